// LDS read throughput of ds_read_b128 by the number of distinct 16-byte addresses
// per wave-instruction (lanes in NA groups of 64/NA share an address), with a
// VALU load beside it like the plane scan's (bitop3 chains on the loaded words).
// usage: hipcc --offload-arch=gfx950 -O3 tools/ubench_lds.hip -o /tmp/ubench_lds && /tmp/ubench_lds
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int NA, int VALU>
__global__ __launch_bounds__(512) void k_lds(uint32_t* out, int iters) {
    __shared__ __attribute__((aligned(16))) uint32_t buf[8192];
    for (int i = threadIdx.x; i < 8192; i += blockDim.x) buf[i] = i * 2654435761u;
    __syncthreads();
    const int lane = threadIdx.x & 63, grp = lane / (64 / NA);
    // group g reads at a stride of 216 dwords (the plane scan's record layout)
    const uint32_t* base = buf + grp * 216;
    uint32_t acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = lane * (2 * i + 1);
    for (int it = 0; it < iters; ++it) {
#pragma unroll 2
        for (int r = 0; r < 26; ++r) {
            const uint4 a = *reinterpret_cast<const uint4*>(base + r * 8);
            const uint4 b = *reinterpret_cast<const uint4*>(base + r * 8 + 4);
            const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
            // 8 independent chains, like the plane scan's interleaved borrow chains
#pragma unroll
            for (int v = 0; v < 4 + 4 * VALU; ++v)
                acc[v % 8] = __builtin_amdgcn_bitop3_b32(acc[v % 8], w[v % 8], w[(v + 3) % 8], 0x8E);
        }
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) x ^= acc[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <int NA, int VALU>
void run(uint32_t* d, int cus) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 200, blocks = 2 * cus;
    hipLaunchKernelGGL((k_lds<NA, VALU>), dim3(blocks), dim3(512), 0, 0, d, 10);
    hipEventRecord(e0);
    hipLaunchKernelGGL((k_lds<NA, VALU>), dim3(blocks), dim3(512), 0, 0, d, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double reads = 2.0 * 26 * iters * blocks * 8;          // wave-instructions
    const double valu = (4.0 + 4.0 * VALU) * 26 * iters * blocks * 8;
    printf("addresses/instr %d, valu/row %3d: %.3f ms, %.2f ds_read_b128/CU/ns, %.3f VALU/SIMD/cycle@2.4GHz\n",
           NA, 4 + 4 * VALU, ms, reads / cus / (ms * 1e6), valu / (cus * 4.0) / (ms * 1e-3 * 2.4e9));
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t* d;
    hipMalloc(&d, sizeof(uint32_t) * 512 * 2 * cus);
    run<1, 0>(d, cus); run<2, 0>(d, cus); run<4, 0>(d, cus); run<8, 0>(d, cus);
    run<1, 7>(d, cus); run<2, 7>(d, cus); run<4, 7>(d, cus); run<8, 7>(d, cus);
    run<1, 16>(d, cus); run<8, 16>(d, cus);
    hipFree(d);
    return 0;
}
