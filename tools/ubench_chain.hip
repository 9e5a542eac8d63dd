// Microbenchmark: chip-wide issue rate of interleaved v_bitop3_b32 borrow chains
// with a scalar operand (the bit-plane scan's inner loop), by waves per SIMD (w)
// and by how far the loop is unrolled (U: body = 16*U instructions, 8 bytes each),
// to separate VALU issue limits from instruction-fetch limits.
// Rate = all wave-instructions / (kernel event time x shader clock x SIMDs).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_chain.hip -o tools/ubench_chain
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int ITERS = 4096;

template <int U, int MODE>
__global__ __launch_bounds__(256) void chain(unsigned* out, unsigned long long* clk, unsigned s0) {
    unsigned b[4], t[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) { b[i] = threadIdx.x + i; t[i] = threadIdx.x * (i + 3); }
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll U
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int rep = 0; rep < 4; ++rep)
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (MODE == 0)
                    asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x8e" : "+v"(b[k]) : "v"(t[k]), "s"(s0));
                else if (MODE == 1)
                    asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x8e" : "+v"(b[k]) : "v"(t[k]), "v"(t[(k + 1) & 3]));
                else if (MODE == 2)
                    asm volatile("v_xor_b32 %0, %1, %0" : "+v"(b[k]) : "v"(t[k]));
                else
                    asm volatile("v_add_u32 %0, %1, %0" : "+v"(b[k]) : "s"(s0));
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = b[0] ^ b[1] ^ b[2] ^ b[3];
    if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = c1 - c0; clk[1] = r1 - r0; }
}

template <int U, int MODE>
void run(int w) {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount, blocks = cus * w;
    unsigned* out;
    unsigned long long* clk;
    hipMalloc(&out, sizeof(unsigned) * blocks * 256);
    hipMalloc(&clk, 16);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL((chain<U, MODE>), dim3(blocks), dim3(256), 0, 0, out, clk, 3u);
    hipEventRecord(e0);
    hipLaunchKernelGGL((chain<U, MODE>), dim3(blocks), dim3(256), 0, 0, out, clk, 3u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c[2];
    hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
    const double ghz = c[0] / (c[1] * 10.0);
    const double insns = (double)blocks * 4 * ITERS * 16;
    static const char* names[] = {"bitop3 s", "bitop3 v", "xor v", "add s"};
    printf("%-9s U=%4d (body %6d B) w=%d: %.3f wave-insn/SIMD-cycle (clock %.2f GHz, %.1f us)\n", names[MODE], U,
           16 * U * 8, w, insns / (ms * 1e-3 * ghz * 1e9 * cus * 4), ghz, ms * 1e3);
    hipFree(out);
    hipFree(clk);
}

int main() {
    for (int w : {2, 3, 4, 8}) {
        run<16, 0>(w); run<16, 1>(w); run<16, 2>(w); run<16, 3>(w);
    }
    return 0;
}
