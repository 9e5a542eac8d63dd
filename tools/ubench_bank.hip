// Microbenchmark: does VGPR bank placement of v_bitop3_b32's three sources change
// its issue rate on gfx950?  Eight independent chains per wave in fixed physical
// registers (inline asm), grid fills every SIMD with `waves` waves; also the
// shader clock (s_memtime vs s_memrealtime) so rates are per real SIMD-cycle.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_bank.hip -o /tmp/ubb && /tmp/ubb
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                          \
    do {                                                                  \
        hipError_t e = (x);                                               \
        if (e != hipSuccess) {                                            \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));      \
            exit(1);                                                      \
        }                                                                 \
    } while (0)

constexpr int ITERS = 2048;
// dst chains in v40..v47 (banks 0,1,2,3,0,1,2,3); sources chosen per variant
#define B8(S1, S2)                                              \
    "v_bitop3_b32 v40, " S1 ", " S2 ", v40 bitop3:0x8e\n\t"     \
    "v_bitop3_b32 v41, " S1 ", " S2 ", v41 bitop3:0x8e\n\t"     \
    "v_bitop3_b32 v42, " S1 ", " S2 ", v42 bitop3:0x8e\n\t"     \
    "v_bitop3_b32 v43, " S1 ", " S2 ", v43 bitop3:0x8e\n\t"     \
    "v_bitop3_b32 v44, " S1 ", " S2 ", v44 bitop3:0x8e\n\t"     \
    "v_bitop3_b32 v45, " S1 ", " S2 ", v45 bitop3:0x8e\n\t"     \
    "v_bitop3_b32 v46, " S1 ", " S2 ", v46 bitop3:0x8e\n\t"     \
    "v_bitop3_b32 v47, " S1 ", " S2 ", v47 bitop3:0x8e\n\t"
// same-bank for every instruction: sources in the destination's bank
#define SAME8                                                   \
    "v_bitop3_b32 v40, v48, v52, v40 bitop3:0x8e\n\t"           \
    "v_bitop3_b32 v41, v49, v53, v41 bitop3:0x8e\n\t"           \
    "v_bitop3_b32 v42, v50, v54, v42 bitop3:0x8e\n\t"           \
    "v_bitop3_b32 v43, v51, v55, v43 bitop3:0x8e\n\t"           \
    "v_bitop3_b32 v44, v48, v52, v44 bitop3:0x8e\n\t"           \
    "v_bitop3_b32 v45, v49, v53, v45 bitop3:0x8e\n\t"           \
    "v_bitop3_b32 v46, v50, v54, v46 bitop3:0x8e\n\t"           \
    "v_bitop3_b32 v47, v51, v55, v47 bitop3:0x8e\n\t"
// all three sources in distinct banks
#define DIFF8                                                   \
    "v_bitop3_b32 v40, v49, v54, v40 bitop3:0x8e\n\t"           \
    "v_bitop3_b32 v41, v50, v55, v41 bitop3:0x8e\n\t"           \
    "v_bitop3_b32 v42, v51, v52, v42 bitop3:0x8e\n\t"           \
    "v_bitop3_b32 v43, v48, v53, v43 bitop3:0x8e\n\t"           \
    "v_bitop3_b32 v44, v49, v54, v44 bitop3:0x8e\n\t"           \
    "v_bitop3_b32 v45, v50, v55, v45 bitop3:0x8e\n\t"           \
    "v_bitop3_b32 v46, v51, v52, v46 bitop3:0x8e\n\t"           \
    "v_bitop3_b32 v47, v48, v53, v47 bitop3:0x8e\n\t"
// two sources share a bank, third differs
#define PAIR8                                                   \
    "v_bitop3_b32 v40, v48, v53, v40 bitop3:0x8e\n\t"           \
    "v_bitop3_b32 v41, v49, v54, v41 bitop3:0x8e\n\t"           \
    "v_bitop3_b32 v42, v50, v55, v42 bitop3:0x8e\n\t"           \
    "v_bitop3_b32 v43, v51, v52, v43 bitop3:0x8e\n\t"           \
    "v_bitop3_b32 v44, v48, v53, v44 bitop3:0x8e\n\t"           \
    "v_bitop3_b32 v45, v49, v54, v45 bitop3:0x8e\n\t"           \
    "v_bitop3_b32 v46, v50, v55, v46 bitop3:0x8e\n\t"           \
    "v_bitop3_b32 v47, v51, v52, v47 bitop3:0x8e\n\t"
#define BCNT8                                                   \
    "v_bcnt_u32_b32 v40, v49, v40\n\t"                          \
    "v_bcnt_u32_b32 v41, v50, v41\n\t"                          \
    "v_bcnt_u32_b32 v42, v51, v42\n\t"                          \
    "v_bcnt_u32_b32 v43, v48, v43\n\t"                          \
    "v_bcnt_u32_b32 v44, v49, v44\n\t"                          \
    "v_bcnt_u32_b32 v45, v50, v45\n\t"                          \
    "v_bcnt_u32_b32 v46, v51, v46\n\t"                          \
    "v_bcnt_u32_b32 v47, v48, v47\n\t"

#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", \
             "v51", "v52", "v53", "v54", "v55"

template <int K>
__global__ void ubench(unsigned* out, unsigned long long* clk) {
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    asm volatile("v_mov_b32 v48, %0\n\tv_mov_b32 v49, %0\n\tv_mov_b32 v50, %0\n\tv_mov_b32 v51, %0\n\t"
                 "v_mov_b32 v52, %0\n\tv_mov_b32 v53, %0\n\tv_mov_b32 v54, %0\n\tv_mov_b32 v55, %0\n\t"
                 "v_mov_b32 v40, %0\n\tv_mov_b32 v41, %0\n\tv_mov_b32 v42, %0\n\tv_mov_b32 v43, %0\n\t"
                 "v_mov_b32 v44, %0\n\tv_mov_b32 v45, %0\n\tv_mov_b32 v46, %0\n\tv_mov_b32 v47, %0"
                 :: "v"(threadIdx.x) : CLOB);
    for (int i = 0; i < ITERS; ++i) {
        if (K == 0) asm volatile(SAME8 SAME8 SAME8 SAME8 ::: CLOB);
        if (K == 1) asm volatile(DIFF8 DIFF8 DIFF8 DIFF8 ::: CLOB);
        if (K == 2) asm volatile(PAIR8 PAIR8 PAIR8 PAIR8 ::: CLOB);
        if (K == 3) asm volatile(DIFF8 DIFF8 DIFF8 DIFF8 DIFF8 DIFF8 DIFF8 DIFF8 BCNT8 ::: CLOB);
        if (K == 4) asm volatile(BCNT8 BCNT8 BCNT8 BCNT8 ::: CLOB);
    }
    unsigned r;
    asm volatile("v_xor_b32 %0, v40, v47" : "=v"(r) :: CLOB);
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        clk[0] = __builtin_amdgcn_s_memtime() - t0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

template <int K>
void run(const char* name, int insn_per_iter, int waves_per_simd) {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const int blocks = cus * waves_per_simd;
    unsigned* out;
    unsigned long long* clk;
    CHECK(hipMalloc(&out, sizeof(unsigned) * blocks * 256));
    CHECK(hipMalloc(&clk, 16));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(ubench<K>, dim3(blocks), dim3(256), 0, 0, out, clk);
    CHECK(hipEventRecord(e0));
    const int reps = 5;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(ubench<K>, dim3(blocks), dim3(256), 0, 0, out, clk);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long c[2];
    CHECK(hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost));
    const double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;  // memtime ticks at shader clock? see note
    const double insns = (double)blocks * 4 * reps * ITERS * insn_per_iter;
    const double rate = insns / (ms * 1e-3);
    printf("%-10s waves/SIMD=%d  %.3e wave-insn/s  %.3f per SIMD-cycle @2.4GHz  (memtime/realtime %.3f GHz)\n",
           name, waves_per_simd, rate, rate / ((double)cus * 4 * 2.4e9), ghz);
    CHECK(hipFree(out));
    CHECK(hipFree(clk));
}

int main() {
    for (int w : {2, 4}) {
        run<0>("same-bank", 32, w);
        run<1>("diff-bank", 32, w);
        run<2>("pair-bank", 32, w);
        run<3>("64b+8bcnt", 72, w);
        run<4>("bcnt", 32, w);
    }
    return 0;
}
