// Microbenchmark: chip-wide issue rate of the VALU instructions the template
// scan is built from (gfx950).  Each lane runs 8 independent dependency chains
// of one instruction (inline asm, so nothing is folded), the grid fills every
// SIMD with `waves` waves.  Prints wave-instructions per second and per SIMD-cycle.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip -o /tmp/ubench && /tmp/ubench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                     \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

constexpr int ITERS = 4096;

#define CHAIN8(INSN)                                                                 \
    _Pragma("unroll 8") for (int i = 0; i < ITERS; ++i) {                            \
        INSN(a0); INSN(a1); INSN(a2); INSN(a3); INSN(a4); INSN(a5); INSN(a6); INSN(a7); \
    }

#define SAD(r) asm volatile("v_sad_u8 %0, %1, %2, %0" : "+v"(r) : "v"(x), "v"(y))
#define ADD(r) asm volatile("v_add_u32 %0, %1, %0" : "+v"(r) : "v"(x))
#define BOP3(r) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(r) : "v"(x), "v"(y))
#define XOR(r) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(r) : "v"(x))
#define DOT4(r) asm volatile("v_dot4_u32_u8 %0, %1, %2, %0" : "+v"(r) : "v"(x), "v"(y))
#define BCNT(r) asm volatile("v_bcnt_u32_b32 %0, %1, %0" : "+v"(r) : "v"(x))
#define ADD3(r) asm volatile("v_add3_u32 %0, %1, %2, %0" : "+v"(r) : "v"(x), "v"(y))
#define PERM(r) asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(r) : "v"(x), "v"(y))
#define CARRY(r)                                                                     \
    asm volatile("v_add_u32 %0, %1, %0\n\tv_bitop3_b32 %0, %1, %2, %0 bitop3:0xe8\n\t" \
                 "v_bcnt_u32_b32 %0, %0, %0" : "+v"(r) : "v"(x), "v"(y))
#define MIX(r)                                                                       \
    asm volatile("v_add_u32 %0, %1, %0\n\tv_bitop3_b32 %0, %0, %1, %2 bitop3:0x96\n\t" \
                 "v_sad_u8 %0, %0, 0, %0" : "+v"(r) : "v"(x), "v"(y))

template <int K>
__global__ void ubench(unsigned* out, unsigned x, unsigned y) {
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
             a6 = a0 + 6, a7 = a0 + 7;
    if (K == 0) CHAIN8(SAD)
    if (K == 1) CHAIN8(ADD)
    if (K == 2) CHAIN8(BOP3)
    if (K == 3) CHAIN8(XOR)
    if (K == 4) CHAIN8(DOT4)
    if (K == 5) CHAIN8(MIX)
    if (K == 6) CHAIN8(BCNT)
    if (K == 7) CHAIN8(ADD3)
    if (K == 8) CHAIN8(PERM)
    if (K == 9) CHAIN8(CARRY)
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <int K>
void run(const char* name, int insn_per_body, int waves_per_simd) {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const int blocks = cus * waves_per_simd;  // 256-thread blocks = 4 waves = 1 per SIMD
    unsigned* out;
    CHECK(hipMalloc(&out, sizeof(unsigned) * blocks * 256));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipLaunchKernelGGL(ubench<K>, dim3(blocks), dim3(256), 0, 0, out, 0x01020304u, 0x80706050u);
    CHECK(hipEventRecord(e0));
    const int reps = 5;
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL(ubench<K>, dim3(blocks), dim3(256), 0, 0, out, 0x01020304u, 0x80706050u);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double waves = (double)blocks * 4 * reps;
    const double insns = waves * ITERS * 8.0 * insn_per_body;
    const double rate = insns / (ms * 1e-3);
    const double simd_cycles = (double)cus * 4 * 2.4e9;
    printf("%-8s waves/SIMD=%d  %.3e wave-insn/s  %.3f wave-insn per SIMD-cycle @2.4GHz\n", name,
           waves_per_simd, rate, rate / simd_cycles);
    CHECK(hipFree(out));
}

int main() {
    for (int w : {2, 4, 8}) {
        run<0>("sad_u8", 1, w);
        run<1>("add_u32", 1, w);
        run<2>("bitop3", 1, w);
        run<6>("bcnt", 1, w);
        run<7>("add3", 1, w);
        run<8>("perm", 1, w);
        run<5>("mix3", 3, w);
        run<9>("carry3", 3, w);
    }
    return 0;
}
