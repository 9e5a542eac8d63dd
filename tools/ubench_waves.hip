// Microbenchmark: back-to-back cost of a dependent empty launch on one stream as a
// function of the block size and of the LDS a block allocates (gfx950), at the
// pose-cell column kernels' grid of 256 blocks: does the launch floor grow with
// the waves a grid dispatches?
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_waves.hip -o /tmp/ubw && /tmp/ubw
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                     \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

__global__ void k_empty(float* p) {
    extern __shared__ float lds[];
    if (p && threadIdx.x == 100000) p[0] = lds[threadIdx.x];
}

static double stream_us(int blocks, int threads, int lds, float* buf, hipStream_t s, int reps) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(threads), lds, s, buf);
    CHECK(hipEventRecord(e0, s));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(threads), lds, s, buf);
    CHECK(hipEventRecord(e1, s));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return 1e3 * ms / reps;
}

int main() {
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_empty),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    float* buf;
    CHECK(hipMalloc(&buf, 1 << 20));
    const int threads[] = {64, 256, 512, 768, 1024};
    const int ldss[] = {0, 80 * 1024, 150 * 1024};
    for (int blocks : {256, 512}) {
        for (int lds : ldss) {
            printf("blocks %d  LDS %6d B:", blocks, lds);
            for (int t : threads) printf("  %4d thr %.2f", t, stream_us(blocks, t, lds, buf, s, 2000));
            printf("  us/launch\n");
        }
    }
    CHECK(hipFree(buf));
    return 0;
}
