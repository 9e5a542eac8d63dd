// Microbenchmark: what a kernel boundary costs on one stream (gfx950), for the
// pose-cell step's two launches per step -- back-to-back stream launches versus
// the same launches captured once in a hipGraph and replayed, at the step
// kernels' grids (256 x 768 threads: column form at 128x128x72; 192 x 768: rows
// form at 64x64x36), for empty kernels and for kernels that store 16 KiB per
// block write-through (sc1) or plain (dirty lines at the boundary).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_launch.hip -o /tmp/ubl && /tmp/ubl
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
    if (p && threadIdx.x == 100000) p[0] = 1.f;
}

// 16 KiB per block: each of the block's threads stores 16 B (768 threads: 12 KiB)
template <bool WT>
__global__ void k_store(float* p) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    f4 v = {1.f, 2.f, 3.f, (float)i};
    if (WT) {
        typedef unsigned v4u __attribute__((ext_vector_type(4)));
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(p, (short)0, 0x7FFFFFFF, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), r, (int)(i * 16), 0, 16);
    } else {
        reinterpret_cast<f4*>(p)[i] = v;
    }
}

template <typename K>
double stream_us(K kern, int blocks, int threads, float* buf, hipStream_t s, int reps) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, s, buf);
    CHECK(hipEventRecord(e0, s));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, s, buf);
    CHECK(hipEventRecord(e1, s));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return 1e3 * ms / reps;
}

template <typename K>
double graph_us(K kern, int blocks, int threads, float* buf, hipStream_t s, int per_graph, int reps) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < per_graph; ++i) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, s, buf);
    CHECK(hipStreamEndCapture(s, &g));
    CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int i = 0; i < 3; ++i) CHECK(hipGraphLaunch(ge, s));
    CHECK(hipStreamSynchronize(s));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0, s));
    for (int i = 0; i < reps; ++i) CHECK(hipGraphLaunch(ge, s));
    CHECK(hipEventRecord(e1, s));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    CHECK(hipGraphExecDestroy(ge));
    CHECK(hipGraphDestroy(g));
    return 1e3 * ms / ((double)reps * per_graph);
}

int main() {
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    float* buf;
    CHECK(hipMalloc(&buf, (size_t)256 * 1024 * 16));
    const int grids[2][2] = {{256, 768}, {192, 768}};
    for (auto& gr : grids) {
        const int b = gr[0], t = gr[1];
        printf("grid %d x %d\n", b, t);
        printf("  empty   stream %.2f us/kernel   graph(64) %.2f   graph(400) %.2f\n",
               stream_us(k_empty, b, t, buf, s, 2000), graph_us(k_empty, b, t, buf, s, 64, 40),
               graph_us(k_empty, b, t, buf, s, 400, 10));
        printf("  sc1 st  stream %.2f us/kernel   graph(64) %.2f   graph(400) %.2f\n",
               stream_us(k_store<true>, b, t, buf, s, 2000), graph_us(k_store<true>, b, t, buf, s, 64, 40),
               graph_us(k_store<true>, b, t, buf, s, 400, 10));
        printf("  plain st stream %.2f us/kernel  graph(64) %.2f   graph(400) %.2f\n",
               stream_us(k_store<false>, b, t, buf, s, 2000), graph_us(k_store<false>, b, t, buf, s, 64, 40),
               graph_us(k_store<false>, b, t, buf, s, 400, 10));
    }
    printf("grid 256 x 256\n  empty   stream %.2f us/kernel   graph(64) %.2f\n",
           stream_us(k_empty, 256, 256, buf, s, 2000), graph_us(k_empty, 256, 256, buf, s, 64, 40));
    printf("grid 1 x 64\n  empty   stream %.2f us/kernel   graph(64) %.2f\n",
           stream_us(k_empty, 1, 64, buf, s, 2000), graph_us(k_empty, 1, 64, buf, s, 64, 40));
    CHECK(hipFree(buf));
    return 0;
}
