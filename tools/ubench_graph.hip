// Microbenchmark: host-synchronous round trips of a pose-cell update() (three
// launches -- excite, path, export -- then a stream synchronisation), as direct
// stream launches versus one hipGraph launch, and the host cost of updating one
// kernel node's arguments (per-step control as kernel arguments) before a launch.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_graph.hip -o /tmp/ubg && /tmp/ubg
#include <hip/hip_runtime.h>

#include <chrono>
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

struct Ctl {  // ~700 B, like PcCtlInline
    short ox[128], oy[128];
    unsigned char f[128];
    double zf[8];
};

__global__ void k_a(float* p) {
    if (p && threadIdx.x == 100000) p[0] = 1.f;
}
__global__ void k_b(float* p, Ctl c) {
    if (p && threadIdx.x == 100000) p[0] = (float)c.ox[blockIdx.x & 127];
}
__global__ void k_c(float* p) {
    if (p && threadIdx.x == 100000) p[1] = 1.f;
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    float* buf;
    CHECK(hipMalloc(&buf, 1024));
    Ctl c{};
    const int reps = 2000;
    for (int grid : {192, 256}) {
        // (a) direct launches + sync
        for (int i = 0; i < 100; ++i) {
            hipLaunchKernelGGL(k_a, dim3(grid), dim3(768), 0, s, buf);
            hipLaunchKernelGGL(k_b, dim3(grid), dim3(768), 0, s, buf, c);
            hipLaunchKernelGGL(k_c, dim3(1), dim3(64), 0, s, buf);
            CHECK(hipStreamSynchronize(s));
        }
        double t0 = now_us();
        for (int i = 0; i < reps; ++i) {
            c.ox[i & 127] = (short)i;
            hipLaunchKernelGGL(k_a, dim3(grid), dim3(768), 0, s, buf);
            hipLaunchKernelGGL(k_b, dim3(grid), dim3(768), 0, s, buf, c);
            hipLaunchKernelGGL(k_c, dim3(1), dim3(64), 0, s, buf);
            CHECK(hipStreamSynchronize(s));
        }
        const double direct = (now_us() - t0) / reps;
        // (b) graph of the three + sync; (c) with one node's arguments set per call
        hipGraph_t g;
        hipGraphExec_t ge;
        CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        hipLaunchKernelGGL(k_a, dim3(grid), dim3(768), 0, s, buf);
        hipLaunchKernelGGL(k_b, dim3(grid), dim3(768), 0, s, buf, c);
        hipLaunchKernelGGL(k_c, dim3(1), dim3(64), 0, s, buf);
        CHECK(hipStreamEndCapture(s, &g));
        CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        size_t nn = 0;
        CHECK(hipGraphGetNodes(g, nullptr, &nn));
        hipGraphNode_t nodes[8];
        CHECK(hipGraphGetNodes(g, nodes, &nn));
        hipGraphNode_t nb = nullptr;
        hipKernelNodeParams kp{};
        for (size_t i = 0; i < nn; ++i) {
            hipKernelNodeParams q{};
            if (hipGraphKernelNodeGetParams(nodes[i], &q) == hipSuccess &&
                q.func == reinterpret_cast<void*>(&k_b)) {
                nb = nodes[i];
                kp = q;
            }
        }
        for (int i = 0; i < 100; ++i) {
            CHECK(hipGraphLaunch(ge, s));
            CHECK(hipStreamSynchronize(s));
        }
        t0 = now_us();
        for (int i = 0; i < reps; ++i) {
            CHECK(hipGraphLaunch(ge, s));
            CHECK(hipStreamSynchronize(s));
        }
        const double graph = (now_us() - t0) / reps;
        double setp = -1, graph_set = -1;
        if (nb) {
            void* args[2] = {&buf, &c};
            kp.kernelParams = args;
            t0 = now_us();
            for (int i = 0; i < reps; ++i) {
                c.ox[i & 127] = (short)i;
                CHECK(hipGraphExecKernelNodeSetParams(ge, nb, &kp));
            }
            setp = (now_us() - t0) / reps;
            t0 = now_us();
            for (int i = 0; i < reps; ++i) {
                c.ox[i & 127] = (short)i;
                CHECK(hipGraphExecKernelNodeSetParams(ge, nb, &kp));
                CHECK(hipGraphLaunch(ge, s));
                CHECK(hipStreamSynchronize(s));
            }
            graph_set = (now_us() - t0) / reps;
        }
        printf("grid %d: direct 3 launches + sync %.2f us; graph launch + sync %.2f us; "
               "node SetParams %.2f us; SetParams + graph + sync %.2f us\n",
               grid, direct, graph, setp, graph_set);
        CHECK(hipGraphExecDestroy(ge));
        CHECK(hipGraphDestroy(g));
    }
    return 0;
}
