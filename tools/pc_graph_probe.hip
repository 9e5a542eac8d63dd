// Probe (not part of the library): per-step time of the pose-cell step kernels
// launched on the handle's stream (rs_pc_run) versus the same launches captured
// once into a hipGraph and replayed, at a given grid.  Control from the device
// ring (same for every step), results exported as in rs_pc_run.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Ipyratslam_amd/csrc \
//         tools/pc_graph_probe.hip pyratslam_amd/csrc/rs_common.cpp -o /tmp/pcg && /tmp/pcg 128 128 72
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <vector>

#include "posecell.hip"

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    int X = 64, Y = 64, TH = 36;
    if (argc >= 4) {
        X = atoi(argv[1]);
        Y = atoi(argv[2]);
        TH = atoi(argv[3]);
    }
    rs_pc_params p{};
    p.precision = RS_PREC_F32;
    p.global_inhibition = 0.2;
    double norm = 0;
    for (int t = 0; t < 7; ++t) {
        p.ge[t] = std::exp(-(t - 3) * (t - 3) / 2.0) / std::sqrt(2 * M_PI);
        p.gi[t] = std::exp(-(t - 3) * (t - 3) / 8.0) / (2 * std::sqrt(2 * M_PI));
    }
    for (int a = 0; a < 7; ++a)
        for (int b = 0; b < 7; ++b)
            for (int c = 0; c < 7; ++c) norm += p.ge[a] * p.ge[b] * p.ge[c] - p.gi[a] * p.gi[b] * p.gi[c];
    p.k_scale = 1.0 / std::fabs(norm);
    std::vector<double> filt(4 * 49, 1.0 / 49);
    p.nfilters = 4;
    p.xy_filters = filt.data();
    rs_pc* h = nullptr;
    if (rs_pc_create(X, Y, TH, &p, 0, &h) != RS_OK) {
        fprintf(stderr, "create: %s\n", rs_last_error());
        return 1;
    }
    rs_pc_inject(h, 1.0, X / 2, Y / 2, TH / 2);
    const int n = 256;
    std::vector<int32_t> ox(n * TH, 1), oy(n * TH, -1), f(n * TH, 0), out(3 * n);
    std::vector<double> zf(n * 7, 0.1);
    for (int s = 0; s < n; ++s) zf[s * 7 + 3] = 0.4;
    fprintf(stderr, "created, form %s\n", rs_pc_step_form(h));
    for (int rep = 0; rep < 3; ++rep)
        if (rs_pc_run(h, n, ox.data(), oy.data(), f.data(), zf.data(), out.data()) != RS_OK) {
            fprintf(stderr, "run: %s\n", rs_last_error());
            return 1;
        }
    double t0 = now_us();
    const int reps = 10;
    for (int rep = 0; rep < reps; ++rep)
        if (rs_pc_run(h, n, ox.data(), oy.data(), f.data(), zf.data(), out.data()) != RS_OK) return 1;
    const double direct = (now_us() - t0) / (reps * n);
    fprintf(stderr, "rs_pc_run timed\n");
    // the same n steps captured (ring control uploaded once, outside the graph)
    if (pc_grow_steps(h, n) != RS_OK) return 1;
    pc_pack_ctl(h, n, ox.data(), oy.data(), f.data(), zf.data());
    CK(hipMemcpy(h->dCtl, h->hCtl, h->ctlStride * n, hipMemcpyHostToDevice));
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(h->stream, hipStreamCaptureModeGlobal));
    for (int s = 0; s < n; ++s) {
        const PcCtlRing c = make_ctl_ring(h, s);
        if (pc_launch_step<float, PcCtlRing>(h, step_out(h, s), &c, -1) != RS_OK) return 1;
    }
    hipLaunchKernelGGL(pc_res_export, dim3(n), dim3(64), 0, h->stream, h->dRes, n, h->hResDev);
    CK(hipStreamEndCapture(h->stream, &g));
    fprintf(stderr, "captured\n");
    double ti = now_us();
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    const double inst = now_us() - ti;
    CK(hipGraphLaunch(ge, h->stream));
    CK(hipStreamSynchronize(h->stream));
    t0 = now_us();
    for (int rep = 0; rep < reps; ++rep) CK(hipGraphLaunch(ge, h->stream));
    CK(hipStreamSynchronize(h->stream));
    const double graph = (now_us() - t0) / (reps * n);
    // the same with the ring form kernels launched directly (no inline control)
    t0 = now_us();
    for (int rep = 0; rep < reps; ++rep) {
        for (int s = 0; s < n; ++s) {
            const PcCtlRing c = make_ctl_ring(h, s);
            if (pc_launch_step<float, PcCtlRing>(h, step_out(h, s), &c, -1) != RS_OK) return 1;
        }
        hipLaunchKernelGGL(pc_res_export, dim3(n), dim3(64), 0, h->stream, h->dRes, n, h->hResDev);
    }
    CK(hipStreamSynchronize(h->stream));
    const double ring = (now_us() - t0) / (reps * n);
    printf("grid %dx%dx%d form %s: rs_pc_run %.2f us/step; ring launches %.2f us/step; "
           "one graph of all steps %.2f "
           "us/step (instantiate %.0f us for %d steps)\n",
           X, Y, TH, rs_pc_step_form(h), direct, ring, graph, inst, n);
    rs_pc_destroy(h);
    return 0;
}
