// Diagnostic probe for the pose-cell step kernels (not part of the library).
// Builds posecell.hip with its PC_STAMP hook defined so the step kernels write s_memrealtime
// stamps (100 MHz) at their phase boundaries, then reports per-phase times
// over the blocks of one step, and back-to-back launch costs of each kernel
// alone and of an empty kernel with the same grid.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-kernarg-preload-count=9 -Iinclude -Ipyratslam_amd/csrc \
//         tools/pc_probe.hip pyratslam_amd/csrc/rs_common.cpp -o /tmp/pc_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

// the library's phase-stamp hook (posecell.hip leaves it empty)
__device__ unsigned long long* pc_dbg;
#define PC_STAMP(kid, sid)                                                              \
    do {                                                                                \
        if (threadIdx.x == 0) {                                                         \
            const unsigned b_ = blockIdx.y * gridDim.x + blockIdx.x;                    \
            pc_dbg[((kid) * 4096 + b_) * 8 + (sid)] = __builtin_amdgcn_s_memrealtime(); \
        }                                                                               \
    } while (0)
// per-wave stamp: wave w of the block at (kid + w / 8, w % 8)
#define PC_STAMPW(kid)                                                                        \
    do {                                                                                      \
        if ((threadIdx.x & 63) == 0) {                                                        \
            const unsigned b_ = blockIdx.y * gridDim.x + blockIdx.x, w_ = threadIdx.x >> 6;   \
            pc_dbg[((kid + w_ / 8) * 4096 + b_) * 8 + w_ % 8] = __builtin_amdgcn_s_memrealtime(); \
        }                                                                                     \
    } while (0)
#include "posecell.hip"

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                          \
        }                                                                      \
    } while (0)

__global__ void empty_kernel(int* p) {
    if (p && threadIdx.x == 1023) p[0] = 1;
}

static double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0 : v[v.size() / 2];
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
            for (int c = 0; c < 7; ++c)
                norm += p.ge[a] * p.ge[b] * p.ge[c] - p.gi[a] * p.gi[b] * p.gi[c];
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
    // the halo form's last step of a call would also write its per-block records (a
    // one-call-end extra): settle every call, so the stamped last step is a batch step
    rs_pc_debug(h, RS_PC_DBG_HALO_SETTLE);
    unsigned long long* dbg;
    constexpr int NKID = 16;  // stamp slots: kernel id x 4096 blocks x 8 stamps
    const size_t ndbg = (size_t)NKID * 4096 * 8;
    CK(hipMalloc(&dbg, ndbg * 8));
    CK(hipMemset(dbg, 0, ndbg * 8));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(pc_dbg), &dbg, sizeof(dbg)));
    const int n = 200;
    std::vector<int32_t> ox(n * TH, 1), oy(n * TH, -1), f(n * TH, 0), out(3 * n);
    // argv[4] = translation in cells: the per-layer shifts of that step, round(vt cos),
    // round(vt sin) of each layer's heading (posecell_network.py:257-265), as run() sees
    if (argc >= 5) {
        const double vt = atof(argv[4]);
        for (int s = 0; s < n; ++s)
            for (int k = 0; k < TH; ++k) {
                const double a = (k - TH / 2) * 2 * M_PI / TH;
                ox[s * TH + k] = (int)std::nearbyint(vt * std::cos(a));
                oy[s * TH + k] = (int)std::nearbyint(vt * std::sin(a));
            }
    }
    std::vector<double> zf(n * 7, 0.1);
    for (int s = 0; s < n; ++s) zf[s * 7 + 3] = 0.4;
    for (int rep = 0; rep < 3; ++rep)
        if (rs_pc_run(h, n, ox.data(), oy.data(), f.data(), zf.data(), out.data()) != RS_OK) {
            fprintf(stderr, "run: %s\n", rs_last_error());
            return 1;
        }
    double ms = 0;
    rs_pc_last_ms(h, &ms);
    printf("grid %dx%dx%d  form %s  blocks %d  run(%d): %.2f us/step\n", X, Y, TH,
           rs_pc_step_form(h), h->nPart, n, 1e3 * ms / n);
    // stamps of the last step
    std::vector<unsigned long long> st(ndbg);
    CK(hipMemcpy(st.data(), dbg, ndbg * 8, hipMemcpyDeviceToHost));
    const int nb = h->nPart;
    auto slot = [&](int kid, int b, int i) { return st[((size_t)kid * 4096 + b) * 8 + i]; };
    // only the kernels of this handle's form, and of those only the stamps every block
    // wrote: a slot no block stamped (a phase this build does not stamp) is reported as
    // such, never as a difference against zero
    static const char* kname[NKID] = {"excite_rows", "path_rows", "excite_stream", "path_stream", "",
                                      "excite_cols", "path_cols", "halo"};
    static const int kns[NKID] = {4, 6, 5, 5, 0, 5, 5, 7};
    std::vector<int> kids;
    if (h->halo) kids = {7};
    else if (h->cols) kids = {5, 6};
    else if (h->streamed) kids = {2, 3};
    else if (h->tiling) kids = {0, 1};
    auto stamped = [&](int kid, int i) {
        for (int b = 0; b < nb; ++b)
            if (slot(kid, b, i) == 0) return false;
        return true;
    };
    for (int kid : kids) {
        const int ns = kns[kid];
        if (!stamped(kid, 0) || !stamped(kid, ns - 1)) {
            printf("%s: start/end not stamped by this build\n", kname[kid]);
            continue;
        }
        unsigned long long t0 = ~0ull, t1 = 0;
        std::vector<double> starts;
        for (int b = 0; b < nb; ++b) {
            t0 = std::min(t0, slot(kid, b, 0));
            t1 = std::max(t1, slot(kid, b, ns - 1));
        }
        for (int b = 0; b < nb; ++b) starts.push_back((slot(kid, b, 0) - t0) * 10.0);
        printf("%s: first start -> last end %.2f us; start spread median %.2f max %.2f us\n",
               kname[kid], (t1 - t0) * 1e-2, median(starts) * 1e-3,
               *std::max_element(starts.begin(), starts.end()) * 1e-3);
        for (int i = 1; i < ns; ++i) {
            if (!stamped(kid, i - 1) || !stamped(kid, i)) {
                printf("   phase %d: not stamped\n", i);
                continue;
            }
            std::vector<double> ph;
            for (int b = 0; b < nb; ++b) ph.push_back((double)(slot(kid, b, i) - slot(kid, b, i - 1)) * 10.0);
            printf("   phase %d: median %.2f us  max %.2f us\n", i, median(ph) * 1e-3,
                   *std::max_element(ph.begin(), ph.end()) * 1e-3);
        }
    }
    // the last step's kernel boundary: excitation's last block end -> path's first block start
    if (kids.size() == 2 && stamped(kids[0], kns[kids[0]] - 1) && stamped(kids[1], 0)) {
        const int ek = kids[0], pk = kids[1];
        unsigned long long e1 = 0, p0 = ~0ull, e0 = ~0ull, p1 = 0;
        for (int b = 0; b < nb; ++b) {
            e0 = std::min(e0, slot(ek, b, 0));
            e1 = std::max(e1, slot(ek, b, kns[ek] - 1));
            p0 = std::min(p0, slot(pk, b, 0));
            p1 = std::max(p1, slot(pk, b, kns[pk] - 1));
        }
        printf("boundary %s -> %s: %.2f us (excite first start -> path last end %.2f us)\n", kname[ek],
               kname[pk], ((double)p0 - (double)e1) * 1e-2, ((double)p1 - (double)e0) * 1e-2);
    }
    if (h->halo && stamped(11, 0) && stamped(11, 1) && stamped(10, 0) && stamped(10, 1) && stamped(7, 1)) {
        // the halo kernel's phase-1 DMA (stamps 10, 0..1) and theta pass (11, 0..1)
        std::vector<double> a, b;
        for (int bb = 0; bb < h->nPart; ++bb) {
            const unsigned long long* r4 = &st[((size_t)11 * 4096 + bb) * 8];
            const unsigned long long* r7 = &st[((size_t)7 * 4096 + bb) * 8];
            a.push_back((double)(r4[0] - r7[1]) * 10.0);
            b.push_back((double)(r4[1] - r4[0]) * 10.0);
        }
        printf("   halo phase 2: barrier end -> task loop %.2f us, task loop %.2f us (wave 0, median)\n",
               median(a) * 1e-3, median(b) * 1e-3);
        {
            std::vector<double> i1, w1;
            for (int bb = 0; bb < h->nPart; ++bb) {
                const unsigned long long* r3 = &st[((size_t)10 * 4096 + bb) * 8];
                const unsigned long long* r7 = &st[((size_t)7 * 4096 + bb) * 8];
                i1.push_back((double)(r3[0] - r7[0]) * 10.0);
                w1.push_back((double)(r3[1] - r7[0]) * 10.0);
            }
            printf("   halo phase 1 (wave 0): LDS-DMA issued after %.2f us, landed after %.2f us (median)\n",
                   median(i1) * 1e-3, median(w1) * 1e-3);
        }
        if (stamped(11, 2)) {   // the two-group image (round 6): wave 0's segment A, to the group-B wait
            std::vector<double> sa;
            for (int bb = 0; bb < h->nPart; ++bb)
                sa.push_back((double)(st[((size_t)11 * 4096 + bb) * 8 + 2] - st[((size_t)7 * 4096 + bb) * 8 + 1]) * 10.0);
            printf("   halo phase 2 (wave 0): group-A barrier -> segment A done %.2f us (median)\n", median(sa) * 1e-3);
        }
        if (stamped(14, 0) && stamped(14, 1) && stamped(14, 2) && stamped(7, 5)) {   // phase 6's parts (wave 0)
            std::vector<double> f, r, b;
            for (int bb = 0; bb < h->nPart; ++bb) {
                const unsigned long long* r13 = &st[((size_t)14 * 4096 + bb) * 8];
                const unsigned long long p5 = st[((size_t)7 * 4096 + bb) * 8 + 5];
                f.push_back((double)(r13[0] - p5) * 10.0);
                r.push_back((double)(r13[1] - r13[0]) * 10.0);
                b.push_back((double)(r13[2] - r13[1]) * 10.0);
            }
            printf("   halo phase 6 (wave 0): theta filter + store %.2f, reductions %.2f, barrier %.2f us (median)\n",
                   median(f) * 1e-3, median(r) * 1e-3, median(b) * 1e-3);
        }
        printf("   halo phase 2 per wave, task loop end after phase 1 (median us):");
        for (int w = 0; w < 9; ++w) {
            std::vector<double> c;
            if (!stamped(12 + w / 8, w % 8)) {
                printf(" -");
                continue;
            }
            for (int bb = 0; bb < h->nPart; ++bb)
                c.push_back((double)(st[((size_t)(12 + w / 8) * 4096 + bb) * 8 + w % 8] -
                                     st[((size_t)7 * 4096 + bb) * 8 + 1]) * 10.0);
            printf(" %.2f", median(c) * 1e-3);
        }
        printf("\n");
    }
    if (h->halo) {  // back-to-back launch cost of the halo kernel alone, and of an empty one
        hipEvent_t c0, c1;
        CK(hipEventCreate(&c0));
        CK(hipEventCreate(&c1));
        const dim3 g(h->cgx * h->cgy), b(HF_NT);
        const int reps = 500;
        float t = 0;
        CK(hipEventRecord(c0, h->stream));
        for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(empty_kernel, g, b, 0, h->stream, nullptr);
        CK(hipEventRecord(c1, h->stream));
        CK(hipEventSynchronize(c1));
        CK(hipEventElapsedTime(&t, c0, c1));
        printf("empty kernel, same grid: %.2f us/launch\n", 1e3 * t / reps);
        PcCtlHalo c;
        make_ctl_halo(h, 0, ox.data(), oy.data(), f.data(), zf.data(), &c);
        CK(hipEventRecord(c0, h->stream));
        for (int i = 0; i < reps; ++i)
            hf_launch<false>(h->TH, g, h->stream, (const float*)h->dP, hf_pack(X, Y),
                               hf_pack(h->cgx, g.x), hf_pack(c.ux, c.uy), hf_pack(c.uw, c.uh), hf_magic(h->cgx),
                               hf_magic(c.uh), h->dPart, h->nPart, (float*)h->dQ, h->dPart + h->nPart, h->dRes, h->dRes + RES_SLOTS,
                               (const float*)h->dFilt, h->nf, c, h->kf, nullptr);
        CK(hipEventRecord(c1, h->stream));
        CK(hipEventSynchronize(c1));
        CK(hipEventElapsedTime(&t, c0, c1));
        printf("halo step alone: %.2f us/launch\n", 1e3 * t / reps);
        rs_pc_destroy(h);
        return 0;
    }
    if (h->streamed) {
        printf("stream tile BX=%d WR=%d KC=%d grid %d blocks\n", h->sbx, h->swr, h->sg.KC,
               h->sg.gx * h->sg.gy * h->sg.gz);
        rs_pc_destroy(h);
        return 0;
    }
    if (h->cols && h->coKC >= TH) {  // back-to-back launch costs of the column kernels
        hipEvent_t c0, c1;
        CK(hipEventCreate(&c0));
        CK(hipEventCreate(&c1));
        const dim3 g(h->cgx * h->cgy), b(64 * CO_NW), bp(64 * CO_NW);
        constexpr int THF = co_thmax<float>();
        const int reps = 500;
        float t = 0;
        CK(hipEventRecord(c0, h->stream));
        for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(empty_kernel, g, b, 0, h->stream, nullptr);
        CK(hipEventRecord(c1, h->stream));
        CK(hipEventSynchronize(c1));
        CK(hipEventElapsedTime(&t, c0, c1));
        printf("empty kernel, same grid: %.2f us/launch\n", 1e3 * t / reps);
        const PcCtlRing ctl = make_ctl_ring(h, 0);
        CK(hipEventRecord(c0, h->stream));
        for (int i = 0; i < reps; ++i)
            hipLaunchKernelGGL((pc_excite_cols<float, CO_TX, CO_TY, CO_NW, THF, false>), g, b, 0, h->stream,
                               (const float*)h->dP, X, Y, TH, h->cgx, h->cgy, (int)g.x, (float*)h->dQ,
                               h->dPart, h->dRes, h->coKC, h->kf);
        CK(hipEventRecord(c1, h->stream));
        CK(hipEventSynchronize(c1));
        CK(hipEventElapsedTime(&t, c0, c1));
        printf("excite alone: %.2f us/launch\n", 1e3 * t / reps);
        CK(hipEventRecord(c0, h->stream));
        for (int i = 0; i < reps; ++i)
            hipLaunchKernelGGL((pc_path_cols<float, CO_TX, CO_TY, CO_NW, THF, false, PcCtlRing>), g, bp, 0, h->stream,
                               (const float*)h->dQ, X, Y, TH, h->cgx, h->cgy, (int)g.x, (float*)h->dP, h->dPart,
                               h->nPart, (const float*)h->dFilt, h->nf, ctl, h->dRes, (float*)nullptr,
                               (unsigned*)nullptr, h->coKC);
        CK(hipEventRecord(c1, h->stream));
        CK(hipEventSynchronize(c1));
        CK(hipEventElapsedTime(&t, c0, c1));
        printf("path alone: %.2f us/launch\n", 1e3 * t / reps);
        rs_pc_destroy(h);
        return 0;
    }
    if (h->cols) {
        rs_pc_destroy(h);
        return 0;
    }
    if (Y > 64) {
        rs_pc_destroy(h);
        return 0;
    }
    // back-to-back launch costs (rows form, Y <= 64)
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const dim3 g((X + RT_BX - 1) / RT_BX, (TH + RT_BK - 1) / RT_BK);
    const int reps = 500;
    float t = 0;
    CK(hipEventRecord(e0, h->stream));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL(empty_kernel, g, dim3(256), 0, h->stream, nullptr);
    CK(hipEventRecord(e1, h->stream));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&t, e0, e1));
    printf("empty kernel, same grid: %.2f us/launch\n", 1e3 * t / reps);
    const PcCtlRing ctl = make_ctl_ring(h, 0);
    CK(hipEventRecord(e0, h->stream));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((pc_excite_rows<float, 64>), g, dim3(RT_NT), 0, h->stream,
                           (const float*)h->dP, (float*)h->dQ, h->dPart, h->dRes, X, Y, TH, h->kf);
    CK(hipEventRecord(e1, h->stream));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&t, e0, e1));
    printf("excite alone: %.2f us/launch\n", 1e3 * t / reps);
    CK(hipEventRecord(e0, h->stream));
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((pc_path_rows<float, 64, PcCtlRing>), g, dim3(RT_NT), 0, h->stream,
                           (const float*)h->dQ, (float*)h->dP, h->dPart, h->nPart,
                           (const float*)h->dFilt, h->nf, ctl, h->dRes, (float*)nullptr,
                           (unsigned*)nullptr, X, Y, TH);
    CK(hipEventRecord(e1, h->stream));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&t, e0, e1));
    printf("path alone: %.2f us/launch\n", 1e3 * t / reps);
    rs_pc_destroy(h);
    return 0;
}
