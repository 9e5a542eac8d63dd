// Diagnostic (not part of the library): does a revision of posecell.hip read step
// scratch it did not write, or return a result word the export never stored?
// Compiled against any revision's sources (the -I path picks the revision):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I<rev>/include -I<rev>/pyratslam_amd/csrc \
//         -x hip -fno-slp-vectorize tools/poison_probe.hip <rev>/pyratslam_amd/csrc/rs_common.cpp -o probe
// For each scratch buffer (the excited volume Q, the normalisation partials, the
// argmax slots) a fresh handle has that buffer filled with all-ones bytes (NaN /
// the largest key) right after create; it then takes the same injected start and
// the same steps as a handle whose scratch was zeroed, and the peaks and states are
// compared bit for bit.  A last pass writes a fake key into the host result word
// before every update() and counts the updates that returned it (an export store
// not visible to the host after the stream synchronised).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
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

static rs_pc_params params(std::vector<double>& filt) {
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
    filt.assign(2 * 49, 0.0);
    for (int i = 0; i < 49; ++i) {
        const int a = i / 7 - 3, b = i % 7 - 3;
        filt[i] = std::exp(-(a * a + b * b) / 3.0);
        filt[49 + i] = std::exp(-((a + 1) * (a + 1) + (b + 1) * (b + 1)) / 3.0);
    }
    p.nfilters = 2;
    p.xy_filters = filt.data();
    return p;
}

int main(int argc, char** argv) {
    const int X = argc > 1 ? atoi(argv[1]) : 128, Y = argc > 2 ? atoi(argv[2]) : 128;
    const int TH = argc > 3 ? atoi(argv[3]) : 72, steps = 4;
    std::vector<double> filt;
    const rs_pc_params p = params(filt);
    // the steps: a 1.2-cell translation at heading 0.3 rad, per-layer shifts as
    // posecell_network.py:257-265 forms them, filter 0/1 by the sign of the residual
    std::vector<int32_t> ox(steps * TH), oy(steps * TH), fi(steps * TH);
    std::vector<double> zf(steps * 7, 0.0);
    for (int s = 0; s < steps; ++s) {
        for (int k = 0; k < TH; ++k) {
            const double a = (k - TH / 2) * 2 * M_PI / TH + 0.3, ex = 1.2 * std::cos(a), ey = 1.2 * std::sin(a);
            ox[s * TH + k] = (int)std::nearbyint(ex);
            oy[s * TH + k] = (int)std::nearbyint(ey);
            fi[s * TH + k] = ex - std::nearbyint(ex) < 0 ? 1 : 0;
        }
        for (int z = 0; z < 7; ++z) zf[s * 7 + z] = std::exp(-(z - 3) * (z - 3) / 2.0) / 2.5;
    }
    const char* what[4] = {"zeroed scratch", "excited volume Q poisoned", "partials poisoned",
                           "argmax slots poisoned"};
    std::vector<float> ref, got(size_t(X) * Y * TH);
    std::vector<int32_t> refpk, pk(3 * steps);
    int bad = 0;
    for (int v = 0; v < 4; ++v) {
        rs_pc* h = nullptr;
        if (rs_pc_create(X, Y, TH, &p, 0, &h) != RS_OK) {
            fprintf(stderr, "create: %s\n", rs_last_error());
            return 1;
        }
        if (pc_grow_steps(h, steps) != RS_OK) return 1;   // the argmax slots exist now
        const size_t nres = sizeof(unsigned long long) * RES_SLOTS * h->resCap;
        CK(hipMemsetAsync(h->dQ, v == 1 ? 0xFF : 0, h->n * h->esz, h->stream));
        CK(hipMemsetAsync(h->dPart, v == 2 ? 0xFF : 0, sizeof(double) * h->nPart, h->stream));
        CK(hipMemsetAsync(h->dRes, v == 3 ? 0xFF : 0, nres, h->stream));
        CK(hipStreamSynchronize(h->stream));
        rs_pc_inject(h, 1.0, X / 2, Y / 2, TH / 2);
        for (int s = 0; s < steps; ++s)
            if (rs_pc_update(h, &ox[s * TH], &oy[s * TH], &fi[s * TH], &zf[s * 7], &pk[3 * s]) != RS_OK) {
                fprintf(stderr, "update: %s\n", rs_last_error());
                return 1;
            }
        CK(hipMemcpy(got.data(), h->dP, h->n * h->esz, hipMemcpyDeviceToHost));
        int nan = 0;
        for (float x : got) nan += std::isnan(x);
        if (v == 0) {
            ref = got;
            refpk = pk;
        }
        const bool same = v == 0 || (pk == refpk && !memcmp(got.data(), ref.data(), got.size() * 4));
        printf("%-28s form %-6s peaks", what[v], rs_pc_step_form(h));
        for (int s = 0; s < steps; ++s) printf(" (%d,%d,%d)", pk[3 * s], pk[3 * s + 1], pk[3 * s + 2]);
        printf("  NaN cells %d  %s\n", nan, same ? "identical to zeroed" : "DIFFERENT");
        bad += !same;
        rs_pc_destroy(h);
    }
    // host result word: a fake key written before each update(); count returns of it
    {
        rs_pc* h = nullptr;
        if (rs_pc_create(X, Y, TH, &p, 0, &h) != RS_OK) return 1;
        if (pc_grow_steps(h, steps) != RS_OK) return 1;
        rs_pc_inject(h, 1.0, X / 2, Y / 2, TH / 2);
        const unsigned lin = (1u * Y + 2u) * TH + 3u;  // cell (1, 2, 3)
        const float half = 0.5f;
        unsigned hb;
        memcpy(&hb, &half, 4);
        const unsigned long long fake = ((unsigned long long)hb << 32) | (0xFFFFFFFFu - lin);
        int stale = 0;
        const int n = 20000;
        for (int i = 0; i < n; ++i) {
            h->hRes[0] = fake;
            const int s = i % steps;
            if (rs_pc_update(h, &ox[s * TH], &oy[s * TH], &fi[s * TH], &zf[s * 7], &pk[0]) != RS_OK) {
                fprintf(stderr, "update: %s\n", rs_last_error());
                return 1;
            }
            stale += pk[0] == 1 && pk[1] == 2 && pk[2] == 3;
        }
        printf("host result word: %d of %d updates returned the fake key written before them\n", stale, n);
        bad += stale != 0;
        rs_pc_destroy(h);
    }
    printf("%s\n", bad ? "FOUND" : "clean");
    return 0;
}
