/*
 * C restatement of the pyratslam hot path -- TEST INFRASTRUCTURE / CPU BASELINE ONLY.
 * Never linked by the product (pyratslam_amd).  Built by oracle/c/Makefile into
 * oracle/lib/libratslam_oracle.so; used by tests (as a second checker) and by
 * bench.py's cpu_baseline leg (OpenMP over the host's cores).
 *
 * Restates, in float64 and in the reference kernels' tap order:
 *   ro_conv3d   OpenCL kernel `conv`                   convolution.py:228-246
 *   ro_conv_xy  OpenCL kernel `conv_xy_origin_filters`  convolution.py:320-340
 *   ro_conv_z   OpenCL kernel `conv_z`                  convolution.py:344-359
 *   ro_update   PoseCellNetwork.update                  posecell_network.py:326-353
 *               (host control scalars are inputs, computed as the reference does)
 *   ro_vt_*     ViewTemplate.match / first argmin      view_templates.py:16-28, 63-75
 * The periodic wrap is taken modulo the grid (the reference's padded buffers).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define FL 7
#define HALF 3

static inline int wrapi(int v, int n) {
    int r = v % n;
    return r < 0 ? r + n : r;
}

int ro_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* bench.py's cpu_baseline picks the thread count (OMP_NUM_THREADS or the affinity
 * mask's size, whichever runs faster on the box) */
void ro_set_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

void ro_conv3d(const double* P, const double* K, double* out, int X, int Y, int TH) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < X; ++i)
        for (int j = 0; j < Y; ++j)
            for (int k = 0; k < TH; ++k) {
                double sum = 0;
                for (int x = 0; x < FL; ++x) {
                    const int ii = wrapi(i + x - HALF, X);
                    for (int y = 0; y < FL; ++y) {
                        const int jj = wrapi(j + y - HALF, Y);
                        const double* row = P + ((size_t)ii * Y + jj) * TH;
                        const double* kr = K + (x * FL + y) * FL;
                        for (int z = 0; z < FL; ++z) sum += row[wrapi(k + z - HALF, TH)] * kr[z];
                    }
                }
                out[((size_t)i * Y + j) * TH + k] = sum;
            }
}

/* F: (7, 7, TH) C order, F[x][y][k] */
void ro_conv_xy(const double* P, const int* ox, const int* oy, const double* F, double* out,
                int X, int Y, int TH) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < X; ++i)
        for (int j = 0; j < Y; ++j)
            for (int k = 0; k < TH; ++k) {
                double sum = 0;
                for (int x = 0; x < FL; ++x) {
                    const int ii = wrapi(i + x - HALF + ox[k], X);
                    for (int y = 0; y < FL; ++y) {
                        const int jj = wrapi(j + y - HALF + oy[k], Y);
                        sum += P[((size_t)ii * Y + jj) * TH + k] * F[(x * FL + y) * TH + k];
                    }
                }
                out[((size_t)i * Y + j) * TH + k] = sum;
            }
}

void ro_conv_z(const double* P, const double* zf, double* out, int X, int Y, int TH) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < X; ++i)
        for (int j = 0; j < Y; ++j) {
            const double* row = P + ((size_t)i * Y + j) * TH;
            for (int k = 0; k < TH; ++k) {
                double sum = 0;
                for (int z = 0; z < FL; ++z) sum += row[wrapi(k + z - HALF, TH)] * zf[z];
                out[((size_t)i * Y + j) * TH + k] = sum;
            }
        }
}

/* One update (posecell_network.py:326-353).  P is updated in place; tmp has X*Y*TH
 * doubles.  The normalisation total is a plain sequential sum (numpy uses a
 * pairwise sum: results agree to rounding).  Returns the argmax in out_xyz. */
void ro_update(double* P, double* tmp, const double* K, double inhib, const int* ox,
               const int* oy, const double* F, const double* zf, int X, int Y, int TH,
               int* out_xyz) {
    const size_t n = (size_t)X * Y * TH;
    ro_conv3d(P, K, tmp, X, Y, TH);
    double total = 0;
#pragma omp parallel for reduction(+ : total) schedule(static)
    for (size_t e = 0; e < n; ++e) {
        double v = tmp[e];
        v = v < inhib ? 0.0 : v - inhib;
        tmp[e] = v;
        total += v;
    }
    if (total != 0) {
#pragma omp parallel for schedule(static)
        for (size_t e = 0; e < n; ++e) tmp[e] /= total;
    }
    ro_conv_xy(tmp, ox, oy, F, P, X, Y, TH);
#pragma omp parallel for schedule(static)
    for (size_t e = 0; e < n; ++e)
        if (P[e] < 0) P[e] = 0;
    ro_conv_z(P, zf, tmp, X, Y, TH);
    size_t best = 0;
    for (size_t e = 0; e < n; ++e) {
        double v = tmp[e] < 0 ? 0 : tmp[e];
        P[e] = v;
        if (v > P[best]) best = e;
    }
    out_xyz[2] = (int)(best % TH);
    out_xyz[1] = (int)((best / TH) % Y);
    out_xyz[0] = (int)(best / ((size_t)TH * Y));
}

/* ViewTemplate.match for uint8 data: min over o of sum((T[m+o+r] - Q[m+r]) & 0xFF) */
static uint64_t vt_score(const uint8_t* t, const uint8_t* q, int H, int W, int M) {
    uint64_t best = UINT64_MAX;
    for (int o = -(M - 1); o <= M - 1; ++o) {
        uint64_t acc = 0;
        for (int r = M; r < H - M; ++r) {
            const uint8_t* a = t + (size_t)(r + o) * W;
            const uint8_t* b = q + (size_t)r * W;
            for (int c = 0; c < W; ++c) acc += (uint8_t)(a[c] - b[c]);
        }
        if (acc < best) best = acc;
    }
    return H - 2 * M > 0 ? best : 0;
}

void ro_vt_scores(const uint8_t* lib, int64_t T, const uint8_t* q, int H, int W, int M,
                  uint64_t* out) {
#pragma omp parallel for schedule(static)
    for (int64_t t = 0; t < T; ++t) out[t] = vt_score(lib + (size_t)t * H * W, q, H, W, M);
}

/* first argmin per query over a frozen library */
void ro_vt_best(const uint8_t* lib, int64_t T, const uint8_t* queries, int nq, int H, int W,
                int M, uint64_t* best_score, int64_t* best_index) {
    for (int i = 0; i < nq; ++i) {
        const uint8_t* q = queries + (size_t)i * H * W;
        uint64_t bs = UINT64_MAX;
        int64_t bi = -1;
#pragma omp parallel
        {
            uint64_t ls = UINT64_MAX;
            int64_t li = -1;
#pragma omp for schedule(static) nowait
            for (int64_t t = 0; t < T; ++t) {
                const uint64_t s = vt_score(lib + (size_t)t * H * W, q, H, W, M);
                if (s < ls || (s == ls && t < li)) {
                    ls = s;
                    li = t;
                }
            }
#pragma omp critical
            if (li >= 0 && (ls < bs || (ls == bs && li < bi))) {
                bs = ls;
                bi = li;
            }
        }
        best_score[i] = bs;
        best_index[i] = bi;
    }
}
