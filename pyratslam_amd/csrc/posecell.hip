// Pose-cell network step on MI355X (gfx950).
//
// Replaces PoseCellNetwork.update (/root/reference/ratslam/posecell_network.py:326-353)
// and the three OpenCL kernels it drives through Convolution.conv_im
// (convolution.py:228-246 `conv`, :320-340 `conv_xy_origin_filters`,
// :344-359 `conv_z`) plus the host-side numpy passes between them.
//
// Device layout: the volume is stored layer-major, P[th][x][y] (y fastest), so
// each theta layer -- the unit the path-integration shift acts on -- is one
// contiguous periodic 2-D image.  The reference's C-order (x, y, th) appears
// only at the boundary (rs_pc_read/write) and in the argmax tie-break index.
//
// One update() = two kernels on one stream:
//   pc_excite : 3-D DoG excitation as the exact rank-2 separable form
//               (ge^3 - gi^3)*scale, three 7-tap passes per Gaussian staged in
//               LDS, fused with the global inhibition relu(v - 0.2) and a
//               per-block float64 partial sum (normalisation total).
//   pc_path   : sums the partials (-> total), per-layer shifted 7x7 filter
//               (path integration), clamp, 7-tap theta filter, clamp, divide by
//               total, write the new state, fused argmax (first max in the
//               reference's C order) via a packed 64-bit atomicMax.
// max(conv(Q/t), 0) == max(conv(Q), 0)/t for t > 0, so the normalisation is
// applied once, at the end of the step.
#include <type_traits>
#include <utility>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <limits>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "rs_common.h"

namespace {

constexpr int FL = RS_FILTER_LEN;  // 7 taps
constexpr int HALF = FL / 2;       // 3
constexpr int NT = 256;            // threads per block (4 waves)
constexpr int FT = FL * FL;        // 49 taps of a 2-D filter

template <typename T>
struct SepKernel {
    T ge[FL];
    T gi[FL];
    T scale;
    T inhib;
};

// The normalisation P /= total (posecell_network.py:343-345).  float32: a product with
// the reciprocal of the total, rounded once from double (within an ulp of the division;
// one VALU op per value); where that reciprocal is not a finite float (a total below
// about 2.9e-39) each value is divided instead.  float64: the division, as the reference.
// A zero total leaves the volume as it is (:344).
template <typename T>
struct PcNorm;
template <>
struct PcNorm<float> {
    float r, t;
    bool div;
    __device__ PcNorm(float r_, float t_, bool div_) : r(r_), t(t_), div(div_) {}
    __device__ explicit PcNorm(double tot) {
        const float rf = (float)(tot != 0.0 ? 1.0 / tot : 1.0);
        // wave-uniform (every lane formed the same total): a scalar branch below, so the
        // division is never speculated into the common path
        div = __builtin_amdgcn_readfirstlane((int)!__builtin_isfinite(rf)) != 0;
        r = div ? 1.0f : rf;
        t = div ? (float)tot : 1.0f;
    }
    __device__ float operator()(float x) const {
        float y = x * r;
        if (div) {
            asm volatile("" ::: "memory");
            y = x / t;
        }
        return y;
    }
    template <int N>
    __device__ void operator()(float (&p)[N]) const {
        if (div) {
            asm volatile("" ::: "memory");
#pragma unroll
            for (int q = 0; q < N; ++q) p[q] = p[q] / t;
        } else {
#pragma unroll
            for (int q = 0; q < N; ++q) p[q] = p[q] * r;
        }
    }
};
template <>
struct PcNorm<double> {
    double t;
    __device__ explicit PcNorm(double tot) : t(tot != 0.0 ? tot : 1.0) {}
    __device__ double operator()(double x) const { return x / t; }
};

// Per-step control of the path-integration kernel: inline by value (one launch
// carries its step's shifts, filter rows and theta filter; no copy, no extra
// dependency) when TH <= CTL_INLINE_MAX, else pointers into a device ring.
constexpr int CTL_INLINE_MAX = 128;
struct PcCtlInline {     // single update(): the launch carries the control (~700 B kernarg)
    short iox[CTL_INLINE_MAX];
    short ioy[CTL_INLINE_MAX];
    unsigned char ifi[CTL_INLINE_MAX];
    double izf[FL];
    // the union of the step's per-layer shifted windows (column form, whole theta
    // extent: every block holds every layer, so it is the same for all blocks):
    // smallest centred shifts and the union's extent in cells, formed on the host
    // (make_ctl_inline) so the path kernel issues its window loads first thing
    short umx, umy, uwx, uwy;
};
struct PcCtlRing {       // batched run(): one record per step, uploaded once per batch
    const int* ox;
    const int* oy;
    const int* f;
    const double* zf;
};

__device__ inline int ctl_ox(const PcCtlInline& c, int L) { return c.iox[L]; }
__device__ inline int ctl_oy(const PcCtlInline& c, int L) { return c.ioy[L]; }
__device__ inline int ctl_fi(const PcCtlInline& c, int L) { return c.ifi[L]; }
__device__ inline double ctl_zf(const PcCtlInline& c, int z) { return c.izf[z]; }
__device__ inline int ctl_ox(const PcCtlRing& c, int L) { return c.ox[L]; }
__device__ inline int ctl_oy(const PcCtlRing& c, int L) { return c.oy[L]; }
__device__ inline int ctl_fi(const PcCtlRing& c, int L) { return c.f[L]; }
__device__ inline double ctl_zf(const PcCtlRing& c, int z) { return c.zf[z]; }

// float32 argmax: one packed key per block, max-reduced into slot b % RES_SLOTS;
// pc_res_export takes each step's max.  256 slots: one block per slot on the
// column and rows grids (with 8 slots, 32 contending 64-bit atomics per address
// held each step's end back: 64x64x36 13.35 -> 12.32 us per batched step,
// 128x128x72 27.7 -> 26.8, tools/pc_ab.py).
constexpr int RES_SLOTS = 256;
// No step's packed key is ever 0: float32 keys are (value bits << 32 | ~lin) and
// float64 keys ~lin, with lin < X*Y*TH < 2^32 - 1 (rs_pc_create).  The host writes
// RES_NONE into each step's result word before the launch and refuses a result
// still holding it after the stream has synchronised.
constexpr unsigned long long RES_NONE = 0ull;
// Step outputs are >= 0 or NaN (every step ends in a clamp), so the value bits order
// like the values (-0 taken as +0); every NaN is given one bit pattern above +inf, so
// that, as in numpy's argmax, a NaN beats every number and the first NaN wins.
__device__ inline unsigned long long argmax_key(float v, unsigned lin) {
    const unsigned bits = v != v ? 0x7FC00000u : v == 0.f ? 0u : __float_as_uint(v);  // -0 as +0
    return ((unsigned long long)bits << 32) | (0xFFFFFFFFu - lin);
}
// The clamps P[P < 0] = 0 (posecell_network.py:300,314): as the reference, a NaN stays
// a NaN (x > 0 ? x : 0 would zero it)
template <typename T>
__device__ inline T pc_clamp(T x) {
    return x < T(0) ? T(0) : x;
}
// The same order for (value, index) pairs (float64 steps, get_pc_max): a NaN beats every
// number, ties and NaNs among themselves go to the lower index; start from (-inf, ~0u).
template <typename T>
__device__ inline bool pc_better(T v, unsigned l, T bv, unsigned bl) {
    const bool vn = v != v, bn = bv != bv;
    return vn ? (!bn || l < bl) : (!bn && (v > bv || (v == bv && l < bl)));
}

// Phase-stamp hooks, empty in the library.  tools/pc_probe.hip defines them (a
// per-block s_memrealtime stamp) before it includes this file.
#ifndef PC_STAMP
#define PC_STAMP(kid, sid) \
    do {                   \
    } while (0)
#endif
#ifndef PC_STAMPW
#define PC_STAMPW(kid) \
    do {               \
    } while (0)
#endif

// A step's small result words (the normalisation partials, the argmax slots zeroed
// for the path kernel) stored write-through: an agent-scope relaxed atomic store is a
// plain store with sc1 on gfx950, so the line leaves the XCD's L2 at once and the
// kernel ends with nothing of these left dirty to write back at its boundary
// (tools/pc_ab.py, 5 rounds: 16.65 -> 16.49 us per 128x128x72 step, 11.41 -> 11.18 us
// per 64x64x36 step).
template <typename V>
__device__ inline void st_wt(V* p, V v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Tile shapes (output cells per block = BK layers x BX rows x BY cols).
constexpr int EX_BX = 8, EX_BY = 16, EX_BK = 4;
constexpr int PI_BX = 8, PI_BY = 16, PI_BK = 4;

// Deterministic block sum of one double per thread (same value returned to all).
__device__ inline double block_sum(double v, double* s_red) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) s_red[w] = v;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) t += s_red[i];
    __syncthreads();
    return t;
}

// ---------------------------------------------------------------------------
// Kernel 1: excitation (3-D DoG, separable) + global inhibition + partial sums
// posecell_network.py:336-343 (conv -> inhibit -> sum)
// ---------------------------------------------------------------------------
template <typename T, int BX, int BY, int BK>
__global__ __launch_bounds__(NT) void pc_excite_kernel(const T* __restrict__ P, T* __restrict__ Q,
                                                        double* __restrict__ part,
                                                        unsigned long long* __restrict__ res_slot,
                                                        int X, int Y, int TH, SepKernel<T> k) {
    constexpr int HX = BX + 2 * HALF, HY = BY + 2 * HALF, HK = BK + 2 * HALF;
    __shared__ T s_in[HK * HX * HY];
    __shared__ T s_ey[HK * HX * BY];
    __shared__ T s_iy[HK * HX * BY];
    __shared__ T s_exy[HK * BX * BY];
    __shared__ T s_ixy[HK * BX * BY];
    __shared__ double s_red[NT / 64];

    const int tid = threadIdx.x;
    const int j0 = blockIdx.x * BY, i0 = blockIdx.y * BX, k0 = blockIdx.z * BK;
    if (res_slot != nullptr && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0)
        for (int i = tid; i < RES_SLOTS; i += NT) st_wt(&res_slot[i], 0ull);  // this step's path kernel max-reduces into them

    for (int idx = tid; idx < HK * HX * HY; idx += NT) {
        const int kk = idx / (HX * HY);
        const int rem = idx - kk * (HX * HY);
        const int a = rem / HY, b = rem - a * HY;
        const int L = rs::wrapi(k0 - HALF + kk, TH);
        const int r = rs::wrapi(i0 - HALF + a, X);
        const int c = rs::wrapi(j0 - HALF + b, Y);
        s_in[idx] = P[((size_t)L * X + r) * Y + c];
    }
    __syncthreads();

    // pass along y (contiguous axis)
    for (int idx = tid; idx < HK * HX * BY; idx += NT) {
        const int row = idx / BY, j = idx - row * BY;
        const T* src = s_in + row * HY + j;
        T e = 0, g = 0;
#pragma unroll
        for (int t = 0; t < FL; ++t) {
            const T v = src[t];
            e += k.ge[t] * v;
            g += k.gi[t] * v;
        }
        s_ey[idx] = e;
        s_iy[idx] = g;
    }
    __syncthreads();

    // pass along x
    for (int idx = tid; idx < HK * BX * BY; idx += NT) {
        const int kk = idx / (BX * BY);
        const int rem = idx - kk * (BX * BY);
        const int i = rem / BY, j = rem - i * BY;
        const int base = (kk * HX + i) * BY + j;
        T e = 0, g = 0;
#pragma unroll
        for (int t = 0; t < FL; ++t) {
            e += k.ge[t] * s_ey[base + t * BY];
            g += k.gi[t] * s_iy[base + t * BY];
        }
        s_exy[idx] = e;
        s_ixy[idx] = g;
    }
    __syncthreads();

    // pass along theta, then relu(v - inhib) (posecell_network.py:339-340)
    double sum = 0.0;
    for (int idx = tid; idx < BK * BX * BY; idx += NT) {
        const int kq = idx / (BX * BY);
        const int rem = idx - kq * (BX * BY);
        const int i = rem / BY, j = rem - i * BY;
        const int gk = k0 + kq, gi = i0 + i, gj = j0 + j;
        if (gk < TH && gi < X && gj < Y) {
            T e = 0, g = 0;
#pragma unroll
            for (int t = 0; t < FL; ++t) {
                e += k.ge[t] * s_exy[idx + t * BX * BY];
                g += k.gi[t] * s_ixy[idx + t * BX * BY];
            }
            const T v = (e - g) * k.scale;
            const T q = (v < k.inhib) ? T(0) : v - k.inhib;
            Q[((size_t)gk * X + gi) * Y + gj] = q;
            sum += (double)q;
        }
    }
    sum = block_sum(sum, s_red);
    if (tid == 0) st_wt(&part[(blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x], sum);
}

// ---------------------------------------------------------------------------
// Kernel 2: path integration (posecell_network.py:252-314) + normalisation
// (:343-345, applied at the end) + argmax (:317-319)
// ---------------------------------------------------------------------------
template <typename T, int BX, int BY, int BK, typename CTL>
__global__ __launch_bounds__(NT) void pc_path_kernel(
    const T* __restrict__ Q, T* __restrict__ P, const double* __restrict__ part, int npart,
    const T* __restrict__ filt, CTL ctl, unsigned long long* __restrict__ res_slot,
    T* __restrict__ bmax, unsigned* __restrict__ bidx, int X, int Y, int TH) {
    constexpr int HX = BX + 2 * HALF, HY = BY + 2 * HALF, HK = BK + 2 * HALF;
    __shared__ T s_win[HK * HX * HY];
    __shared__ T s_r[HK * BX * BY];
    __shared__ T s_f[HK * FT];
    __shared__ int s_ox[HK], s_oy[HK];
    __shared__ T s_zf[FL];
    __shared__ double s_red[NT / 64];
    __shared__ T s_bv[NT / 64];
    __shared__ unsigned s_bl[NT / 64];

    const int tid = threadIdx.x;
    const int j0 = blockIdx.x * BY, i0 = blockIdx.y * BX, k0 = blockIdx.z * BK;

    // normalisation total = sum of the excitation kernel's partials (fixed order)
    double tot = 0.0;
    for (int i = tid; i < npart; i += NT) tot += part[i];
    tot = block_sum(tot, s_red);

    if (tid < HK) {
        const int L = rs::wrapi(k0 - HALF + tid, TH);
        s_ox[tid] = ctl_ox(ctl, L);
        s_oy[tid] = ctl_oy(ctl, L);
    }
    if (tid < FL) s_zf[tid] = (T)ctl_zf(ctl, tid);
    for (int idx = tid; idx < HK * FT; idx += NT) {
        const int kk = idx / FT, tap = idx - kk * FT;
        const int L = rs::wrapi(k0 - HALF + kk, TH);
        s_f[idx] = filt[ctl_fi(ctl, L) * FT + tap];
    }
    __syncthreads();

    // shifted window of every layer this tile (plus theta halo) needs
    for (int idx = tid; idx < HK * HX * HY; idx += NT) {
        const int kk = idx / (HX * HY);
        const int rem = idx - kk * (HX * HY);
        const int a = rem / HY, b = rem - a * HY;
        const int L = rs::wrapi(k0 - HALF + kk, TH);
        const int r = rs::wrapi(i0 - HALF + s_ox[kk] + a, X);
        const int c = rs::wrapi(j0 - HALF + s_oy[kk] + b, Y);
        s_win[idx] = Q[((size_t)L * X + r) * Y + c];
    }
    __syncthreads();

    // per-layer 7x7 correlation with the layer's filter, clamp (:300)
    for (int idx = tid; idx < HK * BX * BY; idx += NT) {
        const int kk = idx / (BX * BY);
        const int rem = idx - kk * (BX * BY);
        const int i = rem / BY, j = rem - i * BY;
        const T* w = s_win + (kk * HX + i) * HY + j;
        const T* f = s_f + kk * FT;
        T acc = 0;
#pragma unroll
        for (int x = 0; x < FL; ++x)
#pragma unroll
            for (int y = 0; y < FL; ++y) acc += w[x * HY + y] * f[x * FL + y];
        s_r[idx] = pc_clamp(acc);
    }
    __syncthreads();

    // theta filter, clamp (:310-314), normalise, store, argmax
    T bv = -std::numeric_limits<T>::infinity();
    unsigned bl = 0xFFFFFFFFu;
    const PcNorm<T> nrm(tot);
    for (int idx = tid; idx < BK * BX * BY; idx += NT) {
        const int kq = idx / (BX * BY);
        const int rem = idx - kq * (BX * BY);
        const int i = rem / BY, j = rem - i * BY;
        const int gk = k0 + kq, gi = i0 + i, gj = j0 + j;
        if (gk < TH && gi < X && gj < Y) {
            T acc = 0;
#pragma unroll
            for (int z = 0; z < FL; ++z) acc += s_r[idx + z * BX * BY] * s_zf[z];
            T v = pc_clamp(acc);
            v = nrm(v);
            P[((size_t)gk * X + gi) * Y + gj] = v;
            const unsigned lin = ((unsigned)gi * Y + gj) * TH + gk;
            if (pc_better(v, lin, bv, bl)) {
                bv = v;
                bl = lin;
            }
        }
    }
    {
        // wave argmax, then block argmax: one (value, index) partial per block,
        // reduced per step by pc_argmax_steps (no same-address atomics)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const T ov = __shfl_xor(bv, off);
            const unsigned ol = __shfl_xor(bl, off);
            if (pc_better(ov, ol, bv, bl)) {
                bv = ov;
                bl = ol;
            }
        }
        if ((tid & 63) == 0) {
            s_bv[tid >> 6] = bv;
            s_bl[tid >> 6] = bl;
        }
        __syncthreads();
        if (tid == 0) {
            for (int w = 1; w < NT / 64; ++w)
                if (pc_better(s_bv[w], s_bl[w], bv, bl)) {
                    bv = s_bv[w];
                    bl = s_bl[w];
                }
            const int b = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
            if constexpr (sizeof(T) == 4) {
                atomicMax(res_slot + (b & (RES_SLOTS - 1)), argmax_key((float)bv, bl));
            } else {
                bmax[b] = bv;
                bidx[b] = bl;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Row-tiled forms (the fast path for Y <= 128).  A block (512 threads = 8
// waves) owns BK layers x BX rows x the whole Y extent; lanes own columns, so
// the periodic wrap in y is a 3-cell LDS halo and no hot loop divides.  The
// wrapped layer/row index of every halo row is computed once per block (one
// modulo per thread) into LDS; then every global load of a wave is issued
// unconditionally (column clamped) before the first use, so each phase costs
// one memory round trip.  One halo layer per wave for the stencil passes, which
// are register-blocked per column (a lane walks the x direction).
// ---------------------------------------------------------------------------
// Row-tile shape: BK layers x BX rows per block, BK + 6 = BK * BX waves (one
// window layer per wave in the y/x passes, one output row per wave in the theta
// pass).  6 x 2 (12 waves) keeps the 64x64x36 grid at 192 blocks, one per CU:
// 2 x 4 (8 waves) made 288 blocks, and the CUs that ran two of them set the
// kernels' span (path 8.7 -> 5.2 us, excitation 4.6 -> 3.8 us first block start
// to last block end; it also re-evaluates fewer halo rows and layers per output).
constexpr int RT_BX = 2, RT_BK = 6, RT_NW = RT_BK + 6, RT_NT = 64 * RT_NW;
constexpr int RT_NFMAX = 8;  // filter tables up to this size are preloaded whole

template <int NW>
__device__ inline double block_sum_w(double v, double* s_red) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < NW; ++i) t += s_red[i];
    return t;
}

// Block barrier for LDS traffic only: waits for this wave's LDS operations, not
// for its global stores (a __syncthreads fence would drain those too).
__device__ inline void co_lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Wave-wide reductions by DPP row operations instead of ds_bpermute shuffles (six
// dependent LDS round trips each): within every 16-lane row by quad_perm xor 1,
// xor 2, row_half_mirror and row_mirror, then over the 4 rows by readlane.  Every
// lane computes the same additions on the same two operands at each step, so the
// result is identical in all lanes (wave-uniform) and deterministic.
template <int CTRL>
__device__ inline unsigned long long co_dpp64(unsigned long long v) {
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)v, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(v >> 32), CTRL, 0xF, 0xF, false);
    return ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
}
__device__ inline unsigned long long co_readlane64(unsigned long long v, int l) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), l);
    return ((unsigned long long)hi << 32) | lo;
}
__device__ inline double co_wave_sum(double v) {
    v += __longlong_as_double((long long)co_dpp64<0xB1>((unsigned long long)__double_as_longlong(v)));
    v += __longlong_as_double((long long)co_dpp64<0x4E>((unsigned long long)__double_as_longlong(v)));
    v += __longlong_as_double((long long)co_dpp64<0x141>((unsigned long long)__double_as_longlong(v)));
    v += __longlong_as_double((long long)co_dpp64<0x140>((unsigned long long)__double_as_longlong(v)));
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    return (__longlong_as_double((long long)co_readlane64(b, 0)) +
            __longlong_as_double((long long)co_readlane64(b, 16))) +
           (__longlong_as_double((long long)co_readlane64(b, 32)) +
            __longlong_as_double((long long)co_readlane64(b, 48)));
}
__device__ inline unsigned long long co_wave_max(unsigned long long v) {
    v = max(v, co_dpp64<0xB1>(v));
    v = max(v, co_dpp64<0x4E>(v));
    v = max(v, co_dpp64<0x141>(v));
    v = max(v, co_dpp64<0x140>(v));
    return max(max(co_readlane64(v, 0), co_readlane64(v, 16)),
               max(co_readlane64(v, 32), co_readlane64(v, 48)));
}

template <typename T, int YP>
__global__ __launch_bounds__(RT_NT) void pc_excite_rows(const T* __restrict__ P, T* __restrict__ Q,
                                                         double* __restrict__ part,
                                                         unsigned long long* __restrict__ res_slot,
                                                         int X, int Y, int TH, SepKernel<T> k) {
    constexpr int BX = RT_BX, BK = RT_BK, HX = BX + 2 * HALF, HK = BK + 2 * HALF, NW = RT_NW;
    constexpr int RW = YP + 2 * HALF, JC = YP / 64, NR = HK * HX, RPW = NR / NW;
    static_assert(NR % NW == 0 && HK == NW && BK * BX == NW, "row tile / wave mapping");
    __shared__ T s_in[NR * RW];
    __shared__ T s_e[HK * BX * YP];
    __shared__ T s_i[HK * BX * YP];
    __shared__ int s_row[NR];
    __shared__ double s_red[NW];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int i0 = blockIdx.x * BX, k0 = blockIdx.y * BK;
    PC_STAMP(0, 0);
    if (res_slot != nullptr && blockIdx.x == 0 && blockIdx.y == 0)
        for (int i = tid; i < RES_SLOTS; i += blockDim.x) st_wt(&res_slot[i], 0ull);  // this step's path kernel max-reduces into them
    if (tid < NR) {
        const int kk = tid / HX, a = tid - kk * HX;
        s_row[tid] = rs::wrapi(k0 - HALF + kk, TH) * X + rs::wrapi(i0 - HALF + a, X);
    }
    co_lds_barrier();

    T v[RPW][JC];
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        const T* src = P + (size_t)s_row[wave + NW * q] * Y;
#pragma unroll
        for (int jc = 0; jc < JC; ++jc) v[q][jc] = src[min(lane + 64 * jc, Y - 1)];
    }
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        T* dst = s_in + (wave + NW * q) * RW;
#pragma unroll
        for (int jc = 0; jc < JC; ++jc) {
            const int c = lane + 64 * jc;
            if (c < Y) {
                dst[HALF + c] = v[q][jc];
                if (c < HALF) dst[HALF + Y + c] = v[q][jc];
                if (c >= Y - HALF) dst[c - (Y - HALF)] = v[q][jc];
            }
        }
    }
    co_lds_barrier();
    PC_STAMP(0, 1);

    // y pass (7 taps along the row) then x pass (7 rows) in registers; one layer per wave
    {
        const int kk = wave;
#pragma unroll
        for (int jc = 0; jc < JC; ++jc) {
            const int j = lane + 64 * jc;
            if (j >= Y) continue;
            T ey[HX], iy[HX];
#pragma unroll
            for (int a = 0; a < HX; ++a) {
                const T* rw = s_in + (kk * HX + a) * RW + j;
                T e = 0, g = 0;
#pragma unroll
                for (int t = 0; t < FL; ++t) {
                    const T x = rw[t];
                    e += k.ge[t] * x;
                    g += k.gi[t] * x;
                }
                ey[a] = e;
                iy[a] = g;
            }
#pragma unroll
            for (int i = 0; i < BX; ++i) {
                T e = 0, g = 0;
#pragma unroll
                for (int t = 0; t < FL; ++t) {
                    e += k.ge[t] * ey[i + t];
                    g += k.gi[t] * iy[i + t];
                }
                s_e[(kk * BX + i) * YP + j] = e;
                s_i[(kk * BX + i) * YP + j] = g;
            }
        }
    }
    co_lds_barrier();
    PC_STAMP(0, 2);

    // theta pass + relu(v - inhib) (posecell_network.py:339-340) + partial sum; one row per wave
    double sum = 0.0;
    {
        const int kq = wave / BX, i = wave - kq * BX;
        const int gk = k0 + kq, gi = i0 + i;
        if (gk < TH && gi < X) {
#pragma unroll
            for (int jc = 0; jc < JC; ++jc) {
                const int j = lane + 64 * jc;
                if (j >= Y) continue;
                T e = 0, g = 0;
#pragma unroll
                for (int t = 0; t < FL; ++t) {
                    e += k.ge[t] * s_e[((kq + t) * BX + i) * YP + j];
                    g += k.gi[t] * s_i[((kq + t) * BX + i) * YP + j];
                }
                const T val = (e - g) * k.scale;
                const T q = (val < k.inhib) ? T(0) : val - k.inhib;
                // write-through (sc1): nothing dirty left for the kernel's end to write back
                st_wt(&Q[((size_t)gk * X + gi) * Y + j], q);
                sum += (double)q;
            }
        }
    }
    sum = co_wave_sum(sum);
    if (lane == 0) s_red[wave] = sum;
    co_lds_barrier();  // the Q stores drain meanwhile
    if (tid == 0) {
        double t = 0.0;
#pragma unroll
        for (int w = 0; w < NW; ++w) t += s_red[w];
        st_wt(&part[blockIdx.y * gridDim.x + blockIdx.x], t);
    }
    PC_STAMP(0, 3);
}

template <typename T, int YP, typename CTL>
__global__ __launch_bounds__(RT_NT) void pc_path_rows(
    const T* __restrict__ Q, T* __restrict__ P, const double* __restrict__ part, int npart,
    const T* __restrict__ filt, int nf, CTL ctl, unsigned long long* __restrict__ res_slot,
    T* __restrict__ bmax, unsigned* __restrict__ bidx, int X, int Y, int TH) {
    constexpr int BX = RT_BX, BK = RT_BK, HX = BX + 2 * HALF, HK = BK + 2 * HALF, NW = RT_NW;
    constexpr int RW = YP + 2 * HALF, JC = YP / 64, NR = HK * HX, RPW = NR / NW;
    constexpr int NPP = 4;  // normalisation partials held per thread (npart <= NPP * RT_NT)
    static_assert(NR % NW == 0 && HK == NW && BK * BX == NW, "row tile / wave mapping");
    __shared__ T s_win[NR * RW];
    __shared__ T s_r[HK * BX * YP];
    __shared__ int s_row[NR];
    __shared__ int s_oy[HK], s_fi[HK];
    __shared__ double s_red[NW];
    __shared__ T s_bv[NW];
    __shared__ unsigned s_bl[NW];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    (void)nf;  // filter indices are validated on the host (pc_check_ctl)
    const int i0 = blockIdx.x * BX, k0 = blockIdx.y * BK;
    PC_STAMP(1, 0);

    // the block's control, and the row table straight from it (one barrier)
    if (tid < HK) {
        const int L = rs::wrapi(k0 - HALF + tid, TH);
        s_oy[tid] = rs::wrapi(ctl_oy(ctl, L), Y);
        s_fi[tid] = ctl_fi(ctl, L);
    }
    if (tid < NR) {
        const int kk = tid / HX, a = tid - kk * HX, L = rs::wrapi(k0 - HALF + kk, TH);
        // shifts may exceed the grid (vtrans large)
        s_row[tid] = L * X + rs::wrapi(i0 - HALF + a + rs::wrapi(ctl_ox(ctl, L), X), X);
    }
    co_lds_barrier();
    PC_STAMP(1, 1);
    PC_STAMP(1, 2);

    // shifted window rows: s_win[kk][a][HALF + d] = Q[L][(i0-3+a+ox) % X][(d + oy) % Y]
    T v[RPW][JC];
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        const T* src = Q + (size_t)s_row[wave + NW * q] * Y;
#pragma unroll
        for (int jc = 0; jc < JC; ++jc) v[q][jc] = src[min(lane + 64 * jc, Y - 1)];
    }
    // this wave's layer filter and the normalisation partials (reduced only at the
    // end), issued behind the window loads: a barrier waits for every load in
    // flight, so nothing global is loaded before the control barriers above
    T f[FT];
    {
        const T* fsrc = filt + (size_t)s_fi[wave] * FT;
#pragma unroll
        for (int t = 0; t < FT; ++t) f[t] = fsrc[t];
    }
    double pt[NPP];
#pragma unroll
    for (int u = 0; u < NPP; ++u) {
        const int i = tid + u * RT_NT;
        pt[u] = part[min(i, npart - 1)];  // unconditional (a guarded load got its wait hoisted)
    }
    double pextra = 0.0;  // npart beyond NPP * RT_NT (huge grids)
    for (int i = tid + NPP * RT_NT; i < npart; i += RT_NT) pextra += part[i];
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
        const int row = wave + NW * q;
        const int oy = s_oy[row / HX];
        T* dst = s_win + row * RW;
#pragma unroll
        for (int jc = 0; jc < JC; ++jc) {
            const int c = lane + 64 * jc;
            if (c >= Y) continue;
            int d = c - oy;
            if (d < 0) d += Y;
            dst[HALF + d] = v[q][jc];
            if (d < HALF) dst[HALF + Y + d] = v[q][jc];
            if (d >= Y - HALF) dst[d - (Y - HALF)] = v[q][jc];
        }
    }
    co_lds_barrier();
    PC_STAMP(1, 3);

    // 7x7 per-layer correlation (:273-274), register-blocked over the BX rows, clamp (:300)
    {
        const int kk = wave;
#pragma unroll
        for (int jc = 0; jc < JC; ++jc) {
            const int j = lane + 64 * jc;
            if (j >= Y) continue;
            T acc[BX];
#pragma unroll
            for (int i = 0; i < BX; ++i) acc[i] = 0;
#pragma unroll
            for (int a = 0; a < HX; ++a) {
                T w[FL];
                const T* rw = s_win + (kk * HX + a) * RW + j;
#pragma unroll
                for (int t = 0; t < FL; ++t) w[t] = rw[t];
#pragma unroll
                for (int i = 0; i < BX; ++i) {
                    const int x = a - i;
                    if (x < 0 || x >= FL) continue;
#pragma unroll
                    for (int t = 0; t < FL; ++t) acc[i] += w[t] * f[x * FL + t];
                }
            }
#pragma unroll
            for (int i = 0; i < BX; ++i) s_r[(kk * BX + i) * YP + j] = pc_clamp(acc[i]);
        }
    }
    // normalisation total (its loads were issued at entry): per thread, then per
    // wave by DPP, then over the waves through LDS behind the barrier that also
    // publishes s_r
    double tot = pextra;
#pragma unroll
    for (int u = 0; u < NPP; ++u) tot += tid + u * RT_NT < npart ? pt[u] : 0.0;
    tot = co_wave_sum(tot);
    if (lane == 0) s_red[wave] = tot;
    co_lds_barrier();
    tot = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) tot += s_red[w];
    PC_STAMP(1, 4);

    // theta filter (:310), clamp (:314), normalise (:343-345), store, argmax (:317-319):
    // float32 as the largest packed (value, ~index) key, float64 as value/index pairs
    T bv = -std::numeric_limits<T>::infinity();
    unsigned bl = 0xFFFFFFFFu;
    unsigned long long bk = 0ull;
    {
        const PcNorm<T> nrm(tot);
        const int kq = wave / BX, i = wave - kq * BX;
        const int gk = k0 + kq, gi = i0 + i;
        if (gk < TH && gi < X) {
#pragma unroll
            for (int jc = 0; jc < JC; ++jc) {
                const int j = lane + 64 * jc;
                if (j >= Y) continue;
                T acc = 0;
#pragma unroll
                for (int z = 0; z < FL; ++z) acc += s_r[((kq + z) * BX + i) * YP + j] * (T)ctl_zf(ctl, z);
                T val = pc_clamp(acc);
                val = nrm(val);
                st_wt(&P[((size_t)gk * X + gi) * Y + j], val);
                const unsigned lin = ((unsigned)gi * Y + j) * TH + gk;
                if constexpr (sizeof(T) == 4) {
                    bk = max(bk, argmax_key((float)val, lin));
                } else if (pc_better(val, lin, bv, bl)) {
                    bv = val;
                    bl = lin;
                }
            }
        }
    }
    const int b = blockIdx.y * gridDim.x + blockIdx.x;
    if constexpr (sizeof(T) == 4) {
        __shared__ unsigned long long s_bk[NW];
        bk = co_wave_max(bk);
        if (lane == 0) s_bk[wave] = bk;
        co_lds_barrier();
        if (tid == 0) {
            for (int w = 1; w < NW; ++w) bk = max(bk, s_bk[w]);
            atomicMax(res_slot + (b & (RES_SLOTS - 1)), bk);
        }
    } else {
        // block argmax -> one (value, index) partial per block (pc_argmax_steps reduces)
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const T ov = __shfl_xor(bv, off);
            const unsigned ol = __shfl_xor(bl, off);
            if (pc_better(ov, ol, bv, bl)) {
                bv = ov;
                bl = ol;
            }
        }
        if (lane == 0) {
            s_bv[wave] = bv;
            s_bl[wave] = bl;
        }
        co_lds_barrier();
        if (tid == 0) {
            for (int w = 1; w < NW; ++w)
                if (pc_better(s_bv[w], s_bl[w], bv, bl)) {
                    bv = s_bv[w];
                    bl = s_bl[w];
                }
            bmax[b] = bv;
            bidx[b] = bl;
        }
    }
    PC_STAMP(1, 5);
}

// ---------------------------------------------------------------------------
// Layer-streaming forms (large grids).  A block of WR x WC waves owns BXB = BX*WR
// rows x YT = 64*WC columns x KC layers of the output and walks its KC + 6
// input layers in order.  Per input layer only 2-D work is done (window load
// into double-buffered LDS, then the y and x passes or the 7x7 filter); the
// 7-tap theta pass runs on a 7-deep register ring of per-lane results, so the
// 2-D passes are evaluated (KC+6)/KC times per cell instead of the rows form's
// (BK+6)/BK = 4x.  Lane <-> column; each wave register-blocks BX rows.
// Window loads run ST_PF layers ahead of use (a 7-slot register ring, so the
// slot of every stage is a compile-time index of the 7-way unrolled layer loop).
// Every stage is straight-line: unconditional loads and LDS stores, and the
// outputs go to an LDS buffer written back after the loop, so the only
// vector-memory operations in the loop are the in-order window loads and the
// compiler's vmcnt wait at each stage covers just that stage's slot (a global
// store in flight makes it drain every prefetch).  The per-layer control
// (shifts, filter index) and the filter table are staged in LDS once per block.
// Tiles are numbered XCD-aware: dispatch is round-robin over the 8 XCDs, and
// XCD x takes a contiguous run of tiles, so neighbouring tiles' halo rows and
// layers meet in the same L2.
// ---------------------------------------------------------------------------
constexpr int ST_PF = 3;                  // window prefetch distance (layers)
// The streaming grids hold 1-2 blocks per CU, so occupancy buys nothing: let the
// scheduler spend registers on keeping LDS reads in flight (at the default
// occupancy target it serialises every ds_read behind an lgkmcnt(0)).
#define PC_ST_WAVES __attribute__((amdgpu_waves_per_eu(1, 2)))
constexpr int ST_MAXKC = 12;              // layers per block (outputs buffered in LDS)
constexpr int ST_MAXL = ST_MAXKC + 2 * 3 + ST_PF + 1;  // control entries staged in LDS
constexpr int ST_OUT_BYTES = 24 * 1024;   // LDS output buffer per block
// layers per block that fit the output buffer for a tile of bxb x yt cells of esz bytes
__host__ __device__ constexpr int st_maxkc(int esz, int bxb, int yt) {
    return ST_OUT_BYTES / (esz * bxb * yt) < ST_MAXKC ? ST_OUT_BYTES / (esz * bxb * yt) : ST_MAXKC;
}
constexpr int ST_FTP = 52;                // filter stride in LDS: 49 taps padded to 13 x 16 B
constexpr int NPP_MAX_BLOCKS = 4 * 512 * 64;
constexpr size_t ST_MIN_CELLS = 512 * 1024;  // default form: streamed from this grid size
constexpr int ST_DEF_BX = 2, ST_DEF_WR = 8, ST_DEF_WC = 1;  // default streaming tile (float32)
static_assert(ST_PF >= 1 && ST_PF < FL, "prefetch ring has 7 slots");

struct StreamGrid {  // tiles along x, y and theta chunks; layers per chunk
    int gx, gy, gz, KC;
};

__device__ inline int st_tile(int b, int nb) {
    if ((nb & 7) != 0) return b;
    return (b & 7) * (nb >> 3) + (b >> 3);
}

// Window loads.  Plain loads: hipcc counts them and places the waits.  (An
// earlier inline-asm form with hand-placed vmcnt waits is unsafe: hipcc treats an
// asm load's destination as written at the statement and may copy or reuse that
// register before the data lands.  It was the suspected cause of an illegal-address
// fault with two processes on one GPU; the plain form measures within 2%.)
template <typename T>
__device__ inline T st_load(const T* base, unsigned idx) {
    return base[idx];
}

// Excitation (posecell_network.py:336 -> convolution.py:228-246), inhibition
// (:339-340) and the normalisation partial sum (:343), streamed over layers.
template <typename T, int BX, int WR, int WC>
__global__ __launch_bounds__(64 * WR * WC) PC_ST_WAVES void pc_excite_stream(const T* __restrict__ P, T* __restrict__ Q,
                                                           double* __restrict__ part,
                                                           unsigned long long* __restrict__ res_slot,
                                                           int X, int Y, int TH, StreamGrid G,
                                                           SepKernel<T> k) {
    constexpr int NW = WR * WC, NT = 64 * NW, YT = 64 * WC, BXB = BX * WR;
    constexpr int HR = BXB + 2 * HALF, RW = YT + 2 * HALF, WN = HR * RW;
    constexpr int LPT = (WN + NT - 1) / NT;
    __shared__ T s_in[2][LPT * NT];  // padded: every thread stores every stage
    __shared__ T s_ye[2][HR * YT];
    __shared__ T s_yi[2][HR * YT];
    __shared__ T s_out[st_maxkc(sizeof(T), BXB, YT) * BXB * YT];
    __shared__ double s_red[NW];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int rg = wave % WR, col = (wave / WR) * 64 + lane;
    const int tile = st_tile(blockIdx.x, gridDim.x);
    const int bx = tile % G.gx, rest = tile / G.gx;
    const int i0 = bx * BXB, y0 = (rest % G.gy) * YT, k0 = (rest / G.gy) * G.KC;
    const int nL = min(G.KC, TH - k0) + 2 * HALF;
    const int gy = y0 + col;
    PC_STAMP(2, 0);
    if (res_slot != nullptr && blockIdx.x == 0)
        for (int i = tid; i < RES_SLOTS; i += blockDim.x) st_wt(&res_slot[i], 0ull);  // this step's path kernel max-reduces into them

    // window element e = (row r, col c) <-> P[L][(i0-3+r) % X][(y0-3+c) % Y]: the
    // in-layer offset is fixed over layers
    unsigned off[LPT];
#pragma unroll
    for (int u = 0; u < LPT; ++u) {
        const int e = min(tid + u * NT, WN - 1), r = e / RW, c = e - r * RW;
        off[u] = (unsigned)(rs::wrapi(i0 - HALF + r, X) * Y + rs::wrapi(y0 - HALF + c, Y));
    }
    const size_t lstride = (size_t)X * Y;
    T pre[FL][LPT];
#pragma unroll
    for (int d = 0; d < ST_PF; ++d) {
        const T* src = P + (size_t)rs::wrapi(k0 - HALF + d, TH) * lstride;
#pragma unroll
        for (int u = 0; u < LPT; ++u) pre[d][u] = st_load(src, off[u]);
    }

    T re[FL][BX], ri[FL][BX];
    double sum = 0.0;
    // software-pipelined over layers, one barrier per iteration: iteration it
    // stores window it+1, runs the y pass of layer it and the x / theta passes of
    // layer it-1 (its y pass landed before the previous barrier)
#pragma unroll
    for (int u = 0; u < LPT; ++u) s_in[0][tid + u * NT] = pre[0][u];
    {
        const T* src = P + (size_t)rs::wrapi(k0 - HALF + ST_PF, TH) * lstride;
#pragma unroll
        for (int u = 0; u < LPT; ++u) pre[ST_PF % FL][u] = st_load(src, off[u]);
    }
    __syncthreads();
    PC_STAMP(2, 1);
    for (int base = 0; base <= nL; base += FL) {
#pragma unroll
        for (int s = 0; s < FL; ++s) {
            const int it = base + s;
            if (it > nL) break;
            if (it < nL) {
                const int b = it & 1;
                // window it+1 (layers past the chunk are valid wrapped addresses: every
                // load is issued, so the counted waits stay in step)
#pragma unroll
                for (int u = 0; u < LPT; ++u) s_in[b ^ 1][tid + u * NT] = pre[(s + 1) % FL][u];
                {
                    const T* src = P + (size_t)rs::wrapi(k0 - HALF + it + 1 + ST_PF, TH) * lstride;
#pragma unroll
                    for (int u = 0; u < LPT; ++u) pre[(s + 1 + ST_PF) % FL][u] = st_load(src, off[u]);
                }
                // y pass of layer it: window rows rg, rg + WR, ... (both Gaussians share the loads)
                for (int r = rg; r < HR; r += WR) {
                    const T* rw = &s_in[b][r * RW + col];
                    T e = 0, g = 0;
#pragma unroll
                    for (int t = 0; t < FL; ++t) {
                        const T x = rw[t];
                        e += k.ge[t] * x;
                        g += k.gi[t] * x;
                    }
                    s_ye[b][r * YT + col] = e;
                    s_yi[b][r * YT + col] = g;
                }
            }
            if (it >= 1) {
                // x pass of layer it-1 (ring slot (s+6) % 7): this wave's BX rows,
                // register-blocked over the BX + 6 window rows
                const int b = (it - 1) & 1;
                T ye[BX + 2 * HALF], yi[BX + 2 * HALF];
#pragma unroll
                for (int a = 0; a < BX + 2 * HALF; ++a) {
                    ye[a] = s_ye[b][(rg * BX + a) * YT + col];
                    yi[a] = s_yi[b][(rg * BX + a) * YT + col];
                }
#pragma unroll
                for (int i = 0; i < BX; ++i) {
                    T e = 0, g = 0;
#pragma unroll
                    for (int t = 0; t < FL; ++t) {
                        e += k.ge[t] * ye[i + t];
                        g += k.gi[t] * yi[i + t];
                    }
                    re[(s + 6) % FL][i] = e;
                    ri[(s + 6) % FL][i] = g;
                }
                // theta pass for output layer o = it-7 over the ring (input o+t sits in
                // slot (s+t) % 7), relu(v - inhib), partial sum; the output waits in LDS
                if (it >= 2 * HALF + 1) {
                    const int o = it - 2 * HALF - 1;
#pragma unroll
                    for (int i = 0; i < BX; ++i) {
                        T e = 0, g = 0;
#pragma unroll
                        for (int t = 0; t < FL; ++t) {
                            e += k.ge[t] * re[(s + t) % FL][i];
                            g += k.gi[t] * ri[(s + t) % FL][i];
                        }
                        const T v = (e - g) * k.scale;
                        const T q = (v < k.inhib) ? T(0) : v - k.inhib;
                        s_out[(o * BXB + rg * BX + i) * YT + col] = q;
                        if (i0 + rg * BX + i < X && gy < Y) sum += (double)q;
                    }
                }
            }
            __syncthreads();
            if (it == 0) PC_STAMP(2, 2);
        }
    }
    PC_STAMP(2, 3);
    // write-back: each thread stores the cells it computed (its own LDS slots)
    for (int o = 0; o < nL - 2 * HALF; ++o)
#pragma unroll
        for (int i = 0; i < BX; ++i) {
            const int gi = i0 + rg * BX + i;
            if (gi < X && gy < Y)
                Q[((size_t)(k0 + o) * X + gi) * Y + gy] = s_out[(o * BXB + rg * BX + i) * YT + col];
        }
    sum = block_sum_w<NW>(sum, s_red);
    if (tid == 0) st_wt(&part[blockIdx.x], sum);
    PC_STAMP(2, 4);
}

// 49 filter taps from LDS (uniform address: broadcast reads, 16 B each for float)
template <typename T>
__device__ inline void st_filter(const T* __restrict__ src, T (&f)[FT]) {
    if constexpr (sizeof(T) == 4) {
        const float4* s4 = reinterpret_cast<const float4*>(src);
#pragma unroll
        for (int q = 0; q < ST_FTP / 4; ++q) {
            const float4 v = s4[q];
            if (4 * q + 0 < FT) f[4 * q + 0] = v.x;
            if (4 * q + 1 < FT) f[4 * q + 1] = v.y;
            if (4 * q + 2 < FT) f[4 * q + 2] = v.z;
            if (4 * q + 3 < FT) f[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (int t = 0; t < FT; ++t) f[t] = src[t];
    }
}

// Path integration (posecell_network.py:252-314): per-layer shifted 7x7 filter
// (:273 -> convolution.py:320-340), clamp (:300), 7-tap theta filter (:310 ->
// convolution.py:344-359), clamp (:314), normalisation by the excitation total
// (:343-345, applied at the end), fused argmax (:317-319), streamed over layers.
template <typename T, int BX, int WR, int WC, typename CTL>
__global__ __launch_bounds__(64 * WR * WC) PC_ST_WAVES void pc_path_stream(
    const T* __restrict__ Q, T* __restrict__ P, const double* __restrict__ part, int npart,
    const T* __restrict__ filt, int nf, CTL ctl, unsigned long long* __restrict__ res_slot,
    T* __restrict__ bmax, unsigned* __restrict__ bidx, int X, int Y, int TH, StreamGrid G) {
    constexpr int NW = WR * WC, NT = 64 * NW, YT = 64 * WC, BXB = BX * WR;
    constexpr int HR = BXB + 2 * HALF, RW = YT + 2 * HALF, WN = HR * RW;
    constexpr int LPT = (WN + NT - 1) / NT;
    constexpr int NPP = 4;  // normalisation partials per thread (npart <= NPP * NT)
    __shared__ T s_win[2][LPT * NT];  // padded: every thread stores every stage
    __shared__ T s_out[st_maxkc(sizeof(T), BXB, YT) * BXB * YT];
    __shared__ __attribute__((aligned(16))) T s_ftab[RT_NFMAX * ST_FTP];
    __shared__ int s_ox[ST_MAXL], s_oy[ST_MAXL], s_fo[ST_MAXL];
    __shared__ double s_red[NW];
    __shared__ T s_bv[NW];
    __shared__ unsigned s_bl[NW];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int rg = wave % WR, col = (wave / WR) * 64 + lane;
    const int tile = st_tile(blockIdx.x, gridDim.x);
    const int bx = tile % G.gx, rest = tile / G.gx;
    const int i0 = bx * BXB, y0 = (rest % G.gy) * YT, k0 = (rest / G.gy) * G.KC;
    const int nL = min(G.KC, TH - k0) + 2 * HALF;
    const int gy = y0 + col;
    const size_t lstride = (size_t)X * Y;
    PC_STAMP(3, 0);

    // stage the block's control and the filter table; issue the normalisation
    // partials' loads (reduced after the first windows are in flight)
    if (tid < nL + ST_PF + 1) {  // + the prefetches issued past the chunk
        const int L = rs::wrapi(k0 - HALF + tid, TH);
        s_ox[tid] = rs::wrapi(ctl_ox(ctl, L), X);   // shifts may exceed the grid (vtrans large)
        s_oy[tid] = rs::wrapi(ctl_oy(ctl, L), Y);
        s_fo[tid] = ctl_fi(ctl, L) * ST_FTP;
    }
    for (int i = tid; i < nf * FT; i += NT) {
        const int fi = i / FT;
        s_ftab[fi * ST_FTP + (i - fi * FT)] = filt[i];
    }
    double pt[NPP];
#pragma unroll
    for (int u = 0; u < NPP; ++u) {
        const int i = tid + u * NT;
        pt[u] = part[min(i, npart - 1)];  // unconditional (a guarded load got its wait hoisted)
    }
    double pextra = 0.0;
    for (int i = tid + NPP * NT; i < npart; i += NT) pextra += part[i];
    T zf[FL];
#pragma unroll
    for (int z = 0; z < FL; ++z) zf[z] = (T)ctl_zf(ctl, z);
    __syncthreads();

    // window element e = (row r, col c) <-> Q[L][(i0-3+r+ox[L]) % X][(y0-3+c+oy[L]) % Y]
    // unshifted window coordinates, wrapped once: (a + o) % n == (a % n + o) % n with
    // o in [0, n), so a shifted coordinate needs one conditional subtraction
    int er[LPT], ec[LPT];
#pragma unroll
    for (int u = 0; u < LPT; ++u) {
        const int e = min(tid + u * NT, WN - 1), r = e / RW;
        er[u] = rs::wrapi(i0 - HALF + r, X);
        ec[u] = rs::wrapi(y0 - HALF + (e - r * RW), Y);
    }
    T pre[FL][LPT];
    auto load = [&](int it, T(&dst)[LPT]) {
        const int ox = s_ox[it], oy = s_oy[it];
        const T* src = Q + (size_t)rs::wrapi(k0 - HALF + it, TH) * lstride;
#pragma unroll
        for (int u = 0; u < LPT; ++u) {
            int gx = er[u] + ox, gc = ec[u] + oy;
            gx -= gx >= X ? X : 0;
            gc -= gc >= Y ? Y : 0;
            dst[u] = st_load(src, (unsigned)(gx * Y + gc));
        }
    };
#pragma unroll
    for (int d = 0; d < ST_PF; ++d) load(d, pre[d]);
    double tot = pextra;
#pragma unroll
    for (int u = 0; u < NPP; ++u) tot += tid + u * NT < npart ? pt[u] : 0.0;
    tot = block_sum_w<NW>(tot, s_red);
    const PcNorm<T> nrm(tot);

    T ring[FL][BX];
    T bv = -std::numeric_limits<T>::infinity();
    unsigned bl = 0xFFFFFFFFu;
    // software-pipelined: iteration it stores window it+1 while filtering window it;
    // one barrier per iteration
#pragma unroll
    for (int u = 0; u < LPT; ++u) s_win[0][tid + u * NT] = pre[0][u];
    load(ST_PF, pre[ST_PF % FL]);
    __syncthreads();
    PC_STAMP(3, 1);
    for (int base = 0; base < nL; base += FL) {
#pragma unroll
        for (int s = 0; s < FL; ++s) {
            const int it = base + s;
            if (it >= nL) break;
            const int b = it & 1;
            // window it+1 (every load is issued, past the chunk too, so the vmcnt
            // count always holds: see pc_excite_stream)
#pragma unroll
            for (int u = 0; u < LPT; ++u) s_win[b ^ 1][tid + u * NT] = pre[(s + 1) % FL][u];
            load(it + 1 + ST_PF, pre[(s + 1 + ST_PF) % FL]);
            if (it == 0) PC_STAMP(3, 2);
            T f[FT];
            st_filter<T>(s_ftab + s_fo[it], f);
            T acc[BX];
#pragma unroll
            for (int i = 0; i < BX; ++i) acc[i] = 0;
#pragma unroll
            for (int a = 0; a < BX + 2 * HALF; ++a) {
                T w[FL];
                const T* rw = &s_win[b][(rg * BX + a) * RW + col];
#pragma unroll
                for (int t = 0; t < FL; ++t) w[t] = rw[t];
#pragma unroll
                for (int i = 0; i < BX; ++i) {
                    const int x = a - i;
                    if (x < 0 || x >= FL) continue;
#pragma unroll
                    for (int t = 0; t < FL; ++t) acc[i] += w[t] * f[x * FL + t];
                }
            }
#pragma unroll
            for (int i = 0; i < BX; ++i) ring[s][i] = pc_clamp(acc[i]);
            if (it >= 2 * HALF) {
                const int o = it - 2 * HALF, gk = k0 + o;
#pragma unroll
                for (int i = 0; i < BX; ++i) {
                    T v = 0;
#pragma unroll
                    for (int z = 0; z < FL; ++z) v += ring[(s + 1 + z) % FL][i] * zf[z];
                    v = pc_clamp(v);
                    v = nrm(v);
                    s_out[(o * BXB + rg * BX + i) * YT + col] = v;
                    const int gi = i0 + rg * BX + i;
                    const unsigned lin = ((unsigned)gi * Y + gy) * TH + gk;
                    if (gi < X && gy < Y && pc_better(v, lin, bv, bl)) {
                        bv = v;
                        bl = lin;
                    }
                }
            }
            __syncthreads();
        }
    }
    PC_STAMP(3, 3);
    // write-back: each thread stores the cells it computed (its own LDS slots)
    for (int o = 0; o < nL - 2 * HALF; ++o)
#pragma unroll
        for (int i = 0; i < BX; ++i) {
            const int gi = i0 + rg * BX + i;
            if (gi < X && gy < Y)
                P[((size_t)(k0 + o) * X + gi) * Y + gy] = s_out[(o * BXB + rg * BX + i) * YT + col];
        }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const T ov = __shfl_xor(bv, off);
        const unsigned ol = __shfl_xor(bl, off);
        if (pc_better(ov, ol, bv, bl)) {
            bv = ov;
            bl = ol;
        }
    }
    if (lane == 0) {
        s_bv[wave] = bv;
        s_bl[wave] = bl;
    }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < NW; ++w)
            if (pc_better(s_bv[w], s_bl[w], bv, bl)) {
                bv = s_bv[w];
                bl = s_bl[w];
            }
        if constexpr (sizeof(T) == 4) {
            atomicMax(res_slot + (blockIdx.x & (RES_SLOTS - 1)), argmax_key((float)bv, bl));
        } else {
            bmax[blockIdx.x] = bv;
            bidx[blockIdx.x] = bl;
        }
    }
    PC_STAMP(3, 4);
}

// ---------------------------------------------------------------------------
// Column forms (large grids).  A block of CO_NW waves owns a TX x TY tile of
// cells through ALL TH layers, so neither theta pass needs halo layers and no
// layer waits on another: the block loads its whole (TX+6) x (TY+6) x TH window
// at once (every load in flight together, one global round trip), then runs each
// pass over all layers in parallel with one barrier between passes.  The xy halo
// is re-read by neighbouring tiles ((TX+6)(TY+6) / (TX*TY) loads per cell) and
// the y pass runs over the TX+6 window rows; the theta passes are not repeated.
// The stream form's walk over KC+6 layers in sequence (one barrier and one LDS
// round trip chain per layer) is what bounds it at 128x128x72; here a block has
// four phases whatever TH is.  Tiles are numbered XCD-aware (st_tile).
// Window rows/cols wrap with one conditional add/subtract, so X >= TX+6 and
// Y >= TY+6 (checked on the host); TH <= co_thmax (the window in LDS).
// ---------------------------------------------------------------------------
// 12 waves per block (768 threads; 9, 10, 11, 13, 14, 16: 20.6, 20.3, 20.2, 20.5,
// 20.3, 20.2 us vs 19.8 per 128x128x72 step)
constexpr int CO_TX = 8, CO_TY = 8, CO_NW = 12;
// float64 whole-extent blocks: 8 waves (2 per SIMD), so the path kernel's 7x7 filter
// taps and its window loads fit the 256 VGPRs per wave without spilling
template <typename T>
__host__ __device__ constexpr int co_nw() { return sizeof(T) == 4 ? CO_NW : 8; }
// 7x7 filter tasks of the path kernel: 2 tasks per output column (4-row halves),
// 2 output columns per task, window rows scheduled 2 at a time
constexpr int CO_FSPLIT = 2, CO_FCOLS = 2, CO_FROWS = 2;
constexpr int CO_CH = 8;                        // layers per theta-pass task (scalar stream/rows helpers)
constexpr int CO_LDS = 150 * 1024;              // LDS budget of the excitation kernel
// Window rows are loaded as 16-byte vectors of VEC = 16 / sizeof(T) cells from a
// VEC-aligned start (Y % VEC == 0, so a vector never straddles the wrap): a row of
// HY cells starting d = start % VEC cells into its first vector takes
// ceil((HY + d) / VEC) vectors.  The excitation window starts at y0 - 3 with y0 a
// multiple of 8 (d = VEC - 3 % VEC); the path windows are shifted per layer (any d).
template <typename T>
__host__ __device__ constexpr int co_vec() { return 16 / (int)sizeof(T); }
template <typename T, bool SHIFTED>
__host__ __device__ constexpr int co_ncp() {  // vectors per window row
    return (CO_TY + 2 * HALF + (SHIFTED ? co_vec<T>() - 1 : (co_vec<T>() - HALF % co_vec<T>()) % co_vec<T>()) +
            co_vec<T>() - 1) / co_vec<T>();
}
// Layers of LDS window per block: the whole theta extent in one block per CU
// (co_thmax), or a theta chunk plus its 6 halo layers with two blocks per CU
// (co_thmax_chunk).  The excitation kernel's window + y-pass outputs set the size.
template <typename T>
__host__ __device__ constexpr int co_layer_bytes(bool padded) {
    return ((CO_TX + 2 * HALF) * (co_ncp<T, false>() + (padded ? 1 : 0)) * co_vec<T>() +
            2 * (CO_TX + 2 * HALF) * CO_TY) * (int)sizeof(T);
}
template <typename T>
__host__ __device__ constexpr int co_thmax() { return CO_LDS / co_layer_bytes<T>(true); }
constexpr int CO_LDS_CHUNK = 76 * 1024;   // two blocks per CU
constexpr int CO_NW_CHUNK = 8;            // 16 waves per CU: the path kernel's VGPRs allow 4 per SIMD
template <typename T>
__host__ __device__ constexpr int co_thmax_chunk() { return CO_LDS_CHUNK / co_layer_bytes<T>(false); }

// window coordinate a in [-n, 2n) -> [0, n)
__device__ inline int co_wrap(int a, int n) {
    a += a < 0 ? n : 0;
    return a - (a >= n ? n : 0);
}

// A 16-byte output vector at element offset e of a volume of nbytes bytes, stored
// write-through (sc1: the line leaves the XCD's L2 at once, so the kernel ends with
// nothing dirty to write back -- 128x128x72: 27.7 -> 24.3 us per batched step with
// the 16-byte theta-pass stores, tools/pc_ab.py; the excite -> path boundary gap
// 3.5 -> 2.1 us, tools/pc_probe.hip); volumes of 2 GiB or more: plain stores.
template <typename T, typename V>
__device__ inline void co_put(T* __restrict__ base, size_t e, V v, bool wt, int nbytes) {
    if (wt) {
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, nbytes, 0x00020000);
        if constexpr (sizeof(V) == 8) {
            typedef unsigned v2u __attribute__((ext_vector_type(2)));
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, v), r, (int)(e * sizeof(T)), 0, 16);
        } else {
            typedef unsigned v4u __attribute__((ext_vector_type(4)));
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v), r, (int)(e * sizeof(T)), 0, 16);
        }
        return;
    }
    (void)wt;
    (void)nbytes;
    *reinterpret_cast<V*>(base + e) = v;
}

template <typename T>
struct CoVec;
// native vector types: their copies are vector loads/stores, not memcpys (a window
// array of HIP_vector_type kept live across a loop stayed in scratch)
typedef float co_f4 __attribute__((ext_vector_type(4)));
typedef double co_d2 __attribute__((ext_vector_type(2)));
template <>
struct CoVec<float> { using type = co_f4; };
template <>
struct CoVec<double> { using type = co_d2; };


// Layers of one column block: nl = nout + 2*halo window layers, local layer L
// holding global layer k0 - halo + L (wrapped); CHUNK: the block holds a theta
// chunk (halo 3), else the whole periodic extent (k0 = 0, nout = TH, halo 0).
template <bool CHUNK>
struct CoLayers {
    int k0, nout, nl;
    __device__ inline int global(int L, int TH) const { return CHUNK ? co_wrap(k0 - HALF + L, TH) : L; }
    // local layer of theta tap a (0..13) for the outputs of chunk j (8 per task)
    __device__ inline int tap(int j, int a, int TH) const {
        return CHUNK ? min(j * 8 + a, nl - 1) : co_wrap(j * 8 - HALF + a, TH);
    }
    // the same for chunks of cl output layers
    __device__ inline int tapc(int j, int a, int cl, int TH) const {
        return CHUNK ? min(j * cl + a, nl - 1) : co_wrap(j * cl - HALF + a, TH);
    }
};

template <bool CHUNK>
__device__ inline CoLayers<CHUNK> co_layers(int ch, int KC, int TH) {
    CoLayers<CHUNK> c;
    c.k0 = CHUNK ? ch * KC : 0;
    c.nout = CHUNK ? min(KC, TH - c.k0) : TH;
    c.nl = c.nout + (CHUNK ? 2 * HALF : 0);
    return c;
}

// Excitation (posecell_network.py:336 -> convolution.py:228-246), inhibition
// (:339-340) and the normalisation partial sum (:343) for one column tile.
// FIX_TH > 0: the instance for TH == FIX_TH (the x-pass output rows then have pitch
// TH + 64: a cell's row starts TH dwords modulo the 64 banks after the previous one, as
// if the rows were contiguous, so the theta pass's 16-byte reads of consecutive groups
// of consecutive cells are conflict-free)
template <typename T, int TX, int TY, int NW, int THM, bool CHUNK, int FIX_TH = 0>
__global__ __launch_bounds__(64 * NW) void pc_excite_cols(const T* __restrict__ P, int X, int Y, int TH,
                                                          int gx, int gy, int nblk, T* __restrict__ Q,
                                                          double* __restrict__ part,
                                                          unsigned long long* __restrict__ res_slot, int KC,
                                                          SepKernel<T> k) {
    constexpr int NT = 64 * NW, HX = TX + 2 * HALF, HY = TY + 2 * HALF;
    constexpr int VEC = co_vec<T>();
    static_assert(TY % VEC == 0, "row vectors");
    static_assert(FIX_TH == 0 || (FIX_TH == THM && !CHUNK && FIX_TH % 4 == 0), "fixed-extent instance");
    constexpr int SPO = 4, PP = FIX_TH ? FIX_TH + 64 : (THM + 12 + 3) / 4 * 4;
    __shared__ __attribute__((aligned(16))) T s_in[2 * TX * TY * PP];  // x-pass outputs (e, i)
    __shared__ __attribute__((aligned(16))) T s_ye[THM * HX * TY];  // [r][c][L]
    __shared__ __attribute__((aligned(16))) T s_yi[THM * HX * TY];
    __shared__ double s_red[NW];
    using V = typename CoVec<T>::type;
    const int tid = threadIdx.x;
    const int tile = st_tile(blockIdx.x, nblk), xy = tile % (gx * gy);
    const int x0 = (xy % gx) * TX, y0 = (xy / gx) * TY;
    const CoLayers<CHUNK> ly = co_layers<CHUNK>(tile / (gx * gy), KC, TH);
    // the fixed-extent instance's layer count is compile-time (no division per task)
    const int nlc = FIX_TH > 0 ? FIX_TH : ly.nl;
    if (res_slot != nullptr && blockIdx.x == 0)
        for (int i = tid; i < RES_SLOTS; i += blockDim.x) st_wt(&res_slot[i], 0ull);  // this step's path kernel max-reduces into them
    // the taps and constants in scalar registers for the whole kernel (float32): hipcc
    // otherwise reloads them from the kernel arguments after each barrier, a scalar
    // round trip at the head of the x and theta passes
    if constexpr (sizeof(T) == 4) {
#pragma unroll
        for (int q = 0; q < FL; ++q) asm volatile("" : "+s"(k.ge[q]), "+s"(k.gi[q]));
        asm volatile("" : "+s"(k.scale), "+s"(k.inhib));
    }
    PC_STAMP(5, 0);
    // y pass straight from the loads.  P is theta-fastest on this form (cell (x, y)
    // holds its TH layers contiguously), so task (r, L) = window row r of layer L
    // puts consecutive lanes on consecutive layers: each load instruction reads
    // consecutive words of one cell's theta column (whole 128-byte lines, where the
    // layer-major rows of 14 cells used a third of each line they touched).  Every
    // row of the block is in flight at once; the window never visits LDS; the y-pass
    // outputs go to LDS as [r][c][L].
    if constexpr (FIX_TH > 0) {
        // the fixed-extent instance: 16-byte loads of 4 consecutive layers of a cell
        // (a quarter of the load instructions), task (row r, layer group g): the row's
        // 14 window cells, 8 outputs x 4 layers, each output one 16-byte LDS store;
        // 14 x TH/4 tasks (252 at TH = 72: 4 waves).  (Half rows on 8 waves loaded 20
        // cells a row, 80 KiB a block through the load path instead of 56: 14.53 ->
        // 14.42 us per 128 x 128 x 72 step, tools/pc_ab.py, round 6)
        constexpr int NG = FIX_TH / 4, TH2 = TY, HW = TH2 + 2 * HALF;
        static_assert(HX * NG <= NT, "one task per thread");
        const int t = tid;
        if (t < HX * NG) {
            const int r = t / NG, h = 0, g = t - r * NG;
            const T* rowp = P + ((size_t)co_wrap(x0 - HALF + r, X) * Y) * FIX_TH + 4 * g;
            V w[HW];
#pragma unroll
            for (int c = 0; c < HW; ++c)
                w[c] = *reinterpret_cast<const V*>(rowp + (size_t)co_wrap(y0 - HALF + h * TH2 + c, Y) * FIX_TH);
#pragma unroll
            for (int c = 0; c < TH2; ++c) {
                V e = {0, 0, 0, 0}, gg = {0, 0, 0, 0};
#pragma unroll
                for (int q = 0; q < FL; ++q) {
                    e += k.ge[q] * w[c + q];
                    gg += k.gi[q] * w[c + q];
                }
                const int o = (r * TY + h * TH2 + c) * THM + 4 * g;
                *reinterpret_cast<V*>(s_ye + o) = e;
                *reinterpret_cast<V*>(s_yi + o) = gg;
            }
        }
    } else {
        constexpr int NR = (THM * HX + NT - 1) / NT;
        const int nrow = ly.nl * HX;
        T w[NR][HY];
#pragma unroll
        for (int u = 0; u < NR; ++u) {
            const int t = min(tid + u * NT, nrow - 1), r = t / ly.nl, L = t - r * ly.nl;
            const T* cell = P + ((size_t)co_wrap(x0 - HALF + r, X) * Y) * TH + ly.global(L, TH);
#pragma unroll
            for (int c = 0; c < HY; ++c) w[u][c] = cell[(size_t)co_wrap(y0 - HALF + c, Y) * TH];
        }
#pragma unroll
        for (int u = 0; u < NR; ++u) {
            const int t = tid + u * NT;
            if (t >= nrow) break;
            const int r = t / ly.nl, L = t - r * ly.nl;
#pragma unroll
            for (int c = 0; c < TY; ++c) {
                T e = 0, g = 0;
#pragma unroll
                for (int q = 0; q < FL; ++q) {
                    e += k.ge[q] * w[u][c + q];
                    g += k.gi[q] * w[u][c + q];
                }
                s_ye[(r * TY + c) * THM + L] = e;   // [r][c][L]: consecutive lanes, consecutive words
                s_yi[(r * TY + c) * THM + L] = g;
            }
        }
    }
    PC_STAMP(5, 1);
    co_lds_barrier();
    PC_STAMP(5, 2);
    // x pass: task (L, c) -> a column of TX outputs from HX y-pass rows, written as
    // [cell p][SPO + L] rows of pitch PP (16-byte aligned: the theta pass reads
    // them as vectors; consecutive lanes take consecutive layers, so the writes are
    // conflict-free).  The whole-extent form also writes each output's wrapped copy
    // (layers TH-4..TH-1 before SPO, 0..7 after SPO + TH), so every theta window is
    // one contiguous aligned run with no extra pass.
    T* s_xe = s_in;
    T* s_xi = s_in + TX * TY * PP;
    // one task: outputs i0 .. i0 + R - 1 of column c, layer L
    auto xtask = [&](int c, int L, int i0, auto r_c) __attribute__((always_inline)) {
        constexpr int R = decltype(r_c)::value;
        T ye[R + 2 * HALF], yi[R + 2 * HALF];
#pragma unroll
        for (int a = 0; a < R + 2 * HALF; ++a) {
            ye[a] = s_ye[((i0 + a) * TY + c) * THM + L];
            yi[a] = s_yi[((i0 + a) * TY + c) * THM + L];
        }
        // wrapped copies (TH >= 10, so at most one of each)
        const int Lw1 = !CHUNK && L < 8 ? nlc + L : INT_MIN, Lw2 = !CHUNK && L >= nlc - 4 ? L - nlc : INT_MIN;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            T e = 0, g = 0;
#pragma unroll
            for (int q = 0; q < FL; ++q) {
                e += k.ge[q] * ye[i + q];
                g += k.gi[q] * yi[i + q];
            }
            const int r = ((i0 + i) * TY + c) * PP + SPO;
            s_xe[r + L] = e;
            s_xi[r + L] = g;
            if (Lw1 != INT_MIN) {
                s_xe[r + Lw1] = e;
                s_xi[r + Lw1] = g;
            }
            if (Lw2 != INT_MIN) {
                s_xe[r + Lw2] = e;
                s_xi[r + Lw2] = g;
            }
        }
    };
    if constexpr (FIX_TH == 72 && TX == 8 && TY == 8 && NW == 12) {
        // the 72-layer instance balances the four SIMDs (wave w runs on SIMD w % 4):
        // waves 0-7 take layers 0-63 (lane = layer) of column w, waves 8-11 layers 64-71
        // (64 + (lane & 7)) of column lane >> 3, two of the eight outputs each; 576 equal
        // tasks on 9 waves put three on SIMD 0
        const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
        if (wave < 8) xtask(wave, lane, 0, std::integral_constant<int, TX>{});
        else xtask(lane >> 3, 64 + (lane & 7), 2 * (wave - 8), std::integral_constant<int, 2>{});
    } else {
        for (int t = tid; t < nlc * TY; t += NT) {
            const int c = t / nlc, L = t - c * nlc;
            xtask(c, L, 0, std::integral_constant<int, TX>{});
        }
    }
    co_lds_barrier();
    PC_STAMP(5, 3);
    // theta pass: task (cell p, group j of VEC layers), consecutive lanes on
    // consecutive groups of one cell: the outputs of a group are one 16-byte
    // write-through store into Q, which is theta-fastest like P (the path kernel
    // then loads whole runs of each cell's layers)
    double sum = 0.0;
    {
        const int ng = FIX_TH > 0 ? FIX_TH / VEC : (ly.nout + VEC - 1) / VEC;
        const int nbytes = (int)min((size_t)X * Y * TH * sizeof(T), (size_t)INT_MAX);
        const bool wt = (size_t)X * Y * TH * sizeof(T) <= (size_t)INT_MAX;
        constexpr int ROFF = CHUNK ? 0 : 1, NRV = (ROFF + VEC + 2 * HALF + VEC - 1) / VEC;
#pragma unroll 1
        for (int t = tid; t < TX * TY * ng; t += NT) {
            const int p = t / ng, j = t - p * ng, i = p / TY;
            const int gi = x0 + i, gy = y0 + p - i * TY;
            // taps of output lo = j * VEC + o: local layers lo - 3 .. lo + 3 (whole
            // extent, from the aligned run starting at lo - 4) or lo .. lo + 6 (a chunk's
            // local layer lo + 3 is its output lo)
            const V* se = reinterpret_cast<const V*>(s_xe + p * PP + SPO + j * VEC - (CHUNK ? 0 : 4));
            const V* si = reinterpret_cast<const V*>(s_xi + p * PP + SPO + j * VEC - (CHUNK ? 0 : 4));
            T re[NRV * VEC], ri[NRV * VEC];
#pragma unroll
            for (int q = 0; q < NRV; ++q) {
                const V a = se[q], b = si[q];
#pragma unroll
                for (int c = 0; c < VEC; ++c) {
                    re[q * VEC + c] = a[c];
                    ri[q * VEC + c] = b[c];
                }
            }
            V qv;
#pragma unroll
            for (int o = 0; o < VEC; ++o) {
                T e = 0, g = 0;
#pragma unroll
                for (int z = 0; z < FL; ++z) {
                    e += k.ge[z] * re[ROFF + o + z];
                    g += k.gi[z] * ri[ROFF + o + z];
                }
                const T v = (e - g) * k.scale;
                qv[o] = (v < k.inhib) ? T(0) : v - k.inhib;
            }
            if (gi < X && gy < Y) {
                const int gk0 = ly.k0 + j * VEC, nv = min(VEC, ly.nout - j * VEC);
                const size_t e0 = ((size_t)gi * Y + gy) * TH + gk0;
                if (nv == VEC && e0 % VEC == 0) {
                    co_put(Q, e0, qv, wt, nbytes);
                } else {  // a ragged or unaligned group (TH or the chunk not a multiple of VEC)
#pragma unroll
                    for (int o = 0; o < VEC; ++o)
                        if (o < nv) Q[e0 + o] = qv[o];
                }
#pragma unroll
                for (int o = 0; o < VEC; ++o)
                    if (o < nv) sum += (double)qv[o];
            }
        }
    }
    sum = co_wave_sum(sum);
    if ((tid & 63) == 0) s_red[tid >> 6] = sum;
    co_lds_barrier();  // the Q stores drain meanwhile
    if (tid == 0) {
        double t = 0.0;
#pragma unroll
        for (int w = 0; w < NW; ++w) t += s_red[w];
        st_wt(&part[blockIdx.x], t);
    }
    PC_STAMP(5, 4);
}

// Path integration (posecell_network.py:252-314) for one column tile: per-layer
// shifted 7x7 filter (:273 -> convolution.py:320-340), clamp (:300), 7-tap theta
// filter (:310 -> convolution.py:344-359), clamp (:314), normalisation by the
// excitation total (:343-345, applied at the end), fused argmax (:317-319).
// Window buffer of the path kernel (bytes): the whole-extent form runs one block per
// CU, the theta-chunked form two.
constexpr int CO_WIN_BYTES = 128 * 1024, CO_WIN_BYTES_CHUNK = 56 * 1024;
// theta extent of the path kernel's LDS-DMA window instance (float32, whole extent,
// control as kernel arguments): BASELINE configs[3]'s 72 layers
constexpr int CO_DMA_TH = 72;

// signed shift in (-n/2, n/2] (control shifts may exceed the grid: vtrans large)
__host__ __device__ inline int co_centre(int o, int n) {
    o = rs::wrapi(o, n);
    return o > n / 2 ? o - n : o;
}

// wave min / max of an int by DPP row operations and readlanes (as co_wave_max)
template <bool MAX>
__device__ inline int co_wave_ext_i(int v) {
    auto op = [](int a, int b) { return MAX ? max(a, b) : min(a, b); };
    v = op(v, __builtin_amdgcn_update_dpp(v, v, 0xB1, 0xF, 0xF, false));
    v = op(v, __builtin_amdgcn_update_dpp(v, v, 0x4E, 0xF, 0xF, false));
    v = op(v, __builtin_amdgcn_update_dpp(v, v, 0x141, 0xF, 0xF, false));
    v = op(v, __builtin_amdgcn_update_dpp(v, v, 0x140, 0xF, 0xF, false));
    return op(op(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
              op(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}

// DMA_TH > 0: the instance for TH == DMA_TH (float32, whole extent, control as kernel
// arguments).  Its window is an LDS image [u][v][layer] with no padding between a
// cell's layers, so each 16-byte piece of a cell's theta run in Q has a fixed place,
// and the pieces go global -> LDS by LDS-DMA (global_load_lds_dwordx4, lane-linear
// 1 KiB per wave-instruction): no register staging and no ds_write (the scalar
// stores into the odd-pitch image were 4-way bank conflicts), issued first thing from
// the host-formed union (PcCtlInline::umx..uwy), in flight together with the
// control's, the partials' and the filter table's loads: one round trip.
template <typename T, int TX, int TY, int NW, int THM, bool CHUNK, typename CTL, int DMA_TH = 0>
__global__ __launch_bounds__(64 * NW) void pc_path_cols(
    const T* __restrict__ Q, int X, int Y, int TH, int gx, int gy, int nblk, T* __restrict__ P,
    const double* __restrict__ part, int npart, const T* __restrict__ filt, int nf, CTL ctl,
    unsigned long long* __restrict__ res_slot, T* __restrict__ bmax, unsigned* __restrict__ bidx, int KC) {
    constexpr int NT = 64 * NW, VEC = co_vec<T>();
    constexpr bool DMA = DMA_TH > 0;
    // Q is theta-fastest, like P: the block loads the union of its layers' shifted
    // windows -- WX x WY cells, each cell's run of layers contiguous in Q -- into LDS
    // as [cell][layer] (every |shift| <= 3 at 128x128x72: 20 x 20 cells x 72 layers,
    // 115 KiB).  Consecutive lanes take consecutive layers: the loads read whole runs
    // of a cell's layers and the filter's LDS reads are conflict-free.  Shifts whose
    // union window does not fit take per-layer 14 x 14 windows instead.
    // (the DMA instance: windows of up to 20 x 20 cells, shifts spread over at most 6
    // cells, plus one wave-instruction of slack for the last pieces)
    constexpr int WBUF = DMA ? 20 * (TY + 2 * HALF + 6) * DMA_TH + 4 * 64
                             : (CHUNK ? CO_WIN_BYTES_CHUNK : CO_WIN_BYTES) / (int)sizeof(T);
    using V = typename CoVec<T>::type;
    __shared__ __attribute__((aligned(16))) T s_w[WBUF];
    // clamped 7x7 outputs [cell p][SPO + L], pitch PP (16-byte rows: the theta pass
    // reads VEC-aligned vectors); the whole-extent form also keeps wrapped copies of
    // the last 4 layers before SPO and of the first 8 after SPO + TH, so every theta
    // window is one contiguous aligned run
    // (the DMA instance: PP = TH + 64, so a cell's row starts TH dwords modulo the 64
    // banks after the previous one, as if the rows were contiguous: the theta pass's
    // 16-byte reads of consecutive groups of consecutive cells are conflict-free)
    constexpr int SPO = 4, PP = DMA ? DMA_TH + 64 : (THM + 12 + 3) / 4 * 4;
    __shared__ __attribute__((aligned(16))) T s_p[TX * TY * PP];
    __shared__ __attribute__((aligned(16))) T s_ftab[RT_NFMAX * ST_FTP];
    __shared__ int s_ox[THM], s_oy[THM], s_fo[THM];
    __shared__ T s_bv[NW];
    __shared__ unsigned s_bl[NW];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int tile = st_tile(blockIdx.x, nblk), xy = tile % (gx * gy);
    const int x0 = (xy % gx) * TX, y0 = (xy / gx) * TY;
    const CoLayers<CHUNK> ly = co_layers<CHUNK>(tile / (gx * gy), KC, TH);
    PC_STAMP(6, 0);
    // window strides are compile-time (the filter's LDS reads take immediate offsets):
    // WYP cells per window row, LPC layers per cell (odd: fewer bank conflicts between
    // lanes whose layers have different shifts; the DMA image: exactly TH), at most
    // WXP rows
    constexpr int WYP = TY + 2 * HALF + 6, LPC = DMA ? DMA_TH : (THM | 1), WXP = WBUF / (WYP * LPC);
    static_assert(WXP >= TX + 2 * HALF, "a per-layer window fits");
    bool dma = false;
    // the union's fields (DMA instance) in scalar registers for the whole kernel: hipcc
    // otherwise reloads them from the kernel arguments after the first barrier
    int cumx = 0, cumy = 0, cuwx = 0, cuwy = 0;
    if constexpr (DMA) {
        cumx = __builtin_amdgcn_readfirstlane((int)ctl.umx);
        cumy = __builtin_amdgcn_readfirstlane((int)ctl.umy);
        cuwx = __builtin_amdgcn_readfirstlane((int)ctl.uwx);
        cuwy = __builtin_amdgcn_readfirstlane((int)ctl.uwy);
        asm volatile("" : "+s"(cumx), "+s"(cumy), "+s"(cuwx), "+s"(cuwy));
    }
    if constexpr (DMA) {
        static_assert(sizeof(T) == 4 && !CHUNK && DMA_TH % 4 == 0 && DMA_TH <= THM, "DMA window form");
        constexpr int PPC = DMA_TH / 4;    // 16-byte pieces per cell
        static_assert(WXP * WYP * PPC + 63 <= WBUF / 4, "the last wave-instruction stays in the buffer");
        const int WX = cuwx, WY = cuwy;
        dma = TH == DMA_TH && WX <= WXP && WY <= WYP && WX <= X && WY <= Y;
        if (dma) {
            // piece p = (u * WYP + v) * PPC + l4 lands at s_w + 4p (the padding cells
            // v >= WY are not loaded); a thread's pieces advance by NT per instruction
            const int ux0 = co_wrap(x0 - HALF + cumx, X), uy0 = co_wrap(y0 - HALF + cumy, Y);
            const int npc = WX * WYP * PPC, wave_u = __builtin_amdgcn_readfirstlane(wave);
            constexpr int DC = NT / PPC, DL = NT % PPC, DU = DC / WYP, DV = DC % WYP;
            constexpr int NK = (WXP * WYP * PPC + NT - 1) / NT;
            const int p0 = wave_u * 64 + lane;
            int c = p0 / PPC, l4 = p0 - c * PPC, u = c / WYP, v = c - u * WYP;
#pragma unroll
            for (int k = 0; k < NK; ++k) {
                const int i0 = k * NT + wave_u * 64;  // wave-uniform
                if (i0 < npc) {
                    if (i0 + lane < npc && v < WY) {
                        int gr = ux0 + u, gc = uy0 + v;
                        gr -= gr >= X ? X : 0;
                        gc -= gc >= Y ? Y : 0;
                        __builtin_amdgcn_global_load_lds(
                            (__attribute__((address_space(1))) const void*)(Q + ((unsigned)gr * Y + gc) * DMA_TH + 4 * l4),
                            (__attribute__((address_space(3))) void*)(s_w + 4 * i0), 16, 0, 0);
                    }
                }
                l4 += DL;
                v += DV;
                u += DU;
                if (l4 >= PPC) {
                    l4 -= PPC;
                    ++v;
                }
                if (v >= WYP) {
                    v -= WYP;
                    ++u;
                }
            }
        }
    }
    // The control first (its loads are the ones the first barrier waits for; clamped
    // unconditional reads, in flight together), then the normalisation partials (a
    // guarded load had its wait hoisted to the kernel's start).  Every wave forms
    // the total itself: no block barrier between the window loads and their use.
    static_assert(THM <= NT, "one layer's control per thread");
    const int Lc = min(tid, ly.nl - 1), gLc = ly.global(Lc, TH);
    const int oxc = ctl_ox(ctl, gLc), oyc = ctl_oy(ctl, gLc), fic = ctl_fi(ctl, gLc);
    constexpr int NPL = 4;  // partials per lane loaded up front (npart <= 256 in one round)
    double pt[NPL];
#pragma unroll
    for (int u = 0; u < NPL; ++u) pt[u] = part[min(lane + 64 * u, npart - 1)];
    if (tid < ly.nl) {
        s_ox[tid] = co_centre(oxc, X);
        s_oy[tid] = co_centre(oyc, Y);
        s_fo[tid] = fic * ST_FTP;
    }
    constexpr int NFR = (RT_NFMAX * FT + NT - 1) / NT;
    T fr[NFR];
#pragma unroll
    for (int u = 0; u < NFR; ++u) fr[u] = tid + u * NT < nf * FT ? filt[tid + u * NT] : T(0);
    T zf[FL];
#pragma unroll
    for (int z = 0; z < FL; ++z) zf[z] = (T)ctl_zf(ctl, z);
    // the normalisation total (every wave forms it itself) and the filter table into
    // LDS before the first barrier, which waits for the control's loads anyway: the
    // window's loads then follow with nothing else to wait for
    // (the DMA instance forms it after the first barrier, in its last wave, which has no
    // filter task: the partials are the youngest loads of every wave, so forming the total
    // here waits for the whole window, and the DPP reduction and reciprocal sat between the
    // window's landing and the barrier)
    auto total = [&]() __attribute__((always_inline)) {
        double tot = 0.0;
#pragma unroll
        for (int u = 0; u < NPL; ++u) tot += lane + 64 * u < npart ? pt[u] : 0.0;
        for (int i = lane + 64 * NPL; i < npart; i += 64) tot += part[i];
        return co_wave_sum(tot);
    };
    // the normalisation (:343-345): PcNorm (float32: the product with the reciprocal)
    __shared__ float s_nrm[3];   // (the DMA instance: r, t, div of the total's PcNorm<float>)
    const PcNorm<T> nrm0(DMA ? 1.0 : total());
#pragma unroll
    for (int u = 0; u < NFR; ++u) {
        const int i = tid + u * NT, fi = i / FT;
        if (i < nf * FT) s_ftab[fi * ST_FTP + (i - fi * FT)] = fr[u];
    }
    // the DMA pieces have landed before any wave passes the barrier and reads them
    // (a wave's waitcnt covers its own LDS-DMA; the barrier, everyone's)
    if (DMA && dma) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    co_lds_barrier();
    PC_STAMP(6, 1);
    // the union window of the block's layers (every wave reduces the shifts itself;
    // the DMA form has it from the host)
    int mnx = INT_MAX, mxx = INT_MIN, mny = INT_MAX, mxy = INT_MIN;
    if (DMA && dma) {
        if constexpr (DMA) {
            mnx = cumx;
            mny = cumy;
            mxx = mnx + cuwx - (TX + 2 * HALF);
            mxy = mny + cuwy - (TY + 2 * HALF);
        }
    } else {
        for (int L = lane; L < ly.nl; L += 64) {
            mnx = min(mnx, s_ox[L]);
            mxx = max(mxx, s_ox[L]);
            mny = min(mny, s_oy[L]);
            mxy = max(mxy, s_oy[L]);
        }
        mnx = co_wave_ext_i<false>(mnx);
        mxx = co_wave_ext_i<true>(mxx);
        mny = co_wave_ext_i<false>(mny);
        mxy = co_wave_ext_i<true>(mxy);
    }
    const int WX = TX + 2 * HALF + mxx - mnx, WY = TY + 2 * HALF + mxy - mny;
    const bool uni = WX <= WXP && WY <= WYP && WX <= X && WY <= Y;
    const int ux0 = co_wrap(x0 - HALF + mnx, X), uy0 = co_wrap(y0 - HALF + mny, Y);

    constexpr int FS = CO_FSPLIT, TXH = TX / FS, CP = CO_FCOLS, NCG = TY / CP;
    static_assert(TX % FS == 0 && TY % CP == 0, "filter task shape");
    const int nl = DMA ? DMA_TH : ly.nl;   // (the DMA instance runs at TH == DMA_TH only: no division per task)
    if (DMA && dma) {
        // the window is in LDS already
    } else if (uni && !CHUNK && TH % VEC == 0) {
        // the common case: the union window (WX x WY cells) with 16-byte loads of VEC
        // consecutive layers of a cell, positions advanced incrementally (no
        // divisions per element); all of a thread's loads in flight together
        constexpr int NV = (WXP * WYP * LPC / VEC + NT - 1) / NT;
        // float64: two rounds of loads (all NV in flight spills the filter's registers)
        constexpr int NR = sizeof(T) == 4 ? 1 : 2, NVR = (NV + NR - 1) / NR;
        const int lcw = nl / VEC, nel = WX * WY * lcw;
        const int c = tid / lcw, dc = NT / lcw, dl = (NT - dc * lcw) * VEC;
        const int dcu = dc / WY, dcv = dc - dcu * WY;
        int cu = c / WY, cv = c - cu * WY, l = (tid - c * lcw) * VEC;   // load cursor
        int su = cu, sv = cv, sl = l;                                   // store cursor
        auto advance = [&](int& u_, int& v_, int& l_) __attribute__((always_inline)) {
            l_ += dl;
            v_ += dcv;
            u_ += dcu;
            if (l_ >= nl) {
                l_ -= nl;
                ++v_;
            }
            if (v_ >= WY) {
                v_ -= WY;
                ++u_;
            }
        };
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            V w[NVR];
#pragma unroll
            for (int k = 0; k < NVR; ++k) {
                const int u = r * NVR + k;
                if (u < NV) {  // straight-line: a thread past the window re-reads element 0
                    int gr = ux0 + cu, gc = uy0 + cv;
                    gr -= gr >= X ? X : 0;
                    gc -= gc >= Y ? Y : 0;
                    const unsigned off = tid + u * NT < nel ? ((unsigned)gr * Y + gc) * TH + l
                                                            : ((unsigned)ux0 * Y + uy0) * TH;
                    w[k] = *reinterpret_cast<const V*>(Q + off);
                }
                advance(cu, cv, l);
            }
#pragma unroll
            for (int k = 0; k < NVR; ++k) {
                const int u = r * NVR + k;
                if (u < NV && tid + u * NT < nel) {
                    T* d = s_w + (su * WYP + sv) * LPC + sl;
#pragma unroll
                    for (int j = 0; j < VEC; ++j) d[j] = w[k][j];
                }
                advance(su, sv, sl);
            }
        }
    } else {
        // theta chunks (a window run may wrap around TH), ragged extents, and shifts
        // whose union window does not fit (each layer then takes its own 14 x 14
        // window): scalar elements, 8 loads in flight per thread
        const int wx = uni ? WX : TX + 2 * HALF, wy = uni ? WY : TY + 2 * HALF, nel = wx * wy * nl;
        for (int e0 = tid; e0 < nel; e0 += 8 * NT) {
            T w[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int e = e0 + u * NT;
                if (e < nel) {
                    const int c = e / nl, L = e - c * nl, cu = c / wy, cv = c - cu * wy;
                    const int bx = uni ? ux0 : co_wrap(x0 - HALF + s_ox[L], X);
                    const int by = uni ? uy0 : co_wrap(y0 - HALF + s_oy[L], Y);
                    w[u] = Q[((size_t)co_wrap(bx + cu, X) * Y + co_wrap(by + cv, Y)) * TH + ly.global(L, TH)];
                }
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int e = e0 + u * NT;
                if (e < nel) {
                    const int c = e / nl, L = e - c * nl, cu = c / wy, cv = c - cu * wy;
                    s_w[(cu * WYP + cv) * LPC + L] = w[u];
                }
            }
        }
    }
    if (!(DMA && dma)) co_lds_barrier();
    PC_STAMP(6, 2);
    if constexpr (DMA) {
        static_assert(DMA_TH * NCG * FS <= 64 * (NW - 1), "the last wave has no filter task");
        if (wave == NW - 1) {
            const PcNorm<float> n1(total());
            if (lane == 0) {
                s_nrm[0] = n1.r;
                s_nrm[1] = n1.t;
                s_nrm[2] = n1.div ? 1.f : 0.f;
            }
        }
    }
    // 7x7 filter: task (layer, column group, row part) -> TX/FS rows x CP columns of
    // outputs from TX/FS + 6 window rows of CP + 6 cells (CP columns share each window
    // row's reads; reads of CO_FROWS rows at a time in flight: hoisting all of them
    // spills at 3 waves per SIMD).  Layer fastest over the lanes.
    // one task: R output rows from tile row x0r, CP columns from c0, of layer L
    auto ftask = [&](int L, int x0r, int c0, auto r_c) __attribute__((always_inline)) {
        constexpr int R = decltype(r_c)::value;
        T f[FT];
        st_filter<T>(s_ftab + s_fo[L], f);
        T acc[R][CP];
#pragma unroll
        for (int i = 0; i < R; ++i)
#pragma unroll
            for (int c = 0; c < CP; ++c) acc[i][c] = 0;
        const int dx = uni ? s_ox[L] - mnx : 0, dy = uni ? s_oy[L] - mny : 0;
        // the base index is opaque to the compiler, so each read keeps its compile-time
        // offset as an immediate (ds_read2_b32 pairs) instead of an address add each
        int wbase = ((x0r + dx) * WYP + c0 + dy) * LPC + L;
        asm volatile("" : "+v"(wbase));
        const T* win = s_w + wbase;
        // the window rows in a rotated order per wave group (waves w, w+4, w+8 share a
        // SIMD): the groups' LDS read bursts and FMA runs interleave instead of
        // running in lockstep behind the barrier
        auto rows = [&](auto rot_c) __attribute__((always_inline)) {
            constexpr int ROT = decltype(rot_c)::value, NRW = R + 2 * HALF;
#pragma unroll
            for (int aa = 0; aa < NRW; ++aa) {
                const int a = (aa + ROT) % NRW;
                T w[FL + CP - 1];
#pragma unroll
                for (int q = 0; q < FL + CP - 1; ++q) w[q] = win[(a * WYP + q) * LPC];
                if (aa % CO_FROWS == CO_FROWS - 1) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int i = 0; i < R; ++i) {
                    const int x = a - i;
                    if (x < 0 || x >= FL) continue;
#pragma unroll
                    for (int c = 0; c < CP; ++c)
#pragma unroll
                        for (int q = 0; q < FL; ++q) acc[i][c] += w[c + q] * f[x * FL + q];
                }
            }
        };
        const int grp = __builtin_amdgcn_readfirstlane(tid >> 8);  // wave / 4
        if (grp == 0) rows(std::integral_constant<int, 0>{});
        else if (grp == 1) rows(std::integral_constant<int, 3>{});
        else rows(std::integral_constant<int, 6>{});
        // with the wrapped copies of the whole-extent form (layers TH-4..TH-1 also
        // before SPO, 0..7 also after SPO + TH; TH >= 10, so at most one of each)
        const int Lw1 = !CHUNK && L < 8 ? nl + L : INT_MIN, Lw2 = !CHUNK && L >= nl - 4 ? L - nl : INT_MIN;
#pragma unroll
        for (int i = 0; i < R; ++i)
#pragma unroll
            for (int c = 0; c < CP; ++c) {
                const T v = pc_clamp(acc[i][c]);
                T* sp = s_p + ((x0r + i) * TY + c0 + c) * PP + SPO;
                sp[L] = v;
                if (Lw1 != INT_MIN) sp[Lw1] = v;
                if (Lw2 != INT_MIN) sp[Lw2] = v;
            }
    };
    if constexpr (DMA) {
        // The DMA instance (72 layers, 8 x 8 tiles, 12 waves) balances the four SIMDs
        // (wave w runs on SIMD w % 4): waves 0-7 take layers 0-63 (lane = layer) in
        // 4-row x 2-column tasks, waves 8-11 layers 64-71 in 1-row x 2-column tasks
        // (layer 64 + (lane & 7), tile row lane >> 3).  Every SIMD issues 2 x 392 + 98
        // filter FMAs per lane, where 576 equal tasks on 9 waves put 3 x 392 on SIMD 0
        static_assert(TX == 8 && TY == 8 && CP == 2 && FS == 2 && NW == 12 && DMA_TH == 72, "DMA instance's task split");
        if (wave < 8) ftask(lane, (wave >> 2) * TXH, (wave & 3) * CP, std::integral_constant<int, TXH>{});
        else ftask(64 + (lane & 7), lane >> 3, (wave - 8) * CP, std::integral_constant<int, 1>{});
    } else {
        for (int t = tid; t < nl * NCG * FS; t += NT) {
            const int L = t % nl, rem = t / nl, hf = rem / NCG, c0 = (rem - hf * NCG) * CP;
            ftask(L, hf * TXH, c0, std::integral_constant<int, TXH>{});
        }
    }
    (void)VEC;
    co_lds_barrier();
    PC_STAMP(6, 3);
    PcNorm<T> nrm = nrm0;
    if constexpr (DMA)   // (div block-uniform: a scalar branch)
        nrm = PcNorm<T>(s_nrm[0], s_nrm[1], __builtin_amdgcn_readfirstlane((int)(s_nrm[2] != 0.f)) != 0);
    // theta pass, clamp, normalisation, argmax: task (cell p, chunk j).  float32:
    // the first maximum as the largest packed (value, ~index) key; float64: value
    // and index pairs
    T bv = -std::numeric_limits<T>::infinity();
    unsigned bl = 0xFFFFFFFFu;
    unsigned long long bk = 0ull;
    {
        // task (cell p, group j of VEC layers), consecutive lanes on consecutive groups
        // of one cell: P is theta-fastest on this form, so a group is one 16-byte
        // store and a wave's stores cover consecutive cells' theta columns
        using V = typename CoVec<T>::type;
        const int ng = DMA ? DMA_TH / VEC : (ly.nout + VEC - 1) / VEC;
        const int nbytes = (int)min((size_t)X * Y * TH * sizeof(T), (size_t)INT_MAX);
        const bool wt = (size_t)X * Y * TH * sizeof(T) <= (size_t)INT_MAX;
#pragma unroll 1
        for (int t = tid; t < TX * TY * ng; t += NT) {
            const int p = t / ng, j = t - p * ng, i = p / TY;
            const int gi = x0 + i, gy = y0 + p - i * TY;
            // taps of output lo = j * VEC + o: local layers lo - 3 .. lo + 3 (whole
            // extent, from the aligned run starting at lo - 4) or lo .. lo + 6 (a chunk's
            // local layer lo + 3 is its output lo)
            constexpr int ROFF = CHUNK ? 0 : 1, NRV = (ROFF + VEC + 2 * HALF + VEC - 1) / VEC;
            const V* sv = reinterpret_cast<const V*>(s_p + p * PP + SPO + j * VEC - (CHUNK ? 0 : 4));
            T rr[NRV * VEC];
#pragma unroll
            for (int q = 0; q < NRV; ++q) {
                const V x = sv[q];
#pragma unroll
                for (int c = 0; c < VEC; ++c) rr[q * VEC + c] = x[c];
            }
            const T* r = rr + ROFF;
            V v;
#pragma unroll
            for (int o = 0; o < VEC; ++o) {
                T x = 0;
#pragma unroll
                for (int z = 0; z < FL; ++z) x += r[o + z] * zf[z];
                x = pc_clamp(x);
                x = nrm(x);
                v[o] = x;
            }
            if (gi < X && gy < Y) {
                const int gk0 = ly.k0 + j * VEC, nv = min(VEC, ly.nout - j * VEC);
                const size_t e0 = ((size_t)gi * Y + gy) * TH + gk0;
                if (nv == VEC && e0 % VEC == 0) {
                    co_put(P, e0, v, wt, nbytes);
                } else {  // a ragged or unaligned group (TH or the chunk not a multiple of VEC)
#pragma unroll
                    for (int o = 0; o < VEC; ++o)
                        if (o < nv) P[e0 + o] = v[o];
                }
#pragma unroll
                for (int o = 0; o < VEC; ++o) {
                    if (o >= nv) break;
                    const unsigned lin = (unsigned)(e0 + o);
                    if constexpr (sizeof(T) == 4) {
                        bk = max(bk, argmax_key((float)v[o], lin));
                    } else if (pc_better(v[o], lin, bv, bl)) {
                        bv = v[o];
                        bl = lin;
                    }
                }
            }
        }
    }
    if constexpr (sizeof(T) == 4) {
        __shared__ unsigned long long s_bk[NW];
        bk = co_wave_max(bk);
        if (lane == 0) s_bk[wave] = bk;
        co_lds_barrier();
        if (tid == 0) {
            for (int w = 1; w < NW; ++w) bk = max(bk, s_bk[w]);
            atomicMax(res_slot + (blockIdx.x & (RES_SLOTS - 1)), bk);
        }
    } else {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const T ov = __shfl_xor(bv, off);
            const unsigned ol = __shfl_xor(bl, off);
            if (pc_better(ov, ol, bv, bl)) {
                bv = ov;
                bl = ol;
            }
        }
        if (lane == 0) {
            s_bv[wave] = bv;
            s_bl[wave] = bl;
        }
        co_lds_barrier();
        if (tid == 0) {
            for (int w = 1; w < NW; ++w)
                if (pc_better(s_bv[w], s_bl[w], bv, bl)) {
                    bv = s_bv[w];
                    bl = s_bl[w];
                }
            bmax[blockIdx.x] = bv;
            bidx[blockIdx.x] = bl;
        }
    }
    PC_STAMP(6, 4);
}

// ---------------------------------------------------------------------------
// Halo form: ONE launch per step (float32; X, Y >= HF_W; TH == HF_TH).
//
// The reference's step (posecell_network.py:326-353) has one global dependency, the
// normalisation total (:343-345), and two local ones: the excitation's 3-cell halo
// (:336) and the path filter's shifted 7 x 7 window (:273).  The two-launch forms
// hand the excited volume Q from one kernel to the next through memory.  Here a
// block recomputes the excitation on its halo instead, so the only hand-off left is
// the one a kernel boundary gives for free: the state and its total.
//  * Between the launches of a batch the state is kept UNNORMALISED,
//    U = relu(conv_z(relu(conv_xy(Q)))), with the per-block partial sums of the
//    total t of Q (max(conv(Q/t), 0) = max(conv(Q), 0)/t for t > 0, which the
//    two-launch forms use too).  The next launch sums the partials and forms
//    P = U * (1/t) as it loads: the same product
//    the two-launch path kernels apply before their store, so P is the same.
//  * The argmax of a step (:317-319) is taken from those scaled values, exactly the
//    values of the state: by the next launch over its own tile, and for the last step
//    of a call by pc_halo_finish, which also stores the normalised state (between
//    calls the handle's state is normalised, as in every other form) and exports the
//    keys of all steps to the host (its last block, by an agent-scope counter).
//  * A block owns a 4 x 4 tile through all TH layers (256 blocks at 64 x 64).  Layer
//    j's path output needs Q on the 10 x 10 window shifted by the layer's (ox, oy),
//    and that Q needs P on the 16 x 16 window around it.  The excitation runs theta
//    pass first: the union of the step's shifted 16 x 16 windows goes global -> LDS
//    by LDS-DMA (each cell's theta column is contiguous, theta-fastest C order, so the
//    pieces are whole 1 KiB runs per wave-instruction); the theta pass reads it in
//    place, a lane per window cell through a run of layers (phase 2 below); then per
//    layer on its own window the y pass (16 x 10), the x pass (10 x 10) with the
//    inhibition, the 7 x 7 path filter and clamp, the theta filter and clamp, and the
//    write-through store.
//  * The partial sums cover, for layer j, the block's tile shifted by layer j's
//    shift (the centre of its Q window): those shifted tiles partition each layer as
//    the tiles do.
// ---------------------------------------------------------------------------
constexpr int HF_T = 4;                       // tile: HF_T x HF_T cells through all layers
constexpr int HF_W = HF_T + 4 * HALF;         // 16: a layer's excitation window
constexpr int HF_Q = HF_T + 2 * HALF;         // 10: a layer's excited (Q) window
constexpr int HF_NW = 9, HF_NT = 64 * HF_NW;  // 576 threads: one task per (layer, window row) at TH = 36
constexpr int HF_TH = 36;                     // the theta extent instantiated (configs[1], the ROS node)
constexpr int HF_UMAX = 22 * 22;              // union cells staged by LDS-DMA (|shifts| spread <= 6)
// theta-pass windows, (e, i) pairs [j][rx][ry], row pitch 18 pairs: the y pass's 16-byte
// row reads (16 lanes on consecutive rows, 36 dwords apart) are conflict-free
constexpr int HF_WP = 18, HF_WJ = HF_W * HF_WP;
constexpr int HF_YC = HF_W + 4;               // y-pass outputs per Q column (16 rows, 16-byte aligned)
constexpr int HF_YL = HF_Q * HF_YC;           // ... per layer, [qc][rx]
constexpr int HF_QJ = HF_Q * HF_Q + 4;        // Q window per layer
constexpr int HF_EXP_MAX = 64;                // steps whose keys pc_halo_finish exports itself
constexpr float HF_NEAR = 0x1p-20f;           // relative margin of a possible rounding tie (pc_halo_export)
// A step's result word when its last-step records cannot settle the first maximum of the
// scaled state (a cell within HF_NEAR of the maximum): never a valid key (a key's low
// word is ~lin >= 2, lin < X*Y*TH < 2^32 - 1, rs_pc_create)
constexpr unsigned long long RES_AMBIG = 1ull;
constexpr unsigned long long REC_SET = 1ull << 63;   // a record's count word: REC_SET | count
// calls of at most this many steps poll their result words (pc_poll_words); longer ones
// wait in the stream synchronisation with the CPU idle (a 4,000-step run: 9.13 polled vs
// 9.02 us per step synchronised, tools/pc_ab.py, round 5)
constexpr int HF_POLL_MAX = 64;
constexpr int HF_FLAGS = 1024;   // pc_halo_finish blocks' flags in pinned host memory

// One step's control, a kernel argument (formed on the host by make_ctl_halo).
struct PcCtlHalo {
    short sx[HF_TH], sy[HF_TH];  // layer j's 16 x 16 window starts at union row sx[j], column sy[j]
    unsigned char fo[HF_TH];     // layer j's path filter (row of the filter table)
    float zf[FL];                // theta filter (posecell_network.py:308)
    short ux, uy;                // union origin = tile origin - 6 + the smallest centred shift
    short uw, uh;                // union extent in cells (at most X, Y)
    int wrap;                    // the union is a whole period in x or y (windows wrap inside it)
};
typedef float hf_f2 __attribute__((ext_vector_type(2)));  // (excitatory, inhibitory) pairs: packed FMAs
// two 16-bit fields in one kernel argument (pc_step_halo's preloaded union origin / extent)
inline int hf_pack(short lo, short hi) {
    return (int)((unsigned)(unsigned short)lo | ((unsigned)(unsigned short)hi << 16));
}

// The normalisation total of a step from its per-block partials, formed by every wave
// itself in one fixed order (so every block gets the same bits): 4 per lane, then DPP.
// Split in two so a kernel can issue the loads first and sum them later, behind other
// loads already in flight (pc_step_halo).
__device__ inline void pc_partials_issue(const double* __restrict__ part, int npart, double (&pt)[4]) {
    const int lane = threadIdx.x & 63, np1 = npart > 0 ? npart - 1 : 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) pt[u] = part[min(lane + 64 * u, np1)];  // unconditional
}
__device__ inline double pc_partials_sum(const double* __restrict__ part, int npart, const double (&pt)[4]) {
    const int lane = threadIdx.x & 63;
    double tot = 0.0;
#pragma unroll
    for (int u = 0; u < 4; ++u) tot += lane + 64 * u < npart ? pt[u] : 0.0;
    for (int i = lane + 256; i < npart; i += 64) tot += part[i];
    return co_wave_sum(tot);
}
__device__ inline double pc_partials_total(const double* __restrict__ part, int npart) {
    double pt[4];
    pc_partials_issue(part, npart, pt);
    return pc_partials_sum(part, npart, pt);
}
// q = n / d for n, d < 2^16, d >= 2, by one high multiply with m = hf_magic(d): the error
// of m / 2^32 against 1 / d is below 2^-32, so n * m / 2^32 stays below the next integer
// when n < 2^32 / d
inline unsigned hf_magic(int d) { return (unsigned)(0xFFFFFFFFull / (unsigned)d + 1ull); }

// EXC: excitation only (rs_pc_excite, the step the reference runs before a LUT
// KeyError): zero shifts, Q of the own cells stored into Uo (theta-fastest), partials.
// The first HF_PRELOAD arguments are everything the union image's LDS-DMA addresses
// need (the state, the grid, the block count, the union's origin and extent packed
// as 16-bit pairs): posecell.hip is built with -amdgpu-kernarg-preload-count, so they
// arrive in scalar registers with the wave and the image's loads issue without a
// kernel-argument round trip (two dependent ones before: the block count, then the
// union, 0.84 us from the block's start to the DMA issue at 64 x 64 x 36).
template <bool EXC, int TH>
__global__ __launch_bounds__(HF_NT) void pc_step_halo(
    const float* __restrict__ U, int xy, int gxnb, int ulo, int uext, unsigned mgx, unsigned muh,
    const double* __restrict__ part_in, int npart_in, float* __restrict__ Uo, double* __restrict__ part_out,
    unsigned long long* __restrict__ slot_prev, unsigned long long* __restrict__ slot_zero,
    const float* __restrict__ filt, int nf, PcCtlHalo ctl, SepKernel<float> k,
    unsigned long long* __restrict__ rec) {
    // TH: 36 (configs[1], the ROS node: the tuned phases below), or another even extent up
    // to HF_TH (18: configs[0]'s grid, 10: simulate.py's), whose theta columns are not
    // whole 16-byte pieces: the image then loads in 4-byte pieces, the theta pass runs a
    // thread per union cell (cell_pass below) and the theta filter in 2-layer groups
    static_assert(TH % 2 == 0 && TH >= FL + HALF && TH <= HF_TH, "an even theta extent, 10 .. HF_TH");
    constexpr bool V4 = TH % 4 == 0;
    constexpr int PW = V4 ? 4 : 1, NV = TH / PW;   // image pieces (PW floats each) per theta column
    constexpr int WBUF = HF_UMAX * TH + 64 * 4;   // union image [cell][layer] (+ a wave-instruction of slack)
    constexpr int YBUF = 2 * TH * HF_YL;
    constexpr int BBUF = WBUF > YBUF ? WBUF : YBUF;
    constexpr int PP = TH + 64;   // path outputs per cell: rows TH dwords apart modulo the 64 banks
    static_assert(HF_T * HF_T * PP <= BBUF && TH * HF_QJ <= 2 * TH * HF_WJ, "buffer reuse");
    // theta-pass (e, i) windows, then a dump slot per thread (a lane outside a layer's
    // window stores there: no branch); then Q
    __shared__ __attribute__((aligned(16))) float s_t[2 * (TH * HF_WJ + HF_NT)];
    __shared__ __attribute__((aligned(16))) float s_b[BBUF];  // union image; then y pass e | i; then path outputs
    __shared__ __attribute__((aligned(16))) float s_ftab[RT_NFMAX * ST_FTP];
    __shared__ int s_fo[TH];
    __shared__ double s_red[HF_NW];
    __shared__ unsigned long long s_rk[HF_NW];
    __shared__ int s_cnt[HF_NW];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int X = xy & 0xFFFF, Y = (int)((unsigned)xy >> 16), gx = gxnb & 0xFFFF, nblk = (int)((unsigned)gxnb >> 16);
    const int tile = st_tile(blockIdx.x, nblk);
    const int ty = (int)__umulhi((unsigned)tile, mgx);   // tile / gx (hf_magic)
    const int x0 = (tile - ty * gx) * HF_T, y0 = ty * HF_T;
    const int tw = min(HF_T, X - x0), tht = min(HF_T, Y - y0);
    const int cux = (short)(ulo & 0xFFFF), cuy = ulo >> 16;   // the union's origin (centred shifts)
    const int UW = uext & 0xFFFF, UH = uext >> 16, nu = UW * UH;
    const int ux0 = co_wrap(x0 - 2 * HALF + cux, X), uy0 = co_wrap(y0 - 2 * HALF + cuy, Y);
    const bool dma = nu <= HF_UMAX;
    PC_STAMP(7, 0);
    // the partial sums of the state entering the step, issued ahead of the union image so
    // they land first and the total is formed while the image is in flight
    double pt[4];
    pc_partials_issue(part_in, npart_in, pt);
    // 1. the union image, issued first: piece p = tid + HF_NT * r is piece p % NVU of union
    //    unit p / NVU (a unit: UC cells of one union row, units row-major, UH / UC per row),
    //    landing at s_b + PWU p.  TH % 4 == 0: a unit is a cell of TH / 4 16-byte pieces.
    //    Otherwise, when the host made the union's start column and width even (and Y is
    //    even: make_ctl_halo), a unit is a cell pair, 2 TH floats from an even cell, 16-byte
    //    aligned (TH / 2 16-byte pieces); else a cell of TH 4-byte pieces.
    auto issue = [&](auto pw_c, auto nvu_c, auto uc_c) __attribute__((always_inline)) {
        constexpr int PWU = decltype(pw_c)::value, NVU = decltype(nvu_c)::value, UC = decltype(uc_c)::value;
        constexpr int DC = HF_NT / NVU, DL = HF_NT % NVU, NR = (HF_UMAX / UC * NVU + HF_NT - 1) / HF_NT;
        // A lane walks its pieces with full-rate 32-bit arithmetic only (no 64-bit,
        // quarter-rate address math; measured neutral: the issue, about 0.95 us from the
        // block's start at 64 x 64 x 36, is not VALU-bound, r4 probe): the row's first cell rb =
        // gr * Y carried incrementally (the union row advances by dU or dU + 1 < X per
        // round and UW <= X, so one wrap suffices), a 32-bit byte offset from the state's
        // base (n * 4 <= INT_MAX, pc_halo_fit) by a 24-bit multiply (cells < 2^24).
        // Units per row: UH / UC, by the same high multiply (UC c / UH, c < 2^15)
        const int UHU = UH / UC, npc = nu / UC * NVU, XY = X * Y;
        const int dU = (int)__umulhi((unsigned)(UC * DC), muh), dV = DC - dU * UHU;
        int c = tid / NVU, l4 = tid - c * NVU, ui = (int)__umulhi((unsigned)(UC * c), muh), vi = c - ui * UHU;
        int rb = ux0 + ui;
        rb = (rb >= X ? rb - X : rb) * Y;
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const int i0 = r * HF_NT + wave * 64;  // wave-uniform
            if (i0 < npc) {
                if (i0 + lane < npc) {
                    int gc = uy0 + UC * vi;
                    gc -= gc >= Y ? Y : 0;
                    const unsigned boff = __umul24((unsigned)(rb + gc), (unsigned)(4 * TH)) + 4u * PWU * (unsigned)l4;
                    const auto gsrc = (__attribute__((address_space(1))) const void*)(reinterpret_cast<const char*>(U) + boff);
                    const auto ldst = (__attribute__((address_space(3))) void*)(s_b + PWU * i0);
                    if constexpr (PWU == 4) __builtin_amdgcn_global_load_lds(gsrc, ldst, 16, 0, 0);
                    else __builtin_amdgcn_global_load_lds(gsrc, ldst, 4, 0, 0);
                }
            }
            l4 += DL;
            vi += dV;
            rb += dU * Y;
            if (l4 >= NVU) {
                l4 -= NVU;
                ++vi;
            }
            if (vi >= UHU) {
                vi -= UHU;
                rb += Y;
            }
            rb -= rb >= XY ? XY : 0;
        }
    };
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I4 = std::integral_constant<int, 4>;
    if (dma) {
        if constexpr (V4) {
            issue(I4{}, std::integral_constant<int, TH / 4>{}, I1{});
        } else {
            if (((cuy | UH | Y) & 1) == 0) issue(I4{}, std::integral_constant<int, TH / 2>{}, I2{});
            else issue(I1{}, std::integral_constant<int, TH>{}, I1{});
        }
    }
    PC_STAMP(10, 0);
    // the normalisation of the state entering the step, the filter table, the control
    // (lane L of every wave holds layer L's window start, read by readlane in phase 2)
    const int lsx = ctl.sx[lane < TH ? lane : 0], lsy = ctl.sy[lane < TH ? lane : 0];
    const float fr = tid < nf * FT ? filt[tid] : 0.f;
    static_assert(RT_NFMAX * FT <= HF_NT, "one filter tap per thread");
    if (tid < TH) s_fo[tid] = ctl.fo[tid] * ST_FTP;
    const PcNorm<float> nrm(pc_partials_sum(part_in, npart_in, pt));
    if (tid < nf * FT) s_ftab[(tid / FT) * ST_FTP + tid % FT] = fr;
    // the tap pairs and the wrap flag (kernel arguments beyond the preloaded ones) in
    // registers before the barrier: hipcc otherwise loads them after it, a scalar round
    // trip at the head of phase 2
    hf_f2 gei[FL];
#pragma unroll
    for (int t = 0; t < FL; ++t) {
        gei[t] = hf_f2{k.ge[t], k.gi[t]};
        asm volatile("" : "+s"(gei[t]));
    }
    int cwrap = ctl.wrap;
    asm volatile("" : "+s"(cwrap));
    // likewise the inhibition's constants (phase 4) and the theta filter (phase 6)
    float kscale = k.scale, kinhib = k.inhib, zf[FL];
    asm volatile("" : "+s"(kscale), "+s"(kinhib));
#pragma unroll
    for (int z = 0; z < FL; ++z) {
        zf[z] = ctl.zf[z];
        asm volatile("" : "+s"(zf[z]));
    }
    if (slot_zero != nullptr && blockIdx.x == 0)
        for (int i = tid; i < RES_SLOTS; i += HF_NT) st_wt(&slot_zero[i], 0ull);  // the next launch max-reduces into them
    if (dma) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's LDS-DMA pieces have landed
    PC_STAMP(10, 1);
    co_lds_barrier();
    PC_STAMP(7, 1);

    // 2. the theta pass of both Gaussians, as packed (e, i) FMAs, into the layers'
    //    windows [j][rx][ry] (row pitch HF_WP).
    hf_f2* s_tw = reinterpret_cast<hf_f2*>(s_t);
    unsigned long long bk = 0ull;
    const bool want_key = slot_prev != nullptr;
    PC_STAMP(11, 0);
    // a thread per union cell (theta extents other than HF_TH; at HF_TH a union larger
    // than the LDS-DMA image)
    auto cell_passes = [&]() __attribute__((always_inline)) {
        // a union spanning a whole period (the windows wrap inside it), or one larger
        // than the LDS-DMA image (columns from memory): thread c takes union cell c's
        // column, scales it, forms all TH theta-pass outputs in registers and stores
        // those of the windows holding the cell (a lane outside a window stores into its
        // own dump slot, a select rather than a branch, so the layers' FMA chains share
        // one basic block and interleave).  The own tile's keys: wave 8 when the union
        // is in LDS (below; HF_UMAX < 512, so wave 8 holds no union cell), else here.
        static_assert(HF_UMAX <= 8 * 64, "wave 8 takes no union cell");
        auto cell_pass = [&](int c, auto wrap_c) __attribute__((always_inline)) {
            constexpr bool WRAP = decltype(wrap_c)::value;
            const int ui = (int)__umulhi((unsigned)c, muh), vi = c - ui * UH;   // c / UH (hf_magic)
            const int cw = ui * HF_WP + vi, dump = TH * HF_WJ + tid;
            // (no wrap) lane L: layer L's window start as packed 16-bit (x, y), and the
            // byte offset of its window cell (0, 0) in layer 0's window image; the lane's
            // cell, packed and in bytes (pinned: one subtraction per layer each)
            const int lsp = (lsx << 16) + lsy, lso8 = 8 * (lsx * HF_WP + lsy - lane * HF_WJ);
            int uvp = (ui << 16) + vi, cw8 = 8 * cw;
            asm volatile("" : "+v"(uvp), "+v"(cw8));
            const int dump8 = 8 * dump;
            int gr = ux0 + ui, gc = uy0 + vi;
            gr -= gr >= X ? X : 0;
            gc -= gc >= Y ? Y : 0;
            float p[TH];
            // the column as 16-byte vectors (TH % 4 == 0) or 8-byte pairs (TH even: a
            // column starts 8-byte aligned)
            using CV = typename std::conditional<V4, co_f4, hf_f2>::type;
            constexpr int CW = V4 ? 4 : 2;
            auto rd = [&](const float* base) __attribute__((always_inline)) {
                const CV* src = reinterpret_cast<const CV*>(base);
#pragma unroll
                for (int v = 0; v < TH / CW; ++v) {
                    const CV x = src[v];
#pragma unroll
                    for (int w = 0; w < CW; ++w) p[CW * v + w] = x[w];
                }
            };
            if (dma) rd(s_b + c * TH);
            else rd(U + ((size_t)gr * Y + gc) * TH);
            nrm(p);
            if (want_key && !dma && (unsigned)(gr - x0) < (unsigned)tw && (unsigned)(gc - y0) < (unsigned)tht) {
                const unsigned lin0 = ((unsigned)gr * Y + gc) * TH;
#pragma unroll
                for (int q = 0; q < TH; ++q) bk = max(bk, argmax_key(p[q], lin0 + q));
            }
            auto store = [&](int j, hf_f2 eg) __attribute__((always_inline)) {
                if constexpr (WRAP) {
                    const int sxj = __builtin_amdgcn_readlane(lsx, j), syj = __builtin_amdgcn_readlane(lsy, j);
                    int rx = ui - sxj, ry = vi - syj;
                    rx += rx < 0 ? UW : 0;
                    ry += ry < 0 ? UH : 0;
                    const int a = j * HF_WJ + (int)__umul24((unsigned)rx, (unsigned)HF_WP) + ry;
                    s_tw[max((unsigned)rx, (unsigned)ry) < (unsigned)HF_W ? a : dump] = eg;
                } else {
                    // in the window: both 16-bit fields of the packed difference in [0, 16)
                    // (a negative y part borrows into bits 4-15 of the low field);
                    // |coordinates| < 2^15
                    static_assert(HF_W == 16, "the packed window test");
                    const int d = uvp - __builtin_amdgcn_readlane(lsp, j);
                    const int a8 = cw8 - __builtin_amdgcn_readlane(lso8, j);
                    *reinterpret_cast<hf_f2*>(reinterpret_cast<char*>(s_tw) + ((d & 0xFFF0FFF0) == 0 ? a8 : dump8)) = eg;
                }
            };
            // layers in pairs: two independent FMA chains interleaved
#pragma unroll
            for (int j = 0; j < TH; j += 2) {
                hf_f2 ea = {0.f, 0.f}, eb = {0.f, 0.f};
#pragma unroll
                for (int t = 0; t < FL; ++t) {
                    ea += gei[t] * p[(j + t + TH - HALF) % TH];
                    eb += gei[t] * p[(j + 1 + t + TH - HALF) % TH];
                }
                store(j, ea);
                store(j + 1, eb);
            }
        };
        if (cwrap) {
#pragma unroll 1
            for (int c = tid; c < nu; c += HF_NT) cell_pass(c, std::true_type{});
        } else {
#pragma unroll 1
            for (int c = tid; c < nu; c += HF_NT) cell_pass(c, std::false_type{});
        }
    };
    if constexpr (TH == HF_TH) {
      if (dma) {
        // the common case, read straight from the union image [cell][layer]: wave w < 8
        // takes window rows 4(w&3) .. +3 (a lane per window cell) through the layers
        // [18(w>>2), +18).  Layer j's window cell (rx, ry) is union cell (rx + sx_j,
        // ry + sy_j); its 7 theta taps are 7 consecutive floats of that cell's column,
        // held as 16-byte quads of the column in registers (conflict-free reads: lanes
        // 144 bytes apart).  While the shift stays the layer before's, a layer needs at
        // most one new quad, read PF layers ahead; a layer with a new shift (a
        // wave-uniform branch, a few per run) reloads the quads its taps and the next
        // PF layers' reach.  Each quad is scaled by 1/t as it arrives (the same products
        // as every other form's); every lane's store is one of a window's own cells.
        if (nrm.div) {   // 1/t not finite (t tiny): divide the image in place first
            for (int c = tid; c < nu; c += HF_NT) {
                co_f4* col = reinterpret_cast<co_f4*>(s_b + c * TH);
#pragma unroll
                for (int v = 0; v < NV; ++v) {
                    co_f4 x = col[v];
#pragma unroll
                    for (int w = 0; w < 4; ++w) x[w] = nrm(x[w]);
                    col[v] = x;
                }
            }
            co_lds_barrier();
        }
        if (wave < 8) {
            constexpr int JH = TH / 2, PF = 3;
            const int rx = 4 * (wave & 3) + (lane >> 4), ry = lane & 15;
            const int loff = (lsx * UH + lsy) * TH;   // lane L: layer L's window place in the union
            const int cbase = (rx * UH + ry) * TH;
            auto run = [&](auto hh, auto wc) __attribute__((always_inline)) {
                constexpr int J0 = decltype(hh)::value * JH;
                constexpr bool WRAP = decltype(wc)::value;
                // quads kq = 0 .. NQ-1 hold layers 4 (QB + kq) .. +3 (mod TH) of the current cell
                constexpr int QB = (J0 - HALF + 4 * TH) / 4 - TH, NQ = (J0 + JH - 1 + HALF - 4 * QB) / 4 + 1;
                co_f4 qd[NQ];
                hf_f2* dst = s_tw + J0 * HF_WJ + (rx * HF_WP + ry);
                // a union spanning a whole period (cwrap: 16 + the shifts' spread exceeds X
                // or Y, so the union is the period): window cell (rx, ry) of layer j is
                // union cell ((rx + sx_j) mod UW, (ry + sy_j) mod UH); else no wrap occurs
                auto colof = [&](int j) __attribute__((always_inline)) {
                    int ux = rx + __builtin_amdgcn_readlane(lsx, j), uy = ry + __builtin_amdgcn_readlane(lsy, j);
                    ux -= ux >= UW ? UW : 0;
                    uy -= uy >= UH ? UH : 0;
                    return s_b + (ux * UH + uy) * TH;
                };
                int prev = __builtin_amdgcn_readlane(loff, J0);
                const float* col = WRAP ? colof(J0) : s_b + cbase + prev;
                auto ld = [&](int kq) {
                    qd[kq] = *reinterpret_cast<const co_f4*>(col + ((4 * (QB + kq) + 4 * TH) % TH)) * nrm.r;
                };
                // quads holding layers lo .. hi (relative to 4 QB), clipped to the run
                auto ld_span = [&](int lo, int hi) __attribute__((always_inline)) {
#pragma unroll
                    for (int kq = 0; kq < NQ; ++kq)
                        if (4 * kq + 3 >= lo && 4 * kq <= hi) ld(kq);
                };
                ld_span(J0 - HALF - 4 * QB, J0 + HALF + PF - 4 * QB);
                auto tapv = [&](int e) { return qd[e / 4][e % 4]; };
                // layer jj's taps (first tap e0 relative to 4 QB) in the reference's order
                auto one = [&](int jj) __attribute__((always_inline)) {
                    const int e0 = J0 + jj - HALF - 4 * QB;
                    hf_f2 eg = {0.f, 0.f};
#pragma unroll
                    for (int t = 0; t < FL; ++t) eg += gei[t] * tapv(e0 + t);
                    dst[jj * HF_WJ] = eg;
                };
                // the new shift of layer jj, if any; else the quad its taps reach PF layers on
                auto enter = [&](int jj, int o) __attribute__((always_inline)) {
                    const int e0 = J0 + jj - HALF - 4 * QB;
                    if (o == prev) {
                        const int e = e0 + 2 * HALF + PF;
                        if (e % 4 == 0 && e / 4 < NQ) ld(e / 4);
                    } else {
                        prev = o;
                        col = WRAP ? colof(J0 + jj) : s_b + cbase + o;
                        ld_span(e0, e0 + 2 * HALF + PF);
                    }
                };
                // layers in pairs: two independent FMA chains interleaved, unless the
                // second layer of the pair takes a new shift (then one after the other,
                // the first before its quads are replaced)
                static_assert(JH % 2 == 0, "layer pairs");
#pragma unroll
                for (int jj = 0; jj < JH; jj += 2) {
                    if (jj > 0) enter(jj, __builtin_amdgcn_readlane(loff, J0 + jj));
                    const int o1 = __builtin_amdgcn_readlane(loff, J0 + jj + 1);
                    if (o1 == prev) {
                        enter(jj + 1, o1);
                        const int e0 = J0 + jj - HALF - 4 * QB;
                        hf_f2 ea = {0.f, 0.f}, eb = {0.f, 0.f};
#pragma unroll
                        for (int t = 0; t < FL; ++t) {
                            ea += gei[t] * tapv(e0 + t);
                            eb += gei[t] * tapv(e0 + 1 + t);
                        }
                        dst[jj * HF_WJ] = ea;
                        dst[(jj + 1) * HF_WJ] = eb;
                    } else {
                        one(jj);
                        enter(jj + 1, o1);
                        one(jj + 1);
                    }
                }
            };
            // (separate code for a wrapped union, so the common case keeps its registers)
            if (!cwrap) {
                if (wave < 4) run(std::integral_constant<int, 0>{}, std::false_type{});
                else run(std::integral_constant<int, 1>{}, std::false_type{});
            } else {
                if (wave < 4) run(std::integral_constant<int, 0>{}, std::true_type{});
                else run(std::integral_constant<int, 1>{}, std::true_type{});
            }
        } else if (want_key) {
            // wave 8: the argmax of the state entering the step over the own tile (lane:
            // cell lane & 15, quads lane >> 4 + 4 m)
            const int i = (lane & 15) >> 2, jc = lane & 3;
            int cu = co_wrap(2 * HALF - cux, X) + i, cv = co_wrap(2 * HALF - cuy, Y) + jc;
            cu -= cu >= X ? X : 0;
            cv -= cv >= Y ? Y : 0;
            if (i < tw && jc < tht && cu < UW && cv < UH) {
                const unsigned lin0 = ((unsigned)(x0 + i) * Y + (y0 + jc)) * TH;
                const co_f4* src = reinterpret_cast<const co_f4*>(s_b + (cu * UH + cv) * TH);
                for (int v = lane >> 4; v < NV; v += 4) {
                    const co_f4 x = src[v];
#pragma unroll
                    for (int w = 0; w < 4; ++w) bk = max(bk, argmax_key(x[w] * nrm.r, lin0 + 4 * v + w));  // (r = 1 once divided)
                }
            }
        }
      } else {
        cell_passes();
      }
    } else {
        cell_passes();
        if (dma && want_key && wave == 8) {
            // the own tile's keys from the image, off the cell-pass waves (lane: cell
            // lane & 15, layers lane >> 4 + 4 m), scaled as cell_pass scales
            const int i = (lane & 15) >> 2, jc = lane & 3;
            int cu = co_wrap(2 * HALF - cux, X) + i, cv = co_wrap(2 * HALF - cuy, Y) + jc;
            cu -= cu >= X ? X : 0;
            cv -= cv >= Y ? Y : 0;
            if (i < tw && jc < tht && cu < UW && cv < UH) {
                const unsigned lin0 = ((unsigned)(x0 + i) * Y + (y0 + jc)) * TH;
                const float* src = s_b + (cu * UH + cv) * TH;
                for (int q = lane >> 4; q < TH; q += 4) bk = max(bk, argmax_key(nrm(src[q]), lin0 + q));
            }
        }
    }
    PC_STAMP(11, 1);
    PC_STAMPW(12);
    if (want_key && tid < tw * tht) {
        // an own cell outside the union (a large uniform shift): its key from memory
        const int i = tid / tht, j = tid - i * tht;
        int cu = co_wrap(2 * HALF - cux, X) + i, cv = co_wrap(2 * HALF - cuy, Y) + j;
        cu -= cu >= X ? X : 0;
        cv -= cv >= Y ? Y : 0;
        if (cu >= UW || cv >= UH) {
            const unsigned lin0 = ((unsigned)(x0 + i) * Y + (y0 + j)) * TH;
            using CV = typename std::conditional<V4, co_f4, hf_f2>::type;
            constexpr int CW = V4 ? 4 : 2;
            const CV* src = reinterpret_cast<const CV*>(U + lin0);
#pragma unroll
            for (int v = 0; v < TH / CW; ++v) {
                const CV x = src[v];
#pragma unroll
                for (int w = 0; w < CW; ++w) bk = max(bk, argmax_key(nrm(x[w]), lin0 + CW * v + w));
            }
        }
    }
    co_lds_barrier();
    PC_STAMP(7, 2);

    // 3. y pass: task (layer j, window row rx) -> 10 outputs of each Gaussian, stored
    //    transposed, [j][qc][rx] (column pitch HF_YC), so that the x pass reads each
    //    column as four 16-byte vectors (conflict-free: lanes on consecutive columns are
    //    20 dwords apart, layers HF_YL apart)
    float* s_ye = s_b;
    float* s_yi = s_b + TH * HF_YL;
    // task (layer j, row rx, outputs QC0 .. QC0 + NQ - 1); the SIMDs are balanced (wave w
    // runs on SIMD w % 4): waves 0-7 take layers 0-31 whole, one wave per SIMD (8, 5, 6, 7)
    // a part of layers 32-35 (576 whole tasks on 9 waves put three on SIMD 0)
    auto ytask = [&](int j, int rx, auto qc0_c, auto nq_c) __attribute__((always_inline)) {
        constexpr int QC0 = decltype(qc0_c)::value, NQ = decltype(nq_c)::value;
        const co_f4* rw = reinterpret_cast<const co_f4*>(s_tw + j * HF_WJ + rx * HF_WP);
        hf_f2 w[HF_W];   // (e, i) of the row's 16 cells (those the outputs reach)
#pragma unroll
        for (int q = QC0 / 2; q <= (QC0 + NQ + 2 * HALF - 1) / 2; ++q) {
            const co_f4 a = rw[q];
            w[2 * q] = hf_f2{a.x, a.y};
            w[2 * q + 1] = hf_f2{a.z, a.w};
        }
        float* de = s_ye + j * HF_YL + rx;
        float* di = s_yi + j * HF_YL + rx;
#pragma unroll
        for (int qc = QC0; qc < QC0 + NQ; ++qc) {
            hf_f2 eg = {0.f, 0.f};
#pragma unroll
            for (int t2 = 0; t2 < FL; ++t2) eg += gei[t2] * w[qc + t2];
            de[qc * HF_YC] = eg.x;
            di[qc * HF_YC] = eg.y;
        }
    };
    static_assert(HF_W == 16 && HF_Q == 10 && HF_NW == 9, "phase 3's task split");
    if constexpr (TH == 18) {
        // waves 0-3 take layers 0-15 whole, one wave per SIMD; layers 16-17 go in 4-, 3-
        // and 3-output pieces to waves 5, 6, 7 (SIMDs 1-3): 288 whole tasks on 5 waves
        // put two on SIMD 0
        using I = std::integral_constant<int, 0>;
        if (wave < 4) ytask(tid >> 4, tid & 15, I{}, std::integral_constant<int, HF_Q>{});
        const int jr = 16 + ((lane >> 4) & 1), rr = lane & 15;
        if (lane < 32) {
            if (wave == 5) ytask(jr, rr, I{}, std::integral_constant<int, 4>{});
            else if (wave == 6) ytask(jr, rr, std::integral_constant<int, 4>{}, std::integral_constant<int, 3>{});
            else if (wave == 7) ytask(jr, rr, std::integral_constant<int, 7>{}, std::integral_constant<int, 3>{});
        }
    } else if constexpr (TH != 36) {
        for (int t = tid; t < TH * HF_W; t += HF_NT)
            ytask(t >> 4, t & 15, std::integral_constant<int, 0>{}, std::integral_constant<int, HF_Q>{});
    } else {
        using I = std::integral_constant<int, 0>;
        if (wave < 8) ytask(tid >> 4, tid & 15, I{}, std::integral_constant<int, HF_Q>{});
        const int jr = 32 + (lane >> 4), rr = lane & 15;
        if (wave == 8) ytask(jr, rr, I{}, std::integral_constant<int, 3>{});
        else if (wave == 5) ytask(jr, rr, std::integral_constant<int, 3>{}, std::integral_constant<int, 3>{});
        else if (wave == 6) ytask(jr, rr, std::integral_constant<int, 6>{}, std::integral_constant<int, 2>{});
        else if (wave == 7) ytask(jr, rr, std::integral_constant<int, 8>{}, std::integral_constant<int, 2>{});
    }
    co_lds_barrier();
    PC_STAMP(7, 3);

    // 4. x pass + inhibition (:339-340): task (layer j, Q column qc) -> 10 Q values;
    //    the partial sum over the layer's shifted own tile (Q rows/columns 3 .. 3+tw)
    float* s_q = s_t;
    double qs = 0.0;
    // task (layer j, Q column qc, Q rows 5H .. 5H + 4), H-uniform per wave; the SIMDs are
    // balanced: H = 0 on waves 0-5, H = 1 on waves 8, 6, 7, 1, 2, 3 (three 5-row tasks
    // per SIMD, where 360 10-row tasks on 6 waves put two on SIMDs 0 and 1)
    auto xtask = [&](int t, auto h_c) __attribute__((always_inline)) {
        constexpr int H = decltype(h_c)::value;
        if (t >= TH * HF_Q) return;
        const int j = t / HF_Q, qc = t - j * HF_Q;
        const co_f4* ce = reinterpret_cast<const co_f4*>(s_ye + j * HF_YL + qc * HF_YC) + H;
        const co_f4* ci = reinterpret_cast<const co_f4*>(s_yi + j * HF_YL + qc * HF_YC) + H;
        hf_f2 w[12];   // rows 4H .. 4H + 11
#pragma unroll
        for (int r4 = 0; r4 < 3; ++r4) {
            const co_f4 a = ce[r4], b = ci[r4];
#pragma unroll
            for (int u = 0; u < 4; ++u) w[4 * r4 + u] = hf_f2{a[u], b[u]};
        }
        const bool ocol = (unsigned)(qc - HALF) < (unsigned)tht;
#pragma unroll
        for (int o = 0; o < 5; ++o) {
            const int qa = 5 * H + o;
            hf_f2 eg = {0.f, 0.f};
#pragma unroll
            for (int a = 0; a < FL; ++a) eg += gei[a] * w[H + o + a];
            const float v = (eg.x - eg.y) * kscale;
            const float q = (v < kinhib) ? 0.f : v - kinhib;
            const bool own = ocol && (unsigned)(qa - HALF) < (unsigned)tw;
            if (own) qs += (double)q;
            if constexpr (EXC) {
                if (own) Uo[((size_t)(x0 + qa - HALF) * Y + (y0 + qc - HALF)) * TH + j] = q;
            } else {
                s_q[j * HF_QJ + qa * HF_Q + qc] = q;
            }
        }
    };
    if constexpr (TH != 36) {
        for (int t = tid; t < 2 * TH * HF_Q; t += HF_NT) {
            if (t < TH * HF_Q) xtask(t, std::integral_constant<int, 0>{});
            else xtask(t - TH * HF_Q, std::integral_constant<int, 1>{});
        }
    } else {
        static_assert(TH * HF_Q <= 6 * 64 && TH * HF_Q > 5 * 64, "phase 4's task split: 6 wave-tasks per half");
        if (wave < 6) xtask(wave * 64 + lane, std::integral_constant<int, 0>{});
        const int s1 = wave == 8 ? 0 : wave == 6 ? 1 : wave == 7 ? 2 : wave == 1 ? 3 : wave == 2 ? 4 : wave == 3 ? 5 : -1;
        if (s1 >= 0) xtask(s1 * 64 + lane, std::integral_constant<int, 1>{});
    }
    float* s_po = s_b;
    // rec (the last step of a call that leaves the state unnormalised, pc_run_halo):
    // the key of the block's largest output U and, below, how many of its outputs lie
    // within a relative 2^-20 of it (HF_NEAR): P = U * (1/t) rounds monotonically, so the
    // first maximum of P is the first maximum of U unless another cell lies that close
    unsigned long long rk = 0ull;
    co_f4 uv = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};   // (lanes past a 2-layer group's stay -inf)
    bool has_uv = false;
    // every thread's partial sum and key, past Q in s_t (free from here on): the last
    // wave, which has no task in phase 5, reduces them there -- lane l adds the values of
    // thread l of every wave in wave order, then one DPP reduction (a fixed order, so
    // every launch gives the same bits) -- and stores the block's partial sum and key, so
    // the block's tail is the theta filter and its store
    constexpr int QSW = (TH * HF_QJ + 1) / 2 * 2;   // (8-byte aligned)
    double* s_qsw = reinterpret_cast<double*>(s_t + QSW);
    unsigned long long* s_bkw = reinterpret_cast<unsigned long long*>(s_qsw + HF_NT);
    static_assert(QSW + 4 * HF_NT <= 2 * (TH * HF_WJ + HF_NT), "per-thread sums and keys in s_t");
    if constexpr (!EXC) {
        s_qsw[tid] = qs;
        s_bkw[tid] = bk;
        co_lds_barrier();
        PC_STAMP(7, 4);
        static_assert(TH * 8 <= (HF_NW - 1) * 64, "the last wave has no phase-5 task");
        if (wave == HF_NW - 1) {
            double v = 0.0;
            unsigned long long kb = 0ull;
#pragma unroll
            for (int w = 0; w < HF_NW; ++w) {
                v += s_qsw[w * 64 + lane];
                kb = max(kb, s_bkw[w * 64 + lane]);
            }
            const double bsum = co_wave_sum(v);
            if (want_key) kb = co_wave_max(kb);
            if (lane == 0) {
                st_wt(&part_out[blockIdx.x], bsum);
                if (want_key) atomicMax(slot_prev + (blockIdx.x & (RES_SLOTS - 1)), kb);
            }
        }
        // 5. 7 x 7 path filter (:273) + clamp (:300): task (layer j, tile column tb,
        //    row pair ap) -> 2 outputs from 8 x 7 Q values; into [cell][3 + j] rows with
        //    wrapped copies (layers TH-3.. before, 0..6 after), so every theta window
        //    below is one contiguous aligned run
        //    The SIMDs are balanced: waves 0-3 take layers 0-31 (2-row tasks), wave 5 layers
        //    32-35 as 1-row tasks (lane: layer 32 + (lane >> 4), row (lane >> 2) & 3, column
        //    lane & 3); 288 2-row tasks on waves 0-4 put two on SIMD 0, beside wave 8
        auto ptask = [&](int j, int tb, int a0, auto n_c) __attribute__((always_inline)) {
            constexpr int NO = decltype(n_c)::value;
            float f[FT];
            st_filter<float>(s_ftab + s_fo[j], f);
            float acc[NO];
#pragma unroll
            for (int h = 0; h < NO; ++h) acc[h] = 0.f;
            const float* qw = s_q + j * HF_QJ + a0 * HF_Q + tb;
#pragma unroll
            for (int r = 0; r < NO + 2 * HALF; ++r) {  // rows of the outputs: h .. h + 6
                float w[FL];
#pragma unroll
                for (int y = 0; y < FL; ++y) w[y] = qw[r * HF_Q + y];
#pragma unroll
                for (int h = 0; h < NO; ++h) {
                    if (r - h < 0 || r - h >= FL) continue;
#pragma unroll
                    for (int y = 0; y < FL; ++y) acc[h] += w[y] * f[(r - h) * FL + y];
                }
            }
#pragma unroll
            for (int h = 0; h < NO; ++h) {
                const float v = pc_clamp(acc[h]);
                float* sp = s_po + ((a0 + h) * HF_T + tb) * PP;
                sp[HALF + j] = v;
                if (j >= TH - HALF) sp[j - TH + HALF] = v;
                if (j < FL) sp[HALF + TH + j] = v;
            }
        };
        static_assert(HF_T == 4, "phase 5's task split");
        if constexpr (TH != 36) {
            for (int t = tid; t < TH * 8; t += HF_NT)
                ptask(t >> 3, t & 3, 2 * ((t >> 2) & 1), std::integral_constant<int, 2>{});
        } else {
            if (wave < 4) ptask(tid >> 3, tid & 3, 2 * ((tid >> 2) & 1), std::integral_constant<int, 2>{});
            else if (wave == 5) ptask(32 + (lane >> 4), lane & 3, (lane >> 2) & 3, std::integral_constant<int, 1>{});
        }
        co_lds_barrier();
        PC_STAMP(7, 5);
        // 6. theta filter (:310) + clamp (:314): task (cell, group of G layers) -> one
        //    write-through store of U (normalised by the next launch): G = 4 (16 bytes),
        //    or 2 (8 bytes) when TH is not a multiple of 4
        const int nbytes = (int)min((size_t)X * Y * TH * sizeof(float), (size_t)INT_MAX);
        const bool wt = (size_t)X * Y * TH * sizeof(float) <= (size_t)INT_MAX;
        constexpr int G = V4 ? 4 : 2, NGR = TH / G, NRD = (G + 2 * HALF + G - 1) / G;
        using GV = typename std::conditional<V4, co_f4, hf_f2>::type;
        static_assert(HF_T * HF_T * NGR <= HF_NT, "one theta-filter task per thread");
        if (tid < HF_T * HF_T * NGR) {
            const int t = tid;
            const int cell = t / NGR, g = t - cell * NGR, ta = cell >> 2, tb = cell & 3;
            if (ta < tw && tb < tht) {
            const GV* sv = reinterpret_cast<const GV*>(s_po + cell * PP + G * g);
            float r[NRD * G];
#pragma unroll
            for (int q = 0; q < NRD; ++q) {
                const GV x = sv[q];
#pragma unroll
                for (int w = 0; w < G; ++w) r[G * q + w] = x[w];
            }
            GV v;
#pragma unroll
            for (int o = 0; o < G; ++o) {
                float x = 0.f;
#pragma unroll
                for (int z = 0; z < FL; ++z) x += r[o + z] * zf[z];
                v[o] = pc_clamp(x);
            }
            const unsigned lin = ((unsigned)(x0 + ta) * Y + (y0 + tb)) * TH + G * g;
            co_put(Uo, lin, v, wt, nbytes);
            if (rec) {
#pragma unroll
                for (int o = 0; o < G; ++o) {
                    rk = max(rk, argmax_key(v[o], lin + o));
                    uv[o] = v[o];
                }
                has_uv = true;
            }
            }
        }
    }
    PC_STAMP(14, 0);
    if constexpr (EXC) {   // (the excitation-only instance: the block's partial sum at its end)
        qs = co_wave_sum(qs);
        if (lane == 0) s_red[wave] = qs;
        co_lds_barrier();
        if (tid == 0) {
            double bsum = 0.0;
#pragma unroll
            for (int w = 0; w < HF_NW; ++w) bsum += s_red[w];
            st_wt(&part_out[blockIdx.x], bsum);
        }
    }
    if (rec) {
        rk = co_wave_max(rk);
        if (lane == 0) s_rk[wave] = rk;
        co_lds_barrier();
    }
    PC_STAMP(14, 1);
    PC_STAMP(14, 2);
    if (rec) {
        // the block's record: its largest U's key and the count of its outputs within
        // HF_NEAR of that value (the maximum itself included)
        unsigned long long m = s_rk[0];
#pragma unroll
        for (int w = 1; w < HF_NW; ++w) m = max(m, s_rk[w]);
        const float mv = __uint_as_float((unsigned)(m >> 32)), thr = mv - mv * HF_NEAR;
        int c = 0;
#pragma unroll
        for (int o = 0; o < 4; ++o) c += __popcll(__ballot(has_uv && uv[o] >= thr));
        if (lane == 0) s_cnt[wave] = c;
        co_lds_barrier();
        if (tid == 0) {
            int cnt = 0;
#pragma unroll
            for (int w = 0; w < HF_NW; ++w) cnt += s_cnt[w];
            // one 16-byte store: the record may live in pinned host memory (a one-step
            // call, pc_run_halo, whose host polls it: fine-grained host memory, which the
            // store writes through).  The count word carries REC_SET, so that neither word
            // of a landed record is zero and the host waits for both.  (Two 8-byte
            // system-scope atomic stores instead: update() 20.2-22.2 us against
            // 16.8-18.9 us, tools/pc_ab.py --mode update, round 5.)
            typedef unsigned long long u2 __attribute__((ext_vector_type(2)));
            *reinterpret_cast<u2*>(rec + 2 * blockIdx.x) = u2{m, REC_SET | (unsigned long long)cnt};
        }
    }
    PC_STAMP(7, 6);
}

// The instances of pc_step_halo: HF_TH (configs[1], the ROS node) and the even extents
// of configs[0]'s grid (18) and simulate.py's (10); pc_halo_fit admits these.
inline bool hf_th_ok(int TH) { return TH == HF_TH || TH == 18 || TH == 10; }
template <bool EXC, typename... A>
void hf_launch(int TH, dim3 grid, hipStream_t st, A... a) {
    switch (TH) {
    case 18: hipLaunchKernelGGL((pc_step_halo<EXC, 18>), grid, dim3(HF_NT), 0, st, a...); break;
    case 10: hipLaunchKernelGGL((pc_step_halo<EXC, 10>), grid, dim3(HF_NT), 0, st, a...); break;
    default: hipLaunchKernelGGL((pc_step_halo<EXC, HF_TH>), grid, dim3(HF_NT), 0, st, a...); break;
    }
}

// The end of a halo-form call: the normalised state P = U * (1/t) of the last step
// (written back, so the handle's state is normalised between calls), its argmax key
// per block into the last step's slots, optionally the float64 C-order volume into a
// pinned host array (readback='eager'), and the keys of the call's nexp steps for the
// host (the export kernel of the other forms, folded in: one launch fewer per call):
// block 0 stores the words of steps 0 .. nexp-2, whose slots earlier launches of the
// call completed, and every block stores its own key of the last step into bkey[block],
// which the host max-reduces once it has waited for the launch.  No block reads what
// another block of this launch wrote, so the kernel needs no intra-launch hand-off (the
// round-5 form handed the last step's slots to the block that counted last through an
// agent-scope counter, outside the memory model's release/acquire).
__global__ __launch_bounds__(256) void pc_halo_finish(
    const float* U, float* P,  // may be one buffer: each element is read, then written, by one thread
    int n4, const double* __restrict__ part,
    int npart, unsigned long long* __restrict__ slot, const unsigned long long* __restrict__ res,
    int nexp, unsigned long long* __restrict__ host, unsigned long long* __restrict__ bkey,
    double* __restrict__ xp, int nbytes, unsigned* __restrict__ flag, unsigned seq) {
    __shared__ unsigned long long s_bk[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (nexp > 1 && blockIdx.x == 0) {
        // steps 0 .. nexp-2: each step's max of its RES_SLOTS slots (filled by the launches
        // before this one) straight into the pinned host words
        for (int s = wave; s < nexp - 1; s += 4) {
            const unsigned long long* r = res + (size_t)s * RES_SLOTS;
            unsigned long long m = 0ull;
#pragma unroll
            for (int q = 0; q < RES_SLOTS / 64; ++q) m = max(m, r[lane + 64 * q]);
            m = co_wave_max(m);
            if (lane == 0) __hip_atomic_store(host + s, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    const PcNorm<float> nrm(pc_partials_total(part, npart));
    unsigned long long bk = 0ull;
    typedef double d2 __attribute__((ext_vector_type(2)));
    for (int i = blockIdx.x * 256 + tid; i < n4; i += gridDim.x * 256) {
        const co_f4 u = reinterpret_cast<const co_f4*>(U)[i];
        co_f4 p;
#pragma unroll
        for (int o = 0; o < 4; ++o) {
            p[o] = nrm(u[o]);
            bk = max(bk, argmax_key(p[o], 4u * (unsigned)i + o));
        }
        co_put(P, 4 * (size_t)i, p, true, nbytes);
        if (xp) {
            d2* d = reinterpret_cast<d2*>(xp + 4 * (size_t)i);
            d[0] = d2{(double)p[0], (double)p[1]};
            d[1] = d2{(double)p[2], (double)p[3]};
        }
    }
    bk = co_wave_max(bk);
    if (lane == 0) s_bk[wave] = bk;
    // flag (an eager readback the host polls for, pc_run_halo): every wave's volume
    // stores acknowledged before the block's barrier, then one lane's system-scope
    // release and the block's flag -- the producer form MI355X_MICROARCH.md gives
    // (stores, each wave's vmcnt(0), barrier, release, vmcnt(0), flag store)
    if (flag) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        bk = max(max(s_bk[0], s_bk[1]), max(s_bk[2], s_bk[3]));
        if (slot) atomicMax(slot + (blockIdx.x & (RES_SLOTS - 1)), bk);
        if (bkey) __hip_atomic_store(bkey + blockIdx.x, bk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (flag) {   // after the block's volume and its key
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(flag + blockIdx.x, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// Each step's RES_SLOTS packed argmax keys -> their max, stored straight into the
// pinned host buffer (system-scope stores): one queued launch in place of a
// device-to-host blit copy, which trailed the step by ~10 us (gap + copy kernel).
// One wave per step: each lane takes the max of RES_SLOTS / 64 slots, then DPP.
__global__ __launch_bounds__(64) void pc_res_export(const unsigned long long* __restrict__ res, int n,
                                                    unsigned long long* host) {
    static_assert(RES_SLOTS % 64 == 0, "slots per lane");
    for (int s = blockIdx.x; s < n; s += gridDim.x) {
        const unsigned long long* r = res + (size_t)s * RES_SLOTS;
        unsigned long long m = r[threadIdx.x];
#pragma unroll
        for (int k = 1; k < RES_SLOTS / 64; ++k) m = max(m, r[threadIdx.x + 64 * k]);
        m = co_wave_max(m);
        if (threadIdx.x == 0) __hip_atomic_store(host + s, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// The halo form's key export for a call that leaves its state unnormalised: steps
// 0 .. n-2 as pc_res_export (each keyed by the next launch from the scaled state it
// loaded); step n-1 from the last launch's per-block records of U.  P = U * (1/t) with
// t > 0 (or P = U when t == 0, or U / t where 1/t is not finite) rounds monotonically,
// so P's first maximum is U's, unless some other cell's U lies within HF_NEAR of the
// maximum (it might round to the same P, and the earlier index would win): then the
// word is RES_AMBIG and the host settles the state exactly (pc_halo_finish).  NaN, 0
// and inf maxima are exact (their products are the same value for every such cell).
__global__ __launch_bounds__(64) void pc_halo_export(const unsigned long long* __restrict__ res, int n,
                                                     const unsigned long long* __restrict__ rec, int nrec,
                                                     unsigned long long* host) {
    const int lane = threadIdx.x;
    for (int s = blockIdx.x; s < n; s += gridDim.x) {
        unsigned long long m = 0ull;
        if (s < n - 1 || rec == nullptr) {
            const unsigned long long* r = res + (size_t)s * RES_SLOTS;
#pragma unroll
            for (int k = 0; k < RES_SLOTS / 64; ++k) m = max(m, r[lane + 64 * k]);
            m = co_wave_max(m);
        } else {
            for (int b = lane; b < nrec; b += 64) m = max(m, rec[2 * b]);
            m = co_wave_max(m);
            const float gv = __uint_as_float((unsigned)(m >> 32)), thr = gv - gv * HF_NEAR;
            const bool exact = !(gv > 0.f) || gv == __builtin_inff() || gv != gv;   // 0 (all zero), inf, NaN
            bool amb = false;
            for (int b = lane; b < nrec; b += 64) {
                const unsigned long long kb = rec[2 * b];
                amb |= kb == m ? (rec[2 * b + 1] & ~REC_SET) > 1ull : __uint_as_float((unsigned)(kb >> 32)) >= thr;
            }
            amb = __ballot(amb) != 0ull;
            if (!exact && amb) m = RES_AMBIG;
        }
        if (lane == 0) __hip_atomic_store(host + s, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

template <typename T>
__global__ __launch_bounds__(NT) void pc_argmax_finalize(const T* __restrict__ bmax,
                                                         const unsigned* __restrict__ bidx, int nb,
                                                         unsigned long long* __restrict__ res_slot) {
    __shared__ T s_bv[NT];
    __shared__ unsigned s_bl[NT];
    T bv = -std::numeric_limits<T>::infinity();
    unsigned bl = 0xFFFFFFFFu;
    for (int i = threadIdx.x; i < nb; i += NT) {
        const T v = bmax[i];
        const unsigned l = bidx[i];
        if (pc_better(v, l, bv, bl)) {
            bv = v;
            bl = l;
        }
    }
    s_bv[threadIdx.x] = bv;
    s_bl[threadIdx.x] = bl;
    __syncthreads();
    for (int s = NT / 2; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            const T v = s_bv[threadIdx.x + s];
            const unsigned l = s_bl[threadIdx.x + s];
            if (pc_better(v, l, s_bv[threadIdx.x], s_bl[threadIdx.x])) {
                s_bv[threadIdx.x] = v;
                s_bl[threadIdx.x] = l;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) *res_slot = 0xFFFFFFFFull - s_bl[0];  // same decoding as the packed key
}

// Per-step argmax: block s reduces the nb (value, index) partials of step s.
template <typename T>
__global__ __launch_bounds__(NT) void pc_argmax_steps(const T* __restrict__ bmax,
                                                      const unsigned* __restrict__ bidx, int nb,
                                                      unsigned long long* __restrict__ res) {
    __shared__ T s_bv[NT];
    __shared__ unsigned s_bl[NT];
    const size_t base = (size_t)blockIdx.x * nb;
    T bv = -std::numeric_limits<T>::infinity();
    unsigned bl = 0xFFFFFFFFu;
    for (int i = threadIdx.x; i < nb; i += NT) {
        const T v = bmax[base + i];
        const unsigned l = bidx[base + i];
        if (pc_better(v, l, bv, bl)) {
            bv = v;
            bl = l;
        }
    }
    s_bv[threadIdx.x] = bv;
    s_bl[threadIdx.x] = bl;
    __syncthreads();
    for (int st = NT / 2; st > 0; st >>= 1) {
        if (threadIdx.x < st) {
            const T v = s_bv[threadIdx.x + st];
            const unsigned l = s_bl[threadIdx.x + st];
            if (pc_better(v, l, s_bv[threadIdx.x], s_bl[threadIdx.x])) {
                s_bv[threadIdx.x] = v;
                s_bl[threadIdx.x] = l;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) res[(size_t)blockIdx.x * RES_SLOTS] = 0xFFFFFFFFull - s_bl[0];
}

// Argmax of the stored state (get_pc_max outside update): per-block partials.
template <typename T>
__global__ __launch_bounds__(NT) void pc_argmax_blocks(const T* __restrict__ P, int X, int Y, int TH,
                                                       T* __restrict__ bmax,
                                                       unsigned* __restrict__ bidx, int thfast) {
    __shared__ T s_bv[NT];
    __shared__ unsigned s_bl[NT];
    const size_t n = (size_t)X * Y * TH;
    T bv = -std::numeric_limits<T>::infinity();
    unsigned bl = 0xFFFFFFFFu;
    for (size_t e = blockIdx.x * (size_t)NT + threadIdx.x; e < n; e += (size_t)gridDim.x * NT) {
        const int k = (int)(e / ((size_t)X * Y));
        const int rem = (int)(e - (size_t)k * X * Y);
        const int i = rem / Y, j = rem - i * Y;
        const T v = P[e];
        const unsigned lin = thfast ? (unsigned)e : ((unsigned)i * Y + j) * TH + k;
        if (pc_better(v, lin, bv, bl)) {
            bv = v;
            bl = lin;
        }
    }
    s_bv[threadIdx.x] = bv;
    s_bl[threadIdx.x] = bl;
    __syncthreads();
    for (int s = NT / 2; s > 0; s >>= 1) {
        if (threadIdx.x < s) {
            const T v = s_bv[threadIdx.x + s];
            const unsigned l = s_bl[threadIdx.x + s];
            if (pc_better(v, l, s_bv[threadIdx.x], s_bl[threadIdx.x])) {
                s_bv[threadIdx.x] = v;
                s_bl[threadIdx.x] = l;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        bmax[blockIdx.x] = s_bv[0];
        bidx[blockIdx.x] = s_bl[0];
    }
}

// Element e of the C-order (x, y, th) volume -> its place in a layer-major volume
// (or itself in a theta-fastest one: the column form's P, which is C order).
__device__ inline size_t pc_layer_major(size_t e, int X, int Y, int TH) {
    const int k = (int)(e % TH);
    const size_t xy = e / TH;
    const int j = (int)(xy % Y), i = (int)(xy / Y);
    return ((size_t)k * X + i) * Y + j;
}

// The float64 C-order export with 16-byte stores (two consecutive cells per thread): a wave's
// stores are 1 KiB contiguous, the unit host writes over PCIe favour.  out is
// 16-byte aligned (rs_host_alloc / hipMalloc); an odd last cell goes alone.
// flag (host memory the host polls instead of the stream's completion, pc_poll_flags):
// every wave's volume stores acknowledged, the block's barrier, one lane's system-scope
// release, then the block's flag = seq -- the producer form of pc_halo_finish.
template <typename T>
__global__ void pc_export2_kernel(const T* __restrict__ P, double* __restrict__ out, int X, int Y,
                                  int TH, int thfast, unsigned* __restrict__ flag, unsigned seq) {
    typedef double d2 __attribute__((ext_vector_type(2)));
    const size_t n = (size_t)X * Y * TH, n2 = n / 2;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x) {
        const size_t e = 2 * i;
        d2 v;
        v.x = (double)P[thfast ? e : pc_layer_major(e, X, Y, TH)];
        v.y = (double)P[thfast ? e + 1 : pc_layer_major(e + 1, X, Y, TH)];
        *reinterpret_cast<d2*>(out + e) = v;
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0)
        out[n - 1] = (double)P[thfast ? n - 1 : pc_layer_major(n - 1, X, Y, TH)];
    if (flag) {   // (kernel argument: uniform)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(flag + blockIdx.x, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

template <typename T>
__global__ void pc_import_kernel(const double* __restrict__ in, T* __restrict__ P, int X, int Y,
                                 int TH, int thfast) {
    const size_t n = (size_t)X * Y * TH;
    for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < n;
         e += (size_t)gridDim.x * blockDim.x)
        P[thfast ? e : pc_layer_major(e, X, Y, TH)] = (T)in[e];
}


template <typename T>
__global__ void pc_inject_kernel(T* __restrict__ P, size_t idx, double energy) {
    if (threadIdx.x == 0) P[idx] = (T)((double)P[idx] + energy);
}

template <typename T>
__global__ __launch_bounds__(NT) void pc_total_kernel(const T* __restrict__ P, size_t n,
                                                      double* __restrict__ out) {
    __shared__ double s_red[NT / 64];
    double s = 0.0;
    for (size_t e = threadIdx.x; e < n; e += NT) s += (double)P[e];
    s = block_sum(s, s_red);
    if (threadIdx.x == 0) *out = s;
}

}  // namespace

// ===========================================================================
// Host side
// ===========================================================================
// Tables of path_integration's control (rs_pc_set_odometry_tables): NumPy-evaluated
// cos/sin per layer, the LUT key -> filter row map and the theta filters per origin.
struct OdoTables {
    int TH = 0;
    double vtScale = 0.0, vrScale = 0.0;
    const double* cosA = nullptr;
    const double* sinA = nullptr;
    int keyMin = 0, nKeys = 0;
    const int32_t* keyRows = nullptr;
    int zMin = 0, nZ = 0;
    const double* zfTab = nullptr;
    std::vector<double> own;        // owned copies when held by a handle
    std::vector<int32_t> ownRows;
};

struct rs_pc {
    int X = 0, Y = 0, TH = 0, prec = RS_PREC_F32, device = 0;
    size_t n = 0, esz = 4;
    hipStream_t stream = nullptr;
    void* dP = nullptr;
    void* dQ = nullptr;
    void* dFilt = nullptr;
    int nf = 0;
    double* dPart = nullptr;
    int nPart = 0;               // blocks of the excitation kernel
    int nPathBlocks = 0;         // blocks of the path kernel
    void* dBmax = nullptr;       // f64 argmax partials (max(nPathBlocks, argmax grid))
    unsigned* dBidx = nullptr;
    int nBmaxCap = 0;
    unsigned long long* dRes = nullptr;
    int resCap = 0;
    void* dArgV = nullptr;        // per-step per-block argmax partials [resCap][nPathBlocks]
    unsigned* dArgI = nullptr;
    unsigned long long* hRes = nullptr;  // pinned
    unsigned long long* hResDev = nullptr;  // hRes in the device's address space (pc_res_export)
    unsigned char* dCtl = nullptr;
    unsigned char* hCtl = nullptr;       // pinned
    size_t ctlStride = 0;
    int ctlCap = 0;
    double* dTmp = nullptr;              // export/import staging (n doubles)
    double* dScalar = nullptr;
    SepKernel<float> kf{};
    SepKernel<double> kd{};
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    float lastMs = 0.f;
    bool profiling = false;  // HIP events around the whole call (device_ms)
    bool profKernels = false;  // ... and around every launch (kernel_ms; the events add gaps)
    std::vector<hipEvent_t> evPool;
    double kernelMs[2] = {0.0, 0.0};
    int tiling = 0;  // 64 / 128: row-tiled kernels for Y <= 64 / 128; 0: generic 3-D tiles
    bool streamed = false;  // layer-streaming kernels (default; RS_PC_FORM=rows|tiles|stream:BX,WR,KC)
    bool cols = false;      // column kernels (RS_PC_FORM=cols[:KC]): TX x TY tiles through KC layers;
                            // P and Q are then theta-fastest (C order (x, y, th))
    bool halo = false;      // one launch per step (RS_PC_FORM=halo): HF_T x HF_T tiles through all
                            // layers, the excitation recomputed on each tile's halo; P theta-fastest
    unsigned long long* dRec = nullptr;  // halo: the last launch's per-block (key of max U, near count)
    unsigned long long* hRec = nullptr;  // ... for a one-step call: pinned host records (hRecDev on the device)
    unsigned long long* hRecDev = nullptr;
    unsigned* hFlag = nullptr;      // halo: pc_halo_finish's per-block flags (pinned; eager readback polls)
    unsigned* hFlagDev = nullptr;
    unsigned long long* hKey = nullptr;     // halo: pc_halo_finish's per-block keys of a call's last step (pinned)
    unsigned long long* hKeyDev = nullptr;
    unsigned flagSeq = 0u;
    bool haloPend = false;  // halo: the state is U, unnormalised, in buffer haloCur (0 dP, 1 dQ) with
    int haloCur = 0, haloPart = 0;  // its partial sums in half haloPart of dPart (pc_halo_settle)
    long haloAmbig = 0;     // calls whose last step was keyed by the finishing pass (RES_AMBIG)
    bool haloSettleAlways = false;  // rs_pc_debug(RS_PC_DBG_HALO_SETTLE)
    int cgx = 0, cgy = 0;   // column (or halo) tiles along x and y
    int coKC = 0, coNch = 1;  // layers per theta chunk (KC == TH: whole extent, no halo), chunks
    int sbx = 1, swr = 8, swc = 1;  // streaming tile: BX rows per wave, WR row groups, WC column tiles
    StreamGrid sg{};
    // odometry -> control tables (rs_pc_set_odometry_tables) and per-call scratch
    bool odoReady = false;
    OdoTables odo{};
    std::vector<int32_t> cOx, cOy, cRows;
    std::vector<double> cZf;
    bool dbgSkipExport = false;  // rs_pc_debug(RS_PC_DBG_SKIP_EXPORT): the next run leaves hRes unwritten
    double* exportDev = nullptr;  // rs_pc_update_odom_read: the state export queued behind the step
    double* hRead = nullptr;     // rs_pc_read: pinned float64 volume the export kernel writes in place
    double* hReadDev = nullptr;
};

namespace {

// P (and Q) theta-fastest, the reference's C order (x, y, th): the column and halo
// forms; the others keep P layer-major
inline bool pc_thfast(const rs_pc* h) { return h->cols || h->halo; }

// Per-step buffers of a call of n steps, grown in powers of two: the result slots and
// words always; the control ring (pinned staging + device copy, ctlStride bytes a step)
// only for the forms that read it (ctl): the halo and column forms take each step's
// control as kernel arguments, and a 10,000-step batch's 16 MiB of pinned ring was a
// few milliseconds of page-locking inside its first call.
int pc_grow_steps(rs_pc* h, int n, bool ctl = true) {
    if (n > h->resCap) {
        int cap = h->resCap > 0 ? h->resCap : 16;
        while (cap < n) cap *= 2;
        if (h->dRes) RS_HIP(hipFree(h->dRes));
        if (h->hRes) RS_HIP(hipHostFree(h->hRes));
        if (h->dArgV) RS_HIP(hipFree(h->dArgV));
        if (h->dArgI) RS_HIP(hipFree(h->dArgI));
        h->dRes = nullptr; h->hRes = nullptr; h->hResDev = nullptr;
        h->dArgV = nullptr; h->dArgI = nullptr;
        h->resCap = 0;
        RS_HIP(hipMalloc(&h->dRes, sizeof(unsigned long long) * RES_SLOTS * cap));
        // every slot starts zeroed (the excitation's block 0 zeroes a step's slots again
        // before its path kernel max-reduces into them; no step ever reads freed data)
        RS_HIP(hipMemsetAsync(h->dRes, 0, sizeof(unsigned long long) * RES_SLOTS * cap, h->stream));
        // the export kernel stores each step's key here with a system-scope store:
        // fine-grained (coherent) host memory, so the store is visible once the stream
        // has synchronised; pc_run_impl also checks a sentinel per step (RES_NONE)
        RS_HIP(hipHostMalloc(&h->hRes, sizeof(unsigned long long) * cap,
                             hipHostMallocMapped | hipHostMallocCoherent));
        for (int s = 0; s < cap; ++s) h->hRes[s] = RES_NONE;
        RS_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&h->hResDev), h->hRes, 0));
        if (h->prec == RS_PREC_F64) {  // float64 argmax: per-block partials + pc_argmax_steps
            RS_HIP(hipMalloc(&h->dArgV, h->esz * (size_t)cap * h->nPathBlocks));
            RS_HIP(hipMalloc(&h->dArgI, sizeof(unsigned) * (size_t)cap * h->nPathBlocks));
        }
        h->resCap = cap;
    }
    if (ctl && n > h->ctlCap) {
        int cap = h->ctlCap > 0 ? h->ctlCap : 16;
        while (cap < n) cap *= 2;
        if (h->dCtl) RS_HIP(hipFree(h->dCtl));
        if (h->hCtl) RS_HIP(hipHostFree(h->hCtl));
        h->dCtl = nullptr; h->hCtl = nullptr;
        h->ctlCap = 0;
        RS_HIP(hipMalloc(&h->dCtl, h->ctlStride * cap));
        RS_HIP(hipHostMalloc(&h->hCtl, h->ctlStride * cap, hipHostMallocDefault));
        h->ctlCap = cap;
    }
    return RS_OK;
}

int pc_ensure_events(rs_pc* h, size_t need) {
    while (h->evPool.size() < need) {
        hipEvent_t e;
        RS_HIP(hipEventCreate(&e));
        h->evPool.push_back(e);
    }
    return RS_OK;
}

// control record: int32 ox[TH] | int32 oy[TH] | int32 fidx[TH] | pad | double zf[8]
inline size_t ctl_off_oy(const rs_pc* h) { return sizeof(int32_t) * h->TH; }
inline size_t ctl_off_f(const rs_pc* h) { return 2 * sizeof(int32_t) * h->TH; }
inline size_t ctl_off_zf(const rs_pc* h) { return rs::round_up(3 * sizeof(int32_t) * h->TH, 16); }

int pc_check_ctl(const rs_pc* h, int n, const int32_t* ox, const int32_t* oy,
                 const int32_t* fidx, const double* zf) {
    RS_CHECK(ox && oy && fidx && zf, RS_ERR_ARG, "null control array");
    for (size_t e = 0; e < (size_t)n * h->TH; ++e) {
        const int32_t f = fidx[e];
        RS_CHECK(f >= 0 && f < h->nf, RS_ERR_ARG,
                 "step %d layer %d: filter index %d outside the table [0, %d)", (int)(e / h->TH),
                 (int)(e % h->TH), f, h->nf);
        if (h->TH <= CTL_INLINE_MAX)
            RS_CHECK(ox[e] >= -32768 && ox[e] <= 32767 && oy[e] >= -32768 && oy[e] <= 32767,
                     RS_ERR_ARG, "shift (%d, %d) outside the int16 inline control", ox[e], oy[e]);
    }
    return RS_OK;
}

int pc_pack_ctl(rs_pc* h, int n, const int32_t* ox, const int32_t* oy, const int32_t* fidx,
                const double* zf, unsigned char* dst = nullptr) {
    const int TH = h->TH;
    for (int s = 0; s < n; ++s) {
        unsigned char* rec = (dst ? dst : h->hCtl) + (size_t)s * h->ctlStride;
        std::memcpy(rec, ox + (size_t)s * TH, sizeof(int32_t) * TH);
        std::memcpy(rec + ctl_off_oy(h), oy + (size_t)s * TH, sizeof(int32_t) * TH);
        std::memcpy(rec + ctl_off_f(h), fidx + (size_t)s * TH, sizeof(int32_t) * TH);
        std::memcpy(rec + ctl_off_zf(h), zf + (size_t)s * FL, sizeof(double) * FL);
    }
    return RS_OK;
}

template <typename T>
const SepKernel<T>& sep_of(const rs_pc* h);
template <>
const SepKernel<float>& sep_of<float>(const rs_pc* h) { return h->kf; }
template <>
const SepKernel<double>& sep_of<double>(const rs_pc* h) { return h->kd; }

// Control of step s as a kernel argument (TH <= CTL_INLINE_MAX) ...
void make_ctl_inline(const rs_pc* h, int s, const int32_t* ox, const int32_t* oy,
                     const int32_t* fidx, const double* zf, PcCtlInline* c) {
    const size_t b = (size_t)s * h->TH;
    int mnx = INT_MAX, mxx = INT_MIN, mny = INT_MAX, mxy = INT_MIN;
    for (int k = 0; k < h->TH; ++k) {
        c->iox[k] = (short)ox[b + k];
        c->ioy[k] = (short)oy[b + k];
        c->ifi[k] = (unsigned char)fidx[b + k];
        const int cx = co_centre(ox[b + k], h->X), cy = co_centre(oy[b + k], h->Y);
        mnx = std::min(mnx, cx);
        mxx = std::max(mxx, cx);
        mny = std::min(mny, cy);
        mxy = std::max(mxy, cy);
    }
    for (int z = 0; z < FL; ++z) c->izf[z] = zf[(size_t)s * FL + z];
    c->umx = (short)mnx;
    c->umy = (short)mny;
    c->uwx = (short)(CO_TX + 2 * HALF + mxx - mnx);
    c->uwy = (short)(CO_TY + 2 * HALF + mxy - mny);
}

// ... or as pointers into the device ring record of step s.
PcCtlRing make_ctl_ring(const rs_pc* h, int s, const unsigned char* ring = nullptr) {
    const unsigned char* rec = (ring ? ring : h->dCtl) + (size_t)s * h->ctlStride;
    return PcCtlRing{reinterpret_cast<const int*>(rec),
                     reinterpret_cast<const int*>(rec + ctl_off_oy(h)),
                     reinterpret_cast<const int*>(rec + ctl_off_f(h)),
                     reinterpret_cast<const double*>(rec + ctl_off_zf(h))};
}

void decode_xyz(const rs_pc* h, unsigned long long key, int32_t* out);

// Control of step s for the halo form: the layers' centred shifts as window starts in
// the union of the step's shifted 16 x 16 windows (the same for every block), which the
// kernel loads first thing.
void make_ctl_halo(const rs_pc* h, int s, const int32_t* ox, const int32_t* oy, const int32_t* fidx,
                   const double* zf, PcCtlHalo* c) {
    const size_t b = (size_t)s * h->TH;
    int mnx = INT_MAX, mxx = INT_MIN, mny = INT_MAX, mxy = INT_MIN;
    for (int k = 0; k < h->TH; ++k) {
        const int cx = co_centre(ox[b + k], h->X), cy = co_centre(oy[b + k], h->Y);
        mnx = std::min(mnx, cx);
        mxx = std::max(mxx, cx);
        mny = std::min(mny, cy);
        mxy = std::max(mxy, cy);
    }
    const int uw = std::min(HF_W + mxx - mnx, h->X);
    int uy = mny, uh = std::min(HF_W + mxy - mny, h->Y);
    const bool wrap = HF_W + mxx - mnx > h->X || HF_W + mxy - mny > h->Y;
    // theta extents that are not whole 16-byte pieces (pc_step_halo loads the image in
    // 16-byte pieces of cell pairs then): an even start column and width, one column more
    // on either side where needed, when that stays a union the image holds
    if (h->TH % 4 != 0 && h->Y % 2 == 0 && !wrap) {
        const int py = uy - (uy & 1), ph = (uh + (uy & 1) + 1) & ~1;
        if (ph <= h->Y && uw * ph <= HF_UMAX) {
            uy = py;
            uh = ph;
        }
    }
    for (int k = 0; k < h->TH; ++k) {
        c->sx[k] = (short)(co_centre(ox[b + k], h->X) - mnx);
        c->sy[k] = (short)(co_centre(oy[b + k], h->Y) - uy);
        c->fo[k] = (unsigned char)fidx[b + k];
    }
    for (int z = 0; z < FL; ++z) c->zf[z] = (float)zf[(size_t)s * FL + z];
    c->ux = (short)mnx;
    c->uy = (short)uy;
    c->uw = (short)uw;
    c->uh = (short)uh;
    c->wrap = wrap;
}

// Where step s of a launch sequence leaves its results: its RES_SLOTS argmax
// slots, and (float64) its per-block argmax partials.
struct StepOut {
    unsigned long long* slot;
    void* bmax;
    unsigned* bidx;
};
inline StepOut step_out(unsigned long long* res, void* argv, unsigned* argi, size_t esz, int nblocks, int s) {
    return StepOut{res + (size_t)s * RES_SLOTS,
                   argv ? static_cast<char*>(argv) + esz * (size_t)s * nblocks : nullptr,
                   argi ? argi + (size_t)s * nblocks : nullptr};
}
inline StepOut step_out(const rs_pc* h, int s) {
    return step_out(h->dRes, h->dArgV, h->dArgI, h->esz, h->nPathBlocks, s);
}

// Wait for a call's result words (pinned host memory, each one 8-byte system-scope store
// by the call's last kernel) instead of the stream's completion signal: a bounded spin
// that returns true once every word of steps [s0, s1) holds a key, false when it runs
// out (the caller then synchronises the stream, which returns any error).  Safe for the
// same reason as the halo form's record polling (pc_run_halo): the host reads nothing
// else the call wrote, and every later device access is ordered on the stream.
bool pc_poll_words(const rs_pc* h, int s0, int s1) {
    const volatile unsigned long long* w = h->hRes;
    int s = s0;
    for (long spin = 0; spin < 4000000 && s < s1; ++spin)
        while (s < s1 && w[s] != RES_NONE) ++s;
    return s == s1;
}

// An eager halo call (the volume written into the caller's pinned array) polls the
// finishing blocks' flags instead of the stream's completion when it is short and not
// profiled; RS_PC_HALO_FLAGS=0 keeps the stream synchronisation for it.
bool halo_poll_env() {
    static const bool on = [] {
        const char* e = std::getenv("RS_PC_HALO_POLL");
        return !(e && std::strcmp(e, "0") == 0);
    }();
    return on;
}
bool halo_flags_env() {
    static const bool on = [] {
        const char* e = std::getenv("RS_PC_HALO_FLAGS");
        return !(e && std::strcmp(e, "0") == 0);
    }();
    return on;
}
bool xp_poll_ok(const rs_pc* h, int n, bool poll_env) {
    return poll_env && halo_flags_env() && h->exportDev && h->hFlag && !h->profiling && !h->dbgSkipExport &&
           n <= HF_POLL_MAX && (int)std::min<size_t>(1024, (h->n / 4 + 255) / 256) <= HF_FLAGS;
}

// Spin until pc_halo_finish's nb blocks have each stored flag value seq (bounded; false
// when the spin runs out and the caller must synchronise the stream instead).
bool pc_poll_flags(const rs_pc* h, int nb, unsigned seq) {
    const volatile unsigned* f = h->hFlag;
    int b = 0;
    for (long spin = 0; spin < 4000000 && b < nb; ++spin)
        while (b < nb && f[b] == seq) ++b;
    return b == nb;
}

// The next flag value of a volume-writing launch the host will poll (0 is the flags'
// initial value, never a live one), and whether a launch of nb blocks may be polled.
unsigned pc_next_seq(rs_pc* h) {
    unsigned seq = ++h->flagSeq;
    if (seq == 0u) seq = ++h->flagSeq;
    return seq;
}
bool pc_flags_ok(const rs_pc* h, int nb) {
    return halo_poll_env() && halo_flags_env() && h->hFlag && !h->profiling && nb <= HF_FLAGS;
}
// The export kernel's grid when its flags are polled: at most 128 blocks, each thread
// storing a few 16-byte pieces (fewer blocks, fewer flags; 64x64x36 rows-form read 32-36
// us at 32-128 blocks against 36-37 at 289, within the boxes' spread, tools/node_step.py,
// round 5)
int pc_xflag_nb(int nb) { return std::min(nb, 128); }

// pc_halo_export's last-step rule on the host, over records in pinned host memory: the
// largest key, or RES_AMBIG when another cell may round to the same scaled value; RES_NONE
// when a block's record is missing (a record's key is never 0).
unsigned long long halo_key_from_records(const unsigned long long* rec, int nrec) {
    unsigned long long m = 0ull;
    for (int b = 0; b < nrec; ++b) {
        if (rec[2 * b] == 0ull || rec[2 * b + 1] == 0ull) return RES_NONE;
        m = std::max(m, rec[2 * b]);
    }
    auto val = [](unsigned long long k) {
        const unsigned u = (unsigned)(k >> 32);
        float f;
        std::memcpy(&f, &u, sizeof(f));
        return f;
    };
    const float gv = val(m), thr = gv - gv * HF_NEAR;
    if (!(gv > 0.f) || std::isinf(gv) || std::isnan(gv)) return m;   // 0, inf, NaN maxima are exact
    for (int b = 0; b < nrec; ++b) {
        const unsigned long long kb = rec[2 * b];
        if (kb == m ? (rec[2 * b + 1] & ~REC_SET) > 1ull : val(kb) >= thr) return RES_AMBIG;
    }
    return m;
}

// The halo form's state left unnormalised by a call (U in buffer haloCur, its partial
// sums in half haloPart of dPart), normalised into dP: the entry points that read or
// change the state directly (read, write, inject, get_max, total, excite, debug) settle
// it first.  (The next call's first launch consumes it as it is: it scales on load.)
int pc_halo_settle(rs_pc* h) {
    if (!h->haloPend) return RS_OK;
    float* buf[2] = {static_cast<float*>(h->dP), static_cast<float*>(h->dQ)};
    const int n4 = (int)(h->n / 4), nb = std::min(1024, (n4 + 255) / 256);
    hipLaunchKernelGGL(pc_halo_finish, dim3(nb), dim3(256), 0, h->stream, buf[h->haloCur], buf[0], n4,
                       h->dPart + (size_t)h->haloPart * h->nPart, h->nPart, nullptr, nullptr, 0, nullptr,
                       nullptr, nullptr, (int)(h->n * sizeof(float)), nullptr, 0u);
    RS_HIP(hipGetLastError());
    h->haloPend = false;
    h->haloCur = 0;
    return RS_OK;
}

// A volume read of a state a halo call left unnormalised (the ROS node's `.posecells`
// after update()): the finishing kernel normalises the state and writes the float64
// C-order volume into the pinned destination in the same pass (the eager readback's
// kernel: one launch in place of the settle and the export kernel), and the host waits
// for its blocks' flags -- each released at system scope after the block's volume
// stores -- instead of the stream's completion (RS_PC_HALO_POLL=0 or RS_PC_HALO_FLAGS=0:
// the stream synchronisation).  The host reads only what this kernel wrote, so the
// early return is safe as the eager call's is (pc_run_halo).  *done is false when no
// state is pending (the caller exports as usual).
int pc_halo_settle_read(rs_pc* h, double* xp_dev, bool* done) {
    *done = false;
    if (!h->haloPend) return RS_OK;
    float* buf[2] = {static_cast<float*>(h->dP), static_cast<float*>(h->dQ)};
    const int n4 = (int)(h->n / 4), nb = std::min(1024, (n4 + 255) / 256);
    const bool fl = pc_flags_ok(h, nb);
    const unsigned seq = fl ? pc_next_seq(h) : 0u;
    hipLaunchKernelGGL(pc_halo_finish, dim3(nb), dim3(256), 0, h->stream, buf[h->haloCur], buf[0], n4,
                       h->dPart + (size_t)h->haloPart * h->nPart, h->nPart, nullptr, nullptr, 0, nullptr,
                       nullptr, xp_dev, (int)(h->n * sizeof(float)), fl ? h->hFlagDev : nullptr, seq);
    RS_HIP(hipGetLastError());
    h->haloPend = false;
    h->haloCur = 0;
    if (!(fl && pc_poll_flags(h, nb, seq))) RS_HIP(hipStreamSynchronize(h->stream));
    *done = true;
    return RS_OK;
}

// n steps of the halo form: one launch each (step s reads the state in one buffer,
// scaled by the partials of the step before, and writes U into the other; the partial
// sums ping-pong between the two halves of dPart).  Then, by default, the call ends with
// the state left unnormalised (haloPend) and one small export launch (pc_halo_export):
// steps 0 .. n-2 keyed by the launch after each, step n-1 from the last launch's
// per-block records of U -- the finishing pass over the volume (pc_halo_finish) is off
// the per-call path (update() at 64x64x36: about 4 us of device time per call).  With an
// eager readback (the float64 volume into the caller's pinned array), or when the
// records cannot settle the last step's first maximum (RES_AMBIG: a cell within
// HF_NEAR of the peak), pc_halo_finish normalises the state into dP, keys it and
// exports.  One host sync (two for RES_AMBIG).  RS_PC_HALO_SETTLE=1 always finishes.
int pc_run_halo(rs_pc* h, int n, const int32_t* ox, const int32_t* oy, const int32_t* fidx,
                const double* zf, int32_t* out_xyz) {
    RS_TRY(pc_grow_steps(h, n, false));   // (the control travels as kernel arguments)
    const bool pk = h->profiling && h->profKernels;
    if (pk) RS_TRY(pc_ensure_events(h, (size_t)2 * n + 2));
    for (int s = 0; s < n; ++s) h->hRes[s] = RES_NONE;
    // RS_PC_HALO_POLL=0: a one-step call waits for the kernel's completion signal instead
    // of returning once every block's record has reached host memory (below)
    const bool poll_env = halo_poll_env();
    const bool lazy = h->exportDev == nullptr && !h->haloSettleAlways;
    // a one-step call: the blocks' records go straight to pinned host memory and the host
    // reduces them after its wait (no export launch)
    const bool host_rec = lazy && n == 1 && h->hRec;
    if (host_rec) std::memset(h->hRec, 0, sizeof(unsigned long long) * 2 * h->nPart);
    if (h->profiling) RS_HIP(hipEventRecord(h->ev0, h->stream));
    float* buf[2] = {static_cast<float*>(h->dP), static_cast<float*>(h->dQ)};
    const dim3 grid(h->cgx * h->cgy);
    const bool pend = h->haloPend;
    const int c0 = pend ? h->haloCur : 0;          // the buffer step 0 reads
    const int p0 = pend ? (h->haloPart ^ 1) : 0;   // the partials half step 0 writes
    for (int s = 0; s < n; ++s) {
        PcCtlHalo c;
        make_ctl_halo(h, s, ox, oy, fidx, zf, &c);
        const double* part_in = s > 0 ? h->dPart + (size_t)((p0 + s - 1) & 1) * h->nPart
                                      : h->dPart + (size_t)(pend ? h->haloPart : 0) * h->nPart;
        const int npart_in = s > 0 || pend ? h->nPart : 0;
        if (pk) RS_HIP(hipEventRecord(h->evPool[2 * s], h->stream));
        hf_launch<false>(h->TH, grid, h->stream, static_cast<const float*>(buf[(c0 + s) & 1]),
                           hf_pack(h->X, h->Y), hf_pack(h->cgx, grid.x), hf_pack(c.ux, c.uy), hf_pack(c.uw, c.uh),
                           hf_magic(h->cgx), hf_magic(c.uh), part_in, npart_in, buf[(c0 + s + 1) & 1],
                           h->dPart + (size_t)((p0 + s) & 1) * h->nPart,
                           s == 0 ? nullptr : h->dRes + (size_t)(s - 1) * RES_SLOTS,
                           h->dRes + (size_t)s * RES_SLOTS, static_cast<const float*>(h->dFilt), h->nf, c, h->kf,
                           lazy && s == n - 1 ? (host_rec ? h->hRecDev : h->dRec) : nullptr);
        RS_HIP(hipGetLastError());
        if (pk) RS_HIP(hipEventRecord(h->evPool[2 * s + 1], h->stream));
    }
    const int cl = (c0 + n) & 1, pl = (p0 + n - 1) & 1;   // where the last U and its partials are
    const int n4 = (int)(h->n / 4), nb = std::min(1024, (n4 + 255) / 256);
    // an eager readback the host may poll for (per-block flags behind a system-scope release)
    const bool flag_poll = xp_poll_ok(h, n, poll_env);
    const unsigned seq = flag_poll ? pc_next_seq(h) : 0u;
    // own export: block 0 stores the words of steps 0 .. n-2, every block its key of step
    // n-1 into hKey, reduced here once the launch has been waited for
    auto finish = [&](int nexp_own, double* xp) -> int {
        const bool fl = flag_poll && xp != nullptr;
        if (nexp_own > 0) std::memset(h->hKey, 0, sizeof(unsigned long long) * nb);
        hipLaunchKernelGGL(pc_halo_finish, dim3(nb), dim3(256), 0, h->stream, buf[cl], buf[0], n4,
                           h->dPart + (size_t)pl * h->nPart, h->nPart, h->dRes + (size_t)(n - 1) * RES_SLOTS,
                           h->dRes, nexp_own, h->hResDev, nexp_own > 0 ? h->hKeyDev : nullptr, xp,
                           (int)(h->n * sizeof(float)), fl ? h->hFlagDev : nullptr, seq);
        RS_HIP(hipGetLastError());
        h->haloPend = false;
        h->haloCur = 0;
        return RS_OK;
    };
    if (pk) RS_HIP(hipEventRecord(h->evPool[2 * n], h->stream));
    bool own_export = false;
    if (lazy) {
        if (!h->dbgSkipExport && !host_rec) {
            hipLaunchKernelGGL(pc_halo_export, dim3(n < 1024 ? n : 1024), dim3(64), 0, h->stream, h->dRes, n,
                               h->dRec, (int)grid.x, h->hResDev);
            RS_HIP(hipGetLastError());
        }
        h->haloPend = true;
        h->haloCur = cl;
        h->haloPart = pl;
    } else {
        own_export = !h->dbgSkipExport && n <= HF_EXP_MAX;
        RS_TRY(finish(own_export ? n : 0, h->exportDev));
        if (!h->dbgSkipExport && !own_export) {
            hipLaunchKernelGGL(pc_res_export, dim3(n < 1024 ? n : 1024), dim3(64), 0, h->stream, h->dRes, n,
                               h->hResDev);
            RS_HIP(hipGetLastError());
        }
    }
    const bool skipped = h->dbgSkipExport;
    h->dbgSkipExport = false;
    if (pk) RS_HIP(hipEventRecord(h->evPool[2 * n + 1], h->stream));
    if (h->profiling) RS_HIP(hipEventRecord(h->ev1, h->stream));
    // A one-step call returns as soon as every block's record has reached the pinned host
    // array, without waiting for the kernel's completion signal and the host's wake-up
    // (update() at 64x64x36: 22.5-24.3 -> 16.8-18.9 us, tools/pc_ab.py --mode update,
    // round 5).  What makes the early return safe: the host reads nothing but the
    // records, each block's last store (one 16-byte store, both words non-zero, checked
    // after the host zeroed them); the state and every other result stay on the device,
    // and every later access to them -- the next step, a read, inject, get_max,
    // settle -- is a launch or copy ordered on this stream behind the kernel (the
    // library's volume reads into pinned memory synchronise the stream themselves).
    // A spin that runs out (a slow or faulted kernel) falls back to the stream
    // synchronisation, which returns any error.
    bool polled = false;
    if (flag_poll && !lazy && !skipped) {
        // the eager readback: every finishing block's flag (its volume slice released at
        // system scope before it), then every step's key word
        polled = pc_poll_flags(h, nb, seq) && pc_poll_words(h, 0, n - 1);
    }
    if (lazy && !skipped && poll_env && !h->profiling && n <= HF_POLL_MAX) {
        if (host_rec) {
            const volatile unsigned long long* r = h->hRec;
            const int nr = (int)grid.x;
            int b = 0;
            for (long spin = 0; spin < 4000000 && b < nr; ++spin)
                while (b < nr && r[2 * b] != 0ull && r[2 * b + 1] != 0ull) ++b;
            polled = b == nr;
        } else {
            polled = pc_poll_words(h, 0, n);   // the export kernel's words
        }
    }
    if (!polled) RS_HIP(hipStreamSynchronize(h->stream));
    if (host_rec && !skipped) h->hRes[n - 1] = halo_key_from_records(h->hRec, (int)grid.x);
    if (own_export) {   // the finishing blocks' keys of the last step (a key is never 0)
        unsigned long long m = 0ull;
        bool all = true;
        for (int b = 0; b < nb; ++b) {
            all &= h->hKey[b] != 0ull;
            m = std::max(m, h->hKey[b]);
        }
        h->hRes[n - 1] = all ? m : RES_NONE;
    }
    if (lazy && !skipped && h->hRes[n - 1] == RES_AMBIG) {
        // a cell within HF_NEAR of the last step's peak: key the normalised state itself
        // (its slots were zeroed by the last launch and nothing has reduced into them)
        h->hRes[n - 1] = RES_NONE;
        RS_TRY(finish(0, nullptr));
        hipLaunchKernelGGL(pc_res_export, dim3(1), dim3(64), 0, h->stream, h->dRes + (size_t)(n - 1) * RES_SLOTS, 1,
                           h->hResDev + (n - 1));
        RS_HIP(hipGetLastError());
        if (!(poll_env && pc_poll_words(h, n - 1, n))) RS_HIP(hipStreamSynchronize(h->stream));
        ++h->haloAmbig;
    }
    for (int s = 0; s < n; ++s)
        RS_CHECK(h->hRes[s] != RES_NONE, RS_ERR_HIP,
                 "step %d of %d: its argmax key did not reach the host result buffer after the "
                 "stream synchronised", s, n);
    if (h->profiling) RS_HIP(hipEventElapsedTime(&h->lastMs, h->ev0, h->ev1));
    else h->lastMs = 0.f;  // the call-bracketing events are recorded only while profiling
    if (pk) {
        h->kernelMs[0] = h->kernelMs[1] = 0.0;
        for (int s = 0; s < n; ++s) {
            float a = 0.f;
            RS_HIP(hipEventElapsedTime(&a, h->evPool[2 * s], h->evPool[2 * s + 1]));
            h->kernelMs[0] += a;
        }
        float b = 0.f;
        RS_HIP(hipEventElapsedTime(&b, h->evPool[2 * n], h->evPool[2 * n + 1]));
        h->kernelMs[1] = b;
    }
    if (out_xyz)
        for (int s = 0; s < n; ++s) decode_xyz(h, h->hRes[s], out_xyz + 3 * (size_t)s);
    return RS_OK;
}

// Streaming variants instantiated: (BX rows per wave, WR row groups, WC column tiles of 64).
#define PC_STREAM_VARIANTS(X_) X_(1, 8, 1) X_(2, 8, 1)

template <typename T, typename CTL>
int pc_launch_stream(rs_pc* h, const T* P, T* Q, unsigned long long* slot, T* bmax, unsigned* bidx,
                     const CTL* ctl, int prof_base) {
    const StreamGrid G = h->sg;
    const dim3 grid(G.gx * G.gy * G.gz), block(64 * h->swr * h->swc);
    const SepKernel<T>& k = sep_of<T>(h);
    const T* filt = static_cast<const T*>(h->dFilt);
    bool done = false;
#define PC_EXCITE_CASE(bx_, wr_, wc_)                                                         \
    if (!done && h->sbx == bx_ && h->swr == wr_ && h->swc == wc_) {                           \
        hipLaunchKernelGGL((pc_excite_stream<T, bx_, wr_, wc_>), grid, block, 0, h->stream, P, \
                           Q,                                                                 \
                           h->dPart, slot, h->X, h->Y, h->TH, G, k);                          \
        done = true;                                                                          \
    }
    PC_STREAM_VARIANTS(PC_EXCITE_CASE)
#undef PC_EXCITE_CASE
    RS_CHECK(done, RS_ERR_STATE, "no streaming variant BX=%d WR=%d WC=%d", h->sbx, h->swr, h->swc);
    RS_HIP(hipGetLastError());
    if (prof_base >= 0) RS_HIP(hipEventRecord(h->evPool[prof_base + 1], h->stream));
    if (!ctl) return RS_OK;
    if (prof_base >= 0) RS_HIP(hipEventRecord(h->evPool[prof_base + 2], h->stream));
    done = false;
#define PC_PATH_CASE(bx_, wr_, wc_)                                                              \
    if (!done && h->sbx == bx_ && h->swr == wr_ && h->swc == wc_) {                              \
        hipLaunchKernelGGL((pc_path_stream<T, bx_, wr_, wc_, CTL>), grid, block, 0, h->stream, Q, \
                           static_cast<T*>(h->dP), h->dPart, h->nPart, filt, h->nf, *ctl, slot,  \
                           bmax, bidx, h->X, h->Y, h->TH, G);                                    \
        done = true;                                                                             \
    }
    PC_STREAM_VARIANTS(PC_PATH_CASE)
#undef PC_PATH_CASE
    RS_HIP(hipGetLastError());
    return RS_OK;
}

template <typename T, typename CTL>
int pc_launch_step(rs_pc* h, const StepOut& so, const CTL* ctl, int prof_base) {
    const T* P = static_cast<const T*>(h->dP);
    T* Q = static_cast<T*>(h->dQ);
    const SepKernel<T>& k = sep_of<T>(h);
    unsigned long long* slot = so.slot;
    T* bmax = static_cast<T*>(so.bmax);
    unsigned* bidx = so.bidx;
    const T* filt = static_cast<const T*>(h->dFilt);
    if (prof_base >= 0) RS_HIP(hipEventRecord(h->evPool[prof_base], h->stream));
    if (h->cols) {
        const dim3 g(h->cgx * h->cgy * h->coNch);
        const bool whole = h->coKC >= h->TH;
        constexpr int THF = co_thmax<T>(), THC = co_thmax_chunk<T>();
        bool fixed = false;
        if constexpr (std::is_same<T, float>::value) {
            if (whole && h->TH == CO_DMA_TH) {  // configs[3]'s theta extent
                hipLaunchKernelGGL((pc_excite_cols<float, CO_TX, CO_TY, CO_NW, CO_DMA_TH, false, CO_DMA_TH>), g,
                                   dim3(64 * CO_NW), 0, h->stream, P, h->X, h->Y, h->TH, h->cgx, h->cgy,
                                   (int)g.x, Q, h->dPart, slot, h->coKC, k);
                fixed = true;
            }
        }
        if (fixed) {
        } else if (whole)
            hipLaunchKernelGGL((pc_excite_cols<T, CO_TX, CO_TY, co_nw<T>(), THF, false>), g, dim3(64 * co_nw<T>()), 0,
                               h->stream, P, h->X, h->Y, h->TH, h->cgx, h->cgy, (int)g.x, Q, h->dPart, slot,
                               h->coKC, k);
        else
            hipLaunchKernelGGL((pc_excite_cols<T, CO_TX, CO_TY, CO_NW_CHUNK, THC, true>), g,
                               dim3(64 * CO_NW_CHUNK), 0, h->stream, P, h->X, h->Y, h->TH, h->cgx, h->cgy,
                               (int)g.x, Q, h->dPart, slot, h->coKC, k);
        RS_HIP(hipGetLastError());
        if (prof_base >= 0) RS_HIP(hipEventRecord(h->evPool[prof_base + 1], h->stream));
        if (!ctl) return RS_OK;
        if (prof_base >= 0) RS_HIP(hipEventRecord(h->evPool[prof_base + 2], h->stream));
        bool launched = false;
        if constexpr (std::is_same<T, float>::value && std::is_same<CTL, PcCtlInline>::value) {
            // TH == 72 (configs[3]): the LDS-DMA window instance
            if (whole && h->TH == CO_DMA_TH) {
                hipLaunchKernelGGL((pc_path_cols<float, CO_TX, CO_TY, CO_NW, CO_DMA_TH, false, PcCtlInline, CO_DMA_TH>),
                                   g, dim3(64 * CO_NW), 0, h->stream, Q, h->X, h->Y, h->TH, h->cgx, h->cgy,
                                   (int)g.x, static_cast<T*>(h->dP), h->dPart, h->nPart, filt, h->nf, *ctl, slot,
                                   bmax, bidx, h->coKC);
                launched = true;
            }
        }
        if (launched) {
        } else if (whole)
            hipLaunchKernelGGL((pc_path_cols<T, CO_TX, CO_TY, co_nw<T>(), THF, false, CTL>), g, dim3(64 * co_nw<T>()), 0,
                               h->stream, Q, h->X, h->Y, h->TH, h->cgx, h->cgy, (int)g.x, static_cast<T*>(h->dP),
                               h->dPart, h->nPart, filt, h->nf, *ctl, slot, bmax, bidx, h->coKC);
        else
            hipLaunchKernelGGL((pc_path_cols<T, CO_TX, CO_TY, CO_NW_CHUNK, THC, true, CTL>), g,
                               dim3(64 * CO_NW_CHUNK), 0, h->stream, Q, h->X, h->Y, h->TH, h->cgx, h->cgy,
                               (int)g.x, static_cast<T*>(h->dP), h->dPart, h->nPart, filt, h->nf, *ctl, slot,
                               bmax, bidx, h->coKC);
    } else if (h->streamed) {
        RS_TRY((pc_launch_stream<T, CTL>(h, P, Q, slot, bmax, bidx, ctl, prof_base)));
    } else if (h->tiling == 64 || h->tiling == 128) {
        const dim3 g((h->X + RT_BX - 1) / RT_BX, (h->TH + RT_BK - 1) / RT_BK);
        if (h->tiling == 64)
            hipLaunchKernelGGL((pc_excite_rows<T, 64>), g, dim3(RT_NT), 0, h->stream, P, Q,
                               h->dPart, slot, h->X, h->Y, h->TH, k);
        else
            hipLaunchKernelGGL((pc_excite_rows<T, 128>), g, dim3(RT_NT), 0, h->stream, P, Q,
                               h->dPart, slot, h->X, h->Y, h->TH, k);
        RS_HIP(hipGetLastError());
        if (prof_base >= 0) RS_HIP(hipEventRecord(h->evPool[prof_base + 1], h->stream));
        if (!ctl) return RS_OK;  // rs_pc_excite() normalises with pc_scale_kernel
        if (prof_base >= 0) RS_HIP(hipEventRecord(h->evPool[prof_base + 2], h->stream));
        if (h->tiling == 64)
            hipLaunchKernelGGL((pc_path_rows<T, 64, CTL>), g, dim3(RT_NT), 0, h->stream, Q,
                               static_cast<T*>(h->dP), h->dPart, h->nPart, filt, h->nf, *ctl, slot,
                               bmax, bidx, h->X, h->Y, h->TH);
        else
            hipLaunchKernelGGL((pc_path_rows<T, 128, CTL>), g, dim3(RT_NT), 0, h->stream, Q,
                               static_cast<T*>(h->dP), h->dPart, h->nPart, filt, h->nf, *ctl, slot,
                               bmax, bidx, h->X, h->Y, h->TH);
    } else {
        const dim3 gA((h->Y + EX_BY - 1) / EX_BY, (h->X + EX_BX - 1) / EX_BX,
                      (h->TH + EX_BK - 1) / EX_BK);
        hipLaunchKernelGGL((pc_excite_kernel<T, EX_BX, EX_BY, EX_BK>), gA, dim3(NT), 0, h->stream,
                           P, Q, h->dPart, slot, h->X, h->Y, h->TH, k);
        RS_HIP(hipGetLastError());
        if (prof_base >= 0) RS_HIP(hipEventRecord(h->evPool[prof_base + 1], h->stream));
        if (!ctl) return RS_OK;
        if (prof_base >= 0) RS_HIP(hipEventRecord(h->evPool[prof_base + 2], h->stream));
        const dim3 gB((h->Y + PI_BY - 1) / PI_BY, (h->X + PI_BX - 1) / PI_BX,
                      (h->TH + PI_BK - 1) / PI_BK);
        hipLaunchKernelGGL((pc_path_kernel<T, PI_BX, PI_BY, PI_BK, CTL>), gB, dim3(NT), 0, h->stream, Q,
                           static_cast<T*>(h->dP), h->dPart, h->nPart, filt, *ctl, slot, bmax,
                           bidx, h->X, h->Y, h->TH);
    }
    RS_HIP(hipGetLastError());
    if (prof_base >= 0) RS_HIP(hipEventRecord(h->evPool[prof_base + 3], h->stream));
    return RS_OK;
}

void decode_xyz(const rs_pc* h, unsigned long long key, int32_t* out) {
    const unsigned lin = 0xFFFFFFFFu - (unsigned)(key & 0xFFFFFFFFull);
    out[2] = (int32_t)(lin % (unsigned)h->TH);
    const unsigned xy = lin / (unsigned)h->TH;
    out[1] = (int32_t)(xy % (unsigned)h->Y);
    out[0] = (int32_t)(xy / (unsigned)h->Y);
}

// n steps launched one by one on the handle's stream, then one export and a sync.
int pc_run_direct(rs_pc* h, int n, const int32_t* ox, const int32_t* oy, const int32_t* fidx,
                  const double* zf, int32_t* out_xyz) {
    if (n == 0) return RS_OK;
    if (h->halo) return pc_run_halo(h, n, ox, oy, fidx, zf, out_xyz);
    // Batches: the column form takes each step's control as kernel arguments too (its
    // path kernel then starts its window loads without a global round trip for the
    // shifts: 128x128x72 27.5 -> 27.1 us per step with the filter table staged behind
    // the window); the other forms read the device ring
    const bool inline_ctl = (n == 1 || h->cols) && h->TH <= CTL_INLINE_MAX;
    RS_TRY(pc_grow_steps(h, n, !inline_ctl));
    if (!inline_ctl) {
        RS_TRY(pc_pack_ctl(h, n, ox, oy, fidx, zf));
        RS_HIP(hipMemcpyAsync(h->dCtl, h->hCtl, h->ctlStride * n, hipMemcpyHostToDevice,
                              h->stream));
    }
    const bool pk = h->profiling && h->profKernels;
    if (pk) RS_TRY(pc_ensure_events(h, (size_t)4 * n));
    if (h->profiling) RS_HIP(hipEventRecord(h->ev0, h->stream));
    for (int s = 0; s < n; ++s) {
        const int pb = pk ? 4 * s : -1;
        if (inline_ctl) {
            PcCtlInline c;
            make_ctl_inline(h, s, ox, oy, fidx, zf, &c);
            if (h->prec == RS_PREC_F32)
                RS_TRY((pc_launch_step<float, PcCtlInline>(h, step_out(h, s), &c, pb)));
            else
                RS_TRY((pc_launch_step<double, PcCtlInline>(h, step_out(h, s), &c, pb)));
        } else {
            const PcCtlRing c = make_ctl_ring(h, s);
            if (h->prec == RS_PREC_F32)
                RS_TRY((pc_launch_step<float, PcCtlRing>(h, step_out(h, s), &c, pb)));
            else
                RS_TRY((pc_launch_step<double, PcCtlRing>(h, step_out(h, s), &c, pb)));
        }
    }
    if (h->prec == RS_PREC_F64) {
        hipLaunchKernelGGL((pc_argmax_steps<double>), dim3(n), dim3(NT), 0, h->stream,
                           static_cast<const double*>(h->dArgV), h->dArgI, h->nPathBlocks, h->dRes);
        RS_HIP(hipGetLastError());
    }
    for (int s = 0; s < n; ++s) h->hRes[s] = RES_NONE;
    const bool skipped = h->dbgSkipExport;
    if (!h->dbgSkipExport) {
        hipLaunchKernelGGL(pc_res_export, dim3(n < 1024 ? n : 1024), dim3(64), 0,
                           h->stream, h->dRes, n, h->hResDev);
        RS_HIP(hipGetLastError());
    }
    h->dbgSkipExport = false;
    // the volume after the last step, into the caller's pinned array (the eager
    // readback), its blocks' flags polled when the call may return early
    const bool may_poll = halo_poll_env() && !h->profiling && !skipped && n <= HF_POLL_MAX;
    int xnb = 0;
    unsigned seq = 0u;
    if (h->exportDev) {
        xnb = (int)std::min<size_t>(1024, (h->n / 2 + NT - 1) / NT + 1);
        const bool fl = may_poll && pc_flags_ok(h, xnb);
        if (fl) xnb = pc_xflag_nb(xnb);
        seq = fl ? pc_next_seq(h) : 0u;
        unsigned* flag = fl ? h->hFlagDev : nullptr;
        if (h->prec == RS_PREC_F32)
            hipLaunchKernelGGL((pc_export2_kernel<float>), dim3(xnb), dim3(NT), 0, h->stream,
                               static_cast<const float*>(h->dP), h->exportDev, h->X, h->Y, h->TH, (int)pc_thfast(h),
                               flag, seq);
        else
            hipLaunchKernelGGL((pc_export2_kernel<double>), dim3(xnb), dim3(NT), 0, h->stream,
                               static_cast<const double*>(h->dP), h->exportDev, h->X, h->Y, h->TH, (int)pc_thfast(h),
                               flag, seq);
        RS_HIP(hipGetLastError());
    }
    if (h->profiling) RS_HIP(hipEventRecord(h->ev1, h->stream));
    // the result words polled (pc_poll_words), and with an eager readback the volume's
    // flags first (each block's stores released at system scope before its flag), unless
    // the call is profiled, long or its export was withheld (RS_PC_HALO_POLL=0: always the
    // stream synchronisation; RS_PC_HALO_FLAGS=0: for an eager readback)
    const bool polled = may_poll && (h->exportDev ? seq != 0u && pc_poll_flags(h, xnb, seq) : true) &&
                        pc_poll_words(h, 0, n);
    if (!polled) RS_HIP(hipStreamSynchronize(h->stream));
    for (int s = 0; s < n; ++s)
        RS_CHECK(h->hRes[s] != RES_NONE, RS_ERR_HIP,
                 "step %d of %d: its argmax key did not reach the host result buffer after the "
                 "stream synchronised", s, n);
    if (h->profiling) RS_HIP(hipEventElapsedTime(&h->lastMs, h->ev0, h->ev1));
    else h->lastMs = 0.f;  // the step-bracketing events are recorded only while profiling
    if (pk) {
        h->kernelMs[0] = h->kernelMs[1] = 0.0;
        for (int s = 0; s < n; ++s) {
            float a = 0.f, b = 0.f;
            RS_HIP(hipEventElapsedTime(&a, h->evPool[4 * s], h->evPool[4 * s + 1]));
            RS_HIP(hipEventElapsedTime(&b, h->evPool[4 * s + 2], h->evPool[4 * s + 3]));
            h->kernelMs[0] += a;
            h->kernelMs[1] += b;
        }
    }
    if (out_xyz)
        for (int s = 0; s < n; ++s)
            decode_xyz(h, h->hRes[s], out_xyz + 3 * (size_t)s);
    return RS_OK;
}

int pc_run_impl(rs_pc* h, int n, const int32_t* ox, const int32_t* oy, const int32_t* fidx,
                const double* zf, int32_t* out_xyz) {
    RS_CHECK(h, RS_ERR_STATE, "null pose-cell handle");
    RS_CHECK(n >= 0, RS_ERR_ARG, "negative step count");
    if (n == 0) return RS_OK;
    RS_HIP(hipSetDevice(h->device));
    RS_TRY(pc_check_ctl(h, n, ox, oy, fidx, zf));
    return pc_run_direct(h, n, ox, oy, fidx, zf, out_xyz);
}

// path_integration's control for one step (posecell_network.py:252-308) in the
// operation order of filters.step_control: vt = vtrans/0.2, vr = vrot/(2pi/TH),
// e = vt*cos|sin (:257-261), o = around(e) (:262-265, half-even = rint), key =
// int((e_x - o_x)*10) (:246-249), theta origin floor(vr + .5) (:304).  Each is one
// correctly rounded IEEE operation on the same operands as NumPy's, and
// contraction is off, so the result is bit-identical.  Returns RS_ERR_LUT_KEY on
// a key outside the LUT (the reference's KeyError, :249; checked before the theta
// filter, as the reference builds the xy filters first) and RS_ERR_CTL_RANGE when
// the theta origin or a shift lies outside what the tables cover.
constexpr double PC_LUT_PRECISION = 10.0;  // filter_dict_2d_precision, posecell_network.py:48

static inline __attribute__((always_inline)) int pc_odom_control_body(const OdoTables* h, double vtrans, double vrot,
                                                                      int32_t* ox, int32_t* oy, int32_t* rows, double* zf) {
#pragma clang fp contract(off)
    const double vt = vtrans / h->vtScale;
    const double vr = vrot / h->vrScale;
    for (int k = 0; k < h->TH; ++k) {
        const double ex = vt * h->cosA[k];
        const double ey = vt * h->sinA[k];
        const double rx = std::nearbyint(ex);
        const double ry = std::nearbyint(ey);
        const double key = std::trunc((ex - rx) * PC_LUT_PRECISION);
        if (!(key >= h->keyMin && key < h->keyMin + h->nKeys)) return RS_ERR_LUT_KEY;  // NaN too
        if (!(std::fabs(rx) < 1073741824.0 && std::fabs(ry) < 1073741824.0)) return RS_ERR_CTL_RANGE;
        ox[k] = (int32_t)rx;
        oy[k] = (int32_t)ry;
        rows[k] = h->keyRows[(int)key - h->keyMin];
    }
    const double zo = std::floor(vr + 0.5);
    if (!std::isfinite(zo)) {
        // Python 2's math.floor returns a NaN or infinite argument as it is, and the
        // theta filter built on it is all NaN (filters.theta_filter): the reference runs
        // on with a NaN volume (posecell_network.py:304-310)
        for (int t = 0; t < FL; ++t) zf[t] = std::numeric_limits<double>::quiet_NaN();
        return RS_OK;
    }
    if (!(zo >= h->zMin && zo < h->zMin + h->nZ)) return RS_ERR_CTL_RANGE;
    const double* f = h->zfTab + (size_t)((int)zo - h->zMin) * FL;
    for (int t = 0; t < FL; ++t) zf[t] = f[t];
    return RS_OK;
}
// The same operations compiled for SSE4.1 (nearbyint, trunc and floor become roundsd
// with the same IEEE results: 0.80 -> 0.42 us per 72-layer step on the build host), used
// when the CPU has it
__attribute__((target("sse4.1"))) int pc_odom_control_sse41(const OdoTables* h, double vtrans, double vrot,
                                                           int32_t* ox, int32_t* oy, int32_t* rows, double* zf) {
    return pc_odom_control_body(h, vtrans, vrot, ox, oy, rows, zf);
}
int pc_odom_control_base(const OdoTables* h, double vtrans, double vrot, int32_t* ox, int32_t* oy, int32_t* rows,
                         double* zf) {
    return pc_odom_control_body(h, vtrans, vrot, ox, oy, rows, zf);
}
int pc_odom_control(const OdoTables* h, double vtrans, double vrot, int32_t* ox, int32_t* oy, int32_t* rows,
                    double* zf) {
    static const bool sse41 = __builtin_cpu_supports("sse4.1");
    return sse41 ? pc_odom_control_sse41(h, vtrans, vrot, ox, oy, rows, zf)
                 : pc_odom_control_base(h, vtrans, vrot, ox, oy, rows, zf);
}

template <typename T>
int pc_argmax_impl(rs_pc* h, int32_t* out) {
    const int nb = h->nBmaxCap < 1024 ? h->nBmaxCap : 1024;
    hipLaunchKernelGGL((pc_argmax_blocks<T>), dim3(nb), dim3(NT), 0, h->stream,
                       static_cast<const T*>(h->dP), h->X, h->Y, h->TH, static_cast<T*>(h->dBmax),
                       h->dBidx, (int)pc_thfast(h));
    RS_HIP(hipGetLastError());
    hipLaunchKernelGGL((pc_argmax_finalize<T>), dim3(1), dim3(NT), 0, h->stream,
                       static_cast<const T*>(h->dBmax), h->dBidx, nb, h->dRes);
    RS_HIP(hipGetLastError());
    RS_HIP(hipMemcpyAsync(h->hRes, h->dRes, sizeof(unsigned long long), hipMemcpyDeviceToHost,
                          h->stream));
    RS_HIP(hipStreamSynchronize(h->stream));
    decode_xyz(h, h->hRes[0], out);
    return RS_OK;
}

template <typename T>
void fill_sep(SepKernel<T>& k, const rs_pc_params* p) {
    for (int t = 0; t < FL; ++t) {
        k.ge[t] = (T)p->ge[t];
        k.gi[t] = (T)p->gi[t];
    }
    k.scale = (T)p->k_scale;
    k.inhib = (T)p->global_inhibition;
}

// Scale the excited volume by 1/total in place (rs_pc_excite only).
template <typename T>
__global__ void pc_scale_kernel(T* __restrict__ P, size_t n, const double* __restrict__ part,
                                int npart) {
    __shared__ double s_red[NT / 64];
    double t = 0.0;
    for (int i = threadIdx.x; i < npart; i += NT) t += part[i];
    t = block_sum(t, s_red);
    if (t == 0.0) return;
    const PcNorm<T> nrm(t);
    for (size_t e = blockIdx.x * (size_t)NT + threadIdx.x; e < n; e += (size_t)gridDim.x * NT)
        P[e] = nrm(P[e]);
}

// Step-kernel form.  Default: rows below ST_MIN_CELLS; above it the column form
// where it fits (pc_cols_fit), else layer streaming with one wave per 64 columns
// and 8 row groups of BX rows, KC (layers per block) the smallest chunk that keeps
// the grid within ~2 blocks per CU (fewer, longer blocks re-evaluate fewer halo
// layers).  RS_PC_FORM=rows|tiles|cols|stream:BX,WR[,KC] overrides (A/B, tests).
// Scratch traffic in the layer loop defeats the streaming kernels' prefetch
// pipeline: refuse a variant that spills.
template <typename T>
int pc_stream_scratch(int bx, int wr, int wc, size_t* bytes) {
    hipFuncAttributes a{};
    *bytes = 0;
    bool done = false;
#define PC_SCRATCH(bx_, wr_, wc_)                                                                      \
    if (!done && bx == bx_ && wr == wr_ && wc == wc_) {                                                \
        const void* fns[3] = {                                                                         \
            reinterpret_cast<const void*>(&pc_excite_stream<T, bx_, wr_, wc_>),                        \
            reinterpret_cast<const void*>(&pc_path_stream<T, bx_, wr_, wc_, PcCtlRing>),               \
            reinterpret_cast<const void*>(&pc_path_stream<T, bx_, wr_, wc_, PcCtlInline>)};            \
        for (const void* f : fns) {                                                          \
            RS_HIP(hipFuncGetAttributes(&a, f));                                             \
            *bytes += a.localSizeBytes;                                                      \
        }                                                                                    \
        done = true;                                                                         \
    }
    PC_STREAM_VARIANTS(PC_SCRATCH)
#undef PC_SCRATCH
    return RS_OK;
}

// The column kernels' limits: single-conditional wraps, the window in LDS, the
// filter table in LDS.
bool pc_cols_fit(const rs_pc* h) {
    const int vec = h->esz == 4 ? co_vec<float>() : co_vec<double>();
    return h->X >= CO_TX + 2 * HALF && h->Y >= CO_TY + 2 * HALF + 4 && h->Y % vec == 0 &&
           h->TH >= CO_CH + 2 && h->nf <= RT_NFMAX;
}

// Theta chunking of the column form: kc = 0 picks it.  The whole extent in one
// block per CU when it fits the LDS window (no halo layers); KC < TH puts KC + 6
// layers in each of two blocks per CU.
int pc_cols_set(rs_pc* h, int kc) {
    const int thf = h->esz == 4 ? co_thmax<float>() : co_thmax<double>();
    const int thc = h->esz == 4 ? co_thmax_chunk<float>() : co_thmax_chunk<double>();
    if (kc <= 0) {
        kc = h->TH;
        if (h->TH > thf) {  // more layers than one block holds: the fewest chunks that fit
            const int nch = (h->TH + thc - 2 * HALF - 1) / (thc - 2 * HALF);
            kc = (h->TH + nch - 1) / nch;
        }
    }
    RS_CHECK(kc >= 1 && kc <= h->TH, RS_ERR_ARG, "cols KC=%d outside [1, %d]", kc, h->TH);
    RS_CHECK(kc < h->TH ? kc + 2 * HALF <= thc : h->TH <= thf, RS_ERR_ARG,
             "cols KC=%d: %d window layers exceed the LDS window (%d whole, %d per chunk)", kc,
             kc < h->TH ? kc + 2 * HALF : kc, thf, thc);
    h->streamed = false;
    h->cols = true;
    h->cgx = (h->X + CO_TX - 1) / CO_TX;
    h->cgy = (h->Y + CO_TY - 1) / CO_TY;
    h->coKC = kc;
    h->coNch = (h->TH + kc - 1) / kc;
    return RS_OK;
}

// The halo form's limits: float32, the instantiated theta extent, the 16 x 16 layer
// windows without self-overlap, the filter table in LDS, 32-bit buffer offsets.
bool pc_halo_fit(const rs_pc* h) {
    // (the union's origin and extent travel as 16-bit fields: make_ctl_halo, hf_pack)
    // (so do the grid, the tile count and the block count of pc_step_halo; tile / gx is a
    // high multiply valid below 2^16, hf_magic)
    return h->esz == 4 && hf_th_ok(h->TH) && h->X >= HF_W && h->Y >= HF_W && h->X <= 32767 && h->Y <= 32767 &&
           (size_t)((h->X + HF_T - 1) / HF_T) * ((h->Y + HF_T - 1) / HF_T) <= 65535 &&
           h->nf <= RT_NFMAX && h->n * sizeof(float) <= (size_t)INT_MAX && h->n % 4 == 0;   // (pc_halo_finish: float4s)
}

int pc_halo_set(rs_pc* h) {
    h->streamed = false;
    h->cols = false;
    h->halo = true;
    h->cgx = (h->X + HF_T - 1) / HF_T;
    h->cgy = (h->Y + HF_T - 1) / HF_T;
    return RS_OK;
}

// The halo form by default where it fits and its tiles fill at most one block per CU
// (every block holds ~155 KiB of LDS): 64x64x36 9.49 vs 11.23 us per batched step
// against rows, 21x21x36 10.00 vs 11.12 (tools/pc_ab.py, 3 rounds, one box)
constexpr int HF_DEFAULT_MAX_TILES = 256;
bool pc_halo_default(const rs_pc* h) {
    return pc_halo_fit(h) && (size_t)((h->X + HF_T - 1) / HF_T) * ((h->Y + HF_T - 1) / HF_T) <=
                                 (size_t)HF_DEFAULT_MAX_TILES;
}

int pc_choose_form(rs_pc* h) {
    int bx = 1, wr = 8, wc = 1, kc = 0;
    const char* env = std::getenv("RS_PC_FORM");
    if ((env == nullptr || env[0] == 0) && pc_halo_default(h)) return pc_halo_set(h);
    if (env && std::strcmp(env, "halo") == 0) {
        RS_CHECK(pc_halo_fit(h), RS_ERR_ARG,
                 "RS_PC_FORM=halo needs float32, TH 10, 18 or %d, %d <= X, Y <= 32767 and at most %d path filters", HF_TH,
                 HF_W, RT_NFMAX);
        return pc_halo_set(h);
    }
    if (env && std::strcmp(env, "rows") == 0) {
        RS_CHECK(h->tiling != 0, RS_ERR_ARG, "RS_PC_FORM=rows needs Y <= 128");
        h->streamed = false;
        return RS_OK;
    }
    if (env && std::strcmp(env, "tiles") == 0) {
        h->streamed = false;
        h->tiling = 0;
        return RS_OK;
    }
    if (env && (std::strcmp(env, "cols") == 0 || std::strncmp(env, "cols:", 5) == 0)) {
        RS_CHECK(pc_cols_fit(h), RS_ERR_ARG,
                 "RS_PC_FORM=cols needs X >= %d, Y >= %d and a multiple of %d, TH >= %d and at most %d "
                 "path filters",
                 CO_TX + 2 * HALF, CO_TY + 2 * HALF + 4, h->esz == 4 ? co_vec<float>() : co_vec<double>(),
                 CO_CH + 2, RT_NFMAX);
        return pc_cols_set(h, env[4] == ':' ? std::atoi(env + 5) : 0);
    }
    const bool explicit_stream = env && std::strncmp(env, "stream:", 7) == 0;
    if (explicit_stream) {
        const int n = std::sscanf(env + 7, "%d,%d,%d,%d", &bx, &wr, &wc, &kc);
        RS_CHECK(n >= 3, RS_ERR_ARG, "RS_PC_FORM=stream:BX,WR,WC[,KC], got '%s'", env);
    } else {
        RS_CHECK(env == nullptr || env[0] == 0 || std::strcmp(env, "stream") == 0, RS_ERR_ARG,
                 "unknown RS_PC_FORM '%s' (rows | tiles | cols | halo | stream[:BX,WR,WC[,KC]])", env);
        // default: one pass per kernel (rows) while the whole grid fits in one wave of
        // blocks -- the step is latency-bound there (64x64x36: 17 us rows vs 23 us
        // streamed); streamed once the rows form's 4x theta-halo recompute dominates
        // (128x128x72: 57 us rows vs 41 us streamed)
        const bool big = (size_t)h->X * h->Y * h->TH >= ST_MIN_CELLS;
        if ((env == nullptr || env[0] == 0) && h->tiling != 0 && !big) {
            h->streamed = false;
            return RS_OK;
        }
        // large grids: the column form where it fits (128x128x72: 29.3 us per step
        // vs 38.8 us streamed, tools/pc_sweep.py), else the streamed form
        if ((env == nullptr || env[0] == 0) && big && pc_cols_fit(h)) return pc_cols_set(h, 0);
        bx = h->esz == 4 ? ST_DEF_BX : 1;
        wr = ST_DEF_WR;
        wc = ST_DEF_WC;
    }
    if (h->nf > RT_NFMAX) {  // filter table too large to stage in LDS: rows / tiles forms
        RS_CHECK(env == nullptr || std::strncmp(env, "stream", 6) != 0, RS_ERR_ARG,
                 "stream form stages at most %d path filters, table has %d", RT_NFMAX, h->nf);
        h->streamed = false;
        return RS_OK;
    }
    bool known = false;
#define PC_KNOWN(bx_, wr_, wc_) known = known || (bx == bx_ && wr == wr_ && wc == wc_);
    PC_STREAM_VARIANTS(PC_KNOWN)
#undef PC_KNOWN
    RS_CHECK(known, RS_ERR_ARG, "no streaming variant BX=%d WR=%d WC=%d", bx, wr, wc);
    size_t scratch = 0;
    if (h->esz == 4)
        RS_TRY(pc_stream_scratch<float>(bx, wr, wc, &scratch));
    else
        RS_TRY(pc_stream_scratch<double>(bx, wr, wc, &scratch));
    RS_CHECK(scratch == 0, RS_ERR_ARG,
             "streaming variant BX=%d WR=%d WC=%d spills %zu B to scratch at this precision", bx, wr,
             wc, scratch);
    const int bxb = bx * wr, yt = 64 * wc;
    StreamGrid g;
    g.gx = (h->X + bxb - 1) / bxb;
    g.gy = (h->Y + yt - 1) / yt;
    const int maxkc = st_maxkc((int)h->esz, bxb, yt);
    if (kc <= 0) {
        // smallest chunk that keeps the grid within one block per CU: a second block
        // on some CUs doubles their share (fewer, longer blocks also re-evaluate
        // fewer halo layers)
        const int target = 256;
        kc = 2;
        while (kc < maxkc && kc < h->TH && (long)g.gx * g.gy * ((h->TH + kc - 1) / kc) > target) ++kc;
    }
    RS_CHECK(kc >= 1 && kc <= maxkc, RS_ERR_ARG, "stream KC=%d outside [1, %d]", kc, maxkc);
    if (kc > h->TH) kc = h->TH;
    g.KC = kc;
    g.gz = (h->TH + g.KC - 1) / g.KC;
    RS_CHECK((long)g.gx * g.gy * g.gz <= NPP_MAX_BLOCKS, RS_ERR_ARG,
             "streaming grid of %ld blocks exceeds %d", (long)g.gx * g.gy * g.gz, NPP_MAX_BLOCKS);
    h->streamed = true;
    h->sbx = bx;
    h->swr = wr;
    h->swc = wc;
    h->sg = g;
    return RS_OK;
}

}  // namespace

// ---------------------------------------------------------------------------
// extern "C" entry points
// ---------------------------------------------------------------------------
extern "C" {

int rs_pc_create(int X, int Y, int TH, const rs_pc_params* p, int device, rs_pc** out) {
    rs::clear_error();
    RS_CHECK(out, RS_ERR_ARG, "null output handle pointer");
    *out = nullptr;
    RS_CHECK(p, RS_ERR_ARG, "null parameters");
    RS_CHECK(X >= HALF && Y >= HALF && TH >= HALF, RS_ERR_ARG,
             "grid (%d, %d, %d): every dimension must be >= %d (3-cell wrap halo, convolution.py:52-81)",
             X, Y, TH, HALF);
    RS_CHECK((size_t)X * Y * TH < 0xFFFFFFFFull, RS_ERR_ARG, "grid too large for 32-bit cell index");
    RS_CHECK(p->precision == RS_PREC_F32 || p->precision == RS_PREC_F64, RS_ERR_ARG,
             "precision must be RS_PREC_F32 or RS_PREC_F64");
    RS_CHECK(p->nfilters >= 1 && p->xy_filters, RS_ERR_ARG, "empty path-integration filter table");
    int ndev = 0;
    RS_HIP(hipGetDeviceCount(&ndev));
    RS_CHECK(device >= 0 && device < ndev, RS_ERR_ARG, "device %d not in [0, %d)", device, ndev);
    RS_HIP(hipSetDevice(device));

    rs_pc* h = new rs_pc();
    h->X = X; h->Y = Y; h->TH = TH; h->prec = p->precision; h->device = device;
    h->n = (size_t)X * Y * TH;
    h->esz = p->precision == RS_PREC_F32 ? 4 : 8;
    h->nf = p->nfilters;
    fill_sep(h->kf, p);
    fill_sep(h->kd, p);
    h->ctlStride = rs::round_up(ctl_off_zf(h) + sizeof(double) * 8, 16);
    h->tiling = Y <= 64 ? 64 : (Y <= 128 ? 128 : 0);
    if (int st = pc_choose_form(h); st != RS_OK) {
        delete h;
        return st;
    }
    if (h->halo) {
        h->nPart = h->cgx * h->cgy;
        h->nPathBlocks = h->nPart;
    } else if (h->cols) {
        h->nPart = h->cgx * h->cgy * h->coNch;
        h->nPathBlocks = h->nPart;
    } else if (h->streamed) {
        h->nPart = h->sg.gx * h->sg.gy * h->sg.gz;
        h->nPathBlocks = h->nPart;
    } else if (h->tiling) {
        h->nPart = ((X + RT_BX - 1) / RT_BX) * ((TH + RT_BK - 1) / RT_BK);
        h->nPathBlocks = h->nPart;
    } else {
        h->nPart = ((Y + EX_BY - 1) / EX_BY) * ((X + EX_BX - 1) / EX_BX) * ((TH + EX_BK - 1) / EX_BK);
        h->nPathBlocks =
            ((Y + PI_BY - 1) / PI_BY) * ((X + PI_BX - 1) / PI_BX) * ((TH + PI_BK - 1) / PI_BK);
    }
    h->nBmaxCap = h->nPathBlocks > 1024 ? h->nPathBlocks : 1024;

    auto fail = [&](int code) { rs_pc_destroy(h); return code; };
    hipError_t e = hipSuccess;
#define PC_ALLOC(call)                                                         \
    do {                                                                       \
        e = (call);                                                            \
        if (e != hipSuccess) {                                                 \
            rs::set_error("%s failed: %s", #call, hipGetErrorString(e));       \
            return fail(e == hipErrorOutOfMemory ? RS_ERR_NOMEM : RS_ERR_HIP); \
        }                                                                      \
    } while (0)
    PC_ALLOC(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
    PC_ALLOC(hipMalloc(&h->dP, h->n * h->esz));
    PC_ALLOC(hipMalloc(&h->dQ, h->n * h->esz));
    PC_ALLOC(hipMemsetAsync(h->dP, 0, h->n * h->esz, h->stream));  // zeros(shape), :27
    // Q and the partials are rewritten in full by every excitation before a path
    // kernel reads them; zeroed anyway so that no launch can see a freed handle's data
    // (rs_pc_debug(RS_PC_DBG_POISON) + tests/test_posecell_gpu.py check the former)
    PC_ALLOC(hipMemsetAsync(h->dQ, 0, h->n * h->esz, h->stream));
    // (the halo form keeps two steps' partial sums: the one it reads, the one it writes)
    PC_ALLOC(hipMalloc(&h->dPart, sizeof(double) * h->nPart * 2));
    PC_ALLOC(hipMemsetAsync(h->dPart, 0, sizeof(double) * h->nPart * 2, h->stream));
    PC_ALLOC(hipMalloc(&h->dRec, sizeof(unsigned long long) * 2 * h->nPart));
    if (h->halo) {
        PC_ALLOC(hipHostMalloc(&h->hRec, sizeof(unsigned long long) * 2 * h->nPart,
                               hipHostMallocMapped | hipHostMallocCoherent));
        PC_ALLOC(hipHostGetDevicePointer(reinterpret_cast<void**>(&h->hRecDev), h->hRec, 0));
    }
    // the volume-writing kernels' per-block flags (pc_halo_finish, pc_export2_kernel)
    PC_ALLOC(hipHostMalloc(&h->hFlag, sizeof(unsigned) * HF_FLAGS, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(h->hFlag, 0, sizeof(unsigned) * HF_FLAGS);
    PC_ALLOC(hipHostGetDevicePointer(reinterpret_cast<void**>(&h->hFlagDev), h->hFlag, 0));
    if (h->halo) {
        PC_ALLOC(hipHostMalloc(&h->hKey, sizeof(unsigned long long) * HF_FLAGS,
                               hipHostMallocMapped | hipHostMallocCoherent));
        PC_ALLOC(hipHostGetDevicePointer(reinterpret_cast<void**>(&h->hKeyDev), h->hKey, 0));
    }
    PC_ALLOC(hipMalloc(&h->dBmax, h->esz * h->nBmaxCap));
    PC_ALLOC(hipMalloc(&h->dBidx, sizeof(unsigned) * h->nBmaxCap));
    PC_ALLOC(hipMalloc(&h->dTmp, sizeof(double) * h->n));
    PC_ALLOC(hipMalloc(&h->dScalar, sizeof(double)));
    PC_ALLOC(hipMalloc(&h->dFilt, h->esz * FT * h->nf));
    if (h->prec == RS_PREC_F32) {
        std::vector<float> f(FT * (size_t)h->nf);
        for (size_t i = 0; i < f.size(); ++i) f[i] = (float)p->xy_filters[i];
        PC_ALLOC(hipMemcpy(h->dFilt, f.data(), f.size() * sizeof(float), hipMemcpyHostToDevice));
    } else {
        PC_ALLOC(hipMemcpy(h->dFilt, p->xy_filters, FT * (size_t)h->nf * sizeof(double),
                           hipMemcpyHostToDevice));
    }
    PC_ALLOC(hipEventCreate(&h->ev0));
    PC_ALLOC(hipEventCreate(&h->ev1));
#undef PC_ALLOC
    int s = pc_grow_steps(h, 16);
    if (s != RS_OK) return fail(s);
    e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) {
        rs::set_error("hipStreamSynchronize failed: %s", hipGetErrorString(e));
        return fail(RS_ERR_HIP);
    }
    *out = h;
    return RS_OK;
}

int rs_pc_destroy(rs_pc* h) {
    if (!h) return RS_OK;
    (void)hipSetDevice(h->device);
    // the handle's last queued work: a fault or launch error the early-returning calls
    // left on the stream is reported here instead of being dropped
    const hipError_t se = h->stream ? hipStreamSynchronize(h->stream) : hipSuccess;
    if (h->hRead) (void)hipHostFree(h->hRead);
    for (void* p : {h->dP, h->dQ, h->dFilt, (void*)h->dPart, (void*)h->dRec, h->dBmax,
                    (void*)h->dBidx, h->dArgV,
                    (void*)h->dArgI,
                    (void*)h->dRes, (void*)h->dCtl, (void*)h->dTmp, (void*)h->dScalar})
        if (p) (void)hipFree(p);
    if (h->hRes) (void)hipHostFree(h->hRes);
    if (h->hRec) (void)hipHostFree(h->hRec);
    if (h->hFlag) (void)hipHostFree(h->hFlag);
    if (h->hKey) (void)hipHostFree(h->hKey);
    if (h->hCtl) (void)hipHostFree(h->hCtl);
    if (h->ev0) (void)hipEventDestroy(h->ev0);
    if (h->ev1) (void)hipEventDestroy(h->ev1);
    for (hipEvent_t e : h->evPool) (void)hipEventDestroy(e);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    RS_CHECK(se == hipSuccess, RS_ERR_HIP, "work queued before rs_pc_destroy failed: %s", hipGetErrorString(se));
    return RS_OK;
}

int rs_pc_shape(const rs_pc* h, int* X, int* Y, int* TH) {
    RS_CHECK(h, RS_ERR_STATE, "null pose-cell handle");
    if (X) *X = h->X;
    if (Y) *Y = h->Y;
    if (TH) *TH = h->TH;
    return RS_OK;
}

int rs_pc_update(rs_pc* h, const int32_t* ox, const int32_t* oy, const int32_t* fidx,
                 const double* zf, int32_t out_xyz[3]) {
    rs::clear_error();
    return pc_run_impl(h, 1, ox, oy, fidx, zf, out_xyz);
}

int rs_pc_run(rs_pc* h, int n, const int32_t* ox, const int32_t* oy, const int32_t* fidx,
              const double* zf, int32_t* out_xyz) {
    rs::clear_error();
    return pc_run_impl(h, n, ox, oy, fidx, zf, out_xyz);
}

int rs_pc_excite(rs_pc* h) {
    rs::clear_error();
    RS_CHECK(h, RS_ERR_STATE, "null pose-cell handle");
    RS_HIP(hipSetDevice(h->device));
    RS_TRY(pc_halo_settle(h));  // (halo: a state a call left unnormalised)
    if (h->halo) {
        // the halo kernel's excitation-only instance: no shifts, Q of the own cells
        PcCtlHalo c{};
        c.uw = (short)HF_W;
        c.uh = (short)HF_W;
        hf_launch<true>(h->TH, dim3(h->cgx * h->cgy), h->stream,
                           static_cast<const float*>(h->dP), hf_pack(h->X, h->Y), hf_pack(h->cgx, h->cgx * h->cgy),
                           hf_pack(c.ux, c.uy), hf_pack(c.uw, c.uh), hf_magic(h->cgx), hf_magic(c.uh), h->dPart, 0,
                           static_cast<float*>(h->dQ), h->dPart, nullptr, nullptr, static_cast<const float*>(h->dFilt), h->nf, c, h->kf,
                           nullptr);
        RS_HIP(hipGetLastError());
        hipLaunchKernelGGL((pc_scale_kernel<float>), dim3(64), dim3(NT), 0, h->stream,
                           static_cast<float*>(h->dQ), h->n, h->dPart, h->nPart);
    } else if (h->prec == RS_PREC_F32) {
        RS_TRY((pc_launch_step<float, PcCtlRing>(h, step_out(h, 0), nullptr, -1)));
        hipLaunchKernelGGL((pc_scale_kernel<float>), dim3(64), dim3(NT), 0, h->stream,
                           static_cast<float*>(h->dQ), h->n, h->dPart, h->nPart);
    } else {
        RS_TRY((pc_launch_step<double, PcCtlRing>(h, step_out(h, 0), nullptr, -1)));
        hipLaunchKernelGGL((pc_scale_kernel<double>), dim3(64), dim3(NT), 0, h->stream,
                           static_cast<double*>(h->dQ), h->n, h->dPart, h->nPart);
    }
    RS_HIP(hipGetLastError());
    // Q has P's layout in every form (the column form: both theta-fastest)
    RS_HIP(hipMemcpyAsync(h->dP, h->dQ, h->n * h->esz, hipMemcpyDeviceToDevice, h->stream));
    RS_HIP(hipStreamSynchronize(h->stream));
    return RS_OK;
}

int rs_pc_set_odometry_tables(rs_pc* h, double vtrans_scale, double vrot_scale,
                              const double* cos_a, const double* sin_a, int key_min,
                              int nkeys, const int32_t* key_rows, int zorig_min, int nz,
                              const double* zf_table) {
    rs::clear_error();
    RS_CHECK(h, RS_ERR_STATE, "null pose-cell handle");
    RS_CHECK(cos_a && sin_a && key_rows && zf_table, RS_ERR_ARG, "null table");
    RS_CHECK(nkeys > 0 && nz > 0, RS_ERR_ARG, "empty key or theta-filter table");
    RS_CHECK(vtrans_scale != 0.0 && vrot_scale != 0.0, RS_ERR_ARG, "zero odometry scale");
    for (int i = 0; i < nkeys; ++i)
        RS_CHECK(key_rows[i] >= 0 && key_rows[i] < h->nf, RS_ERR_ARG,
                 "key row %d outside the %d-filter table", key_rows[i], h->nf);
    OdoTables& o = h->odo;
    o.TH = h->TH;
    o.vtScale = vtrans_scale;
    o.vrScale = vrot_scale;
    o.own.assign(cos_a, cos_a + h->TH);
    o.own.insert(o.own.end(), sin_a, sin_a + h->TH);
    o.own.insert(o.own.end(), zf_table, zf_table + (size_t)nz * FL);
    o.ownRows.assign(key_rows, key_rows + nkeys);
    o.cosA = o.own.data();
    o.sinA = o.own.data() + h->TH;
    o.zfTab = o.own.data() + 2 * (size_t)h->TH;
    o.keyMin = key_min;
    o.nKeys = nkeys;
    o.keyRows = o.ownRows.data();
    o.zMin = zorig_min;
    o.nZ = nz;
    h->odoReady = true;
    return RS_OK;
}

int rs_pc_odom_control(int TH, double vtrans_scale, double vrot_scale, const double* cos_a,
                       const double* sin_a, int key_min, int nkeys, const int32_t* key_rows,
                       int zorig_min, int nz, const double* zf_table, int n, const double* odom,
                       int32_t* ox, int32_t* oy, int32_t* fidx, double* zf, int32_t* status) {
    rs::clear_error();
    RS_CHECK(TH > 0 && n >= 0 && nkeys > 0 && nz > 0, RS_ERR_ARG, "bad table or batch size");
    RS_CHECK(cos_a && sin_a && key_rows && zf_table && (n == 0 || (odom && ox && oy && fidx && zf &&
             status)), RS_ERR_ARG, "null argument");
    OdoTables o;
    o.TH = TH;
    o.vtScale = vtrans_scale;
    o.vrScale = vrot_scale;
    o.cosA = cos_a;
    o.sinA = sin_a;
    o.keyMin = key_min;
    o.nKeys = nkeys;
    o.keyRows = key_rows;
    o.zMin = zorig_min;
    o.nZ = nz;
    o.zfTab = zf_table;
    for (int s = 0; s < n; ++s)
        status[s] = pc_odom_control(&o, odom[2 * s], odom[2 * s + 1], ox + (size_t)TH * s,
                                    oy + (size_t)TH * s, fidx + (size_t)TH * s, zf + (size_t)FL * s);
    return RS_OK;
}

int rs_pc_update_odom(rs_pc* h, double vtrans, double vrot, int32_t out_xyz[3]) {
    rs::clear_error();
    RS_CHECK(h, RS_ERR_STATE, "null pose-cell handle");
    RS_CHECK(h->odoReady, RS_ERR_STATE, "rs_pc_set_odometry_tables has not been called");
    h->cOx.resize(h->TH);
    h->cOy.resize(h->TH);
    h->cRows.resize(h->TH);
    h->cZf.resize(FL);
    const int st = pc_odom_control(&h->odo, vtrans, vrot, h->cOx.data(), h->cOy.data(),
                                   h->cRows.data(), h->cZf.data());
    if (st == RS_ERR_LUT_KEY) {
        // the reference raises inside path_integration, after steps 1-4 ran
        RS_TRY(rs_pc_excite(h));
        RS_CHECK(false, RS_ERR_LUT_KEY, "path-integration LUT key outside the table "
                 "(posecell_network.py:249)");
    }
    RS_CHECK(st == RS_OK, st, "odometry (%g, %g) outside the control tables", vtrans, vrot);
    return pc_run_impl(h, 1, h->cOx.data(), h->cOy.data(), h->cRows.data(), h->cZf.data(), out_xyz);
}

int rs_pc_update_odom_read(rs_pc* h, double vtrans, double vrot, int32_t out_xyz[3], double* pinned) {
    rs::clear_error();
    RS_CHECK(h && pinned, RS_ERR_ARG, "null argument");
    RS_CHECK(reinterpret_cast<uintptr_t>(pinned) % 16 == 0, RS_ERR_ARG, "pinned buffer not 16-byte aligned");
    RS_HIP(hipSetDevice(h->device));
    RS_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&h->exportDev), pinned, 0));
    const int st = rs_pc_update_odom(h, vtrans, vrot, out_xyz);
    h->exportDev = nullptr;
    return st;
}

int rs_pc_run_odom(rs_pc* h, int n, const double* odom, int32_t* out_xyz, int* first_bad) {
    rs::clear_error();
    RS_CHECK(h, RS_ERR_STATE, "null pose-cell handle");
    RS_CHECK(h->odoReady, RS_ERR_STATE, "rs_pc_set_odometry_tables has not been called");
    RS_CHECK(n >= 0 && (odom || n == 0), RS_ERR_ARG, "bad odometry batch");
    if (first_bad) *first_bad = -1;
    const size_t th = h->TH;
    h->cOx.resize(th * (n > 0 ? n : 1));
    h->cOy.resize(th * (n > 0 ? n : 1));
    h->cRows.resize(th * (n > 0 ? n : 1));
    h->cZf.resize((size_t)FL * (n > 0 ? n : 1));
    // The batch's control is formed before its first launch (the step kernels take it as
    // kernel arguments), so a long batch forms it on a few threads, each a contiguous range
    // of steps: 10,000 steps at 128x128x72 spent about 6 ms on one (0.6 us per step of the
    // 15 us step, added to the batch's wall time).  The first failing step decides, as in
    // order on one thread.
    int fail = n, fail_st = RS_OK;
    auto range = [&](int s0, int s1, int* fs, int* fst) {
        for (int s = s0; s < s1; ++s) {
            const int st = pc_odom_control(&h->odo, odom[2 * s], odom[2 * s + 1], h->cOx.data() + th * s,
                                           h->cOy.data() + th * s, h->cRows.data() + th * s,
                                           h->cZf.data() + (size_t)FL * s);
            if (st != RS_OK) {
                *fs = s;
                *fst = st;
                return;
            }
        }
    };
    const int nthr = n >= 1024 ? std::min(8, n / 512) : 1;
    if (nthr > 1) {
        std::vector<int> fs(nthr, n), fst(nthr, RS_OK);
        std::vector<std::thread> pool;
        const int per = (n + nthr - 1) / nthr;
        for (int t = 1; t < nthr; ++t) {
            try {
                pool.emplace_back(range, std::min(n, t * per), std::min(n, (t + 1) * per), &fs[t], &fst[t]);
            } catch (...) {   // no thread to be had: this one takes the range
                range(std::min(n, t * per), std::min(n, (t + 1) * per), &fs[t], &fst[t]);
            }
        }
        range(0, std::min(n, per), &fs[0], &fst[0]);
        for (auto& th_ : pool) th_.join();
        for (int t = 0; t < nthr; ++t)
            if (fs[t] < fail) {
                fail = fs[t];
                fail_st = fst[t];
            }
    } else {
        range(0, n, &fail, &fail_st);
    }
    int todo = n;
    if (fail < n) {
        if (fail_st == RS_ERR_LUT_KEY) todo = fail;
        else RS_CHECK(false, fail_st, "odometry of step %d outside the control tables", fail);
    }
    RS_TRY(pc_run_impl(h, todo, h->cOx.data(), h->cOy.data(), h->cRows.data(), h->cZf.data(),
                       out_xyz));
    if (todo < n) {
        RS_TRY(rs_pc_excite(h));
        if (first_bad) *first_bad = todo;
        RS_CHECK(false, RS_ERR_LUT_KEY, "path-integration LUT key outside the table at step %d "
                 "(posecell_network.py:249)", todo);
    }
    return RS_OK;
}

int rs_pc_inject(rs_pc* h, double energy, int x, int y, int th) {
    rs::clear_error();
    RS_CHECK(h, RS_ERR_STATE, "null pose-cell handle");
    RS_CHECK(x >= 0 && x < h->X && y >= 0 && y < h->Y && th >= 0 && th < h->TH, RS_ERR_ARG,
             "inject location (%d, %d, %d) outside grid (%d, %d, %d)", x, y, th, h->X, h->Y, h->TH);
    RS_HIP(hipSetDevice(h->device));
    RS_TRY(pc_halo_settle(h));  // (halo: a state a call left unnormalised)
    // the column form keeps P theta-fastest (C order); the others layer-major
    const size_t idx = pc_thfast(h) ? ((size_t)x * h->Y + y) * h->TH + th : ((size_t)th * h->X + x) * h->Y + y;
    if (h->prec == RS_PREC_F32)
        hipLaunchKernelGGL((pc_inject_kernel<float>), dim3(1), dim3(64), 0, h->stream,
                           static_cast<float*>(h->dP), idx, energy);
    else
        hipLaunchKernelGGL((pc_inject_kernel<double>), dim3(1), dim3(64), 0, h->stream,
                           static_cast<double*>(h->dP), idx, energy);
    RS_HIP(hipGetLastError());
    // no host sync: the add is ordered on the handle's stream before the next step,
    // read or argmax (template -> pose-cell feedback costs one queued launch)
    return RS_OK;
}

int rs_pc_get_max(rs_pc* h, int32_t out_xyz[3]) {
    rs::clear_error();
    RS_CHECK(h && out_xyz, RS_ERR_ARG, "null argument");
    RS_HIP(hipSetDevice(h->device));
    RS_TRY(pc_halo_settle(h));  // (halo: a state a call left unnormalised)
    if (h->prec == RS_PREC_F32) return pc_argmax_impl<float>(h, out_xyz);
    return pc_argmax_impl<double>(h, out_xyz);
}

// The float64 C-order volume into pinned host memory (dst: its device pointer) and the
// host back once it has landed: a pending halo state settled in the same pass
// (pc_halo_settle_read), else the export kernel; either way the writing kernel's
// blocks' flags are polled (pc_poll_flags) where allowed, else the stream synchronised.
int pc_read_volume(rs_pc* h, double* dst) {
    bool done = false;
    RS_TRY(pc_halo_settle_read(h, dst, &done));
    if (done) return RS_OK;
    int nb = (int)std::min<size_t>(1024, (h->n / 2 + NT - 1) / NT + 1);
    const bool fl = pc_flags_ok(h, nb);
    if (fl) nb = pc_xflag_nb(nb);
    const unsigned seq = fl ? pc_next_seq(h) : 0u;
    unsigned* flag = fl ? h->hFlagDev : nullptr;
    if (h->prec == RS_PREC_F32)
        hipLaunchKernelGGL((pc_export2_kernel<float>), dim3(nb), dim3(NT), 0, h->stream,
                           static_cast<const float*>(h->dP), dst, h->X, h->Y, h->TH, (int)pc_thfast(h), flag, seq);
    else
        hipLaunchKernelGGL((pc_export2_kernel<double>), dim3(nb), dim3(NT), 0, h->stream,
                           static_cast<const double*>(h->dP), dst, h->X, h->Y, h->TH, (int)pc_thfast(h), flag, seq);
    RS_HIP(hipGetLastError());
    if (!(fl && pc_poll_flags(h, nb, seq))) RS_HIP(hipStreamSynchronize(h->stream));
    return RS_OK;
}

int rs_pc_read(rs_pc* h, double* host) {
    rs::clear_error();
    RS_CHECK(h && host, RS_ERR_ARG, "null argument");
    RS_HIP(hipSetDevice(h->device));
    // The export kernel writes the float64 C-order volume straight into pinned host
    // memory (one launch, no copy engine), then the host copies it into the caller's
    // array.
    if (!h->hRead) {
        RS_HIP(hipHostMalloc(&h->hRead, sizeof(double) * h->n, hipHostMallocMapped | hipHostMallocCoherent));
        RS_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&h->hReadDev), h->hRead, 0));
    }
    RS_TRY(pc_read_volume(h, h->hReadDev));
    std::memcpy(host, h->hRead, sizeof(double) * h->n);
    return RS_OK;
}

int rs_pc_read_pinned(rs_pc* h, double* pinned) {
    rs::clear_error();
    RS_CHECK(h && pinned, RS_ERR_ARG, "null argument");
    RS_CHECK(reinterpret_cast<uintptr_t>(pinned) % 16 == 0, RS_ERR_ARG, "pinned buffer not 16-byte aligned");
    RS_HIP(hipSetDevice(h->device));
    double* dst = nullptr;
    RS_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&dst), pinned, 0));
    return pc_read_volume(h, dst);
}

int rs_pc_write(rs_pc* h, const double* host) {
    rs::clear_error();
    RS_CHECK(h && host, RS_ERR_ARG, "null argument");
    RS_HIP(hipSetDevice(h->device));
    h->haloPend = false;  // (halo: the whole state is replaced)
    h->haloCur = 0;
    RS_HIP(hipMemcpyAsync(h->dTmp, host, sizeof(double) * h->n, hipMemcpyHostToDevice, h->stream));
    if (h->prec == RS_PREC_F32)
        hipLaunchKernelGGL((pc_import_kernel<float>), dim3(256), dim3(NT), 0, h->stream, h->dTmp,
                           static_cast<float*>(h->dP), h->X, h->Y, h->TH, (int)pc_thfast(h));
    else
        hipLaunchKernelGGL((pc_import_kernel<double>), dim3(256), dim3(NT), 0, h->stream, h->dTmp,
                           static_cast<double*>(h->dP), h->X, h->Y, h->TH, (int)pc_thfast(h));
    RS_HIP(hipGetLastError());
    RS_HIP(hipStreamSynchronize(h->stream));
    return RS_OK;
}

int rs_pc_total(rs_pc* h, double* total) {
    rs::clear_error();
    RS_CHECK(h && total, RS_ERR_ARG, "null argument");
    RS_HIP(hipSetDevice(h->device));
    RS_TRY(pc_halo_settle(h));  // (halo: a state a call left unnormalised)
    if (h->prec == RS_PREC_F32)
        hipLaunchKernelGGL((pc_total_kernel<float>), dim3(1), dim3(NT), 0, h->stream,
                           static_cast<const float*>(h->dP), h->n, h->dScalar);
    else
        hipLaunchKernelGGL((pc_total_kernel<double>), dim3(1), dim3(NT), 0, h->stream,
                           static_cast<const double*>(h->dP), h->n, h->dScalar);
    RS_HIP(hipGetLastError());
    RS_HIP(hipMemcpyAsync(total, h->dScalar, sizeof(double), hipMemcpyDeviceToHost, h->stream));
    RS_HIP(hipStreamSynchronize(h->stream));
    return RS_OK;
}

int rs_pc_last_ms(rs_pc* h, double* ms) {
    RS_CHECK(h && ms, RS_ERR_ARG, "null argument");
    *ms = h->lastMs;
    return RS_OK;
}

int rs_pc_set_profiling(rs_pc* h, int enable) {
    RS_CHECK(h, RS_ERR_STATE, "null pose-cell handle");
    // 1: events around every launch too (kernel_ms); 2: around the whole call only
    h->profiling = enable != 0;
    h->profKernels = enable == 1;
    return RS_OK;
}

int rs_pc_kernel_ms(rs_pc* h, double ms[2]) {
    RS_CHECK(h && ms, RS_ERR_ARG, "null argument");
    ms[0] = h->kernelMs[0];
    ms[1] = h->kernelMs[1];
    return RS_OK;
}

const char* rs_pc_step_form(const rs_pc* h) {
    if (!h) return nullptr;
    if (h->streamed) return "stream";
    if (h->halo) return "halo";
    if (h->cols) return "cols";
    return h->tiling ? "rows" : "tiles";
}

int rs_pc_debug(rs_pc* h, int op) {
    rs::clear_error();
    RS_CHECK(h, RS_ERR_STATE, "null pose-cell handle");
    RS_HIP(hipSetDevice(h->device));
    RS_TRY(pc_halo_settle(h));  // (halo: a state a call left unnormalised)
    if (op == RS_PC_DBG_POISON) {
        // every buffer a step writes before it reads: all bits set (NaN volumes, the
        // largest possible argmax key in every slot of every step)
        RS_HIP(hipMemsetAsync(h->dQ, 0xFF, h->n * h->esz, h->stream));
        RS_HIP(hipMemsetAsync(h->dPart, 0xFF, sizeof(double) * h->nPart * 2, h->stream));
        RS_HIP(hipMemsetAsync(h->dRes, 0xFF, sizeof(unsigned long long) * RES_SLOTS * h->resCap, h->stream));
        RS_HIP(hipMemsetAsync(h->dBmax, 0xFF, h->esz * h->nBmaxCap, h->stream));
        RS_HIP(hipMemsetAsync(h->dBidx, 0xFF, sizeof(unsigned) * h->nBmaxCap, h->stream));
        if (h->dArgV) RS_HIP(hipMemsetAsync(h->dArgV, 0xFF, h->esz * (size_t)h->resCap * h->nPathBlocks, h->stream));
        if (h->dArgI)
            RS_HIP(hipMemsetAsync(h->dArgI, 0xFF, sizeof(unsigned) * (size_t)h->resCap * h->nPathBlocks, h->stream));
        for (int s = 0; s < h->resCap; ++s) h->hRes[s] = ~0ull;
        RS_HIP(hipStreamSynchronize(h->stream));
        return RS_OK;
    }
    if (op == RS_PC_DBG_SKIP_EXPORT) {
        h->dbgSkipExport = true;
        return RS_OK;
    }
    if (op == RS_PC_DBG_HALO_SETTLE) {
        h->haloSettleAlways = true;
        return RS_OK;
    }

    RS_CHECK(false, RS_ERR_ARG, "unknown rs_pc_debug op %d", op);
}

int rs_pc_debug_value(rs_pc* h, int op, int64_t* value) {
    rs::clear_error();
    RS_CHECK(h && value, RS_ERR_ARG, "null argument");
    RS_CHECK(op == RS_PC_DBG_HALO_AMBIG, RS_ERR_ARG, "unknown rs_pc_debug_value op %d", op);
    *value = h->haloAmbig;
    return RS_OK;
}

}  // extern "C"
