// View-template matcher on MI355X (gfx950).
//
// Replaces ViewTemplate.match / ViewTemplates.match
// (/root/reference/ratslam/view_templates.py:16-28, 63-75).
//
// Score of template T against query Q (both H x W uint8):
//   min_{o=-(M-1)..M-1} sum_{r=M..H-M-1, c} (T[r+o][c] - Q[r][c]) mod 256
// (numpy uint8 subtraction wraps and abs() is the identity on uint8).
// Per 4-byte dword this is a carry-free SWAR add of the query's byte negation
// c = -Q (mod 256):  d = ((a & 0x7f7f7f7f) + cL) ^ (a & 0x80808080) ^ cH, then
// v_sad_u8(d, 0, acc) adds the four wrapped bytes: 3 VALU instructions
// (v_add_u32, v_bitop3_b32 XOR3, v_sad_u8) per template-dword x offset pair.
//
// Library layout in HBM (SoA, 16-byte chunks): chunk (tb, c, q, t) at byte
//   (((tb * WD + c) * HQ + q) * 64 + t) * 16
// holds rows 4q..4q+3 (one dword each) of dword column c of template slot
// tb*64 + t.  One global_load_dwordx4 by a wave = 1 KiB contiguous = the same
// 16 bytes of 64 templates.
//
// Result of a scan: per query, the first argmin as a packed key
// (score << 32) | global_index, min-reduced over lanes, waves and (RCCL
// allreduce(min, uint64)) ranks -- exactly numpy's argmin tie-break
// (view_templates.py:73).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rs_common.h"

namespace {

constexpr int FAST_M = 8;  // ViewTemplate.max_offset (view_templates.py:14)
constexpr unsigned long long NO_KEY = ~0ull;

__device__ inline unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(v, off);
        v = o < v ? o : v;
    }
    return v;
}

__device__ inline uint32_t wrapped_pair(uint32_t aL, uint32_t aH, uint2 f, uint32_t acc) {
    return __builtin_amdgcn_sad_u8(__builtin_amdgcn_bitop3_b32(aL + f.x, aH, f.y, 0x96), 0u, acc);
}

// Scatter n raw (H x W) templates into library slots (layout above).
__global__ void vt_store_kernel(const uint8_t* __restrict__ raw, const int32_t* __restrict__ src,
                                const int64_t* __restrict__ dst, int n, uint4* __restrict__ lib,
                                int H, int W, int WD, int HQ) {
    const int64_t total = (int64_t)n * WD * HQ;
    for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int t = (int)(idx / (WD * HQ));
        const int rem = (int)(idx - (int64_t)t * WD * HQ);
        const int c = rem / HQ, q = rem - c * HQ;
        const uint8_t* tpl = raw + (size_t)src[t] * H * W;
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int row = 4 * q + k;
            uint32_t d = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int col = 4 * c + b;
                const uint32_t byte = (row < H && col < W) ? tpl[(size_t)row * W + col] : 0u;
                d |= byte << (8 * b);
            }
            w[k] = d;
        }
        const int64_t slot = dst[t];
        const int64_t tb = slot >> 6, tl = slot & 63;
        lib[((tb * WD + c) * HQ + q) * 64 + tl] = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

// On-device subsampling (view_templates.py:64, input[self.mask].reshape(shape)):
// query f = frame f gathered through the mask's pixel offsets, row-major.
__global__ __launch_bounds__(256) void vt_gather_kernel(const uint8_t* __restrict__ frames,
                                                        size_t frame_bytes,
                                                        const int32_t* __restrict__ pix, int npix,
                                                        uint8_t* __restrict__ out) {
    const uint8_t* f = frames + (size_t)blockIdx.x * frame_bytes;
    uint8_t* o = out + (size_t)blockIdx.x * npix;
    for (int i = threadIdx.x; i < npix; i += blockDim.x) o[i] = f[pix[i]];
}

// Query forms: qf[(n*WD + c)*H + r] = (cL, cH) of c = -Q[r][4c..4c+3] mod 256,
// and qsum[n] = sum over rows [M, H-M) of the bytes of c (carry-count scan).
// One block per query.
__global__ __launch_bounds__(256) void vt_qform_kernel(const uint8_t* __restrict__ raw, int H, int W,
                                                       int WD, int M, uint2* __restrict__ qf,
                                                       uint32_t* __restrict__ qsum) {
    __shared__ uint32_t s_red[4];
    const int qn = blockIdx.x;
    uint32_t part = 0;
    for (int idx = threadIdx.x; idx < WD * H; idx += blockDim.x) {
        const int c = idx / H, r = idx - c * H;
        uint32_t neg = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int col = 4 * c + b;
            const uint32_t byte = col < W ? raw[((size_t)qn * H + r) * W + col] : 0u;
            neg |= ((256u - byte) & 0xFFu) << (8 * b);
        }
        qf[(size_t)qn * WD * H + idx] = make_uint2(neg & 0x7F7F7F7Fu, neg & 0x80808080u);
        if (r >= M && r < H - M) part = __builtin_amdgcn_sad_u8(neg, 0u, part);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off);
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = part;
    __syncthreads();
    if (threadIdx.x == 0) qsum[qn] = s_red[0] + s_red[1] + s_red[2] + s_red[3];
}

// Output of a scan: either min-reduce packed keys per query (best[]) or
// write every (query, slot) score into a matrix.
struct ScanOut {
    unsigned long long* best;  // [nq] packed keys (MATRIX == false)
    uint32_t* mat;             // [nq][ld]          (MATRIX == true)
    int64_t ld;
    // plane scan, MATRIX == false: the block that finishes last hands the keys to the
    // host words and resets them (vt_keys_export folded in); done counts the blocks
    unsigned long long* host = nullptr;
    unsigned* done = nullptr;
};

template <bool MATRIX>
__device__ inline void emit_score(const ScanOut& out, int64_t slot, int64_t count, int qi, int nq,
                                  uint32_t score, int rank, int nranks, bool lane0_after_reduce) {
    if constexpr (MATRIX) {
        if (slot < count && qi < nq) out.mat[(size_t)qi * out.ld + slot] = score;
    } else {
        const unsigned long long g = (unsigned long long)slot * nranks + rank;
        unsigned long long key = slot < count ? (((unsigned long long)score << 32) | g) : NO_KEY;
        key = wave_min_u64(key);
        if (lane0_after_reduce && qi < nq) atomicMin(out.best + qi, key);
    }
}

// --- carry-count forms.  v_sad_u8 issues at half rate on gfx950 (measured,
// tools/ubench_valu.hip), so the byte sum is taken apart exactly:
//   sum_b (a_b + c_b) mod 256 = bytesum(a) + bytesum(c) - 256 * #carries,
// with the carry out of byte b = majority(a_b7, c_b7, bit 7 of (a&0x7f + c&0x7f)_b):
// one v_bitop3 (table 0xE8; zero outside bit 7 since aH, cH are), counted by
// v_bcnt_u32_b32.  Per pair: v_add_u32 + v_bitop3_b32 + v_bcnt_u32_b32, all full
// rate.  bytesum(a) over each offset's row window is a sliding sum per column
// (query-independent), bytesum(c) is qsum[] from vt_qform_kernel.
__device__ inline uint32_t carry_pair(uint32_t aL, uint32_t aH, uint2 f, uint32_t cnt) {
    return __builtin_popcount(__builtin_amdgcn_bitop3_b32(aH, f.y, aL + f.x, 0xE8)) + cnt;
}

template <int H, int NQ, bool MATRIX>
__global__ __launch_bounds__(64) void vt_scan_carry_kernel(const uint4* __restrict__ lib, int ntb,
                                                           int64_t count, int WD,
                                                           const uint2* __restrict__ qf,
                                                           const uint32_t* __restrict__ qsum,
                                                           int nq, ScanOut out, int rank,
                                                           int nranks) {
    constexpr int M = FAST_M, HQ = (H + 3) / 4, NO = 2 * M - 1, R0 = M, R1 = H - M;
    // XCD-aware mapping (speed only): blocks b and b+8 are dealt to the same XCD, so
    // XCD x takes query groups qg = x (mod 8) against the whole library -- its L2
    // holds the library plus 1/8 of the query forms.
    const int j = blockIdx.x >> 3;
    const int tb = j % ntb;
    const int qg = (j / ntb) * 8 + (blockIdx.x & 7);
    if (qg * NQ >= nq) return;
    const int qbase = qg * NQ;
    const int lane = threadIdx.x;
    uint32_t cnt[NQ][NO];
    uint32_t A[NO];
#pragma unroll
    for (int o = 0; o < NO; ++o) {
        A[o] = 0u;
#pragma unroll
        for (int n = 0; n < NQ; ++n) cnt[n][o] = 0u;
    }
    for (int c = 0; c < WD; ++c) {
        const uint4* col = lib + ((size_t)(tb * WD + c) * HQ) * 64 + lane;
        uint32_t aL[4 * HQ], aH[4 * HQ], bs[4 * HQ];
#pragma unroll
        for (int q = 0; q < HQ; ++q) {
            const uint4 v = col[(size_t)q * 64];
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                aL[4 * q + k] = w[k] & 0x7F7F7F7Fu;
                aH[4 * q + k] = w[k] & 0x80808080u;
                bs[4 * q + k] = __builtin_amdgcn_sad_u8(w[k], 0u, 0u);
            }
        }
        uint32_t win = 0u;
#pragma unroll
        for (int s = R0 - (M - 1); s < R1 - (M - 1); ++s) win += bs[s];
        A[0] += win;
#pragma unroll
        for (int o = 1; o < NO; ++o) {
            win += bs[R1 - (M - 1) + o - 1] - bs[R0 - (M - 1) + o - 1];
            A[o] += win;
        }
#pragma unroll
        for (int r = R0; r < R1; ++r) {
#pragma unroll
            for (int n = 0; n < NQ; ++n) {
                const int qi = min(qbase + n, nq - 1);
                const uint2 f = qf[((size_t)qi * WD + c) * H + r];
#pragma unroll
                for (int o = 0; o < NO; ++o) {
                    const int s = r + o - (M - 1);
                    cnt[n][o] = carry_pair(aL[s], aH[s], f, cnt[n][o]);
                }
            }
        }
    }
    const int64_t slot = (int64_t)tb * 64 + lane;
#pragma unroll
    for (int n = 0; n < NQ; ++n) {
        const uint32_t qs = qsum[min(qbase + n, nq - 1)];
        uint32_t sc = 0xFFFFFFFFu;
#pragma unroll
        for (int o = 0; o < NO; ++o) sc = min(sc, A[o] + qs - 256u * cnt[n][o]);
        emit_score<MATRIX>(out, slot, count, qbase + n, nq, sc, rank, nranks, lane == 0);
    }
}

template <int H, int NQ>
__global__ __launch_bounds__(64) void vt_scan_carry_col_kernel(const uint4* __restrict__ lib,
                                                               int64_t count, int WD,
                                                               const uint2* __restrict__ qf,
                                                               const uint32_t* __restrict__ qsum,
                                                               int nq, ScanOut out, int rank,
                                                               int nranks) {
    constexpr int M = FAST_M, HQ = (H + 3) / 4, NO = 2 * M - 1, R0 = M, R1 = H - M;
    const int lane = threadIdx.x;
    const int t8 = lane >> 3, cl = lane & 7;
    const int64_t slot = (int64_t)blockIdx.x * 8 + t8;
    const int64_t tb = slot >> 6, tl = slot & 63;
    const int qbase = blockIdx.y * NQ;
    uint32_t val[NQ][NO];  // bytesum(a) - 256 * carries, mod 2^32, this lane's columns
#pragma unroll
    for (int n = 0; n < NQ; ++n)
#pragma unroll
        for (int o = 0; o < NO; ++o) val[n][o] = 0u;
    for (int c = cl; c < WD; c += 8) {
        const uint4* col = lib + ((size_t)(tb * WD + c) * HQ) * 64 + tl;
        uint32_t aL[4 * HQ], aH[4 * HQ], bs[4 * HQ];
#pragma unroll
        for (int q = 0; q < HQ; ++q) {
            const uint4 v = col[(size_t)q * 64];
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                aL[4 * q + k] = w[k] & 0x7F7F7F7Fu;
                aH[4 * q + k] = w[k] & 0x80808080u;
                bs[4 * q + k] = __builtin_amdgcn_sad_u8(w[k], 0u, 0u);
            }
        }
        uint32_t A[NO];
        uint32_t win = 0u;
#pragma unroll
        for (int s = R0 - (M - 1); s < R1 - (M - 1); ++s) win += bs[s];
        A[0] = win;
#pragma unroll
        for (int o = 1; o < NO; ++o) {
            win += bs[R1 - (M - 1) + o - 1] - bs[R0 - (M - 1) + o - 1];
            A[o] = win;
        }
#pragma unroll
        for (int n = 0; n < NQ; ++n) {
            uint32_t cnt[NO];
#pragma unroll
            for (int o = 0; o < NO; ++o) cnt[o] = 0u;
            const int qi = min(qbase + n, nq - 1);
#pragma unroll
            for (int r = R0; r < R1; ++r) {
                const uint2 f = qf[((size_t)qi * WD + c) * H + r];
#pragma unroll
                for (int o = 0; o < NO; ++o) cnt[o] = carry_pair(aL[r + o - (M - 1)], aH[r + o - (M - 1)], f, cnt[o]);
            }
#pragma unroll
            for (int o = 0; o < NO; ++o) val[n][o] += A[o] - 256u * cnt[o];
        }
    }
#pragma unroll
    for (int n = 0; n < NQ; ++n) {
        const uint32_t qs = qsum[min(qbase + n, nq - 1)];
        uint32_t sc = 0xFFFFFFFFu;
#pragma unroll
        for (int o = 0; o < NO; ++o) {
            uint32_t v = val[n][o];
            v += __shfl_xor(v, 1);
            v += __shfl_xor(v, 2);
            v += __shfl_xor(v, 4);
            sc = min(sc, v + qs);
        }
        const unsigned long long g = (unsigned long long)slot * nranks + rank;
        unsigned long long key =
            (slot < count && cl == 0) ? (((unsigned long long)sc << 32) | g) : NO_KEY;
        key = wave_min_u64(key);
        if (lane == 0 && qbase + n < nq) atomicMin(out.best + qbase + n, key);
    }
}

// --- generic form (any H, max_offset): one thread per (slot, query).
template <bool MATRIX>
__global__ __launch_bounds__(64) void vt_scan_generic_kernel(const uint4* __restrict__ lib, int ntb,
                                                             int64_t count, int H, int M, int WD,
                                                             const uint2* __restrict__ qf, int nq,
                                                             ScanOut out, int rank, int nranks) {
    const int HQ = (H + 3) / 4;
    const int tb = blockIdx.x % ntb;
    const int qi = blockIdx.x / ntb;
    const int lane = threadIdx.x;
    const uint32_t* base = reinterpret_cast<const uint32_t*>(lib);
    uint32_t best = 0xFFFFFFFFu;
    bool any = false;
    for (int o = -(M - 1); o <= M - 1; ++o) {
        uint32_t acc = 0;
        for (int r = M; r < H - M; ++r) {
            const int s = r + o;
            for (int c = 0; c < WD; ++c) {
                const size_t chunk = ((size_t)(tb * WD + c) * HQ + (s >> 2)) * 64 + lane;
                const uint32_t a = base[chunk * 4 + (s & 3)];
                acc = wrapped_pair(a & 0x7F7F7F7Fu, a & 0x80808080u,
                                   qf[((size_t)qi * WD + c) * H + r], acc);
            }
        }
        best = min(best, acc);
        any = true;
    }
    if (!any) best = 0;
    emit_score<MATRIX>(out, (int64_t)tb * 64 + lane, count, qi, nq, best, rank, nranks, lane == 0);
}

// ===========================================================================
// Bit-plane scan (default for W = 32, H in {32, 64}, max_offset 8).
//
// (T - Q) mod 256 = T - Q + 256 [T < Q], so a score is
//   score(o) = TS(o) - QS + 256 * B(o),
// TS(o) = the template's byte sum over rows [M+o, H-M+o) (stored with the
// template), QS = the query's byte sum over rows [M, H-M), and B(o) = the number
// of byte pairs with T < Q.  B is counted bit-sliced: a unit of 4 rows x 8
// columns (32 bytes) is stored as 8 bit planes (plane k, bit i = bit k of byte
// i), and [T < Q] for all 32 pairs of a unit is the borrow out of T - Q,
//   b = maj(~T_k, Q_k, b)  for k = 0..7   (one v_bitop3_b32 each, table 0x8E),
// followed by one v_bcnt_u32_b32 into the offset's counter: 9 VALU per
// 32 byte pairs, against 3 per 4 pairs for the byte-SWAR forms above.
//
// Template planes: uint4 chunk ((((tb*CG + cg)*NU + j)*2 + g)*64 + t) holds
// planes 4g..4g+3 of unit j (rows 4j..4j+3, columns 8cg..8cg+7) of slot
// tb*64 + t.  TS: tsum[(tb*16 + o+M-1)*64 + t].
// Query planes: for every start row s in [M-3, H-M-1] and column group cg, the
// unit of rows s..s+3 with rows outside [M, H-M) zeroed (a zero byte never
// borrows), qp[((q*CG + cg)*NS + s-(M-3))*8 + k]; qsum[q] = QS (raw bytes).
//
// A block is CG waves (one per column group) x 64 templates.  Wave cg keeps
// its NU units x 8 planes in VGPRs and streams query planes through SGPRs
// (wave-uniform scalar loads).  Template unit j meets query unit s at offset
// o = 4j - s.  The CG partial counts per (query, offset, template) meet in LDS.
// ===========================================================================
constexpr int PL_CG = 4;       // column groups of 8 bytes: W = 32

// Per-wave stamp hook, empty in the library: tools/vt_probe.hip defines it (start
// and end of every wave: realtime, shader clock, hw ids) before it includes this file.
#ifndef VT_STAMP
#define VT_STAMP(slot) \
    do {               \
    } while (0)
#endif
constexpr int PL_NB = 4;  // queries per LDS batch (staged planes; one reducing wave each)

// One block per stored template: planes + TS of raw template src[t] into slot dst[t].
__global__ __launch_bounds__(256) void vt_plane_store_kernel(const uint8_t* __restrict__ raw,
                                                             const int32_t* __restrict__ src,
                                                             const int64_t* __restrict__ dst,
                                                             int H, int M,
                                                             uint32_t* __restrict__ planes,
                                                             uint32_t* __restrict__ tsum) {
    constexpr int W = 8 * PL_CG;
    __shared__ uint32_t s_row[256];
    const uint8_t* T = raw + (size_t)src[blockIdx.x] * H * W;
    const int64_t slot = dst[blockIdx.x];
    const int64_t tb = slot >> 6, tl = slot & 63;
    const int NU = H / 4, wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 31;
    for (int u0 = 2 * wave; u0 < PL_CG * NU; u0 += 8) {
        const int u = u0 + (lane >> 5);
        const int cg = u / NU, j = u - cg * NU;
        const uint32_t byte = u < PL_CG * NU ? T[(size_t)(4 * j + (i >> 3)) * W + 8 * cg + (i & 7)] : 0u;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const unsigned long long m = __ballot((byte >> k) & 1u);
            if (i == k && u < PL_CG * NU)
                planes[((((tb * PL_CG + cg) * NU + j) * 2 + (k >> 2)) * 64 + tl) * 4 + (k & 3)] =
                    (uint32_t)(lane < 32 ? m : m >> 32);
        }
    }
    for (int r = threadIdx.x; r < H; r += blockDim.x) {
        uint32_t acc = 0;
        const uint32_t* row = reinterpret_cast<const uint32_t*>(T + (size_t)r * W);
#pragma unroll
        for (int d = 0; d < W / 4; ++d) acc = __builtin_amdgcn_sad_u8(row[d], 0u, acc);
        s_row[r] = acc;
    }
    __syncthreads();
    if (threadIdx.x < 16) {
        const int o = (int)threadIdx.x - (M - 1);
        uint32_t ts = 0;
        if (threadIdx.x < 2 * M - 1)
            for (int r = M + o; r < H - M + o; ++r) ts += s_row[r];
        tsum[(tb * 16 + threadIdx.x) * 64 + tl] = ts;
    }
}

// 8x8 bit-matrix transpose of 8 bytes held as (lo = bytes 0-3, hi = bytes 4-7):
// bit c of byte r  ->  bit r of byte c (three delta swaps, Hacker's Delight 7-3).
__device__ inline void transpose8x8(uint32_t& lo, uint32_t& hi) {
    uint32_t t;
    t = (lo ^ (lo >> 7)) & 0x00AA00AAu;   lo ^= t ^ (t << 7);
    t = (hi ^ (hi >> 7)) & 0x00AA00AAu;   hi ^= t ^ (t << 7);
    t = (lo ^ (lo >> 14)) & 0x0000CCCCu;  lo ^= t ^ (t << 14);
    t = (hi ^ (hi >> 14)) & 0x0000CCCCu;  hi ^= t ^ (t << 14);
    t = (lo ^ (hi << 4)) & 0xF0F0F0F0u;   lo ^= t;  hi ^= t >> 4;
}

// 4x4 byte transpose: out[k] byte q = byte k of in[q].
__device__ inline void transpose4x4_bytes(uint32_t a, uint32_t b, uint32_t c, uint32_t d,
                                          uint32_t (&o)[4]) {
    // pairs: (a,b) -> byte k of a, byte k of b interleaved; likewise (c,d)
    const uint32_t ab_lo = __builtin_amdgcn_perm(b, a, 0x05010400u);  // a0 b0 a1 b1
    const uint32_t ab_hi = __builtin_amdgcn_perm(b, a, 0x07030602u);  // a2 b2 a3 b3
    const uint32_t cd_lo = __builtin_amdgcn_perm(d, c, 0x05010400u);  // c0 d0 c1 d1
    const uint32_t cd_hi = __builtin_amdgcn_perm(d, c, 0x07030602u);  // c2 d2 c3 d3
    o[0] = __builtin_amdgcn_perm(cd_lo, ab_lo, 0x05040100u);          // a0 b0 c0 d0
    o[1] = __builtin_amdgcn_perm(cd_lo, ab_lo, 0x07060302u);          // a1 b1 c1 d1
    o[2] = __builtin_amdgcn_perm(cd_hi, ab_hi, 0x05040100u);
    o[3] = __builtin_amdgcn_perm(cd_hi, ab_hi, 0x07060302u);
}

// One block per query: query planes for every start row, and QS.  Phase 1: each
// thread bit-transposes one 8-byte row segment (row r, column group cg) so byte
// k holds bit k of its 8 pixels (rows outside [M, H-M) become zero), and adds
// the segment to QS.  Phase 2: each thread assembles one unit (4 rows from start
// row S0 + si, column group cg): plane k = byte k of its 4 segments, two 16-byte
// stores.  Bit b of plane k = bit k of pixel (row + b/8, col 8cg + b%8).
__global__ __launch_bounds__(256) void vt_qplane_kernel(const uint8_t* __restrict__ raw, int H,
                                                        int M, uint32_t* __restrict__ qp,
                                                        uint32_t* __restrict__ qsum,
                                                        uint8_t* __restrict__ raw_copy) {
    constexpr int W = 8 * PL_CG;
    __shared__ uint32_t s_red[4];
    __shared__ uint2 s_t[64 * W / 8];   // transposed segments (H <= 64)
    const int NS = H - 2 * M + 3, S0 = M - 3;
    const uint8_t* Q = raw + (size_t)blockIdx.x * H * W;
    uint32_t* out = qp + (size_t)blockIdx.x * PL_CG * NS * 8;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t part = 0;
    for (int d = threadIdx.x; d < H * W / 8; d += blockDim.x) {
        uint2 v = reinterpret_cast<const uint2*>(Q)[d];
        // raw read in place from pinned host memory: its bytes also into the device copy
        if (raw_copy) reinterpret_cast<uint2*>(raw_copy + (size_t)blockIdx.x * H * W)[d] = v;
        const int r = d / (W / 8);
        const bool live = r >= M && r < H - M;
        if (live) part = __builtin_amdgcn_sad_u8(v.y, 0u, __builtin_amdgcn_sad_u8(v.x, 0u, part));
        transpose8x8(v.x, v.y);
        s_t[d] = live ? v : make_uint2(0u, 0u);
    }
    __syncthreads();
    const int NU = PL_CG * NS;
    for (int u = threadIdx.x; u < NU; u += blockDim.x) {
        const int cg = u / NS, r0 = S0 + (u - cg * NS);
        const uint2 q0 = s_t[(r0 + 0) * PL_CG + cg], q1 = s_t[(r0 + 1) * PL_CG + cg];
        const uint2 q2 = s_t[(r0 + 2) * PL_CG + cg], q3 = s_t[(r0 + 3) * PL_CG + cg];
        uint32_t lo[4], hi[4];
        transpose4x4_bytes(q0.x, q1.x, q2.x, q3.x, lo);
        transpose4x4_bytes(q0.y, q1.y, q2.y, q3.y, hi);
        uint4* o = reinterpret_cast<uint4*>(out + (size_t)u * 8);
        o[0] = make_uint4(lo[0], lo[1], lo[2], lo[3]);
        o[1] = make_uint4(hi[0], hi[1], hi[2], hi[3]);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off);
    if (lane == 0) s_red[wave] = part;
    __syncthreads();
    if (threadIdx.x == 0) qsum[blockIdx.x] = s_red[0] + s_red[1] + s_red[2] + s_red[3];
}

// Query start rows [M-3, H-M-1] are split into PL_SPLIT ranges, one wave each
// per column group, so a wave keeps only the template units its rows meet
// (10 of 16 at H = 64): fewer VGPRs, four waves per SIMD.
constexpr int PL_SPLIT = 2;

template <int H, int HALF>
struct PlaneRange {
    static constexpr int M = FAST_M, NU = H / 4, S0 = M - 3, S1 = H - M - 1, NS = S1 - S0 + 1;
    static constexpr int NSH = (NS + PL_SPLIT - 1) / PL_SPLIT;
    static constexpr int SA = S0 + HALF * NSH;
    static constexpr int SB = (SA + NSH - 1) < S1 ? SA + NSH - 1 : S1;
    static constexpr int ja(int s) { return (s - (M - 1)) > 0 ? (s - (M - 1) + 3) / 4 : 0; }
    static constexpr int jb(int s) { return (s + (M - 1)) / 4 < NU - 1 ? (s + (M - 1)) / 4 : NU - 1; }
    static constexpr int JLO = ja(SA), JHI = jb(SB), NUH = JHI - JLO + 1;
};

// One query start row S against the template units it meets (o = 4J - S within
// +-(M-1): 3 or 4 units).  The borrow chains of those units are interleaved
// plane by plane, so consecutive bitop3s are independent (a single chain would
// stall on every instruction).  All indices are compile-time.
template <int H, int HALF, int S>
__device__ __forceinline__ void plane_row(const uint32_t (&P)[PlaneRange<H, HALF>::NUH][8],
                                          const uint32_t* q, uint32_t (&acc)[2 * FAST_M - 1]) {
    using R = PlaneRange<H, HALF>;
    constexpr int M = FAST_M, JA = R::ja(S), JB = R::jb(S), NJ = JB - JA + 1;
    static_assert(NJ >= 1 && NJ <= 4 && JA >= R::JLO && JB <= R::JHI, "units per query row");
    uint32_t b[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) b[j] = __builtin_amdgcn_bitop3_b32(P[JA - R::JLO + j][0], q[0], 0u, 0x8E);
#pragma unroll
    for (int k = 1; k < 8; ++k)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
            b[j] = __builtin_amdgcn_bitop3_b32(P[JA - R::JLO + j][k], q[k], b[j], 0x8E);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        // v_bcnt's own accumulator (asm keeps the compiler from re-associating
        // the counts into half-rate v_add3_u32)
        uint32_t& a = acc[4 * (JA + j) - S + M - 1];
        asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(a) : "v"(b[j]), "v"(a));
    }
}

// Query planes are staged per batch in LDS and read as wave-uniform
// ds_read_b128 broadcasts into VGPRs: on gfx950 a VALU instruction with an SGPR
// operand issues at about half the all-VGPR rate (tools/ubench_chain.hip:
// 0.23 vs 0.36-0.41 wave-instructions per SIMD-cycle), so the chains take both
// operands from VGPRs.
template <int H, int HALF, int S>
__device__ __forceinline__ void plane_rows(const uint32_t (&P)[PlaneRange<H, HALF>::NUH][8],
                                           const uint32_t* sq, uint32_t (&acc)[2 * FAST_M - 1]) {
    using R = PlaneRange<H, HALF>;
    const uint4 lo = *reinterpret_cast<const uint4*>(sq + (S - R::S0) * 8);
    const uint4 hi = *reinterpret_cast<const uint4*>(sq + (S - R::S0) * 8 + 4);
    const uint32_t q[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    plane_row<H, HALF, S>(P, q, acc);
    if constexpr (S < R::SB) plane_rows<H, HALF, S + 1>(P, sq, acc);
}


template <int H>
struct PlaneLds {
    static constexpr int M = FAST_M, NS = H - 2 * M + 3, NO = 2 * M - 1, NK = (NO + 1) / 2;
    static constexpr int QW = PL_CG * NS * 8;                 // query-plane dwords per query
    static constexpr int NW = PL_CG * PL_SPLIT;                // waves per block
    static constexpr int QP = (PL_NB * QW / 4 + 63) / 64 * 64;  // padded to whole 1 KiB wave-instructions
};

// The plane scan's LDS.  Double-buffered: batch i computes from its staged query
// planes and adds its partial counts into part[i&1] while batch i+1 is staged into
// the other plane buffer; one barrier per batch.  Each buffer is its own
// namespace-scope __shared__ variable and every access names one of them at
// compile time (pl_q<H, CUR>, pl_part<CUR>): hipcc waits for an LDS-DMA in flight
// before any LDS access it cannot prove disjoint from the DMA's variable, so
// only distinct, statically named variables let the next batch's DMA stay in
// flight through this batch's compute.
constexpr int PL_NK = PlaneLds<64>::NK;   // the same for every H (it depends on max_offset only)
static_assert(PlaneLds<32>::NK == PL_NK, "partial-count slots independent of H");
// the staged query planes, sized per template height (a kernel allocates only the
// instances it names: the H = 32 scan, the ROS node's geometry, does not carry the
// H = 64 buffers)
template <int H>
__shared__ uint4 vt_pl_qa[PlaneLds<H>::QP];   // even batches
template <int H>
__shared__ uint4 vt_pl_qb[PlaneLds<H>::QP];   // odd batches
__shared__ uint32_t vt_pl_part0[PL_NB][PL_NK][64];  // u16 pairs of partial counts, summed by ds_add
__shared__ uint32_t vt_pl_part1[PL_NB][PL_NK][64];
__shared__ int vt_pl_bidx[3];             // batches taken ahead (ring)
__shared__ uint32_t vt_pl_ts[16][64];     // TS(o) of the block's 64 templates
template <int H, int CUR>
__device__ __forceinline__ uint4* pl_q() {
    if constexpr (CUR == 0) return vt_pl_qa<H>;
    else return vt_pl_qb<H>;
}
template <int CUR>
__device__ __forceinline__ uint32_t (&pl_part())[PL_NB][PL_NK][64] {
    if constexpr (CUR == 0) return vt_pl_part0;
    else return vt_pl_part1;
}

template <int H, int HALF>
__device__ __forceinline__ void plane_load_units(const uint4* __restrict__ planes, int tb, int cg,
                                                 int lane, uint32_t (&P)[PlaneRange<H, HALF>::NUH][8]) {
    using R = PlaneRange<H, HALF>;
    const uint4* src = planes + ((size_t)(tb * PL_CG + cg) * (H / 4) + R::JLO) * 128 + lane;
#pragma unroll
    for (int j = 0; j < R::NUH; ++j) {
        const uint4 a = src[(2 * j) * 64], b = src[(2 * j + 1) * 64];
        P[j][0] = a.x; P[j][1] = a.y; P[j][2] = a.z; P[j][3] = a.w;
        P[j][4] = b.x; P[j][5] = b.y; P[j][6] = b.z; P[j][7] = b.w;
    }
}

// The work of one wave: column group cg, query start rows of range HALF.  One
// barrier per batch: before it, every wave stages its share of the next batch's
// planes and adds this batch's partial counts into LDS (ds_add; the per-half
// sums stay < 2^16, so the packed pairs never carry); after it, wave w < nb
// finishes query w of the batch and clears its partial slots for batch i+2.
// Batches are taken one ahead by thread 0; a block stops taking after its first
// failed take, so every block ends on exactly one failed take (counter rewind).
// One batch of plane_wave: compute from qcur (staged by the previous batch or the
// prologue) while this wave's share of the next batch goes global -> LDS into qnxt.
// CUR is the parity of the iteration (it & 1), so the plane buffers and the
// partial-count slots are compile-time: each LDS read names one __shared__
// variable and each DMA the other, and hipcc leaves the DMA in flight through the
// compute (a runtime choice of buffer made it wait vmcnt(0) before the first read).
// Returns false once the block has no batch left.
template <int H, int HALF, bool MATRIX, int CUR>
__device__ __forceinline__ bool plane_batch(const uint32_t (&P)[PlaneRange<H, HALF>::NUH][8], int it,
                                            int& bi, int nbatch, int64_t slot, int64_t count,
                                            const uint4* __restrict__ qp4, const uint32_t* __restrict__ qsum,
                                            int nq, unsigned* __restrict__ ctr, int G, int g, ScanOut out,
                                            int rank, int nranks, int wave, int cg, int lane,
                                            unsigned& failed) {
    using R = PlaneRange<H, HALF>;
    using LD = PlaneLds<H>;
    constexpr int NO = LD::NO, NK = LD::NK, NS = LD::NS, NT = 64 * LD::NW;
    if (bi >= nbatch) return false;  // block-uniform
    const uint4* qcur = pl_q<H, CUR>();
    uint4* qnxt = pl_q<H, CUR ^ 1>();
    uint32_t(&part)[PL_NB][PL_NK][64] = pl_part<CUR>();
    const int tid = wave * 64 + lane;
    // batch ring: iteration it reads the next batch from slot (it+1) % 3 and thread
    // 0 writes the one after it into slot (it+2) % 3, last read two barriers ago
    const int r1 = (it + 1) % 3, r2 = (it + 2) % 3;
    const int bn = vt_pl_bidx[r1];
    const int qb = (bi * G + g) * PL_NB, nb = min(PL_NB, nq - qb);
    // The take comes first (its result is waited for); with no next batch there is
    // no further take: this block's failed take was bn.
    if (tid == 0) {  // the batch after next
        const unsigned t = bn < nbatch ? atomicAdd(ctr, 1u) : (unsigned)nbatch;
        vt_pl_bidx[r2] = (int)t;
        if (bn < nbatch && (int)t >= nbatch) failed = t;
    }
    // the next batch's planes go global -> LDS directly (global_load_lds, 1 KiB per
    // wave-instruction, lane-linear), in flight through this batch's compute
    if (bn < nbatch) {
        const int qn = (bn * G + g) * PL_NB, nbn = min(PL_NB, nq - qn);
        const int lim = nbn * LD::QW / 4;
        const uint4* src = qp4 + (size_t)qn * (LD::QW / 4);
#pragma unroll
        for (int k = 0; k < (LD::QP + NT - 1) / NT; ++k) {
            const int i0 = wave * 64 + k * NT;  // wave-uniform
            if (i0 < lim)
                __builtin_amdgcn_global_load_lds(
                    (__attribute__((address_space(1))) const void*)(src + min(i0 + lane, lim - 1)),
                    (__attribute__((address_space(3))) void*)(qnxt + i0), 16, 0, 0);
        }
    }
#pragma unroll 1
    for (int b = 0; b < nb; ++b) {
        uint32_t acc[NO];
#pragma unroll
        for (int o = 0; o < NO; ++o) acc[o] = 0u;
        plane_rows<H, HALF, R::SA>(P, reinterpret_cast<const uint32_t*>(qcur) + (b * PL_CG + cg) * NS * 8, acc);
#pragma unroll
        for (int k = 0; k < NK; ++k)
            atomicAdd(&part[b][k][lane], acc[2 * k] | (2 * k + 1 < NO ? acc[2 * k + 1] << 16 : 0u));
    }
    // every wave's DMA into qnxt has landed before any wave passes the barrier and
    // reads it (explicit: nothing else guarantees this wait stays in front of it)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    __syncthreads();
    if (wave < nb) {  // wave w finishes query qb + w of the batch
        const int qi = qb + wave;
        uint32_t best = 0xFFFFFFFFu;
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            const uint32_t t = part[wave][k][lane];
            part[wave][k][lane] = 0u;
            best = min(best, vt_pl_ts[2 * k][lane] + 256u * (t & 0xFFFFu));
            if (2 * k + 1 < NO) best = min(best, vt_pl_ts[2 * k + 1][lane] + 256u * (t >> 16));
        }
        emit_score<MATRIX>(out, slot, count, qi, nq, best - qsum[qi], rank, nranks, lane == 0);
    }
    bi = bn;
    return true;
}

template <int H, int HALF, bool MATRIX>
__device__ __forceinline__ void plane_wave(const uint4* __restrict__ planes,
                                           int tb, int64_t count, const uint4* __restrict__ qp4,
                                           const uint32_t* __restrict__ qsum, int nq,
                                           unsigned* __restrict__ ctr, int G, int g, ScanOut out,
                                           int rank, int nranks, int wave, int cg, int lane,
                                           unsigned& failed) {
    using R = PlaneRange<H, HALF>;
    uint32_t P[R::NUH][8];
    plane_load_units<H, HALF>(planes, tb, cg, lane, P);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the template planes have landed before the loop
    const int nbatch = ((nq + PL_NB - 1) / PL_NB - g + G - 1) / G;
    const int64_t slot = (int64_t)tb * 64 + lane;
    int bi = vt_pl_bidx[0];
    // unrolled by two: even iterations compute from qa and stage into qb, odd ones
    // the other way round (the prologue staged the first batch into qa)
    // The first batch is peeled off the loop: hipcc's wait analysis is exact for the
    // LDS accesses after a DMA issued in the same loop iteration but not across the
    // loop header's merge, so the loop body starts with an odd batch, whose compute
    // follows its own DMA issue, not the header.
    if (!plane_batch<H, HALF, MATRIX, 0>(P, 0, bi, nbatch, slot, count, qp4, qsum, nq, ctr, G, g, out, rank,
                                         nranks, wave, cg, lane, failed))
        return;
    for (int it = 1;; it += 2) {
        if (!plane_batch<H, HALF, MATRIX, 1>(P, it, bi, nbatch, slot, count, qp4, qsum, nq, ctr, G, g, out,
                                             rank, nranks, wave, cg, lane, failed))
            break;
        if (!plane_batch<H, HALF, MATRIX, 0>(P, it + 1, bi, nbatch, slot, count, qp4, qsum, nq, ctr, G, g,
                                             out, rank, nranks, wave, cg, lane, failed))
            break;
    }
}

// nqc blocks serve each template block; they take query batches of PL_NB from
// the template block's counter, so blocks that the SIMDs' oldest-first issue
// favours take more batches and no SIMD is left running a lone straggler.
template <int H, bool MATRIX>
__global__ __launch_bounds__(64 * PL_CG * PL_SPLIT) __attribute__((amdgpu_waves_per_eu(4, 4)))
void vt_scan_plane_kernel(const uint4* __restrict__ planes, const uint32_t* __restrict__ tsum,
                          int ntb, int64_t count, const uint32_t* __restrict__ qp,
                          const uint32_t* __restrict__ qsum, int nq, int nqc,
                          unsigned* __restrict__ next_batch, ScanOut out, int rank, int nranks) {
    static_assert(PL_SPLIT == 2, "two row ranges");
    // The nqc blocks of a template block are adjacent block ids, so they are dispatched
    // together and split its query batches dynamically even when the grid runs in
    // several rounds.  XCD-aware: blocks b and b+8 share an XCD (and its L2); with
    // nqc >= 8 (a multiple of 8) the query batches are split into 8 groups by XCD, so
    // each L2 holds one group's planes
    const int tb = (int)(blockIdx.x / (unsigned)nqc);
    const int G = nqc >= 8 ? 8 : 1, g = nqc >= 8 ? (int)(blockIdx.x & 7) : 0;
    unsigned* ctr = next_batch + (size_t)tb * 8 + g;
    VT_STAMP(0);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, cg = wave % PL_CG, half = wave / PL_CG;
    const int nbatch = ((nq + PL_NB - 1) / PL_NB - g + G - 1) / G;
    for (int i = threadIdx.x; i < 16 * 64; i += blockDim.x) vt_pl_ts[i >> 6][i & 63] = tsum[(size_t)tb * 1024 + i];
    unsigned failed = 0u;  // thread 0: the value of this block's one failed take
    for (int i = threadIdx.x; i < PL_NB * PL_NK * 64; i += blockDim.x) {
        (&vt_pl_part0[0][0][0])[i] = 0u;
        (&vt_pl_part1[0][0][0])[i] = 0u;
    }
    if (threadIdx.x == 0) {  // the first batch and the one after it
        const unsigned a = atomicAdd(ctr, 1u);
        unsigned b = (unsigned)nbatch;
        if ((int)a < nbatch) {
            b = atomicAdd(ctr, 1u);
            if ((int)b >= nbatch) failed = b;
        } else {
            failed = a;
        }
        vt_pl_bidx[0] = (int)a;
        vt_pl_bidx[1] = (int)b;
    }
    __syncthreads();
    if (vt_pl_bidx[0] < nbatch) {  // stage the first batch
        constexpr int QW4 = PlaneLds<H>::QW / 4;
        const int qb = (vt_pl_bidx[0] * G + g) * PL_NB, nb = min(PL_NB, nq - qb);
        const uint4* qp4 = reinterpret_cast<const uint4*>(qp);
        for (int i = threadIdx.x; i < nb * QW4; i += blockDim.x) vt_pl_qa<H>[i] = qp4[(size_t)qb * QW4 + i];
    }
    __syncthreads();
    const uint4* qp4 = reinterpret_cast<const uint4*>(qp);
    if (half == 0)
        plane_wave<H, 0, MATRIX>(planes, tb, count, qp4, qsum, nq, ctr, G, g, out, rank, nranks,
                                 wave, cg, lane, failed);
    else
        plane_wave<H, 1, MATRIX>(planes, tb, count, qp4, qsum, nq, ctr, G, g, out, rank, nranks,
                                 wave, cg, lane, failed);
    // Each of the nqc / G blocks sharing a counter ends on exactly one failed take, so
    // the block whose failed take returned (group batches) + nqc / G - 1 is the
    // counter's last user in this launch: it rewinds the counter for the next launch
    // (no memset).
    if (threadIdx.x == 0 && failed == (unsigned)(nbatch + nqc / G - 1)) *ctr = 0u;
    if constexpr (!MATRIX) {
        if (out.host) {   // (kernel argument: uniform)
            // The key export folded into the scan (small calls, vt_scan_local_impl): the
            // keys are agent-scope atomics (performed at memory, never held in an L2), each
            // wave waits for its own (vmcnt(0)) before the block's counter add, the last
            // adder learns it from the add's return value and reads the keys with sc1
            // loads, then stores them into the pinned host words and resets them.
            // The model's agent-scope release before each block's counter add and acquire
            // in the last block frame the hand-off (a release fence after the block barrier
            // is cumulative over the waves' atomics; the acquire is one cache invalidate in
            // one block of the launch).
            __shared__ int s_last;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (threadIdx.x == 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                s_last = __hip_atomic_fetch_add(out.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                         gridDim.x - 1;
                if (s_last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            }
            __syncthreads();
            if (s_last) {
                for (int i = threadIdx.x; i < nq; i += blockDim.x) {
                    const unsigned long long k =
                        __hip_atomic_load(out.best + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(out.best + i, ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(out.host + i, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                if (threadIdx.x == 0) __hip_atomic_store(out.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    VT_STAMP(1);
}

// ===========================================================================
// Float path of ViewTemplate.match (view_templates.py:16-28 with float arrays):
// no wrap, a true sum of |T - Q| per row offset in the arrays' own precision,
// summed in numpy's order -- np.sum of the contiguous (H-2M) x W difference is
// numpy's pairwise summation over the flattened n elements (blocks of <= 128
// with 8 strided accumulators, halves split at a multiple of 8), so the host
// lowers that recursion for this n into a postfix program of leaf sums and adds
// (int2 (start, len) = push the leaf's sum; (-1, 0) = pop two, push their sum)
// that every thread evaluates: the same additions in the same order, bit-exact.
// Then the first strict minimum over the offsets from +inf, as the reference's
// `if diff < mindiff` loop (an all-NaN pair stays +inf).
// ===========================================================================
template <typename T>
__device__ inline T sad_at(const T* __restrict__ a, const T* __restrict__ b, int W, int M, int o,
                           int i) {
    const int r = i / W, c = i - r * W;
    const T d = a[(size_t)(M + o + r) * W + c] - b[(size_t)(M + r) * W + c];
    if constexpr (sizeof(T) == 4) return fabsf(d);   // numpy's absolute is fabs
    else return fabs(d);
}

template <typename T>
__device__ T sad_leaf(const T* a, const T* b, int W, int M, int o, int s, int n) {
    if (n < 8) {
        T res = T(0);
        for (int i = 0; i < n; ++i) res += sad_at(a, b, W, M, o, s + i);
        return res;
    }
    T r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = sad_at(a, b, W, M, o, s + j);
    int i = 8;
    for (; i < n - (n % 8); i += 8)
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] += sad_at(a, b, W, M, o, s + i + j);
    T res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += sad_at(a, b, W, M, o, s + i);
    return res;
}

constexpr int SAD_STACK = 40;   // pairwise depth: log2(n / 128) + 2 <= 40 for any n < 2^31

// 4 (template, query) pairs per 64-thread block, 16 threads per pair (one per offset)
template <typename T>
__global__ __launch_bounds__(64) void vt_sad_float_kernel(const T* __restrict__ tpl, int64_t nt,
                                                          const T* __restrict__ qry, int nq, int H,
                                                          int W, int M,
                                                          const int2* __restrict__ prog, int nprog,
                                                          T* __restrict__ out) {
    __shared__ T s_d[4][16];
    const int sub = threadIdx.x >> 4, oi = threadIdx.x & 15, NO = 2 * M - 1;
    const int64_t pair = (int64_t)blockIdx.x * 4 + sub;
    const bool live = pair < nt * (int64_t)nq;
    const int64_t t = live ? pair % nt : 0, qi = live ? pair / nt : 0;
    T d = T(INFINITY);
    if (live && oi < NO) {
        const T* a = tpl + (size_t)t * H * W;
        const T* b = qry + (size_t)qi * H * W;
        const int o = oi - (M - 1);
        T st[SAD_STACK];
        int sp = 0;
        for (int k = 0; k < nprog; ++k) {
            const int2 op = prog[k];
            if (op.x >= 0) {
                st[sp++] = sad_leaf(a, b, W, M, o, op.x, op.y);
            } else {
                const T rhs = st[--sp];
                st[sp - 1] = st[sp - 1] + rhs;
            }
        }
        d = st[0];
    }
    if (oi < 16) s_d[sub][oi] = d;
    __syncthreads();
    if (live && oi == 0) {
        T best = T(INFINITY);
        for (int k = 0; k < NO; ++k)
            if (s_d[sub][k] < best) best = s_d[sub][k];
        out[(size_t)qi * nt + t] = best;
    }
}

// The batch's first-argmin keys -> the pinned host buffer (system-scope stores),
// and the device keys reset to UINT64_MAX for the next scan: one queued launch in
// place of a device-to-host blit copy and a memset before the next scan.
__global__ __launch_bounds__(256) void vt_keys_export(unsigned long long* __restrict__ keys, int n,
                                                      unsigned long long* host) {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        __hip_atomic_store(host + i, keys[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        keys[i] = ~0ull;
    }
}

}  // namespace

// ===========================================================================
// Host side
// ===========================================================================
struct rs_vt {
    int H = 0, W = 0, M = 0, WD = 0, HQ = 0;
    // ViewTemplates.match's threshold (view_templates.py:67): a score (< 2^32, exact in
    // a double) makes a new template when score > thr, compared in float64 exactly as
    // numpy compares a uint64 with a Python float (NaN: never; negative: always)
    double thr = 0.0;
    int device = 0;
    int rank = 0, nranks = 1;
    ncclComm_t comm = nullptr;
    int64_t count = 0;     // global number of templates
    int64_t localCap = 0;  // local slots allocated (multiple of 64)
    uint4* dLib = nullptr;
    hipStream_t stream = nullptr;
    // query staging
    int qCap = 0;
    uint8_t* dQraw = nullptr;
    uint8_t* hQraw = nullptr;  // pinned, fine-grained (a small batch's plane kernel reads it in place)
    uint8_t* hQrawDev = nullptr;  // hQraw in the device's address space
    bool qrawBusy = false;     // hQraw read by queued work not yet known to have run
    uint2* dQf = nullptr;
    uint32_t* dQsum = nullptr;
    unsigned long long* dBest = nullptr;
    unsigned long long* hBest = nullptr;  // pinned
    unsigned long long* hBestDev = nullptr;  // hBest in the device's address space
    bool stagingBusy = false;  // copies from hSrc / hDst queued and not yet known to have run
    hipStream_t cstream = nullptr;           // rs_vt_match_stream's collective stream
    hipEvent_t evScan = nullptr, evComm = nullptr;
    hipStream_t ustream = nullptr;           // rs_vt_match_stream: host batches' upload stream
    hipEvent_t evUp[2] = {nullptr, nullptr}, evUsed[2] = {nullptr, nullptr};
    uint8_t* dUp[2] = {nullptr, nullptr};    // ... and its two raw-query group buffers
    size_t upCap = 0;                        // bytes per group buffer
    uint32_t* dQpStream = nullptr;           // rs_vt_match_stream: every batch's query planes
    uint32_t* dQsumStream = nullptr;
    size_t qpStreamCap = 0;                  // queries
    unsigned long long* dStream = nullptr;   // keys of rs_vt_match_stream, one row per batch
    unsigned long long* hStream = nullptr;   // pinned copy (nb * nq)
    unsigned long long* hStreamDev = nullptr;  // hStream in the device's address space
    size_t streamCap = 0;
    bool streamClean = false;                // dStream holds UINT64_MAX (vt_keys_export resets it)
    int bestClean = 0;     // leading dBest entries known to hold UINT64_MAX
    int bestPending = 0;   // bestClean once the keys of the running scan are exported
    // index lists for stores
    int idxCap = 0;
    int32_t* dSrc = nullptr;
    int64_t* dDst = nullptr;
    int32_t* hSrc = nullptr;  // pinned
    int64_t* hDst = nullptr;  // pinned
    // candidate library and score matrix for in-batch resolution
    int64_t candCap = 0;
    uint4* dCand = nullptr;
    size_t matCap = 0;
    uint32_t* dMat = nullptr;
    uint32_t* hMat = nullptr;  // pinned
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timing = false;  // HIP events around every scan (rs_vt_set_timing; off: the keys are polled)
    bool timedScan = false;  // the last scan recorded ev0/ev1
    float lastMs = 0.f;
    int stagedQ = 0;  // queries staged by the last scan
    // bit-plane scan (default when W == 32, H in {32, 64}, max_offset 8; RS_VT_SCAN=plane):
    // planes + TS of the library and candidate slots, query planes + raw sums
    bool planar = false;
    uint32_t* dLibP = nullptr;
    uint32_t* dLibTs = nullptr;
    uint32_t* dCandP = nullptr;
    uint32_t* dCandTs = nullptr;
    uint32_t* dQp = nullptr;
    uint32_t* dQsumRaw = nullptr;
    int planeSlots = 0;  // resident plane-scan blocks on the device (occupancy x CUs)
    unsigned* dCtr = nullptr;  // per template block x query group: next batch (plane scan)
    unsigned* dDone = nullptr; // plane scan blocks finished (the folded key export; reset by the last)
    bool keysFolded = false;   // the running scan exports its own keys (vt_fetch_keys: no export launch)
    int ctrCap = 0;
    // on-device subsampling of camera frames (rs_vt_set_subsample / rs_vt_match_frames)
    int32_t* dPix = nullptr;   // H*W byte offsets of the kept pixels in a frame
    int64_t frameBytes = 0;
    uint8_t* dFrames = nullptr;
    uint8_t* hFrames = nullptr;  // pinned staging for host frames
    int frameCap = 0;
};

namespace {

size_t tblock_bytes(const rs_vt* h) { return (size_t)h->WD * h->HQ * 64 * 16; }
size_t pblock_bytes(const rs_vt* h) { return (size_t)PL_CG * (h->H / 4) * 128 * 16; }
constexpr size_t TS_BLOCK_BYTES = 16 * 64 * sizeof(uint32_t);
int plane_ns(const rs_vt* h) { return h->H - 2 * h->M + 3; }

// (Re)allocate a slot buffer of `blocks` 64-slot blocks of `bb` bytes, keeping
// the first `keep` blocks.
int vt_realloc_blocks(rs_vt* h, void** buf, int64_t keep, int64_t blocks, size_t bb) {
    void* nb = nullptr;
    const size_t bytes = (size_t)blocks * bb;
    hipError_t e = hipMalloc(&nb, bytes);
    if (e != hipSuccess) {
        rs::set_error("template buffer growth to %lld slots (%zu bytes) failed: %s",
                      (long long)blocks * 64, bytes, hipGetErrorString(e));
        return e == hipErrorOutOfMemory ? RS_ERR_NOMEM : RS_ERR_HIP;
    }
    RS_HIP(hipMemsetAsync(nb, 0, bytes, h->stream));
    if (*buf) {
        if (keep > 0)
            RS_HIP(hipMemcpyAsync(nb, *buf, (size_t)keep * bb, hipMemcpyDeviceToDevice, h->stream));
        RS_HIP(hipStreamSynchronize(h->stream));
        RS_HIP(hipFree(*buf));
    }
    *buf = nb;
    return RS_OK;
}

int64_t local_count_of(const rs_vt* h, int64_t global_count) {
    if (global_count <= h->rank) return 0;
    return (global_count - h->rank + h->nranks - 1) / h->nranks;
}

int vt_grow_lib(rs_vt* h, int64_t need_slots) {
    if (need_slots <= h->localCap) return RS_OK;
    int64_t cap = h->localCap > 0 ? h->localCap : 64;
    while (cap < need_slots) cap *= 2;
    cap = (int64_t)rs::round_up((size_t)cap, 64);
    uint4* nl = nullptr;
    const size_t bytes = (size_t)(cap / 64) * tblock_bytes(h);
    hipError_t e = hipMalloc(&nl, bytes);
    if (e != hipSuccess) {
        rs::set_error("template library growth to %lld slots (%zu bytes) failed: %s",
                      (long long)cap, bytes, hipGetErrorString(e));
        return e == hipErrorOutOfMemory ? RS_ERR_NOMEM : RS_ERR_HIP;
    }
    RS_HIP(hipMemsetAsync(nl, 0, bytes, h->stream));
    if (h->dLib) {
        RS_HIP(hipMemcpyAsync(nl, h->dLib, (size_t)(h->localCap / 64) * tblock_bytes(h),
                              hipMemcpyDeviceToDevice, h->stream));
        RS_HIP(hipStreamSynchronize(h->stream));
        RS_HIP(hipFree(h->dLib));
    }
    h->dLib = nl;
    if (h->planar) {
        RS_TRY(vt_realloc_blocks(h, (void**)&h->dLibP, h->localCap / 64, cap / 64, pblock_bytes(h)));
        RS_TRY(vt_realloc_blocks(h, (void**)&h->dLibTs, h->localCap / 64, cap / 64, TS_BLOCK_BYTES));
    }
    h->localCap = cap;
    return RS_OK;
}

// hQraw (pinned) is read by a queued copy (frames, float batches) or, for small batches,
// in place by the plane kernel: before the host writes or frees it again that work must
// have run.  Every call that stages into it waits for its keys before returning
// (vt_fetch_keys clears the flag); after an error between the staging and that wait the
// stream is synchronised here.  (rs_vt_add uploads the caller's array directly.)
int vt_qraw_idle(rs_vt* h) {
    if (h->qrawBusy) {
        RS_HIP(hipStreamSynchronize(h->stream));
        h->qrawBusy = false;
    }
    return RS_OK;
}

int vt_grow_queries(rs_vt* h, int nq) {
    if (nq <= h->qCap) return RS_OK;
    int cap = h->qCap > 0 ? h->qCap : 64;
    while (cap < nq) cap *= 2;
    RS_TRY(vt_qraw_idle(h));
    if (h->dQraw) RS_HIP(hipFree(h->dQraw));
    if (h->hQraw) RS_HIP(hipHostFree(h->hQraw));
    h->hQraw = h->hQrawDev = nullptr;
    if (h->dQf) RS_HIP(hipFree(h->dQf));
    if (h->dQsum) RS_HIP(hipFree(h->dQsum));
    if (h->dBest) RS_HIP(hipFree(h->dBest));
    if (h->hBest) RS_HIP(hipHostFree(h->hBest));
    if (h->dQp) RS_HIP(hipFree(h->dQp));
    if (h->dQsumRaw) RS_HIP(hipFree(h->dQsumRaw));
    h->dQp = h->dQsumRaw = nullptr;
    const size_t qb = (size_t)h->H * h->W;
    if (h->planar) {
        RS_HIP(hipMalloc(&h->dQp, sizeof(uint32_t) * PL_CG * plane_ns(h) * 8 * (size_t)cap));
        RS_HIP(hipMalloc(&h->dQsumRaw, sizeof(uint32_t) * cap));
    }
    RS_HIP(hipMalloc(&h->dQraw, qb * cap));
    RS_HIP(hipHostMalloc(&h->hQraw, qb * cap, hipHostMallocMapped | hipHostMallocCoherent));
    RS_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&h->hQrawDev), h->hQraw, 0));
    RS_HIP(hipMalloc(&h->dQf, sizeof(uint2) * (size_t)h->WD * h->H * cap));
    RS_HIP(hipMalloc(&h->dQsum, sizeof(uint32_t) * cap));
    RS_HIP(hipMalloc(&h->dBest, sizeof(unsigned long long) * cap));
    // fine-grained (coherent): vt_fetch_keys polls the words the export kernel stores
    RS_HIP(hipHostMalloc(&h->hBest, sizeof(unsigned long long) * cap, hipHostMallocMapped | hipHostMallocCoherent));
    RS_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&h->hBestDev), h->hBest, 0));
    h->bestClean = h->bestPending = 0;
    h->qCap = cap;
    return RS_OK;
}

int vt_grow_index(rs_vt* h, int n) {
    if (n <= h->idxCap) return RS_OK;
    int cap = h->idxCap > 0 ? h->idxCap : 64;
    while (cap < n) cap *= 2;
    if (h->dSrc) RS_HIP(hipFree(h->dSrc));
    if (h->dDst) RS_HIP(hipFree(h->dDst));
    if (h->hSrc) RS_HIP(hipHostFree(h->hSrc));
    if (h->hDst) RS_HIP(hipHostFree(h->hDst));
    RS_HIP(hipMalloc(&h->dSrc, sizeof(int32_t) * cap));
    RS_HIP(hipMalloc(&h->dDst, sizeof(int64_t) * cap));
    RS_HIP(hipHostMalloc(&h->hSrc, sizeof(int32_t) * cap, hipHostMallocDefault));
    RS_HIP(hipHostMalloc(&h->hDst, sizeof(int64_t) * cap, hipHostMallocDefault));
    h->idxCap = cap;
    return RS_OK;
}

int vt_grow_matrix(rs_vt* h, size_t elems) {
    if (elems <= h->matCap) return RS_OK;
    size_t cap = h->matCap > 0 ? h->matCap : 4096;
    while (cap < elems) cap *= 2;
    if (h->dMat) RS_HIP(hipFree(h->dMat));
    if (h->hMat) RS_HIP(hipHostFree(h->hMat));
    RS_HIP(hipMalloc(&h->dMat, sizeof(uint32_t) * cap));
    RS_HIP(hipHostMalloc(&h->hMat, sizeof(uint32_t) * cap, hipHostMallocDefault));
    h->matCap = cap;
    return RS_OK;
}

int vt_grow_cand(rs_vt* h, int64_t slots) {
    if (slots <= h->candCap) return RS_OK;
    int64_t cap = h->candCap > 0 ? h->candCap : 64;
    while (cap < slots) cap *= 2;
    if (h->dCand) RS_HIP(hipFree(h->dCand));
    RS_HIP(hipMalloc(&h->dCand, (size_t)(cap / 64) * tblock_bytes(h)));
    if (h->planar) {
        RS_TRY(vt_realloc_blocks(h, (void**)&h->dCandP, 0, cap / 64, pblock_bytes(h)));
        RS_TRY(vt_realloc_blocks(h, (void**)&h->dCandTs, 0, cap / 64, TS_BLOCK_BYTES));
    }
    h->candCap = cap;
    return RS_OK;
}

int vt_build_forms(rs_vt* h, int nq);

// Batches of at most this many queries are read by the plane kernel straight from the
// pinned staging array (one launch in place of a host-to-device copy and the launch;
// the kernel leaves the raw bytes in dQraw for the template stores); RS_VT_ZC=0: always
// the copy.
constexpr int VT_ZC_MAX = 64;
bool vt_zc_env() {
    static const bool on = [] {
        const char* e = std::getenv("RS_VT_ZC");
        return !(e && std::strcmp(e, "0") == 0);
    }();
    return on;
}

// Upload nq raw queries and build their forms on the device.
int vt_stage_queries(rs_vt* h, int nq, const uint8_t* queries) {
    RS_TRY(vt_grow_queries(h, nq));
    RS_TRY(vt_qraw_idle(h));
    const size_t qb = (size_t)h->H * h->W * nq;
    // larger batches: HIP's own upload of the caller's (pageable) array, which returns
    // once the bytes are staged (per-batch PCIe-inclusive rate 4.04-4.12 against 3.44-3.54
    // G compares/s through our memcpy into pinned staging, round 5).  The call waits for
    // its keys, which the scan stores after the copy has run, so a pinned caller array is
    // no longer read when it returns.
    if (h->planar && nq <= VT_ZC_MAX && vt_zc_env()) {
        std::memcpy(h->hQraw, queries, qb);
        h->qrawBusy = true;
        hipLaunchKernelGGL(vt_qplane_kernel, dim3(nq), dim3(256), 0, h->stream, h->hQrawDev, h->H, h->M, h->dQp,
                           h->dQsumRaw, h->dQraw);
        RS_HIP(hipGetLastError());
        return RS_OK;
    }
    RS_HIP(hipMemcpyAsync(h->dQraw, queries, qb, hipMemcpyHostToDevice, h->stream));
    return vt_build_forms(h, nq);
}

// Build the query forms of nq raw queries in device memory (default: dQraw).
// The plane scan reads only the planes; the byte-SWAR forms serve the other scans.
int vt_build_forms(rs_vt* h, int nq, const uint8_t* src) {
    if (!h->planar)
        hipLaunchKernelGGL(vt_qform_kernel, dim3(nq), dim3(256), 0, h->stream, src, h->H, h->W,
                           h->WD, h->M, h->dQf, h->dQsum);
    else
        hipLaunchKernelGGL(vt_qplane_kernel, dim3(nq), dim3(256), 0, h->stream, src, h->H,
                           h->M, h->dQp, h->dQsumRaw, nullptr);
    RS_HIP(hipGetLastError());
    return RS_OK;
}

int vt_build_forms(rs_vt* h, int nq) { return vt_build_forms(h, nq, h->dQraw); }

// Subsample nf frames on the device into the raw query buffer, then build the
// forms.  Host frames go through a pinned staging buffer; device-resident frames
// (a camera / decoder pipeline on the GPU) are gathered in place.
int vt_stage_frames(rs_vt* h, int nf, const uint8_t* frames) {
    RS_CHECK(h->dPix, RS_ERR_STATE, "no subsampling mask: call rs_vt_set_subsample first");
    RS_TRY(vt_grow_queries(h, nf));
    hipPointerAttribute_t attr{};
    const bool on_device = hipPointerGetAttributes(&attr, frames) == hipSuccess &&
                           attr.type == hipMemoryTypeDevice;
    (void)hipGetLastError();  // a host pointer is not an error
    const uint8_t* src = frames;
    if (!on_device) {
        if (nf > h->frameCap) {
            int cap = h->frameCap > 0 ? h->frameCap : 16;
            while (cap < nf) cap *= 2;
            if (h->dFrames) RS_HIP(hipFree(h->dFrames));
            if (h->hFrames) RS_HIP(hipHostFree(h->hFrames));
            h->dFrames = nullptr;
            h->hFrames = nullptr;
            RS_HIP(hipMalloc(&h->dFrames, (size_t)h->frameBytes * cap));
            RS_HIP(hipHostMalloc(&h->hFrames, (size_t)h->frameBytes * cap, hipHostMallocDefault));
            h->frameCap = cap;
        }
        const size_t fb = (size_t)h->frameBytes * nf;
        std::memcpy(h->hFrames, frames, fb);
        RS_HIP(hipMemcpyAsync(h->dFrames, h->hFrames, fb, hipMemcpyHostToDevice, h->stream));
        src = h->dFrames;
    }
    hipLaunchKernelGGL(vt_gather_kernel, dim3(nf), dim3(256), 0, h->stream, src,
                       (size_t)h->frameBytes, h->dPix, h->H * h->W, h->dQraw);
    RS_HIP(hipGetLastError());
    return vt_build_forms(h, nf);
}

// Store raw staged queries src[i] into slots dst[i] of the library (or, with
// `cand`, of the candidate buffer).
int vt_store(rs_vt* h, bool cand, const uint8_t* d_raw, int n) {
    if (n == 0) return RS_OK;
    uint4* lib = cand ? h->dCand : h->dLib;
    RS_HIP(hipMemcpyAsync(h->dSrc, h->hSrc, sizeof(int32_t) * n, hipMemcpyHostToDevice, h->stream));
    RS_HIP(hipMemcpyAsync(h->dDst, h->hDst, sizeof(int64_t) * n, hipMemcpyHostToDevice, h->stream));
    h->stagingBusy = true;
    const int64_t total = (int64_t)n * h->WD * h->HQ;
    const int grid = (int)std::min<int64_t>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(vt_store_kernel, dim3(grid), dim3(256), 0, h->stream, d_raw, h->dSrc,
                       h->dDst, n, lib, h->H, h->W, h->WD, h->HQ);
    if (h->planar)
        hipLaunchKernelGGL(vt_plane_store_kernel, dim3(n), dim3(256), 0, h->stream, d_raw, h->dSrc,
                           h->dDst, h->H, h->M, cand ? h->dCandP : h->dLibP,
                           cand ? h->dCandTs : h->dLibTs);
    RS_HIP(hipGetLastError());
    return RS_OK;
}

// Blocks per template block (nqc) for the plane scan.  A block's fixed cost
// (its template planes, 128 KiB, into VGPRs) is small next to its query batches,
// and the nqc blocks of a template block balance their batches dynamically, so
// finer splits fill the last round of resident blocks better; measured on
// MI355X (tools/scan_split.py, 1,024 queries): nqc = 32 is within 2% of the best
// split from 12.5k to 100k templates (100k: 18.6 ms at nqc = 1, the previous
// choice there, vs 15.0 ms), and small libraries gain from up to 4 rounds of
// blocks (1k: 128 -> 0.183 ms vs 0.199 ms at 32).  nqc >= 8 is a multiple of 8
// (the XCD query groups).  RS_VT_NQC overrides (A/B).
int plane_split(int ntb, int nbatch, int slots) {
    int nqc;
    if (const char* e = std::getenv("RS_VT_NQC")) {
        nqc = std::max(1, std::atoi(e));
    } else {
        const int fill = (slots + ntb - 1) / ntb;  // blocks per template block for one round
        nqc = std::max(32, std::min(4 * fill, std::max(128, fill)));
    }
    nqc = std::min(nqc, std::max(1, nbatch));
    if (nqc >= 8) nqc &= ~7;
    return nqc;
}

// Launch a scan of queries [0, nq) (forms in dQf) against `count` slots of lib.
template <bool MATRIX>
int vt_launch_plane(rs_vt* h, bool cand, int64_t count, int nq, ScanOut out, int rank,
                    int nranks, int64_t tb0) {
    const int ntb = (int)((count + 63) / 64);
    const int nqc = plane_split(ntb, (nq + PL_NB - 1) / PL_NB, h->planeSlots);
    if (8 * ntb > h->ctrCap) {  // counters start at zero and every scan leaves them at zero
        const int cap = std::max(8 * ntb, 2 * h->ctrCap);
        if (h->dCtr) RS_HIP(hipFree(h->dCtr));
        h->dCtr = nullptr;
        h->ctrCap = 0;
        RS_HIP(hipMalloc(&h->dCtr, sizeof(unsigned) * (size_t)cap));
        RS_HIP(hipMemsetAsync(h->dCtr, 0, sizeof(unsigned) * (size_t)cap, h->stream));
        h->ctrCap = cap;
    }
    RS_CHECK((int64_t)ntb * nqc < (1ll << 31), RS_ERR_ARG, "scan grid too large");
    const dim3 grid((unsigned)(ntb * nqc));
    const uint4* planes = reinterpret_cast<const uint4*>(
        reinterpret_cast<const uint8_t*>(cand ? h->dCandP : h->dLibP) + (size_t)tb0 * pblock_bytes(h));
    const uint32_t* ts = (cand ? h->dCandTs : h->dLibTs) + (size_t)tb0 * (TS_BLOCK_BYTES / 4);
    if (h->H == 64)
        hipLaunchKernelGGL((vt_scan_plane_kernel<64, MATRIX>), grid, dim3(64 * PL_CG * PL_SPLIT), 0, h->stream,
                           planes, ts, ntb, count, h->dQp, h->dQsumRaw, nq, nqc, h->dCtr, out, rank,
                           nranks);
    else
        hipLaunchKernelGGL((vt_scan_plane_kernel<32, MATRIX>), grid, dim3(64 * PL_CG * PL_SPLIT), 0, h->stream,
                           planes, ts, ntb, count, h->dQp, h->dQsumRaw, nq, nqc, h->dCtr, out, rank,
                           nranks);
    RS_HIP(hipGetLastError());
    return RS_OK;
}

// Launch a scan of queries [0, nq) against `count` slots of the library (or of
// the candidate buffer), starting at 64-slot block tb0 of it.
template <bool MATRIX>
int vt_launch_scan(rs_vt* h, bool cand, int64_t count, int nq, ScanOut out, int rank,
                   int nranks, int64_t tb0 = 0) {
    if (count <= 0 || nq <= 0) return RS_OK;
    if (h->planar) return vt_launch_plane<MATRIX>(h, cand, count, nq, out, rank, nranks, tb0);
    const uint4* lib = (cand ? h->dCand : h->dLib) + (size_t)tb0 * h->WD * h->HQ * 64;
    const int ntb = (int)((count + 63) / 64);
    const bool fast = h->M == FAST_M && (h->H == 64 || h->H == 32);
    RS_CHECK((int64_t)ntb * nq < (1ll << 31), RS_ERR_ARG, "scan grid too large (%d x %d)", ntb, nq);
    if (fast && !MATRIX && (int64_t)ntb * nq < 2048 && h->WD <= 8) {
        // few waves of work: spread each template over 8 column lanes
        const dim3 grid((unsigned)((count + 7) / 8), nq);
        if (h->H == 64)
            hipLaunchKernelGGL((vt_scan_carry_col_kernel<64, 1>), grid, dim3(64), 0, h->stream,
                               lib, count, h->WD, h->dQf, h->dQsum, nq, out, rank, nranks);
        else
            hipLaunchKernelGGL((vt_scan_carry_col_kernel<32, 1>), grid, dim3(64), 0, h->stream,
                               lib, count, h->WD, h->dQf, h->dQsum, nq, out, rank, nranks);
    } else if (fast) {
        constexpr int NQ = 2;
        const int nqg = (nq + NQ - 1) / NQ;
        const dim3 grid((unsigned)(ntb * ((nqg + 7) / 8) * 8));
        if (h->H == 64)
            hipLaunchKernelGGL((vt_scan_carry_kernel<64, NQ, MATRIX>), grid, dim3(64), 0,
                               h->stream, lib, ntb, count, h->WD, h->dQf, h->dQsum, nq, out,
                               rank, nranks);
        else
            hipLaunchKernelGGL((vt_scan_carry_kernel<32, NQ, MATRIX>), grid, dim3(64), 0,
                               h->stream, lib, ntb, count, h->WD, h->dQf, h->dQsum, nq, out,
                               rank, nranks);
    } else {
        hipLaunchKernelGGL((vt_scan_generic_kernel<MATRIX>), dim3((unsigned)(ntb * nq)), dim3(64),
                           0, h->stream, lib, ntb, count, h->H, h->M, h->WD, h->dQf, nq, out, rank,
                           nranks);
    }
    RS_HIP(hipGetLastError());
    return RS_OK;
}

// The host waits for a call's keys by polling them (pinned, fine-grained; each key one
// 8-byte system-scope store by vt_keys_export, the call's last kernel) instead of the
// stream's completion signal and its own wake-up: the host reads nothing else the call
// wrote, and every later device access is ordered on the stream (the pinned staging
// arrays a call's copies read are guarded by vt_staging_idle).  A spin that runs out
// falls back to the stream synchronisation.  RS_VT_POLL=0: always synchronise.
constexpr unsigned long long KEY_PENDING = 0xFFFFFFFF00000000ull;  // score 2^32-1: never a key
constexpr int VT_POLL_MAX = 4096;
bool vt_poll_env() {
    static const bool on = [] {
        const char* e = std::getenv("RS_VT_POLL");
        return !(e && std::strcmp(e, "0") == 0);
    }();
    return on;
}
bool vt_poll_keys(const unsigned long long* w_, int n) {
    const volatile unsigned long long* w = w_;
    int i = 0;
    for (long spin = 0; spin < 4000000 && i < n; ++spin)
        while (i < n && w[i] != KEY_PENDING) ++i;
    return i == n;
}

// The pinned staging arrays hSrc / hDst are read by asynchronous copies (vt_store):
// before the host writes or reallocates them again, those copies must have run.
int vt_staging_idle(rs_vt* h) {
    if (h->stagingBusy) {
        RS_HIP(hipStreamSynchronize(h->stream));
        h->stagingBusy = false;
    }
    return RS_OK;
}

int vt_append_staged(rs_vt* h, const std::vector<std::pair<int, int64_t>>& news) {
    // news: (staged query index, global index) in order
    int mine = 0;
    RS_TRY(vt_staging_idle(h));
    RS_TRY(vt_grow_index(h, (int)news.size() + 1));
    const int64_t new_count = h->count + (int64_t)news.size();
    RS_TRY(vt_grow_lib(h, local_count_of(h, new_count)));
    for (const auto& p : news) {
        if (p.second % h->nranks != h->rank) continue;
        h->hSrc[mine] = p.first;
        h->hDst[mine] = p.second / h->nranks;
        ++mine;
    }
    RS_TRY(vt_store(h, false, h->dQraw, mine));
    h->count = new_count;
    return RS_OK;
}

// Stage nq queries (raw H x W, or whole frames subsampled on the device) and
// min-reduce their local first-argmin keys into dBest.
int vt_scan_local_impl(rs_vt* h, int nq, const uint8_t* queries, bool frames = false, bool fold_ok = true) {
    RS_CHECK(h, RS_ERR_STATE, "null view-template handle");
    RS_CHECK(nq >= 0, RS_ERR_ARG, "negative query count");
    if (nq == 0) return RS_OK;
    RS_HIP(hipSetDevice(h->device));
    if (frames) {
        RS_CHECK(queries, RS_ERR_ARG, "null frames");
        RS_TRY(vt_stage_frames(h, nq, queries));
    } else if (queries) {
        RS_TRY(vt_stage_queries(h, nq, queries));
    } else {
        // re-match the queries already resident on the device (last staged batch)
        RS_CHECK(nq == h->stagedQ, RS_ERR_STATE, "no staged batch of %d queries (have %d)", nq,
                 h->stagedQ);
    }
    if (h->bestClean < nq) {  // vt_keys_export resets the keys it hands over
        RS_HIP(hipMemsetAsync(h->dBest, 0xFF, sizeof(unsigned long long) * nq, h->stream));
        h->bestClean = nq;
    }
    h->bestPending = h->bestClean;  // [0, nq) is dirty until exported; the rest stays clean
    h->bestClean = 0;
    const int64_t lc = local_count_of(h, h->count);
    ScanOut out{h->dBest, nullptr, 0};
    // a plane scan whose keys the host polls exports them itself (its last block): one
    // launch fewer per call.  Not when they are min-reduced over ranks first.
    h->keysFolded = fold_ok && h->planar && lc > 0 && vt_poll_env() && !h->timing && nq <= VT_POLL_MAX;
    if (h->keysFolded) {
        if (!h->dDone) {
            RS_HIP(hipMalloc(&h->dDone, sizeof(unsigned)));
            RS_HIP(hipMemsetAsync(h->dDone, 0, sizeof(unsigned), h->stream));
        }
        for (int i = 0; i < nq; ++i) h->hBest[i] = KEY_PENDING;
        out.host = h->hBestDev;
        out.done = h->dDone;
    }
    if (h->timing) RS_HIP(hipEventRecord(h->ev0, h->stream));
    RS_TRY(vt_launch_scan<false>(h, false, lc, nq, out, h->rank, h->nranks));
    if (h->timing) RS_HIP(hipEventRecord(h->ev1, h->stream));
    h->timedScan = h->timing;
    h->stagedQ = nq;
    return RS_OK;
}

// Given the global keys of the staged queries, decide hits / new templates in
// ViewTemplates.match order and append the new templates this rank owns.
int vt_resolve_impl(rs_vt* h, int nq, const unsigned long long* keys, int mode,
                    uint64_t* best_score, int64_t* best_index, uint8_t* is_new) {
    RS_CHECK(h, RS_ERR_STATE, "null view-template handle");
    RS_CHECK(mode == RS_VT_FROZEN || mode == RS_VT_SEQUENTIAL, RS_ERR_ARG, "unknown mode %d", mode);
    RS_CHECK(nq == h->stagedQ, RS_ERR_STATE, "resolve of %d queries, %d staged", nq, h->stagedQ);
    if (nq == 0) return RS_OK;
    RS_CHECK(keys, RS_ERR_ARG, "null keys");
    RS_HIP(hipSetDevice(h->device));
    std::vector<unsigned long long> key(keys, keys + nq);
    if (mode == RS_VT_FROZEN) {
        for (int i = 0; i < nq; ++i) {
            if (is_new) is_new[i] = 0;
            if (best_index) best_index[i] = key[i] == NO_KEY ? -1 : (int64_t)(key[i] & 0xFFFFFFFFull);
            if (best_score) best_score[i] = key[i] == NO_KEY ? UINT64_MAX : (key[i] >> 32);
        }
        return RS_OK;
    }
    // Candidates: queries that miss the stored library.  Only they can become
    // templates; a later query may still prefer one of them (first argmin over
    // the grown list, view_templates.py:65-73), so every candidate is scored as
    // a template against every query once (replicated on all ranks).
    std::vector<int> cand;
    for (int i = 0; i < nq; ++i)
        if (key[i] == NO_KEY || (double)(key[i] >> 32) > h->thr) cand.push_back(i);
    std::vector<int> cpos(nq, -1);
    int64_t ldm = 0;
    if (!cand.empty() && cand.front() < nq - 1) {
        RS_TRY(vt_staging_idle(h));
        const int64_t C = (int64_t)cand.size();
        RS_TRY(vt_grow_cand(h, (int64_t)rs::round_up((size_t)C, 64)));
        RS_TRY(vt_grow_index(h, (int)C));
        for (int64_t j = 0; j < C; ++j) {
            h->hSrc[j] = cand[j];
            h->hDst[j] = j;
            cpos[cand[j]] = (int)j;
        }
        RS_TRY(vt_store(h, true, h->dQraw, (int)C));
        ldm = (int64_t)rs::round_up((size_t)C, 64);
        RS_TRY(vt_grow_matrix(h, (size_t)ldm * nq));
        ScanOut mo{nullptr, h->dMat, ldm};
        RS_TRY(vt_launch_scan<true>(h, true, C, nq, mo, 0, 1));
        RS_HIP(hipMemcpyAsync(h->hMat, h->dMat, sizeof(uint32_t) * ldm * nq, hipMemcpyDeviceToHost,
                              h->stream));
        RS_HIP(hipStreamSynchronize(h->stream));
        h->stagingBusy = false;
    }
    std::vector<std::pair<int, int64_t>> news;
    for (int i = 0; i < nq; ++i) {
        unsigned long long k = key[i];
        for (size_t a = 0; a < news.size(); ++a) {
            const int j = news[a].first;
            const unsigned long long kj =
                ((unsigned long long)h->hMat[(size_t)i * ldm + cpos[j]] << 32) |
                (unsigned long long)news[a].second;
            k = kj < k ? kj : k;
        }
        if (k == NO_KEY || (double)(k >> 32) > h->thr) {
            const int64_t g = h->count + (int64_t)news.size();
            news.emplace_back(i, g);
            if (is_new) is_new[i] = 1;
            if (best_index) best_index[i] = g;
        } else {
            if (is_new) is_new[i] = 0;
            if (best_index) best_index[i] = (int64_t)(k & 0xFFFFFFFFull);
        }
        if (best_score) best_score[i] = k == NO_KEY ? UINT64_MAX : (k >> 32);
    }
    RS_TRY(vt_append_staged(h, news));   // (its copies guarded by vt_staging_idle, not a sync)
    return RS_OK;
}

int vt_fetch_keys(rs_vt* h, int nq, bool allreduce) {
    if (allreduce && h->nranks > 1) {
        RS_CHECK(h->comm, RS_ERR_STATE, "sharded handle without a communicator: use "
                 "rs_vt_scan_local + an external min-reduction + rs_vt_resolve");
        ncclResult_t r = ncclAllReduce(h->dBest, h->dBest, (size_t)nq, ncclUint64, ncclMin, h->comm,
                                       h->stream);
        RS_CHECK(r == ncclSuccess, RS_ERR_RCCL, "ncclAllReduce(min) failed: %s",
                 ncclGetErrorString(r));
    }
    const bool poll = vt_poll_env() && !h->timedScan && nq <= VT_POLL_MAX;
    if (h->keysFolded) {   // the scan's last block exports them (vt_scan_local_impl)
        h->keysFolded = false;
    } else {
        if (poll)
            for (int i = 0; i < nq; ++i) h->hBest[i] = KEY_PENDING;
        hipLaunchKernelGGL(vt_keys_export, dim3((nq + 255) / 256 < 64 ? (nq + 255) / 256 : 64), dim3(256), 0,
                           h->stream, h->dBest, nq, h->hBestDev);
        RS_HIP(hipGetLastError());
    }
    if (!(poll && vt_poll_keys(h->hBest, nq))) {
        RS_HIP(hipStreamSynchronize(h->stream));
        h->stagingBusy = false;
    }
    // the keys are the call's last work: everything queued before them has run,
    // the readers of hQraw included (not the staging copies vt_store queues after them)
    h->qrawBusy = false;
    h->bestClean = h->bestPending;
    if (h->timedScan) RS_HIP(hipEventElapsedTime(&h->lastMs, h->ev0, h->ev1));
    return RS_OK;
}

// nb frozen-library batches queued back to back with one host synchronisation:
// per batch the forms are built straight from the raw queries (device-resident
// ones in place; host ones through dQraw) and the library is scanned into that
// batch's row of keys; with a communicator the row is min-reduced over the ranks
// on a second stream, overlapped with the next batch; one copy brings all rows back.
constexpr int VT_UP_GROUP = 16;  // host batches per upload group of rs_vt_match_stream

int vt_match_stream_impl(rs_vt* h, int nb, int nq, const uint8_t* queries, uint64_t* best_score,
                         int64_t* best_index) {
    RS_CHECK(h, RS_ERR_STATE, "null view-template handle");
    RS_CHECK(nb >= 0 && nq >= 0, RS_ERR_ARG, "negative batch or query count");
    if (nb == 0 || nq == 0) return RS_OK;
    RS_CHECK(queries, RS_ERR_ARG, "null queries");
    RS_CHECK(h->nranks == 1 || h->comm, RS_ERR_STATE, "sharded handle without a communicator: "
             "rs_vt_match_stream needs the RCCL reduction (rs_vt_attach_comm)");
    if (h->comm && !h->cstream) {
        RS_HIP(hipStreamCreateWithFlags(&h->cstream, hipStreamNonBlocking));
        RS_HIP(hipEventCreateWithFlags(&h->evScan, hipEventDisableTiming));
        RS_HIP(hipEventCreateWithFlags(&h->evComm, hipEventDisableTiming));
    }
    RS_HIP(hipSetDevice(h->device));
    RS_TRY(vt_grow_queries(h, nq));
    const size_t total = (size_t)nb * nq;
    RS_CHECK(total <= INT32_MAX, RS_ERR_ARG, "too many queries in one stream");
    if (total > h->streamCap) {
        if (h->hStream) RS_HIP(hipHostFree(h->hStream));
        if (h->dStream) RS_HIP(hipFree(h->dStream));
        h->hStream = h->dStream = nullptr;
        h->streamCap = 0;
        RS_HIP(hipHostMalloc(&h->hStream, sizeof(unsigned long long) * total, hipHostMallocDefault));
        RS_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&h->hStreamDev), h->hStream, 0));
        RS_HIP(hipMalloc(&h->dStream, sizeof(unsigned long long) * total));
        h->streamCap = total;
        h->streamClean = false;
    }
    hipPointerAttribute_t attr{};
    const bool on_device = hipPointerGetAttributes(&attr, queries) == hipSuccess &&
                           attr.type == hipMemoryTypeDevice;
    (void)hipGetLastError();  // a host pointer is not an error
    RS_CHECK(!on_device || reinterpret_cast<uintptr_t>(queries) % 8 == 0, RS_ERR_ARG,
             "device-resident queries must be 8-byte aligned");
    const size_t qb = (size_t)h->H * h->W * nq;
    // the keys start at UINT64_MAX: the export of the previous call reset them
    // (one memset after allocation, or after a call that did not reach its export)
    if (!h->streamClean)
        RS_HIP(hipMemsetAsync(h->dStream, 0xFF, sizeof(unsigned long long) * h->streamCap, h->stream));
    h->streamClean = false;
    h->stagedQ = 0;  // the forms no longer match dQraw
    h->timedScan = false;
    const int64_t lc = local_count_of(h, h->count);
    // Device-resident batches of the plane scan: one launch builds every batch's
    // planes (nb * nq blocks) and ONE scan launch covers all nb * nq queries (the
    // batches are independent against a frozen library, and their keys are rows of
    // one array), so the scan's fixed costs -- each block's template planes into
    // VGPRs, the last partial round of blocks -- are paid once per call instead of
    // once per batch; a sharded handle then min-reduces all rows in one collective.
    // Host batches of the plane scan take the same fused path in groups of up to
    // VT_UP_GROUP batches: a group is uploaded on the upload stream into one of two
    // device buffers while the previous group's planes and scan run on the main stream
    // (the upload of pageable memory holds the host, not the GPU), then its planes are
    // built in one launch and scanned in one launch.  One batch per launch with its
    // upload in line (the earlier form) ran at 0.52 of the HBM-resident rate.
    const bool hostgroups = !on_device && h->planar;
    const bool allplanes = (on_device && h->planar && nb > 1) || hostgroups;
    const size_t qpq = (size_t)PL_CG * plane_ns(h) * 8;  // plane dwords per query
    struct PlaneBufRestore {  // h->dQp / dQsumRaw point at the per-batch buffers on return
        rs_vt* h;
        uint32_t* p;
        uint32_t* q;
        ~PlaneBufRestore() { h->dQp = p; h->dQsumRaw = q; }
    } restore{h, h->dQp, h->dQsumRaw};
    if (allplanes) {
        if (total > h->qpStreamCap) {
            if (h->dQpStream) RS_HIP(hipFree(h->dQpStream));
            if (h->dQsumStream) RS_HIP(hipFree(h->dQsumStream));
            h->dQpStream = h->dQsumStream = nullptr;
            h->qpStreamCap = 0;
            RS_HIP(hipMalloc(&h->dQpStream, sizeof(uint32_t) * qpq * total));
            RS_HIP(hipMalloc(&h->dQsumStream, sizeof(uint32_t) * total));
            h->qpStreamCap = total;
        }
        RS_CHECK(total <= INT32_MAX, RS_ERR_ARG, "too many queries in one stream");
        h->dQp = h->dQpStream;
        h->dQsumRaw = h->dQsumStream;
        if (!hostgroups) {
            RS_TRY(vt_build_forms(h, (int)total, queries));
            const ScanOut out{h->dStream, nullptr, 0};
            // the one scan of the call, bracketed by events when timing (rs_vt_last_ms)
            if (h->timing) RS_HIP(hipEventRecord(h->ev0, h->stream));
            RS_TRY(vt_launch_scan<false>(h, false, lc, (int)total, out, h->rank, h->nranks));
            if (h->timing) RS_HIP(hipEventRecord(h->ev1, h->stream));
            h->timedScan = h->timing;
        } else {
            // a first group of one batch (its upload is the only one not hidden behind a
            // scan), then groups of about a third of the rest (2 .. VT_UP_GROUP batches: a
            // scan launch of >= 2 batches keeps the fused launch's efficiency).  10 batches
            // of 1,024 queries from a pageable array: groups (1, 3, 3, 3) 1.674 ms per call
            // against 1.745 for (2, 2, 2, 2, 2), 1.759 for threes, 1.762 for fives, 1.920 for
            // ones, and 1.757 with the caller's array page-locked for the call
            // (hipHostRegister): the uploads are not the bound (tools/stream_ab.py --host)
            const int gb = std::min(nb, std::max(2, std::min(VT_UP_GROUP, (nb - 1) / 3)));
            if (!h->ustream) {
                RS_HIP(hipStreamCreateWithFlags(&h->ustream, hipStreamNonBlocking));
                for (int i = 0; i < 2; ++i) {
                    RS_HIP(hipEventCreateWithFlags(&h->evUp[i], hipEventDisableTiming));
                    RS_HIP(hipEventCreateWithFlags(&h->evUsed[i], hipEventDisableTiming));
                }
            }
            if (qb * gb > h->upCap) {
                RS_HIP(hipStreamSynchronize(h->ustream));
                for (int i = 0; i < 2; ++i) {
                    if (h->dUp[i]) RS_HIP(hipFree(h->dUp[i]));
                    h->dUp[i] = nullptr;
                }
                h->upCap = 0;
                for (int i = 0; i < 2; ++i) RS_HIP(hipMalloc(&h->dUp[i], qb * gb));
                h->upCap = qb * gb;
            }
            const int g1n = nb >= 4 ? 1 : gb;
            for (int g = 0, b0 = 0, n = 0; b0 < nb; ++g, b0 += n) {
                n = std::min(g == 0 ? g1n : gb, nb - b0);
                const int bi = g & 1;
                // the buffer's group before last has had its planes built
                if (g >= 2) RS_HIP(hipStreamWaitEvent(h->ustream, h->evUsed[bi], 0));
                RS_HIP(hipMemcpyAsync(h->dUp[bi], queries + qb * b0, qb * n, hipMemcpyHostToDevice, h->ustream));
                RS_HIP(hipEventRecord(h->evUp[bi], h->ustream));
                RS_HIP(hipStreamWaitEvent(h->stream, h->evUp[bi], 0));
                h->dQp = h->dQpStream + qpq * (size_t)b0 * nq;
                h->dQsumRaw = h->dQsumStream + (size_t)b0 * nq;
                RS_TRY(vt_build_forms(h, n * nq, h->dUp[bi]));
                RS_HIP(hipEventRecord(h->evUsed[bi], h->stream));
                const ScanOut out{h->dStream + (size_t)b0 * nq, nullptr, 0};
                RS_TRY(vt_launch_scan<false>(h, false, lc, n * nq, out, h->rank, h->nranks));
            }
            h->timedScan = false;   // scans interleaved with upload waits: no single duration
        }
        if (h->comm) {
            ncclResult_t r = ncclAllReduce(h->dStream, h->dStream, total, ncclUint64, ncclMin, h->comm,
                                           h->stream);
            RS_CHECK(r == ncclSuccess, RS_ERR_RCCL, "ncclAllReduce(min) failed: %s",
                     ncclGetErrorString(r));
        }
    }
    for (int b = 0; b < nb && !allplanes; ++b) {
        unsigned long long* keys = h->dStream + (size_t)b * nq;
        const ScanOut out{keys, nullptr, 0};
        const uint8_t* src = queries + qb * b;
        if (!on_device) {
            RS_HIP(hipMemcpyAsync(h->dQraw, src, qb, hipMemcpyHostToDevice, h->stream));
            src = h->dQraw;
        }
        RS_TRY(vt_build_forms(h, nq, src));
        RS_TRY(vt_launch_scan<false>(h, false, lc, nq, out, h->rank, h->nranks));
        if (h->comm) {
            // the batch's row is reduced on the collective stream while the next
            // batch's planes and scan run on the main stream (rows are distinct)
            RS_HIP(hipEventRecord(h->evScan, h->stream));
            RS_HIP(hipStreamWaitEvent(h->cstream, h->evScan, 0));
            ncclResult_t r = ncclAllReduce(keys, keys, (size_t)nq, ncclUint64, ncclMin, h->comm,
                                           h->cstream);
            RS_CHECK(r == ncclSuccess, RS_ERR_RCCL, "ncclAllReduce(min) failed: %s",
                     ncclGetErrorString(r));
        }
    }
    if (h->comm && !allplanes) {
        RS_HIP(hipEventRecord(h->evComm, h->cstream));
        RS_HIP(hipStreamWaitEvent(h->stream, h->evComm, 0));
    }
    // keys -> pinned host memory and reset for the next call, in one queued launch
    // (in place of a device-to-host blit and a memset)
    hipLaunchKernelGGL(vt_keys_export, dim3(std::min<size_t>((total + 255) / 256, 256)), dim3(256), 0,
                       h->stream, h->dStream, (int)total, h->hStreamDev);
    RS_HIP(hipGetLastError());
    RS_HIP(hipStreamSynchronize(h->stream));
    h->streamClean = true;
    if (!allplanes) h->timedScan = false;  // several scans: no single duration
    else if (h->timedScan) RS_HIP(hipEventElapsedTime(&h->lastMs, h->ev0, h->ev1));
    for (size_t i = 0; i < total; ++i) {
        const unsigned long long k = h->hStream[i];
        if (best_index) best_index[i] = k == NO_KEY ? -1 : (int64_t)(k & 0xFFFFFFFFull);
        if (best_score) best_score[i] = k == NO_KEY ? UINT64_MAX : (k >> 32);
    }
    return RS_OK;
}

int vt_match_impl(rs_vt* h, int nq, const uint8_t* queries, int mode, uint64_t* best_score,
                  int64_t* best_index, uint8_t* is_new, bool frames = false) {
    RS_CHECK(mode == RS_VT_FROZEN || mode == RS_VT_SEQUENTIAL, RS_ERR_ARG, "unknown mode %d", mode);
    RS_TRY(vt_scan_local_impl(h, nq, queries, frames, h->nranks == 1));
    if (nq == 0) return RS_OK;
    RS_TRY(vt_fetch_keys(h, nq, true));
    return vt_resolve_impl(h, nq, h->hBest, mode, best_score, best_index, is_new);
}

}  // namespace

extern "C" {

int rs_vt_create(int H, int W, int max_offset, uint64_t thr, int64_t capacity, int device,
                 rs_vt** out) {
    rs::clear_error();
    RS_CHECK(out, RS_ERR_ARG, "null output handle pointer");
    *out = nullptr;
    RS_CHECK(H > 0 && W > 0 && H <= 4096 && W <= 4096, RS_ERR_ARG, "bad template shape (%d, %d)", H, W);
    RS_CHECK(max_offset >= 1 && max_offset <= 64, RS_ERR_ARG, "max_offset %d outside [1, 64]", max_offset);
    RS_CHECK(capacity >= 0, RS_ERR_ARG, "negative capacity");
    // max score H*W*255 must fit the 32-bit half of the packed key
    RS_CHECK((uint64_t)H * W * 255u < 0xFFFFFFFFull, RS_ERR_ARG, "template too large");
    int ndev = 0;
    RS_HIP(hipGetDeviceCount(&ndev));
    RS_CHECK(device >= 0 && device < ndev, RS_ERR_ARG, "device %d not in [0, %d)", device, ndev);
    RS_HIP(hipSetDevice(device));
    rs_vt* h = new rs_vt();
    h->H = H; h->W = W; h->M = max_offset; h->thr = (double)thr; h->device = device;
    h->WD = (W + 3) / 4;
    h->HQ = (H + 3) / 4;
    h->planar = W == 8 * PL_CG && (H == 64 || H == 32) && max_offset == FAST_M;
    if (const char* e = std::getenv("RS_VT_SCAN")) {
        // A/B switch: "carry" forces the byte-SWAR carry-count scan; "plane" (or
        // unset) keeps the default
        if (std::strcmp(e, "carry") == 0) h->planar = false;
        else if (std::strcmp(e, "plane") != 0 && e[0] != 0) {
            rs::set_error("RS_VT_SCAN='%s': expected plane or carry", e);
            delete h;
            return RS_ERR_ARG;
        }
    }
    if (h->planar) {
        // resident blocks per CU: the occupancy API, capped by the kernel's own VGPR and
        // LDS arithmetic (the API has read one block high on gfx950 for some SGPR counts)
        int per_cu = 0, cus = 0;
        hipFuncAttributes fa{};
        const void* fn = h->H == 64 ? reinterpret_cast<const void*>(vt_scan_plane_kernel<64, false>)
                                    : reinterpret_cast<const void*>(vt_scan_plane_kernel<32, false>);
        hipError_t oe = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64 * PL_CG * PL_SPLIT, 0);
        if (oe == hipSuccess) oe = hipFuncGetAttributes(&fa, fn);
        if (oe == hipSuccess) oe = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
        if (oe != hipSuccess) {
            rs::set_error("occupancy query failed: %s", hipGetErrorString(oe));
            delete h;
            return RS_ERR_HIP;
        }
        const int vg = std::max(8, (fa.numRegs + 7) / 8 * 8);
        const int by_vgpr = (512 / vg) * 4 / (PL_CG * PL_SPLIT);  // waves/SIMD x 4 SIMDs / waves/block
        const int by_lds = fa.sharedSizeBytes > 0 ? (int)(160 * 1024 / fa.sharedSizeBytes) : per_cu;
        const int api = per_cu;
        per_cu = std::max(1, std::min({api, by_vgpr, by_lds}));
        h->planeSlots = std::max(1, per_cu * cus);
    }
    hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreate(&h->ev0);
    if (e == hipSuccess) e = hipEventCreate(&h->ev1);
    if (e != hipSuccess) {
        rs::set_error("stream/event creation failed: %s", hipGetErrorString(e));
        rs_vt_destroy(h);
        return RS_ERR_HIP;
    }
    int s = vt_grow_lib(h, capacity > 0 ? capacity : 64);
    if (s == RS_OK) s = vt_grow_queries(h, 64);
    if (s == RS_OK) s = vt_grow_index(h, 64);
    if (s != RS_OK) {
        rs_vt_destroy(h);
        return s;
    }
    *out = h;
    return RS_OK;
}

int rs_vt_destroy(rs_vt* h) {
    if (!h) return RS_OK;
    (void)hipSetDevice(h->device);
    // the handle's last queued work: a fault or launch error the early-returning calls
    // left on a stream is reported here instead of being dropped
    hipError_t se = hipSuccess;
    for (hipStream_t st : {h->stream, h->cstream, h->ustream})
        if (st) {
            const hipError_t e = hipStreamSynchronize(st);
            if (se == hipSuccess) se = e;
        }
    if (h->comm) (void)ncclCommDestroy(h->comm);
    for (void* p : {(void*)h->dLib, (void*)h->dQraw, (void*)h->dQf, (void*)h->dQsum, (void*)h->dBest,
                    (void*)h->dSrc, (void*)h->dDst, (void*)h->dCand, (void*)h->dMat, (void*)h->dLibP,
                    (void*)h->dLibTs, (void*)h->dCandP, (void*)h->dCandTs, (void*)h->dQp,
                    (void*)h->dQsumRaw, (void*)h->dCtr, (void*)h->dDone, (void*)h->dPix, (void*)h->dFrames})
        if (p) (void)hipFree(p);
    if (h->hStream) (void)hipHostFree(h->hStream);
    if (h->dStream) (void)hipFree(h->dStream);
    if (h->dQpStream) (void)hipFree(h->dQpStream);
    if (h->dQsumStream) (void)hipFree(h->dQsumStream);
    for (void* p : {(void*)h->hQraw, (void*)h->hBest, (void*)h->hSrc, (void*)h->hDst, (void*)h->hMat,
                    (void*)h->hFrames})
        if (p) (void)hipHostFree(p);
    if (h->ev0) (void)hipEventDestroy(h->ev0);
    if (h->ev1) (void)hipEventDestroy(h->ev1);
    if (h->evScan) (void)hipEventDestroy(h->evScan);
    if (h->evComm) (void)hipEventDestroy(h->evComm);
    if (h->cstream) (void)hipStreamDestroy(h->cstream);
    for (int i = 0; i < 2; ++i) {
        if (h->dUp[i]) (void)hipFree(h->dUp[i]);
        if (h->evUp[i]) (void)hipEventDestroy(h->evUp[i]);
        if (h->evUsed[i]) (void)hipEventDestroy(h->evUsed[i]);
    }
    if (h->ustream) (void)hipStreamDestroy(h->ustream);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    RS_CHECK(se == hipSuccess, RS_ERR_HIP, "work queued before rs_vt_destroy failed: %s", hipGetErrorString(se));
    return RS_OK;
}

int rs_vt_count(const rs_vt* h, int64_t* count) {
    RS_CHECK(h && count, RS_ERR_ARG, "null argument");
    *count = h->count;
    return RS_OK;
}

int rs_vt_add(rs_vt* h, int n, const uint8_t* templates, int64_t* first_index) {
    rs::clear_error();
    RS_CHECK(h, RS_ERR_STATE, "null view-template handle");
    RS_CHECK(n >= 0 && (n == 0 || templates), RS_ERR_ARG, "bad template batch");
    RS_HIP(hipSetDevice(h->device));
    if (first_index) *first_index = h->count;
    if (n == 0) return RS_OK;
    RS_TRY(vt_grow_queries(h, n));
    const size_t qb = (size_t)h->H * h->W * n;
    // A pageable array is uploaded by HIP, which returns once the bytes are staged in its
    // own buffers.  Pinned or registered host memory, or device memory, is read by the
    // DMA engine while the copy runs, after this call would return: those sources are
    // waited for below, so in every case the caller may reuse or free its array at once.
    hipPointerAttribute_t attr{};
    const bool direct_dma = hipPointerGetAttributes(&attr, templates) == hipSuccess &&
                            (attr.type == hipMemoryTypeHost || attr.type == hipMemoryTypeDevice ||
                             attr.type == hipMemoryTypeManaged);
    (void)hipGetLastError();  // a pageable pointer is not an error
    RS_HIP(hipMemcpyAsync(h->dQraw, templates, qb,
                          attr.type == hipMemoryTypeDevice && direct_dma ? hipMemcpyDeviceToDevice
                                                                         : hipMemcpyHostToDevice,
                          h->stream));
    h->stagedQ = 0;  // the staging buffer now holds templates, not a query batch
    std::vector<std::pair<int, int64_t>> news;
    news.reserve(n);
    for (int i = 0; i < n; ++i) news.emplace_back(i, h->count + i);
    RS_TRY(vt_append_staged(h, news));   // (its copies guarded by vt_staging_idle, not a sync)
    if (direct_dma) RS_HIP(hipStreamSynchronize(h->stream));
    return RS_OK;
}

int rs_vt_read(rs_vt* h, int64_t index, uint8_t* out) {
    rs::clear_error();
    RS_CHECK(h && out, RS_ERR_ARG, "null argument");
    RS_CHECK(index >= 0 && index < h->count, RS_ERR_ARG, "template index %lld outside [0, %lld)",
             (long long)index, (long long)h->count);
    RS_CHECK(index % h->nranks == h->rank, RS_ERR_ARG, "template %lld lives on rank %lld",
             (long long)index, (long long)(index % h->nranks));
    RS_HIP(hipSetDevice(h->device));
    const int64_t slot = index / h->nranks;
    const int64_t tb = slot >> 6, tl = slot & 63;
    std::vector<uint4> chunks((size_t)h->WD * h->HQ);
    for (int c = 0; c < h->WD; ++c)
        for (int q = 0; q < h->HQ; ++q)
            RS_HIP(hipMemcpyAsync(&chunks[(size_t)c * h->HQ + q],
                                  h->dLib + ((tb * h->WD + c) * h->HQ + q) * 64 + tl, sizeof(uint4),
                                  hipMemcpyDeviceToHost, h->stream));
    RS_HIP(hipStreamSynchronize(h->stream));
    for (int r = 0; r < h->H; ++r)
        for (int col = 0; col < h->W; ++col) {
            const uint4& ch = chunks[(size_t)(col / 4) * h->HQ + r / 4];
            const uint32_t w[4] = {ch.x, ch.y, ch.z, ch.w};
            out[(size_t)r * h->W + col] = (uint8_t)(w[r & 3] >> (8 * (col & 3)));
        }
    return RS_OK;
}

int rs_vt_match_batch(rs_vt* h, int nq, const uint8_t* queries, int mode, uint64_t* best_score,
                      int64_t* best_index, uint8_t* is_new) {
    rs::clear_error();
    return vt_match_impl(h, nq, queries, mode, best_score, best_index, is_new);
}

int rs_vt_match_stream(rs_vt* h, int nb, int nq, const uint8_t* queries, uint64_t* best_score,
                       int64_t* best_index) {
    rs::clear_error();
    return vt_match_stream_impl(h, nb, nq, queries, best_score, best_index);
}

int rs_vt_match(rs_vt* h, const uint8_t* query, uint64_t* best_score, int64_t* best_index,
                int* is_new) {
    rs::clear_error();
    uint8_t nw = 0;
    const int s = vt_match_impl(h, 1, query, RS_VT_SEQUENTIAL, best_score, best_index, &nw);
    if (is_new) *is_new = nw;
    return s;
}

int rs_vt_set_subsample(rs_vt* h, int64_t frame_bytes, const int32_t* pixels) {
    rs::clear_error();
    RS_CHECK(h && pixels, RS_ERR_ARG, "null argument");
    RS_CHECK(frame_bytes > 0 && frame_bytes <= INT32_MAX, RS_ERR_ARG, "bad frame size %lld",
             (long long)frame_bytes);
    const int npix = h->H * h->W;
    for (int i = 0; i < npix; ++i)
        RS_CHECK(pixels[i] >= 0 && pixels[i] < frame_bytes, RS_ERR_ARG,
                 "pixel offset %d of entry %d outside the %lld-byte frame", pixels[i], i,
                 (long long)frame_bytes);
    RS_HIP(hipSetDevice(h->device));
    if (!h->dPix) RS_HIP(hipMalloc(&h->dPix, sizeof(int32_t) * npix));
    RS_HIP(hipMemcpyAsync(h->dPix, pixels, sizeof(int32_t) * npix, hipMemcpyHostToDevice, h->stream));
    RS_HIP(hipStreamSynchronize(h->stream));
    if (frame_bytes != h->frameBytes) {  // staging buffers are sized per frame
        if (h->dFrames) RS_HIP(hipFree(h->dFrames));
        if (h->hFrames) RS_HIP(hipHostFree(h->hFrames));
        h->dFrames = nullptr;
        h->hFrames = nullptr;
        h->frameCap = 0;
    }
    h->frameBytes = frame_bytes;
    return RS_OK;
}

int rs_vt_match_frames(rs_vt* h, int nf, const uint8_t* frames, int mode, uint64_t* best_score,
                       int64_t* best_index, uint8_t* is_new) {
    rs::clear_error();
    RS_CHECK(h, RS_ERR_STATE, "null view-template handle");
    return vt_match_impl(h, nf, frames, mode, best_score, best_index, is_new, true);
}

int rs_vt_scan_local(rs_vt* h, int nq, const uint8_t* queries, uint64_t* local_keys) {
    rs::clear_error();
    RS_TRY(vt_scan_local_impl(h, nq, queries));
    if (nq == 0) return RS_OK;
    RS_TRY(vt_fetch_keys(h, nq, false));
    if (local_keys) std::memcpy(local_keys, h->hBest, sizeof(uint64_t) * nq);
    return RS_OK;
}

int rs_vt_resolve(rs_vt* h, int nq, const uint64_t* global_keys, int mode, uint64_t* best_score,
                  int64_t* best_index, uint8_t* is_new) {
    rs::clear_error();
    static_assert(sizeof(uint64_t) == sizeof(unsigned long long), "key width");
    return vt_resolve_impl(h, nq, reinterpret_cast<const unsigned long long*>(global_keys), mode,
                           best_score, best_index, is_new);
}

int rs_vt_set_shard(rs_vt* h, int rank, int nranks) {
    rs::clear_error();
    RS_CHECK(h, RS_ERR_STATE, "null view-template handle");
    RS_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, RS_ERR_ARG, "bad rank %d of %d", rank, nranks);
    RS_CHECK(h->count == 0 && h->comm == nullptr, RS_ERR_STATE,
             "set the shard before adding templates, once");
    h->rank = rank;
    h->nranks = nranks;
    return RS_OK;
}

int rs_vt_rank(const rs_vt* h, int* rank, int* nranks) {
    RS_CHECK(h, RS_ERR_STATE, "null view-template handle");
    if (rank) *rank = h->rank;
    if (nranks) *nranks = h->nranks;
    return RS_OK;
}

int rs_vt_scores(rs_vt* h, int nq, const uint8_t* queries, int64_t t0, int64_t nt,
                 uint64_t* scores) {
    rs::clear_error();
    RS_CHECK(h, RS_ERR_STATE, "null view-template handle");
    RS_CHECK(h->nranks == 1, RS_ERR_STATE, "rs_vt_scores needs an unsharded library");
    RS_CHECK(nq >= 0 && t0 >= 0 && nt >= 0 && t0 + nt <= h->count, RS_ERR_ARG,
             "template range [%lld, %lld) outside [0, %lld)", (long long)t0,
             (long long)(t0 + nt), (long long)h->count);
    if (nq == 0 || nt == 0) return RS_OK;
    RS_CHECK(queries && scores, RS_ERR_ARG, "null argument");
    RS_HIP(hipSetDevice(h->device));
    RS_TRY(vt_stage_queries(h, nq, queries));
    h->stagedQ = 0;  // the staging buffer no longer holds the last match batch
    // only the 64-slot blocks that hold [t0, t0 + nt) are scanned
    const int64_t tb0 = t0 / 64, lo = t0 - tb0 * 64, span = lo + nt;
    const int64_t ld = (int64_t)rs::round_up((size_t)span, 64);
    RS_TRY(vt_grow_matrix(h, (size_t)ld * nq));
    ScanOut mo{nullptr, h->dMat, ld};
    RS_HIP(hipEventRecord(h->ev0, h->stream));
    RS_TRY(vt_launch_scan<true>(h, false, span, nq, mo, 0, 1, tb0));
    RS_HIP(hipEventRecord(h->ev1, h->stream));
    RS_HIP(hipMemcpy2DAsync(h->hMat, sizeof(uint32_t) * nt, h->dMat + lo, sizeof(uint32_t) * ld,
                            sizeof(uint32_t) * nt, nq, hipMemcpyDeviceToHost, h->stream));
    RS_HIP(hipStreamSynchronize(h->stream));
    RS_HIP(hipEventElapsedTime(&h->lastMs, h->ev0, h->ev1));
    h->timedScan = true;
    for (size_t i = 0; i < (size_t)nq * nt; ++i) scores[i] = h->hMat[i];
    return RS_OK;
}

int rs_vt_set_threshold(rs_vt* h, double threshold) {
    rs::clear_error();
    RS_CHECK(h, RS_ERR_STATE, "null view-template handle");
    h->thr = threshold;
    return RS_OK;
}

const char* rs_vt_scan_form(const rs_vt* h) {
    if (!h) return nullptr;
    if (h->planar) return "plane";
    if (h->M != FAST_M || (h->H != 64 && h->H != 32)) return "generic";
    return "carry";
}

int rs_vt_last_ms(rs_vt* h, double* ms) {
    RS_CHECK(h && ms, RS_ERR_ARG, "null argument");
    *ms = h->timedScan ? h->lastMs : -1.0;
    return RS_OK;
}

int rs_vt_set_timing(rs_vt* h, int enable) {
    rs::clear_error();
    RS_CHECK(h, RS_ERR_STATE, "null view-template handle");
    h->timing = enable != 0;
    return RS_OK;
}

int rs_comm_unique_id(uint8_t id[RS_UNIQUE_ID_BYTES]) {
    rs::clear_error();
    RS_CHECK(id, RS_ERR_ARG, "null id buffer");
    static_assert(sizeof(ncclUniqueId) == RS_UNIQUE_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    ncclResult_t r = ncclGetUniqueId(&u);
    RS_CHECK(r == ncclSuccess, RS_ERR_RCCL, "ncclGetUniqueId failed: %s", ncclGetErrorString(r));
    std::memcpy(id, &u, sizeof(u));
    return RS_OK;
}

int rs_vt_attach_comm(rs_vt* h, int rank, int nranks, const uint8_t id[RS_UNIQUE_ID_BYTES]) {
    rs::clear_error();
    RS_CHECK(h && id, RS_ERR_ARG, "null argument");
    RS_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, RS_ERR_ARG, "bad rank %d of %d", rank, nranks);
    RS_CHECK(h->count == 0 && h->comm == nullptr, RS_ERR_STATE,
             "attach the communicator before adding templates, once");
    RS_HIP(hipSetDevice(h->device));
    {  // also for nranks == 1: rs_vt_match_stream then runs its collective path
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        ncclComm_t comm = nullptr;  // kept only on success: destroy never sees a failed init
        ncclResult_t r = ncclCommInitRank(&comm, nranks, u, rank);
        RS_CHECK(r == ncclSuccess, RS_ERR_RCCL, "ncclCommInitRank failed: %s", ncclGetErrorString(r));
        h->comm = comm;
    }
    h->rank = rank;
    h->nranks = nranks;
    return RS_OK;
}

// host side of the float path: numpy's pairwise program for n elements
static void sad_program(int start, int n, std::vector<int2>& prog) {
    if (n <= 128) {
        prog.push_back(make_int2(start, n));
        return;
    }
    int n2 = n / 2;
    n2 -= n2 % 8;
    sad_program(start, n2, prog);
    sad_program(start + n2, n - n2, prog);
    prog.push_back(make_int2(-1, 0));
}

int rs_sad_scores(int device, int dtype, int H, int W, int max_offset, int64_t nt,
                  const void* templates, int nq, const void* queries, void* scores) {
    rs::clear_error();
    RS_CHECK(dtype == RS_DT_F32 || dtype == RS_DT_F64, RS_ERR_TYPE, "dtype %d is not F32/F64", dtype);
    RS_CHECK(H > 0 && W > 0 && max_offset >= 1 && max_offset <= 16 && H > 2 * max_offset,
             RS_ERR_ARG, "bad shape (%d, %d) for max_offset %d", H, W, max_offset);
    RS_CHECK((int64_t)H * W < (1ll << 31), RS_ERR_ARG, "template too large");
    RS_CHECK(nt >= 0 && nq >= 0, RS_ERR_ARG, "negative count");
    if (nt == 0 || nq == 0) return RS_OK;
    RS_CHECK(templates && queries && scores, RS_ERR_ARG, "null argument");
    int ndev = 0;
    RS_HIP(hipGetDeviceCount(&ndev));
    RS_CHECK(device >= 0 && device < ndev, RS_ERR_ARG, "device %d not in [0, %d)", device, ndev);
    RS_HIP(hipSetDevice(device));
    std::vector<int2> prog;
    sad_program(0, (H - 2 * max_offset) * W, prog);
    const size_t es = dtype == RS_DT_F32 ? 4 : 8;
    const size_t tb = (size_t)nt * H * W * es, qb = (size_t)nq * H * W * es, ob = (size_t)nt * nq * es;
    void *dT = nullptr, *dQ = nullptr, *dO = nullptr, *dP = nullptr;
    hipStream_t st = nullptr;
    int rc = RS_OK;
    auto run = [&]() -> int {
        RS_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        RS_HIP(hipMalloc(&dT, tb));
        RS_HIP(hipMalloc(&dQ, qb));
        RS_HIP(hipMalloc(&dO, ob));
        RS_HIP(hipMalloc(&dP, sizeof(int2) * prog.size()));
        RS_HIP(hipMemcpyAsync(dT, templates, tb, hipMemcpyHostToDevice, st));
        RS_HIP(hipMemcpyAsync(dQ, queries, qb, hipMemcpyHostToDevice, st));
        RS_HIP(hipMemcpyAsync(dP, prog.data(), sizeof(int2) * prog.size(), hipMemcpyHostToDevice, st));
        const int64_t pairs = nt * (int64_t)nq;
        RS_CHECK((pairs + 3) / 4 < (1ll << 31), RS_ERR_ARG, "too many pairs");
        const dim3 grid((unsigned)((pairs + 3) / 4));
        if (dtype == RS_DT_F32)
            hipLaunchKernelGGL(vt_sad_float_kernel<float>, grid, dim3(64), 0, st,
                               static_cast<const float*>(dT), nt, static_cast<const float*>(dQ), nq,
                               H, W, max_offset, static_cast<const int2*>(dP), (int)prog.size(),
                               static_cast<float*>(dO));
        else
            hipLaunchKernelGGL(vt_sad_float_kernel<double>, grid, dim3(64), 0, st,
                               static_cast<const double*>(dT), nt, static_cast<const double*>(dQ),
                               nq, H, W, max_offset, static_cast<const int2*>(dP), (int)prog.size(),
                               static_cast<double*>(dO));
        RS_HIP(hipGetLastError());
        RS_HIP(hipMemcpyAsync(scores, dO, ob, hipMemcpyDeviceToHost, st));
        RS_HIP(hipStreamSynchronize(st));
        return RS_OK;
    };
    rc = run();
    for (void* p : {dT, dQ, dO, dP})
        if (p) (void)hipFree(p);
    if (st) (void)hipStreamDestroy(st);
    return rc;
}

}  // extern "C"
