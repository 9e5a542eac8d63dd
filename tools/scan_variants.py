#!/usr/bin/env python3
"""The round-6 plane-scan variants (profiles/r6_scan/): edited copies of
view_templates.hip in abtmp/ -- two query rows' borrow chains interleaved (s*r2), and
12- / 16-wave blocks of 3 / 4 query-row ranges (s3*, s4*).  Run from the repository
root; build each with tools/build_vt_edit.sh's hipcc lines (no edits) and time them
with tools/stream_ab.py, which checks every build's keys against the first."""
import sys
src = open('pyratslam_amd/csrc/view_templates.hip').read()
row2 = '''
// Two query start rows S and S + 1 against the units each meets, their borrow chains
// interleaved (6 - 8 independent chains; distinct accumulators: 4J - S != 4J' - S - 1)
template <int H, int HALF, int S>
__device__ __forceinline__ void plane_row2(const uint32_t (&P)[PlaneRange<H, HALF>::NUH][8],
                                           const uint32_t* q0, const uint32_t* q1, uint32_t (&acc)[2 * FAST_M - 1]) {
    using R = PlaneRange<H, HALF>;
    constexpr int M = FAST_M, JA0 = R::ja(S), JB0 = R::jb(S), N0 = JB0 - JA0 + 1;
    constexpr int JA1 = R::ja(S + 1), JB1 = R::jb(S + 1), N1 = JB1 - JA1 + 1;
    uint32_t b0[N0], b1[N1];
#pragma unroll
    for (int j = 0; j < N0; ++j) b0[j] = __builtin_amdgcn_bitop3_b32(P[JA0 - R::JLO + j][0], q0[0], 0u, 0x8E);
#pragma unroll
    for (int j = 0; j < N1; ++j) b1[j] = __builtin_amdgcn_bitop3_b32(P[JA1 - R::JLO + j][0], q1[0], 0u, 0x8E);
#pragma unroll
    for (int k = 1; k < 8; ++k) {
#pragma unroll
        for (int j = 0; j < N0; ++j) b0[j] = __builtin_amdgcn_bitop3_b32(P[JA0 - R::JLO + j][k], q0[k], b0[j], 0x8E);
#pragma unroll
        for (int j = 0; j < N1; ++j) b1[j] = __builtin_amdgcn_bitop3_b32(P[JA1 - R::JLO + j][k], q1[k], b1[j], 0x8E);
    }
#pragma unroll
    for (int j = 0; j < N0; ++j) {
        uint32_t& a = acc[4 * (JA0 + j) - S + M - 1];
        asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(a) : "v"(b0[j]), "v"(a));
    }
#pragma unroll
    for (int j = 0; j < N1; ++j) {
        uint32_t& a = acc[4 * (JA1 + j) - (S + 1) + M - 1];
        asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(a) : "v"(b1[j]), "v"(a));
    }
}
'''
old_rows = '''    const uint4 lo = *reinterpret_cast<const uint4*>(sq + (S - R::S0) * 8);
    const uint4 hi = *reinterpret_cast<const uint4*>(sq + (S - R::S0) * 8 + 4);
    const uint32_t q[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    plane_row<H, HALF, S>(P, q, acc);
    if constexpr (S < R::SB) plane_rows<H, HALF, S + 1>(P, sq, acc);'''
new_rows = '''    const uint4 lo = *reinterpret_cast<const uint4*>(sq + (S - R::S0) * 8);
    const uint4 hi = *reinterpret_cast<const uint4*>(sq + (S - R::S0) * 8 + 4);
    const uint32_t q[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    if constexpr (S < R::SB) {
        const uint4 lo1 = *reinterpret_cast<const uint4*>(sq + (S + 1 - R::S0) * 8);
        const uint4 hi1 = *reinterpret_cast<const uint4*>(sq + (S + 1 - R::S0) * 8 + 4);
        const uint32_t q1[8] = {lo1.x, lo1.y, lo1.z, lo1.w, hi1.x, hi1.y, hi1.z, hi1.w};
        plane_row2<H, HALF, S>(P, q, q1, acc);
        if constexpr (S + 1 < R::SB) plane_rows<H, HALF, S + 2>(P, sq, acc);
    } else {
        plane_row<H, HALF, S>(P, q, acc);
    }'''
def variant(name, split, row2flag, wpe):
    s = src
    assert old_rows in s
    if row2flag:
        s = s.replace("// Query planes are staged per batch in LDS and read as wave-uniform", row2 + "\n// Query planes are staged per batch in LDS and read as wave-uniform", 1)
        s = s.replace(old_rows, new_rows)
    if split != 2:
        s = s.replace("constexpr int PL_SPLIT = 2;", "constexpr int PL_SPLIT = %d;" % split)
        s = s.replace('    static_assert(PL_SPLIT == 2, "two row ranges");\n', '')
        old = '''    if (half == 0)
        plane_wave<H, 0, MATRIX>(planes, tb, count, qp4, qsum, nq, ctr, G, g, out, rank, nranks,
                                 wave, cg, lane, failed);
    else
        plane_wave<H, 1, MATRIX>(planes, tb, count, qp4, qsum, nq, ctr, G, g, out, rank, nranks,
                                 wave, cg, lane, failed);'''
        assert old in s
        new = '''    if (half == 0)
        plane_wave<H, 0, MATRIX>(planes, tb, count, qp4, qsum, nq, ctr, G, g, out, rank, nranks,
                                 wave, cg, lane, failed);
    else if (half == 1)
        plane_wave<H, 1, MATRIX>(planes, tb, count, qp4, qsum, nq, ctr, G, g, out, rank, nranks,
                                 wave, cg, lane, failed);
    else if (half == 2)
        plane_wave<H, 2, MATRIX>(planes, tb, count, qp4, qsum, nq, ctr, G, g, out, rank, nranks,
                                 wave, cg, lane, failed);
    else if constexpr (PL_SPLIT > 3)
        plane_wave<H, 3, MATRIX>(planes, tb, count, qp4, qsum, nq, ctr, G, g, out, rank, nranks,
                                 wave, cg, lane, failed);'''
        s = s.replace(old, new)
    s = s.replace("__attribute__((amdgpu_waves_per_eu(4, 4)))", "__attribute__((amdgpu_waves_per_eu(%d, %d)))" % (wpe, wpe))
    open('abtmp/%s_vt.hip' % name, 'w').write(s)
for name, split, r2, wpe in [('s2r2', 2, True, 4), ('s3r1', 3, False, 3), ('s3r2', 3, True, 3), ('s4r1', 4, False, 4), ('s4r2', 4, True, 4)]:
    variant(name, split, r2, wpe)
print('ok')
