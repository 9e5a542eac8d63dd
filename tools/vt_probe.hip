// Diagnostic probe for the bit-plane template scan (not part of the library).
// Builds view_templates.hip with its VT_STAMP hook defined so every wave of vt_scan_plane_kernel
// stamps its start and end (realtime 100 MHz, shader clock, hw ids), then
// reports the kernel span, wave durations, waves per SIMD and the clock.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Ipyratslam_amd/csrc \
//         tools/vt_probe.hip pyratslam_amd/csrc/rs_common.cpp -lrccl -o tools/vt_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <random>
#include <vector>

// the library's per-wave stamp hook (view_templates.hip leaves it empty)
__device__ unsigned long long* vt_dbg;
#define VT_STAMP(slot)                                                                     \
    do {                                                                                   \
        if ((threadIdx.x & 63) == 0) {                                                     \
            unsigned hw_, xcc_;                                                            \
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_));              \
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_));            \
            unsigned long long* d_ = vt_dbg + ((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 6; \
            d_[(slot) * 3 + 0] = __builtin_amdgcn_s_memrealtime();                         \
            d_[(slot) * 3 + 1] = __builtin_amdgcn_s_memtime();                             \
            d_[(slot) * 3 + 2] = ((unsigned long long)xcc_ << 32) | hw_;                   \
        }                                                                                  \
    } while (0)
#include "view_templates.hip"

int main(int argc, char** argv) {
    const int T = argc > 1 ? atoi(argv[1]) : 1000, Q = argc > 2 ? atoi(argv[2]) : 1024;
    const int H = 64, W = 32;
    rs_vt* h = nullptr;
    if (rs_vt_create(H, W, 8, 45000, T, 0, &h) != RS_OK) {
        fprintf(stderr, "create: %s\n", rs_last_error());
        return 1;
    }
    std::mt19937 rng(1);
    std::vector<uint8_t> lib((size_t)T * H * W), qs((size_t)Q * H * W);
    for (auto& b : lib) b = (uint8_t)rng();
    for (auto& b : qs) b = (uint8_t)rng();
    if (rs_vt_add(h, T, lib.data(), nullptr) != RS_OK) return 1;
    const size_t nslots = 1 << 16;
    unsigned long long* dbg;
    if (hipMalloc(&dbg, nslots * 6 * 8) != hipSuccess) return 1;
    hipMemset(dbg, 0, nslots * 6 * 8);
    hipMemcpyToSymbol(HIP_SYMBOL(vt_dbg), &dbg, sizeof(dbg));
    std::vector<uint64_t> sc(Q);
    std::vector<int64_t> ix(Q);
    std::vector<uint8_t> nw(Q);
    double ms = 0;
    for (int rep = 0; rep < 5; ++rep) {
        if (rs_vt_match_batch(h, Q, rep ? nullptr : qs.data(), RS_VT_FROZEN, sc.data(), ix.data(),
                              nw.data()) != RS_OK) {
            fprintf(stderr, "match: %s\n", rs_last_error());
            return 1;
        }
        rs_vt_last_ms(h, &ms);
    }
    std::vector<unsigned long long> d(nslots * 6);
    hipMemcpy(d.data(), dbg, d.size() * 8, hipMemcpyDeviceToHost);
    unsigned long long t0 = ~0ull, t1 = 0;
    std::vector<double> dur, clk;
    std::map<unsigned long long, std::vector<std::pair<unsigned long long, unsigned long long>>> simd;
    int nw_ = 0;
    for (size_t i = 0; i < nslots; ++i) {
        const unsigned long long* e = &d[i * 6];
        if (!e[0] || !e[3]) continue;
        ++nw_;
        t0 = std::min(t0, e[0]);
        t1 = std::max(t1, e[3]);
        dur.push_back((e[3] - e[0]) * 0.01);  // us
        clk.push_back((double)(e[4] - e[1]) / ((e[3] - e[0]) * 10.0));  // GHz
        const unsigned hw = (unsigned)e[2], xcc = (unsigned)(e[2] >> 32);
        const unsigned long long key = ((unsigned long long)xcc << 16) | ((hw >> 13) & 7) << 12 |
                                       ((hw >> 12) & 1) << 11 | ((hw >> 8) & 15) << 4 | ((hw >> 4) & 3);
        simd[key].push_back({e[0], e[3]});
    }
    std::sort(dur.begin(), dur.end());
    std::sort(clk.begin(), clk.end());
    printf("waves %d  kernel (event) %.1f us  stamped span %.1f us\n", nw_, ms * 1e3, (t1 - t0) * 0.01);
    if (dur.empty()) return 0;
    printf("wave duration us: min %.1f  p10 %.1f  median %.1f  p90 %.1f  max %.1f\n", dur.front(),
           dur[dur.size() / 10], dur[dur.size() / 2], dur[dur.size() * 9 / 10], dur.back());
    printf("shader clock GHz (per wave): median %.2f\n", clk[clk.size() / 2]);
    std::map<int, int> hist;
    double busy = 0;
    for (auto& kv : simd) {
        hist[(int)kv.second.size()]++;
        // time-averaged concurrent waves on this SIMD over the stamped span
        for (auto& p : kv.second) busy += (double)(p.second - p.first);
    }
    printf("SIMDs seen %zu; waves per SIMD histogram:", simd.size());
    for (auto& kv : hist) printf("  %d:%d", kv.first, kv.second);
    printf("\navg concurrent waves per SIMD seen (over span) %.2f\n", busy / simd.size() / (double)(t1 - t0));
    // start-time spread
    std::vector<double> st;
    for (size_t i = 0; i < nslots; ++i)
        if (d[i * 6] && d[i * 6 + 3]) st.push_back((d[i * 6] - t0) * 0.01);
    std::sort(st.begin(), st.end());
    printf("start offset us: median %.2f  p90 %.2f  max %.2f\n", st[st.size() / 2], st[st.size() * 9 / 10], st.back());
    rs_vt_destroy(h);
    return 0;
}
