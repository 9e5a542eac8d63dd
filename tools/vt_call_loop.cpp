// A C loop over rs_vt_match_stream (no Python, no ctypes): the per-call cost of the
// library alone around its fused scan, for tools/vt_call_anatomy.py.  Built on the fly:
//   g++ -O2 -shared -fPIC tools/vt_call_loop.cpp -Iinclude -Lpyratslam_amd -lratslam_hip -o /tmp/...
#include <chrono>
#include <cstdint>

#include "ratslam_abi.h"

extern "C" int vt_call_loop(rs_vt* h, int calls, int nb, int nq, const uint8_t* queries, uint64_t* score,
                            int64_t* index, double* us_per_call) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < calls; ++i) {
        const int st = rs_vt_match_stream(h, nb, nq, queries, score, index);
        if (st != 0) return st;
    }
    const auto t1 = std::chrono::steady_clock::now();
    *us_per_call = std::chrono::duration<double, std::micro>(t1 - t0).count() / calls;
    return 0;
}
