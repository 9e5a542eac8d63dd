// A C loop over rs_pc_update_odom (no Python, no ctypes): the per-call cost of the
// library alone, for tools/pc_call_anatomy.py.  Built on the fly:
//   g++ -O2 -shared -fPIC tools/pc_call_loop.cpp -Iinclude -Lpyratslam_amd -lratslam_hip -o /tmp/...
#include <chrono>
#include <cstdint>

#include "ratslam_abi.h"

extern "C" int pc_call_loop(rs_pc* h, int n, const double* odom, double* us_per_call) {
    int32_t out[3];
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) {
        const int st = rs_pc_update_odom(h, odom[2 * i], odom[2 * i + 1], out);
        if (st != 0) return st;
    }
    const auto t1 = std::chrono::steady_clock::now();
    *us_per_call = std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
    return 0;
}
