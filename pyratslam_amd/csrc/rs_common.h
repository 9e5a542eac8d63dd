// Shared helpers of libratslam_hip: error state and HIP call checking.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "ratslam_abi.h"

namespace rs {

void set_error(const char* fmt, ...);
void clear_error();

// Return-on-failure wrappers for the extern "C" entry points.
#define RS_HIP(call)                                                              \
    do {                                                                          \
        hipError_t e_ = (call);                                                   \
        if (e_ != hipSuccess) {                                                   \
            ::rs::set_error("%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), \
                            __FILE__, __LINE__);                                  \
            return RS_ERR_HIP;                                                    \
        }                                                                         \
    } while (0)

#define RS_CHECK(cond, code, ...)            \
    do {                                     \
        if (!(cond)) {                       \
            ::rs::set_error(__VA_ARGS__);    \
            return (code);                   \
        }                                    \
    } while (0)

#define RS_TRY(expr)                 \
    do {                             \
        int s_ = (expr);             \
        if (s_ != RS_OK) return s_;  \
    } while (0)

// Positive modulo for (possibly negative) halo coordinates.
__host__ __device__ inline int wrapi(int v, int n) {
    int r = v % n;
    return r < 0 ? r + n : r;
}

inline size_t round_up(size_t v, size_t m) { return (v + m - 1) / m * m; }

}  // namespace rs
