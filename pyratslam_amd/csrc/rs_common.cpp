// Error state and library-level entry points of libratslam_hip.
#include "rs_common.h"

#include <cstring>

namespace rs {

static thread_local char g_err[1024] = {0};

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

void clear_error() { g_err[0] = 0; }

}  // namespace rs

extern "C" {

int rs_version(void) { return 100; }

const char* rs_last_error(void) { return rs::g_err; }

int rs_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

}  // extern "C"
