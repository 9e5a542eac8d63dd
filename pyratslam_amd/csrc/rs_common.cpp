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

int rs_dev_malloc(int device, size_t bytes, void** ptr) {
    rs::clear_error();
    RS_CHECK(ptr, RS_ERR_ARG, "null output pointer");
    *ptr = nullptr;
    RS_HIP(hipSetDevice(device));
    RS_HIP(hipMalloc(ptr, bytes));
    return RS_OK;
}

int rs_dev_free(void* ptr) {
    rs::clear_error();
    if (ptr) RS_HIP(hipFree(ptr));
    return RS_OK;
}

int rs_dev_copy(void* dst, const void* src, size_t bytes) {
    rs::clear_error();
    RS_CHECK(dst && src, RS_ERR_ARG, "null pointer");
    RS_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDefault));
    return RS_OK;
}

int rs_host_alloc(size_t bytes, void** ptr) {
    rs::clear_error();
    RS_CHECK(ptr, RS_ERR_ARG, "null output pointer");
    *ptr = nullptr;
    RS_HIP(hipHostMalloc(ptr, bytes, hipHostMallocMapped | hipHostMallocCoherent));
    return RS_OK;
}

int rs_host_free(void* ptr) {
    rs::clear_error();
    if (ptr) RS_HIP(hipHostFree(ptr));
    return RS_OK;
}

}  // extern "C"
