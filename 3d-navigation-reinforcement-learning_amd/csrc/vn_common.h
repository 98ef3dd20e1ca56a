// vn_common.h -- helpers shared by the libvoxnav translation units
// (error reporting across the C-ABI: negative VN_ERR_* codes plus a
// thread-local message returned by vn_last_error()).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "voxnav.h"

namespace vn_detail {

inline thread_local std::string g_last_error;

inline int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

}  // namespace vn_detail

#define VN_HIP(expr)                                                                                    \
    do {                                                                                                \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess) return vn_detail::fail(VN_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)
