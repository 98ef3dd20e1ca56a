// vn_common.h -- helpers shared by the libvoxnav translation units
// (error reporting across the C-ABI: negative VN_ERR_* codes plus a
// thread-local message returned by vn_last_error()).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "voxnav.h"

// Compile-time knobs -- the ablations (VN_ABLATE), timing diagnostics
// (VN_*_DIAG, VN_*_PROF) and the A/B layout switches -- exist for the
// diagnostics builds of scripts/build_variants.py (voxnav/_build.py
// build_variant, which defines VN_DIAG) only.  The product library is built
// with every knob at its default: a knob set without VN_DIAG does not build.
#ifndef VN_DIAG
#if defined(VN_ABLATE) || defined(VN_ENV_PROF) || defined(VN_SIMPLE_PROF) || defined(VN_LF_DIAG) || \
    defined(VN_PF_DIAG) || defined(VN_LDS_PAD_U64) || defined(VN_PHILOX16) || defined(VN_REWARD_STRIPE) || \
    defined(VN_PC_BLOCK) || defined(VN_PC_MIN_WAVES) || defined(VN_MIN_WAVES_PER_SIMD) || defined(VN_PREMOVE) || \
    defined(VN_STAGE_OBS) || defined(VN_LF_ROWS) || defined(VN_LF_KC) || defined(VN_LF_RAW_BARRIER) || \
    defined(VN_LF_MIN_WAVES) || defined(VN_LF_WPE) || defined(VN_STOOD) || defined(VN_DPP) || \
    defined(VN_TAB_SWZ) || defined(VN_PF_FAST) || defined(VN_PF_PREF) || defined(VN_OBS_STORE) || \
    defined(VN_LDS_BARRIER)
#error "compile-time knobs are for the diagnostics build only (define VN_DIAG)"
#endif
#endif

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
