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
    defined(VN_LDS_BARRIER) || defined(VN_ROW_WB) || defined(VN_SETPRIO) || \
    defined(VN_SETPRIO_FLUSH) || defined(VN_ENV_WT) || defined(VN_DFLUSH_DEFAULT) || defined(VN_STOOD_PART) || defined(VN_WIMG_REP) || \
    defined(VN_BRICK_T) || defined(VN_WREC_K_DEFAULT) || defined(VN_WREC) || defined(VN_DM_CODES) || defined(VN_GEMM_ASM) || \
    defined(VN_ROWS_RAWBAR) || defined(VN_ROWS_PRELOAD) || defined(VN_ROWS_FLAGS)
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

// Philox4x32-10 (same rounds as the env's random policy), word 0: the
// collector's Categorical draws.  The sampler's counter is (global agent id,
// t | 2^63), so it never collides with the env's random-policy stream (gid,
// t / 4) under the same key.
__device__ __forceinline__ uint32_t philox_word0(uint64_t key, uint64_t gid, uint64_t ctr_hi) {
    uint32_t c0 = (uint32_t)gid, c1 = (uint32_t)(gid >> 32), c2 = (uint32_t)ctr_hi, c3 = (uint32_t)(ctr_hi >> 32);
    uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
        const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
        c0 = hi1 ^ c1 ^ k0;
        c1 = lo1;
        c2 = hi0 ^ c3 ^ k1;
        c3 = lo0;
    }
    return c0;
}

}  // namespace vn_detail

#define VN_HIP(expr)                                                                                    \
    do {                                                                                                \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess) return vn_detail::fail(VN_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)
