// voxnav_collect.hip -- the on-device PPO rollout collector around the env
// step.
//
// The reference collects rollouts with sb3_contrib's
// RecurrentPPO.collect_rollouts (third-party, reached from model.learn at
// train/Grid_Train.py:228; policy "MlpLstmPolicy", net_arch
// pi/vf=[256,256,128], lstm_hidden_size=256 at :68-80, :196-204).  Per step
// it runs the actor and critic LSTMs on the observation batch (with the
// state of every env whose previous step ended an episode zeroed), samples a
// Categorical action, steps the VecEnv, bootstraps the reward of every env
// that was truncated with gamma * V(terminal_obs) under that env's critic
// state, and appends (obs, action, reward, episode_start, value, log_prob,
// lstm states) to the rollout buffer.  Here the matrix products run as
// library GEMMs (hipBLASLt through torch, f32 -- the reference's dtype) and
// everything between them is one of these kernels:
//
//   lstm_cell_kernel      gate pre-activations (x GEMM + h GEMM + biases)
//                         -> i,f,g,o -> (h, c), optional buffer store
//   policy_head_kernel    action logits + value head (GEMVs from LDS),
//                         log-softmax, Philox inverse-CDF Categorical
//                         sample (or argmax), log-prob
//   boot_compact_kernel   ordered compaction of the truncated envs
//                         (SB3: done and info["TimeLimit.truncated"])
//   bootstrap_kernel      rewards[idx] += gamma * V(terminal_obs)
//   episode_start_kernel  episode_starts[t+1] = done; zero (h, c) of done envs
//
// All f32, compiled with -ffp-contract=off (no fused multiply-add), so the
// bootstrap add rounds exactly like SB3's numpy `rewards[idx] += gamma * v`.

#include <hip/hip_runtime.h>

#include <cstdint>

#include "vn_common.h"

using vn_detail::fail;

namespace {

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

// bf16 (stored as uint16_t) <-> f32; f32 -> bf16 rounds to nearest even
// (torch's rounding; the values here are finite)
__device__ __forceinline__ float bf2f(uint32_t b) { return __uint_as_float(b << 16); }
__device__ __forceinline__ uint32_t f2bf(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}

template <typename T>
__device__ __forceinline__ float4 load4(const T *p);
template <>
__device__ __forceinline__ float4 load4<float>(const float *p) {
    return *reinterpret_cast<const float4 *>(p);
}
template <>
__device__ __forceinline__ float4 load4<uint16_t>(const uint16_t *p) {
    const uint2 v = *reinterpret_cast<const uint2 *>(p);
    return make_float4(bf2f(v.x & 0xffffu), bf2f(v.x >> 16), bf2f(v.y & 0xffffu), bf2f(v.y >> 16));
}

using vn_detail::philox_word0;

// ----------------------------------------------------------------------------
// LSTM cell, torch gate order (i, f, g, o):
//   pre = gx + gh + b_ih + b_hh;  c' = f*c + i*g;  h' = o*tanh(c')
// One thread per (lstm b, agent n, 4 hidden units): float4 loads of the four
// gate slices, coalesced along the hidden dimension.
//   gx  element (b, n, j) at gx[n*gx_row + b*4H + j]   (one GEMM for all LSTMs)
//   gh  [B][N][4H] or NULL (state was zero)
//   h, c, h_store, c_store  [B][N][H]
// T = float, or uint16_t for bf16 gate pre-activations (the bf16 policy
// path, which also writes h in bf16 for the next GEMMs into h_bf).
// ----------------------------------------------------------------------------
// MASK (the rollout entry vn_lstm_cell_masked): the state is read from c_in
// (!= c) and gh was computed from the UNMASKED h; agents with start[n] != 0
// take h = c = 0, i.e. no gh term (h_masked @ W_hh^T = 0 exactly) and c_in 0.
template <typename T, bool MASK>
__global__ __launch_bounds__(256) void lstm_cell_kernel(const T *__restrict__ gx, int64_t gx_row,
                                                        const T *__restrict__ gh, const float *__restrict__ b_ih,
                                                        const float *__restrict__ b_hh, float *__restrict__ h,
                                                        const float *__restrict__ c_in, const float *__restrict__ start,
                                                        float *__restrict__ c, uint16_t *__restrict__ h_bf,
                                                        float *__restrict__ h_store, float *__restrict__ c_store,
                                                        int B, int N, int H) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int H4 = H >> 2;
    const int64_t per_b = (int64_t)N * H4;
    if (q >= per_b * B) return;
    const int b = (int)(q / per_b);
    const int64_t r = q - (int64_t)b * per_b;
    const int64_t n = r / H4;
    const int j = (int)(r - n * H4) * 4;
    const int G = 4 * H;
    const T *px = gx + n * gx_row + (int64_t)b * G + j;
    const bool zero = MASK && start[n] != 0.0f;
    const T *ph = (gh && !zero) ? gh + ((int64_t)b * N + n) * G + j : nullptr;
    const float *pbi = b_ih + (int64_t)b * G + j;
    const float *pbh = b_hh + (int64_t)b * G + j;
    float4 pre[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float4 x = load4<T>(px + k * H);
        const float4 bi = *reinterpret_cast<const float4 *>(pbi + k * H);
        const float4 bh = *reinterpret_cast<const float4 *>(pbh + k * H);
        float4 s = x;
        if (ph) {
            const float4 y = load4<T>(ph + k * H);
            s.x += y.x; s.y += y.y; s.z += y.z; s.w += y.w;
        }
        s.x += bi.x; s.y += bi.y; s.z += bi.z; s.w += bi.w;
        s.x += bh.x; s.y += bh.y; s.z += bh.z; s.w += bh.w;
        pre[k] = s;
    }
    const int64_t so = ((int64_t)b * N + n) * H + j;
    float4 cv = zero ? make_float4(0.f, 0.f, 0.f, 0.f) : *reinterpret_cast<const float4 *>((MASK ? c_in : c) + so);
    float4 hv;
#define VN_CELL(comp)                                                                 \
    {                                                                                 \
        const float ig = sigm(pre[0].comp), fg = sigm(pre[1].comp);                    \
        const float gg = tanhf(pre[2].comp), og = sigm(pre[3].comp);                   \
        const float fc = fg * cv.comp, ig2 = ig * gg;                                 \
        cv.comp = fc + ig2;                                                           \
        hv.comp = og * tanhf(cv.comp);                                                \
    }
    VN_CELL(x) VN_CELL(y) VN_CELL(z) VN_CELL(w)
#undef VN_CELL
    *reinterpret_cast<float4 *>(c + so) = cv;
    *reinterpret_cast<float4 *>(h + so) = hv;
    if (h_bf)
        *reinterpret_cast<uint2 *>(h_bf + so) =
            make_uint2(f2bf(hv.x) | (f2bf(hv.y) << 16), f2bf(hv.z) | (f2bf(hv.w) << 16));
    if (h_store) *reinterpret_cast<float4 *>(h_store + so) = hv;
    if (c_store) *reinterpret_cast<float4 *>(c_store + so) = cv;
}

// ----------------------------------------------------------------------------
// Fused LSTM step on the matrix cores (bf16 policy path): for each LSTM b,
//   gates[n][4H] = [x_n | h_n] @ [W_ih | W_hh]^T + (b_ih + b_hh)
// with v_mfma_f32_32x32x16_bf16 (f32 accumulation), and the cell update as
// the epilogue, so the 4H gate pre-activations never leave the registers.
// Block: 4 waves (VN_LF_ROWS 64), 64 agents x 64 hidden units x 4 gates; wave w owns rows
// 32*(w&1).. and units 32*(w>>1).., one 32x32 accumulator per gate, so the
// four gates of a (row, unit) sit in the same lane and register.  K is
// streamed in chunks of 64 through LDS (rows padded to 72 bf16), the next
// chunk prefetched into registers during the current chunk's MFMAs.  x is read as f32 (the env's obs) and rounded to bf16 on the way
// into LDS; W is pre-packed [B][4H][Kp] with x in columns [0, obs_dim),
// h in [kx, kx+H) (kx = obs_dim rounded up to 8), zeros elsewhere.
//   hin / hout  bf16 [B][N][H] (ping-pong: other blocks still read hin)
//   c           f32 [B][N][H] in/out;  h32, h_store, c_store f32, optional
// ----------------------------------------------------------------------------
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(16))) float f32x16_t;

#ifndef VN_LF_ROWS
#define VN_LF_ROWS 64   // 96 / 128 / 192 rows measured 432 / 357 / 363 vs 347 us
#endif
constexpr int LF_ROWS = VN_LF_ROWS, LF_UNITS = 64;
constexpr int LF_WAVES = (LF_ROWS / 32) * (LF_UNITS / 32), LF_T = 64 * LF_WAVES;   // threads per block
#ifndef VN_LF_KC
#define VN_LF_KC 64
#endif
constexpr int LF_KC = VN_LF_KC;           // K per chunk (bf16 elements)
constexpr int LF_LDK = LF_KC + 8;         // LDS row pitch (+16 B against bank conflicts)
constexpr int LF_GPR = LF_KC / 8;         // 16-byte groups per row and chunk
constexpr int LF_BTOT = 4 * LF_UNITS * LF_GPR;    // 16-byte W groups per chunk
constexpr int LF_NA = LF_ROWS * LF_GPR / LF_T, LF_NB = (LF_BTOT + LF_T - 1) / LF_T;   // groups per thread

// gate nonlinearities of the bf16 path on the hardware exp / rcp (~1e-6
// relative; the operands are bf16 already): 5 per (row, unit), 80 per lane
__device__ __forceinline__ float fast_sigm(float x) { return __frcp_rn(1.0f + __expf(-x)); }
__device__ __forceinline__ float fast_tanh(float x) { return 2.0f * fast_sigm(2.0f * x) - 1.0f; }

#ifndef VN_LF_RAW_BARRIER
#define VN_LF_RAW_BARRIER 1
#endif
#ifndef VN_LF_MIN_WAVES
#define VN_LF_MIN_WAVES 3   // waves per SIMD the register budget is sized for (12 per CU)
#endif
template <bool VEC_X, bool MASK>   // obs_dim % 8 == 0: branch-free staging loads; MASK: episode-start mask on c_in
#ifdef VN_LF_WPE
#define LF_WPE_ATTR __attribute__((amdgpu_waves_per_eu(VN_LF_WPE, VN_LF_WPE)))
#else
#define LF_WPE_ATTR
#endif
__global__ __launch_bounds__(LF_T, VN_LF_MIN_WAVES) LF_WPE_ATTR void lstm_fused_bf16_kernel(
    const float *__restrict__ x, int obs_dim, int kx, const uint16_t *__restrict__ hin,
    // MASK: the state is read from c_in (never the array c); !MASK (the
    // in/out entry): c_in is unused (null) and the state is read from c itself,
    // so no two restrict pointers alias
    const uint16_t *__restrict__ w, int Kp, const float *__restrict__ bias, const float *__restrict__ c_in,
    const float *__restrict__ start, float *__restrict__ c, uint16_t *__restrict__ hout, float *__restrict__ h32,
    float *__restrict__ h_store, float *__restrict__ c_store, int N, int H, int ncombo) {
    // one LDS buffer; the next chunk is prefetched into registers during
    // the current chunk's MFMAs
    __shared__ __attribute__((aligned(16))) uint16_t lds[(LF_ROWS + 4 * LF_UNITS) * LF_LDK];
    uint16_t *As = lds, *Bs = lds + LF_ROWS * LF_LDK;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    // 1-D grid over (row tile, combo = LSTM x unit block).  Blocks are dealt
    // to the 8 XCDs round-robin by id; when the tile count allows, the combos
    // of one row tile get ids of the same residue mod 8 (same XCD, close in
    // time), so the tile's x / h rows are fetched into that XCD's L2 once.
    const int ublocks = H / LF_UNITS;
    const int ntiles = (N + LF_ROWS - 1) / LF_ROWS;
    const int id = (int)blockIdx.x;
    int tile, combo;
    if ((ntiles & 7) == 0) {
        const int xcd = id & 7, local = id >> 3;
        tile = xcd + 8 * (local / ncombo);
        combo = local - (local / ncombo) * ncombo;
    } else {
        tile = id / ncombo;
        combo = id - tile * ncombo;
    }
    const int b = combo / ublocks;
    const int u_base = (combo - b * ublocks) * LF_UNITS;
    const int n_base = tile * LF_ROWS;
    const int K = kx + H;
    const int nchunks = Kp / LF_KC;
    const uint16_t *wb = w + (size_t)b * 4 * H * Kp;
    const uint16_t *hb = hin + (size_t)b * N * H;

    static_assert(LF_NA == 2 && LF_NB <= 8 && LF_ROWS * LF_GPR == 2 * LF_T, "staging registers are spelled out for LF_KC = 64");
    // raw staging registers: an A group is 8 obs floats (x columns) or 8 bf16
    // of h (in lo); it is converted when written to LDS, so no wait sits
    // between issuing the next chunk's loads and this chunk's MFMAs
    float4 ra0lo, ra0hi, ra1lo, ra1hi;
    uint4 rb0, rb1, rb2, rb3, rb4, rb5, rb6, rb7;   // named: an indexed array would live in scratch
#define LF_A_LOAD(lo, hi, i)                                                                                \
    if (VEC_X) {                                                                                            \
        /* unconditional loads from a clamped address, zeroed when written to LDS: */                       \
        /* a loaded value merged across branches would force a wait right here     */                       \
        const int gi_ = tid + LF_T * (i), k_ = k0_ + (gi_ % LF_GPR) * 8;                                    \
        const int n_ = min(n_base + gi_ / LF_GPR, N - 1);                                                   \
        const bool isx_ = k_ < kx;                                                                          \
        const float *p_ = isx_ ? x + (size_t)n_ * obs_dim + k_                                              \
                               : reinterpret_cast<const float *>(hb + (size_t)n_ * H + min(k_ - kx, H - 8)); \
        lo = *reinterpret_cast<const float4 *>(p_);                                                         \
        hi = *reinterpret_cast<const float4 *>(p_ + (isx_ ? 4 : 0));                                        \
    } else {                                                                                                \
        const int gi_ = tid + LF_T * (i), k_ = k0_ + (gi_ % LF_GPR) * 8;                                    \
        const int n_ = n_base + gi_ / LF_GPR;                                                               \
        lo = make_float4(0.f, 0.f, 0.f, 0.f);                                                               \
        hi = lo;                                                                                            \
        if (n_ < N) {                                                                                       \
            if (k_ < kx) {                                                                                  \
                const float *px_ = x + (size_t)n_ * obs_dim + k_;                                           \
                lo.x = k_ + 0 < obs_dim ? px_[0] : 0.0f; lo.y = k_ + 1 < obs_dim ? px_[1] : 0.0f;          \
                lo.z = k_ + 2 < obs_dim ? px_[2] : 0.0f; lo.w = k_ + 3 < obs_dim ? px_[3] : 0.0f;          \
                hi.x = k_ + 4 < obs_dim ? px_[4] : 0.0f; hi.y = k_ + 5 < obs_dim ? px_[5] : 0.0f;          \
                hi.z = k_ + 6 < obs_dim ? px_[6] : 0.0f; hi.w = k_ + 7 < obs_dim ? px_[7] : 0.0f;          \
            } else if (k_ < K) {                                                                            \
                lo = *reinterpret_cast<const float4 *>(hb + (size_t)n_ * H + (k_ - kx));                    \
            }                                                                                               \
        }                                                                                                   \
    }
#define LF_B(dst, i)                                                                                        \
    if (LF_NB > (i)) {                                                                                      \
        const int gi_ = tid + LF_T * (i), lrow_ = gi_ / LF_GPR, gate_ = lrow_ / LF_UNITS;                   \
        const int uu_ = lrow_ - gate_ * LF_UNITS;                                                           \
        if (LF_BTOT % LF_T == 0 || gi_ < LF_BTOT) /* wave-uniform */                                       \
            dst = *reinterpret_cast<const uint4 *>(wb + (size_t)(gate_ * H + u_base + uu_) * Kp + k0_ +     \
                                                   (gi_ % LF_GPR) * 8);                                     \
    }
#define LF_LOAD_CHUNK(ch)                                                                                   \
    {                                                                                                       \
        const int k0_ = (ch) * LF_KC;                                                                       \
        LF_B(rb0, 0) LF_B(rb1, 1) LF_B(rb2, 2) LF_B(rb3, 3) LF_B(rb4, 4) LF_B(rb5, 5) LF_B(rb6, 6) LF_B(rb7, 7) \
        LF_A_LOAD(ra0lo, ra0hi, 0) LF_A_LOAD(ra1lo, ra1hi, 1)                                               \
    }
#define LF_A_PUT(lo, hi, i)                                                                                 \
    {                                                                                                       \
        const int gi_ = tid + LF_T * (i), k_ = k0_ + (gi_ % LF_GPR) * 8;                                    \
        uint4 v_;                                                                                           \
        if (VEC_X && (n_base + gi_ / LF_GPR >= N || k_ >= K)) {                                             \
            v_ = make_uint4(0u, 0u, 0u, 0u);                                                                \
        } else if (k_ < kx) {                                                                               \
            v_ = make_uint4(f2bf(lo.x) | (f2bf(lo.y) << 16), f2bf(lo.z) | (f2bf(lo.w) << 16),              \
                            f2bf(hi.x) | (f2bf(hi.y) << 16), f2bf(hi.z) | (f2bf(hi.w) << 16));             \
        } else {                                                                                            \
            v_ = make_uint4(__float_as_uint(lo.x), __float_as_uint(lo.y), __float_as_uint(lo.z),            \
                            __float_as_uint(lo.w));                                                         \
        }                                                                                                   \
        *reinterpret_cast<uint4 *>(&As[(gi_ / LF_GPR) * LF_LDK + (gi_ % LF_GPR) * 8]) = v_;                 \
    }
#define LF_PUT(base, src, i)                                                                                \
    if (LF_NB > (i)) {                                                                                      \
        const int gi_ = tid + LF_T * (i);                                                                    \
        if (LF_BTOT % LF_T == 0 || gi_ < LF_BTOT)                                                           \
            *reinterpret_cast<uint4 *>(&base[(gi_ / LF_GPR) * LF_LDK + (gi_ % LF_GPR) * 8]) = src;          \
    }
#define LF_STORE_CHUNK(ch)                                                                                   \
    {                                                                                                       \
        const int k0_ = (ch) * LF_KC;                                                                       \
        LF_A_PUT(ra0lo, ra0hi, 0) LF_A_PUT(ra1lo, ra1hi, 1)                                                 \
        LF_PUT(Bs, rb0, 0) LF_PUT(Bs, rb1, 1) LF_PUT(Bs, rb2, 2) LF_PUT(Bs, rb3, 3)                         \
        LF_PUT(Bs, rb4, 4) LF_PUT(Bs, rb5, 5) LF_PUT(Bs, rb6, 6) LF_PUT(Bs, rb7, 7)                         \
    }

    f32x16_t acc[4];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[g][r] = 0.0f;
    const int wr = (wv % (LF_ROWS / 32)) * 32, wu = (wv / (LF_ROWS / 32)) * 32;
#ifndef VN_LF_DIAG
#define VN_LF_DIAG 0   // timing diagnostics: 1 skips the K loop, 2 a cheap epilogue (results invalid)
#endif
    // Block barriers that order only LDS (lgkmcnt(0) + s_barrier): a
    // __syncthreads() also waits vmcnt(0), i.e. for the next chunk's
    // prefetch, so that prefetch could only overlap one chunk's MFMAs
#if VN_LF_RAW_BARRIER
#define LF_BARRIER()                                                                                        \
    {                                                                                                       \
        asm volatile("" ::: "memory");                                                                      \
        __builtin_amdgcn_s_waitcnt(0xC07F);                                                                 \
        __builtin_amdgcn_s_barrier();                                                                       \
        asm volatile("" ::: "memory");                                                                      \
    }
#else
#define LF_BARRIER() __syncthreads();
#endif
    LF_LOAD_CHUNK(0)
    for (int ch = 0; ch < (VN_LF_DIAG == 1 ? 0 : nchunks); ++ch) {
        LF_STORE_CHUNK(ch)
        LF_BARRIER()
        // next chunk, in flight during this chunk's MFMAs (the last iteration
        // reloads its own chunk: unconditional, so the staging stays in
        // registers); the scheduling barrier keeps the loads ahead of the MFMAs
        LF_LOAD_CHUNK(ch + 1 < nchunks ? ch + 1 : ch)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ks = 0; ks < LF_KC / 16; ++ks) {
            const int kk = ks * 16 + 8 * (lane >> 5);
            const bf16x8_t a = *reinterpret_cast<const bf16x8_t *>(&As[(wr + (lane & 31)) * LF_LDK + kk]);
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const bf16x8_t bv =
                    *reinterpret_cast<const bf16x8_t *>(&Bs[(g * LF_UNITS + wu + (lane & 31)) * LF_LDK + kk]);
                acc[g] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bv, acc[g], 0, 0, 0);
            }
        }
        LF_BARRIER()
    }
#undef LF_BARRIER
#undef LF_LOAD_CHUNK
#undef LF_STORE_CHUNK
#undef LF_A_LOAD
#undef LF_A_PUT
#undef LF_B
#undef LF_PUT

    // epilogue: lane holds unit u for 16 rows; gate g of (row, u) in acc[g][reg]
    const int u = u_base + wu + (lane & 31);
    // the 16 cell states loaded together first: loaded row by row, each load
    // would wait behind the previous row's five stores (vmcnt retires in order)
    float cin[16];
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int n = min(n_base + wr + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5), N - 1);
        const float v = (MASK ? c_in : c)[((size_t)b * N + n) * H + u];
        cin[reg] = (MASK && start[n] != 0.0f) ? 0.0f : v;   // the episode-start mask, applied on read
    }
    const float *bb = bias + (size_t)b * 4 * H;
    const float bi = bb[u], bf = bb[H + u], bg = bb[2 * H + u], bo = bb[3 * H + u];
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int n = n_base + wr + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
        if (n < N) {
            const size_t so = ((size_t)b * N + n) * H + u;
#if VN_LF_DIAG == 2
            const float ig = acc[0][reg] + bi, fg = acc[1][reg] + bf, gg = acc[2][reg] + bg, og = acc[3][reg] + bo;
#else
            const float ig = fast_sigm(acc[0][reg] + bi), fg = fast_sigm(acc[1][reg] + bf);
            const float gg = fast_tanh(acc[2][reg] + bg), og = fast_sigm(acc[3][reg] + bo);
#endif
            const float fc = fg * cin[reg], ig2 = ig * gg;
            const float cn = fc + ig2;
#if VN_LF_DIAG == 2
            const float hn = og * cn;
#else
            const float hn = og * fast_tanh(cn);
#endif
            c[so] = cn;
            hout[so] = (uint16_t)f2bf(hn);
            if (h32) h32[so] = hn;
            if (h_store) h_store[so] = hn;
            if (c_store) c_store[so] = cn;
        }
    }
}

// ----------------------------------------------------------------------------
// Action + value heads and the Categorical draw.  16 lanes per agent (16
// agents per 256-thread block): lane l reads float4s l, l+16, ... of the
// agent's latent rows (coalesced 256-B segments), dot products against the
// head weights held in LDS, butterfly-reduced over the 16 lanes.
//   logits_a = b_a + sum_k lat_pi[k] * W_a[a][k]      (action_net, 128 -> A)
//   value    = b_v + sum_k lat_vf[k] * w_v[k]         (value_net,  128 -> 1)
//   lse = max + log(sum exp(logit - max)); log_prob = logit[action] - lse
//   action: first a with u < cdf[a] (cdf over exp(logit - lse)), u from
//   Philox; argmax when deterministic.  lat_pi NULL -> value only.
// ----------------------------------------------------------------------------
constexpr int HEAD_MAX_A = 8;

template <typename T>
__global__ __launch_bounds__(256) void policy_head_kernel(const T *__restrict__ lat_pi,
                                                          const T *__restrict__ lat_vf, int N, int P,
                                                          const float *__restrict__ wa, const float *__restrict__ ba,
                                                          int A, const float *__restrict__ wv,
                                                          const float *__restrict__ bv, uint64_t seed, uint64_t t,
                                                          int64_t gid_base, int deterministic,
                                                          int32_t *__restrict__ actions, float *__restrict__ values,
                                                          float *__restrict__ logp) {
    extern __shared__ float sw[];  // [A][P] action weights, then [P] value weights
    const int nw = (lat_pi ? A * P : 0);
    for (int i = threadIdx.x; i < nw; i += blockDim.x) sw[i] = wa[i];
    if (lat_vf)
        for (int i = threadIdx.x; i < P; i += blockDim.x) sw[A * P + i] = wv[i];
    __syncthreads();
    const int g = threadIdx.x >> 4, l = threadIdx.x & 15;
    const int64_t n = (int64_t)blockIdx.x * 16 + g;
    const bool live = n < N;
    float acc[HEAD_MAX_A + 1];
#pragma unroll
    for (int a = 0; a <= HEAD_MAX_A; ++a) acc[a] = 0.0f;
    if (live) {
        for (int k = l * 4; k < P; k += 64) {
            if (lat_pi) {
                const float4 x = load4<T>(lat_pi + n * P + k);
#pragma unroll
                for (int a = 0; a < HEAD_MAX_A; ++a) {
                    if (a < A) {
                        const float *w = sw + a * P + k;
                        acc[a] += x.x * w[0];
                        acc[a] += x.y * w[1];
                        acc[a] += x.z * w[2];
                        acc[a] += x.w * w[3];
                    }
                }
            }
            if (lat_vf) {
                const float4 x = load4<T>(lat_vf + n * P + k);
                const float *w = sw + A * P + k;
                acc[HEAD_MAX_A] += x.x * w[0];
                acc[HEAD_MAX_A] += x.y * w[1];
                acc[HEAD_MAX_A] += x.z * w[2];
                acc[HEAD_MAX_A] += x.w * w[3];
            }
        }
    }
#pragma unroll
    for (int a = 0; a <= HEAD_MAX_A; ++a) {
#pragma unroll
        for (int m = 8; m >= 1; m >>= 1) acc[a] += __shfl_xor(acc[a], m, 16);
    }
    if (!live || l != 0) return;
    if (lat_vf) values[n] = acc[HEAD_MAX_A] + bv[0];
    if (!lat_pi) return;
    float lg[HEAD_MAX_A];
    float mx = -INFINITY;
#pragma unroll
    for (int a = 0; a < HEAD_MAX_A; ++a) {
        lg[a] = (a < A) ? acc[a] + ba[a] : -INFINITY;
        mx = fmaxf(mx, lg[a]);
    }
    float se = 0.0f;
#pragma unroll
    for (int a = 0; a < HEAD_MAX_A; ++a)
        if (a < A) se += expf(lg[a] - mx);
    const float lse = mx + logf(se);
    int act = A - 1;
    if (deterministic) {
        float best = lg[0];
        act = 0;
#pragma unroll
        for (int a = 1; a < HEAD_MAX_A; ++a)
            if (a < A && lg[a] > best) {
                best = lg[a];
                act = a;
            }
    } else {
        const uint64_t gid = (uint64_t)(gid_base + n);
        const uint32_t w0 = philox_word0(seed, gid, t | (1ull << 63));
        const float u = (float)(w0 >> 8) * (1.0f / 16777216.0f);
        float cdf = 0.0f;
#pragma unroll
        for (int a = 0; a < HEAD_MAX_A; ++a) {
            if (a < A - 1) {
                cdf += expf(lg[a] - lse);
                if (u < cdf && act == A - 1) act = a;
            }
        }
        // first a with u < cdf: the loop above keeps the FIRST crossing
        // because act only leaves A-1 once.
    }
    actions[n] = act;
    logp[n] = lg[act] - lse;
}

// ----------------------------------------------------------------------------
// Ordered compaction of the envs whose step was a time-limit truncation:
// SB3 bootstraps `done and info["TimeLimit.truncated"]`, where the VecEnv
// wrapper sets TimeLimit.truncated = truncated and not terminated.
// One 1024-thread block; thread i owns the 16-byte-aligned chunks i,
// i+1024, ... of the flag arrays (one uint4 load per array per chunk; the
// flags are 0/1 bytes, so a chunk's boot mask is tr & ~te & 0x01 per byte).
// A block-wide exclusive scan of the per-thread counts orders the output by
// agent index, so the gathered batch (and its GEMM) is the same every run.
// ----------------------------------------------------------------------------
__device__ __forceinline__ uint4 boot_bytes(const uint8_t *__restrict__ term, const uint8_t *__restrict__ trunc,
                                            int base, int N) {
    uint4 m;
    if (base + 16 <= N) {
        const uint4 te = *reinterpret_cast<const uint4 *>(term + base);
        const uint4 tr = *reinterpret_cast<const uint4 *>(trunc + base);
        m.x = tr.x & ~te.x & 0x01010101u;
        m.y = tr.y & ~te.y & 0x01010101u;
        m.z = tr.z & ~te.z & 0x01010101u;
        m.w = tr.w & ~te.w & 0x01010101u;
    } else {
        uint32_t w[4] = {0u, 0u, 0u, 0u};
        for (int k = 0; k < 16 && base + k < N; ++k)
            w[k >> 2] |= (uint32_t)((trunc[base + k] != 0) & (term[base + k] == 0)) << (8 * (k & 3));
        m = make_uint4(w[0], w[1], w[2], w[3]);
    }
    return m;
}

__global__ __launch_bounds__(1024) void boot_compact_kernel(const uint8_t *__restrict__ term,
                                                            const uint8_t *__restrict__ trunc, int N,
                                                            int32_t *__restrict__ idx, int32_t *__restrict__ count) {
    __shared__ int wsum[16];
    const int tid = threadIdx.x;
    const int nchunk = (N + 15) >> 4;
    // thread tid owns chunks [c0, c1): contiguous, so the output order is
    // the agent order after the scan
    const int per = (nchunk + 1023) >> 10;
    const int c0 = min(nchunk, tid * per), c1 = min(nchunk, c0 + per);
    int cnt = 0;
    for (int ch = c0; ch < c1; ++ch) {
        const uint4 m = boot_bytes(term, trunc, ch << 4, N);
        cnt += __popc(m.x) + __popc(m.y) + __popc(m.z) + __popc(m.w);
    }
    const int lane = tid & 63, wv = tid >> 6;
    int inc = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(inc, d, 64);
        if (lane >= d) inc += y;
    }
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    if (tid == 0) {
        int run = 0;
        for (int w = 0; w < 16; ++w) {
            const int v = wsum[w];
            wsum[w] = run;
            run += v;
        }
        *count = run;
    }
    __syncthreads();
    if (cnt == 0) return;
    int pos = wsum[wv] + inc - cnt;
    for (int ch = c0; ch < c1; ++ch) {
        const uint4 m = boot_bytes(term, trunc, ch << 4, N);
        const uint32_t w[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            uint32_t b = w[q];
            while (b) {
                const int bit = __ffs(b) - 1;
                idx[pos++] = (ch << 4) + q * 4 + (bit >> 3);
                b &= b - 1;
            }
        }
    }
}

// rewards[idx[i]] = rewards[idx[i]] + (gamma * v[i])   (two f32 roundings,
// as numpy `rewards[idx] += self.gamma * terminal_value`)
__global__ __launch_bounds__(256) void bootstrap_kernel(const int32_t *__restrict__ idx, const float *__restrict__ v,
                                                        int M, float g32, float *__restrict__ rew) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M) return;
    const int a = idx[i];
    const float gv = g32 * v[i];
    rew[a] = rew[a] + gv;
}

// The step's truncated agents appended to the rollout's bootstrap stash, so
// the truncation bootstrap runs once per rollout (no per-step host read of the
// count): row base[t] + j gets agent a = idx[j]'s terminal obs, its critic
// state (h in h_bytes-byte elements, c f32) and the flat reward index
// t * N + a; block 0 thread 0 sets base[t + 1] = base[t] + count.  Rows past
// `cap` are dropped (the caller checks base[T] <= cap).  One wave per row.
__global__ __launch_bounds__(256) void collect_stash_kernel(const int32_t *__restrict__ idx,
                                                            const int32_t *__restrict__ count,
                                                            const int32_t *__restrict__ base_in,
                                                            int32_t *__restrict__ base_out, int t, int N,
                                                            const float *__restrict__ tobs, int obs_dim,
                                                            const uint8_t *__restrict__ h, int h_bytes,
                                                            const float *__restrict__ c, int H,
                                                            float *__restrict__ st_obs, uint8_t *__restrict__ st_h,
                                                            float *__restrict__ st_c, int32_t *__restrict__ st_flat,
                                                            int cap) {
    const int cnt = *count, base = *base_in;
    if (blockIdx.x == 0 && threadIdx.x == 0) *base_out = base + cnt;
    const int lane = threadIdx.x & 63;
    const int nw = (int)(gridDim.x * blockDim.x) >> 6;
    for (int j = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6); j < cnt; j += nw) {
        const int r = base + j;
        if (r >= cap) break;
        const int a = idx[j];
        if (lane == 0) st_flat[r] = t * N + a;
        for (int k = lane; k < obs_dim; k += 64) st_obs[(size_t)r * obs_dim + k] = tobs[(size_t)a * obs_dim + k];
        if (h) {
            const int hw = H * h_bytes / 4;          // 32-bit words of a row
            const uint32_t *hs = reinterpret_cast<const uint32_t *>(h) + (size_t)a * hw;
            uint32_t *hd = reinterpret_cast<uint32_t *>(st_h) + (size_t)r * hw;
            for (int k = lane; k < hw; k += 64) hd[k] = hs[k];
            for (int k = lane; k < H; k += 64) st_c[(size_t)r * H + k] = c[(size_t)a * H + k];
        }
    }
}

// episode_starts[n] = done; (h, c)[b][n][:] = 0 for done agents
// (RecurrentActorCriticPolicy._process_sequence masks the state with
// (1 - episode_start) before the next LSTM step).
__global__ __launch_bounds__(256) void episode_start_kernel(const uint8_t *__restrict__ term,
                                                            const uint8_t *__restrict__ trunc, int N,
                                                            float *__restrict__ starts, float *__restrict__ h,
                                                            float *__restrict__ c, uint16_t *__restrict__ h_bf,
                                                            int B, int H) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int H4 = H >> 2;
    if (B == 0) {
        if (q < N) starts[q] = (term[q] | trunc[q]) ? 1.0f : 0.0f;
        return;
    }
    const int64_t per_b = (int64_t)N * H4;
    if (q >= per_b * B) return;
    const int b = (int)(q / per_b);
    const int64_t r = q - (int64_t)b * per_b;
    const int64_t n = r / H4;
    const int j = (int)(r - n * H4) * 4;
    const bool done = (term[n] | trunc[n]) != 0;
    if (b == 0 && j == 0 && starts) starts[n] = done ? 1.0f : 0.0f;
    if (done) {
        const int64_t so = ((int64_t)b * N + n) * H + j;
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        *reinterpret_cast<float4 *>(h + so) = z;
        *reinterpret_cast<float4 *>(c + so) = z;
        if (h_bf) *reinterpret_cast<uint2 *>(h_bf + so) = make_uint2(0u, 0u);
    }
}

unsigned blocks_for(int64_t threads, int per_block = 256) { return (unsigned)((threads + per_block - 1) / per_block); }

}  // namespace

extern "C" {

}  // extern "C"

namespace {

template <typename T>
int lstm_cell_launch(const T *gx, int64_t gx_row_stride, const T *gh, const float *b_ih, const float *b_hh, float *h,
                     float *c, uint16_t *h_bf, float *h_store, float *c_store, int32_t n_lstm, int32_t N, int32_t H,
                     void *stream, const float *c_in = nullptr, const float *start = nullptr) {
    if (!gx || !b_ih || !b_hh || !h || !c) return fail(VN_ERR_INVALID, "NULL argument");
    if (n_lstm < 1 || N < 1 || H < 4 || (H & 3)) return fail(VN_ERR_INVALID, "bad sizes n_lstm=%d N=%d H=%d", n_lstm, N, H);
    if (gx_row_stride < (int64_t)n_lstm * 4 * H || (gx_row_stride & 3))
        return fail(VN_ERR_INVALID, "gx_row_stride %lld too small / unaligned", (long long)gx_row_stride);
    const int64_t threads = (int64_t)n_lstm * N * (H / 4);
    if (start)
        hipLaunchKernelGGL((lstm_cell_kernel<T, true>), dim3(blocks_for(threads)), dim3(256), 0, (hipStream_t)stream,
                           gx, gx_row_stride, gh, b_ih, b_hh, h, c_in, start, c, h_bf, h_store, c_store, (int)n_lstm,
                           (int)N, (int)H);
    else
        hipLaunchKernelGGL((lstm_cell_kernel<T, false>), dim3(blocks_for(threads)), dim3(256), 0, (hipStream_t)stream,
                           gx, gx_row_stride, gh, b_ih, b_hh, h, nullptr, nullptr, c, h_bf, h_store, c_store, (int)n_lstm,
                           (int)N, (int)H);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

template <typename T>
int policy_head_launch(const T *latent_pi, const T *latent_vf, int32_t N, int32_t P, const float *w_action,
                       const float *b_action, int32_t n_actions, const float *w_value, const float *b_value,
                       uint64_t sample_seed, uint64_t t, int64_t agent_id_base, int32_t deterministic,
                       int32_t *actions, float *values, float *log_probs, void *stream) {
    if (!latent_pi && !latent_vf) return fail(VN_ERR_INVALID, "latent_pi and latent_vf are both NULL");
    if (latent_pi && (!w_action || !b_action || !actions || !log_probs))
        return fail(VN_ERR_INVALID, "NULL action-head argument");
    if (latent_vf && (!w_value || !b_value || !values)) return fail(VN_ERR_INVALID, "NULL value-head argument");
    if (N < 1 || P < 4 || (P & 3) || P > 4096) return fail(VN_ERR_INVALID, "bad sizes N=%d P=%d", N, P);
    if (latent_pi && (n_actions < 1 || n_actions > HEAD_MAX_A))
        return fail(VN_ERR_INVALID, "n_actions must be in 1..%d (got %d)", HEAD_MAX_A, n_actions);
    const int A = latent_pi ? n_actions : 0;
    const size_t lds = (size_t)(A + 1) * P * sizeof(float);
    hipLaunchKernelGGL(policy_head_kernel<T>, dim3(blocks_for(N, 16)), dim3(256), lds, (hipStream_t)stream,
                       latent_pi, latent_vf, (int)N, (int)P, w_action, b_action, A, w_value, b_value, sample_seed, t,
                       agent_id_base, (int)deterministic, actions, values, log_probs);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

}  // namespace


// One launch after the collector's env step (vn_collect_post_step): what
// episode_start_kernel, monitor_kernel, boot_compact_kernel and
// collect_stash_kernel did in four, one lane per agent.  The truncated
// agents' stash rows are claimed with one atomic per wave (rows are in wave
// order within a wave, waves in completion order: the bootstrap is per row,
// so the order does not change any value).  Done agents' state rows are
// zeroed by their wave together (zB LSTMs; 0: none).
__global__ __launch_bounds__(256) void collect_post_kernel(
    const uint8_t *__restrict__ term, const uint8_t *__restrict__ trunc, int N, int t, float *__restrict__ starts,
    const double *__restrict__ r64, const float *__restrict__ r32, double *__restrict__ ep_ret,
    int32_t *__restrict__ ep_len, double *__restrict__ rec_ret, int32_t *__restrict__ rec_len,
    const float *__restrict__ tobs, int obs_dim, const uint8_t *h, int h_bytes,
    const float *c, int H, float *__restrict__ st_obs, uint8_t *__restrict__ st_h,
    float *__restrict__ st_c, int32_t *__restrict__ st_flat, int cap, int32_t *__restrict__ st_count,
    float *zh, float *zc, uint16_t *zh_bf, int zB) {
    // h / c (the stash's source) may be the very rows zh / zc / zh_bf zero
    // below (the collector's non-buffer paths pass the live state arrays for
    // both): no __restrict__ on them, so the zeroing stores stay behind the
    // stash's loads of the same rows (same wave, program order)
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const int a0 = i - lane;
    const bool live = i < N;
    const bool te = live && term[i] != 0, tr = live && trunc[i] != 0;
    const bool done = te || tr;
    if (live && starts) starts[i] = done ? 1.0f : 0.0f;
    if (live && ep_ret) {                         // SB3 Monitor (as monitor_kernel)
        const double r = ep_ret[i] + (r64 ? r64[i] : (double)r32[i]);
        const int32_t l = ep_len[i] + 1;
        rec_ret[i] = done ? r : 0.0;
        rec_len[i] = done ? l : 0;
        ep_ret[i] = done ? 0.0 : r;
        ep_len[i] = done ? 0 : l;
    }
    // the truncated (not terminated) agents' terminal obs + critic state into the stash
    uint64_t m = __ballot(tr && !te);
    if (m) {
        int base = 0;
        if (lane == 0) base = atomicAdd(st_count, __popcll(m));
        base = __shfl(base, 0);
        while (m) {
            const int src = __ffsll((unsigned long long)m) - 1;
            m &= m - 1;
            const int r = base++;
            if (r >= cap) continue;                  // dropped; the caller checks the count against cap
            const int a = a0 + src;
            if (lane == 0) st_flat[r] = t * N + a;
            for (int k = lane; k < obs_dim; k += 64) st_obs[(size_t)r * obs_dim + k] = tobs[(size_t)a * obs_dim + k];
            if (h) {
                const int hw = H * h_bytes / 4;
                const uint32_t *hs = reinterpret_cast<const uint32_t *>(h) + (size_t)a * hw;
                uint32_t *hd = reinterpret_cast<uint32_t *>(st_h) + (size_t)r * hw;
                for (int k = lane; k < hw; k += 64) hd[k] = hs[k];
                for (int k = lane; k < H; k += 64) st_c[(size_t)r * H + k] = c[(size_t)a * H + k];
            }
        }
    }
    // zero the (h, c) rows of done agents where the next step reads the state arrays
    uint64_t md = __ballot(done && zB > 0);
    while (md) {
        const int src = __ffsll((unsigned long long)md) - 1;
        md &= md - 1;
        const int a = a0 + src;
        for (int b = 0; b < zB; ++b) {
            const size_t so = ((size_t)b * N + a) * H;
            for (int k = lane; k < H; k += 64) {
                zh[so + k] = 0.0f;
                zc[so + k] = 0.0f;
                if (zh_bf) zh_bf[so + k] = 0;
            }
        }
    }
}

// SB3 Monitor (stable_baselines3/common/monitor.py, wrapping every worker at
// train/Grid_Train.py:125): per agent the running episode return (f64, summed
// in step order from 0 like Monitor's sum(self.rewards)) and length; on
// terminated | truncated the finished episode's (return, length) goes to this
// step's record row and the counters restart (Monitor.reset via the VecEnv
// auto-reset).  rec_len 0 = no episode ended at this step.
__global__ __launch_bounds__(256) void monitor_kernel(const double *__restrict__ r64, const float *__restrict__ r32,
                                                      const uint8_t *__restrict__ term,
                                                      const uint8_t *__restrict__ trunc, int N,
                                                      double *__restrict__ ep_ret, int32_t *__restrict__ ep_len,
                                                      double *__restrict__ rec_ret, int32_t *__restrict__ rec_len) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const double r = ep_ret[i] + (r64 ? r64[i] : (double)r32[i]);
    const int32_t l = ep_len[i] + 1;
    const bool done = (term[i] | trunc[i]) != 0;
    rec_ret[i] = done ? r : 0.0;
    rec_len[i] = done ? l : 0;
    ep_ret[i] = done ? 0.0 : r;
    ep_len[i] = done ? 0 : l;
}

extern "C" {

int vn_lstm_cell(const float *gx, int64_t gx_row_stride, const float *gh, const float *b_ih, const float *b_hh,
                 float *h, float *c, float *h_store, float *c_store, int32_t n_lstm, int32_t N, int32_t H,
                 void *stream) {
    return lstm_cell_launch<float>(gx, gx_row_stride, gh, b_ih, b_hh, h, c, nullptr, h_store, c_store, n_lstm, N, H,
                                   stream);
}

int vn_lstm_cell_masked(const float *gx, int64_t gx_row_stride, const float *gh, const float *b_ih,
                        const float *b_hh, const float *c_in, const float *start, float *h_out, float *c_out,
                        int32_t n_lstm, int32_t N, int32_t H, void *stream) {
    if (!c_in || !start || !gh) return fail(VN_ERR_INVALID, "NULL argument");
    if (c_in == c_out) return fail(VN_ERR_INVALID, "c_in and c_out must differ");
    return lstm_cell_launch<float>(gx, gx_row_stride, gh, b_ih, b_hh, h_out, c_out, nullptr, nullptr, nullptr, n_lstm,
                                   N, H, stream, c_in, start);
}

int vn_lstm_cell_bf16(const uint16_t *gx, int64_t gx_row_stride, const uint16_t *gh, const float *b_ih,
                      const float *b_hh, float *h, float *c, uint16_t *h_bf16, float *h_store, float *c_store,
                      int32_t n_lstm, int32_t N, int32_t H, void *stream) {
    return lstm_cell_launch<uint16_t>(gx, gx_row_stride, gh, b_ih, b_hh, h, c, h_bf16, h_store, c_store, n_lstm, N,
                                      H, stream);
}

namespace {
int lstm_fused_launch(const float *x, int32_t obs_dim, const uint16_t *h_in, const uint16_t *w_cat, int32_t Kp,
                      const float *bias, const float *c_in, const float *start, float *c, uint16_t *h_out,
                      float *h32, float *h_store, float *c_store, int32_t n_lstm, int32_t N, int32_t H,
                      void *stream) {
    if (!x || !h_in || !w_cat || !bias || !c || !h_out || (start && !c_in)) return fail(VN_ERR_INVALID, "NULL argument");
    if (h_in == h_out) return fail(VN_ERR_INVALID, "h_in and h_out must differ (other blocks read h_in)");
    const int kx = (obs_dim + 7) & ~7;
    if (n_lstm < 1 || N < 1 || obs_dim < 1 || H < 64 || (H % LF_UNITS) || (Kp % LF_KC) || Kp < kx + H)
        return fail(VN_ERR_INVALID, "bad sizes n_lstm=%d N=%d obs_dim=%d H=%d Kp=%d (H %% 64, Kp %% %d, Kp >= %d)",
                    n_lstm, N, obs_dim, H, Kp, LF_KC, kx + H);
    // one block per (row tile, combo = LSTM x 64-unit block)
    const int ncombo = n_lstm * (H / LF_UNITS);
    const dim3 grid((unsigned)((N + LF_ROWS - 1) / LF_ROWS) * (unsigned)ncombo);
#define VN_LF_LAUNCH(VX, MK)                                                                                \
    hipLaunchKernelGGL((lstm_fused_bf16_kernel<VX, MK>), grid, dim3(LF_T), 0, (hipStream_t)stream, x,           \
                       (int)obs_dim, kx, h_in, w_cat, (int)Kp, bias, c_in, start, c, h_out, h32, h_store, c_store, \
                       (int)N, (int)H, ncombo)
    if ((obs_dim & 7) == 0) {
        if (start) VN_LF_LAUNCH(true, true);
        else VN_LF_LAUNCH(true, false);
    } else {
        if (start) VN_LF_LAUNCH(false, true);
        else VN_LF_LAUNCH(false, false);
    }
#undef VN_LF_LAUNCH
    VN_HIP(hipGetLastError());
    return VN_OK;
}
}  // namespace

int vn_lstm_fused_bf16(const float *x, int32_t obs_dim, const uint16_t *h_in, const uint16_t *w_cat, int32_t Kp,
                       const float *bias, float *c, uint16_t *h_out, float *h32, float *h_store, float *c_store,
                       int32_t n_lstm, int32_t N, int32_t H, void *stream) {
    return lstm_fused_launch(x, obs_dim, h_in, w_cat, Kp, bias, nullptr, nullptr, c, h_out, h32, h_store, c_store,
                             n_lstm, N, H, stream);
}

int vn_lstm_fused_bf16_masked(const float *x, int32_t obs_dim, const uint16_t *h_in, const uint16_t *w_cat,
                              int32_t Kp, const float *bias, const float *c_in, const float *start, float *c_out,
                              uint16_t *h_out, float *h_store, int32_t n_lstm, int32_t N, int32_t H, void *stream) {
    if (!start) return fail(VN_ERR_INVALID, "NULL argument (start)");
    if (c_in == c_out) return fail(VN_ERR_INVALID, "c_in and c_out must differ");
    return lstm_fused_launch(x, obs_dim, h_in, w_cat, Kp, bias, c_in, start, c_out, h_out, nullptr, h_store, nullptr,
                             n_lstm, N, H, stream);
}


int vn_policy_head(const float *latent_pi, const float *latent_vf, int32_t N, int32_t P, const float *w_action,
                   const float *b_action, int32_t n_actions, const float *w_value, const float *b_value,
                   uint64_t sample_seed, uint64_t t, int64_t agent_id_base, int32_t deterministic, int32_t *actions,
                   float *values, float *log_probs, void *stream) {
    return policy_head_launch<float>(latent_pi, latent_vf, N, P, w_action, b_action, n_actions, w_value, b_value,
                                     sample_seed, t, agent_id_base, deterministic, actions, values, log_probs, stream);
}

int vn_policy_head_bf16(const uint16_t *latent_pi, const uint16_t *latent_vf, int32_t N, int32_t P,
                        const float *w_action, const float *b_action, int32_t n_actions, const float *w_value,
                        const float *b_value, uint64_t sample_seed, uint64_t t, int64_t agent_id_base,
                        int32_t deterministic, int32_t *actions, float *values, float *log_probs, void *stream) {
    return policy_head_launch<uint16_t>(latent_pi, latent_vf, N, P, w_action, b_action, n_actions, w_value, b_value,
                                        sample_seed, t, agent_id_base, deterministic, actions, values, log_probs,
                                        stream);
}

int vn_collect_compact(const uint8_t *terminated, const uint8_t *truncated, int32_t N, int32_t *boot_idx,
                       int32_t *boot_count, void *stream) {
    if (!terminated || !truncated || !boot_idx || !boot_count) return fail(VN_ERR_INVALID, "NULL argument");
    if (N < 1) return fail(VN_ERR_INVALID, "N must be >= 1 (got %d)", N);
    if (((uintptr_t)terminated | (uintptr_t)truncated) & 15)
        return fail(VN_ERR_INVALID, "terminated / truncated must be 16-byte aligned");
    hipLaunchKernelGGL(boot_compact_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, terminated, truncated,
                       (int)N, boot_idx, boot_count);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

int vn_collect_stash(const int32_t *boot_idx, const int32_t *boot_count, const int32_t *base_in, int32_t *base_out,
                     int32_t t, int32_t N, const float *terminal_obs, int32_t obs_dim, const void *h_critic,
                     int32_t h_bytes, const float *c_critic, int32_t H, float *stash_obs, void *stash_h,
                     float *stash_c, int32_t *stash_flat, int32_t cap, void *stream) {
    if (!boot_idx || !boot_count || !base_in || !base_out || !terminal_obs || !stash_obs || !stash_flat)
        return fail(VN_ERR_INVALID, "NULL argument");
    if (N < 1 || t < 0 || obs_dim < 1 || cap < 0) return fail(VN_ERR_INVALID, "bad sizes N=%d t=%d obs_dim=%d", N, t, obs_dim);
    if (h_critic && (!c_critic || !stash_h || !stash_c || H < 1 || (h_bytes != 2 && h_bytes != 4) || (H * h_bytes) % 4))
        return fail(VN_ERR_INVALID, "critic state: c, stash rows, H and h_bytes (2 or 4) required");
    if ((int64_t)t * N + N > 0x7fffffff) return fail(VN_ERR_INVALID, "t * N overflows the flat index");
    hipLaunchKernelGGL(collect_stash_kernel, dim3(256), dim3(256), 0, (hipStream_t)stream, boot_idx, boot_count,
                       base_in, base_out, (int)t, (int)N, terminal_obs, (int)obs_dim,
                       reinterpret_cast<const uint8_t *>(h_critic), (int)h_bytes, c_critic, (int)H, stash_obs,
                       reinterpret_cast<uint8_t *>(stash_h), stash_c, stash_flat, (int)cap);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

int vn_collect_bootstrap(const int32_t *boot_idx, const float *terminal_values, int32_t M, double gamma,
                         float *rewards, void *stream) {
    if (M < 0) return fail(VN_ERR_INVALID, "M must be >= 0 (got %d)", M);
    if (M == 0) return VN_OK;
    if (!boot_idx || !terminal_values || !rewards) return fail(VN_ERR_INVALID, "NULL argument");
    hipLaunchKernelGGL(bootstrap_kernel, dim3(blocks_for(M)), dim3(256), 0, (hipStream_t)stream, boot_idx,
                       terminal_values, (int)M, (float)gamma, rewards);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

int vn_episode_start(const uint8_t *terminated, const uint8_t *truncated, int32_t N, float *episode_starts,
                     float *h, float *c, uint16_t *h_bf16, int32_t n_lstm, int32_t H, void *stream) {
    if (!terminated || !truncated) return fail(VN_ERR_INVALID, "NULL argument");
    if (N < 1 || n_lstm < 0) return fail(VN_ERR_INVALID, "bad sizes N=%d n_lstm=%d", N, n_lstm);
    if (n_lstm > 0 && (!h || !c || H < 4 || (H & 3))) return fail(VN_ERR_INVALID, "bad LSTM state arguments");
    if (n_lstm == 0 && !episode_starts) return VN_OK;
    const int64_t threads = n_lstm ? (int64_t)n_lstm * N * (H / 4) : (int64_t)N;
    hipLaunchKernelGGL(episode_start_kernel, dim3(blocks_for(threads)), dim3(256), 0, (hipStream_t)stream,
                       terminated, truncated, (int)N, episode_starts, h, c, h_bf16, (int)n_lstm, (int)H);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

int vn_collect_post_step(const uint8_t *terminated, const uint8_t *truncated, int32_t N, int32_t t,
                         float *episode_starts, const double *reward64, const float *reward, double *ep_return,
                         int32_t *ep_length, double *rec_return, int32_t *rec_length, const float *terminal_obs,
                         int32_t obs_dim, const void *h_critic, int32_t h_bytes, const float *c_critic, int32_t H,
                         float *stash_obs, void *stash_h, float *stash_c, int32_t *stash_flat, int32_t cap,
                         int32_t *stash_count, float *h, float *c, uint16_t *h_bf16, int32_t n_lstm, void *stream) {
    if (!terminated || !truncated || !terminal_obs || !stash_obs || !stash_flat || !stash_count)
        return fail(VN_ERR_INVALID, "NULL argument");
    if (N < 1 || t < 0 || obs_dim < 1 || cap < 0) return fail(VN_ERR_INVALID, "bad sizes N=%d t=%d obs_dim=%d", N, t, obs_dim);
    if (ep_return && (!ep_length || !rec_return || !rec_length || (!reward64 && !reward)))
        return fail(VN_ERR_INVALID, "incomplete monitor arguments");
    if (h_critic && (!c_critic || !stash_h || !stash_c || H < 1 || (h_bytes != 2 && h_bytes != 4) || ((H * h_bytes) & 3)))
        return fail(VN_ERR_INVALID, "bad critic-state arguments");
    if (n_lstm < 0 || (n_lstm > 0 && (!h || !c || H < 1))) return fail(VN_ERR_INVALID, "bad state-zeroing arguments");
    hipLaunchKernelGGL(collect_post_kernel, dim3(blocks_for(N)), dim3(256), 0, (hipStream_t)stream, terminated,
                       truncated, (int)N, (int)t, episode_starts, reward64, reward, ep_return, ep_length, rec_return,
                       rec_length, terminal_obs, (int)obs_dim, reinterpret_cast<const uint8_t *>(h_critic),
                       (int)h_bytes, c_critic, (int)H, stash_obs, reinterpret_cast<uint8_t *>(stash_h), stash_c,
                       stash_flat, (int)cap, stash_count, h, c, h_bf16, (int)n_lstm);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

int vn_monitor_step(const double *reward64, const float *reward, const uint8_t *terminated, const uint8_t *truncated,
                    int32_t N, double *ep_return, int32_t *ep_length, double *rec_return, int32_t *rec_length,
                    void *stream) {
    if ((!reward64 && !reward) || !terminated || !truncated || !ep_return || !ep_length || !rec_return || !rec_length)
        return fail(VN_ERR_INVALID, "NULL argument");
    if (N < 1) return fail(VN_ERR_INVALID, "bad size N=%d", N);
    hipLaunchKernelGGL(monitor_kernel, dim3(blocks_for(N)), dim3(256), 0, (hipStream_t)stream, reward64,
                       reward64 ? nullptr : reward, terminated, truncated, (int)N, ep_return, ep_length, rec_return,
                       rec_length);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

}  // extern "C"
