// voxnav_learn_rows.hip -- the PPO learner's LSTM re-run as ONE persistent
// launch per direction, weights held in registers for the whole sequence
// (sb3_contrib RecurrentPPO.train -> evaluate_actions -> _process_sequence,
// reached from model.learn at train/Grid_Train.py:228).
//
// Row layout.  A minibatch of batch_size = R * T env-major samples (T the
// rollout length) covers R whole env rollouts, the first and the last one
// split at the same step s by the random roll: row r is env e0 + r over all T
// steps, and row 0 holds env e0 + R for t < s.  A row restarts its LSTM state
// wherever sb3 starts a sequence (t = 0, an episode start, the seam of row
// 0): h, c := the buffer's stored state x (1 - episode_start) -- so a row is a
// run of whole sb3 sequences laid end to end, and the outputs equal sb3's
// padded per-sequence re-run without any padding.
//
// Work split: block (LSTM l, unit block ub of 32 units, row tile rt of 32
// rows); the 8 unit blocks of one (l, rt) form a group that exchanges h each
// step.  Every block of the grid (2 x 8 x R/32 <= 256, one per CU) is
// resident for the whole launch (checked on the host), and the hand-off is
// the agent-scope protocol of the HIP guide's Guideline 16 (R1, counter form):
// the payload (h_t; in the backward the partial dh of step t-1) is written
// with 16-B write-through (sc1) stores, every storing wave drains vmcnt, the
// block synchronises, ONE lane adds to the group's counter (agent scope); a
// consumer polls the counter with relaxed sc1 loads and reads the payload
// with sc1 loads only.  Spins are bounded: a timeout sets *err and the launch
// runs to its end (the host raises).
//
// forward   wave w = gate w: the 32 x 32 tile [x_t | h_{t-1}] @ W[gate w, 32
//           units]^T on v_mfma_f32_32x32x2_f32, W (168 VGPRs) resident; the
//           x part runs while the group's h_{t-1} is still being produced;
//           the cell (i, f, g, o, c, h) as the epilogue, c carried in
//           registers (a block owns its units' cells).
// backward  per step in reverse: dh = dh_out + sum of the 8 partials of step
//           t+1 (fixed order), the cell backward (dG_t, dc carried in
//           registers), then this block's partial dh_{t-1} = dG_t[:, its 128
//           gate columns] @ W_hh[those rows, 256 units] (W_hh slice resident,
//           128 VGPRs); rows whose step t starts a sequence pass no gradient
//           back (their h_{t-1}, c_{t-1} came from the buffer).
// f32 throughout (the reference's dtype); the nonlinearities on the hardware exp / rcp.

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "vn_common.h"

using vn_detail::fail;

namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16_t;

constexpr int RW = 32;      // rows per tile
constexpr int UBK = 32;     // units per block
constexpr int NUB = 8;      // unit blocks per LSTM (H = 256)
constexpr uint32_t kSpinLimit = 1u << 22;   // ~0.3 s per wait at s_sleep 2
// one 256-B line per group counter: the counters of all groups in one line put
// every poll and add of the launch on one memory channel (measured: with two
// blocks per CU every memory section of a step ran 3-6x slower)
constexpr int CSTRIDE = 64;

// gate / cell nonlinearities on the hardware exp and reciprocal (|err| <= ~4e-7,
// the collector's f32 policy step uses the same: csrc/voxnav_policy_f32.hip)
__device__ __forceinline__ float sigm(float x) { return __frcp_rn(1.0f + __expf(-x)); }
__device__ __forceinline__ float tanh_fast(float x) { return 1.0f - 2.0f * __frcp_rn(1.0f + __expf(2.0f * x)); }

__device__ __forceinline__ f32x16_t zero16() {
    f32x16_t z;
#pragma unroll
    for (int r = 0; r < 16; ++r) z[r] = 0.0f;
    return z;
}

__device__ __forceinline__ float4 f4(float a) { return make_float4(a, a, a, a); }
__device__ __forceinline__ float4 operator+(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ float4 operator*(float4 a, float4 b) { return make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w); }

__device__ __forceinline__ float4 as_f4(__attribute__((ext_vector_type(4))) float v) { return make_float4(v[0], v[1], v[2], v[3]); }

// 16-B write-through (sc1) store / sc1 load through a buffer resource (aux 16 = sc1)
__device__ __forceinline__ void st_sc1(__amdgpu_buffer_rsrc_t rs, uint32_t off, float4 v) {
    __attribute__((ext_vector_type(4))) float w = {v.x, v.y, v.z, v.w};
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, w), rs, off,
                                           0, 16);
}
__device__ __forceinline__ float4 ld_sc1(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
    const auto u = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);
    const auto v = __builtin_bit_cast(__attribute__((ext_vector_type(4))) float, u);
    return as_f4(v);
}

// one lane: wait until *cnt >= target (relaxed agent-scope loads = sc1), bounded
// (a timed-out launch sets *err; every later wait of every block then returns
// at once, so the launch drains instead of timing out step after step)
__device__ __forceinline__ bool wait_ge(uint32_t *cnt, uint32_t target, int32_t *err) {
    uint32_t spins = 0;
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(2);
        ++spins;
        if ((spins & 1023u) == 0u && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
        if (spins > kSpinLimit) {
            __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
    }
    return true;
}

// Block barrier for LDS data only.  With a global -> LDS (LDS-DMA) load in
// flight __syncthreads() compiles to `s_waitcnt vmcnt(0) lgkmcnt(0); s_barrier`
// (the DMA counts as an LDS write): the backward's h_{t-1} / x_t rows, issued
// before the hand-off wait for the off-path weight gradients, then completed
// in front of the step's partial-dh loads -- one more memory round trip on the
// recurrence of the block that arrives last.  Those rows are waited for
// explicitly where they are read.
#ifndef VN_ROWS_RAWBAR
#define VN_ROWS_RAWBAR 1
#endif
#ifndef VN_ROWS_PRELOAD
#define VN_ROWS_PRELOAD 1
#endif
#ifndef VN_ROWS_FLAGS
#define VN_ROWS_FLAGS 1
#endif
__device__ __forceinline__ void lds_barrier() {
#if VN_ROWS_RAWBAR
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#else
    __syncthreads();
#endif
}

// after this block's payload stores: drain (every wave), block barrier, one add
__device__ __forceinline__ void publish(uint32_t *cnt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct RowsFwd {
    const float *x;          // [L][B][D]
    const float *w_ih;       // [2][4H][D]
    const float *w_hh;       // [2][4H][H]
    const float *bias;       // [2][4H]  (b_ih + b_hh)
    const float *h_store;    // [T][2][N][H]  the rollout buffer's LSTM states
    const float *c_store;
    const int32_t *env;      // [L][B]  the row's env at each step
    const uint8_t *start;    // [L][B]  1: a sequence starts at this step
    const float *keep;       // [L][B]  1 - episode_start of that sample
    float *hout;             // [2][L][B][H]  h_t (the handed-off payload)
    float *hprev;            // [2][L][B][H]  the h_{t-1} each step used
    float *cprev, *cnew;     // [2][L][B][H]
    float *act;              // [2][L][B][4H] i, f, g, o
    uint32_t *cnt;           // [2 * NT * CSTRIDE] group counters, a line each (zeroed per call)
    int32_t *err;
    int64_t n_env;
    int L, B, NT;
    int prio;                // 16-unit layout: issue priority on the hand-off path (VOXNAV_ROWS_PRIO)
    uint32_t *diag;          // diagnostics (NULL): placement + per-step clocks
};

template <int D, int H>
__global__ __launch_bounds__(256, 1) void lstm_rows_fwd_kernel(RowsFwd a) {
    constexpr int NCX = D / 8, NCH = H / 8, NC = NCX + NCH;
    constexpr int XP = D + 4, HP = H + 4, GP = 36;
    static_assert(D % 8 == 0 && H == NUB * UBK, "shape");
    __shared__ __attribute__((aligned(16))) float xs[2][RW][XP];
    __shared__ __attribute__((aligned(16))) float hsl[RW][HP];
    __shared__ __attribute__((aligned(16))) float gts[4][RW][GP];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);   // this wave's gate
    const int hh = lane >> 5, cl = lane & 31;
    const int G = 2 * a.NT;
    const int ub = (int)blockIdx.x / G, g = (int)blockIdx.x - ub * G;   // blocks of a group: equal index mod 8 when G % 8 == 0
    const int l = g / a.NT, rt = g - l * a.NT;
    const int row0 = rt * RW, u0 = ub * UBK;
    const int B = a.B, L = a.L;

    // resident weights: B operand of gate wv, unit u0 + cl, k = 8 ch + 4 hh + j
    float4 wr[NC];
    {
        const float *wi = a.w_ih + ((size_t)l * 4 * H + (size_t)wv * H + u0 + cl) * D;
        const float *wh = a.w_hh + ((size_t)l * 4 * H + (size_t)wv * H + u0 + cl) * H;
#pragma unroll
        for (int ch = 0; ch < NC; ++ch) {
            const int k = 8 * ch + 4 * hh;
            wr[ch] = ch < NCX ? *reinterpret_cast<const float4 *>(wi + k)
                              : *reinterpret_cast<const float4 *>(wh + (k - D));
        }
    }
    // epilogue mapping: row er of the tile, units u0 + 4 eq .. + 3
    const int er = tid >> 3, eq = tid & 7;
    const int erow = row0 + er;
    const bool elive = erow < B;
    const int eu = u0 + 4 * eq;
    float4 bs[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) bs[q] = *reinterpret_cast<const float4 *>(a.bias + (size_t)l * 4 * H + q * H + eu);
    float4 cc = f4(0.0f);

    const __amdgpu_buffer_rsrc_t hrs =
        __builtin_amdgcn_make_buffer_rsrc(a.hout, 0, (int)((size_t)2 * L * B * H * 4), 0x00020000);
    uint32_t *cnt = a.cnt + (size_t)g * CSTRIDE;

    // x rows of a step: RW x D floats, float4 f -> (row f / (D/4), col 4 (f % (D/4)))
    constexpr int XF = RW * D / 4, XPT = (XF + 255) / 256;
    auto load_x = [&](int t, float4 *r) {
#pragma unroll
        for (int i = 0; i < XPT; ++i) {
            const int f = tid + 256 * i;
            const int rr = f / (D / 4), c4 = f - rr * (D / 4);
            r[i] = (f < XF && row0 + rr < B)
                       ? *reinterpret_cast<const float4 *>(a.x + ((size_t)t * B + row0 + rr) * D + 4 * c4)
                       : f4(0.0f);
        }
    };
    auto store_x = [&](int buf, const float4 *r) {
#pragma unroll
        for (int i = 0; i < XPT; ++i) {
            const int f = tid + 256 * i;
            const int rr = f / (D / 4), c4 = f - rr * (D / 4);
            if (f < XF) *reinterpret_cast<float4 *>(&xs[buf][rr][4 * c4]) = r[i];
        }
    };
    {
        float4 r[XPT];
        load_x(0, r);
        store_x(0, r);
    }
    __syncthreads();

#if VN_ROWS_FLAGS
    // the tile's sequence-start flags, double-buffered: step t reads stf[t & 1];
    // step t + 1's are loaded at the top of step t and written to LDS after the
    // step's h loads (whose wait completes them).  Consumed at the top of the
    // same step (below), the load was waited for at once -- together with the
    // previous step's 7 result stores -- in front of the x part.
    __shared__ uint8_t stf2[2][RW];
    if (tid < RW) stf2[0][tid] = row0 + tid < B ? 1 : 0;   // step 0: every row starts
    const int frow = min(row0 + (tid & (RW - 1)), B - 1);
#else
    __shared__ uint8_t stf[RW];       // the tile's sequence-start flags of the step
    // loaded a step ahead (a load consumed in the same step stalled the x part)
    uint8_t st_next = (tid < RW && row0 + tid < B) ? 1 : 0;
#endif
    for (int t = 0; t < L; ++t) {
        const int xb = t & 1;
#if VN_ROWS_FLAGS
        const uint8_t *stf = stf2[t & 1];
        const uint8_t st_ld = a.start[(size_t)min(t + 1, L - 1) * B + frow];
#else
        if (tid < RW) stf[tid] = st_next;
        if (tid < RW && t + 1 < L) st_next = (row0 + tid < B && a.start[(size_t)(t + 1) * B + row0 + tid]) ? 1 : 0;
#endif
        float4 xn[XPT];
        if (t + 1 < L) load_x(t + 1, xn);
        // the x part of the product (needs nothing from the group)
        f32x16_t acc = zero16();
#pragma unroll
        for (int ch = 0; ch < NCX; ++ch) {
            const float4 av = *reinterpret_cast<const float4 *>(&xs[xb][cl][8 * ch + 4 * hh]);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, wr[ch].x, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, wr[ch].y, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, wr[ch].z, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, wr[ch].w, acc, 0, 0, 0);
        }
        // h_{t-1} of the tile's rows: the group's output of step t-1 (sc1 loads
        // after the counter shows all 8 blocks done), or the stored state at a
        // sequence start
        if (t > 0) {
            if (tid == 0) wait_ge(cnt, (uint32_t)(NUB * t), a.err);
            __syncthreads();
        }
        // every row's h_{t-1} from the group's output, all 8 loads in flight at
        // once (rows past B read row B - 1; a step-0 tile reads nothing) ...
        float4 hv[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int f = tid + 256 * i;
            const int rr = f >> 6, c4 = f & 63;          // H / 4 = 64 float4 per row
            const int row = min(row0 + rr, B - 1);
            hv[i] = t > 0 ? ld_sc1(hrs, (uint32_t)((((size_t)l * L + (t - 1)) * B + row) * H + 4 * c4) * 4u)
                          : f4(0.0f);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int f = tid + 256 * i;
            *reinterpret_cast<float4 *>(&hsl[f >> 6][4 * (f & 63)]) = hv[i];
        }
#if VN_ROWS_FLAGS
        if (tid < RW) stf2[(t + 1) & 1][tid] = (t + 1 < L && row0 + tid < B && st_ld) ? 1 : 0;
#endif
        __syncthreads();
        // ... then the rows that start a sequence at t (all of them at t = 0)
        // take the buffer's stored state x keep: one row per 64 threads
#pragma unroll
        for (int i = 0; i < RW / 4; ++i) {
            const int rr = (tid >> 6) + 4 * i, c4 = tid & 63;
            const int row = row0 + rr;
            if (stf[rr]) {
                const size_t o = (size_t)t * B + row;
                const float4 sv = *reinterpret_cast<const float4 *>(
                    a.h_store + (((size_t)t * 2 + l) * a.n_env + a.env[o]) * H + 4 * c4);
                *reinterpret_cast<float4 *>(&hsl[rr][4 * c4]) = sv * f4(a.keep[o]);
            } else if (row >= B) {
                *reinterpret_cast<float4 *>(&hsl[rr][4 * c4]) = f4(0.0f);
            }
        }
        __syncthreads();
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
            const float4 av = *reinterpret_cast<const float4 *>(&hsl[cl][8 * ch + 4 * hh]);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, wr[NCX + ch].x, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, wr[NCX + ch].y, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, wr[NCX + ch].z, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, wr[NCX + ch].w, acc, 0, 0, 0);
        }
        if (t + 1 < L) store_x(xb ^ 1, xn);
        // gate tile -> LDS: register v = row 8 (v / 4) + 4 hh + v % 4, unit cl
#pragma unroll
        for (int v = 0; v < 16; ++v) gts[wv][8 * (v >> 2) + 4 * hh + (v & 3)][cl] = acc[v];
        __syncthreads();
        if (elive) {
            const size_t o = (size_t)t * B + erow;
            float4 pre[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) pre[q] = *reinterpret_cast<const float4 *>(&gts[q][er][4 * eq]) + bs[q];
            float4 cp = cc;
            if (stf[er]) {
                const float k = a.keep[o];
                cp = *reinterpret_cast<const float4 *>(a.c_store + (((size_t)t * 2 + l) * a.n_env + a.env[o]) * H + eu) *
                     f4(k);
            }
            float4 ig, fg, gg, og, cn, hn;
#define VN_CELL(c)                                 \
    ig.c = sigm(pre[0].c);                         \
    fg.c = sigm(pre[1].c);                         \
    gg.c = tanh_fast(pre[2].c);                        \
    og.c = sigm(pre[3].c);                         \
    {                                              \
        const float fc_ = fg.c * cp.c, ig_ = ig.c * gg.c; \
        cn.c = fc_ + ig_;                          \
    }                                              \
    hn.c = og.c * tanh_fast(cn.c);
            VN_CELL(x) VN_CELL(y) VN_CELL(z) VN_CELL(w)
#undef VN_CELL
            cc = cn;
            const size_t so = (((size_t)l * L + t) * B + erow) * H + eu;
            st_sc1(hrs, (uint32_t)(so * 4u), hn);          // the payload first
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            *reinterpret_cast<float4 *>(a.cnew + so) = cn;
            *reinterpret_cast<float4 *>(a.cprev + so) = cp;
            *reinterpret_cast<float4 *>(a.hprev + so) = *reinterpret_cast<const float4 *>(&hsl[er][eu]);
            float *pa = a.act + (((size_t)l * L + t) * B + erow) * 4 * H + eu;
            *reinterpret_cast<float4 *>(pa) = ig;
            *reinterpret_cast<float4 *>(pa + H) = fg;
            *reinterpret_cast<float4 *>(pa + 2 * H) = gg;
            *reinterpret_cast<float4 *>(pa + 3 * H) = og;
        }
        // h_t published (the payload stores were drained above; the barrier
        // inside publish orders every wave's drain before the one add)
        __syncthreads();
        if (tid == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---------------------------------------------------------------------------
// Two blocks per CU (the default).  The same recurrence with HALF the units
// per block (16: 64 gate columns) on v_mfma_f32_16x16x4_f32, so the grid is
// 2 x 16 x R/32 = 512 blocks, two resident per CU.  A group (LSTM, row tile)
// is now 16 blocks; the two blocks sharing a CU are different groups (the
// grid's second half takes the other LSTM of the same row tile), i.e. two
// independent recurrences, so one's MFMAs run while the other's hand-off is
// in flight -- in the one-block-per-CU layout each SIMD held one wave and
// idled for every hand-off.  Same payloads, same protocol; a group's counter
// counts 16 adds per step.
// ---------------------------------------------------------------------------
constexpr int UB2 = 16;     // units per block
constexpr int NUB2 = 16;    // unit blocks per LSTM

typedef __attribute__((ext_vector_type(4))) float f32x4_t;

__device__ __forceinline__ f32x4_t zero4() { return f32x4_t{0.0f, 0.0f, 0.0f, 0.0f}; }
__device__ __forceinline__ float2 operator+(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 operator*(float2 a, float2 b) { return make_float2(a.x * b.x, a.y * b.y); }
__device__ __forceinline__ float2 f2(float a) { return make_float2(a, a); }

__device__ __forceinline__ void st_sc1_b64(__amdgpu_buffer_rsrc_t rs, uint32_t off, float2 v) {
    __attribute__((ext_vector_type(2))) float w = {v.x, v.y};
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) uint32_t, w), rs, off,
                                          0, 16);
}
__device__ __forceinline__ float2 ld_sc1_b64(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
    const auto u = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 16);
    const auto v = __builtin_bit_cast(__attribute__((ext_vector_type(2))) float, u);
    return make_float2(v[0], v[1]);
}

// block -> (unit block, group): the first half of the grid takes unit blocks
// 0..7 of every group, the second half 8..15 with the LSTMs swapped, so block
// b and block b + grid/2 (which the dispatcher places on the same CU,
// scripts/rows_diag.py) belong to different recurrences.  (They still run in
// phase: a plain order and a delayed start of LSTM 1 measured the same.)
// Blocks of one group share blockIdx mod 8 (one XCD's L2 carries the group's
// hand-offs) when NT % 8 == 0.
__device__ __forceinline__ void rows2_map(int NT, int &ub, int &g) {
    const int G = 2 * NT, half = (NUB2 / 2) * G;
    int b = (int)blockIdx.x;
    const bool second = b >= half;
    if (second) b -= half;
    ub = b / G + (second ? NUB2 / 2 : 0);
    g = b - (b / G) * G;
    if (second) g = (g + NT) % G;
}

template <int D, int H>
__global__ __launch_bounds__(256, 2) void lstm_rows_fwd2_kernel(RowsFwd a) {
    constexpr int NCX = D / 16, NCH = H / 16, NC = NCX + NCH;   // 16-deep k chunks
    constexpr int XP = D + 4, HP = H + 4, GP = UB2 + 4;
    static_assert(D % 16 == 0 && H == NUB2 * UB2, "shape");
    __shared__ __attribute__((aligned(16))) float xs[2][RW][XP];
    __shared__ __attribute__((aligned(16))) float hsl[RW][HP];
    __shared__ __attribute__((aligned(16))) float gts[4][RW][GP];
#if !VN_ROWS_FLAGS
    __shared__ uint8_t stf[RW];
#endif
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);   // this wave's gate
    const int q = lane >> 4, ci = lane & 15;
    int ub, g;
    rows2_map(a.NT, ub, g);
    if (a.diag && tid == 0) {
        a.diag[2 * blockIdx.x] = __builtin_amdgcn_s_getreg((31 << 11) | 4);        // HW_ID
        a.diag[2 * blockIdx.x + 1] = __builtin_amdgcn_s_getreg((31 << 11) | 20);   // XCC_ID
    }
    const int l = g / a.NT, rt = g - l * a.NT;
    const int row0 = rt * RW, u0 = ub * UB2;
    const int B = a.B, L = a.L;

    // resident weights: B operand of gate wv, unit u0 + ci; chunk c, step jj
    // takes k = 16 c + 4 q + jj (the A reads use the same k order)
    float4 wr[NC];
    {
        const float *wi = a.w_ih + ((size_t)l * 4 * H + (size_t)wv * H + u0 + ci) * D;
        const float *wh = a.w_hh + ((size_t)l * 4 * H + (size_t)wv * H + u0 + ci) * H;
#pragma unroll
        for (int c = 0; c < NC; ++c)
            wr[c] = c < NCX ? *reinterpret_cast<const float4 *>(wi + 16 * c + 4 * q)
                            : *reinterpret_cast<const float4 *>(wh + 16 * (c - NCX) + 4 * q);
    }
    // epilogue mapping: row er of the tile, units u0 + 2 eq, + 1
    const int er = tid >> 3, eq = tid & 7;
    const int erow = row0 + er;
    const bool elive = erow < B;
    const int eu = u0 + 2 * eq;
    float2 bs[4];
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) bs[gq] = *reinterpret_cast<const float2 *>(a.bias + (size_t)l * 4 * H + gq * H + eu);
    float2 cc = f2(0.0f);

    const __amdgpu_buffer_rsrc_t hrs =
        __builtin_amdgcn_make_buffer_rsrc(a.hout, 0, (int)((size_t)2 * L * B * H * 4), 0x00020000);
    uint32_t *cnt = a.cnt + (size_t)g * CSTRIDE;

    constexpr int XF = RW * D / 4, XPT = (XF + 255) / 256;
    auto load_x = [&](int t, float4 *r) {
#pragma unroll
        for (int i = 0; i < XPT; ++i) {
            const int f = tid + 256 * i;
            const int rr = f / (D / 4), c4 = f - rr * (D / 4);
            r[i] = (f < XF && row0 + rr < B)
                       ? *reinterpret_cast<const float4 *>(a.x + ((size_t)t * B + row0 + rr) * D + 4 * c4)
                       : f4(0.0f);
        }
    };
    auto store_x = [&](int buf, const float4 *r) {
#pragma unroll
        for (int i = 0; i < XPT; ++i) {
            const int f = tid + 256 * i;
            const int rr = f / (D / 4), c4 = f - rr * (D / 4);
            if (f < XF) *reinterpret_cast<float4 *>(&xs[buf][rr][4 * c4]) = r[i];
        }
    };
    {
        float4 r[XPT];
        load_x(0, r);
        store_x(0, r);
    }
    __syncthreads();

#define VN_DMARK(k_)                                                                          \
    if (a.diag && tid == 0)                                                                   \
        a.diag[2 * gridDim.x + ((size_t)blockIdx.x * L + t) * 8 + (k_)] = (uint32_t)__builtin_amdgcn_s_memrealtime();
    // the tile's sequence-start flags, loaded a step ahead (a load consumed in
    // the same step stalled the x part behind its round trip)
#if VN_ROWS_FLAGS
    // (double-buffered in LDS as in lstm_rows_fwd_kernel)
    __shared__ uint8_t stf2[2][RW];
    if (tid < RW) stf2[0][tid] = row0 + tid < B ? 1 : 0;
    const int frow = min(row0 + (tid & (RW - 1)), B - 1);
#else
    uint8_t st_next = (tid < RW && row0 + tid < B) ? 1 : 0;
#endif
    for (int t = 0; t < L; ++t) {
        const int xb = t & 1;
        VN_DMARK(0);
#if VN_ROWS_FLAGS
        const uint8_t *stf = stf2[t & 1];
        const uint8_t st_ld = a.start[(size_t)min(t + 1, L - 1) * B + frow];
#else
        if (tid < RW) stf[tid] = st_next;
        if (tid < RW && t + 1 < L) st_next = (row0 + tid < B && a.start[(size_t)(t + 1) * B + row0 + tid]) ? 1 : 0;
#endif
        float4 xn[XPT];
        if (t + 1 < L) load_x(t + 1, xn);
        // the x part (needs nothing from the group): rows ci and 16 + ci
        f32x4_t acc0 = zero4(), acc1 = zero4();
#pragma unroll
        for (int c = 0; c < NCX; ++c) {
            const float4 a0 = *reinterpret_cast<const float4 *>(&xs[xb][ci][16 * c + 4 * q]);
            const float4 a1 = *reinterpret_cast<const float4 *>(&xs[xb][16 + ci][16 * c + 4 * q]);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, wr[c].x, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, wr[c].x, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, wr[c].y, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, wr[c].y, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, wr[c].z, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, wr[c].z, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, wr[c].w, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, wr[c].w, acc1, 0, 0, 0);
        }
        VN_DMARK(1);
        if (a.prio) __builtin_amdgcn_s_setprio(2);   // the hand-off path: wait, rows, products, cell, publish
        if (t > 0) {
            if (tid == 0) wait_ge(cnt, (uint32_t)(NUB2 * t), a.err);
            __syncthreads();
        }
        VN_DMARK(2);
        float4 hv[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int f = tid + 256 * i;
            const int rr = f >> 6, c4 = f & 63;
            const int row = min(row0 + rr, B - 1);
            hv[i] = t > 0 ? ld_sc1(hrs, (uint32_t)((((size_t)l * L + (t - 1)) * B + row) * H + 4 * c4) * 4u)
                          : f4(0.0f);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int f = tid + 256 * i;
            *reinterpret_cast<float4 *>(&hsl[f >> 6][4 * (f & 63)]) = hv[i];
        }
#if VN_ROWS_FLAGS
        if (tid < RW) stf2[(t + 1) & 1][tid] = (t + 1 < L && row0 + tid < B && st_ld) ? 1 : 0;
#endif
        __syncthreads();
        VN_DMARK(3);
#pragma unroll
        for (int i = 0; i < RW / 4; ++i) {
            const int rr = (tid >> 6) + 4 * i, c4 = tid & 63;
            const int row = row0 + rr;
            if (stf[rr]) {
                const size_t o = (size_t)t * B + row;
                const float4 sv = *reinterpret_cast<const float4 *>(
                    a.h_store + (((size_t)t * 2 + l) * a.n_env + a.env[o]) * H + 4 * c4);
                *reinterpret_cast<float4 *>(&hsl[rr][4 * c4]) = sv * f4(a.keep[o]);
            } else if (row >= B) {
                *reinterpret_cast<float4 *>(&hsl[rr][4 * c4]) = f4(0.0f);
            }
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const float4 a0 = *reinterpret_cast<const float4 *>(&hsl[ci][16 * c + 4 * q]);
            const float4 a1 = *reinterpret_cast<const float4 *>(&hsl[16 + ci][16 * c + 4 * q]);
            const float4 w = wr[NCX + c];
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, w.x, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, w.x, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, w.y, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, w.y, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, w.z, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, w.z, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, w.w, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, w.w, acc1, 0, 0, 0);
        }
        if (t + 1 < L) store_x(xb ^ 1, xn);
        // gate tiles -> LDS: register r = row 4 q + r (+ 16 for acc1), unit ci
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            gts[wv][4 * q + r][ci] = acc0[r];
            gts[wv][16 + 4 * q + r][ci] = acc1[r];
        }
        __syncthreads();
        VN_DMARK(4);
        if (elive) {
            const size_t o = (size_t)t * B + erow;
            float2 pre[4];
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) pre[gq] = *reinterpret_cast<const float2 *>(&gts[gq][er][2 * eq]) + bs[gq];
            float2 cp = cc;
            if (stf[er]) {
                const float k = a.keep[o];
                cp = *reinterpret_cast<const float2 *>(a.c_store + (((size_t)t * 2 + l) * a.n_env + a.env[o]) * H + eu) *
                     f2(k);
            }
            float2 ig, fg, gg, og, cn, hn;
#define VN_CELL2(c)                                       \
    ig.c = sigm(pre[0].c);                                \
    fg.c = sigm(pre[1].c);                                \
    gg.c = tanh_fast(pre[2].c);                           \
    og.c = sigm(pre[3].c);                                \
    {                                                     \
        const float fc_ = fg.c * cp.c, ig_ = ig.c * gg.c; \
        cn.c = fc_ + ig_;                                 \
    }                                                     \
    hn.c = og.c * tanh_fast(cn.c);
            VN_CELL2(x) VN_CELL2(y)
#undef VN_CELL2
            cc = cn;
            const size_t so = (((size_t)l * L + t) * B + erow) * H + eu;
            st_sc1_b64(hrs, (uint32_t)(so * 4u), hn);      // the payload first
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            *reinterpret_cast<float2 *>(a.cnew + so) = cn;
            *reinterpret_cast<float2 *>(a.cprev + so) = cp;
            *reinterpret_cast<float2 *>(a.hprev + so) = *reinterpret_cast<const float2 *>(&hsl[er][eu]);
            float *pa = a.act + (((size_t)l * L + t) * B + erow) * 4 * H + eu;
            *reinterpret_cast<float2 *>(pa) = ig;
            *reinterpret_cast<float2 *>(pa + H) = fg;
            *reinterpret_cast<float2 *>(pa + 2 * H) = gg;
            *reinterpret_cast<float2 *>(pa + 3 * H) = og;
        }
        VN_DMARK(5);
        __syncthreads();
        if (tid == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a.prio) __builtin_amdgcn_s_setprio(0);
        VN_DMARK(6);
    }
#undef VN_DMARK
}

struct RowsBwd {
    const float *dh_out;     // [2][L][B][H]
    const float *w_hh;       // [2][4H][H]
    const float *act;        // [2][L][B][4H]
    const float *cprev, *cnew;
    const float *hprev;      // [2][L][B][H]  the h_{t-1} each forward step used
    const float *x;          // [L][B][D]
    const uint8_t *start;    // [L][B]
    float *dG;               // [2][L][B][4H] out (may be NULL)
    float *part;             // [2 slots][2][NT][NUB][RW][H] partial dh
    float *wpart;            // [NT][2][4H][H + D] per-row-tile [dW_hh | dW_ih]
    float *bpart;            // [NT][2][4H] per-row-tile db
    uint32_t *cnt;           // [2 * NT * CSTRIDE]
    int32_t *err;
    int L, B, NT;
    int prio;
};

// Backward.  Besides the recurrence, each block accumulates the weight
// gradients of its 128 gate rows over all steps and its 32 rows: dW_hh +=
// dG_t^T h_{t-1}, dW_ih += dG_t^T x_t, db += sum dG_t, on the matrix cores
// with the accumulators resident (wave w: gate w's 32 rows, 8 + 3 tiles of
// 32 x 32).  Those products do not feed the recurrence, so they are issued
// after the step's partial is published and run while the group's next
// hand-off is in flight.  Per-row-tile partials are summed (fixed order) by
// rows_wsum_kernel.
template <int D, int H>
__global__ __launch_bounds__(256, 1) void lstm_rows_bwd_kernel(RowsBwd a) {
    constexpr int GC = 4 * UBK;   // this block's gate columns (K of the partial product)
    constexpr int NCK = GC / 8;   // 16 chunks
    constexpr int DP = GC + 4, PP = H + 4, XP = 96;   // xs padded to 3 tiles of 32 (zeros past D)
    constexpr int NXT = (D + 31) / 32;                 // dW_ih column tiles
    static_assert(H == NUB * UBK && D <= XP && D % 4 == 0 && H == 256 && D / 4 <= 64, "shape: a row per wave load");
    __shared__ __attribute__((aligned(16))) float dgs[RW][DP];
    __shared__ __attribute__((aligned(16))) float pst[RW][PP];
    __shared__ __attribute__((aligned(16))) float hsl[RW][PP];
    __shared__ __attribute__((aligned(16))) float xsl[RW][XP];
    __shared__ uint8_t stf[RW];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);   // output units 64 wv .. + 63; dW gate wv
    const int hh = lane >> 5, cl = lane & 31;
    const int G = 2 * a.NT;
    const int ub = (int)blockIdx.x / G, g = (int)blockIdx.x - ub * G;
    const int l = g / a.NT, rt = g - l * a.NT;
    const int row0 = rt * RW, u0 = ub * UBK;
    const int B = a.B, L = a.L;

    // resident W_hh slice: B operand [k = gate * 32 + unit32][n = 64 wv + 32 j + cl],
    // k = 8 ch + 4 hh + jj
    float4 wb[2][NCK];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ch = 0; ch < NCK; ++ch) {
            float v[4];
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                const int k = 8 * ch + 4 * hh + jj;
                const int grow = (k >> 5) * H + u0 + (k & 31);
                v[jj] = a.w_hh[((size_t)l * 4 * H + grow) * H + 64 * wv + 32 * j + cl];
            }
            wb[j][ch] = make_float4(v[0], v[1], v[2], v[3]);
        }
    const int er = tid >> 3, eq = tid & 7;
    const int erow = row0 + er;
    const bool elive = erow < B;
    const int eu = u0 + 4 * eq;
    float4 dc = f4(0.0f);
    float4 dbs[4] = {f4(0.0f), f4(0.0f), f4(0.0f), f4(0.0f)};
    f32x16_t wacc[8], xacc[NXT];
#pragma unroll
    for (int j = 0; j < 8; ++j) wacc[j] = zero16();
#pragma unroll
    for (int j = 0; j < NXT; ++j) xacc[j] = zero16();
    const size_t slot_f = (size_t)2 * a.NT * NUB * RW * H;     // floats per slot
    const __amdgpu_buffer_rsrc_t prs =
        __builtin_amdgcn_make_buffer_rsrc(a.part, 0, (int)(2 * slot_f * 4), 0x00020000);
    uint32_t *cnt = a.cnt + (size_t)g * CSTRIDE;
    auto pofs = [&](int slot, int ubb, int row, int unit) -> uint32_t {   // byte offset in part
        return (uint32_t)(((size_t)slot * slot_f + ((((size_t)l * a.NT + rt) * NUB + ubb) * RW + row) * H + unit) * 4u);
    };
    // zero the padding columns of xs once (never written by the staging)
#pragma unroll
    for (int i = tid; i < RW * (XP - D); i += 256) xsl[i / (XP - D)][D + i % (XP - D)] = 0.0f;

    for (int s = 0; s < L; ++s) {
        const int t = L - 1 - s;
        // the step's sequence-start flag, loaded ahead of the hand-off wait
        const bool st_ld = !elive || t == 0 || a.start[(size_t)t * B + erow];
        // the step's h_{t-1} and x_t rows (the weight gradients' B operands; rows
        // past B clamped: their dG is zero), copied global -> LDS directly (no
        // registers: the kernel sits at the VGPR cap, and register staging made
        // the compiler serialise the loads), issued before the hand-off wait so
        // they land while it is awaited (the previous step's weight-gradient
        // reads of hsl / xsl ended at its closing barrier).  One wave
        // instruction = one row.
#pragma unroll
        for (int i = 0; i < RW / 4; ++i) {
            const int rr = (RW / 4) * wv + i;
            const int row = min(row0 + rr, B - 1);
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)(a.hprev + (((size_t)l * L + t) * B + row) * H + 4 * lane),
                (__attribute__((address_space(3))) void *)&hsl[rr][0], 16, 0, 0);
            if (lane < D / 4)
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)(a.x + ((size_t)t * B + row) * D + 4 * lane),
                    (__attribute__((address_space(3))) void *)&xsl[rr][0], 16, 0, 0);
        }
        if (s > 0) {
            if (tid == 0) wait_ge(cnt, (uint32_t)(NUB * s), a.err);
            __syncthreads();
        }
        float4 dG4[4] = {f4(0.0f), f4(0.0f), f4(0.0f), f4(0.0f)};
        bool st = true;
        if (elive) {
            st = st_ld;
            float4 dhr = f4(0.0f);
            if (s > 0) {
                // the 8 partials of step t+1 (sc1 loads), summed in unit-block order
#pragma unroll
                for (int k = 0; k < NUB; ++k) dhr = dhr + ld_sc1(prs, pofs((t + 1) & 1, k, er, eu));
            }
            const size_t so = (((size_t)l * L + t) * B + erow) * H + eu;
            const float4 dh = *reinterpret_cast<const float4 *>(a.dh_out + so) + dhr;
            const float *pa = a.act + (((size_t)l * L + t) * B + erow) * 4 * H + eu;
            const float4 ig = *reinterpret_cast<const float4 *>(pa), fg = *reinterpret_cast<const float4 *>(pa + H);
            const float4 gg = *reinterpret_cast<const float4 *>(pa + 2 * H);
            const float4 og = *reinterpret_cast<const float4 *>(pa + 3 * H);
            const float4 cp = *reinterpret_cast<const float4 *>(a.cprev + so);
            const float4 cn = *reinterpret_cast<const float4 *>(a.cnew + so);
#define VN_CELLB(c)                                                   \
    {                                                                 \
        const float tc = tanh_fast(cn.c);                                 \
        const float dtc = dh.c * og.c;                                \
        const float dcc = dc.c + dtc * (1.0f - tc * tc);              \
        dG4[0].c = dcc * gg.c * (ig.c * (1.0f - ig.c));               \
        dG4[1].c = dcc * cp.c * (fg.c * (1.0f - fg.c));               \
        dG4[2].c = dcc * ig.c * (1.0f - gg.c * gg.c);                 \
        dG4[3].c = dh.c * tc * (og.c * (1.0f - og.c));                \
        dc.c = dcc * fg.c;                                            \
    }
            VN_CELLB(x) VN_CELLB(y) VN_CELLB(z) VN_CELLB(w)
#undef VN_CELLB
            if (st) dc = f4(0.0f);   // c_{t-1} of this row came from the buffer
            if (a.dG) {
                float *pg = a.dG + (((size_t)l * L + t) * B + erow) * 4 * H + eu;
#pragma unroll
                for (int q = 0; q < 4; ++q) *reinterpret_cast<float4 *>(pg + q * H) = dG4[q];
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) dbs[q] = dbs[q] + dG4[q];
        }
        // dG (the partial product's and the weight gradients' A operand) and
        // the sequence-start flags to LDS
#pragma unroll
        for (int q = 0; q < 4; ++q) *reinterpret_cast<float4 *>(&dgs[er][q * UBK + 4 * eq]) = dG4[q];
        if (eq == 0) stf[er] = st ? 1 : 0;
        __syncthreads();
        if (t > 0) {
            f32x16_t acc0 = zero16(), acc1 = zero16();
#pragma unroll
            for (int ch = 0; ch < NCK; ++ch) {
                const float4 av = *reinterpret_cast<const float4 *>(&dgs[cl][8 * ch + 4 * hh]);
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, wb[0][ch].x, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, wb[1][ch].x, acc1, 0, 0, 0);
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, wb[0][ch].y, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, wb[1][ch].y, acc1, 0, 0, 0);
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, wb[0][ch].z, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, wb[1][ch].z, acc1, 0, 0, 0);
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, wb[0][ch].w, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, wb[1][ch].w, acc1, 0, 0, 0);
            }
            // rows whose step t starts a sequence pass no gradient back
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const int r = 8 * (v >> 2) + 4 * hh + (v & 3);
                const bool cut = stf[r] != 0;
                pst[r][64 * wv + cl] = cut ? 0.0f : acc0[v];
                pst[r][64 * wv + 32 + cl] = cut ? 0.0f : acc1[v];
            }
            __syncthreads();
            // the partial [RW][H] of this block: 16-B sc1 stores, then publish
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int f = tid + 256 * i;
                const int rr = f >> 6, c4 = f & 63;
                st_sc1(prs, pofs(t & 1, ub, rr, 4 * c4), *reinterpret_cast<const float4 *>(&pst[rr][4 * c4]));
            }
            publish(cnt);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // weight gradients of gate wv's 32 rows (while the next hand-off is in flight):
        // A = dG^T [gate unit][row], B = h_{t-1} / x_t [row][col], K = the 32 rows
#pragma unroll
        for (int ks = 0; ks < RW / 2; ++ks) {
            const int r = 2 * ks + hh;
            const float av = dgs[r][wv * UBK + cl];
#pragma unroll
            for (int j = 0; j < 8; ++j)
                wacc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, hsl[r][32 * j + cl], wacc[j], 0, 0, 0);
#pragma unroll
            for (int j = 0; j < NXT; ++j)
                xacc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, xsl[r][32 * j + cl], xacc[j], 0, 0, 0);
        }
        // every wave done reading hsl / xsl before the next step's copies into them
        __syncthreads();
        if (t == 0) break;
    }
    // per-row-tile weight-gradient partials: register v of a tile = gate row
    // 8 (v / 4) + 4 hh + v % 4 of gate wv's 32, column 32 j + cl
    float *wp = a.wpart + (((size_t)rt * 2 + l) * 4 * H) * (H + D);
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        const int grow = wv * H + u0 + 8 * (v >> 2) + 4 * hh + (v & 3);
        float *prow = wp + (size_t)grow * (H + D);
#pragma unroll
        for (int j = 0; j < 8; ++j) prow[32 * j + cl] = wacc[j][v];
#pragma unroll
        for (int j = 0; j < NXT; ++j)
            if (32 * j + cl < D) prow[H + 32 * j + cl] = xacc[j][v];
    }
    // db: the 32 rows' sums (threads of one eq hold a row each), reduced through LDS
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) *reinterpret_cast<float4 *>(&pst[er][q * UBK + 4 * eq]) = dbs[q];
    __syncthreads();
    if (tid < 4 * UBK) {
        float sum = 0.0f;
        for (int r = 0; r < RW; ++r) sum += pst[r][tid];
        a.bpart[((size_t)rt * 2 + l) * 4 * H + (tid >> 5) * H + u0 + (tid & 31)] = sum;
    }
}

// Backward, two blocks per CU (block = 16 units: 64 gate columns; the grid
// mapping of the forward).  The partial dh_{t-1} [32 rows][256 units] of a
// block is dG_t[:, its 64 gate columns] @ W_hh[those rows] on 16x16x4 tiles
// (wave w: units 64 w .. + 63, W_hh slice resident in 64 registers), staged
// through LDS 16 rows at a time; the weight gradients of gate wv's 16 rows
// over the 336 [h | x] columns are 21 16x16 accumulators.  Row order of the
// weight-gradient products: k-step s, lane group q takes row 4 q + (s & 3) +
// 16 (s >> 2) (the two rows a 32-lane LDS read touches sit 16 banks apart).
template <int D, int H>
__global__ __launch_bounds__(256, 2) void lstm_rows_bwd2_kernel(RowsBwd a) {
    constexpr int GC = 4 * UB2;                  // this block's gate columns (64)
    constexpr int DP = GC + 4, PP = H + 4, XP = D + 4;
    constexpr int NHT = H / 16, NXT = D / 16;    // weight-gradient column tiles (16 + 5)
    static_assert(H == NUB2 * UB2 && D % 16 == 0 && H == 256 && D / 4 <= 64, "shape: a row per wave load");
    __shared__ __attribute__((aligned(16))) float dgs[RW][DP];
    __shared__ __attribute__((aligned(16))) float pst[RW / 2][PP];
    __shared__ __attribute__((aligned(16))) float hsl[RW][PP];
    __shared__ __attribute__((aligned(16))) float xsl[RW][XP];
    __shared__ uint8_t stf[RW];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);   // partial: units 64 wv .. + 63; dW: gate wv
    // wave wv's cell operands [7][8 rows][16 units] (3.5 KB, inside pst)
    static_assert(4 * 7 * 8 * UB2 <= (RW / 2) * PP && UB2 == 16, "cell operands fit the pst area");
    float *const cops = &pst[0][0] + 7 * 8 * UB2 * wv;
    const int q = lane >> 4, ci = lane & 15;
    int ub, g;
    rows2_map(a.NT, ub, g);
    const int l = g / a.NT, rt = g - l * a.NT;
    const int row0 = rt * RW, u0 = ub * UB2;
    const int B = a.B, L = a.L;

    // resident W_hh slice: B operand [k = gate c * 16 + unit16][n = 64 wv + 16 j + ci],
    // chunk c = the gate, step jj: k = 16 c + 4 q + jj
    float4 wb[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            float v[4];
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                const int grow = c * H + u0 + 4 * q + jj;
                v[jj] = a.w_hh[((size_t)l * 4 * H + grow) * H + 64 * wv + 16 * j + ci];
            }
            wb[j][c] = make_float4(v[0], v[1], v[2], v[3]);
        }
    const int er = tid >> 3, eq = tid & 7;
    const int erow = row0 + er;
    const bool elive = erow < B;
    const int eu = u0 + 2 * eq;
    float2 dc = f2(0.0f);
    float2 dbs[4] = {f2(0.0f), f2(0.0f), f2(0.0f), f2(0.0f)};
    f32x4_t wacc[NHT + NXT];
#pragma unroll
    for (int j = 0; j < NHT + NXT; ++j) wacc[j] = zero4();
    const size_t slot_f = (size_t)2 * a.NT * NUB2 * RW * H;     // floats per slot
    const __amdgpu_buffer_rsrc_t prs =
        __builtin_amdgcn_make_buffer_rsrc(a.part, 0, (int)(2 * slot_f * 4), 0x00020000);
    uint32_t *cnt = a.cnt + (size_t)g * CSTRIDE;
    auto pofs = [&](int slot, int ubb, int row, int unit) -> uint32_t {   // byte offset in part
        return (uint32_t)(((size_t)slot * slot_f + ((((size_t)l * a.NT + rt) * NUB2 + ubb) * RW + row) * H + unit) * 4u);
    };

    for (int s = 0; s < L; ++s) {
        const int t = L - 1 - s;
        const bool st_ld = !elive || t == 0 || a.start[(size_t)t * B + erow];
        // the step's h_{t-1} and x_t rows (the weight gradients' B operands),
        // global -> LDS, issued before the hand-off wait
#pragma unroll
        for (int i = 0; i < RW / 4; ++i) {
            const int rr = (RW / 4) * wv + i;
            const int row = min(row0 + rr, B - 1);
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)(a.hprev + (((size_t)l * L + t) * B + row) * H + 4 * lane),
                (__attribute__((address_space(3))) void *)&hsl[rr][0], 16, 0, 0);
            if (lane < D / 4)
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)(a.x + ((size_t)t * B + row) * D + 4 * lane),
                    (__attribute__((address_space(3))) void *)&xsl[rr][0], 16, 0, 0);
        }
#if VN_ROWS_PRELOAD
        // the step's own cell operands (dh_out, the 4 gates, c_{t-1}, c_t) need
        // nothing from the group: global -> LDS before the hand-off wait, each
        // wave the 8 rows its cell lanes read (so no barrier is needed, only the
        // wave's own vmcnt), into the pst area (free until the partial below).
        // The partial-dh loads are then the one round trip after the wait (from
        // registers the compiler issued these behind that wait: 3 round trips;
        // the kernel sits at 256 VGPRs).  Lanes 0-31 / 32-63: operands 2 k, 2 k + 1.
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int op = 2 * k + (lane >> 5);
            const int row = min(row0 + 8 * wv + ((lane >> 2) & 7), B - 1);
            const size_t rb = ((size_t)l * L + t) * B + row;
            const float *src = op == 0 ? a.dh_out + rb * H : op == 5 ? a.cprev + rb * H : op == 6 ? a.cnew + rb * H
                                                                                               : a.act + rb * 4 * H + (op - 1) * H;
            if (op < 7)
                __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(src + u0 + 4 * (lane & 3)),
                                                 (__attribute__((address_space(3))) void *)(cops + 256 * k), 16, 0, 0);
        }
#endif
        if (a.prio) __builtin_amdgcn_s_setprio(2);   // the hand-off path up to the publish
        if (s > 0) {
            if (tid == 0) wait_ge(cnt, (uint32_t)(NUB2 * s), a.err);
            lds_barrier();
        }
        float2 dG2[4] = {f2(0.0f), f2(0.0f), f2(0.0f), f2(0.0f)};
        bool st = true;
        if (elive) {
            st = st_ld;
            float2 dhr = f2(0.0f);
            if (s > 0) {
#pragma unroll
                for (int k = 0; k < NUB2; ++k) dhr = dhr + ld_sc1_b64(prs, pofs((t + 1) & 1, k, er, eu));
            }
#if VN_ROWS_PRELOAD
            auto cop = [&](int op) {   // this lane's 2 units of operand op
                return *reinterpret_cast<const float2 *>(cops + 128 * op + 16 * (lane >> 3) + 2 * eq);
            };
            const float2 dh = cop(0) + dhr;
            const float2 ig = cop(1), fg = cop(2), gg = cop(3), og = cop(4), cp = cop(5), cn = cop(6);
#else
            const size_t so = (((size_t)l * L + t) * B + erow) * H + eu;
            const float2 dh = *reinterpret_cast<const float2 *>(a.dh_out + so) + dhr;
            const float *pa = a.act + (((size_t)l * L + t) * B + erow) * 4 * H + eu;
            const float2 ig = *reinterpret_cast<const float2 *>(pa), fg = *reinterpret_cast<const float2 *>(pa + H);
            const float2 gg = *reinterpret_cast<const float2 *>(pa + 2 * H);
            const float2 og = *reinterpret_cast<const float2 *>(pa + 3 * H);
            const float2 cp = *reinterpret_cast<const float2 *>(a.cprev + so);
            const float2 cn = *reinterpret_cast<const float2 *>(a.cnew + so);
#endif
#define VN_CELLB2(c)                                                  \
    {                                                                 \
        const float tc = tanh_fast(cn.c);                             \
        const float dtc = dh.c * og.c;                                \
        const float dcc = dc.c + dtc * (1.0f - tc * tc);              \
        dG2[0].c = dcc * gg.c * (ig.c * (1.0f - ig.c));               \
        dG2[1].c = dcc * cp.c * (fg.c * (1.0f - fg.c));               \
        dG2[2].c = dcc * ig.c * (1.0f - gg.c * gg.c);                 \
        dG2[3].c = dh.c * tc * (og.c * (1.0f - og.c));                \
        dc.c = dcc * fg.c;                                            \
    }
            VN_CELLB2(x) VN_CELLB2(y)
#undef VN_CELLB2
            if (st) dc = f2(0.0f);
            if (a.dG) {
                float *pg = a.dG + (((size_t)l * L + t) * B + erow) * 4 * H + eu;
#pragma unroll
                for (int gq = 0; gq < 4; ++gq) *reinterpret_cast<float2 *>(pg + gq * H) = dG2[gq];
            }
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) dbs[gq] = dbs[gq] + dG2[gq];
        }
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) *reinterpret_cast<float2 *>(&dgs[er][gq * UB2 + 2 * eq]) = dG2[gq];
        if (eq == 0) stf[er] = st ? 1 : 0;
        __syncthreads();   // (a full one: every wave's operand DMA has landed before pst is reused)
        if (t > 0) {
            f32x4_t acc[2][4];
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[h][j] = zero4();
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const float4 a0 = *reinterpret_cast<const float4 *>(&dgs[ci][16 * c + 4 * q]);
                const float4 a1 = *reinterpret_cast<const float4 *>(&dgs[16 + ci][16 * c + 4 * q]);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, wb[j][c].x, acc[0][j], 0, 0, 0);
                    acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, wb[j][c].x, acc[1][j], 0, 0, 0);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, wb[j][c].y, acc[0][j], 0, 0, 0);
                    acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, wb[j][c].y, acc[1][j], 0, 0, 0);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, wb[j][c].z, acc[0][j], 0, 0, 0);
                    acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, wb[j][c].z, acc[1][j], 0, 0, 0);
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, wb[j][c].w, acc[0][j], 0, 0, 0);
                    acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, wb[j][c].w, acc[1][j], 0, 0, 0);
                }
            }
            // the partial [RW][H], 16 rows at a time through LDS, 16-B sc1
            // stores; rows whose step t starts a sequence pass no gradient back
#pragma unroll
            for (int h = 0; h < 2; ++h) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const bool cut = stf[16 * h + 4 * q + r] != 0;
#pragma unroll
                    for (int j = 0; j < 4; ++j) pst[4 * q + r][64 * wv + 16 * j + ci] = cut ? 0.0f : acc[h][j][r];
                }
                __syncthreads();
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int f = tid + 256 * i;
                    const int rr = f >> 6, c4 = f & 63;
                    st_sc1(prs, pofs(t & 1, ub, 16 * h + rr, 4 * c4), *reinterpret_cast<const float4 *>(&pst[rr][4 * c4]));
                }
                if (h == 0) __syncthreads();
            }
            publish(cnt);
        }
        if (a.prio) __builtin_amdgcn_s_setprio(0);       // the weight gradients: off the critical path
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // weight gradients of gate wv's 16 rows: A = dG^T [unit][row], B = the
        // h_{t-1} | x_t rows [row][col], K = the 32 rows
#pragma unroll
        for (int s4 = 0; s4 < RW / 4; ++s4) {
            const int r = 4 * q + (s4 & 3) + 16 * (s4 >> 2);
            const float av = dgs[r][wv * UB2 + ci];
#pragma unroll
            for (int j = 0; j < NHT; ++j)
                wacc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, hsl[r][16 * j + ci], wacc[j], 0, 0, 0);
#pragma unroll
            for (int j = 0; j < NXT; ++j)
                wacc[NHT + j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, xsl[r][16 * j + ci], wacc[NHT + j], 0, 0, 0);
        }
        __syncthreads();
        if (t == 0) break;
    }
    // per-row-tile weight-gradient partials: register r of tile j = gate row
    // u0 + 4 q + r of gate wv, column 16 j + ci
    float *wp = a.wpart + (((size_t)rt * 2 + l) * 4 * H) * (H + D);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int grow = wv * H + u0 + 4 * q + r;
        float *prow = wp + (size_t)grow * (H + D);
#pragma unroll
        for (int j = 0; j < NHT; ++j) prow[16 * j + ci] = wacc[j][r];
#pragma unroll
        for (int j = 0; j < NXT; ++j) prow[H + 16 * j + ci] = wacc[NHT + j][r];
    }
    // db: the 32 rows' sums, reduced through LDS (dgs reused)
    __syncthreads();
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) *reinterpret_cast<float2 *>(&dgs[er][gq * UB2 + 2 * eq]) = dbs[gq];
    __syncthreads();
    if (tid < GC) {
        float sum = 0.0f;
        for (int r = 0; r < RW; ++r) sum += dgs[r][tid];
        a.bpart[((size_t)rt * 2 + l) * 4 * H + (tid >> 4) * H + u0 + (tid & 15)] = sum;
    }
}

// sum over row tiles (in order) of the [2][4H][H + D] weight-gradient partials,
// written straight into the two parameters' layouts: dW_hh [2][4H][H] and
// dW_ih [2][4H][D]
__global__ void rows_wsum_kernel(const float *__restrict__ part, int nt, int G, int H, int D,
                                 float *__restrict__ dw_hh, float *__restrict__ dw_ih) {
    const int64_t per = (int64_t)2 * G * (H + D);
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= per) return;
    float s = part[i];
    for (int k = 1; k < nt; ++k) s += part[(int64_t)k * per + i];
    const int64_t row = i / (H + D);
    const int c = (int)(i - row * (H + D));
    if (c < H) dw_hh[row * H + c] = s;
    else dw_ih[row * D + (c - H)] = s;
}

// the bias gradient (sum over row tiles, in order) into both bias parameters
__global__ void rows_bsum_kernel(const float *__restrict__ part, int nt, int64_t per, float *__restrict__ db_ih,
                                 float *__restrict__ db_hh) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= per) return;
    float s = part[i];
    for (int k = 1; k < nt; ++k) s += part[(int64_t)k * per + i];
    db_ih[i] = s;
    db_hh[i] = s;
}

int rows_supported(int D, int H) { return D == 80 && H == 256; }

// which layout a direction runs: the 16-unit blocks (v2) whenever their grid
// is at most one block per CU (measured 6.8 vs 9.4 us per forward step at 256
// rows); at two per CU the two blocks of a CU run their steps in phase (their
// matrix work shares the SIMDs, an offset start decays to alignment within ~8
// steps), so the forward keeps the 32-unit blocks there (9.4 vs 9.9 us) and the
// backward the 16-unit ones (14.8 vs 15.4 us).  VOXNAV_ROWS_V1=1 / _V2=1 force
// one layout (A/B and tests; read per call).
bool rows_v2(int NT, bool fwd) {
    const char *e1 = getenv("VOXNAV_ROWS_V1");
    if (e1 && e1[0] == '1') return false;
    const char *e2 = getenv("VOXNAV_ROWS_V2");
    if (e2 && e2[0] == '1') return true;
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return false;
    return 2 * NUB2 * NT <= ncu || !fwd;
}

// the 16-unit kernels raise the issue priority on the hand-off path (wait,
// rows, products, cell, publish) and drop it for the off-path weight
// gradients / x part: at two blocks per CU the publishing block goes first
// (backward 15.1 -> 14.2 us per step at 512 rows).  VOXNAV_ROWS_PRIO=0: off.
int rows_prio() {
    const char *e = getenv("VOXNAV_ROWS_PRIO");
    return (e && e[0] == '0') ? 0 : 1;
}

uint32_t *g_rows_diag = nullptr;   // vn_lstm_rows_set_diag (diagnostics)

int rows_grid_ok(int B, int NT, bool v2, int *grid) {
    *grid = 2 * (v2 ? NUB2 : NUB) * NT;
    if (B < 1 || NT < 1 || B > NT * RW) return 0;
    int dev = 0, ncu = 0, per_fwd = 0, per_bwd = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    if (v2) {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_fwd, lstm_rows_fwd2_kernel<80, 256>, 256, 0) != hipSuccess)
            return 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_bwd, lstm_rows_bwd2_kernel<80, 256>, 256, 0) != hipSuccess)
            return 0;
    } else {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_fwd, lstm_rows_fwd_kernel<80, 256>, 256, 0) != hipSuccess)
            return 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_bwd, lstm_rows_bwd_kernel<80, 256>, 256, 0) != hipSuccess)
            return 0;
    }
    const int cap = ncu * (per_fwd < per_bwd ? per_fwd : per_bwd);
    return *grid <= cap;
}

}  // namespace

extern "C" {

int vn_lstm_rows_supported(int32_t D, int32_t H, int32_t B) {
    if (!rows_supported(D, H)) return 0;
    int grid = 0;
    const int NT = (B + RW - 1) / RW;
    return rows_grid_ok(B, NT, rows_v2(NT, true), &grid) && rows_grid_ok(B, NT, rows_v2(NT, false), &grid);
}

// diagnostics: the forward (two-per-CU layout) records each block's HW_ID /
// XCC_ID in diag[2 b], diag[2 b + 1] and the 100-MHz clock at 7 points of
// its step t in diag[2 grid + (b L + t) 8 + k]; NULL turns it off.  Not in voxnav.h.
int vn_lstm_rows_set_diag(void *diag) {
    g_rows_diag = (uint32_t *)diag;
    return VN_OK;
}

int vn_lstm_rows_part_floats(int32_t B, int64_t *floats) {
    if (!floats || B < 1) return fail(VN_ERR_INVALID, "bad argument");
    const int NT = (B + RW - 1) / RW;
    // the two partial-dh slots, the per-row-tile [dW_hh | dW_ih] and db partials
    *floats = (int64_t)2 * 2 * NT * NUB2 * RW * 256 + (int64_t)NT * 2 * 1024 * (256 + 80) + (int64_t)NT * 2 * 1024;
    return VN_OK;
}

int vn_lstm_rows_fwd(const float *x, int32_t D, const float *w_ih, const float *w_hh, const float *bias,
                     const float *h_store, const float *c_store, int64_t n_env, const int32_t *env,
                     const uint8_t *start, const float *keep, float *hout, float *hprev, float *cprev, float *cnew,
                     float *act, uint32_t *cnt, int32_t *err, int32_t L, int32_t B, int32_t H, void *stream) {
    if (!x || !w_ih || !w_hh || !bias || !h_store || !c_store || !env || !start || !keep || !hout || !hprev ||
        !cprev || !cnew || !act || !cnt || !err)
        return fail(VN_ERR_INVALID, "NULL argument");
    if (!rows_supported(D, H)) return fail(VN_ERR_INVALID, "row-layout LSTM: D 80 and H 256 only (got %d, %d)", D, H);
    if (L < 1) return fail(VN_ERR_INVALID, "L < 1");
    const int NT = (B + RW - 1) / RW;
    const bool v2 = rows_v2(NT, true);
    int grid = 0;
    if (!rows_grid_ok(B, NT, v2, &grid))
        return fail(VN_ERR_INVALID, "row-layout LSTM: %d blocks are not co-resident (B = %d)", grid, B);
    if ((size_t)2 * L * B * H * 4 >= (1ull << 31)) return fail(VN_ERR_INVALID, "row-layout LSTM: hout over 2 GB");
    const hipStream_t st = (hipStream_t)stream;
    VN_HIP(hipMemsetAsync(cnt, 0, (size_t)2 * NT * CSTRIDE * sizeof(uint32_t), st));
    RowsFwd a{x, w_ih, w_hh, bias, h_store, c_store, env, start, keep, hout, hprev, cprev, cnew, act, cnt, err,
              n_env, L, B, NT, rows_prio(), g_rows_diag};
    if (v2) hipLaunchKernelGGL((lstm_rows_fwd2_kernel<80, 256>), dim3((unsigned)grid), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((lstm_rows_fwd_kernel<80, 256>), dim3((unsigned)grid), dim3(256), 0, st, a);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

int vn_lstm_rows_bwd(const float *dh_out, const float *w_hh, const float *act, const float *cprev, const float *cnew,
                     const float *hprev, const float *x, const uint8_t *start, float *dG, float *dw_hh,
                     float *dw_ih, float *db_ih, float *db_hh, float *part, uint32_t *cnt, int32_t *err, int32_t L,
                     int32_t B, int32_t H, void *stream) {
    if (!dh_out || !w_hh || !act || !cprev || !cnew || !hprev || !x || !start || !dw_hh || !dw_ih || !db_ih ||
        !db_hh || !part || !cnt || !err)
        return fail(VN_ERR_INVALID, "NULL argument");
    if (!rows_supported(80, H)) return fail(VN_ERR_INVALID, "row-layout LSTM: H 256 only (got %d)", H);
    if (L < 1) return fail(VN_ERR_INVALID, "L < 1");
    const int NT = (B + RW - 1) / RW;
    const bool v2 = rows_v2(NT, false);
    int grid = 0;
    if (!rows_grid_ok(B, NT, v2, &grid))
        return fail(VN_ERR_INVALID, "row-layout LSTM: %d blocks are not co-resident (B = %d)", grid, B);
    const hipStream_t st = (hipStream_t)stream;
    constexpr int D = 80;
    const size_t slot_f = (size_t)2 * NT * (v2 ? NUB2 : NUB) * RW * H;
    float *wpart = part + 2 * slot_f;
    float *bpart = wpart + (size_t)NT * 2 * 4 * H * (H + D);
    VN_HIP(hipMemsetAsync(cnt, 0, (size_t)2 * NT * CSTRIDE * sizeof(uint32_t), st));
    RowsBwd a{dh_out, w_hh, act, cprev, cnew, hprev, x, start, dG, part, wpart, bpart, cnt, err, L, B, NT, rows_prio()};
    if (v2) hipLaunchKernelGGL((lstm_rows_bwd2_kernel<80, 256>), dim3((unsigned)grid), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((lstm_rows_bwd_kernel<80, 256>), dim3((unsigned)grid), dim3(256), 0, st, a);
    const int64_t pw = (int64_t)2 * 4 * H * (H + D), pb = (int64_t)2 * 4 * H;
    hipLaunchKernelGGL(rows_wsum_kernel, dim3((unsigned)((pw + 255) / 256)), dim3(256), 0, st, wpart, NT, 4 * H, H, D,
                       dw_hh, dw_ih);
    hipLaunchKernelGGL(rows_bsum_kernel, dim3((unsigned)((pb + 255) / 256)), dim3(256), 0, st, bpart, NT, pb, db_ih,
                       db_hh);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

}  // extern "C"
