// voxnav_policy_f32.hip -- the reference-dtype (f32) policy step of the
// rollout collector on the f32 matrix cores.
//
// sb3_contrib's MlpLstmPolicy (train/Grid_Train.py:68-80, :199-205; SURVEY.md
// Appendix D.4) runs per step, per agent, in f32:
//   actor / critic LSTM(80 -> 256):  gates = x W_ih^T + b_ih + h W_hh^T + b_hh
//                                    c' = f c + i g,  h' = o tanh(c')
//   pi / vf MLP 256 -> 256 -> 256 -> 128, Tanh after every layer
// (then the action / value heads, vn_policy_head).  gfx950 has no xf32: the
// f32 matrix instruction v_mfma_f32_32x32x2_f32 runs at the f32 vector rate
// (64 FLOP/clk/SIMD, 157 TF/s) and computes exact f32 FMA chains, so the
// policy math is bound by that rate (2.03 MFLOP per agent-step).  Two kernels:
//
//   lstm_fused_f32_kernel  [x | h] @ [W_ih | W_hh]^T for both LSTMs with the
//                          cell update as the epilogue: the 4H gate
//                          pre-activations (2 x 1 GB per step at 65,536
//                          agents through library GEMMs) never reach memory;
//                          the episode-start mask is applied on read (h rows
//                          and c of agents starting an episode are zero)
//   linear_f32_kernel      y = tanh(x W^T + b) for one MLP layer of both
//                          branches (pi, vf) in one launch, the bias and
//                          Tanh in the epilogue (no standalone tanh pass)
//
// Both stream K through LDS in chunks of 16 (double-buffered, the next
// chunk's global loads in flight during this chunk's MFMAs, one barrier per
// chunk).  A-operand chunks are stored k-major ([k][row]) and B chunks
// ([k][col]) so that every MFMA operand is one conflict-free ds_read_b32:
// for v_mfma_f32_32x32x2_f32, lane l supplies A[row l%32][k l/32] and
// B[k l/32][col l%32], and receives D[8(v/4) + 4(l/32) + v%4][l%32] in
// accumulator register v.  Weights are pre-packed on the host into the LDS
// chunk layout (contiguous 16-row slabs), so a B chunk is a straight copy.

#include <hip/hip_runtime.h>

#include <cstdint>

#include "vn_common.h"

using vn_detail::fail;

namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16_t;

#ifndef VN_PF_FAST
#define VN_PF_FAST 1   // gate / Tanh nonlinearities on the hardware exp and rcp (|err| <= ~4e-7)
#endif
#ifndef VN_PF_DIAG
#define VN_PF_DIAG 0   // timing diagnostics (results invalid): 1 no K loop, 2 no nonlinearities
#endif
#if VN_PF_FAST
__device__ __forceinline__ float sigm_f32(float x) { return __frcp_rn(1.0f + __expf(-x)); }
__device__ __forceinline__ float tanh_f32(float x) { return 1.0f - 2.0f * __frcp_rn(1.0f + __expf(2.0f * x)); }
#else
__device__ __forceinline__ float sigm_f32(float x) { return 1.0f / (1.0f + expf(-x)); }
__device__ __forceinline__ float tanh_f32(float x) { return tanhf(x); }
#endif
#if VN_PF_DIAG == 2
#define PF_SIGM(v) (v)
#define PF_TANH(v) (v)
#else
#define PF_SIGM(v) sigm_f32(v)
#define PF_TANH(v) tanh_f32(v)
#endif

constexpr int PF_KC = 16;          // K per LDS chunk (8 MFMA k-steps)
constexpr int PF_AP = 128 + 4;     // A chunk pitch in floats (128 rows + pad)

__device__ __forceinline__ f32x16_t zero16() {
    f32x16_t z;
#pragma unroll
    for (int r = 0; r < 16; ++r) z[r] = 0.0f;
    return z;
}

// ---------------------------------------------------------------------------
// LSTM step.  Block: 256 threads (4 waves), 128 agents x 64 units x 4 gates;
// wave w owns rows 64*(w&1) .. +63 (two 32-row MFMA tiles) and units
// 32*(w>>1) .. +31, one accumulator per (row tile, gate): the four gates of a
// (row, unit) sit in the same lane and register, so the cell update needs no
// exchange.  8 accumulators = 128 registers: 2 waves per SIMD, 2 blocks per CU.
//   x      f32 [N][obs_dim]
//   hin    f32 [n_lstm][N][H] (unmasked with MASK: rows with start != 0 are
//          read as zero)
//   wp     f32 [n_lstm][H/64][Kp][4][64]: wp[b][ub][k][g][uu] =
//          [W_ih | 0 | W_hh][g*H + 64 ub + uu][k], W_ih in k < obs_dim,
//          W_hh in [kx, kx + H), kx = obs_dim rounded up to 16, Kp = kx + H
//   bias   f32 [n_lstm][4H] = b_ih + b_hh
//   c_in   f32 [n_lstm][N][H] (may equal c_out); c_out, h_out f32 [n_lstm][N][H]
// ---------------------------------------------------------------------------
constexpr int LS_ROWS = 128, LS_UNITS = 64, LS_COLS = 4 * LS_UNITS;
constexpr int LS_RT = LS_ROWS / 64;             // 32-row MFMA tiles per wave = A float4 staged per thread
constexpr int LS_AP = LS_ROWS + 4;              // A chunk pitch

// A work item: one (row tile, LSTM, 64-unit block).  Items are dealt to the
// persistent blocks with stride gridDim.x (a multiple of 8), so a block's
// items stay on its XCD; when the tile count allows, the items of one round on
// one XCD are all the unit blocks of a few row tiles (their x / h rows are
// fetched into that XCD's L2 once).
struct LsItem {
    int n_base, b, u_base;
    const float *wblk, *hb;
};

__device__ __forceinline__ LsItem ls_decode(int id, int ntiles, int ncombo, int ublocks, int N, int H, int Kp,
                                            const float *wp, const float *hin) {
    int tile, combo;
    if ((ntiles & 7) == 0) {
        const int xcd = id & 7, local = id >> 3;
        tile = xcd + 8 * (local / ncombo);
        combo = local - (local / ncombo) * ncombo;
    } else {
        tile = id / ncombo;
        combo = id - tile * ncombo;
    }
    LsItem d;
    d.b = combo / ublocks;
    const int ub = combo - d.b * ublocks;
    d.n_base = tile * LS_ROWS;
    d.u_base = ub * LS_UNITS;
    d.wblk = wp + ((size_t)d.b * ublocks + ub) * (size_t)Kp * LS_COLS;
    d.hb = hin + (size_t)d.b * N * H;
    return d;
}

// Persistent: gridDim.x blocks (the co-resident count, 2 per CU) walk the
// items.  The chunk stream runs on across items: the last chunk of an item
// stages the next item's first chunk, and the epilogue's state stores drain
// behind the next item's MFMAs.
template <bool VEC_X, bool MASK>
__global__ __launch_bounds__(256, 2) void lstm_fused_f32_kernel(const float *__restrict__ x, int obs_dim, int kx,
                                                                const float *__restrict__ hin,
                                                                const float *__restrict__ wp, int Kp,
                                                                const float *__restrict__ bias, const float *c_in,
                                                                const float *__restrict__ start, float *c_out,
                                                                float *h_out, int N, int H, int ncombo, int n_items) {
    __shared__ float As[2][PF_KC][LS_AP];
    __shared__ __attribute__((aligned(16))) float Bs[2][PF_KC][LS_COLS];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int ublocks = H / LS_UNITS;
    const int ntiles = (N + LS_ROWS - 1) / LS_ROWS;
    const int nchunks = Kp / PF_KC;
    const int kq = (tid & 3) * 4;
    const int wr = (wv & 1) * (LS_ROWS / 2), wu = (wv >> 1) * 32;
    const int col = lane & 31, kh = lane >> 5;

    int item = (int)blockIdx.x;
    if (item >= n_items) return;
    LsItem cur = ls_decode(item, ntiles, ncombo, ublocks, N, H, Kp, wp, hin);

    // staging rows of the item being staged: thread covers (row q>>2, k 4(q&3)
    // .. +3) for q = tid, tid + 256
    int arow0, arow1;
    bool az0 = false, az1 = false;
#define LS_ROWS_FOR(d)                                                                                       \
    {                                                                                                        \
        arow0 = min((d).n_base + (tid >> 2), N - 1);                                                         \
        arow1 = min((d).n_base + ((tid + 256) >> 2), N - 1);                                                 \
        if (MASK) {                                                                                          \
            az0 = start[arow0] != 0.0f;                                                                      \
            az1 = start[arow1] != 0.0f;                                                                      \
        }                                                                                                    \
    }
    // staging registers, named (an indexed array lives in scratch); the loads
    // are unconditional from a selected address and the zeroing happens when
    // the registers are written to LDS, so nothing waits between issuing the
    // next chunk's loads and this chunk's MFMAs
    float4 ra0, ra1, rb0, rb1, rb2, rb3;
#define LS_A_LOAD(dst, arow, hb_)                                                                            \
    {                                                                                                        \
        if (VEC_X) {                                                                                         \
            const float *p_ = isx_ ? x + (size_t)(arow) * obs_dim + min(k_, obs_dim - 4)                     \
                                   : (hb_) + (size_t)(arow) * H + (k_ - kx);                                 \
            dst = *reinterpret_cast<const float4 *>(p_);                                                     \
        } else {                                                                                             \
            const float *p_ = isx_ ? x + (size_t)(arow) * obs_dim : (hb_) + (size_t)(arow) * H - kx;         \
            const int lim_ = isx_ ? obs_dim - 1 : 0x7fffffff;                                                \
            dst.x = p_[min(k_ + 0, lim_)];                                                                   \
            dst.y = p_[min(k_ + 1, lim_)];                                                                   \
            dst.z = p_[min(k_ + 2, lim_)];                                                                   \
            dst.w = p_[min(k_ + 3, lim_)];                                                                   \
        }                                                                                                    \
    }
    // chunk ch of the item d into the staging registers
#define LS_LOAD(d, ch)                                                                                       \
    {                                                                                                        \
        const int k_ = (ch) * PF_KC + kq;                                                                    \
        const bool isx_ = (ch) * PF_KC < kx; /* block-uniform: a chunk is all x or all h (kx % 16 == 0) */   \
        LS_A_LOAD(ra0, arow0, (d).hb) LS_A_LOAD(ra1, arow1, (d).hb)                                          \
        const float4 *pb_ = reinterpret_cast<const float4 *>((d).wblk + (size_t)(ch) * PF_KC * LS_COLS) + tid; \
        rb0 = pb_[0];                                                                                        \
        rb1 = pb_[256];                                                                                      \
        rb2 = pb_[512];                                                                                      \
        rb3 = pb_[768];                                                                                      \
    }
#define LS_A_PUT(v, i, az)                                                                                   \
    {                                                                                                        \
        const int r_ = (tid + 256 * (i)) >> 2;                                                               \
        float4 v_ = v;                                                                                       \
        if (isx_) {                                                                                          \
            if (k_ + 0 >= obs_dim) v_.x = 0.0f;                                                              \
            if (k_ + 1 >= obs_dim) v_.y = 0.0f;                                                              \
            if (k_ + 2 >= obs_dim) v_.z = 0.0f;                                                              \
            if (k_ + 3 >= obs_dim) v_.w = 0.0f;                                                              \
        } else if (MASK && (az)) {                                                                           \
            v_ = make_float4(0.f, 0.f, 0.f, 0.f);                                                            \
        }                                                                                                    \
        As[buf_][kq + 0][r_] = v_.x;                                                                         \
        As[buf_][kq + 1][r_] = v_.y;                                                                         \
        As[buf_][kq + 2][r_] = v_.z;                                                                         \
        As[buf_][kq + 3][r_] = v_.w;                                                                         \
    }
    // the staging registers (chunk ch) into LDS buffer bf
#define LS_STORE(bf, ch)                                                                                     \
    {                                                                                                        \
        const int buf_ = (bf);                                                                               \
        const int k_ = (ch) * PF_KC + kq;                                                                    \
        const bool isx_ = (ch) * PF_KC < kx;                                                                 \
        LS_A_PUT(ra0, 0, az0) LS_A_PUT(ra1, 1, az1)                                                          \
        float4 *pl_ = reinterpret_cast<float4 *>(&Bs[buf_][0][0]) + tid;                                     \
        pl_[0] = rb0;                                                                                        \
        pl_[256] = rb1;                                                                                      \
        pl_[512] = rb2;                                                                                      \
        pl_[768] = rb3;                                                                                      \
    }

    f32x16_t acc[LS_RT][4];
#define LS_RD(bf, s_, A0, A1, B0, B1, B2, B3)                                                                \
    {                                                                                                        \
        const int kk_ = 2 * (s_) + kh;                                                                       \
        A0 = As[bf][kk_][wr + col];                                                                          \
        A1 = As[bf][kk_][wr + 32 + col];                                                                     \
        B0 = Bs[bf][kk_][wu + col];                                                                          \
        B1 = Bs[bf][kk_][LS_UNITS + wu + col];                                                               \
        B2 = Bs[bf][kk_][2 * LS_UNITS + wu + col];                                                           \
        B3 = Bs[bf][kk_][3 * LS_UNITS + wu + col];                                                           \
    }
#define LS_MM(A0, A1, B0, B1, B2, B3)                                                                        \
    {                                                                                                        \
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(A0, B0, acc[0][0], 0, 0, 0);                        \
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(A0, B1, acc[0][1], 0, 0, 0);                        \
        acc[0][2] = __builtin_amdgcn_mfma_f32_32x32x2f32(A0, B2, acc[0][2], 0, 0, 0);                        \
        acc[0][3] = __builtin_amdgcn_mfma_f32_32x32x2f32(A0, B3, acc[0][3], 0, 0, 0);                        \
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(A1, B0, acc[1][0], 0, 0, 0);                        \
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(A1, B1, acc[1][1], 0, 0, 0);                        \
        acc[1][2] = __builtin_amdgcn_mfma_f32_32x32x2f32(A1, B2, acc[1][2], 0, 0, 0);                        \
        acc[1][3] = __builtin_amdgcn_mfma_f32_32x32x2f32(A1, B3, acc[1][3], 0, 0, 0);                        \
    }
    // the MFMAs of one chunk in LDS buffer bf: two operand sets, k-step s+1's
    // reads issued before k-step s's MFMAs (3 LDS reads -- one ds_read2 of A,
    // two of B -- per k-step, enforced on the scheduler)
#define LS_COMPUTE(bf)                                                                                       \
    {                                                                                                        \
        float pa0, pa1, pb0, pb1, pb2, pb3, qa0, qa1, qb0, qb1, qb2, qb3;                                    \
        LS_RD(bf, 0, pa0, pa1, pb0, pb1, pb2, pb3)                                                           \
        _Pragma("unroll") for (int s = 0; s < PF_KC / 2; s += 2) {                                           \
            LS_RD(bf, s + 1, qa0, qa1, qb0, qb1, qb2, qb3)                                                   \
            LS_MM(pa0, pa1, pb0, pb1, pb2, pb3)                                                              \
            if (s + 2 < PF_KC / 2) LS_RD(bf, s + 2, pa0, pa1, pb0, pb1, pb2, pb3)                            \
            LS_MM(qa0, qa1, qb0, qb1, qb2, qb3)                                                              \
        }                                                                                                    \
        __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);                                                   \
        _Pragma("unroll") for (int s = 0; s < PF_KC / 2; ++s) {                                              \
            if (s + 1 < PF_KC / 2) __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);                        \
            __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);                                               \
        }                                                                                                    \
    }

    LS_ROWS_FOR(cur)
    LS_LOAD(cur, 0)
    LS_STORE(0, 0)
    __syncthreads();
    int g = 0;        // chunks computed so far: chunk g sits in LDS buffer g & 1
    for (;;) {
#pragma unroll
        for (int t = 0; t < LS_RT; ++t)
#pragma unroll
            for (int gg = 0; gg < 4; ++gg) acc[t][gg] = zero16();
        const int nitem = item + (int)gridDim.x;
        const bool more = nitem < n_items;
        const LsItem nxt = more ? ls_decode(nitem, ntiles, ncombo, ublocks, N, H, Kp, wp, hin) : cur;
        for (int ch = 0; ch < (VN_PF_DIAG == 1 ? 0 : nchunks - 1); ++ch) {
            LS_LOAD(cur, ch + 1)
            __builtin_amdgcn_sched_barrier(0);
            LS_COMPUTE(g & 1)
            LS_STORE((g + 1) & 1, ch + 1)
            __syncthreads();
            ++g;
        }
        // the item's last chunk: stage the next item's first chunk (this
        // item's own first chunk again when there is none: into the idle
        // buffer, unconditional) and load this item's cell states
        LS_ROWS_FOR(nxt)
        LS_LOAD(nxt, 0)
        __builtin_amdgcn_sched_barrier(0);
        if (VN_PF_DIAG != 1) LS_COMPUTE(g & 1)
        LS_STORE((g + 1) & 1, 0)
        __syncthreads();
        ++g;

        // epilogue: lane holds unit u; gate gg of (row, u) in acc[t][gg][reg].
        // A row tile's 16 states are loaded together before any store (vmcnt
        // retires in order: a load issued after a store waits for it); the
        // stores drain behind the next item's MFMAs
        const int u = cur.u_base + wu + col;
        const float *bb = bias + (size_t)cur.b * 4 * H;
        const float bi = bb[u], bf = bb[H + u], bg = bb[2 * H + u], bo = bb[3 * H + u];
#pragma unroll
        for (int t = 0; t < LS_RT; ++t) {
            float cin[16];
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int n = min(cur.n_base + wr + 32 * t + (reg & 3) + 8 * (reg >> 2) + 4 * kh, N - 1);
                const float v = c_in[((size_t)cur.b * N + n) * H + u];
                cin[reg] = (MASK && start[n] != 0.0f) ? 0.0f : v;      // the episode-start mask, on read
            }
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int n = cur.n_base + wr + 32 * t + (reg & 3) + 8 * (reg >> 2) + 4 * kh;
                if (n < N) {
                    const size_t so = ((size_t)cur.b * N + n) * H + u;
                    const float cv = cin[reg];
                    const float ig = PF_SIGM(acc[t][0][reg] + bi), fg = PF_SIGM(acc[t][1][reg] + bf);
                    const float gg = PF_TANH(acc[t][2][reg] + bg), og = PF_SIGM(acc[t][3][reg] + bo);
                    const float fc = fg * cv, ig2 = ig * gg;
                    const float cn = fc + ig2;
                    c_out[so] = cn;
                    h_out[so] = og * PF_TANH(cn);
                }
            }
        }
        if (!more) break;
        item = nitem;
        cur = nxt;
    }
#undef LS_ROWS_FOR
#undef LS_A_LOAD
#undef LS_A_PUT
#undef LS_LOAD
#undef LS_STORE
#undef LS_RD
#undef LS_MM
#undef LS_COMPUTE
}

// ---------------------------------------------------------------------------
// One Linear (+ Tanh) layer for up to two branches: y[br] = act(x[br] W[br]^T
// + b[br]).  Block: 256 threads, 128 rows x 128 output columns; wave w owns
// rows 64*(w&1) and columns 64*(w>>1) as 2 x 2 accumulators (64 registers):
// 4 waves per SIMD.
//   x   f32 [M][K] rows (row stride ldx), K a multiple of 16
//   wp  f32 [Nout/128][K][128]: wp[cb][k][j] = W[128 cb + j][k]
//   y   f32 [M][Nout]
// ---------------------------------------------------------------------------
constexpr int LN_ROWS = 128, LN_COLS = 128;

struct LinearArgs {
    const float *x[2];
    const float *wp[2];
    const float *bias[2];
    float *y[2];
};

template <bool TANH>
__global__ __launch_bounds__(256, 4) void linear_f32_kernel(LinearArgs a, int64_t ldx, int M, int K, int Nout,
                                                            int ncb) {
    __shared__ float As[2][PF_KC][PF_AP];
    __shared__ __attribute__((aligned(16))) float Bs[2][PF_KC][LN_COLS];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int br = (int)blockIdx.y;
    const float *__restrict__ x = a.x[br];
    const float *__restrict__ wp = a.wp[br];
    const int ntiles = (M + LN_ROWS - 1) / LN_ROWS;
    const int id = (int)blockIdx.x;
    int tile, cb;
    if ((ntiles & 7) == 0) {   // column blocks of one row tile on one XCD (see the LSTM kernel)
        const int xcd = id & 7, local = id >> 3;
        tile = xcd + 8 * (local / ncb);
        cb = local - (local / ncb) * ncb;
    } else {
        tile = id / ncb;
        cb = id - tile * ncb;
    }
    const int n_base = tile * LN_ROWS;
    const float *wblk = wp + (size_t)cb * K * LN_COLS;
    const int nchunks = K / PF_KC;
    int arow[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) arow[i] = min(n_base + ((tid + 256 * i) >> 2), M - 1);
    const int kq = (tid & 3) * 4;
    float4 ra0, ra1, rb0, rb1;   // named staging registers (see the LSTM kernel)
#define LN_LOAD(ch)                                                                                          \
    {                                                                                                        \
        const int k_ = (ch) * PF_KC + kq;                                                                    \
        ra0 = *reinterpret_cast<const float4 *>(x + (size_t)arow[0] * ldx + k_);                             \
        ra1 = *reinterpret_cast<const float4 *>(x + (size_t)arow[1] * ldx + k_);                             \
        const float4 *pb_ = reinterpret_cast<const float4 *>(wblk + (size_t)(ch) * PF_KC * LN_COLS) + tid;   \
        rb0 = pb_[0];                                                                                        \
        rb1 = pb_[256];                                                                                      \
    }
#define LN_A_PUT(v, i)                                                                                       \
    {                                                                                                        \
        const int r_ = (tid + 256 * (i)) >> 2;                                                               \
        As[buf_][kq + 0][r_] = v.x;                                                                          \
        As[buf_][kq + 1][r_] = v.y;                                                                          \
        As[buf_][kq + 2][r_] = v.z;                                                                          \
        As[buf_][kq + 3][r_] = v.w;                                                                          \
    }
#define LN_STORE(ch)                                                                                         \
    {                                                                                                        \
        const int buf_ = (ch) & 1;                                                                           \
        LN_A_PUT(ra0, 0) LN_A_PUT(ra1, 1)                                                                    \
        float4 *pl_ = reinterpret_cast<float4 *>(&Bs[buf_][0][0]) + tid;                                     \
        pl_[0] = rb0;                                                                                        \
        pl_[256] = rb1;                                                                                      \
    }
    f32x16_t acc[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int c = 0; c < 2; ++c) acc[t][c] = zero16();
    const int wr = (wv & 1) * 64, wc = (wv >> 1) * 64;
    const int col = lane & 31, kh = lane >> 5;

    LN_LOAD(0)
    LN_STORE(0)
    __syncthreads();
    for (int ch = 0; ch < (VN_PF_DIAG == 1 ? 0 : nchunks); ++ch) {
        const int nx = ch + 1 < nchunks ? ch + 1 : ch;
        LN_LOAD(nx)
        __builtin_amdgcn_sched_barrier(0);
        const int buf = ch & 1;
#define LN_RD(s_, A0, A1, B0, B1)                                                                            \
    {                                                                                                        \
        const int kk_ = 2 * (s_) + kh;                                                                       \
        A0 = As[buf][kk_][wr + col];                                                                         \
        A1 = As[buf][kk_][wr + 32 + col];                                                                    \
        B0 = Bs[buf][kk_][wc + col];                                                                         \
        B1 = Bs[buf][kk_][wc + 32 + col];                                                                    \
    }
#define LN_MM(A0, A1, B0, B1)                                                                                \
    {                                                                                                        \
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(A0, B0, acc[0][0], 0, 0, 0);                        \
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(A0, B1, acc[0][1], 0, 0, 0);                        \
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(A1, B0, acc[1][0], 0, 0, 0);                        \
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(A1, B1, acc[1][1], 0, 0, 0);                        \
    }
        float pa0, pa1, pb0, pb1;
#if VN_PF_PREF
        float qa0, qa1, qb0, qb1;
        LN_RD(0, pa0, pa1, pb0, pb1)
#pragma unroll
        for (int s = 0; s < PF_KC / 2; s += 2) {
            LN_RD(s + 1, qa0, qa1, qb0, qb1)
            LN_MM(pa0, pa1, pb0, pb1)
            if (s + 2 < PF_KC / 2) LN_RD(s + 2, pa0, pa1, pb0, pb1)
            LN_MM(qa0, qa1, qb0, qb1)
        }
        // 2 LDS reads (ds_read2 of A, of B) per k-step, one k-step ahead of its 4 MFMAs
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
#pragma unroll
        for (int s = 0; s < PF_KC / 2; ++s) {
            if (s + 1 < PF_KC / 2) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        }
#else
#pragma unroll
        for (int s = 0; s < PF_KC / 2; ++s) {
            LN_RD(s, pa0, pa1, pb0, pb1)
            LN_MM(pa0, pa1, pb0, pb1)
        }
#endif
#undef LN_RD
#undef LN_MM
        LN_STORE(nx)
        __syncthreads();
    }
#undef LN_A_PUT
#undef LN_LOAD
#undef LN_STORE

    float *__restrict__ y = a.y[br];
    const float *__restrict__ bias = a.bias[br];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const int j = cb * LN_COLS + wc + 32 * c + col;
        const float bj = bias[j];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int n = n_base + wr + 32 * t + (reg & 3) + 8 * (reg >> 2) + 4 * kh;
                if (n < M) {
                    const float v = acc[t][c][reg] + bj;
                    y[(size_t)n * Nout + j] = TANH ? PF_TANH(v) : v;
                }
            }
    }
}


// ---------------------------------------------------------------------------
// The policy MLP of both branches and the heads in one launch: per step of
// the collector, after the LSTM (ActorCriticPolicy.forward: mlp_extractor ->
// action_net / value_net -> distribution.get_actions / log_prob; net_arch
// pi/vf [256, 256, 128] with Tanh, train/Grid_Train.py:68-80).  Block: 256
// threads, 32 rows of one branch (blockIdx.y: pi, vf).  The rows'
// activations stay in LDS from the input through every Linear + Tanh layer to
// the head, so no latent reaches memory (vn_linear_f32 x 3 + vn_policy_head
// wrote and re-read [M][256] f32 per layer and branch).
//   A operand: act [32][260] in LDS; within a group of 8 k the two lane halves
//     take k 0..3 and 4..7 over the 4 k-steps (a reordering of the dot
//     product's terms, the same for both operands), so one ds_read_b128 of a
//     lane's row carries its 4 k-steps (pitch 260: rows 0..15 of a 16-lane
//     group land on 16 distinct 16-B bank slots).
//   B operand: the weights packed per lane on the host (vn_mlp_head_f32
//     layout: [N/32][K/8][64 lanes][4]): each wave streams its own columns
//     through its own LDS ring (global_load_lds, MH_D k-groups ahead, one
//     ds_read_b128 per lane per 4 k-steps and 32-column tile) -- no register
//     staging and no barrier inside a layer.
//   wave w owns columns 64w .. 64w + 63 (N = 256: two 32x32 tiles) or 32w ..
//   32w + 31 (N = 128: one tile, even / odd k-groups in two accumulators,
//   summed in the epilogue); the epilogue writes tanh(acc + b) over act.
//   head: 8 lanes per row (features j = p, p + 8, ...) with the head weights
//     in LDS, xor-reduced over the 8; pi rows: logits, log-sum-exp, the Philox
//     inverse-CDF draw (argmax when deterministic) and its log-prob, as
//     vn_policy_head; vf rows: the value.
// LDS 49 KB: three blocks per CU.
// ---------------------------------------------------------------------------
constexpr int MH_R = 32, MH_P = 260, MH_MAXL = 4, MH_MAXA = 8, MH_MAXP = 256, MH_D = 2;

struct MlpHeadArgs {
    const float *x[2];                 // branch inputs [M][ldx] (pi, vf)
    const float *wp[2][MH_MAXL];       // packed weights per branch and layer
    const float *bias[2][MH_MAXL];     // b_l [N_l]
    int width[MH_MAXL];                // N_l: 128 or 256
    const float *wa, *ba, *wv, *bv;    // action_net [A][P], [A]; value_net [P], [1]
    int32_t *actions;
    float *log_probs, *values;
    uint64_t seed, t;
    int64_t gid_base, ldx;
    int K0, n_layers, A, M, br0, deterministic;
};

// One layer's K loop of a wave: A from the act rows (one ds_read_b128 per
// k-group of 8), B from the per-lane packed weights through a ring of MH_D
// k-groups in registers (refilled MH_D ahead; past the end the slot reloads a
// k-group already read, so the loop has no branch and the waits are counted).
// WIDE: two column tiles; else one tile, even / odd k-groups into acc0 / acc1.
typedef float mh_f4 __attribute__((ext_vector_type(4)));

// the MLP layers' Tanh on the hardware exp and reciprocal (v_rcp_f32, 1 ulp;
// |err| <= ~3e-7 absolute) -- the correctly rounded __frcp_rn costs a
// division sequence per element in the epilogues
__device__ __forceinline__ float mh_tanh(float x) { return 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + __expf(2.0f * x)); }

// One layer's K loop of a wave: A from the act rows (one ds_read_b128 per
// k-group of 8), B from the per-lane packed weights through the wave's own
// LDS ring of MH_D k-groups (global_load_lds, 16 B per lane; each wave reads
// only what it loaded, so no barrier -- its own vmcnt says the group landed).
// Past the end a slot reloads a k-group already read (no branch; drained at
// the end).  WIDE: two column tiles; else one tile, even / odd k-groups into
// acc0 / acc1.
template <bool WIDE>
__device__ __forceinline__ void mh_layer(const float *Ar, const float4 *B0, const float4 *B1, int KG, float *ring0,
                                         float *ring1, int lane, f32x16_t &acc0, f32x16_t &acc1) {
    static_assert(MH_D == 2, "two ring slots, each its own LDS object (the waits then see they do not alias)");
    constexpr int PER = WIDE ? 2 : 1;                      // 1-KB loads per k-group
    auto issue = [&](int kg, int slot) {
        float *ring = slot == 0 ? ring0 : ring1;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(B0 + kg * 64 + lane),
                                         (__attribute__((address_space(3))) void *)ring, 16, 0, 0);
        if (WIDE)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(B1 + kg * 64 + lane),
                                             (__attribute__((address_space(3))) void *)(ring + 256), 16, 0, 0);
    };
#pragma unroll
    for (int j = 0; j < MH_D; ++j) issue(j, j);
    for (int kg0 = 0; kg0 < KG; kg0 += MH_D) {
        const int nbase = kg0 + MH_D < KG ? kg0 + MH_D : kg0;
#pragma unroll
        for (int j = 0; j < MH_D; ++j) {
            // k-group kg0 + j landed: the later groups' loads may still be in flight
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER * (MH_D - 1)) : "memory");
            const float4 av = *reinterpret_cast<const float4 *>(Ar + 8 * (kg0 + j));
            // the ring reads in asm: the compiler would otherwise wait for every
            // LDS-DMA load in flight (vmcnt(0)) before them
            const float *ring = j == 0 ? ring0 : ring1;
            mh_f4 b0v, b1v;
            asm volatile("ds_read_b128 %0, %1" : "=v"(b0v) : "v"((uint32_t)(uintptr_t)(ring + lane * 4)) : "memory");
            if (WIDE) {
                asm volatile("ds_read_b128 %0, %1 offset:1024" : "=v"(b1v) : "v"((uint32_t)(uintptr_t)(ring + lane * 4))
                             : "memory");
                // the slot's reads are done before the next load overwrites it
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(b0v), "+v"(b1v)::"memory");
            } else {
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(b0v)::"memory");
                b1v = b0v;
            }
            const float4 b0 = make_float4(b0v[0], b0v[1], b0v[2], b0v[3]);
            const float4 b1 = make_float4(b1v[0], b1v[1], b1v[2], b1v[3]);
            issue(nbase + j, j);
            if (WIDE) {
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, b0.x, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, b1.x, acc1, 0, 0, 0);
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, b0.y, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, b1.y, acc1, 0, 0, 0);
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, b0.z, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, b1.z, acc1, 0, 0, 0);
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, b0.w, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, b1.w, acc1, 0, 0, 0);
            } else if ((j & 1) == 0) {
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, b0.x, acc0, 0, 0, 0);
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, b0.y, acc0, 0, 0, 0);
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, b0.z, acc0, 0, 0, 0);
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, b0.w, acc0, 0, 0, 0);
            } else {
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, b0.x, acc1, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, b0.y, acc1, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, b0.z, acc1, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, b0.w, acc1, 0, 0, 0);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the trailing reloads landed: the ring is free
}

__global__ __launch_bounds__(256, 3) void mlp_head_f32_kernel(MlpHeadArgs a) {
    __shared__ __attribute__((aligned(16))) float act[MH_R * MH_P];
    // per wave the B ring (2 slots, each k-group x 2 tiles x 1 KB); after the
    // last layer the head's weights (action weights in slot 0, value weights in 1)
    __shared__ __attribute__((aligned(16))) float ring0s[4 * 2 * 256];
    __shared__ __attribute__((aligned(16))) float ring1s[4 * 2 * 256];
    static_assert(4 * 2 * 256 >= MH_MAXA * MH_MAXP && 4 * 2 * 256 >= MH_MAXP, "head weights fit the ring");
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: the ring and weight bases in SGPRs
    const int col = lane & 31, kh = lane >> 5;
    const int br = a.br0 + (int)blockIdx.y;
    const int m0 = (int)blockIdx.x * MH_R;
    const int P = a.width[a.n_layers - 1];
    {   // the input rows (rows past M repeat row M - 1; their outputs are not stored)
        const float *x = a.x[br];
        const int q4 = a.K0 / 4;
        for (int f = tid; f < MH_R * q4; f += 256) {
            const int r = f / q4, k = 4 * (f - r * q4);
            const int m = min(m0 + r, a.M - 1);
            *reinterpret_cast<float4 *>(act + r * MH_P + k) = *reinterpret_cast<const float4 *>(x + (size_t)m * a.ldx + k);
        }
        const int qp = ((a.K0 + 8 * MH_D - 1) / (8 * MH_D) * (8 * MH_D)) / 4;   // zero columns up to the padded K
        for (int f = tid; f < MH_R * (qp - q4); f += 256) {
            const int r = f / (qp - q4), k = 4 * (q4 + f - r * (qp - q4));
            *reinterpret_cast<float4 *>(act + r * MH_P + k) = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
    __syncthreads();
    int K = (a.K0 + 8 * MH_D - 1) / (8 * MH_D) * (8 * MH_D);   // layer 0's K: whole ring rounds (zero rows / weights)
    for (int l = 0; l < a.n_layers; ++l) {
        const int N = a.width[l];
        const bool wide = N == 256;
        const int KG = K / 8;
        const int cb0 = wide ? 2 * wv : wv;                     // this wave's first 32-column block
        const float4 *B0 = reinterpret_cast<const float4 *>(a.wp[br][l]) + (size_t)cb0 * KG * 64;   // uniform
        const float *Ar = act + col * MH_P + 4 * kh;
        f32x16_t acc0 = zero16(), acc1 = zero16();
        float *r0 = ring0s + wv * 512, *r1 = ring1s + wv * 512;
        if (wide) mh_layer<true>(Ar, B0, B0 + (size_t)KG * 64, KG, r0, r1, lane, acc0, acc1);
        else mh_layer<false>(Ar, B0, B0, KG, r0, r1, lane, acc0, acc1);
        __syncthreads();                // every wave has read layer l's input rows
        // epilogue: register v of a tile = row 8 (v / 4) + 4 kh + v % 4, column col
        const float *bias = a.bias[br][l];
        const int n0 = 32 * cb0;
        if (wide) {
            const float bj0 = bias[n0 + col], bj1 = bias[n0 + 32 + col];
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                float *d = act + (8 * (reg >> 2) + 4 * kh + (reg & 3)) * MH_P + n0 + col;
                d[0] = mh_tanh(acc0[reg] + bj0);
                d[32] = mh_tanh(acc1[reg] + bj1);
            }
        } else {
            const float bj = bias[n0 + col];
#pragma unroll
            for (int reg = 0; reg < 16; ++reg)
                act[(8 * (reg >> 2) + 4 * kh + (reg & 3)) * MH_P + n0 + col] = mh_tanh((acc0[reg] + acc1[reg]) + bj);
        }
        __syncthreads();
        K = N;
    }
    // ---- head: the weights into the (drained) ring space, then 8 lanes per row ----
    float *hwa = ring0s, *hwv = ring1s;
    if (br == 0)
        for (int f = tid; f < a.A * P; f += 256) hwa[f] = a.wa[f];
    else
        for (int f = tid; f < P; f += 256) hwv[f] = a.wv[f];
    __syncthreads();
    const int r = tid >> 3, p = tid & 7;
    const int m = m0 + r;
    const float *h = act + r * MH_P;
    if (br == 0) {
        float lg[MH_MAXA];
#pragma unroll
        for (int k = 0; k < MH_MAXA; ++k) lg[k] = 0.0f;
        for (int j = p; j < P; j += 8) {
            const float hv = h[j];
#pragma unroll
            for (int k = 0; k < MH_MAXA; ++k)
                if (k < a.A) lg[k] += hv * hwa[k * P + j];
        }
#pragma unroll
        for (int k = 0; k < MH_MAXA; ++k) {
            lg[k] += __shfl_xor(lg[k], 1, 8);
            lg[k] += __shfl_xor(lg[k], 2, 8);
            lg[k] += __shfl_xor(lg[k], 4, 8);
        }
        if (p != 0 || m >= a.M) return;
        float mx = -INFINITY;
#pragma unroll
        for (int k = 0; k < MH_MAXA; ++k) {
            lg[k] = k < a.A ? lg[k] + a.ba[k] : -INFINITY;
            mx = fmaxf(mx, lg[k]);
        }
        float se = 0.0f;
#pragma unroll
        for (int k = 0; k < MH_MAXA; ++k)
            if (k < a.A) se += expf(lg[k] - mx);
        const float lse = mx + logf(se);
        int act_i = a.A - 1;
        if (a.deterministic) {
            float best = lg[0];
            act_i = 0;
#pragma unroll
            for (int k = 1; k < MH_MAXA; ++k)
                if (k < a.A && lg[k] > best) {
                    best = lg[k];
                    act_i = k;
                }
        } else {
            const uint32_t w0 = vn_detail::philox_word0(a.seed, (uint64_t)(a.gid_base + m), a.t | (1ull << 63));
            const float u = (float)(w0 >> 8) * (1.0f / 16777216.0f);
            float cdf = 0.0f;
#pragma unroll
            for (int k = 0; k < MH_MAXA; ++k)
                if (k < a.A - 1) {
                    cdf += expf(lg[k] - lse);
                    if (u < cdf && act_i == a.A - 1) act_i = k;   // the first crossing
                }
        }
        float lp = lg[0];
#pragma unroll
        for (int k = 1; k < MH_MAXA; ++k)
            if (k == act_i) lp = lg[k];
        a.actions[m] = act_i;
        a.log_probs[m] = lp - lse;
    } else {
        float v = 0.0f;
        for (int j = p; j < P; j += 8) v += h[j] * hwv[j];
        v += __shfl_xor(v, 1, 8);
        v += __shfl_xor(v, 2, 8);
        v += __shfl_xor(v, 4, 8);
        if (p == 0 && m < a.M) a.values[m] = v + a.bv[0];
    }
}

}  // namespace

extern "C" {

int vn_lstm_fused_f32(const float *x, int32_t obs_dim, const float *h_in, const float *w_packed, int32_t Kp,
                      const float *bias, const float *c_in, const float *start, float *c_out, float *h_out,
                      int32_t n_lstm, int32_t N, int32_t H, void *stream) {
    if (!x || !h_in || !w_packed || !bias || !c_in || !c_out || !h_out) return fail(VN_ERR_INVALID, "NULL argument");
    if (h_in == h_out) return fail(VN_ERR_INVALID, "h_in and h_out must differ (other blocks read h_in)");
    const int kx = (obs_dim + PF_KC - 1) / PF_KC * PF_KC;
    if (n_lstm < 1 || N < 1 || obs_dim < 4 || H < LS_UNITS || (H % LS_UNITS) || Kp != kx + H)
        return fail(VN_ERR_INVALID, "bad sizes n_lstm=%d N=%d obs_dim=%d H=%d Kp=%d (H %% 64 == 0, Kp == %d)",
                    n_lstm, N, obs_dim, H, Kp, kx + H);
    if ((reinterpret_cast<uintptr_t>(h_in) | reinterpret_cast<uintptr_t>(w_packed) |
         ((obs_dim & 3) == 0 ? reinterpret_cast<uintptr_t>(x) : 0)) & 15)
        return fail(VN_ERR_INVALID, "x / h_in / w_packed must be 16-byte aligned");
    const int ncombo = n_lstm * (H / LS_UNITS);
    const int n_items = (N + LS_ROWS - 1) / LS_ROWS * ncombo;
    // persistent grid: the co-resident block count (2 per CU), a multiple of 8
    // so a block's items stay on one XCD
    int dev = 0, cus = 0;
    VN_HIP(hipGetDevice(&dev));
    VN_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int slots = (2 * cus + 7) / 8 * 8;
    const dim3 grid((unsigned)(n_items < slots ? n_items : slots));
#define VN_LS_LAUNCH(VX, MK)                                                                                    \
    hipLaunchKernelGGL((lstm_fused_f32_kernel<VX, MK>), grid, dim3(256), 0, (hipStream_t)stream, x,             \
                       (int)obs_dim, kx, h_in, w_packed, (int)Kp, bias, c_in, start, c_out, h_out, (int)N, (int)H, \
                       ncombo, n_items)
    if ((obs_dim & 3) == 0) {
        if (start) VN_LS_LAUNCH(true, true);
        else VN_LS_LAUNCH(true, false);
    } else {
        if (start) VN_LS_LAUNCH(false, true);
        else VN_LS_LAUNCH(false, false);
    }
#undef VN_LS_LAUNCH
    VN_HIP(hipGetLastError());
    return VN_OK;
}

int vn_linear_f32(int32_t n_branch, const float *const *x, int64_t ldx, const float *const *w_packed,
                  const float *const *bias, float *const *y, int32_t M, int32_t K, int32_t Nout, int32_t tanh_act,
                  void *stream) {
    if (n_branch < 1 || n_branch > 2 || !x || !w_packed || !bias || !y) return fail(VN_ERR_INVALID, "bad arguments");
    if (M < 1 || K < PF_KC || (K % PF_KC) || Nout < LN_COLS || (Nout % LN_COLS) || ldx < K || (ldx & 3))
        return fail(VN_ERR_INVALID, "bad sizes M=%d K=%d Nout=%d ldx=%lld (K %% 16, Nout %% 128, ldx %% 4)", M, K,
                    Nout, (long long)ldx);
    LinearArgs a{};
    for (int i = 0; i < n_branch; ++i) {
        if (!x[i] || !w_packed[i] || !bias[i] || !y[i]) return fail(VN_ERR_INVALID, "NULL argument (branch %d)", i);
        if ((reinterpret_cast<uintptr_t>(x[i]) | reinterpret_cast<uintptr_t>(w_packed[i])) & 15)
            return fail(VN_ERR_INVALID, "x / w_packed must be 16-byte aligned");
        a.x[i] = x[i];
        a.wp[i] = w_packed[i];
        a.bias[i] = bias[i];
        a.y[i] = y[i];
    }
    const int ncb = Nout / LN_COLS;
    const dim3 grid((unsigned)((M + LN_ROWS - 1) / LN_ROWS) * (unsigned)ncb, (unsigned)n_branch);
    if (tanh_act)
        hipLaunchKernelGGL((linear_f32_kernel<true>), grid, dim3(256), 0, (hipStream_t)stream, a, ldx, (int)M, (int)K,
                           (int)Nout, ncb);
    else
        hipLaunchKernelGGL((linear_f32_kernel<false>), grid, dim3(256), 0, (hipStream_t)stream, a, ldx, (int)M,
                           (int)K, (int)Nout, ncb);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

int vn_mlp_head_f32(int32_t n_branch, const float *const *x, int64_t ldx, int32_t K0, int32_t n_layers,
                    const int32_t *widths, const float *const *w_t, const float *const *bias, const float *w_action,
                    const float *b_action, int32_t n_actions, const float *w_value, const float *b_value,
                    uint64_t sample_seed, uint64_t t, int64_t agent_id_base, int32_t deterministic, int32_t *actions,
                    float *log_probs, float *values, int32_t M, void *stream) {
    if ((n_branch != 1 && n_branch != 2) || !x || !widths || !w_t || !bias || !w_value || !b_value || !values)
        return fail(VN_ERR_INVALID, "bad arguments");
    if (n_layers < 1 || n_layers > MH_MAXL) return fail(VN_ERR_INVALID, "n_layers %d outside 1..%d", n_layers, MH_MAXL);
    if (M < 1 || K0 < 16 || K0 > 256 || (K0 % 16) || ldx < K0 || (ldx & 3))
        return fail(VN_ERR_INVALID, "bad sizes M=%d K0=%d ldx=%lld (K0 %% 16, <= 256; ldx %% 4)", M, K0,
                    (long long)ldx);
    if (n_branch == 2 && (!w_action || !b_action || !actions || !log_probs || n_actions < 1 || n_actions > MH_MAXA))
        return fail(VN_ERR_INVALID, "the pi branch needs the action head (1 <= n_actions <= %d) and outputs", MH_MAXA);
    MlpHeadArgs a{};
    a.ldx = ldx;
    a.K0 = K0;
    a.n_layers = n_layers;
    for (int l = 0; l < n_layers; ++l) {
        if (widths[l] != 128 && widths[l] != 256) return fail(VN_ERR_INVALID, "layer %d width %d: 128 or 256", l, widths[l]);
        a.width[l] = widths[l];
    }
    if (a.width[n_layers - 1] > MH_MAXP) return fail(VN_ERR_INVALID, "head width > %d", MH_MAXP);
    const int br0 = n_branch == 2 ? 0 : 1;
    for (int b = 0; b < n_branch; ++b) {
        if (!x[b] || (reinterpret_cast<uintptr_t>(x[b]) & 15)) return fail(VN_ERR_INVALID, "x[%d]: NULL or not 16-B aligned", b);
        a.x[br0 + b] = x[b];
        for (int l = 0; l < n_layers; ++l) {
            const float *w = w_t[b * n_layers + l];
            if (!w || (reinterpret_cast<uintptr_t>(w) & 15) || !bias[b * n_layers + l])
                return fail(VN_ERR_INVALID, "branch %d layer %d: NULL or unaligned weights", b, l);
            a.wp[br0 + b][l] = w;
            a.bias[br0 + b][l] = bias[b * n_layers + l];
        }
    }
    a.wa = w_action;
    a.ba = b_action;
    a.wv = w_value;
    a.bv = b_value;
    a.actions = actions;
    a.log_probs = log_probs;
    a.values = values;
    a.seed = sample_seed;
    a.t = t;
    a.gid_base = agent_id_base;
    a.A = n_branch == 2 ? n_actions : 0;
    a.M = M;
    a.br0 = br0;
    a.deterministic = deterministic;
    const dim3 grid((unsigned)((M + MH_R - 1) / MH_R), (unsigned)n_branch);
    hipLaunchKernelGGL(mlp_head_f32_kernel, grid, dim3(256), 0, (hipStream_t)stream, a);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

}  // extern "C"
