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

__device__ __forceinline__ float sigm_f32(float x) { return 1.0f / (1.0f + expf(-x)); }

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

template <bool VEC_X, bool MASK>
__global__ __launch_bounds__(256, 2) void lstm_fused_f32_kernel(const float *__restrict__ x, int obs_dim, int kx,
                                                                const float *__restrict__ hin,
                                                                const float *__restrict__ wp, int Kp,
                                                                const float *__restrict__ bias, const float *c_in,
                                                                const float *__restrict__ start, float *c_out,
                                                                float *h_out, int N, int H, int ncombo) {
    __shared__ float As[2][PF_KC][PF_AP];
    __shared__ __attribute__((aligned(16))) float Bs[2][PF_KC][LS_COLS];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int ublocks = H / LS_UNITS;
    const int ntiles = (N + LS_ROWS - 1) / LS_ROWS;
    // 1-D grid over (row tile, combo = LSTM x 64-unit block).  Blocks go to the
    // 8 XCDs round-robin by id; when the tile count allows, the combos of one
    // row tile get ids of one residue mod 8 (same XCD, close in time), so the
    // tile's x / h rows are fetched into that XCD's L2 once.
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
    const int b = combo / ublocks, ub = combo - b * ublocks;
    const int n_base = tile * LS_ROWS, u_base = ub * LS_UNITS;
    const float *wblk = wp + ((size_t)b * ublocks + ub) * (size_t)Kp * LS_COLS;
    const float *hb = hin + (size_t)b * N * H;
    const int nchunks = Kp / PF_KC;

    // A staging: thread covers (row q>>2, k 4(q&3) .. +3) for q = tid, tid + 256
    int arow[2];
    bool azero[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int q = tid + 256 * i;
        const int n = min(n_base + (q >> 2), N - 1);
        arow[i] = n;
        azero[i] = MASK && start[n] != 0.0f;
    }
    const int kq = (tid & 3) * 4;
    // staging registers, named (an indexed array lives in scratch); the loads
    // are unconditional from a selected address and the zeroing happens when
    // the registers are written to LDS, so nothing waits between issuing the
    // next chunk's loads and this chunk's MFMAs
    float4 ra0, ra1, rb0, rb1, rb2, rb3;
#define LS_A_LOAD(dst, i)                                                                                    \
    {                                                                                                        \
        if (VEC_X) {                                                                                         \
            const float *p_ = isx_ ? x + (size_t)arow[i] * obs_dim + min(k_, obs_dim - 4)                    \
                                   : hb + (size_t)arow[i] * H + (k_ - kx);                                   \
            dst = *reinterpret_cast<const float4 *>(p_);                                                     \
        } else {                                                                                             \
            const float *p_ = isx_ ? x + (size_t)arow[i] * obs_dim : hb + (size_t)arow[i] * H - kx;          \
            const int lim_ = isx_ ? obs_dim - 1 : 0x7fffffff;                                                \
            dst.x = p_[min(k_ + 0, lim_)];                                                                   \
            dst.y = p_[min(k_ + 1, lim_)];                                                                   \
            dst.z = p_[min(k_ + 2, lim_)];                                                                   \
            dst.w = p_[min(k_ + 3, lim_)];                                                                   \
        }                                                                                                    \
    }
#define LS_LOAD(ch)                                                                                          \
    {                                                                                                        \
        const int k_ = (ch) * PF_KC + kq;                                                                    \
        const bool isx_ = (ch) * PF_KC < kx; /* block-uniform: a chunk is all x or all h (kx % 16 == 0) */   \
        LS_A_LOAD(ra0, 0) LS_A_LOAD(ra1, 1)                                                                  \
        const float4 *pb_ = reinterpret_cast<const float4 *>(wblk + (size_t)(ch) * PF_KC * LS_COLS) + tid;   \
        rb0 = pb_[0];                                                                                        \
        rb1 = pb_[256];                                                                                      \
        rb2 = pb_[512];                                                                                      \
        rb3 = pb_[768];                                                                                      \
    }
#define LS_A_PUT(v, i)                                                                                       \
    {                                                                                                        \
        const int r_ = (tid + 256 * (i)) >> 2;                                                               \
        float4 v_ = v;                                                                                       \
        if (isx_) {                                                                                          \
            if (k_ + 0 >= obs_dim) v_.x = 0.0f;                                                              \
            if (k_ + 1 >= obs_dim) v_.y = 0.0f;                                                              \
            if (k_ + 2 >= obs_dim) v_.z = 0.0f;                                                              \
            if (k_ + 3 >= obs_dim) v_.w = 0.0f;                                                              \
        } else if (MASK && azero[i]) {                                                                       \
            v_ = make_float4(0.f, 0.f, 0.f, 0.f);                                                            \
        }                                                                                                    \
        As[buf_][kq + 0][r_] = v_.x;                                                                         \
        As[buf_][kq + 1][r_] = v_.y;                                                                         \
        As[buf_][kq + 2][r_] = v_.z;                                                                         \
        As[buf_][kq + 3][r_] = v_.w;                                                                         \
    }
#define LS_STORE(ch)                                                                                         \
    {                                                                                                        \
        const int buf_ = (ch) & 1;                                                                           \
        const int k_ = (ch) * PF_KC + kq;                                                                    \
        const bool isx_ = (ch) * PF_KC < kx;                                                                 \
        LS_A_PUT(ra0, 0) LS_A_PUT(ra1, 1)                                                                    \
        float4 *pl_ = reinterpret_cast<float4 *>(&Bs[buf_][0][0]) + tid;                                     \
        pl_[0] = rb0;                                                                                        \
        pl_[256] = rb1;                                                                                      \
        pl_[512] = rb2;                                                                                      \
        pl_[768] = rb3;                                                                                      \
    }

    f32x16_t acc[2][4];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[t][g] = zero16();
    const int wr = (wv & 1) * 64, wu = (wv >> 1) * 32;
    const int col = lane & 31, kh = lane >> 5;

    LS_LOAD(0)
    LS_STORE(0)
    __syncthreads();
    for (int ch = 0; ch < nchunks; ++ch) {
        // the next chunk's loads, in flight during this chunk's MFMAs (the last
        // iteration reloads its own chunk into the idle buffer: unconditional,
        // so the staging stays in registers)
        const int nx = ch + 1 < nchunks ? ch + 1 : ch;
        LS_LOAD(nx)
        __builtin_amdgcn_sched_barrier(0);
        const int buf = ch & 1;
#pragma unroll
        for (int s = 0; s < PF_KC / 2; ++s) {
            const int kk = 2 * s + kh;
            const float a0 = As[buf][kk][wr + col], a1 = As[buf][kk][wr + 32 + col];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float bv = Bs[buf][kk][g * LS_UNITS + wu + col];
                acc[0][g] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, bv, acc[0][g], 0, 0, 0);
                acc[1][g] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, bv, acc[1][g], 0, 0, 0);
            }
        }
        LS_STORE(nx)
        __syncthreads();
    }
#undef LS_A_LOAD
#undef LS_A_PUT
#undef LS_LOAD
#undef LS_STORE

    // epilogue: lane holds unit u; gate g of (row, u) in acc[t][g][reg]
    const int u = u_base + wu + col;
    const float *bb = bias + (size_t)b * 4 * H;
    const float bi = bb[u], bf = bb[H + u], bg = bb[2 * H + u], bo = bb[3 * H + u];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        // the 16 states of this row tile loaded together before any store
        // (vmcnt retires in order: a load issued after a store waits for it)
        float cin[16];
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int n = min(n_base + wr + 32 * t + (reg & 3) + 8 * (reg >> 2) + 4 * kh, N - 1);
            const float v = c_in[((size_t)b * N + n) * H + u];
            cin[reg] = (MASK && start[n] != 0.0f) ? 0.0f : v;
        }
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int n = n_base + wr + 32 * t + (reg & 3) + 8 * (reg >> 2) + 4 * kh;
            if (n < N) {
                const size_t so = ((size_t)b * N + n) * H + u;
                const float ig = sigm_f32(acc[t][0][reg] + bi), fg = sigm_f32(acc[t][1][reg] + bf);
                const float gg = tanhf(acc[t][2][reg] + bg), og = sigm_f32(acc[t][3][reg] + bo);
                const float fc = fg * cin[reg], ig2 = ig * gg;
                const float cn = fc + ig2;
                c_out[so] = cn;
                h_out[so] = og * tanhf(cn);
            }
        }
    }
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
    for (int ch = 0; ch < nchunks; ++ch) {
        const int nx = ch + 1 < nchunks ? ch + 1 : ch;
        LN_LOAD(nx)
        __builtin_amdgcn_sched_barrier(0);
        const int buf = ch & 1;
#pragma unroll
        for (int s = 0; s < PF_KC / 2; ++s) {
            const int kk = 2 * s + kh;
            const float a0 = As[buf][kk][wr + col], a1 = As[buf][kk][wr + 32 + col];
            const float b0 = Bs[buf][kk][wc + col], b1 = Bs[buf][kk][wc + 32 + col];
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
        }
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
                    y[(size_t)n * Nout + j] = TANH ? tanhf(v) : v;
                }
            }
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
    const dim3 grid((unsigned)((N + LS_ROWS - 1) / LS_ROWS) * (unsigned)ncombo);
#define VN_LS_LAUNCH(VX, MK)                                                                                    \
    hipLaunchKernelGGL((lstm_fused_f32_kernel<VX, MK>), grid, dim3(256), 0, (hipStream_t)stream, x,             \
                       (int)obs_dim, kx, h_in, w_packed, (int)Kp, bias, c_in, start, c_out, h_out, (int)N, (int)H, \
                       ncombo)
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

}  // extern "C"
