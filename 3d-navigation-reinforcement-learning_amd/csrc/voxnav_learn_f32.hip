// voxnav_learn_f32.hip -- the PPO learner's LSTM time loops on the f32 matrix
// cores (sb3_contrib RecurrentPPO.train -> evaluate_actions ->
// _process_sequence, reached from model.learn at train/Grid_Train.py:228;
// hyperparameters train/Grid_Train.py:84-87).
//
// The learner re-runs the actor and critic LSTM (80 -> 256 each) over a
// minibatch's padded sequences [L, B] (B ~ 512 sequences of <= 128 steps for
// a 65,536-sample minibatch) and back-propagates through them.  A step's work
// is small (B x 2048 gate columns x K 336: 0.7 GFLOP) and strictly sequential,
// so the two loops are one launch per step, each spread over the whole chip:
//
//   lstm_fwd_step_kernel   block (LSTM, 32-unit block, 32-row tile): the four
//                          32 x 32 gate tiles of [x_t | h_{t-1}] @ [W_ih |
//                          W_hh]^T on v_mfma_f32_32x32x2_f32, K split over the
//                          block's 4 waves (one per SIMD), partial sums reduced
//                          through LDS, then the cell update (bias, i f g o,
//                          c, h) as the epilogue.  The input projection is part
//                          of the product (no separate gx GEMM / gx array).
//   lstm_bwd_step_kernel   block (LSTM, 32-unit block, 32-row tile): the
//                          recurrent gradient dh_{t} += dG_{t+1} @ W_hh (K =
//                          4H split over the 4 waves, reduced through LDS),
//                          then the cell backward (dG_t, dc_{t-1}) as the
//                          epilogue.
//
// Operands go global -> registers with no LDS staging: for the f32 MFMA lane
// l supplies A[row l%32][k] and B[k][col l%32] for the k of its half (l/32),
// and the sum over k is order-free across instructions, so lane (h, r) takes
// k = 8c + 4h + s at k-step s of chunk c -- four consecutive floats of its A
// row (one float4) -- and the weights are packed per lane so its B values are
// one float4 per gate (lstm_pack_*_kernel, once per loop).  f32 throughout
// (the reference's dtype; exact f32 products), accurate expf / tanhf in the
// epilogues, -ffp-contract=off like the rest of the library.

#include <hip/hip_runtime.h>

#include <cstdint>

#include "vn_common.h"

using vn_detail::fail;

namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16_t;

constexpr int LQ_ROWS = 32;    // rows per block (one MFMA row tile)
constexpr int LQ_UNITS = 32;   // hidden units per block
constexpr int LQ_KC = 8;       // K per chunk: 4 MFMA k-steps (2 k each, one per half-wave)

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

__device__ __forceinline__ f32x16_t zero16() {
    f32x16_t z;
#pragma unroll
    for (int r = 0; r < 16; ++r) z[r] = 0.0f;
    return z;
}

// Block -> (LSTM l, unit block ub, row tile rt).  Blocks b and b + 8 share an
// XCD: the row tiles of one (l, ub) -- which read the same weight slice every
// step -- are dealt to one XCD when the combination count allows.
struct LqBlock {
    int l, ub, rt;
};
__device__ __forceinline__ LqBlock lq_block(int id, int ncombo, int ntiles, int UB) {
    int combo, rt;
    if ((ncombo & 7) == 0) {
        const int xcd = id & 7, local = id >> 3;
        combo = xcd + 8 * (local / ntiles);
        rt = local - (local / ntiles) * ntiles;
    } else {
        combo = id / ntiles;
        rt = id - combo * ntiles;
    }
    LqBlock b;
    b.l = combo / UB;
    b.ub = combo - b.l * UB;
    b.rt = rt;
    return b;
}

// ---------------------------------------------------------------------------
// weight packing (once per loop).  UB = ceil(H / 32) unit blocks; units >= H
// and k beyond the operand are packed as zeros.
//   forward:  wpf[l][ub][c][h][u][g][s] = Wcat[l][g*H + 32 ub + u][8c + 4h + s]
//             Wcat = [W_ih | 0 (kx - D) | W_hh | 0], k < Kp = kx + Hp
//             (kx = D and Hp = H rounded up to 8)
//   backward: wpb[l][ub][c][h][u][s]    = W_hh[l][8c + 4h + s][32 ub + u], k < 4H
// ---------------------------------------------------------------------------
__global__ void lstm_pack_fwd_kernel(const float *__restrict__ w_ih, const float *__restrict__ w_hh, int n_lstm,
                                     int D, int kx, int H, int Kp, float *__restrict__ wpf) {
    const int NC = Kp / LQ_KC, UB = (H + LQ_UNITS - 1) / LQ_UNITS;
    const int64_t total = (int64_t)n_lstm * UB * NC * 2 * LQ_UNITS * 16;
    if (blockIdx.x == 0 && threadIdx.x < 64) wpf[total + threadIdx.x] = 0.0f;   // the zero block
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t r = i;
        const int s = (int)(r & 3);
        r >>= 2;
        const int g = (int)(r & 3);
        r >>= 2;
        const int u = (int)(r % LQ_UNITS);
        r /= LQ_UNITS;
        const int h = (int)(r & 1);
        r >>= 1;
        const int c = (int)(r % NC);
        r /= NC;
        const int ub = (int)(r % UB);
        const int l = (int)(r / UB);
        const int k = LQ_KC * c + 4 * h + s;
        const int uu = LQ_UNITS * ub + u;
        const int row = g * H + uu;
        float v = 0.0f;
        if (uu < H) {
            if (k < D) v = w_ih[((int64_t)l * 4 * H + row) * D + k];
            else if (k >= kx && k - kx < H) v = w_hh[((int64_t)l * 4 * H + row) * H + (k - kx)];
        }
        wpf[i] = v;
    }
}

__global__ void lstm_pack_bwd_kernel(const float *__restrict__ w_hh, int n_lstm, int H, int NC,
                                     float *__restrict__ wpb) {
    const int UB = (H + LQ_UNITS - 1) / LQ_UNITS;
    const int64_t total = (int64_t)n_lstm * UB * NC * 2 * LQ_UNITS * 4;
    if (blockIdx.x == 0 && threadIdx.x < 64) wpb[total + threadIdx.x] = 0.0f;   // the zero block
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t r = i;
        const int s = (int)(r & 3);
        r >>= 2;
        const int u = (int)(r % LQ_UNITS);
        r /= LQ_UNITS;
        const int h = (int)(r & 1);
        r >>= 1;
        const int c = (int)(r % NC);
        r /= NC;
        const int ub = (int)(r % UB);
        const int l = (int)(r / UB);
        const int k = LQ_KC * c + 4 * h + s;
        const int uu = LQ_UNITS * ub + u;
        wpb[i] = (uu < H && k < 4 * H) ? w_hh[((int64_t)l * 4 * H + k) * H + uu] : 0.0f;
    }
}

// ---------------------------------------------------------------------------
// forward step.  Per LSTM l (lstm strides in floats):
//   x_t     [B][D]                          (shared by the LSTMs; D % 4 == 0)
//   h_prev  l * s_state + [B][H]            c_prev likewise
//   h_new, c_new  l * s_state + [B][H]
//   act     l * s_act + [B][4H]             out: i, f, g, o (after the nonlinearity)
//   wpf     packed (above), bias [n_lstm][4H] = b_ih + b_hh
// Operand loads are unconditional (a chunk index past the wave's last is
// clamped, its data unused) and four chunks deep, so the compiler's vmcnt
// waits stay exact and ~4 x 16 MFMAs cover each load's latency.
// ---------------------------------------------------------------------------
// NCT > 0: the chunk count as a compile-time constant (the policy's shape;
// the chunk loop fully unrolled, so no loop back edge makes the waitcnt pass
// drain every load), 0: run time.
template <int NCT>
__global__ __launch_bounds__(256, 2) void lstm_fwd_step_kernel(const float *__restrict__ x_t, int D, int kx,
                                                               const float *__restrict__ h_prev,
                                                               const float *__restrict__ c_prev,
                                                               float *__restrict__ h_new, float *__restrict__ c_new,
                                                               int64_t s_state, float *__restrict__ act,
                                                               int64_t s_act, const float *__restrict__ wpf,
                                                               const float *__restrict__ zero,
                                                               const float *__restrict__ bias, int B, int H,
                                                               int NC_rt, int ncombo, int ntiles) {
    const int NC = NCT > 0 ? NCT : NC_rt;
    __shared__ float red[4][4][16][64];   // [wave][gate][acc register][lane]: 64 KiB
    // the wave index as a scalar: the chunk loop and its guards are then
    // wave-uniform branches (no exec masking, no accumulator copies)
    const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int hh = lane >> 5, c32 = lane & 31;
    const int UB = (H + LQ_UNITS - 1) / LQ_UNITS;
    const LqBlock blk = lq_block((int)blockIdx.x, ncombo, ntiles, UB);
    const int row0 = blk.rt * LQ_ROWS;
    const int arow = min(row0 + c32, B - 1);
    const float *xa = x_t + (int64_t)arow * D;
    const float *ha = h_prev + (int64_t)blk.l * s_state + (int64_t)arow * H;
    const float4 *wb = reinterpret_cast<const float4 *>(wpf) +
                       (((int64_t)blk.l * UB + blk.ub) * NC * 2 + hh) * (LQ_UNITS * 4) + c32 * 4;
    // named accumulators (an indexed array made the compiler copy all 64
    // registers at the loop back edge)
    f32x16_t acc0 = zero16(), acc1 = zero16(), acc2 = zero16(), acc3 = zero16();
    // one chunk: A = 4 consecutive k of the lane's row ([x | h], zero past
    // either part: a clamped address and a select, no branch), B = one float4 per gate
#define LQ_LD(S, cidx)                                                                                       \
    {                                                                                                        \
        const int cr_ = (cidx);                                                                              \
        const int cc_ = min(cr_, NC - 1);                                                                    \
        const int k_ = LQ_KC * cc_ + 4 * hh;                                                                 \
        /* past the wave's last chunk, or past the h part: the zero block (pointer select, no wait) */       \
        const float *p_ = cr_ >= NC ? zero : k_ < kx ? xa + k_ : (k_ - kx < H ? ha + (k_ - kx) : zero);      \
        S##a = *reinterpret_cast<const float4 *>(p_);                                                        \
        const float4 *pw_ = cr_ >= NC ? reinterpret_cast<const float4 *>(zero)                               \
                                      : wb + (int64_t)cc_ * (2 * LQ_UNITS * 4);                              \
        S##b0 = pw_[0];                                                                                      \
        S##b1 = pw_[1];                                                                                      \
        S##b2 = pw_[2];                                                                                      \
        S##b3 = pw_[3];                                                                                      \
    }
#define LQ_MM4(a, b0, b1, b2, b3)                                                                            \
    {                                                                                                        \
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b0, acc0, 0, 0, 0);                                   \
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b1, acc1, 0, 0, 0);                                   \
        acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b2, acc2, 0, 0, 0);                                   \
        acc3 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b3, acc3, 0, 0, 0);                                   \
    }
#define LQ_MM(S)                                                                                             \
    {                                                                                                        \
        LQ_MM4(S##a.x, S##b0.x, S##b1.x, S##b2.x, S##b3.x)                                                   \
        LQ_MM4(S##a.y, S##b0.y, S##b1.y, S##b2.y, S##b3.y)                                                   \
        LQ_MM4(S##a.z, S##b0.z, S##b1.z, S##b2.z, S##b3.z)                                                   \
        LQ_MM4(S##a.w, S##b0.w, S##b1.w, S##b2.w, S##b3.w)                                                   \
    }
    float4 s0a, s0b0, s0b1, s0b2, s0b3, s1a, s1b0, s1b1, s1b2, s1b3;
    float4 s2a, s2b0, s2b1, s2b2, s2b3, s3a, s3b0, s3b1, s3b2, s3b3;
    // this wave's chunks: wv, wv + 4, wv + 8, ...
    LQ_LD(s0, wv)
    LQ_LD(s1, wv + 4)
    LQ_LD(s2, wv + 8)
    LQ_LD(s3, wv + 12)
    // no guards in the loop: a stage past the wave's last chunk multiplies zeros
    // the same trip count for every wave (a stage past a wave's last chunk
    // multiplies zeros), a constant when NCT is
    const int n_it = (NC + 15) / 16;
#pragma unroll
    for (int it = 0; it < n_it; ++it) {
        const int c = wv + 16 * it;
        LQ_MM(s0)
        LQ_LD(s0, c + 16)
        __builtin_amdgcn_sched_barrier(0);
        LQ_MM(s1)
        LQ_LD(s1, c + 20)
        __builtin_amdgcn_sched_barrier(0);
        LQ_MM(s2)
        LQ_LD(s2, c + 24)
        __builtin_amdgcn_sched_barrier(0);
        LQ_MM(s3)
        LQ_LD(s3, c + 28)
        __builtin_amdgcn_sched_barrier(0);
    }
#undef LQ_LD
#undef LQ_MM4
#undef LQ_MM
    // reduce the 4 waves' partial tiles: wave w finishes accumulator registers
    // 4w .. 4w+3, i.e. rows 8w + 4hh + i (i < 4) of the tile, unit c32
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        red[wv][0][v][lane] = acc0[v];
        red[wv][1][v][lane] = acc1[v];
        red[wv][2][v][lane] = acc2[v];
        red[wv][3][v][lane] = acc3[v];
    }
    __syncthreads();
    const int u = LQ_UNITS * blk.ub + c32;
    if (u >= H) return;
    const float *bb = bias + (int64_t)blk.l * 4 * H;
    const float bi = bb[u], bf = bb[H + u], bg = bb[2 * H + u], bo = bb[3 * H + u];
    float cp[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {   // the c_prev loads together, before any store
        const int row = min(row0 + 8 * wv + 4 * hh + i, B - 1);
        cp[i] = c_prev[(int64_t)blk.l * s_state + (int64_t)row * H + u];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int v = 4 * wv + i;
        float pre[4];
#pragma unroll
        for (int g = 0; g < 4; ++g)
            pre[g] = ((red[0][g][v][lane] + red[1][g][v][lane]) + red[2][g][v][lane]) + red[3][g][v][lane];
        const int row = row0 + 8 * wv + 4 * hh + i;
        if (row < B) {
            const int64_t so = (int64_t)blk.l * s_state + (int64_t)row * H + u;
            const float ig = sigm(pre[0] + bi), fg = sigm(pre[1] + bf);
            const float gg = tanhf(pre[2] + bg), og = sigm(pre[3] + bo);
            const float fc = fg * cp[i], igg = ig * gg;
            const float cn = fc + igg;
            c_new[so] = cn;
            h_new[so] = og * tanhf(cn);
            float *pa = act + (int64_t)blk.l * s_act + (int64_t)row * 4 * H + u;
            pa[0] = ig;
            pa[H] = fg;
            pa[2 * H] = gg;
            pa[3 * H] = og;
        }
    }
}

// ---------------------------------------------------------------------------
// backward step.  Per LSTM l:
//   dG_next  l * s_dg + [B][4H]     dG of step t+1 (NULL at the last step: dh_rec = 0)
//   dh_out   l * s_dho + [B][H]     gradient of the step's output h_t
//   dc       l * B * H + [B][H]     in: dL/dc_t, out: dL/dc_{t-1} (each element by one thread)
//   act      l * s_act + [B][4H]    i, f, g, o of step t
//   c_prev, c_new  l * s_state + [B][H]
//   dG       l * s_dg + [B][4H]     out: dG_t
//   wpb      packed W_hh (above), NC = 4H / 8 chunks (4H % 8 == 0)
// dh_only != NULL: only dh_rec = dG_next @ W_hh is computed and stored there
// ([n_lstm][B][H]; the gradient of h0).  Eight chunks in flight per wave
// (unconditional, clamped loads as in the forward kernel).
// ---------------------------------------------------------------------------
template <int NCT>
__global__ __launch_bounds__(256, 2) void lstm_bwd_step_kernel(const float *__restrict__ dG_next, int64_t s_dg,
                                                               const float *__restrict__ dh_out, int64_t s_dho,
                                                               float *__restrict__ dc,
                                                               const float *__restrict__ act, int64_t s_act,
                                                               const float *__restrict__ c_prev,
                                                               const float *__restrict__ c_new, int64_t s_state,
                                                               float *__restrict__ dG, float *__restrict__ dh_only,
                                                               const float *__restrict__ wpb,
                                                               const float *__restrict__ zero, int B, int H,
                                                               int NC_rt, int ncombo, int ntiles) {
    const int NC = NCT > 0 ? NCT : NC_rt;
    __shared__ float red[4][16][64];   // 16 KiB
    // the wave index as a scalar: the chunk loop and its guards are then
    // wave-uniform branches (no exec masking, no accumulator copies)
    const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int hh = lane >> 5, c32 = lane & 31;
    const int UB = (H + LQ_UNITS - 1) / LQ_UNITS, K = 4 * H;
    const LqBlock blk = lq_block((int)blockIdx.x, ncombo, ntiles, UB);
    const int row0 = blk.rt * LQ_ROWS;
    f32x16_t acc = zero16();
    if (dG_next) {
        const int arow = min(row0 + c32, B - 1);
        const float4 *pa = reinterpret_cast<const float4 *>(dG_next + (int64_t)blk.l * s_dg + (int64_t)arow * K) + hh;
        const float4 *pb = reinterpret_cast<const float4 *>(wpb) +
                           (((int64_t)blk.l * UB + blk.ub) * NC * 2 + hh) * LQ_UNITS + c32;
        const float4 *z4 = reinterpret_cast<const float4 *>(zero);   // past the wave's last chunk
#define LB_LD(j, cidx)                                                                                       \
    {                                                                                                        \
        const int cr_ = (cidx);                                                                              \
        const int cc_ = min(cr_, NC - 1);                                                                    \
        const float4 *pa_ = cr_ >= NC ? z4 : pa + 2 * cc_;   /* pointer select, then one load */          \
        const float4 *pb_ = cr_ >= NC ? z4 : pb + (int64_t)cc_ * 2 * LQ_UNITS;                               \
        a##j = *pa_;                                                                                         \
        b##j = *pb_;                                                                                         \
    }
#define LB_MM(j)                                                                                             \
    {                                                                                                        \
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a##j.x, b##j.x, acc, 0, 0, 0);                            \
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a##j.y, b##j.y, acc, 0, 0, 0);                            \
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a##j.z, b##j.z, acc, 0, 0, 0);                            \
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a##j.w, b##j.w, acc, 0, 0, 0);                            \
    }
#define LB_STAGE(j, c)                                                                                       \
    {                                                                                                        \
        LB_MM(j)                                                                                             \
        LB_LD(j, (c) + 4 * ((j) + 8))                                                                        \
        __builtin_amdgcn_sched_barrier(0); /* keep the loads 8 stages ahead (not sunk to their use) */       \
    }
        float4 a0, a1, a2, a3, a4, a5, a6, a7, b0, b1, b2, b3, b4, b5, b6, b7;
        LB_LD(0, wv) LB_LD(1, wv + 4) LB_LD(2, wv + 8) LB_LD(3, wv + 12)
        LB_LD(4, wv + 16) LB_LD(5, wv + 20) LB_LD(6, wv + 24) LB_LD(7, wv + 28)
        const int n_it = (NC + 31) / 32;   // same for every wave, a constant when NCT is
#pragma unroll
        for (int it = 0; it < n_it; ++it) {
            const int c = wv + 32 * it;
            LB_STAGE(0, c) LB_STAGE(1, c) LB_STAGE(2, c) LB_STAGE(3, c)
            LB_STAGE(4, c) LB_STAGE(5, c) LB_STAGE(6, c) LB_STAGE(7, c)
        }
#undef LB_LD
#undef LB_MM
#undef LB_STAGE
    }
#pragma unroll
    for (int v = 0; v < 16; ++v) red[wv][v][lane] = acc[v];
    __syncthreads();
    const int u = LQ_UNITS * blk.ub + c32;
    if (u >= H) return;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int v = 4 * wv + i;
        const float dh_rec = ((red[0][v][lane] + red[1][v][lane]) + red[2][v][lane]) + red[3][v][lane];
        const int row = row0 + 8 * wv + 4 * hh + i;
        if (row >= B) continue;
        if (dh_only) {
            dh_only[((int64_t)blk.l * B + row) * H + u] = dh_rec;
            continue;
        }
        const float dh = dh_out[(int64_t)blk.l * s_dho + (int64_t)row * H + u] + dh_rec;
        const int64_t so = (int64_t)blk.l * s_state + (int64_t)row * H + u;
        const int64_t sd = ((int64_t)blk.l * B + row) * H + u;
        const float *pa = act + (int64_t)blk.l * s_act + (int64_t)row * 4 * H + u;
        const float ig = pa[0], fg = pa[H], gg = pa[2 * H], og = pa[3 * H];
        const float cp = c_prev[so], tc = tanhf(c_new[so]);
        const float dtc = dh * og;
        const float dcc = dc[sd] + dtc * (1.0f - tc * tc);
        float *pg = dG + (int64_t)blk.l * s_dg + (int64_t)row * K + u;
        pg[0] = dcc * gg * (ig * (1.0f - ig));
        pg[H] = dcc * cp * (fg * (1.0f - fg));
        pg[2 * H] = dcc * ig * (1.0f - gg * gg);
        pg[3 * H] = dh * tc * (og * (1.0f - og));
        dc[sd] = dcc * fg;
    }
}

int check_dims(int n_lstm, int L, int B, int H) {
    if (n_lstm < 1 || L < 1 || B < 1 || H < 4 || (H % 4))
        return fail(VN_ERR_INVALID, "bad sizes n_lstm=%d L=%d B=%d H=%d (H a multiple of 4)", n_lstm, L, B, H);
    return VN_OK;
}

struct LqGeom {
    int kx, Kp, NCf, NCb, UB;
    int64_t fwd_floats, bwd_floats;
};
LqGeom lq_geom(int n_lstm, int D, int H) {
    LqGeom g;
    g.kx = D;                                              // D % 4 == 0 (checked): x and h parts float4-aligned
    const int Hp = (H + LQ_KC - 1) / LQ_KC * LQ_KC;
    g.Kp = (g.kx + Hp + LQ_KC - 1) / LQ_KC * LQ_KC;
    g.NCf = g.Kp / LQ_KC;
    g.NCb = (4 * H + LQ_KC - 1) / LQ_KC;
    g.UB = (H + LQ_UNITS - 1) / LQ_UNITS;
    // + a 64-float zero block (the operand of chunks past a wave's last one)
    g.fwd_floats = (int64_t)n_lstm * g.UB * g.NCf * 2 * LQ_UNITS * 16 + 64;
    g.bwd_floats = (int64_t)n_lstm * g.UB * g.NCb * 2 * LQ_UNITS * 4 + 64;
    return g;
}

}  // namespace

extern "C" {

int vn_lstm_seq_pack_size(int32_t n_lstm, int32_t D, int32_t H, int64_t *fwd_floats, int64_t *bwd_floats) {
    if (!fwd_floats || !bwd_floats) return fail(VN_ERR_INVALID, "NULL argument");
    const LqGeom g = lq_geom(n_lstm, D, H);
    *fwd_floats = g.fwd_floats;
    *bwd_floats = g.bwd_floats;
    return VN_OK;
}

int vn_lstm_seq_fwd_mfma(const float *x, int32_t D, const float *w_ih, const float *w_hh, const float *bias,
                         float *wpack, float *hs, float *cs, float *act, int32_t n_lstm, int32_t L, int32_t B,
                         int32_t H, void *stream) {
    if (!x || !w_ih || !w_hh || !bias || !wpack || !hs || !cs || !act) return fail(VN_ERR_INVALID, "NULL argument");
    if (int rc = check_dims(n_lstm, L, B, H)) return rc;
    if (D < 4 || (D % 4)) return fail(VN_ERR_INVALID, "D must be a positive multiple of 4 (got %d)", D);
    const hipStream_t st = (hipStream_t)stream;
    const LqGeom g = lq_geom(n_lstm, D, H);
    const int64_t pb = (g.fwd_floats + 255) / 256;
    hipLaunchKernelGGL(lstm_pack_fwd_kernel, dim3((unsigned)(pb < 4096 ? pb : 4096)), dim3(256), 0, st, w_ih, w_hh,
                       n_lstm, D, g.kx, H, g.Kp, wpack);
    const int ncombo = n_lstm * g.UB, ntiles = (B + LQ_ROWS - 1) / LQ_ROWS;
    const dim3 grid((unsigned)(ncombo * ntiles));
    const int64_t s_state = (int64_t)(L + 1) * B * H, s_act = (int64_t)B * 4 * H;
    for (int t = 0; t < L; ++t) {
        const int64_t o = (int64_t)t * B * H;
        auto kern = g.NCf == 42 ? lstm_fwd_step_kernel<42> : lstm_fwd_step_kernel<0>;   // 42: D 80, H 256
        hipLaunchKernelGGL(kern, grid, dim3(256), 0, st, x + (int64_t)t * B * D, D, g.kx, hs + o, cs + o,
                           hs + o + (int64_t)B * H, cs + o + (int64_t)B * H, s_state,
                           act + (int64_t)t * n_lstm * B * 4 * H, s_act, wpack, wpack + g.fwd_floats - 64, bias, B,
                           H, g.NCf, ncombo, ntiles);
    }
    VN_HIP(hipGetLastError());
    return VN_OK;
}

int vn_lstm_seq_bwd_mfma(const float *dh_out, const float *w_hh, float *wpack, const float *act, const float *cs,
                         float *dG, float *dc, float *dh0, int32_t n_lstm, int32_t L, int32_t B, int32_t H,
                         void *stream) {
    if (!dh_out || !w_hh || !wpack || !act || !cs || !dG || !dc) return fail(VN_ERR_INVALID, "NULL argument");
    if (int rc = check_dims(n_lstm, L, B, H)) return rc;
    const hipStream_t st = (hipStream_t)stream;
    const LqGeom g = lq_geom(n_lstm, 4, H);
    const int64_t pb = (g.bwd_floats + 255) / 256;
    hipLaunchKernelGGL(lstm_pack_bwd_kernel, dim3((unsigned)(pb < 4096 ? pb : 4096)), dim3(256), 0, st, w_hh, n_lstm,
                       H, g.NCb, wpack);
    const int ncombo = n_lstm * g.UB, ntiles = (B + LQ_ROWS - 1) / LQ_ROWS;
    const dim3 grid((unsigned)(ncombo * ntiles));
    const int64_t G = 4 * (int64_t)H;
    const int64_t s_state = (int64_t)(L + 1) * B * H, s_act = (int64_t)B * G, s_dg = (int64_t)L * B * G;
    const int64_t s_dho = (int64_t)L * B * H;
    auto kern = g.NCb == 128 ? lstm_bwd_step_kernel<128> : lstm_bwd_step_kernel<0>;   // 128: H 256
    for (int t = L - 1; t >= 0; --t) {
        hipLaunchKernelGGL(kern, grid, dim3(256), 0, st,
                           t < L - 1 ? dG + (int64_t)(t + 1) * B * G : nullptr, s_dg, dh_out + (int64_t)t * B * H,
                           s_dho, dc, act + (int64_t)t * n_lstm * B * G, s_act, cs + (int64_t)t * B * H,
                           cs + (int64_t)(t + 1) * B * H, s_state, dG + (int64_t)t * B * G, nullptr, wpack,
                           wpack + g.bwd_floats - 64, B, H, g.NCb, ncombo, ntiles);
    }
    if (dh0)
        hipLaunchKernelGGL(kern, grid, dim3(256), 0, st, dG, s_dg, dh_out, s_dho, dc, act, s_act, cs,
                           cs, s_state, dG, dh0, wpack, wpack + g.bwd_floats - 64, B, H, g.NCb, ncombo, ntiles);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

}  // extern "C"
