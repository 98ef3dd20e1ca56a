// voxnav_gemm_f32.hip -- the PPO learner's matrix products on the f32 matrix
// cores (v_mfma_f32_32x32x2_f32: exact f32 products at the f32 peak), the
// reference's dtype (SB3 policies are f32; train/Grid_Train.py:74-80).
//
// One kernel family covers every product of the learner step (sb3
// RecurrentPPO.train / PPO.train) -- no library GEMM:
//   forward   Y = act(X W^T + b)          X [M][K] row-major, W [N][K] row-major
//   backward  dX = dZ W                   dZ [M][K=out] row-major, W [K][N] k-major
//             dW = dZ^T X  (split-K)      dZ [K=rows][M] k-major, X [K][N] k-major
//   with dZ = dY (1 - Y^2) formed on load (AGRAD: the Tanh's backward fused
//   into the operand fetch, no dZ array) and, for dW, the bias gradient
//   sum_k dZ[k][m] from the same staged tiles.
//
// Block: 256 threads, a 128 x 128 tile of C, wave w owns rows 64 (w & 1) and
// columns 64 (w >> 1) as 2 x 2 accumulators.  K is staged through LDS in
// chunks of 16, double-buffered (the next chunk's global loads in flight
// during this chunk's MFMAs).  Both operands are staged k-major ([k][row],
// [k][col]) so every MFMA operand is one conflict-free ds_read_b32 (lane l
// supplies A[row l%32][k l/32], B[k l/32][col l%32]); a row-major operand is
// transposed on its way into LDS.  Split-K (gridDim.z > 1 along K) writes
// per-split partials that gemm_reduce_kernel sums in a fixed order (the result
// does not depend on timing).

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "vn_common.h"

using vn_detail::fail;

namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16_t;

constexpr int GT = 128;        // tile rows / cols
// K per chunk: 16 for the Linear forward and dX products (K = 80 .. 256:
// half the LDS, 4 waves per SIMD; measured 10-38 % faster than 32), 32 for the
// split-K weight gradients (long K per split; 16 measured no faster there)
constexpr int GK_LIN = 16, GK_TN = 32;
constexpr int GP = GT + 4;     // LDS pitch

__device__ __forceinline__ f32x16_t zero16() {
    f32x16_t z;
#pragma unroll
    for (int r = 0; r < 16; ++r) z[r] = 0.0f;
    return z;
}

struct GemmArgs {
    const float *a, *a2;   // A (and Y for AGRAD: element = a * (1 - a2 * a2))
    const float *b;
    const float *bias;     // EPI 1/2: [N]
    float *c;              // C [M][N] (ldc) or split partials [splits][M][N]
    float *colsum;         // optional (AGRAD, A k-major): split partials of sum_k A[k][m], [splits][M]
    int64_t lda, ldb, ldc;
    int64_t sa, sb, sc, sbias;   // batch strides (blockIdx.y = batch)
    int M, N, K, kper;     // kper: K per split (multiple of GK_TN, except the last split)
};

// EPI: 0 store, 1 tanh(acc + bias), 2 acc + bias, 3 split partial (c + split * M * N)
template <int GK, bool A_KM, bool B_KM, bool AGRAD, int EPI>
__global__ __launch_bounds__(256, 2) void gemm_f32_kernel(GemmArgs g) {
    constexpr int GNF = GK * GT / 4 / 256;   // float4 of one operand chunk per thread
    constexpr int GKQ = GK / 4;              // float4 per row of a row-major chunk
    __shared__ float As[2][GK][GP];
    __shared__ float Bs[2][GK][GP];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    // XCD-aware block order: blocks are dealt round-robin over the 8 XCDs
    // (b and b + 8 share one), so the linear id is re-dealt to make each
    // XCD's blocks one contiguous run of (split, batch, row tile, column
    // tile): the column tiles of a row tile -- and for split-K every tile of
    // a split -- then read their shared operand rows into ONE L2 (speed only;
    // any placement gives the same result)
    const int ntn = (g.N + GT - 1) / GT;
    const int nblk = (int)(gridDim.x * gridDim.y * gridDim.z);
    int vb = (int)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z));
    if ((nblk & 7) == 0) vb = (vb & 7) * (nblk >> 3) + (vb >> 3);
    const int tiles = (int)gridDim.x;
    const int tm = (vb % tiles) / ntn, tn = (vb % tiles) - tm * ntn;
    const int bt = (vb / tiles) % (int)gridDim.y, split = vb / (tiles * (int)gridDim.y);
    const int m0 = tm * GT, n0 = tn * GT;
    const int k0 = split * g.kper;
    const int k1 = min(g.K, k0 + g.kper);
    const float *A = g.a + bt * g.sa;
    const float *A2 = AGRAD ? g.a2 + bt * g.sa : nullptr;
    const float *Bm = g.b + bt * g.sb;
    const int nchunks = (k1 - k0 + GK - 1) / GK;
    // staging: thread covers 8 floats of each operand chunk (2 float4)
    //  k-major operand: chunk [GK][GT]: float4 f = tid + 256 i -> (k = f / 32, col 4 (f % 32))
    //  row-major operand: chunk [GT][GK]: float4 f -> (row = f / GKQ, k 4 (f % GKQ))
    float4 ra[GNF], rb[GNF];
    auto ld_op = [&](const float *P, const float *P2, int64_t ld, int base, int lim, bool km, bool grad, int kc,
                     float4 *r) {
#pragma unroll
        for (int i = 0; i < GNF; ++i) {
            const int f = tid + 256 * i;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f), y = v;
            if (km) {
                const int k = kc + (f >> 5), cc = base + 4 * (f & 31);
                if (k < k1) {
                    const int64_t o = (int64_t)k * ld + cc;
                    if (cc + 3 < lim && (ld & 3) == 0) {
                        v = *reinterpret_cast<const float4 *>(P + o);
                        if (grad) y = *reinterpret_cast<const float4 *>(P2 + o);
                    } else {
                        v.x = cc + 0 < lim ? P[o + 0] : 0.f;
                        v.y = cc + 1 < lim ? P[o + 1] : 0.f;
                        v.z = cc + 2 < lim ? P[o + 2] : 0.f;
                        v.w = cc + 3 < lim ? P[o + 3] : 0.f;
                        if (grad) {
                            y.x = cc + 0 < lim ? P2[o + 0] : 0.f;
                            y.y = cc + 1 < lim ? P2[o + 1] : 0.f;
                            y.z = cc + 2 < lim ? P2[o + 2] : 0.f;
                            y.w = cc + 3 < lim ? P2[o + 3] : 0.f;
                        }
                    }
                }
            } else {
                const int rr = base + f / GKQ, k = kc + 4 * (f % GKQ);
                if (rr < lim) {
                    const int64_t o = (int64_t)rr * ld + k;
                    if (k + 3 < k1 && (ld & 3) == 0) {
                        v = *reinterpret_cast<const float4 *>(P + o);
                        if (grad) y = *reinterpret_cast<const float4 *>(P2 + o);
                    } else {
                        v.x = k + 0 < k1 ? P[o + 0] : 0.f;
                        v.y = k + 1 < k1 ? P[o + 1] : 0.f;
                        v.z = k + 2 < k1 ? P[o + 2] : 0.f;
                        v.w = k + 3 < k1 ? P[o + 3] : 0.f;
                        if (grad) {
                            y.x = k + 0 < k1 ? P2[o + 0] : 0.f;
                            y.y = k + 1 < k1 ? P2[o + 1] : 0.f;
                            y.z = k + 2 < k1 ? P2[o + 2] : 0.f;
                            y.w = k + 3 < k1 ? P2[o + 3] : 0.f;
                        }
                    }
                }
            }
            if (grad) {   // dZ = dY (1 - Y^2): the Tanh backward, as torch's tanh_backward
                v.x = v.x * (1.0f - y.x * y.x);
                v.y = v.y * (1.0f - y.y * y.y);
                v.z = v.z * (1.0f - y.z * y.z);
                v.w = v.w * (1.0f - y.w * y.w);
            }
            r[i] = v;
        }
    };
    auto st_op = [&](float (*S)[GP], bool km, const float4 *r) {
#pragma unroll
        for (int i = 0; i < GNF; ++i) {
            const int f = tid + 256 * i;
            if (km) {
                *reinterpret_cast<float4 *>(&S[f >> 5][4 * (f & 31)]) = r[i];
            } else {
                const int rr = f / GKQ, k = 4 * (f % GKQ);
                S[k + 0][rr] = r[i].x;
                S[k + 1][rr] = r[i].y;
                S[k + 2][rr] = r[i].z;
                S[k + 3][rr] = r[i].w;
            }
        }
    };
    // column sums of A (the bias gradient of dW = dZ^T X): thread owns A column
    // tid & 127 (k-major A only), half the chunk's k each
    float csum = 0.0f;

    f32x16_t acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = zero16();
    const int wr = 64 * (wv & 1), wc = 64 * (wv >> 1);
    const int col = lane & 31, kh = lane >> 5;

    if (nchunks > 0) {
        ld_op(A, A2, g.lda, m0, g.M, A_KM, AGRAD, k0, ra);
        ld_op(Bm, nullptr, g.ldb, n0, g.N, B_KM, false, k0, rb);
        st_op(As[0], A_KM, ra);
        st_op(Bs[0], B_KM, rb);
    }
    __syncthreads();
    for (int ch = 0; ch < nchunks; ++ch) {
        const int bf = ch & 1;
        if (ch + 1 < nchunks) {
            ld_op(A, A2, g.lda, m0, g.M, A_KM, AGRAD, k0 + (ch + 1) * GK, ra);
            ld_op(Bm, nullptr, g.ldb, n0, g.N, B_KM, false, k0 + (ch + 1) * GK, rb);
        }
        if (g.colsum && A_KM && tn == 0) {
            const int cc = tid & 127, kb = (tid >> 7) * (GK / 2);
#pragma unroll
            for (int k = 0; k < GK / 2; ++k) csum += As[bf][kb + k][cc];
        }
        {
            // k-step s + 1's operands read before k-step s's MFMAs (4 LDS reads,
            // then 4 MFMAs, enforced on the scheduler)
            float pa0, pa1, pb0, pb1, qa0, qa1, qb0, qb1;
#define GM_RD(s_, A0, A1, B0, B1)                                                                            \
    {                                                                                                        \
        const int kk_ = 2 * (s_) + kh;                                                                       \
        A0 = As[bf][kk_][wr + col];                                                                          \
        A1 = As[bf][kk_][wr + 32 + col];                                                                     \
        B0 = Bs[bf][kk_][wc + col];                                                                          \
        B1 = Bs[bf][kk_][wc + 32 + col];                                                                     \
    }
#define GM_MM(A0, A1, B0, B1)                                                                                \
    {                                                                                                        \
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(A0, B0, acc[0][0], 0, 0, 0);                        \
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(A0, B1, acc[0][1], 0, 0, 0);                        \
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(A1, B0, acc[1][0], 0, 0, 0);                        \
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(A1, B1, acc[1][1], 0, 0, 0);                        \
    }
            GM_RD(0, pa0, pa1, pb0, pb1)
#pragma unroll
            for (int s = 0; s < GK / 2; s += 2) {
                GM_RD(s + 1, qa0, qa1, qb0, qb1)
                GM_MM(pa0, pa1, pb0, pb1)
                if (s + 2 < GK / 2) GM_RD(s + 2, pa0, pa1, pb0, pb1)
                GM_MM(qa0, qa1, qb0, qb1)
            }
            __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
            for (int s = 0; s < GK / 2; ++s) {
                if (s + 1 < GK / 2) __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
                __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
            }
#undef GM_RD
#undef GM_MM
        }
        if (ch + 1 < nchunks) {
            st_op(As[bf ^ 1], A_KM, ra);
            st_op(Bs[bf ^ 1], B_KM, rb);
        }
        __syncthreads();
    }
    if (g.colsum && A_KM && tn == 0) {   // (block-uniform) one column tile per row block writes the sums
        // the two halves of each column: pairs of threads tid, tid + 128
        __shared__ float cs2[GT];
        if (tid >= 128) cs2[tid - 128] = csum;
        __syncthreads();
        if (tid < 128 && m0 + tid < g.M) g.colsum[((int64_t)split * gridDim.y + bt) * g.M + m0 + tid] = csum + cs2[tid];
    }
    // epilogue: acc[i][j] register v = C[wr + 32 i + 8 (v / 4) + 4 kh + v % 4][wc + 32 j + col]
    float *C = g.c + bt * g.sc;
    if (EPI == 3) C = g.c + ((int64_t)split * gridDim.y + bt) * (int64_t)g.M * g.N;
    const int64_t ldc = EPI == 3 ? g.N : g.ldc;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int n = n0 + wc + 32 * j + col;
        if (n >= g.N) continue;
        const float bv = (EPI == 1 || EPI == 2) ? g.bias[bt * g.sbias + n] : 0.0f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const int m = m0 + wr + 32 * i + 8 * (v >> 2) + 4 * kh + (v & 3);
                if (m >= g.M) continue;
                float r = acc[i][j][v];
                if (EPI == 1) r = tanhf(r + bv);
                else if (EPI == 2) r = r + bv;
                C[(int64_t)m * ldc + n] = r;
            }
    }
}

// out[i] = sum over splits of part[s][i] (+ out if accumulate), deterministic:
// a block owns 64 consecutive outputs; its 4 waves each sum one contiguous
// quarter of the splits in order (loads 8 deep), and the quarters are added in
// order through LDS -- so a tiny output over hundreds of splits (the heads'
// weight gradients) is not one thread's serial chain of loads.
__global__ __launch_bounds__(256) void gemm_reduce_kernel(const float *__restrict__ part, int splits, int64_t per,
                                                          float *__restrict__ out, int accumulate) {
    __shared__ float q[4][64];
    const int o = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t i = (int64_t)blockIdx.x * 64 + o;
    const int per_q = (splits + 3) / 4;
    const int k0 = w * per_q, k1 = min(splits, k0 + per_q);
    float s = 0.0f;
    if (i < per) {
        int k = k0;
        for (; k + 8 <= k1; k += 8) {
            float v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = part[(int64_t)(k + j) * per + i];
#pragma unroll
            for (int j = 0; j < 8; ++j) s += v[j];
        }
        for (; k < k1; ++k) s += part[(int64_t)k * per + i];
    }
    q[w][o] = s;
    __syncthreads();
    if (w == 0 && i < per) {
        const float r = ((q[0][o] + q[1][o]) + q[2][o]) + q[3][o];
        out[i] = accumulate ? out[i] + r : r;
    }
}

#ifndef VN_GEMM_ASM
#define VN_GEMM_ASM 1        // gemm_dl_kernel: raw barriers + asm fragment reads (the double buffering kept)
#endif
typedef float gm_f4 __attribute__((ext_vector_type(4)));
// the LDS offset of a __shared__ pointer (the low 32 bits of its flat address)
__device__ __forceinline__ uint32_t lds_addr(const void *p) { return (uint32_t)(uintptr_t)p; }
__device__ __forceinline__ gm_f4 lds_b128(uint32_t a) {
    gm_f4 r;
    asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(a) : "memory");
    return r;
}
__device__ __forceinline__ float lds_b32(uint32_t a) {
    float r;
    asm volatile("ds_read_b32 %0, %1" : "=v"(r) : "v"(a) : "memory");
    return r;
}

// ----------------------------------------------------------------------------
// Direct-load variant (the aligned shapes of the learner: K per split a
// multiple of GKD, 16-B aligned rows, 4-aligned k-major column counts).  Same
// 128 x 128 block tile and 2 x 2 32x32x2 accumulators per wave, but the
// operand chunks go global -> LDS with global_load_lds (16 B per lane, no
// register staging, no LDS store instructions, no per-chunk address
// arithmetic beyond one add), double-buffered.  LDS layouts (16-B units):
//   row-major operand  [row][GKD/4 units] with the unit index XOR-swizzled
//     by the row (u ^ (row / (16 / NU)) % NU), so a fragment read -- 32 rows,
//     one unit each, ds_read_b128 -- hits 16 distinct bank groups per 16 lanes;
//     one read carries 4 k-steps of the lane's row;
//   k-major operand    [k][32 units] with the unit XOR-swizzled by 8 on every
//     other group of 4 k (the two lane halves of a b32 read then hit disjoint
//     banks).
// The k order inside a chunk is permuted identically for both operands (lane
// half kh at k-step s takes k = 4 (kh + 2 (s / 4)) + s % 4), which is a
// reordering of the dot product's terms only.  With AGRAD the Y tile is
// staged beside dY and dZ = dY (1 - Y^2) is formed on the fragment read.
template <int GKD, bool A_KM, bool B_KM, bool AGRAD, int EPI>
__global__ __launch_bounds__(256, 2) void gemm_dl_kernel(GemmArgs g) {
    constexpr int NU = GKD / 4;              // units per row of a row-major chunk
    constexpr int UNITS = GT * NU;           // 16-B units per operand chunk
    constexpr int PER = UNITS / 256;         // units per thread per operand
    constexpr int RPB = 16 / NU;             // rows per 16-unit bank cycle
    __shared__ float4 sA[2][UNITS], sB[2][UNITS];
    __shared__ float4 sY[AGRAD ? 2 : 1][AGRAD ? UNITS : 1];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int ntn = (g.N + GT - 1) / GT;
    const int nblk = (int)(gridDim.x * gridDim.y * gridDim.z);
    int vb = (int)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z));
    if ((nblk & 7) == 0) vb = (vb & 7) * (nblk >> 3) + (vb >> 3);
    const int tiles = (int)gridDim.x;
    const int tm = (vb % tiles) / ntn, tn = (vb % tiles) - tm * ntn;
    const int bt = (vb / tiles) % (int)gridDim.y, split = vb / (tiles * (int)gridDim.y);
    const int m0 = tm * GT, n0 = tn * GT;
    const int k0 = split * g.kper;
    const int k1 = min(g.K, k0 + g.kper);
    const int nchunks = (k1 - k0) / GKD;
    const float *A = g.a + bt * g.sa;
    const float *Y = AGRAD ? g.a2 + bt * g.sa : nullptr;
    const float *Bm = g.b + bt * g.sb;

    // this thread's source offsets (floats, at chunk k = k0) for its PER units of each operand
    int64_t oa[PER], ob[PER];
    auto src_off = [&](bool km, int p, int base, int lim, int64_t ld) -> int64_t {
        if (km) {            // [k][cols]: p = k * 32 + swizzled unit
            const int k = p >> 5, u = (p & 31) ^ (8 * ((k >> 2) & 1));
            const int c = min(base + 4 * u, lim - 4);
            return (int64_t)(k0 + k) * ld + c;
        }
        const int r = p / NU, u = (p % NU) ^ ((r / RPB) % NU);
        const int rr = min(base + r, lim - 1);
        return (int64_t)rr * ld + k0 + 4 * u;
    };
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int p = (i * 4 + wv) * 64 + lane;
        oa[i] = src_off(A_KM, p, m0, g.M, g.lda);
        ob[i] = src_off(B_KM, p, n0, g.N, g.ldb);
    }
    const int64_t stepA = A_KM ? (int64_t)GKD * g.lda : GKD, stepB = B_KM ? (int64_t)GKD * g.ldb : GKD;
    auto issue = [&](int ch, int st) {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int w0 = (i * 4 + wv) * 64;
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)(A + oa[i] + ch * stepA),
                (__attribute__((address_space(3))) void *)&sA[st][w0], 16, 0, 0);
            if (AGRAD)
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)(Y + oa[i] + ch * stepA),
                    (__attribute__((address_space(3))) void *)&sY[st][w0], 16, 0, 0);
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)(Bm + ob[i] + ch * stepB),
                (__attribute__((address_space(3))) void *)&sB[st][w0], 16, 0, 0);
        }
    };

    f32x16_t acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = zero16();
    const int wr = 64 * (wv & 1), wc = 64 * (wv >> 1);
    const int col = lane & 31, kh = lane >> 5;
    // column sums of dZ (k-major A; the bias gradient of dW): waves with wc == 0
    // cover every A column of the tile once, each lane half its k's
    float csum[2] = {0.0f, 0.0f};
    const bool do_cs = g.colsum && A_KM && tn == 0 && wc == 0;

    if (nchunks > 0) issue(0, 0);
#if VN_GEMM_ASM
    // The chunk loop with raw barriers and the fragment reads in asm.  A
    // __syncthreads() is a workgroup-scope fence, and the compiler drains
    // vmcnt(0) before it -- and before any LDS read that may alias an LDS-DMA
    // load in flight -- so the next chunk's loads were waited for before this
    // chunk's MFMAs (no double buffering left).  Here the waits are explicit:
    // before the barrier that opens chunk ch, this wave's loads of chunk ch
    // landed (vmcnt leaves chunk ch + 1's in flight); the barrier then says
    // every wave's did; before the barrier that frees a stage for the next
    // chunk's loads, this wave's reads of it completed (lgkmcnt(0)).  The
    // reads are asm (invisible to the compiler's wait insertion), so each read
    // batch is waited for with lgkmcnt(0) and its registers tied after the wait.
    constexpr int OPS = AGRAD ? 3 : 2;           // LDS-DMA loads per unit of a chunk
    const uint32_t aA[2] = {lds_addr(sA[0]), lds_addr(sA[1])}, aB[2] = {lds_addr(sB[0]), lds_addr(sB[1])};
    const uint32_t aY[2] = {AGRAD ? lds_addr(sY[0]) : 0u, AGRAD ? lds_addr(sY[AGRAD ? 1 : 0]) : 0u};
    // byte offset of row-major unit (r, u) and of k-major value (c, s) in a stage
    auto rm_off = [&](int r, int u) -> uint32_t { return (uint32_t)(r * NU + (u ^ ((r / RPB) % NU))) * 16u; };
    auto km_off = [&](int c, int s) -> uint32_t {
        const int k = 4 * (kh + 2 * (s >> 2)) + (s & 3);
        return (uint32_t)((k * 32 + ((c >> 2) ^ (8 * kh))) * 4 + (c & 3)) * 4u;
    };
    struct PassRegs {
        gm_f4 ra[2], rb[2], ry[2];               // row-major fragments (A, B, and Y for AGRAD)
        float ka[2][4], kb[2][4], ky[2][4];      // k-major values
    };
    auto pass_read = [&](int st, int sq, PassRegs &R) {
#pragma unroll
        for (int f = 0; f < 2; ++f) {
            if (!A_KM) {
                const uint32_t o = rm_off(wr + 32 * f + col, kh + 2 * sq);
                R.ra[f] = lds_b128(aA[st] + o);
                if (AGRAD) R.ry[f] = lds_b128(aY[st] + o);
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint32_t o = km_off(wr + 32 * f + col, 4 * sq + e);
                    R.ka[f][e] = lds_b32(aA[st] + o);
                    if (AGRAD) R.ky[f][e] = lds_b32(aY[st] + o);
                }
            }
            if (!B_KM) {
                R.rb[f] = lds_b128(aB[st] + rm_off(wc + 32 * f + col, kh + 2 * sq));
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) R.kb[f][e] = lds_b32(aB[st] + km_off(wc + 32 * f + col, 4 * sq + e));
            }
        }
    };
    // after lgkmcnt(0): tie the registers, so no use moves above the wait
    auto pass_tie = [&](PassRegs &R) {
#pragma unroll
        for (int f = 0; f < 2; ++f) {
            if (!A_KM) {
                asm volatile("" : "+v"(R.ra[f]));
                if (AGRAD) asm volatile("" : "+v"(R.ry[f]));
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    asm volatile("" : "+v"(R.ka[f][e]));
                    if (AGRAD) asm volatile("" : "+v"(R.ky[f][e]));
                }
            }
            if (!B_KM) {
                asm volatile("" : "+v"(R.rb[f]));
            } else {
#pragma unroll
                for (int e = 0; e < 4; ++e) asm volatile("" : "+v"(R.kb[f][e]));
            }
        }
    };
    auto pass_mfma = [&](const PassRegs &R) {
        float av[2][4], bv[2][4];
#pragma unroll
        for (int f = 0; f < 2; ++f)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float v = A_KM ? R.ka[f][e] : R.ra[f][e];
                if (AGRAD) {
                    const float y = A_KM ? R.ky[f][e] : R.ry[f][e];
                    v = v * (1.0f - y * y);
                }
                av[f][e] = v;
                if (A_KM && do_cs) csum[f] += v;
                bv[f][e] = B_KM ? R.kb[f][e] : R.rb[f][e];
            }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[0][e], bv[0][e], acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[0][e], bv[1][e], acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[1][e], bv[0][e], acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[1][e], bv[1][e], acc[1][1], 0, 0, 0);
        }
    };
    for (int ch = 0; ch < nchunks; ++ch) {
        const int st = ch & 1;
        if (ch + 1 < nchunks) {
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // stage st ^ 1 (chunk ch - 1) read by every wave
            issue(ch + 1, st ^ 1);
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(OPS * PER) : "memory");  // this wave's chunk-ch loads landed
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        asm volatile("s_barrier" ::: "memory");                               // ... and every wave's
        // pass sq + 1's reads in flight during pass sq's MFMAs
        PassRegs rr[2];
        pass_read(st, 0, rr[0]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        pass_tie(rr[0]);
#pragma unroll
        for (int sq = 0; sq < GKD / 8; ++sq) {
            if (sq + 1 < GKD / 8) pass_read(st, sq + 1, rr[(sq + 1) & 1]);
            pass_mfma(rr[sq & 1]);
            if (sq + 1 < GKD / 8) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                pass_tie(rr[(sq + 1) & 1]);
            }
        }
    }
#else
    for (int ch = 0; ch < nchunks; ++ch) {
        const int st = ch & 1;
        if (ch + 1 < nchunks) {
            __syncthreads();               // every wave is done reading stage st ^ 1 (chunk ch - 1)
            issue(ch + 1, st ^ 1);
            if (AGRAD) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PER) : "memory");
            else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();                   // chunk ch is in LDS for every wave
        const float *fA = reinterpret_cast<const float *>(sA[st]);
        const float *fB = reinterpret_cast<const float *>(sB[st]);
        const float *fY = AGRAD ? reinterpret_cast<const float *>(sY[st]) : nullptr;
        // operand value of fragment f (rows / cols base + 32 f + col) at k-step s
        auto rm_unit = [&](const float4 *T, int r, int u) { return T[r * NU + (u ^ ((r / RPB) % NU))]; };
        auto km_val = [&](const float *T, int c, int s) {
            const int k = 4 * (kh + 2 * (s >> 2)) + (s & 3);
            return T[(k * 32 + ((c >> 2) ^ (8 * kh))) * 4 + (c & 3)];
        };
#pragma unroll
        for (int sq = 0; sq < GKD / 8; ++sq) {      // 4 k-steps per pass (one row-major unit)
            float av[2][4], bv[2][4];
#pragma unroll
            for (int f = 0; f < 2; ++f) {
                if (!A_KM) {
                    const int r = wr + 32 * f + col;
                    float4 v = rm_unit(sA[st], r, kh + 2 * sq);
                    if (AGRAD) {
                        const float4 y = rm_unit(sY[st], r, kh + 2 * sq);
                        v.x = v.x * (1.0f - y.x * y.x);
                        v.y = v.y * (1.0f - y.y * y.y);
                        v.z = v.z * (1.0f - y.z * y.z);
                        v.w = v.w * (1.0f - y.w * y.w);
                    }
                    av[f][0] = v.x; av[f][1] = v.y; av[f][2] = v.z; av[f][3] = v.w;
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        float v = km_val(fA, wr + 32 * f + col, 4 * sq + e);
                        if (AGRAD) {
                            const float y = km_val(fY, wr + 32 * f + col, 4 * sq + e);
                            v = v * (1.0f - y * y);
                        }
                        av[f][e] = v;
                        if (do_cs) csum[f] += v;
                    }
                }
                if (!B_KM) {
                    const float4 v = rm_unit(sB[st], wc + 32 * f + col, kh + 2 * sq);
                    bv[f][0] = v.x; bv[f][1] = v.y; bv[f][2] = v.z; bv[f][3] = v.w;
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e) bv[f][e] = km_val(fB, wc + 32 * f + col, 4 * sq + e);
                }
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[0][e], bv[0][e], acc[0][0], 0, 0, 0);
                acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[0][e], bv[1][e], acc[0][1], 0, 0, 0);
                acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[1][e], bv[0][e], acc[1][0], 0, 0, 0);
                acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[1][e], bv[1][e], acc[1][1], 0, 0, 0);
            }
        }
        (void)fA; (void)fB; (void)fY;
    }
#endif
    if (g.colsum && A_KM && tn == 0) {   // (block-uniform) lanes l, l ^ 32 hold the two k halves of column wr + 32 f + l % 32
        if (do_cs) {
#pragma unroll
            for (int f = 0; f < 2; ++f) {
                const float t = csum[f] + __shfl_xor(csum[f], 32, 64);
                const int m = m0 + wr + 32 * f + col;
                if (kh == 0 && m < g.M) g.colsum[((int64_t)split * gridDim.y + bt) * g.M + m] = t;
            }
        }
    }
    float *C = g.c + bt * g.sc;
    if (EPI == 3) C = g.c + ((int64_t)split * gridDim.y + bt) * (int64_t)g.M * g.N;
    const int64_t ldc = EPI == 3 ? g.N : g.ldc;
    const bool full = m0 + GT <= g.M && n0 + GT <= g.N;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int n = n0 + wc + 32 * j + col;
        if (!full && n >= g.N) continue;
        const float bv = (EPI == 1 || EPI == 2) ? g.bias[bt * g.sbias + n] : 0.0f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const int m = m0 + wr + 32 * i + 8 * (v >> 2) + 4 * kh + (v & 3);
                if (!full && m >= g.M) continue;
                float r = acc[i][j][v];
                if (EPI == 1) r = tanhf(r + bv);
                else if (EPI == 2) r = r + bv;
                C[(int64_t)m * ldc + n] = r;
            }
    }
}

template <bool A_KM, bool B_KM, bool AGRAD, int EPI>
void launch(const GemmArgs &g, int batch, int splits, hipStream_t s) {
    const int tiles = ((g.M + GT - 1) / GT) * ((g.N + GT - 1) / GT);
    const dim3 grid((unsigned)tiles, (unsigned)batch, (unsigned)splits);
    // the direct-load kernel takes 16-B aligned operands whose K per split is
    // a whole number of chunks (VN_GEMM_DL=0: the register-staged kernel, A/B knob)
    constexpr int GKD = 16;
    auto al = [](const void *p) { return ((uintptr_t)p & 15) == 0; };
    static const bool dl_on = [] {
        const char *e = getenv("VN_GEMM_DL");
        return !(e && e[0] == '0');
    }();
    // VN_GEMM_GKD=32: 32-deep chunks where K allows (A/B knob; half the barriers, twice the LDS)
    static const bool gk32 = [] {
        const char *e = getenv("VN_GEMM_GKD");
        return e && e[0] == '3';
    }();
    const bool dl = dl_on && g.K % GKD == 0 && g.kper % GKD == 0 && g.lda % 4 == 0 && g.ldb % 4 == 0 &&
                    g.sa % 4 == 0 && g.sb % 4 == 0 && al(g.a) && al(g.b) && (!AGRAD || al(g.a2)) &&
                    (!A_KM || g.M % 4 == 0) && (!B_KM || g.N % 4 == 0);
    if (dl && gk32 && g.K % 32 == 0 && g.kper % 32 == 0)
        hipLaunchKernelGGL((gemm_dl_kernel<32, A_KM, B_KM, AGRAD, EPI>), grid, dim3(256), 0, s, g);
    else if (dl)
        hipLaunchKernelGGL((gemm_dl_kernel<GKD, A_KM, B_KM, AGRAD, EPI>), grid, dim3(256), 0, s, g);
    else
        hipLaunchKernelGGL((gemm_f32_kernel<EPI == 3 ? GK_TN : GK_LIN, A_KM, B_KM, AGRAD, EPI>), grid, dim3(256), 0,
                           s, g);
}

}  // namespace

extern "C" {

// C = act(A_rm [M][K] @ B_rm[N][K]^T + bias): the forward Linear (+ Tanh).
//   act: 0 none (bias may be NULL), 1 tanh.  Batched over blockIdx.y with strides.
int vn_gemm_f32_linear(const float *a, int64_t lda, int64_t sa, const float *w, int64_t ldw, int64_t sw,
                       const float *bias, int64_t sbias, float *c, int64_t ldc, int64_t sc, int32_t M, int32_t N,
                       int32_t K, int32_t batch, int32_t act, void *stream) {
    if (!a || !w || !c) return fail(VN_ERR_INVALID, "NULL argument");
    if (M < 1 || N < 1 || K < 1 || batch < 1) return fail(VN_ERR_INVALID, "bad sizes M=%d N=%d K=%d", M, N, K);
    if (act == 1 && !bias) return fail(VN_ERR_INVALID, "tanh epilogue needs a bias");
    GemmArgs g{};
    g.a = a; g.b = w; g.bias = bias; g.c = c;
    g.lda = lda; g.ldb = ldw; g.ldc = ldc; g.sa = sa; g.sb = sw; g.sc = sc; g.sbias = sbias;
    g.M = M; g.N = N; g.K = K; g.kper = K;
    const hipStream_t s = (hipStream_t)stream;
    if (act == 1) launch<false, false, false, 1>(g, batch, 1, s);
    else if (bias) launch<false, false, false, 2>(g, batch, 1, s);
    else launch<false, false, false, 0>(g, batch, 1, s);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

// C = dZ [M][K] @ W [K][N], dZ = dy (1 - y^2) when y != NULL (the Tanh
// backward fused into the load), else dZ = dy.  Batched.
int vn_gemm_f32_dx(const float *dy, const float *y, int64_t ldd, int64_t sd, const float *w, int64_t ldw, int64_t sw,
                   float *c, int64_t ldc, int64_t sc, int32_t M, int32_t N, int32_t K, int32_t batch, void *stream) {
    if (!dy || !w || !c) return fail(VN_ERR_INVALID, "NULL argument");
    if (M < 1 || N < 1 || K < 1 || batch < 1) return fail(VN_ERR_INVALID, "bad sizes M=%d N=%d K=%d", M, N, K);
    GemmArgs g{};
    g.a = dy; g.a2 = y; g.b = w; g.c = c;
    g.lda = ldd; g.ldb = ldw; g.ldc = ldc; g.sa = sd; g.sb = sw; g.sc = sc;
    g.M = M; g.N = N; g.K = K; g.kper = K;
    const hipStream_t s = (hipStream_t)stream;
    if (y) launch<false, true, true, 0>(g, batch, 1, s);
    else launch<false, true, false, 0>(g, batch, 1, s);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

// Weight gradient over a tall sample axis: C [M][N] = A^T B, A = dZ [K][M]
// (k-major; dZ = dy (1 - y^2) when y != NULL), B [K][N] k-major; the K axis is
// split into `splits` parts whose partials (workspace: splits * batch * M * N
// floats) are summed in order; colsum [batch][M] (optional) receives sum_k
// dZ[k][m] (workspace2: splits * batch * M floats).  accumulate: C += result.
int vn_gemm_f32_tn(const float *dy, const float *y, int64_t ldd, int64_t sd, const float *b, int64_t ldb, int64_t sb,
                   float *c, int64_t sc, float *colsum, int32_t M, int32_t N, int32_t K, int32_t batch, int32_t splits,
                   float *workspace, float *workspace2, int32_t accumulate, void *stream) {
    if (!dy || !b || !c || !workspace) return fail(VN_ERR_INVALID, "NULL argument");
    if (colsum && !workspace2) return fail(VN_ERR_INVALID, "colsum needs workspace2");
    if (M < 1 || N < 1 || K < 1 || batch < 1 || splits < 1) return fail(VN_ERR_INVALID, "bad sizes");
    if (sc != (int64_t)M * N) return fail(VN_ERR_INVALID, "C must be contiguous [batch][M][N]");
    int kper = (K + splits - 1) / splits;
    kper = (kper + GK_TN - 1) / GK_TN * GK_TN;
    splits = (K + kper - 1) / kper;
    GemmArgs g{};
    g.a = dy; g.a2 = y; g.b = b; g.c = workspace; g.colsum = colsum ? workspace2 : nullptr;
    g.lda = ldd; g.ldb = ldb; g.ldc = N; g.sa = sd; g.sb = sb; g.sc = 0;
    g.M = M; g.N = N; g.K = K; g.kper = kper;
    const hipStream_t s = (hipStream_t)stream;
    if (y) launch<true, true, true, 3>(g, batch, splits, s);
    else launch<true, true, false, 3>(g, batch, splits, s);
    const int64_t per = (int64_t)batch * M * N;
    hipLaunchKernelGGL(gemm_reduce_kernel, dim3((unsigned)((per + 63) / 64)), dim3(256), 0, s, workspace, splits,
                       per, c, accumulate);
    if (colsum) {
        const int64_t pc = (int64_t)batch * M;
        hipLaunchKernelGGL(gemm_reduce_kernel, dim3((unsigned)((pc + 63) / 64)), dim3(256), 0, s, workspace2,
                           splits, pc, colsum, accumulate);
    }
    VN_HIP(hipGetLastError());
    return VN_OK;
}

}  // extern "C"
