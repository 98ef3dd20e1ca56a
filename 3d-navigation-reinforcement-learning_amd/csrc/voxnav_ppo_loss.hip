// voxnav_ppo_loss.hip -- the PPO learner's per-minibatch kernels around the
// matrix products (f32, the reference's dtype): the loss and its gradient down
// to the MLP latents in three launches, the gradient norm of the clip, the Adam
// step, and the feed-forward minibatch gather (each below its own header).
//
// Restates, per minibatch, what sb3 RecurrentPPO.train / PPO.train run after
// the MLP extractor (train/Grid_Train.py:228 -> model.learn; SURVEY.md App.
// D.3/D.4): the heads (action_net Linear -> Categorical, value_net Linear),
// the advantage normalisation, the clipped surrogate, the value MSE and the
// entropy bonus, and -- instead of autograd -- their gradient written
// directly:
//   z = h_pi Wa^T + ba,  lp_all = log_softmax(z),  v = h_vf wv + bv
//   H = -sum p lp_all,   ratio = exp(lp_all[a] - old_lp)
//   loss = -mean(min(A r, A clamp(r, 1-c, 1+c))) - ent_coef mean(H)
//          + vf_coef mean((ret - v)^2)
//   dz_j = g_lp (d_ja - p_j) + (ent_coef / n) p_j (lp_j + H)
//   g_lp = -(1/n) A r (m1 + m2 [1-c <= r <= 1+c])      (torch's min / clamp
//          backward: the smaller branch, a tie split in halves)
//   dv   = vf_coef 2 (v - ret) / n
//   dh_pi = dz Wa, dh_vf = dv wv, dWa = dz^T h_pi, dba = sum dz, dwv, dbv
// with A = (adv - mean) / (std + 1e-8) over the minibatch (unbiased std).
//
// Launches: (1) 64 blocks: f64 sums of the minibatch's advantages and their
// squares (each loss block folds the 64 pairs, in order, into mean / std);
// (2) the samples, one wave per SPW samples, 16 lanes per sample across the
// latent features (a float4 each; coalesced row loads and stores), the head
// dot products reduced over the 16 lanes by xor butterflies (every lane ends
// with the same bits, so the per-sample scalar work runs redundantly without
// a broadcast); per-block partials of the head-weight gradients (f32) and of the
// logged sums (f64); (3) the partials summed in a fixed order (results do not
// depend on scheduling).
//
// HBM per sample: the two latent rows read (2 F 4 B) and their gradient rows
// written (2 F 4 B) + 16 B of gathered buffer scalars + the 8 B row index.

#include <hip/hip_runtime.h>

#include <cstdint>

#include "vn_common.h"

using vn_detail::fail;

namespace {

constexpr int kSPW = 32;       // samples per wave
constexpr int kPass = 1;       // 4-sample passes whose loads are issued together
constexpr int kWaves = 4;      // waves per block
constexpr int kMaxA = 8;       // actions
constexpr int kAdvBlocks = 64; // blocks of the advantage sums
constexpr int kStats = 5;      // per-block f64 sums: min-surrogate, squared value error, entropy, kl, clipped

struct LossArgs {
    const float *hp, *hv;       // latents [M][F] (row stride ldh)
    int64_t ldh;
    const float *wa, *ba, *wv, *bv;   // action_net [A][F], [A]; value_net [F], [1]
    const int64_t *src;         // [M] rows of the buffers (NULL: identity)
    const int32_t *act;
    const float *adv, *old_lp, *ret;
    const double *asum;         // [kAdvBlocks][2] advantage sums
    int normalize;
    float *dhp, *dhv;           // [M][F] contiguous
    float *part;                // [blocks][PG]
    double *spart;              // [blocks][kStats]
    int M, F, A;
    float clip, ent_coef, vf_coef;
};

// per-block f64 sums of the minibatch's advantages and their squares
// (kAdvBlocks blocks, a contiguous range each); every loss block adds the
// kAdvBlocks pairs in the same order
__global__ __launch_bounds__(256) void adv_sum_kernel(const float *__restrict__ adv, const int64_t *__restrict__ src,
                                                      int M, double *__restrict__ asum) {
    __shared__ double s1[256], s2[256];
    const int t = threadIdx.x;
    const int per = (M + kAdvBlocks - 1) / kAdvBlocks;
    const int i0 = blockIdx.x * per, i1 = min(M, i0 + per);
    double a1 = 0.0, a2 = 0.0;
    for (int i = i0 + t; i < i1; i += 256) {
        const double a = adv[src ? src[i] : i];
        a1 += a;
        a2 += a * a;
    }
    s1[t] = a1;
    s2[t] = a2;
    __syncthreads();
    for (int h = 128; h >= 1; h >>= 1) {
        if (t < h) {
            s1[t] += s1[t + h];
            s2[t] += s2[t + h];
        }
        __syncthreads();
    }
    if (t == 0) {
        asum[2 * blockIdx.x] = s1[0];
        asum[2 * blockIdx.x + 1] = s2[0];
    }
}

// Q = F / 64: lane l of a 16-lane group holds latent features
// 64 q + 4 (l & 15) .. +3 (q < Q) -- one float4 per q, 256 B contiguous per
// group; the wave's 4 groups take 4 samples at once.  AM: A rounded up to
// even (the per-action registers); the action weights are read from LDS.
template <int Q, int AM>
__global__ __launch_bounds__(256) void ppo_loss_kernel(LossArgs g) {
    extern __shared__ float red[];            // [kWaves][PG], then action weights [AM][F]
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int grp = lane >> 4, gl = lane & 15;
    const int F = g.F, A = g.A, PG = A * F + A + F + 1;
    const float inv_n = 1.0f / (float)g.M;
    float *wsh = red + kWaves * PG;
    for (int i = threadIdx.x; i < AM * F; i += 256) wsh[i] = i < A * F ? g.wa[i] : 0.0f;
    auto wa = [&](int a, int q) { return *reinterpret_cast<const float4 *>(wsh + a * F + 64 * q + 4 * gl); };
    float4 wvv[Q];
    float ba[AM];
#pragma unroll
    for (int a = 0; a < AM; ++a) ba[a] = a < A ? g.ba[a] : 0.0f;
#pragma unroll
    for (int q = 0; q < Q; ++q) wvv[q] = *reinterpret_cast<const float4 *>(g.wv + 64 * q + 4 * gl);
    const float bv = g.bv[0];
    // the advantage mean and std + 1e-8 (unbiased std; NaN for one sample, as torch)
    __shared__ float adv_ms[2];
    if (threadIdx.x == 0) {
        float mf = 0.0f, df = 1.0f;
        if (g.normalize) {
            double a1 = 0.0, a2 = 0.0;
            for (int b = 0; b < kAdvBlocks; ++b) {
                a1 += g.asum[2 * b];
                a2 += g.asum[2 * b + 1];
            }
            const double n = g.M, mean = a1 / n;
            const double var = g.M > 1 ? fmax(0.0, a2 - a1 * mean) / (n - 1.0) : __builtin_nan("");
            mf = (float)mean;
            df = (float)sqrt(var) + 1e-8f;
        }
        adv_ms[0] = mf;
        adv_ms[1] = df;
    }
    __syncthreads();
    const float mean = adv_ms[0], den = adv_ms[1];

    float4 gwa[AM][Q], gwv[Q];
    float gba[AM], gbv = 0.0f;
#pragma unroll
    for (int a = 0; a < AM; ++a) {
        gba[a] = 0.0f;
#pragma unroll
        for (int q = 0; q < Q; ++q) gwa[a][q] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) gwv[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    double st[kStats] = {0.0, 0.0, 0.0, 0.0, 0.0};

    auto dot4 = [](float4 x, float4 y) { return x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w; };
    auto fma4 = [](float4 &acc, float s, float4 x) {
        acc.x += s * x.x;
        acc.y += s * x.y;
        acc.z += s * x.z;
        acc.w += s * x.w;
    };
    // sum over the 16 lanes of a group; every lane of the group ends with the same bits
    auto gsum = [](float v) {
#pragma unroll
        for (int off = 8; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
        return v;
    };

    const int s0 = (blockIdx.x * kWaves + wv) * kSPW;
    const int ns = max(0, min(kSPW, g.M - s0));
    for (int j0 = 0; j0 < ns; j0 += 4 * kPass) {
        // kPass passes of 4 samples (one per group), their loads issued first
        float4 hp[kPass][Q], hv[kPass][Q];
        int64_t rsrc[kPass];
        bool ok[kPass];
#pragma unroll
        for (int u = 0; u < kPass; ++u) {
            const int j = j0 + 4 * u + grp;
            ok[u] = j < ns;
            const int64_t row = (int64_t)(s0 + (ok[u] ? j : 0));
            rsrc[u] = g.src ? g.src[row] : row;
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                hp[u][q] = *reinterpret_cast<const float4 *>(g.hp + row * g.ldh + 64 * q + 4 * gl);
                hv[u][q] = *reinterpret_cast<const float4 *>(g.hv + row * g.ldh + 64 * q + 4 * gl);
            }
        }
#pragma unroll
        for (int u = 0; u < kPass; ++u) {
            // keep the LDS weight reads inside the loop (hoisted, they would hold
            // A Q float4 registers for the whole kernel)
            asm volatile("" ::: "memory");
            const int64_t r = rsrc[u];
            const int act = g.act[r];
            const float adv = (g.adv[r] - mean) / den, olp = g.old_lp[r], ret = g.ret[r];
            float z[AM];
#pragma unroll
            for (int a = 0; a < AM; ++a) {
                float sacc = 0.0f;
#pragma unroll
                for (int q = 0; q < Q; ++q) sacc += dot4(hp[u][q], wa(a, q));
                z[a] = a < A ? gsum(sacc) + ba[a] : -INFINITY;
            }
            float sv = 0.0f;
#pragma unroll
            for (int q = 0; q < Q; ++q) sv += dot4(hv[u][q], wvv[q]);
            const float v = gsum(sv) + bv;
            // log_softmax, entropy (uniform over the group)
            float zmax = z[0];
#pragma unroll
            for (int a = 1; a < AM; ++a) zmax = fmaxf(zmax, z[a]);
            float se = 0.0f;
#pragma unroll
            for (int a = 0; a < AM; ++a) se += a < A ? expf(z[a] - zmax) : 0.0f;
            const float lse = logf(se);
            float lpa[AM], p[AM], ent = 0.0f;
#pragma unroll
            for (int a = 0; a < AM; ++a) {
                lpa[a] = z[a] - zmax - lse;
                p[a] = a < A ? expf(lpa[a]) : 0.0f;
                ent -= a < A ? p[a] * lpa[a] : 0.0f;
            }
            float lp = 0.0f;
#pragma unroll
            for (int a = 0; a < AM; ++a) lp = a == act ? lpa[a] : lp;
            const float lr = lp - olp;
            const float ratio = expf(lr);
            const float rc = fminf(fmaxf(ratio, 1.0f - g.clip), 1.0f + g.clip);
            const float l1 = adv * ratio, l2 = adv * rc;
            const float m1 = l1 < l2 ? 1.0f : (l1 > l2 ? 0.0f : 0.5f);
            const float inr = (ratio >= 1.0f - g.clip && ratio <= 1.0f + g.clip) ? 1.0f : 0.0f;
            const float w = ok[u] ? 1.0f : 0.0f;     // a padding pass contributes nothing
            const float glp = -inv_n * adv * ratio * (m1 + (1.0f - m1) * inr) * w;
            const float gent = g.ent_coef * inv_n * w;
            const float dv = g.vf_coef * 2.0f * (v - ret) * inv_n * w;
            float4 dh[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) dh[q] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int a = 0; a < AM; ++a) {
                if (a >= A) break;
                const float dz = glp * ((a == act ? 1.0f : 0.0f) - p[a]) + gent * p[a] * (lpa[a] + ent);
                gba[a] += dz;
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    fma4(dh[q], dz, wa(a, q));
                    fma4(gwa[a][q], dz, hp[u][q]);
                }
            }
            gbv += dv;
            if (ok[u]) {
                const int64_t row = (int64_t)(s0 + j0 + 4 * u + grp) * F;
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    *reinterpret_cast<float4 *>(g.dhp + row + 64 * q + 4 * gl) = dh[q];
                    *reinterpret_cast<float4 *>(g.dhv + row + 64 * q + 4 * gl) =
                        make_float4(dv * wvv[q].x, dv * wvv[q].y, dv * wvv[q].z, dv * wvv[q].w);
                }
                if (gl == 0) {
                    st[0] += (double)fminf(l1, l2);
                    st[1] += (double)((ret - v) * (ret - v));
                    st[2] += (double)ent;
                    st[3] += (double)((ratio - 1.0f) - lr);
                    st[4] += fabsf(ratio - 1.0f) > g.clip ? 1.0 : 0.0;
                }
            }
#pragma unroll
            for (int q = 0; q < Q; ++q) fma4(gwv[q], dv, hv[u][q]);
        }
    }
    // the 4 groups' sums (lanes l, l ^ 16, l ^ 32, l ^ 48), then the waves in order
    auto xsum = [](float v) {
        v += __shfl_xor(v, 16, 64);
        return v + __shfl_xor(v, 32, 64);
    };
    float *my = red + wv * PG;
#pragma unroll
    for (int a = 0; a < AM; ++a) {
        if (a >= A) break;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const float4 t = make_float4(xsum(gwa[a][q].x), xsum(gwa[a][q].y), xsum(gwa[a][q].z), xsum(gwa[a][q].w));
            if (grp == 0) *reinterpret_cast<float4 *>(my + a * F + 64 * q + 4 * gl) = t;
        }
        // bias sums: every lane of a group holds its group's sum; one lane per group adds in
        const float b = gba[a];
        const float bs = __shfl(b, 0, 64) + __shfl(b, 16, 64) + __shfl(b, 32, 64) + __shfl(b, 48, 64);
        if (lane == 0) my[A * F + a] = bs;
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const float4 t = make_float4(xsum(gwv[q].x), xsum(gwv[q].y), xsum(gwv[q].z), xsum(gwv[q].w));
        if (grp == 0) *reinterpret_cast<float4 *>(my + A * F + A + 64 * q + 4 * gl) = t;
    }
    {
        const float bs = __shfl(gbv, 0, 64) + __shfl(gbv, 16, 64) + __shfl(gbv, 32, 64) + __shfl(gbv, 48, 64);
        if (lane == 0) my[PG - 1] = bs;
    }
    __shared__ double sred[kWaves][kStats];
#pragma unroll
    for (int k = 0; k < kStats; ++k) {
        const double v0 = __shfl(st[k], 0, 64), v1 = __shfl(st[k], 16, 64), v2 = __shfl(st[k], 32, 64),
                     v3 = __shfl(st[k], 48, 64);
        if (lane == 0) sred[wv][k] = ((v0 + v1) + v2) + v3;
    }
    __syncthreads();
    float *out = g.part + (int64_t)blockIdx.x * PG;
    for (int i = threadIdx.x; i < PG; i += 256)
        out[i] = ((red[i] + red[PG + i]) + red[2 * PG + i]) + red[3 * PG + i];
    if (threadIdx.x < kStats)
        g.spart[(int64_t)blockIdx.x * kStats + threadIdx.x] =
            ((sred[0][threadIdx.x] + sred[1][threadIdx.x]) + sred[2][threadIdx.x]) + sred[3][threadIdx.x];
}

// gout[i] = sum_b part[b][i] (blocks 0 .. nred-1, 64 outputs each, the 4 waves
// summing quarters of the block range in order); the last block sums the f64
// logged values and writes stats [6] = policy loss, value loss, entropy
// loss, loss, approx kl, clip fraction.
__global__ __launch_bounds__(256) void ppo_loss_reduce_kernel(const float *__restrict__ part, const double *__restrict__ spart,
                                                              int nb, int PG, int M, float ent_coef, float vf_coef,
                                                              float *__restrict__ gout, double *__restrict__ stats) {
    const int t = threadIdx.x;
    if (blockIdx.x + 1 == gridDim.x) {
        __shared__ double sr[256];
        double v[kStats];
        for (int k = 0; k < kStats; ++k) {
            double s = 0.0;
            for (int b = t; b < nb; b += 256) s += spart[(int64_t)b * kStats + k];
            sr[t] = s;
            __syncthreads();
            for (int h = 128; h >= 1; h >>= 1) {
                if (t < h) sr[t] += sr[t + h];
                __syncthreads();
            }
            v[k] = sr[0];
            __syncthreads();
        }
        if (t == 0) {
            const double n = M;
            const double pl = -v[0] / n, vl = v[1] / n, el = -v[2] / n;
            stats[0] = pl;
            stats[1] = vl;
            stats[2] = el;
            stats[3] = pl + (double)ent_coef * el + (double)vf_coef * vl;
            stats[4] = v[3] / n;
            stats[5] = v[4] / n;
        }
        return;
    }
    __shared__ float q[4][64];
    const int o = t & 63, w = t >> 6;
    const int i = blockIdx.x * 64 + o;
    const int per_q = (nb + 3) / 4, b0 = w * per_q, b1 = min(nb, b0 + per_q);
    float s = 0.0f;
    if (i < PG) {
        int b = b0;
        for (; b + 8 <= b1; b += 8) {
            float x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) x[u] = part[(int64_t)(b + u) * PG + i];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += x[u];
        }
        for (; b < b1; ++b) s += part[(int64_t)b * PG + i];
    }
    q[w][o] = s;
    __syncthreads();
    if (w == 0 && i < PG) gout[i] = ((q[0][o] + q[1][o]) + q[2][o]) + q[3][o];
}


// ---- gradient clipping (torch.nn.utils.clip_grad_norm_, sb3 max_grad_norm) ----
// The total 2-norm over every parameter gradient (f64 sums: per-block
// partials over all tensors, then one block in a fixed order) and the
// divisor the fused Adam step applies to the gradients (its grad_scale):
// max(1, (norm + 1e-6) / max_norm) = 1 / clip_grad_norm_'s clamped coefficient.
constexpr int kMaxGradTensors = 64;
constexpr int kNormBlocks = 256;

struct GradList {
    const float *p[kMaxGradTensors];
    int64_t n[kMaxGradTensors];
    int count;
};

__global__ __launch_bounds__(256) void grad_sq_kernel(GradList gl, double *__restrict__ part) {
    __shared__ double sr[256];
    const int t = threadIdx.x;
    double acc = 0.0;
    for (int k = 0; k < gl.count; ++k) {
        const float *g = gl.p[k];
        const int64_t n = gl.n[k];
        const int64_t n4 = ((((uintptr_t)g) & 15) == 0) ? n / 4 : 0;
        for (int64_t i = (int64_t)blockIdx.x * 256 + t; i < n4; i += (int64_t)gridDim.x * 256) {
            const float4 v = reinterpret_cast<const float4 *>(g)[i];
            acc += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
        }
        for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * 256 + t; i < n; i += (int64_t)gridDim.x * 256)
            acc += (double)g[i] * g[i];
    }
    sr[t] = acc;
    __syncthreads();
    for (int h = 128; h >= 1; h >>= 1) {
        if (t < h) sr[t] += sr[t + h];
        __syncthreads();
    }
    if (t == 0) part[blockIdx.x] = sr[0];
}

__global__ __launch_bounds__(256) void grad_norm_kernel(const double *__restrict__ part, float max_norm,
                                                        float *__restrict__ norm, float *__restrict__ scale) {
    __shared__ double sr[256];
    const int t = threadIdx.x;
    sr[t] = part[t];
    __syncthreads();
    for (int h = 128; h >= 1; h >>= 1) {
        if (t < h) sr[t] += sr[t + h];
        __syncthreads();
    }
    if (t == 0) {
        const float nv = (float)sqrt(sr[0]);
        norm[0] = nv;
        scale[0] = fmaxf(1.0f, (nv + 1e-6f) / max_norm);
    }
}

// ---- Adam step (torch.optim.Adam, the update sb3's policy optimizer runs) ----
// One launch over every parameter (pointers by value): with the clip divisor
// s (vn_grad_norm; 1 when NULL) and the step's bias corrections from the host,
// per element, in torch's fused-Adam order:
//   g = grad / s;  m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g g
//   p -= (lr / bc1) m / (sqrt(v) / sqrt(bc2) + eps)
// The gradients are read, not rewritten (the learner drops them after the step).
struct AdamList {
    float *p[kMaxGradTensors];
    const float *g[kMaxGradTensors];
    float *m[kMaxGradTensors];
    float *v[kMaxGradTensors];
    float *step[kMaxGradTensors];   // torch's per-parameter step counters (device f32 scalars)
    int64_t n[kMaxGradTensors];
    int count;
};

__global__ __launch_bounds__(256) void adam_kernel(AdamList al, const float *__restrict__ scale,
                                                   const int32_t *__restrict__ skip, float lr, float b1, float b2,
                                                   float eps, float bc1, float bc2_sqrt, float step_value) {
    if (skip && skip[0] != 0) return;   // gradients from a failed launch: leave every tensor as it was
    const bool div = scale != nullptr;
    const float s = scale ? scale[0] : 1.0f;
    const float step_size = lr / bc1;
    const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x, stride = (int64_t)gridDim.x * 256;
    if (gid < al.count && al.step[gid]) al.step[gid][0] = step_value;
    auto upd = [&](float &pp, float g, float &mm, float &vv) {
        if (div) g = g / s;
        mm = b1 * mm + (1.0f - b1) * g;
        vv = b2 * vv + (1.0f - b2) * g * g;
        const float denom = sqrtf(vv) / bc2_sqrt + eps;
        pp = pp - step_size * (mm / denom);
    };
    for (int k = 0; k < al.count; ++k) {
        const int64_t n = al.n[k];
        float *P = al.p[k], *M = al.m[k], *V = al.v[k];
        const float *G = al.g[k];
        const bool vec = ((((uintptr_t)P) | ((uintptr_t)G) | ((uintptr_t)M) | ((uintptr_t)V)) & 15) == 0;
        const int64_t n4 = vec ? n / 4 : 0;
        for (int64_t i = gid; i < n4; i += stride) {
            float4 pp = reinterpret_cast<float4 *>(P)[i], mm = reinterpret_cast<float4 *>(M)[i],
                   vv = reinterpret_cast<float4 *>(V)[i];
            const float4 gg = reinterpret_cast<const float4 *>(G)[i];
            upd(pp.x, gg.x, mm.x, vv.x);
            upd(pp.y, gg.y, mm.y, vv.y);
            upd(pp.z, gg.z, mm.z, vv.z);
            upd(pp.w, gg.w, mm.w, vv.w);
            reinterpret_cast<float4 *>(P)[i] = pp;
            reinterpret_cast<float4 *>(M)[i] = mm;
            reinterpret_cast<float4 *>(V)[i] = vv;
        }
        for (int64_t i = 4 * n4 + gid; i < n; i += stride) upd(P[i], G[i], M[i], V[i]);
    }
}

// ---- minibatch gather (PPO.train: rollout_buffer.get(batch_size) on the
// swap_and_flatten'ed, env-major buffer) ----
// sample i of the minibatch is env-major flat id idx[i] = env * T + t; its row
// in the collector's [T, N]-major buffers is t * N + env.  One block per 16
// samples: the rows (src) and the observation rows copied, 16 B per lane.
__global__ __launch_bounds__(256) void minibatch_rows_kernel(const int64_t *__restrict__ idx, int M, int T, int N,
                                                             const float *__restrict__ obs, int D,
                                                             float *__restrict__ out, int64_t *__restrict__ src) {
    const int lane = threadIdx.x & 15, s = blockIdx.x * 16 + (threadIdx.x >> 4);
    if (s >= M) return;
    const int64_t id = idx[s];
    const int64_t env = id / T, t = id - env * T;
    const int64_t r = t * N + env;
    if (lane == 0) src[s] = r;
    const float4 *in = reinterpret_cast<const float4 *>(obs + r * D);
    float4 *o = reinterpret_cast<float4 *>(out + (int64_t)s * D);
    for (int c = lane; c < D / 4; c += 16) o[c] = in[c];
}
}  // namespace

extern "C" {

int vn_ppo_loss_part_floats(int32_t M, int32_t F, int32_t A, int64_t *n_part, int64_t *n_spart) {
    if (M < 1 || F < 1 || A < 1) return fail(VN_ERR_INVALID, "bad sizes M=%d F=%d A=%d", M, F, A);
    const int64_t nb = (M + kWaves * kSPW - 1) / (kWaves * kSPW);
    if (n_part) *n_part = nb * ((int64_t)A * F + A + F + 1);
    if (n_spart) *n_spart = nb * kStats + 2 * kAdvBlocks;   // + the advantage sums
    return VN_OK;
}

int vn_ppo_loss(const float *hp, const float *hv, int64_t ldh, const float *wa, const float *ba, const float *wv,
                const float *bv, const int64_t *src, const int32_t *actions, const float *advantages,
                const float *old_log_prob, const float *returns, int32_t M, int32_t F, int32_t A, float clip_range,
                float ent_coef, float vf_coef, int32_t normalize_advantage, float *dhp, float *dhv, float *grad_heads,
                double *stats, double *adv_sums, float *part, double *spart, void *stream) {
    if (!hp || !hv || !wa || !ba || !wv || !bv || !actions || !advantages || !old_log_prob || !returns || !dhp ||
        !dhv || !grad_heads || !stats || !adv_sums || !part || !spart)
        return fail(VN_ERR_INVALID, "NULL argument");
    if (M < 1 || A < 1 || A > kMaxA) return fail(VN_ERR_INVALID, "bad sizes M=%d A=%d (A <= %d)", M, A, kMaxA);
    if (F < 64 || F > 256 || F % 64) return fail(VN_ERR_INVALID, "latent width F=%d: a multiple of 64 up to 256", F);
    if (ldh < F) return fail(VN_ERR_INVALID, "latent row stride %lld < F", (long long)ldh);
    const hipStream_t s = (hipStream_t)stream;
    if (normalize_advantage)
        hipLaunchKernelGGL(adv_sum_kernel, dim3(kAdvBlocks), dim3(256), 0, s, advantages, src, M, adv_sums);
    LossArgs g{};
    g.hp = hp; g.hv = hv; g.ldh = ldh; g.wa = wa; g.ba = ba; g.wv = wv; g.bv = bv;
    g.src = src; g.act = actions; g.adv = advantages; g.old_lp = old_log_prob; g.ret = returns;
    g.asum = adv_sums; g.normalize = normalize_advantage; g.dhp = dhp; g.dhv = dhv; g.part = part; g.spart = spart;
    g.M = M; g.F = F; g.A = A; g.clip = clip_range; g.ent_coef = ent_coef; g.vf_coef = vf_coef;
    const int nb = (M + kWaves * kSPW - 1) / (kWaves * kSPW);
    const int PG = A * F + A + F + 1;
    const int AM = (A + 1) / 2 * 2;
    const size_t lds = ((size_t)kWaves * PG + (size_t)AM * F) * sizeof(float);
#define VN_LOSS_Q(Q_)                                                                                   \
    switch (AM) {                                                                                       \
        case 2: hipLaunchKernelGGL((ppo_loss_kernel<Q_, 2>), dim3(nb), dim3(256), lds, s, g); break;    \
        case 4: hipLaunchKernelGGL((ppo_loss_kernel<Q_, 4>), dim3(nb), dim3(256), lds, s, g); break;    \
        case 6: hipLaunchKernelGGL((ppo_loss_kernel<Q_, 6>), dim3(nb), dim3(256), lds, s, g); break;    \
        default: hipLaunchKernelGGL((ppo_loss_kernel<Q_, 8>), dim3(nb), dim3(256), lds, s, g); break;   \
    }
    switch (F / 64) {
        case 1: VN_LOSS_Q(1) break;
        case 2: VN_LOSS_Q(2) break;
        case 3: VN_LOSS_Q(3) break;
        default: VN_LOSS_Q(4) break;
    }
#undef VN_LOSS_Q
    hipLaunchKernelGGL(ppo_loss_reduce_kernel, dim3((unsigned)((PG + 63) / 64 + 1)), dim3(256), 0, s, part, spart, nb,
                       PG, M, ent_coef, vf_coef, grad_heads, stats);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

int vn_grad_norm(const float *const *grads, const int64_t *sizes, int32_t count, float max_norm, float *norm,
                 float *scale, double *work, void *stream) {
    if (!grads || !sizes || !norm || !scale || !work) return fail(VN_ERR_INVALID, "NULL argument");
    if (count < 1 || count > kMaxGradTensors)
        return fail(VN_ERR_INVALID, "gradient count %d outside 1..%d", count, kMaxGradTensors);
    if (!(max_norm > 0.0f)) return fail(VN_ERR_INVALID, "max_norm must be > 0");
    GradList gl{};
    gl.count = count;
    for (int k = 0; k < count; ++k) {
        if (!grads[k] || sizes[k] < 0) return fail(VN_ERR_INVALID, "gradient %d: NULL or negative size", k);
        gl.p[k] = grads[k];
        gl.n[k] = sizes[k];
    }
    const hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(grad_sq_kernel, dim3(kNormBlocks), dim3(256), 0, s, gl, work);
    hipLaunchKernelGGL(grad_norm_kernel, dim3(1), dim3(256), 0, s, work, max_norm, norm, scale);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

int vn_adam_step(float *const *params, const float *const *grads, float *const *exp_avg, float *const *exp_avg_sq,
                 float *const *steps, const int64_t *sizes, int32_t count, const float *clip_scale,
                 const int32_t *skip, float lr, float beta1, float beta2, float eps, int64_t step, void *stream) {
    if (!params || !grads || !exp_avg || !exp_avg_sq || !sizes) return fail(VN_ERR_INVALID, "NULL argument");
    if (count < 1 || count > kMaxGradTensors)
        return fail(VN_ERR_INVALID, "parameter count %d outside 1..%d", count, kMaxGradTensors);
    if (step < 1) return fail(VN_ERR_INVALID, "step must be >= 1");
    AdamList al{};
    al.count = count;
    int64_t total = 0;
    for (int k = 0; k < count; ++k) {
        if (!params[k] || !grads[k] || !exp_avg[k] || !exp_avg_sq[k] || sizes[k] < 0)
            return fail(VN_ERR_INVALID, "parameter %d: NULL or negative size", k);
        al.p[k] = params[k];
        al.g[k] = grads[k];
        al.m[k] = exp_avg[k];
        al.v[k] = exp_avg_sq[k];
        al.step[k] = steps ? steps[k] : nullptr;
        al.n[k] = sizes[k];
        total += sizes[k];
    }
    const double bc1 = 1.0 - pow((double)beta1, (double)step), bc2 = 1.0 - pow((double)beta2, (double)step);
    int blocks = (int)((total / 4 + 255) / 256);
    blocks = blocks < 1 ? 1 : (blocks > 2048 ? 2048 : blocks);
    hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, al, clip_scale, skip, lr, beta1,
                       beta2, eps, (float)bc1, (float)sqrt(bc2), (float)step);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

int vn_minibatch_rows(const int64_t *idx, int32_t M, int32_t T, int32_t N, const float *obs, int32_t D, float *out,
                      int64_t *src, void *stream) {
    if (!idx || !obs || !out || !src) return fail(VN_ERR_INVALID, "NULL argument");
    if (M < 1 || T < 1 || N < 1 || D < 4 || D % 4) return fail(VN_ERR_INVALID, "bad sizes M=%d T=%d N=%d D=%d", M, T, N, D);
    if ((((uintptr_t)obs) | ((uintptr_t)out)) & 15) return fail(VN_ERR_INVALID, "obs / out must be 16-B aligned");
    hipLaunchKernelGGL(minibatch_rows_kernel, dim3((unsigned)((M + 15) / 16)), dim3(256), 0, (hipStream_t)stream, idx,
                       M, T, N, obs, D, out, src);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

}  // extern "C"
