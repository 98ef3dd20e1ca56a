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

// Philox4x32-10 (same rounds as the env's random policy); the sampler's
// counter is (global agent id, t | 2^63) so it never collides with the
// env's random-policy stream (gid, t / 4) under the same key.
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
template <typename T>
__global__ __launch_bounds__(256) void lstm_cell_kernel(const T *__restrict__ gx, int64_t gx_row,
                                                        const T *__restrict__ gh, const float *__restrict__ b_ih,
                                                        const float *__restrict__ b_hh, float *__restrict__ h,
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
    const T *ph = gh ? gh + ((int64_t)b * N + n) * G + j : nullptr;
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
    float4 cv = *reinterpret_cast<const float4 *>(c + so);
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
                     void *stream) {
    if (!gx || !b_ih || !b_hh || !h || !c) return fail(VN_ERR_INVALID, "NULL argument");
    if (n_lstm < 1 || N < 1 || H < 4 || (H & 3)) return fail(VN_ERR_INVALID, "bad sizes n_lstm=%d N=%d H=%d", n_lstm, N, H);
    if (gx_row_stride < (int64_t)n_lstm * 4 * H || (gx_row_stride & 3))
        return fail(VN_ERR_INVALID, "gx_row_stride %lld too small / unaligned", (long long)gx_row_stride);
    const int64_t threads = (int64_t)n_lstm * N * (H / 4);
    hipLaunchKernelGGL(lstm_cell_kernel<T>, dim3(blocks_for(threads)), dim3(256), 0, (hipStream_t)stream, gx,
                       gx_row_stride, gh, b_ih, b_hh, h, c, h_bf, h_store, c_store, (int)n_lstm, (int)N, (int)H);
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

extern "C" {

int vn_lstm_cell(const float *gx, int64_t gx_row_stride, const float *gh, const float *b_ih, const float *b_hh,
                 float *h, float *c, float *h_store, float *c_store, int32_t n_lstm, int32_t N, int32_t H,
                 void *stream) {
    return lstm_cell_launch<float>(gx, gx_row_stride, gh, b_ih, b_hh, h, c, nullptr, h_store, c_store, n_lstm, N, H,
                                   stream);
}

int vn_lstm_cell_bf16(const uint16_t *gx, int64_t gx_row_stride, const uint16_t *gh, const float *b_ih,
                      const float *b_hh, float *h, float *c, uint16_t *h_bf16, float *h_store, float *c_store,
                      int32_t n_lstm, int32_t N, int32_t H, void *stream) {
    return lstm_cell_launch<uint16_t>(gx, gx_row_stride, gh, b_ih, b_hh, h, c, h_bf16, h_store, c_store, n_lstm, N,
                                      H, stream);
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

}  // extern "C"
