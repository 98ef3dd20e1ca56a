// voxnav_learn.hip -- the PPO learner's LSTM re-run (sb3_contrib
// RecurrentPPO.train -> RecurrentActorCriticPolicy.evaluate_actions ->
// _process_sequence, reached from model.learn at train/Grid_Train.py:228).
//
// The learner re-runs the actor and the critic LSTM over every minibatch's
// padded sequences and back-propagates through them.  The matrix products
// are library GEMMs issued by the caller (voxnav/lstm_seq.py):
//   forward   X @ [W_ih_actor | W_ih_critic]^T once for all steps, then per
//             step h_{t-1} @ W_hh^T for both LSTMs as one batched GEMM;
//   backward  per step dG_t @ W_hh (batched), then the weight gradients as
//             three large GEMMs over all steps (dG^T X, dG^T H_prev) and a
//             column sum for the biases;
// and these two kernels are the per-step work in between:
//   seq_cell_fwd_kernel   pre = gx + gh + b;  i,f,g,o;  c = f*c + i*g;
//                         h = o*tanh(c); the activations are kept for the
//                         backward pass
//   seq_cell_bwd_kernel   dh = dh_out + dh_rec;  dc += dh*o*(1-tanh(c)^2);
//                         dG = (dc*g*i(1-i), dc*c_prev*f(1-f),
//                               dc*i*(1-g^2), dh*tanh(c)*o(1-o));
//                         dc_prev = dc*f
// Both LSTMs (n_lstm = 2) of a step in one launch; a thread owns 4
// consecutive hidden units of one (LSTM, row), float4 loads and stores.
// f32 throughout (the reference's dtype), -ffp-contract=off like the rest.

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <cstdint>
#include <mutex>

#include "vn_common.h"

using vn_detail::fail;

namespace {

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ void st4(float *p, const float4 &v) { *reinterpret_cast<float4 *>(p) = v; }

#define VN_F4(op)  \
    op(x) op(y) op(z) op(w)

// gx: element (l, b, j) at gx[b * gx_row + l * gx_lstm + j]  (j < 4H)
// gates: [n_lstm][B][4H] at lstm stride s4 -- in: h_{t-1} @ W_hh^T, out: the
//   activations (i, f, g, o) kept for the backward pass (in place)
// c_prev, c_new, h_new: [n_lstm][B][H] at lstm stride s1
__global__ __launch_bounds__(256) void seq_cell_fwd_kernel(const float *__restrict__ gx, int64_t gx_row,
                                                           int64_t gx_lstm, float *__restrict__ gates,
                                                           const float *__restrict__ bias,
                                                           const float *__restrict__ c_prev, float *__restrict__ c_new,
                                                           float *__restrict__ h_new, int64_t s4, int64_t s1,
                                                           int n_lstm, int B, int H) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int H4 = H >> 2;
    const int64_t per_l = (int64_t)B * H4;
    if (q >= per_l * n_lstm) return;
    const int l = (int)(q / per_l);
    const int64_t r = q - (int64_t)l * per_l;
    const int b = (int)(r / H4);
    const int j = (int)(r - (int64_t)b * H4) * 4;
    const int G = 4 * H;
    const float *px = gx + (int64_t)b * gx_row + (int64_t)l * gx_lstm + j;
    float *pg = gates + (int64_t)l * s4 + (int64_t)b * G + j;
    const float *pb = bias + (int64_t)l * G + j;
    float4 a[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float4 s = ld4(px + k * H);
        const float4 y = ld4(pg + k * H);
        const float4 bb = ld4(pb + k * H);
#define ADD(c) s.c += y.c; s.c += bb.c;
        VN_F4(ADD)
#undef ADD
        a[k] = s;
    }
    const int64_t so = (int64_t)l * s1 + (int64_t)b * H + j;
    const float4 cp = ld4(c_prev + so);
    float4 cn, hn;
#define CELL(c)                                                     \
    {                                                               \
        a[0].c = sigm(a[0].c);                                      \
        a[1].c = sigm(a[1].c);                                      \
        a[2].c = tanhf(a[2].c);                                     \
        a[3].c = sigm(a[3].c);                                      \
        const float fc = a[1].c * cp.c, ig = a[0].c * a[2].c;       \
        cn.c = fc + ig;                                             \
        hn.c = a[3].c * tanhf(cn.c);                                \
    }
    VN_F4(CELL)
#undef CELL
    st4(c_new + so, cn);
    st4(h_new + so, hn);
#pragma unroll
    for (int k = 0; k < 4; ++k) st4(pg + k * H, a[k]);
}

// dh_out: gradient of the step's output h, [n_lstm][B][H] (lstm stride so1,
// row stride H); dh_rec: [n_lstm][B][H] contiguous from the later step (NULL
// at the last step); dc: [n_lstm][B][H] in/out (dc of c_t in, dc of c_{t-1}
// out); act, dG: [n_lstm][B][4H] at lstm strides sa, sg; c_prev, c_new:
// lstm stride s1.
__global__ __launch_bounds__(256) void seq_cell_bwd_kernel(const float *__restrict__ dh_out, int64_t so1,
                                                           const float *__restrict__ dh_rec, float *__restrict__ dc,
                                                           const float *__restrict__ act, int64_t sa,
                                                           const float *__restrict__ c_prev,
                                                           const float *__restrict__ c_new, int64_t s1,
                                                           float *__restrict__ dG, int64_t sg, int n_lstm, int B,
                                                           int H) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int H4 = H >> 2;
    const int64_t per_l = (int64_t)B * H4;
    if (q >= per_l * n_lstm) return;
    const int l = (int)(q / per_l);
    const int64_t r = q - (int64_t)l * per_l;
    const int b = (int)(r / H4);
    const int j = (int)(r - (int64_t)b * H4) * 4;
    const int G = 4 * H;
    const int64_t sd = ((int64_t)l * B + b) * H + j;          // contiguous [n_lstm][B][H]
    float4 dh = ld4(dh_out + (int64_t)l * so1 + (int64_t)b * H + j);
    if (dh_rec) {
        const float4 y = ld4(dh_rec + sd);
#define ADD(c) dh.c += y.c;
        VN_F4(ADD)
#undef ADD
    }
    float4 dcv = ld4(dc + sd);
    const int64_t so = (int64_t)l * s1 + (int64_t)b * H + j;
    const float4 cp = ld4(c_prev + so), cn = ld4(c_new + so);
    const float *pa = act + (int64_t)l * sa + (int64_t)b * G + j;
    const float4 ig = ld4(pa), fg = ld4(pa + H), gg = ld4(pa + 2 * H), og = ld4(pa + 3 * H);
    float4 di, df, dg, dov, dcp;
#define BWD(c)                                                      \
    {                                                               \
        const float tc = tanhf(cn.c);                               \
        const float dtc = dh.c * og.c;                              \
        const float dcc = dcv.c + dtc * (1.0f - tc * tc);           \
        dov.c = dh.c * tc * (og.c * (1.0f - og.c));                 \
        di.c = dcc * gg.c * (ig.c * (1.0f - ig.c));                 \
        df.c = dcc * cp.c * (fg.c * (1.0f - fg.c));                 \
        dg.c = dcc * ig.c * (1.0f - gg.c * gg.c);                   \
        dcp.c = dcc * fg.c;                                         \
    }
    VN_F4(BWD)
#undef BWD
    st4(dc + sd, dcp);
    float *pg = dG + (int64_t)l * sg + (int64_t)b * G + j;
    st4(pg, di);
    st4(pg + H, df);
    st4(pg + 2 * H, dg);
    st4(pg + 3 * H, dov);
}

#undef VN_F4

int grid_for(int n_lstm, int B, int H, dim3 &grid) {
    const int64_t threads = (int64_t)n_lstm * B * (H / 4);
    grid = dim3((unsigned)((threads + 255) / 256));
    return 0;
}

// ----------------------------------------------------------------------------
// The whole time loop in native code (vn_lstm_seq_fwd / vn_lstm_seq_bwd): per
// step one strided-batched rocBLAS SGEMM for both LSTMs and the cell kernel.
// Issued from Python, the two launches of a step cost ~30 us of host time
// against ~20 us of GPU work, so the GPU idled a third of the loop.  rocBLAS
// is bound at run time (dlopen by soname): in a PyTorch process that is the
// copy torch already loaded, so the process keeps one rocBLAS / HIP runtime
// and libvoxnav.so has no link-time BLAS dependency.
// ----------------------------------------------------------------------------
struct Blas {
    decltype(&rocblas_create_handle) create = nullptr;
    decltype(&rocblas_destroy_handle) destroy = nullptr;
    decltype(&rocblas_set_stream) set_stream = nullptr;
    decltype(&rocblas_sgemm_strided_batched) sgemm_sb = nullptr;
    bool ok = false;
};

Blas &blas() {
    static Blas b;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("librocblas.so.5", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librocblas.so.5", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("librocblas.so", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        b.create = reinterpret_cast<decltype(&rocblas_create_handle)>(dlsym(h, "rocblas_create_handle"));
        b.destroy = reinterpret_cast<decltype(&rocblas_destroy_handle)>(dlsym(h, "rocblas_destroy_handle"));
        b.set_stream = reinterpret_cast<decltype(&rocblas_set_stream)>(dlsym(h, "rocblas_set_stream"));
        b.sgemm_sb =
            reinterpret_cast<decltype(&rocblas_sgemm_strided_batched)>(dlsym(h, "rocblas_sgemm_strided_batched"));
        b.ok = b.create && b.destroy && b.set_stream && b.sgemm_sb;
    });
    return b;
}

// The calling thread's handles, one per device, destroyed when the thread
// exits (a thread pool's short-lived workers do not leak them).
struct ThreadHandles {
    rocblas_handle h[64] = {};
    ~ThreadHandles() {
        Blas &b = blas();
        for (int d = 0; d < 64; ++d)
            if (h[d] && b.destroy) {
                int cur = -1;
                if (hipGetDevice(&cur) == hipSuccess && cur != d) (void)hipSetDevice(d);
                (void)b.destroy(h[d]);
                if (cur >= 0 && cur != d) (void)hipSetDevice(cur);
            }
    }
};

// the calling thread's handle for its current device, bound to `stream`.
// One handle per (thread, device): a handle carries its stream, so a handle
// shared between threads driving different streams would let one thread's
// GEMMs run on the other's stream.
int blas_handle(hipStream_t stream, rocblas_handle &out) {
    Blas &b = blas();
    if (!b.ok) return fail(VN_ERR_HIP, "rocBLAS (librocblas.so.5) could not be loaded");
    int dev = 0;
    VN_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return fail(VN_ERR_INVALID, "device %d out of range", dev);
    thread_local ThreadHandles th;
    rocblas_handle *handles = th.h;
    if (!handles[dev] && b.create(&handles[dev]) != rocblas_status_success)
        return fail(VN_ERR_HIP, "rocblas_create_handle failed");
    if (b.set_stream(handles[dev], stream) != rocblas_status_success) return fail(VN_ERR_HIP, "rocblas_set_stream failed");
    out = handles[dev];
    return VN_OK;
}

}  // namespace

extern "C" {

int vn_lstm_seq_fwd_cell(const float *gx, int64_t gx_row_stride, int64_t gx_lstm_stride, float *gates,
                         int64_t gate_lstm_stride, const float *bias, const float *c_prev, float *c_new, float *h_new,
                         int64_t state_lstm_stride, int32_t n_lstm, int32_t B, int32_t H, void *stream) {
    if (!gx || !gates || !bias || !c_prev || !c_new || !h_new) return fail(VN_ERR_INVALID, "NULL argument");
    if (n_lstm < 1 || B < 1 || H < 4 || (H % 4)) return fail(VN_ERR_INVALID, "bad sizes n_lstm=%d B=%d H=%d", n_lstm, B, H);
    if ((gx_row_stride | gx_lstm_stride | gate_lstm_stride | state_lstm_stride) & 3)
        return fail(VN_ERR_INVALID, "strides must be multiples of 4 floats");
    dim3 grid;
    grid_for(n_lstm, B, H, grid);
    hipLaunchKernelGGL(seq_cell_fwd_kernel, grid, dim3(256), 0, (hipStream_t)stream, gx, gx_row_stride,
                       gx_lstm_stride, gates, bias, c_prev, c_new, h_new, gate_lstm_stride, state_lstm_stride,
                       n_lstm, B, H);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

int vn_lstm_seq_bwd_cell(const float *dh_out, int64_t dh_out_lstm_stride, const float *dh_rec, float *dc,
                         const float *act, int64_t act_lstm_stride, const float *c_prev, const float *c_new,
                         int64_t state_lstm_stride, float *dG, int64_t dG_lstm_stride, int32_t n_lstm, int32_t B,
                         int32_t H, void *stream) {
    if (!dh_out || !dc || !act || !c_prev || !c_new || !dG) return fail(VN_ERR_INVALID, "NULL argument");
    if (n_lstm < 1 || B < 1 || H < 4 || (H % 4)) return fail(VN_ERR_INVALID, "bad sizes n_lstm=%d B=%d H=%d", n_lstm, B, H);
    if ((dh_out_lstm_stride | act_lstm_stride | state_lstm_stride | dG_lstm_stride) & 3)
        return fail(VN_ERR_INVALID, "strides must be multiples of 4 floats");
    dim3 grid;
    grid_for(n_lstm, B, H, grid);
    hipLaunchKernelGGL(seq_cell_bwd_kernel, grid, dim3(256), 0, (hipStream_t)stream, dh_out, dh_out_lstm_stride,
                       dh_rec, dc, act, act_lstm_stride, c_prev, c_new, state_lstm_stride, dG, dG_lstm_stride, n_lstm,
                       B, H);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

int vn_lstm_seq_fwd(const float *gx, const float *w_hh, const float *bias, float *hs, float *cs, float *act,
                    int32_t n_lstm, int32_t L, int32_t B, int32_t H, void *stream) {
    if (!gx || !w_hh || !bias || !hs || !cs || !act) return fail(VN_ERR_INVALID, "NULL argument");
    if (n_lstm < 1 || L < 1 || B < 1 || H < 4 || (H % 4)) return fail(VN_ERR_INVALID, "bad sizes n_lstm=%d L=%d B=%d H=%d", n_lstm, L, B, H);
    const hipStream_t st = (hipStream_t)stream;
    rocblas_handle h;
    int rc = blas_handle(st, h);
    if (rc) return rc;
    const int64_t G = 4 * (int64_t)H, sstate = (int64_t)(L + 1) * B * H;
    dim3 grid;
    grid_for(n_lstm, B, H, grid);
    const float one = 1.0f, zero = 0.0f;
    for (int t = 0; t < L; ++t) {
        // act[t][l] (B x 4H, row-major) = hs[l][t] (B x H) @ W_hh[l]^T: column-major, act^T = W_hh (op T) x hs^T
        float *at = act + (int64_t)t * n_lstm * B * G;
        if (blas().sgemm_sb(h, rocblas_operation_transpose, rocblas_operation_none, (rocblas_int)G, B, H, &one, w_hh, H,
                            G * H, hs + (int64_t)t * B * H, H, sstate, &zero, at, (rocblas_int)G, (int64_t)B * G,
                            n_lstm) != rocblas_status_success)
            return fail(VN_ERR_HIP, "rocblas_sgemm_strided_batched (forward step %d) failed", t);
        hipLaunchKernelGGL(seq_cell_fwd_kernel, grid, dim3(256), 0, st, gx + (int64_t)t * B * n_lstm * G,
                           (int64_t)n_lstm * G, G, at, bias, cs + (int64_t)t * B * H, cs + (int64_t)(t + 1) * B * H,
                           hs + (int64_t)(t + 1) * B * H, (int64_t)B * G, sstate, n_lstm, B, H);
    }
    VN_HIP(hipGetLastError());
    return VN_OK;
}

int vn_lstm_seq_bwd(const float *dh_out, const float *w_hh, const float *act, const float *cs, float *dG, float *dc,
                    float *dh, int32_t need_dh0, int32_t n_lstm, int32_t L, int32_t B, int32_t H, void *stream) {
    if (!dh_out || !w_hh || !act || !cs || !dG || !dc || !dh) return fail(VN_ERR_INVALID, "NULL argument");
    if (n_lstm < 1 || L < 1 || B < 1 || H < 4 || (H % 4)) return fail(VN_ERR_INVALID, "bad sizes n_lstm=%d L=%d B=%d H=%d", n_lstm, L, B, H);
    const hipStream_t st = (hipStream_t)stream;
    rocblas_handle h;
    int rc = blas_handle(st, h);
    if (rc) return rc;
    const int64_t G = 4 * (int64_t)H, sstate = (int64_t)(L + 1) * B * H;
    dim3 grid;
    grid_for(n_lstm, B, H, grid);
    const float one = 1.0f, zero = 0.0f;
    for (int t = L - 1; t >= 0; --t) {
        float *dgt = dG + (int64_t)t * B * G;
        hipLaunchKernelGGL(seq_cell_bwd_kernel, grid, dim3(256), 0, st, dh_out + (int64_t)t * B * H, (int64_t)L * B * H,
                           t < L - 1 ? dh : nullptr, dc, act + (int64_t)t * n_lstm * B * G, (int64_t)B * G,
                           cs + (int64_t)t * B * H, cs + (int64_t)(t + 1) * B * H, sstate, dgt, (int64_t)L * B * G,
                           n_lstm, B, H);
        if (t > 0 || need_dh0) {
            // dh[l] (B x H) = dG[l][t] (B x 4H) @ W_hh[l] (4H x H): column-major, dh^T = W_hh^T (as stored) x dG^T
            if (blas().sgemm_sb(h, rocblas_operation_none, rocblas_operation_none, H, B, (rocblas_int)G, &one, w_hh, H,
                                G * H, dgt, (rocblas_int)G, (int64_t)L * B * G, &zero, dh, H, (int64_t)B * H,
                                n_lstm) != rocblas_status_success)
                return fail(VN_ERR_HIP, "rocblas_sgemm_strided_batched (backward step %d) failed", t);
        }
    }
    VN_HIP(hipGetLastError());
    return VN_OK;
}

}  // extern "C"
