"""The PPO learner's matrix products on the f32 matrix cores (no library GEMM).

Autograd functions over the HIP kernels of csrc/voxnav_gemm_f32.hip for the
learner's Linear layers (SB3 ``MlpExtractor`` + ``action_net`` /
``value_net``, reached from ``RecurrentPPO.train`` / ``PPO.train`` at
train/Grid_Train.py:228) and the LSTM weight gradients:

* ``linear_tanh_pair``: one Tanh layer of BOTH branches (pi, vf) per launch,
  forward ``tanh(x W^T + b)``; backward ``dX = (dY (1 - Y^2)) W`` with the
  Tanh backward formed on the operand load, ``dW = dZ^T X`` split over the
  sample axis (per-split partials summed in order) and ``db = sum dZ`` from
  the same staged tiles;
* ``linear``: a Linear without activation (the heads), same backward;
* ``mm_tn``: ``a^T b`` over a tall sample axis (+ the column sums of a).

f32 throughout (the reference's dtype).  CUDA tensors only; the CPU path
(the CPU parity tests) uses torch's own ops.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Tuple

import torch

from . import _native

SPLIT_ROWS = 256         # minimum rows of the sample axis per split of a weight-gradient product


def _p(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream(dev):
    return C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _splits(K: int, tiles: int) -> int:
    """Split count for a K-long reduction whose output has `tiles` 128x128 tiles:
    enough blocks to fill the chip (>= ~512), at least SPLIT_ROWS rows each."""
    want = max(1, -(-512 // max(1, tiles)))
    sp = max(1, min(want, 256, K // SPLIT_ROWS))
    # a multiple of 8 when it can be: the kernel then deals whole splits to one
    # XCD each (csrc/voxnav_gemm_f32.hip), so a split's operand rows are read
    # into one L2
    return sp if sp < 8 else sp // 8 * 8


def mm_tn(a: torch.Tensor, b: torch.Tensor, y: Optional[torch.Tensor] = None, colsum: bool = False,
          out: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Batched ``z^T b`` with z = a (1 - y^2) if y is given else a.
    a, y: [batch, K, M]; b: [batch, K, N] (batch stride 0 allowed via expand);
    returns ([batch, M, N], [batch, M] column sums of z or None)."""
    lib = _native.load()
    Bt, K, M = a.shape
    N = b.shape[2]
    dev = a.device
    if a.stride(2) != 1 or a.stride(1) != M or b.stride(2) != 1 or b.stride(1) != N:
        raise ValueError("mm_tn: operands must be row-contiguous [batch, K, cols]")
    tiles = -(-M // 128) * -(-N // 128) * Bt
    sp = _splits(K, tiles)
    out = torch.empty((Bt, M, N), dtype=torch.float32, device=dev) if out is None else out
    ws = torch.empty(sp * Bt * M * N, dtype=torch.float32, device=dev)
    cs = torch.empty((Bt, M), dtype=torch.float32, device=dev) if colsum else None
    ws2 = torch.empty(sp * Bt * M, dtype=torch.float32, device=dev) if colsum else None
    _native.check(lib.vn_gemm_f32_tn(_p(a), _p(y), M, a.stride(0), _p(b), N, b.stride(0), _p(out), M * N, _p(cs),
                                     M, N, K, Bt, sp, _p(ws), _p(ws2), 0, _stream(dev)), "vn_gemm_f32_tn")
    return out, cs


def _pair_stride(a: torch.Tensor, b: torch.Tensor) -> int:
    """Element offset from tensor a to tensor b (same shape, contiguous f32):
    the kernels' batch stride, so the two branches' parameters are read in
    place instead of stacked into a [2, ...] copy every minibatch."""
    d = b.data_ptr() - a.data_ptr()
    if d % 4 or a.shape != b.shape or not (a.is_contiguous() and b.is_contiguous()):
        raise ValueError("pair operands must be contiguous f32 tensors of one shape")
    return d // 4


class _LinearTanhPair(torch.autograd.Function):
    """y[br] = tanh(x[br] W[br]^T + b[br]) for br in (pi, vf): x [2, M, K]
    (batch stride 0 when both branches read the same input), W_pi, W_vf
    [N, K], b_pi, b_vf [N] (read in place: the batch stride is the distance
    between the two tensors)."""

    @staticmethod
    def forward(ctx, x, wa, wb, ba, bb, tanh: bool):
        lib = _native.load()
        _, M, K = x.shape
        N = wa.shape[0]
        dev = x.device
        y = torch.empty((2, M, N), dtype=torch.float32, device=dev)
        sw, sb = _pair_stride(wa, wb), _pair_stride(ba, bb)
        _native.check(lib.vn_gemm_f32_linear(_p(x), K, x.stride(0), _p(wa), K, sw, _p(ba), sb, _p(y), N, M * N, M, N,
                                             K, 2, 1 if tanh else 0, _stream(dev)), "vn_gemm_f32_linear")
        ctx.save_for_backward(x, wa, wb, y)
        ctx.tanh = tanh
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _native.load()
        x, wa, wb, y = ctx.saved_tensors
        _, M, K = x.shape
        N = wa.shape[0]
        dev = x.device
        st = _stream(dev)
        dy = dy.contiguous()
        yy = y if ctx.tanh else None
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty((2, M, K), dtype=torch.float32, device=dev)
            # dX = dZ W: W [N][K] row-major is the k-major operand of this product
            _native.check(lib.vn_gemm_f32_dx(_p(dy), _p(yy), N, M * N, _p(wa), K, _pair_stride(wa, wb), _p(dx), K,
                                             M * K, M, K, N, 2, st), "vn_gemm_f32_dx")
            # (a shared input was expanded outside: expand's backward sums the branches)
        dw, db = mm_tn(dy, x, y=yy, colsum=True)
        return dx, dw[0], dw[1], db[0], db[1], None


def linear_tanh_pair(x: torch.Tensor, w, b, tanh: bool = True) -> torch.Tensor:
    """x [2, M, K] (or [M, K], shared by both branches); w = (W_pi, W_vf) [N, K]
    each (or one stacked [2, N, K]), b = (b_pi, b_vf) [N] (or [2, N]) -> [2, M, N]."""
    if x.dim() == 2:
        x = x.contiguous().unsqueeze(0).expand(2, *x.shape)
    elif not x.is_contiguous():
        x = x.contiguous()
    if isinstance(w, torch.Tensor):
        w = (w[0], w[1])
    if isinstance(b, torch.Tensor):
        b = (b[0], b[1])
    return _LinearTanhPair.apply(x, w[0], w[1], b[0], b[1], tanh)


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        lib = _native.load()
        M, K = x.shape
        N = w.shape[0]
        dev = x.device
        y = torch.empty((M, N), dtype=torch.float32, device=dev)
        _native.check(lib.vn_gemm_f32_linear(_p(x), K, 0, _p(w), K, 0, _p(b), 0, _p(y), N, 0, M, N, K, 1, 0,
                                             _stream(dev)), "vn_gemm_f32_linear")
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _native.load()
        x, w = ctx.saved_tensors
        M, K = x.shape
        N = w.shape[0]
        dev = x.device
        dy = dy.contiguous()
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty((M, K), dtype=torch.float32, device=dev)
            _native.check(lib.vn_gemm_f32_dx(_p(dy), None, N, 0, _p(w), K, 0, _p(dx), K, 0, M, K, N, 1, _stream(dev)),
                          "vn_gemm_f32_dx")
        dw, db = mm_tn(dy.unsqueeze(0), x.unsqueeze(0), colsum=True)
        return dx, dw[0], db[0]


def linear(x: torch.Tensor, module: torch.nn.Linear) -> torch.Tensor:
    """``module(x)`` for 2-D x on the matrix-core kernels (CUDA), torch otherwise."""
    if x.device.type != "cuda":
        return module(x)
    return _Linear.apply(x.contiguous(), module.weight, module.bias)


def mlp_pair(pi_net: torch.nn.Sequential, vf_net: torch.nn.Sequential, x_pi: torch.Tensor,
             x_vf: Optional[torch.Tensor] = None, x_pair: Optional[torch.Tensor] = None, stacked: bool = False):
    """Both SB3 MLP branches (Linear + Tanh layers of equal widths) layer by
    layer, the two branches of a layer in one launch.  ``x_vf is None``: both
    read ``x_pi`` (MlpPolicy's observation).  ``x_pair`` [2, M, K]: the two
    branches' inputs already stacked (the row-layout LSTM's output), used
    as is -- no stacking copy forward, no gradient accumulation backward.
    Returns (h_pi, h_vf); with ``stacked`` the [2, M, F] pair itself, or None
    when the branches do not take the paired kernels."""
    def tanh_layers(seq):   # [Linear, Tanh] * n, or None
        mods = list(seq)
        if len(mods) % 2 or not all(isinstance(a, torch.nn.Linear) and a.bias is not None and
                                    isinstance(t, torch.nn.Tanh) for a, t in zip(mods[0::2], mods[1::2])):
            return None
        return mods[0::2]
    lin_pi, lin_vf = tanh_layers(pi_net), tanh_layers(vf_net)
    if x_pair is not None:
        x_pi, x_vf = x_pair[0], x_pair[1]
    if (x_pi.device.type != "cuda" or lin_pi is None or lin_vf is None or len(lin_pi) != len(lin_vf) or
            any(a.weight.shape != b.weight.shape for a, b in zip(lin_pi, lin_vf))):
        if stacked:
            return None
        return pi_net(x_pi), vf_net(x_pi if x_vf is None else x_vf)
    h = x_pair if x_pair is not None else (x_pi if x_vf is None else torch.stack([x_pi, x_vf]))
    for a, b in zip(lin_pi, lin_vf):
        h = linear_tanh_pair(h, (a.weight, b.weight), (a.bias, b.bias), tanh=True)
    return h if stacked else (h[0], h[1])


def ppo_loss_supported(action_net: torch.nn.Linear, value_net: torch.nn.Linear, F: int) -> bool:
    """The fused loss kernel takes these heads (F = latent width)."""
    return (F % 64 == 0 and 64 <= F <= 256 and action_net.in_features == F and value_net.in_features == F and
            value_net.out_features == 1 and 1 <= action_net.out_features <= 8 and action_net.bias is not None and
            value_net.bias is not None)


def ppo_loss(h: torch.Tensor, action_net: torch.nn.Linear, value_net: torch.nn.Linear, src: Optional[torch.Tensor],
             actions: torch.Tensor, advantages: torch.Tensor, old_log_prob: torch.Tensor, returns: torch.Tensor,
             clip_range: float, ent_coef: float, vf_coef: float, normalize_advantage: bool):
    """The PPO minibatch loss and its gradient (csrc/voxnav_ppo_loss.hip): the
    heads, the advantage normalisation, the clipped surrogate, value MSE and
    entropy bonus of sb3 (Recurrent)PPO.train, in three launches.

    h [2, M, F]: the (actor, critic) latents; src [M] int64 (or None): the
    samples' rows in the flat rollout buffers ``actions`` (int32),
    ``advantages``, ``old_log_prob``, ``returns``.  Returns (dh [2, M, F],
    (d action_net.weight, d action_net.bias, d value_net.weight,
    d value_net.bias), stats f64 [6]: policy loss, value loss, entropy loss,
    loss, approx kl, clip fraction).  Nothing is differentiated here: the
    caller backpropagates dh from h and assigns the head gradients."""
    lib = _native.load()
    _, M, F = h.shape
    A = action_net.out_features
    dev = h.device
    if h.stride(2) != 1 or h.stride(1) != F:
        raise ValueError("ppo_loss: latents must be row-contiguous [2, M, F]")
    for t, dt in ((actions, torch.int32), (advantages, torch.float32), (old_log_prob, torch.float32),
                  (returns, torch.float32)):
        if t.dtype != dt or not t.is_contiguous() or t.device != dev:
            raise ValueError("ppo_loss: buffers must be contiguous int32 actions / f32 values on the latents' device")
    if src is not None and (src.dtype != torch.int64 or src.numel() != M or not src.is_contiguous()):
        raise ValueError("ppo_loss: src must be [M] contiguous int64")
    npart, nspart = C.c_int64(), C.c_int64()
    _native.check(lib.vn_ppo_loss_part_floats(M, F, A, C.byref(npart), C.byref(nspart)), "vn_ppo_loss_part_floats")
    dh = torch.empty((2, M, F), dtype=torch.float32, device=dev)
    gh = torch.empty(A * F + A + F + 1, dtype=torch.float32, device=dev)
    dbl = torch.empty(6 + 128 + nspart.value, dtype=torch.float64, device=dev)
    part = torch.empty(npart.value, dtype=torch.float32, device=dev)
    stats = dbl[:6]
    wa, ba = action_net.weight.detach(), action_net.bias.detach()
    wv, bv = value_net.weight.detach(), value_net.bias.detach()
    _native.check(lib.vn_ppo_loss(_p(h[0]), _p(h[1]), F, _p(wa.contiguous()), _p(ba), _p(wv.contiguous()), _p(bv),
                                  _p(src), _p(actions), _p(advantages), _p(old_log_prob), _p(returns), M, F, A,
                                  float(clip_range), float(ent_coef), float(vf_coef), int(bool(normalize_advantage)),
                                  _p(dh[0]), _p(dh[1]), _p(gh), _p(stats), _p(dbl[6:134]), _p(part), _p(dbl[134:]),
                                  _stream(dev)), "vn_ppo_loss")
    grads = (gh[:A * F].view(A, F), gh[A * F:A * F + A], gh[A * F + A:A * F + A + F].view(1, F), gh[-1:])
    return dh, grads, stats


def grad_norm_scale(params, max_norm: float, work: Optional[torch.Tensor] = None):
    """The total 2-norm of the parameters' gradients and the divisor that
    clips them to ``max_norm`` (csrc/voxnav_ppo_loss.hip vn_grad_norm): two
    launches, device scalars (norm, scale) -- handed to the fused Adam step as
    its grad_scale instead of rescaling every gradient in place
    (torch.nn.utils.clip_grad_norm_'s update, folded into the step)."""
    lib = _native.load()
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        raise ValueError("grad_norm_scale: no gradients")
    dev = grads[0].device
    for g in grads:
        if g.dtype != torch.float32 or not g.is_contiguous() or g.device != dev:
            raise ValueError("grad_norm_scale: gradients must be contiguous f32 on one device")
    n = len(grads)
    ptrs = (C.c_void_p * n)(*[g.data_ptr() for g in grads])
    sizes = (C.c_int64 * n)(*[g.numel() for g in grads])
    out = torch.empty(2, dtype=torch.float32, device=dev)
    work = torch.empty(256, dtype=torch.float64, device=dev) if work is None else work
    _native.check(lib.vn_grad_norm(ptrs, sizes, n, float(max_norm), _p(out[0:1]), _p(out[1:2]), _p(work),
                                   _stream(dev)), "vn_grad_norm")
    return out[0], out[1]


def adam_step(optimizer: torch.optim.Adam, clip_scale: Optional[torch.Tensor] = None,
              skip: Optional[torch.Tensor] = None) -> None:
    """``optimizer.step()`` for a single-group ``torch.optim.Adam`` (no
    amsgrad / weight decay / maximize) on the library's kernel
    (csrc/voxnav_ppo_loss.hip vn_adam_step): one launch over every parameter,
    the gradients divided by ``clip_scale`` (``grad_norm_scale``'s divisor) on
    the way.  The optimizer's own state tensors are updated in place
    (``exp_avg``, ``exp_avg_sq``, ``step``), so ``state_dict()`` / checkpoints
    are torch's.  ``skip``: a device int32 word; when it is nonzero at run
    time the step changes nothing (the row-layout LSTM's error word: the
    gradients of a timed-out launch are never applied)."""
    lib = _native.load()
    if len(optimizer.param_groups) != 1:
        raise ValueError("adam_step: one parameter group")
    grp = optimizer.param_groups[0]
    if grp.get("amsgrad") or grp.get("weight_decay") or grp.get("maximize"):
        raise ValueError("adam_step: plain Adam only (no amsgrad, weight decay or maximize)")
    params = [p for p in grp["params"] if p.grad is not None]
    if not params:
        return
    dev = params[0].device
    steps = []
    for p in params:
        st = optimizer.state[p]
        if not st:
            st["step"] = torch.zeros((), dtype=torch.float32, device=dev)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        if skip is not None and (st["step"].device != dev or st["step"].dtype != torch.float32):
            # a gated step: the counter must live on the device, where the kernel
            # advances it only when the step is applied
            st["step"] = st["step"].to(device=dev, dtype=torch.float32)
        steps.append(st["step"])
        for t in (p, p.grad, st["exp_avg"], st["exp_avg_sq"]):
            if t.dtype != torch.float32 or not t.is_contiguous() or t.device != dev:
                raise ValueError("adam_step: contiguous f32 parameters, gradients and moments on one device")
    # the step count, kept on the host (read back once after a fresh state or a load_state_dict)
    cache = getattr(optimizer, "_vn_adam_t", None)
    if cache is None or cache[0] is not steps[0]:
        t = int(round(float(steps[0].item())))
    else:
        t = cache[1]
    t += 1
    optimizer._vn_adam_t = (steps[0], t)
    n = len(params)
    arr = lambda ts: (C.c_void_p * n)(*[x.data_ptr() for x in ts])  # noqa: E731
    st_ptrs = [s if (s.device == dev and s.dtype == torch.float32) else None for s in steps]
    steps_arr = (C.c_void_p * n)(*[(x.data_ptr() if x is not None else None) for x in st_ptrs])
    sizes = (C.c_int64 * n)(*[p.numel() for p in params])
    b1, b2 = grp["betas"]
    _native.check(lib.vn_adam_step(arr(params), arr([p.grad for p in params]),
                                   arr([optimizer.state[p]["exp_avg"] for p in params]),
                                   arr([optimizer.state[p]["exp_avg_sq"] for p in params]), steps_arr, sizes, n,
                                   _p(clip_scale), _p(skip), float(grp["lr"]), float(b1), float(b2), float(grp["eps"]), t,
                                   _stream(dev)), "vn_adam_step")
    for s, x in zip(steps, st_ptrs):
        if x is None:                       # a CPU / other-dtype step counter (a loaded state): set on the host
            s.fill_(float(t))


def minibatch_rows(idx: torch.Tensor, T: int, N: int, obs: torch.Tensor):
    """(src, obs rows) of a feed-forward PPO minibatch in one launch
    (vn_minibatch_rows): idx [M] env-major flat ids (int64), obs [T, N, D]
    -> src [M] int64 rows of the [T, N]-major buffers, [M, D] observations."""
    lib = _native.load()
    M = idx.numel()
    D = obs.shape[-1]
    dev = idx.device
    if idx.dtype != torch.int64 or not idx.is_contiguous() or not obs.is_contiguous() or obs.dtype != torch.float32:
        raise ValueError("minibatch_rows: contiguous int64 ids and f32 observations")
    out = torch.empty((M, D), dtype=torch.float32, device=dev)
    src = torch.empty(M, dtype=torch.int64, device=dev)
    _native.check(lib.vn_minibatch_rows(_p(idx), M, T, N, _p(obs), D, _p(out), _p(src), _stream(dev)),
                  "vn_minibatch_rows")
    return src, out
