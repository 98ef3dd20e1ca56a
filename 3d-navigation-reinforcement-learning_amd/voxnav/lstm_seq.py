"""The PPO learner's LSTM re-run on the GPU, forward and backward.

sb3_contrib ``RecurrentPPO.train`` re-runs the actor and the critic LSTM of
``RecurrentActorCriticPolicy`` over each minibatch's sequences
(``evaluate_actions`` -> ``_process_sequence``; reached from ``model.learn``
at train/Grid_Train.py:228) and back-propagates through them.  Here both
LSTMs run together over the padded ``[L, B]`` batch:

forward   ``vn_lstm_seq_fwd_mfma``: the time loop in native code, one
          launch per step: ``[x_t | h_{t-1}] @ [W_ih | W_hh]^T`` for both
          LSTMs on the f32 matrix cores with the cell update (gates, c, h;
          the activations are kept for the backward pass) as the epilogue;
backward  ``vn_lstm_seq_bwd_mfma``: per step, in reverse, ``dh_t +=
          dG_{t+1} @ W_hh`` on the matrix cores with the backward cell
          (gate gradients dG_t, dc_{t-1}) as the epilogue; then the weight
          gradients over all steps at once: ``dW_hh = dG^T H_prev``,
          ``dW_ih = dG^T X``, ``db = sum dG``.

The loop kernels are csrc/voxnav_learn_f32.hip (f32, the reference's dtype);
the loops are native because issued from Python each step's launch costs
more host time than its GPU time.
Padded steps sit after each sequence's real steps and get zero output
gradient from the masked losses, so they never influence the real ones --
the same result as sb3's per-step masked loop (a sequence only begins with
an episode start or the minibatch's first step of an env).

There is no fallback for CUDA tensors: the HIP library must be loaded.
CPU tensors (the CPU parity tests) run torch's own ``nn.LSTM``.
"""
from __future__ import annotations

import ctypes as C
from typing import Tuple

import torch

from . import _native, learn_ops


def _p(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream(dev):
    return C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


class _DualLSTM(torch.autograd.Function):
    """Actor and critic LSTM (one layer each, same input) over [L, B, D]."""

    @staticmethod
    def forward(ctx, x, h0, c0, w_ih_a, w_hh_a, b_ih_a, b_hh_a, w_ih_c, w_hh_c, b_ih_c, b_hh_c):
        lib = _native.load()
        L, B, D = x.shape
        H = w_hh_a.shape[1]
        G = 4 * H
        dev = x.device
        st = _stream(dev)
        xc = x.contiguous()
        w_ih = torch.stack([w_ih_a, w_ih_c])                         # [2, 4H, D]
        D0 = D
        if D % 4:
            # the kernels read x and W_ih in float4s: zero-pad the input width
            # (e.g. simpleEnv's 6L + 7 observation) -- zero columns add nothing
            D = (D + 3) // 4 * 4
            xc = torch.nn.functional.pad(xc, (0, D - D0))
            w_ih = torch.nn.functional.pad(w_ih, (0, D - D0))
        w_ih = w_ih.contiguous()
        w_hh = torch.stack([w_hh_a, w_hh_c]).contiguous()            # [2, 4H, H]
        bias = torch.stack([b_ih_a + b_hh_a, b_ih_c + b_hh_c]).contiguous()
        nf, nb = C.c_int64(), C.c_int64()
        _native.check(lib.vn_lstm_seq_pack_size(2, D, H, C.byref(nf), C.byref(nb)), "vn_lstm_seq_pack_size")
        wpack = torch.empty(nf.value, dtype=torch.float32, device=dev)
        hs = torch.empty((2, L + 1, B, H), dtype=torch.float32, device=dev)
        cs = torch.empty_like(hs)
        hs[:, 0] = h0
        cs[:, 0] = c0
        act = torch.empty((L, 2, B, G), dtype=torch.float32, device=dev)   # step-major: act[t] contiguous
        # [x_t | h_{t-1}] @ [W_ih | W_hh]^T and the cell, one fused launch per step
        _native.check(lib.vn_lstm_seq_fwd_mfma(_p(xc), D, _p(w_ih), _p(w_hh), _p(bias), _p(wpack), _p(hs), _p(cs),
                                               _p(act), 2, L, B, H, st), "vn_lstm_seq_fwd_mfma")
        xf = xc.view(L * B, D)
        ctx.save_for_backward(xf, w_ih_a, w_ih_c, w_hh, hs, cs, act)
        ctx.dims = (L, B, D, D0, H)
        ctx.bwd_pack = nb.value
        return hs[:, 1:]

    @staticmethod
    def backward(ctx, d_out):
        lib = _native.load()
        xf, w_ih_a, w_ih_c, w_hh, hs, cs, act = ctx.saved_tensors
        L, B, D, D0, H = ctx.dims
        G = 4 * H
        dev = xf.device
        st = _stream(dev)
        dh_out = d_out.contiguous()                                 # [2, L, B, H]
        dG = torch.empty((2, L, B, G), dtype=torch.float32, device=dev)
        dc = torch.zeros((2, B, H), dtype=torch.float32, device=dev)
        dh = torch.empty((2, B, H), dtype=torch.float32, device=dev)
        need_h0 = ctx.needs_input_grad[1]
        wpack = torch.empty(ctx.bwd_pack, dtype=torch.float32, device=dev)
        # per step (reverse): dh_t += dG_{t+1} @ W_hh and the cell backward, one fused launch
        _native.check(lib.vn_lstm_seq_bwd_mfma(_p(dh_out), _p(w_hh), _p(wpack), _p(act), _p(cs), _p(dG), _p(dc),
                                               _p(dh) if need_h0 else None, 2, L, B, H, st), "vn_lstm_seq_bwd_mfma")
        dGf = dG.view(2, L * B, G)
        # weight gradients over all steps on the matrix cores (split over the
        # samples): dW_hh = dG^T H_prev (hs[:, :L] is a strided view), dW_ih =
        # dG^T X, db = sum dG (the column sums of the same staged dG tiles)
        d_w_hh, _ = learn_ops.mm_tn(dGf, hs[:, :L].reshape(2, L * B, H))
        d_w_ih, db = learn_ops.mm_tn(dGf, xf.unsqueeze(0).expand(2, L * B, D), colsum=True)
        d_w_ih_a, d_w_ih_c = d_w_ih[0, :, :D0], d_w_ih[1, :, :D0]
        d_w_hh = (d_w_hh[0], d_w_hh[1])
        dx = None
        if ctx.needs_input_grad[0]:
            dx = (dGf[0] @ w_ih_a + dGf[1] @ w_ih_c).view(L, B, D0)
        dh0 = dh.clone() if need_h0 else None
        dc0 = dc.clone() if ctx.needs_input_grad[2] else None
        # b_ih and b_hh get the same gradient, but as separate tensors:
        # autograd may keep an incoming gradient as the leaf's .grad without
        # copying, and the in-place grad clipping would then scale a shared
        # tensor twice
        return (dx, dh0, dc0, d_w_ih_a, d_w_hh[0], db[0].clone(), db[0].clone(), d_w_ih_c, d_w_hh[1],
                db[1].clone(), db[1].clone())


class _DualLSTMRows(torch.autograd.Function):
    """Actor and critic LSTM over the row layout (csrc/voxnav_learn_rows.hip):
    x [L, B, D]; a row restarts from the stored state (h_store / c_store
    [T, 2, N, H] at (t, env[t, r])) times keep[t, r] wherever start[t, r]."""

    @staticmethod
    def forward(ctx, x, env, start, keep, h_store, c_store, w_ih_a, w_hh_a, b_ih_a, b_hh_a, w_ih_c, w_hh_c, b_ih_c,
                b_hh_c):
        lib = _native.load()
        L, B, D = x.shape
        H = w_hh_a.shape[1]
        G = 4 * H
        dev = x.device
        st = _stream(dev)
        xc = x.contiguous()
        w_ih = torch.stack([w_ih_a, w_ih_c]).contiguous()
        w_hh = torch.stack([w_hh_a, w_hh_c]).contiguous()
        bias = torch.stack([b_ih_a + b_hh_a, b_ih_c + b_hh_c]).contiguous()
        nt = -(-B // 32)                        # row tiles of 32 (csrc/voxnav_learn_rows.hip RW)
        hout = torch.empty((2, L, B, H), dtype=torch.float32, device=dev)
        hprev, cprev, cnew = torch.empty_like(hout), torch.empty_like(hout), torch.empty_like(hout)
        act = torch.empty((2, L, B, G), dtype=torch.float32, device=dev)
        cnt = torch.empty(2 * nt * 64, dtype=torch.int32, device=dev)   # a 256-B line per group counter
        err = _rows_err(dev)
        _native.check(lib.vn_lstm_rows_fwd(_p(xc), D, _p(w_ih), _p(w_hh), _p(bias), _p(h_store), _p(c_store),
                                           h_store.shape[2], _p(env), _p(start), _p(keep), _p(hout), _p(hprev),
                                           _p(cprev), _p(cnew), _p(act), _p(cnt), _p(err), L, B, H, st),
                      "vn_lstm_rows_fwd")
        ctx.save_for_backward(xc, w_hh, start, hprev, cprev, cnew, act, w_ih_a, w_ih_c)
        ctx.dims = (L, B, D, H)
        return hout

    @staticmethod
    def backward(ctx, d_out):
        lib = _native.load()
        xc, w_hh, start, hprev, cprev, cnew, act, w_ih_a, w_ih_c = ctx.saved_tensors
        L, B, D, H = ctx.dims
        G = 4 * H
        dev = xc.device
        st = _stream(dev)
        dh_out = d_out.contiguous()
        # dG itself only for an input gradient (the learner's x never needs one)
        need_dx = ctx.needs_input_grad[0]
        dG = torch.empty((2, L, B, G), dtype=torch.float32, device=dev) if need_dx else None
        nf = C.c_int64()
        _native.check(lib.vn_lstm_rows_part_floats(B, C.byref(nf)), "vn_lstm_rows_part_floats")
        part = torch.empty(nf.value, dtype=torch.float32, device=dev)
        cnt = torch.empty(2 * -(-B // 32) * 64, dtype=torch.int32, device=dev)
        # dG and, inside the same persistent launch, the weight and bias gradients,
        # written in the parameters' own layouts (no slicing copies)
        d_w_hh = torch.empty((2, G, H), dtype=torch.float32, device=dev)
        d_w_ih = torch.empty((2, G, D), dtype=torch.float32, device=dev)
        db_ih = torch.empty((2, G), dtype=torch.float32, device=dev)
        db_hh = torch.empty((2, G), dtype=torch.float32, device=dev)
        _native.check(lib.vn_lstm_rows_bwd(_p(dh_out), _p(w_hh), _p(act), _p(cprev), _p(cnew), _p(hprev), _p(xc),
                                           _p(start), _p(dG), _p(d_w_hh), _p(d_w_ih), _p(db_ih), _p(db_hh), _p(part),
                                           _p(cnt), _p(_rows_err(dev)), L, B, H, st), "vn_lstm_rows_bwd")
        dx = None
        if need_dx:
            dGf = dG.view(2, L * B, G)
            dx = (dGf[0] @ w_ih_a + dGf[1] @ w_ih_c).view(L, B, D)
        return (dx, None, None, None, None, None, d_w_ih[0], d_w_hh[0], db_ih[0], db_hh[0], d_w_ih[1], d_w_hh[1],
                db_ih[1], db_hh[1])


_ERR = {}


def _rows_err(dev) -> torch.Tensor:
    """The row kernels' device error word (1: an in-launch hand-off timed out)."""
    key = str(dev)
    if key not in _ERR:
        _ERR[key] = torch.zeros(1, dtype=torch.int32, device=dev)
    return _ERR[key]


def rows_err_word(dev):
    """The device error word of the row-layout launches on ``dev`` (None before
    the first one): what the learner's Adam step is gated on."""
    return _ERR.get(str(dev))


def rows_check(dev) -> None:
    """Raise if a row-layout launch on `dev` timed out (one host read)."""
    e = _ERR.get(str(dev))
    if e is not None and int(e.item()) != 0:
        e.zero_()
        raise _native.VoxnavError("row-layout LSTM: an in-launch hand-off timed out (blocks not co-resident?)")


def rows_supported(policy, D: int, B: int) -> bool:
    """Whether the row-layout kernels take this policy / minibatch on this device."""
    la, lc = policy.lstm_actor, policy.lstm_critic
    if la.num_layers != 1 or lc.num_layers != 1 or la.bidirectional or lc.bidirectional or not la.bias:
        return False
    return bool(_native.load().vn_lstm_rows_supported(D, la.hidden_size, B))


def dual_lstm_rows_pair(policy, x: torch.Tensor, env: torch.Tensor, start: torch.Tensor, keep: torch.Tensor,
                        h_store: torch.Tensor, c_store: torch.Tensor) -> torch.Tensor:
    """``dual_lstm_rows`` as one stacked [2, L, B, H] tensor (actor, critic)."""
    la, lc = policy.lstm_actor, policy.lstm_critic
    return _DualLSTMRows.apply(x, env, start, keep, h_store, c_store, la.weight_ih_l0, la.weight_hh_l0, la.bias_ih_l0,
                               la.bias_hh_l0, lc.weight_ih_l0, lc.weight_hh_l0, lc.bias_ih_l0, lc.bias_hh_l0)


def dual_lstm_rows(policy, x: torch.Tensor, env: torch.Tensor, start: torch.Tensor, keep: torch.Tensor,
                   h_store: torch.Tensor, c_store: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(out_actor, out_critic), each [L, B, H], of ``policy.lstm_actor`` /
    ``lstm_critic`` over the row layout (see ``_DualLSTMRows``)."""
    la, lc = policy.lstm_actor, policy.lstm_critic
    out = _DualLSTMRows.apply(x, env, start, keep, h_store, c_store, la.weight_ih_l0, la.weight_hh_l0, la.bias_ih_l0,
                              la.bias_hh_l0, lc.weight_ih_l0, lc.weight_hh_l0, lc.bias_ih_l0, lc.bias_hh_l0)
    return out[0], out[1]


def dual_lstm(policy, x: torch.Tensor, h0: torch.Tensor, c0: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(out_actor, out_critic), each [L, B, H], of ``policy.lstm_actor`` and
    ``policy.lstm_critic`` over x [L, B, D] from states h0, c0 [2, B, H]
    (actor, critic) -- ``nn.LSTM`` semantics, differentiable w.r.t. the
    LSTM parameters."""
    la, lc = policy.lstm_actor, policy.lstm_critic
    if x.device.type != "cuda":
        out_pi, _ = la(x, (h0[0:1].contiguous(), c0[0:1].contiguous()))
        out_vf, _ = lc(x, (h0[1:2].contiguous(), c0[1:2].contiguous()))
        return out_pi, out_vf
    if la.num_layers != 1 or lc.num_layers != 1 or la.bidirectional or lc.bidirectional or not la.bias:
        raise ValueError("dual_lstm supports one-layer unidirectional LSTMs with biases")
    out = _DualLSTM.apply(x, h0, c0, la.weight_ih_l0, la.weight_hh_l0, la.bias_ih_l0, la.bias_hh_l0,
                          lc.weight_ih_l0, lc.weight_hh_l0, lc.bias_ih_l0, lc.bias_hh_l0)
    return out[0], out[1]
