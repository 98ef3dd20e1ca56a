"""Weight gradients over tall minibatches, split along the sample axis.

The learner's weight gradients are ``dY^T X`` products whose reduction axis
is the minibatch (65,536 samples) and whose outputs are small (256 x 256,
1024 x 256 ...).  As one GEMM, the library tiles only the small output: a
256 x 256 result is 32 workgroups on a 256-CU chip, 240 us per product
(`profiles/r02/learner_native_loops_kernel_stats.csv`).  Cutting the sample
axis into chunks and summing the chunk products gives the GEMM chunks x more
workgroups.  Same math, f32 accumulation, a different summation order (the
parity tests hold it to the f64 oracle's tolerance).

``linear`` is ``F.linear`` with this backward; ``mm_tn`` is ``a^T @ b``.
"""
from __future__ import annotations

import torch

MIN_ROWS = 8192          # below this, one GEMM
CHUNK_ROWS = 2048        # rows per chunk product


def mm_tn(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """``a^T @ b`` for a [K, M], b [K, N] (K the sample axis)."""
    K = a.shape[0]
    c = K // CHUNK_ROWS
    if K < MIN_ROWS or c < 2:
        return a.t() @ b
    main = c * CHUNK_ROWS
    out = torch.bmm(a[:main].reshape(c, CHUNK_ROWS, a.shape[1]).transpose(1, 2),
                    b[:main].reshape(c, CHUNK_ROWS, b.shape[1])).sum(0)
    if main < K:
        out += a[main:].t() @ b[main:]
    return out


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        y = x @ weight.t()
        if bias is not None:
            y += bias
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dy = dy.contiguous()
        dx = dy @ weight if ctx.needs_input_grad[0] else None
        dw = mm_tn(dy, x.contiguous()) if ctx.needs_input_grad[1] else None
        db = dy.sum(0) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return dx, dw, db


def linear(x: torch.Tensor, module: torch.nn.Linear) -> torch.Tensor:
    """``module(x)`` for 2-D x; split-K weight gradient on CUDA tall batches."""
    if x.dim() != 2 or x.device.type != "cuda" or x.shape[0] < MIN_ROWS:
        return module(x)
    return _Linear.apply(x, module.weight, module.bias)


def sequential(seq: torch.nn.Sequential, x: torch.Tensor) -> torch.Tensor:
    """``seq(x)`` with every ``nn.Linear`` through ``linear``."""
    for m in seq:
        x = linear(x, m) if isinstance(m, torch.nn.Linear) else m(x)
    return x
