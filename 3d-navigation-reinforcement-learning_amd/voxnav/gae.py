"""GAE advantage/return scan on the GPU (vn_gae).

Restates SB3 ``RolloutBuffer.compute_returns_and_advantage`` (third-party,
reached from ``model.learn`` at train/Grid_Train.py:228; Grid_Train's
gamma=0.99, gae_lambda=0.95 at :84-85) in float32 with numpy's operation
order:  delta = r + (g*V' )*nnt - V ;  A = delta + ((g*l)*nnt)*A' ;  R = A + V.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _native


def compute_gae(rewards: torch.Tensor, values: torch.Tensor, episode_starts: torch.Tensor,
                last_values: torch.Tensor, dones: torch.Tensor, gamma: float = 0.99, gae_lambda: float = 0.95):
    """All inputs f32 on one GPU; rewards/values/episode_starts [T, N], last_values/dones [N].

    Returns (advantages, returns), both f32 [T, N].
    """
    lib = _native.load()
    dev = rewards.device
    if dev.type != "cuda":
        raise ValueError("compute_gae expects GPU tensors")
    T, N = rewards.shape
    f = lambda t: t.to(device=dev, dtype=torch.float32).contiguous()  # noqa: E731
    r, v, s, lv, d = f(rewards), f(values), f(episode_starts), f(last_values).reshape(N), f(dones).reshape(N)
    if v.shape != (T, N) or s.shape != (T, N):
        raise ValueError("values / episode_starts must be [T, N] like rewards")
    adv = torch.empty((T, N), dtype=torch.float32, device=dev)
    ret = torch.empty((T, N), dtype=torch.float32, device=dev)
    p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    with torch.cuda.device(dev):
        _native.check(lib.vn_gae(p(r), p(v), p(s), p(lv), p(d), int(T), int(N), float(gamma), float(gae_lambda),
                                 p(adv), p(ret), stream), "vn_gae")
    return adv, ret
