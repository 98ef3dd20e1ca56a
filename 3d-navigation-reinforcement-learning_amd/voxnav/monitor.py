"""Episode statistics: the SB3 ``Monitor`` every training worker is wrapped
in (train/Grid_Train.py:125), for N agents on the device.

SB3's ``Monitor.step`` appends each step's reward to a list and, when the
episode ends (terminated or truncated), emits
``info["episode"] = {"r": round(sum(rewards), 6), "l": len(rewards),
"t": round(time.time() - t_start, 6)}``; ``OnPolicyAlgorithm`` keeps the
last 100 of those (``ep_info_buffer``, in step order, workers in index
order within a step) and logs ``rollout/ep_rew_mean`` / ``ep_len_mean``
as their means.

Here the running return (f64, summed in step order from 0 exactly as the
Python ``sum``) and length live on the device per agent; ``vn_monitor_step``
(csrc/voxnav_collect.hip) updates them after every env step and writes the
finished episodes of that step into row t of a [T, N] record buffer.  At
the rollout's end ``harvest`` pulls the finished episodes in (step, agent)
order -- SB3's order -- into ``ep_info_buffer``.

Build-defined: ``t`` is the wall time since the monitor started at the end
of the rollout step that finished the episode, interpolated linearly over
the rollout (the device does not read the clock per step).
"""
from __future__ import annotations

import ctypes as C
import time
from collections import deque
from typing import Dict, Optional

import numpy as np
import torch

from . import _native


def _p(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


class EpisodeMonitor:
    def __init__(self, lib, n_agents: int, n_steps: int, device, info_buffer: int = 100):
        self.lib = lib
        self.N = int(n_agents)
        self.T = int(n_steps)
        self.device = device
        z = lambda *s, dt: torch.zeros(s, dtype=dt, device=device)  # noqa: E731
        self.ep_return = z(self.N, dt=torch.float64)
        self.ep_length = z(self.N, dt=torch.int32)
        self.rec_return = z(self.T, self.N, dt=torch.float64)
        self.rec_length = z(self.T, self.N, dt=torch.int32)
        self.t_start = time.time()
        self.ep_info_buffer: deque = deque(maxlen=int(info_buffer))
        self.last_episodes: Dict[str, torch.Tensor] = {}
        self.total_episodes = 0
        self._t0 = None
        self._warm()

    def _warm(self):
        """Run harvest's device ops once on a tiny record with finished
        episodes: ROCm loads a kernel's code object at its first launch
        (measured: ~40 ms for these, which otherwise land in the first rollout
        whose episodes finish)."""
        rr = torch.zeros((2, 3), dtype=torch.float64, device=self.device)
        rl = torch.zeros((2, 3), dtype=torch.int32, device=self.device)
        rl[1, 2] = 4
        rr[1, 2] = 1.5
        idx = torch.nonzero(rl > 0)
        rec = (rr[idx[:, 0], idx[:, 1]], rl[idx[:, 0], idx[:, 1]])
        rec[0][0:].tolist(), rec[1][0:].tolist(), idx[:, 0][0:].tolist()

    def begin(self):
        self._t0 = time.time()

    def step(self, t: int, terminated: torch.Tensor, truncated: torch.Tensor, reward64: Optional[torch.Tensor] = None,
             reward: Optional[torch.Tensor] = None):
        """After env step t of the rollout: accumulate and record (stream-ordered)."""
        s = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        _native.check(self.lib.vn_monitor_step(_p(reward64), _p(reward), _p(terminated), _p(truncated), self.N,
                                               _p(self.ep_return), _p(self.ep_length), _p(self.rec_return[t]),
                                               _p(self.rec_length[t]), s), "vn_monitor_step")

    def harvest(self, steps: Optional[int] = None) -> Dict[str, torch.Tensor]:
        """Finished episodes of the rollout's first ``steps`` rows in SB3's
        order, as device tensors ``return`` (exact f64 sum), ``length``,
        ``step`` (rollout row) and ``agent``; the last ``maxlen`` of them join
        ``ep_info_buffer`` as SB3 info dicts."""
        T = self.T if steps is None else int(steps)
        t1 = time.time()
        t0 = self._t0 if self._t0 is not None else t1
        lens = self.rec_length[:T]
        idx = torch.nonzero(lens > 0)                      # row-major: (step, agent) order
        rec = {"return": self.rec_return[:T][idx[:, 0], idx[:, 1]], "length": lens[idx[:, 0], idx[:, 1]],
               "step": idx[:, 0], "agent": idx[:, 1]}
        n = int(idx.shape[0])
        self.total_episodes += n
        self.last_episodes = rec
        keep = min(n, self.ep_info_buffer.maxlen)
        if keep:
            rs = rec["return"][n - keep:].tolist()
            ls = rec["length"][n - keep:].tolist()
            ks = rec["step"][n - keep:].tolist()
            for r, l, k in zip(rs, ls, ks):
                when = t0 + (t1 - t0) * (k + 1) / T
                self.ep_info_buffer.append({"r": round(r, 6), "l": int(l), "t": round(when - self.t_start, 6)})
        return rec

    def ep_rew_mean(self) -> Optional[float]:
        if not self.ep_info_buffer:
            return None
        return float(np.mean([e["r"] for e in self.ep_info_buffer]))     # SB3 safe_mean

    def ep_len_mean(self) -> Optional[float]:
        if not self.ep_info_buffer:
            return None
        return float(np.mean([e["l"] for e in self.ep_info_buffer]))
