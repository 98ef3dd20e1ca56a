"""Agent sharding across GPUs (one process per GPU, torch.distributed).

The reference runs one env per OS process (train/Grid_Train.py:191-192);
agents never interact.  Here GPU ``rank`` of ``world`` owns global agents
``[rank * n_local, (rank + 1) * n_local)``; seeds and the random-policy
stream are keyed by the global agent id, so the union of the shards is
bitwise identical to a single-GPU run over the same ids.  The env step has
NO collective.  The only data exchange is at the rollout boundary:
``allgather_rollout`` gathers the trajectory buffers (RCCL over xGMI with
the "nccl" backend; gloo on CPU in tests).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional

import torch
import torch.distributed as dist


@dataclass(frozen=True)
class Shard:
    rank: int
    world: int
    n_local: int

    @property
    def agent_id_base(self) -> int:
        return self.rank * self.n_local

    @property
    def n_global(self) -> int:
        return self.n_local * self.world

    @property
    def seed_stride(self) -> int:
        """Seed increment between consecutive episodes of one agent."""
        return self.n_global


def shard_for(n_local: int, rank: Optional[int] = None, world: Optional[int] = None) -> Shard:
    if rank is None or world is None:
        if dist.is_available() and dist.is_initialized():
            rank, world = dist.get_rank(), dist.get_world_size()
        else:
            rank, world = 0, 1
    return Shard(int(rank), int(world), int(n_local))


def allgather_rollout(buffers: Dict[str, torch.Tensor], agent_dim: int = 1, group=None,
                      flat: bool = True) -> Dict[str, torch.Tensor]:
    """All-gather per-shard trajectory buffers along the agent dimension.

    Each tensor is [T, n_local, ...] (agent dim ``agent_dim``), contiguous.
    One ``all_gather_into_tensor`` per buffer straight from the buffer into
    a [world * T, n_local, ...] output (ranks concatenated: no copy before
    the collective).  The default (``flat=True``) returns [T, n_global, ...]
    in global-id order (one copy after the collective; with one rank the
    buffer itself).  ``flat=False`` skips that copy and returns a zero-copy
    strided view with the rank as a new dimension in front of the agent
    dimension: [T, world, n_local, ...], so ``out[:, r, i]`` is global agent
    ``r * n_local + i`` (the view's C-order bytes are those of the flat
    buffer); the bench's timed gather uses it.  Large
    messages, back to back: the xGMI ring is per-link bound, so few big
    transfers.
    """
    world = dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1
    out = {}
    for name, t in buffers.items():
        if not t.is_contiguous():
            raise ValueError(f"{name}: allgather_rollout gathers contiguous buffers in place")
        if world == 1 and flat:
            out[name] = t
            continue
        if world == 1:
            g = t.unsqueeze(0)
        else:
            g = torch.empty((world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
            dist.all_gather_into_tensor(g.view((world * t.shape[0],) + tuple(t.shape[1:])), t, group=group)
        v = g.movedim(0, agent_dim)                     # [..., world, n_local, ...]
        if flat:
            v = v.reshape(tuple(t.shape[:agent_dim]) + (world * t.shape[agent_dim],) + tuple(t.shape[agent_dim + 1:]))
        out[name] = v
    return out


def max_over_ranks(value: float, device=None, group=None) -> float:
    """Max of a scalar over ranks (the bench's timing rule)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return float(value)
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def reduce_episode_stats(result: Dict[str, object], device=None, group=None) -> Dict[str, object]:
    """Global evaluation averages from per-rank ``evaluate_policy`` results
    (episode statistics by a tiny all-reduce): sums of
    score / bumps / finished / discovered / steps and the episode count are
    summed over ranks (one 6-float all-reduce) and re-averaged.  The local
    per-episode list stays as it is."""
    eps = result["episodes"]
    t = torch.tensor([sum(e["score"] for e in eps), sum(e["bumps"] for e in eps),
                      sum(bool(e["finished"]) for e in eps), sum(e["discovered_cells"] for e in eps),
                      sum(e["steps"] for e in eps), len(eps)], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    s = t.tolist()
    n = max(1.0, s[5])
    out = dict(result)
    out.update(avg_score=s[0] / n, avg_bumps=s[1] / n, finished_pct=100.0 * s[2] / n, avg_discovered=s[3] / n,
               avg_steps=s[4] / n, n_episodes_global=int(s[5]))
    return out
