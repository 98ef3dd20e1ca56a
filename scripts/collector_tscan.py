#!/usr/bin/env python3
"""Marginal per-step cost of the PPO-LSTM collector (C4 shape) vs its
per-rollout fixed cost: wall time of collect() at two rollout lengths."""
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "3d-navigation-reinforcement-learning_amd"))
import torch  # noqa: E402

from voxnav.collector import RolloutCollector  # noqa: E402
from voxnav.env import BatchedGridEnv  # noqa: E402
from voxnav.policy import RecurrentActorCriticPolicy  # noqa: E402
from voxnav.rooms import load_archive_set  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
dev = "cuda:0"
res = {}
for T in (64, 192):
    torch.manual_seed(42)
    pol = RecurrentActorCriticPolicy().to(dev)
    env = BatchedGridEnv(num_agents=N, rooms=load_archive_set("P3_training"), local_map_length=10, autoreset=True,
                         device=dev)
    col = RolloutCollector(env, pol, n_steps=T, sample_seed=42, reset_seed=42)
    col.collect()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(2):
        col.collect()
    torch.cuda.synchronize()
    res[T] = (time.perf_counter() - t0) / 2
    env.close()
    del col, env, pol
    torch.cuda.empty_cache()
step = (res[192] - res[64]) / 128
print(json.dumps({"rollout_s": {str(k): round(v, 5) for k, v in res.items()}, "marginal_ms_per_step": round(step * 1e3, 4),
                  "per_rollout_fixed_ms": round((res[64] - 64 * step) * 1e3, 3)}))
