#!/usr/bin/env python3
"""Learner throughput: one PPO-LSTM rollout (collector) then timed PPO
minibatch updates on it.  python scripts/ppo_bench.py --agents 16384 --batch 16384"""
import argparse
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "3d-navigation-reinforcement-learning_amd"))
sys.path.insert(0, str(REPO))
import torch  # noqa: E402

from voxnav.collector import RolloutCollector  # noqa: E402
from voxnav.env import BatchedGridEnv  # noqa: E402
from voxnav.policy import ActorCriticPolicy, RecurrentActorCriticPolicy  # noqa: E402
from voxnav.ppo import PPOLearner  # noqa: E402
from voxnav.rooms import load_archive_set  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, default=16384)
    ap.add_argument("--T", type=int, default=128)
    ap.add_argument("--batch", default="4096,16384")
    ap.add_argument("--minibatches", type=int, default=24)
    ap.add_argument("--policy", default="lstm")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    pol = (RecurrentActorCriticPolicy() if a.policy == "lstm" else ActorCriticPolicy()).to(dev)
    env = BatchedGridEnv(num_agents=a.agents, rooms=load_archive_set("P3_training"), local_map_length=10,
                         autoreset=True, device=dev)
    col = RolloutCollector(env, pol, n_steps=a.T)
    buf = col.collect()
    torch.cuda.synchronize()
    from bench import lstm_flops_per_agent_step, mlp_flops_per_agent_step
    fwd = lstm_flops_per_agent_step() if a.policy == "lstm" else mlp_flops_per_agent_step()
    for B in map(int, a.batch.split(",")):
        ln = PPOLearner(pol, n_epochs=1, batch_size=B, seed=0)
        total = a.T * a.agents
        nmb = min(a.minibatches, total // B)
        split = 12345 % total
        # time individual minibatches through the learner's internals
        idx_all = torch.roll(torch.arange(total, device=dev), -split)
        ln.optimizer.zero_grad()
        ln.update_many(buf, [idx_all[w * B:(w + 1) * B] for w in range(2)], windows=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ln.update_many(buf, [idx_all[m * B:(m + 1) * B] for m in range(nmb)], windows=True)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        sps = nmb * B / el
        print(f"policy={a.policy} batch={B}: {el / nmb * 1e3:.2f} ms/minibatch, {sps / 1e6:.3f} M samples/s, "
              f"~{3 * fwd * sps / 1e12:.2f} TFLOP/s (fwd+bwd = 3x fwd)", flush=True)


def _one(ln, buf, idx):
    ln.update(buf, idx)


if __name__ == "__main__":
    main()
