"""Policy evaluation with the reference's metrics.

Restates train/evaluate_grid.py:180-247 for a batch of episodes run side by
side on the device: each of ``n_episodes`` agents plays one episode with
``model.predict(..., deterministic=True)`` (argmax of the policy logits,
recurrent state starting from zeros at ``episode_start``), and per episode
the script's statistics are recorded --

* ``score``: sum of the step rewards (f64, :202-203)
* ``steps``: steps until ``done or truncated`` (:204)
* ``bumps`` / ``discovered_cells`` / ``finished``: the agent's
  ``bump_count`` / ``visited_count`` / ``done`` when the episode ends
  (:213-215)

and aggregated as the script's text table does: average score, average
bumps, finished %, average discovered cells, average steps (:257-268).
The EvalCallback of train/Grid_Train.py:218-226 (10 deterministic
episodes, best mean reward) is the same call with ``n_episodes=10``.

Episodes are seeded (agent i resets with ``seed + i``) so an evaluation is
reproducible; the reference's evaluation resets draw from the unseeded
global ``random``.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch

from .collector import RolloutCollector
from .env import BatchedGridEnv


@torch.no_grad()
def evaluate_policy(policy, rooms, n_episodes: int = 10, local_map_length: int = 10, seed: int = 0,
                    device="cuda:0", variant: str = "cubic", crash_penalty: float = -2.0,
                    deterministic: bool = True, max_steps: Optional[int] = None,
                    record_actions: bool = False) -> Dict[str, object]:
    """Run ``n_episodes`` episodes in parallel; returns ``{"episodes": [...],
    "avg_score", "avg_bumps", "finished_pct", "avg_discovered", "avg_steps"}``
    (plus ``"actions"`` [steps, n_episodes] when ``record_actions``)."""
    env = BatchedGridEnv(num_agents=n_episodes, rooms=rooms, local_map_length=local_map_length, autoreset=False,
                         device=device, crash_penalty=crash_penalty, variant=variant)
    try:
        col = RolloutCollector(env, policy, n_steps=1, deterministic=deterministic, store_lstm_states=False,
                               reset_seed=seed)
        dev = env.device
        obs = col._obs[0].clone()
        alive = torch.ones(n_episodes, dtype=torch.bool, device=dev)
        score = torch.zeros(n_episodes, dtype=torch.float64, device=dev)
        steps = torch.zeros(n_episodes, dtype=torch.int64, device=dev)
        final = torch.zeros((n_episodes, 3), dtype=torch.int64, device=dev)   # bumps, visited, done
        limit = int(max_steps) if max_steps is not None else int(env.total_free_cells.max()) + 1
        acts: List[torch.Tensor] = []
        for t in range(limit):
            a = col.act(obs)
            if record_actions:
                acts.append(a.clone())
            res = env.step(a, reward_f64=True, terminal_obs=False)
            obs = res.obs
            score += torch.where(alive, res.reward, torch.zeros_like(res.reward))
            steps += alive.to(torch.int64)
            ended = alive & (res.terminated.bool() | res.truncated.bool())
            st = env.export_state()
            final = torch.where(ended.view(-1, 1), st[:, [7, 6, 8]], final)
            alive &= ~ended
            if (t & 63) == 63 and not bool(alive.any()):
                break
        f = final.cpu().tolist()
        sc, sp = score.cpu().tolist(), steps.cpu().tolist()
        eps = [dict(score=sc[i], bumps=f[i][0], discovered_cells=f[i][1], finished=bool(f[i][2]), steps=sp[i])
               for i in range(n_episodes)]
        n = max(1, n_episodes)
        out = dict(episodes=eps,
                   avg_score=sum(e["score"] for e in eps) / n,
                   avg_bumps=sum(e["bumps"] for e in eps) / n,
                   finished_pct=100.0 * sum(e["finished"] for e in eps) / n,
                   avg_discovered=sum(e["discovered_cells"] for e in eps) / n,
                   avg_steps=sum(e["steps"] for e in eps) / n)
        if record_actions:
            out["actions"] = torch.stack(acts).cpu().numpy() if acts else None
        return out
    finally:
        env.close()


RESULTS_HEADER = (f"{'Model Name':<40} | {'Avg Score':>12} | {'Avg Bumps':>12} | {'Finished (%)':>15} | "
                  f"{'Avg Discovered':>18} | {'Avg Steps':>12}")


def results_table_row(name: str, r: Dict[str, object]) -> str:
    """One line of evaluate_grid.py's aggregated text table (header :106,
    row :268)."""
    return (f"{name:<40} | {r['avg_score']:>12.2f} | {r['avg_bumps']:>12.2f} | {r['finished_pct']:>14.1f}% | "
            f"{r['avg_discovered']:>18.2f} | {r['avg_steps']:>12.2f}")
