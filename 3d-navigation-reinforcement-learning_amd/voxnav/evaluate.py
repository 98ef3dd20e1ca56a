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
                               reset_seed=seed, monitor=False)
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


def evals_due(calls_before: int, calls_after: int, eval_freq: int) -> int:
    """How many multiples of ``eval_freq`` the step-call counter crossed
    (SB3 EvalCallback evaluates when ``n_calls % eval_freq == 0``)."""
    if eval_freq <= 0:
        return 0
    return calls_after // eval_freq - calls_before // eval_freq


class EvalCallback:
    """SB3 ``EvalCallback`` as train/Grid_Train.py:218-226 configures it:
    every ``eval_freq`` vectorized env steps (``max(EVAL_FREQ // NUM_ENVS, 1)``
    with EVAL_FREQ = 100_000, :42), ``n_eval_episodes`` deterministic episodes
    on the evaluation rooms; the episode rewards / lengths are logged to
    ``log_path/evaluations.npz`` (``timesteps``, ``results``, ``ep_lengths``)
    and the policy is saved to ``best_model_save_path/best_model.zip``
    whenever the mean reward beats the best so far.

    SB3 calls ``_on_step`` after every vectorized step of the rollout; the
    policy weights do not change inside a rollout (the update comes after
    it), so ``learn`` asks at the rollout's end and the evaluation sees the
    same weights.  Several multiples of ``eval_freq`` inside one rollout
    (eval_freq < n_steps) give one evaluation, logged at the rollout's
    timestep count.  Episode rewards are the Monitor's ``round(sum, 6)``
    (SB3 ``evaluate_policy`` reads them from the Monitor); episodes run
    side by side with seeds ``seed + n_evals * n_eval_episodes + i``.
    """

    def __init__(self, eval_rooms, eval_freq: int, n_eval_episodes: int = 10, deterministic: bool = True,
                 best_model_save_path=None, log_path=None, local_map_length: int = 10, seed: int = 1_000_000,
                 crash_penalty: float = -2.0, device=None, verbose: int = 0):
        self.rooms = eval_rooms
        self.eval_freq = int(eval_freq)
        self.n_eval_episodes = int(n_eval_episodes)
        self.deterministic = bool(deterministic)
        self.best_model_save_path = best_model_save_path
        self.log_path = log_path
        self.local_map_length = int(local_map_length)
        self.seed = int(seed)
        self.crash_penalty = float(crash_penalty)
        self.device = device
        self.verbose = int(verbose)
        self.n_calls = 0
        self.best_mean_reward = float("-inf")
        self.last_mean_reward = float("-inf")
        self.evaluations_timesteps: List[int] = []
        self.evaluations_results: List[List[float]] = []
        self.evaluations_length: List[List[int]] = []

    def on_rollout_end(self, policy, num_timesteps: int, n_steps: int, optimizer=None) -> Optional[Dict[str, float]]:
        before = self.n_calls
        self.n_calls += int(n_steps)
        if evals_due(before, self.n_calls, self.eval_freq) == 0:
            return None
        import numpy as np
        dev = self.device if self.device is not None else next(policy.parameters()).device
        r = evaluate_policy(policy, self.rooms, n_episodes=self.n_eval_episodes,
                            local_map_length=self.local_map_length,
                            seed=self.seed + len(self.evaluations_timesteps) * self.n_eval_episodes, device=dev,
                            crash_penalty=self.crash_penalty, deterministic=self.deterministic)
        rewards = [round(e["score"], 6) for e in r["episodes"]]
        lengths = [int(e["steps"]) for e in r["episodes"]]
        self.evaluations_timesteps.append(int(num_timesteps))
        self.evaluations_results.append(rewards)
        self.evaluations_length.append(lengths)
        if self.log_path is not None:
            from pathlib import Path
            Path(self.log_path).mkdir(parents=True, exist_ok=True)
            np.savez(Path(self.log_path) / "evaluations.npz", timesteps=np.asarray(self.evaluations_timesteps),
                     results=np.asarray(self.evaluations_results), ep_lengths=np.asarray(self.evaluations_length))
        mean, std = float(np.mean(rewards)), float(np.std(rewards))
        mean_len = float(np.mean(lengths))
        self.last_mean_reward = mean
        new_best = mean > self.best_mean_reward
        if self.verbose:
            print(f"Eval num_timesteps={num_timesteps}, episode_reward={mean:.2f} +/- {std:.2f}")
            print(f"Episode length: {mean_len:.2f} +/- {float(np.std(lengths)):.2f}")
        if new_best:
            self.best_mean_reward = mean
            if self.best_model_save_path is not None:
                from pathlib import Path
                from .checkpoint import save_checkpoint
                save_checkpoint(Path(self.best_model_save_path) / "best_model.zip", policy, optimizer,
                                num_timesteps=num_timesteps)
        return {"eval/mean_reward": mean, "eval/std_reward": std, "eval/mean_ep_length": mean_len,
                "eval/new_best": new_best}
