"""CPU oracle for the rollout collector -- TEST INFRASTRUCTURE ONLY.

Only ``tests/`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module; the product (``voxnav.collector``) never does.

Restates, in float64 numpy, the third-party pieces the reference's training
loop runs per step (sb3_contrib and SB3 are not
installed and not vendored, so this restatement is "parity unpinned" by the
reference -- it is pinned by known-answer tests in tests/test_collector.py
and by the torch fp32 module it mirrors):

* ``RecurrentActorCriticPolicy.forward``: states *= (1 - episode_start);
  actor and critic LSTM steps (torch gate order i, f, g, o); Tanh MLPs;
  action_net / value_net; Categorical log-probs (log-softmax)
* ``RecurrentPPO.collect_rollouts``: truncation bootstrap
  ``r += gamma * V(terminal_obs; critic state after the step)`` for
  ``done and TimeLimit.truncated`` (= truncated and not terminated), buffer
  of (obs, action, reward, episode_start, value, log_prob), last values
  under ``episode_starts = dones``
* the build-defined Categorical draw: Philox4x32-10(key=sample_seed,
  counter=(gid, t | 2^63)) word 0 -> u = (w >> 8) / 2^24, first a with
  u < cdf[a]

The env part is replayed through ``oracle.OracleEnv.run_random`` with the
actions under test, so the env comparison stays bit-exact while the float
comparisons carry a tolerance.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np

from .oracle import philox4x32_10


def _sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


class PolicyOracle:
    """float64 forward of the SB3 (Recurrent)ActorCriticPolicy parameters."""

    def __init__(self, weights: Dict[str, np.ndarray]):
        self.w = {k: np.asarray(v, np.float64) for k, v in weights.items()}
        self.recurrent = "lstm_actor.weight_ih_l0" in self.w
        self.H = self.w["lstm_actor.weight_hh_l0"].shape[1] if self.recurrent else 0

    def _lstm(self, name, x, h, c):
        w = self.w
        pre = (x @ w[f"{name}.weight_ih_l0"].T + h @ w[f"{name}.weight_hh_l0"].T
               + w[f"{name}.bias_ih_l0"] + w[f"{name}.bias_hh_l0"])
        H = h.shape[-1]
        i, f, g, o = (pre[:, k * H:(k + 1) * H] for k in range(4))
        c2 = _sigmoid(f) * c + _sigmoid(i) * np.tanh(g)
        h2 = _sigmoid(o) * np.tanh(c2)
        return h2, c2

    def _mlp(self, branch, x):
        k = 0
        while f"mlp_extractor.{branch}.{k}.weight" in self.w:
            x = np.tanh(x @ self.w[f"mlp_extractor.{branch}.{k}.weight"].T + self.w[f"mlp_extractor.{branch}.{k}.bias"])
            k += 2
        return x

    def forward(self, obs, h=None, c=None, episode_starts=None):
        """-> (logits [N, A], values [N], h' [2, N, H], c' [2, N, H])."""
        obs = np.asarray(obs, np.float64)
        if self.recurrent:
            m = (1.0 - np.asarray(episode_starts, np.float64))[None, :, None]
            h, c = h * m, c * m
            hp, cp = self._lstm("lstm_actor", obs, h[0], c[0])
            hv, cv = self._lstm("lstm_critic", obs, h[1], c[1])
            xp, xv = hp, hv
            h2, c2 = np.stack([hp, hv]), np.stack([cp, cv])
        else:
            xp = xv = obs
            h2 = c2 = None
        lp, lv = self._mlp("policy_net", xp), self._mlp("value_net", xv)
        logits = lp @ self.w["action_net.weight"].T + self.w["action_net.bias"]
        values = (lv @ self.w["value_net.weight"].T + self.w["value_net.bias"])[:, 0]
        return logits, values, h2, c2

    def predict_values(self, obs, h_vf=None, c_vf=None):
        """Critic only, from the critic state (no masking)."""
        obs = np.asarray(obs, np.float64)
        if self.recurrent:
            x, _ = self._lstm("lstm_critic", obs, h_vf, c_vf)
        else:
            x = obs
        lv = self._mlp("value_net", x)
        return (lv @ self.w["value_net.weight"].T + self.w["value_net.bias"])[:, 0]


def log_softmax(logits):
    m = logits.max(axis=1, keepdims=True)
    return logits - (m + np.log(np.exp(logits - m).sum(axis=1, keepdims=True)))


def sample_uniform(seed: int, gid: int, t: int) -> float:
    hi = (int(t) | (1 << 63)) & ((1 << 64) - 1)
    ctr = [gid & 0xFFFFFFFF, (gid >> 32) & 0xFFFFFFFF, hi & 0xFFFFFFFF, hi >> 32]
    key = [seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF]
    w = int(philox4x32_10(ctr, key)[0])
    return (w >> 8) / 16777216.0


def categorical_draw(logp_row: np.ndarray, u: float):
    """First a with u < cdf[a] (last action if none); also the distance of u
    to the nearest cdf boundary (how close the draw was to flipping)."""
    p = np.exp(logp_row)
    cdf = np.cumsum(p)
    A = len(p)
    act = A - 1
    for a in range(A - 1):
        if u < cdf[a]:
            act = a
            break
    margin = float(np.min(np.abs(cdf[:A - 1] - u))) if A > 1 else 1.0
    return act, margin


def collect(policy: PolicyOracle, env_rollout: dict, obs0: np.ndarray, starts0: np.ndarray, actions: np.ndarray,
            gamma: float = 0.99, h0: Optional[np.ndarray] = None, c0: Optional[np.ndarray] = None,
            sample_seed: int = 42, t0: int = 0, gid_base: int = 0):
    """Replay one rollout: env outputs (from OracleEnv.run_random with
    ``actions`` and ``terminal_obs=True``) + the policy in float64.

    Returns dict(values, log_probs, rewards (bootstrapped, f32 arithmetic as
    SB3), episode_starts, last_values, dones, oracle_actions, margins,
    h, c (final states))."""
    T, N = actions.shape
    obs_seq = np.concatenate([obs0[None], env_rollout["obs"]], 0)
    te, tr = env_rollout["terminated"].astype(bool), env_rollout["truncated"].astype(bool)
    H = policy.H
    h = np.zeros((2, N, H)) if h0 is None else np.asarray(h0, np.float64)
    c = np.zeros((2, N, H)) if c0 is None else np.asarray(c0, np.float64)
    starts = np.zeros((T + 1, N), np.float32)
    starts[0] = starts0
    values = np.zeros((T, N))
    logps = np.zeros((T, N))
    rewards = env_rollout["reward"].astype(np.float32).copy()   # VecEnv buf_rews is float32
    oacts = np.zeros((T, N), np.int32)
    margins = np.zeros((T, N))
    for t in range(T):
        logits, v, h2, c2 = policy.forward(obs_seq[t], h, c, starts[t])
        lsm = log_softmax(logits)
        values[t] = v
        logps[t] = lsm[np.arange(N), actions[t]]
        for n in range(N):
            oacts[t, n], margins[t, n] = categorical_draw(lsm[n], sample_uniform(sample_seed, gid_base + n, t0 + t))
        if policy.recurrent:
            h, c = h2, c2
        boot = tr[t] & ~te[t]
        if boot.any():
            idx = np.nonzero(boot)[0]
            tv = policy.predict_values(env_rollout["terminal_obs"][t][idx],
                                       h[1][idx] if policy.recurrent else None,
                                       c[1][idx] if policy.recurrent else None)
            gv = (np.float32(gamma) * tv.astype(np.float32)).astype(np.float32)
            rewards[t, idx] = (rewards[t, idx] + gv).astype(np.float32)
        done = te[t] | tr[t]
        starts[t + 1] = done
        if policy.recurrent:
            m = (~done)[None, :, None]
            h, c = h * m, c * m
    last_values = policy.predict_values(obs_seq[T], h[1] if policy.recurrent else None,
                                        c[1] if policy.recurrent else None)
    return dict(values=values, log_probs=logps, rewards=rewards, episode_starts=starts[:T], last_values=last_values,
                dones=starts[T], oracle_actions=oacts, margins=margins, h=h, c=c)


def gae64(rewards, values, episode_starts, last_values, dones, gamma=0.99, gae_lambda=0.95):
    """SB3 compute_returns_and_advantage (Appendix D.2) in float64."""
    T, N = rewards.shape
    adv = np.zeros((T, N))
    last = np.zeros(N)
    for t in range(T - 1, -1, -1):
        if t == T - 1:
            nnt, nv = 1.0 - dones, last_values
        else:
            nnt, nv = 1.0 - episode_starts[t + 1], values[t + 1]
        delta = rewards[t] + gamma * nv * nnt - values[t]
        last = delta + gamma * gae_lambda * nnt * last
        adv[t] = last
    return adv, adv + values
