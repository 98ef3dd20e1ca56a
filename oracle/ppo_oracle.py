"""CPU oracle for the PPO learner -- TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module; the product (``voxnav.ppo``) never
does.

Restates, in float64 on the CPU, the training step the reference runs
through ``model.learn`` (train/Grid_Train.py:228) with the hyperparameters
of train/Grid_Train.py:84-86 (lr 3e-4, batch_size 64, n_epochs 10, clip
0.2, ent_coef 0.01, vf_coef 0.5; SB3 defaults max_grad_norm 0.5,
normalize_advantage True, Adam eps 1e-5).  The algorithm lives in
third-party packages that are not installed and not vendored here
(sb3_contrib ``RecurrentPPO.train`` + ``RecurrentRolloutBuffer.get`` /
``_get_samples`` + ``create_sequencers`` / ``pad`` / ``pad_and_flatten``
+ ``RecurrentActorCriticPolicy.evaluate_actions`` / ``_process_sequence``;
SB3 ``PPO.train`` + ``RolloutBuffer.get`` for the feed-forward policy), so
this restatement follows their published code structure and is **parity
unpinned** by the reference; tests pin it with
hand-computed sequencer cases and invariants.

Deliberately written the way sb3_contrib writes it: the minibatch is cut
from the env-major flattened buffer, split into sequences at episode starts
and env changes, padded (numpy), and the LSTM is stepped one position at a
time with the ``(1 - episode_start)`` state mask; Adam and the grad-norm
clip are written out by hand.  Gradients come from torch autograd in
float64 (a generic tool, not the algorithm under test).

Minibatch order: sb3 draws ``split_index`` (recurrent) or a permutation
(feed-forward) from the global numpy generator per epoch; here they are
arguments, so the product learner and the oracle use the same ones.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import torch

F64 = torch.float64


# ---------------------------------------------------------------- sequencers
def swap_and_flatten(arr: np.ndarray) -> np.ndarray:
    """(n_steps, n_envs, ...) -> (n_envs * n_steps, ...) keeping each env's
    steps contiguous (sb3 ``BaseBuffer.swap_and_flatten``)."""
    shape = arr.shape
    if len(shape) < 3:
        shape = shape + (1,)
    return arr.swapaxes(0, 1).reshape(shape[0] * shape[1], *shape[2:])


def create_sequencers(episode_starts: np.ndarray, env_change: np.ndarray):
    """sb3_contrib ``create_sequencers``: (seq_start_indices, seq_end_indices)."""
    seq_start = np.logical_or(episode_starts, env_change).flatten()
    seq_start[0] = True
    seq_start_indices = np.where(seq_start)[0]
    seq_end_indices = np.concatenate([(seq_start_indices - 1)[1:], np.array([len(episode_starts)])])
    return seq_start_indices, seq_end_indices


def pad(starts, ends, tensor: np.ndarray, padding_value: float = 0.0) -> np.ndarray:
    """sb3_contrib ``pad`` (``pad_sequence(batch_first=True)``)."""
    seqs = [tensor[s:e + 1] for s, e in zip(starts, ends)]
    n, m = len(seqs), max(len(q) for q in seqs)
    out = np.full((n, m) + tensor.shape[1:], padding_value, dtype=np.float64)
    for i, q in enumerate(seqs):
        out[i, :len(q)] = q
    return out


def pad_and_flatten(starts, ends, tensor: np.ndarray) -> np.ndarray:
    return pad(starts, ends, tensor).reshape(-1)


# ---------------------------------------------------------------- policy
def _lstm_step(w, name, x, h, c):
    pre = (x @ w[f"{name}.weight_ih_l0"].T + h @ w[f"{name}.weight_hh_l0"].T
           + w[f"{name}.bias_ih_l0"] + w[f"{name}.bias_hh_l0"])
    H = h.shape[-1]
    i, f, g, o = (pre[:, k * H:(k + 1) * H] for k in range(4))
    c2 = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(g)
    return torch.sigmoid(o) * torch.tanh(c2), c2


def _process_sequence(w, name, features, h0, c0, episode_starts, n_seq):
    """sb3_contrib ``_process_sequence`` (the masked per-step loop)."""
    fs = features.reshape(n_seq, -1, features.shape[-1]).swapaxes(0, 1)       # (L, n_seq, F)
    es = episode_starts.reshape(n_seq, -1).swapaxes(0, 1)                      # (L, n_seq)
    h, c = h0, c0
    outs = []
    for x, e in zip(fs, es):
        m = (1.0 - e).view(n_seq, 1)
        h, c = _lstm_step(w, name, x, m * h, m * c)
        outs.append(h)
    return torch.stack(outs, 0).transpose(0, 1).reshape(-1, h.shape[-1])


def _mlp(w, branch, x):
    k = 0
    while f"mlp_extractor.{branch}.{k}.weight" in w:
        x = torch.tanh(x @ w[f"mlp_extractor.{branch}.{k}.weight"].T + w[f"mlp_extractor.{branch}.{k}.bias"])
        k += 2
    return x


def evaluate_actions(w, obs, actions, lstm=None, episode_starts=None, n_seq=None):
    """-> values, log_prob, entropy (Categorical)."""
    if lstm is not None:
        (hp, cp), (hv, cv) = lstm
        lat_pi = _process_sequence(w, "lstm_actor", obs, hp, cp, episode_starts, n_seq)
        lat_vf = _process_sequence(w, "lstm_critic", obs, hv, cv, episode_starts, n_seq)
    else:
        lat_pi = lat_vf = obs
    logits = _mlp(w, "policy_net", lat_pi) @ w["action_net.weight"].T + w["action_net.bias"]
    values = (_mlp(w, "value_net", lat_vf) @ w["value_net.weight"].T + w["value_net.bias"]).flatten()
    logp_all = torch.log_softmax(logits, dim=-1)
    log_prob = logp_all.gather(1, actions.view(-1, 1)).flatten()
    entropy = -(logp_all.exp() * logp_all).sum(-1)
    return values, log_prob, entropy


# ---------------------------------------------------------------- optimizer
class Adam:
    """torch.optim.Adam (amsgrad off, no weight decay), written out."""

    def __init__(self, names: List[str], lr: float, eps: float = 1e-5, betas=(0.9, 0.999)):
        self.lr, self.eps, (self.b1, self.b2) = lr, eps, betas
        self.m = {k: None for k in names}
        self.v = {k: None for k in names}
        self.t = 0

    def step(self, params: Dict[str, torch.Tensor], grads: Dict[str, torch.Tensor]):
        self.t += 1
        bc1 = 1.0 - self.b1 ** self.t
        bc2 = 1.0 - self.b2 ** self.t
        for k, g in grads.items():
            if self.m[k] is None:
                self.m[k] = torch.zeros_like(g)
                self.v[k] = torch.zeros_like(g)
            self.m[k] = self.b1 * self.m[k] + (1.0 - self.b1) * g
            self.v[k] = self.b2 * self.v[k] + (1.0 - self.b2) * g * g
            denom = self.v[k].sqrt() / np.sqrt(bc2) + self.eps
            params[k] = params[k] - (self.lr / bc1) * self.m[k] / denom


def clip_grad_norm(grads: Dict[str, torch.Tensor], max_norm: float):
    total = torch.sqrt(sum((g * g).sum() for g in grads.values()))
    coef = min(1.0, float(max_norm / (total + 1e-6)))
    return {k: g * coef for k, g in grads.items()}, float(total)


# ---------------------------------------------------------------- train
def train(weights: Dict[str, np.ndarray], buf: Dict[str, np.ndarray], epoch_orders: List[np.ndarray], *,
          learning_rate=3e-4, batch_size=64, clip_range=0.2, ent_coef=0.01, vf_coef=0.5, max_grad_norm=0.5,
          normalize_advantage=True, adam: Optional[Adam] = None):
    """One ``train()`` call.

    ``buf``: numpy [T, N]-major arrays obs, actions, episode_starts, values,
    log_probs, advantages, returns, and for the recurrent policy lstm_h /
    lstm_c [T, 2, N, H] (states entering step t before the mask).
    ``epoch_orders``: per epoch the split index (recurrent, an int) or the
    index permutation (feed-forward).
    Returns (new weights, stats list per minibatch, adam)."""
    w = {k: torch.tensor(np.asarray(v), dtype=F64) for k, v in weights.items()}
    recurrent = "lstm_actor.weight_ih_l0" in w
    T, N = buf["actions"].shape
    total = T * N
    flat = {k: swap_and_flatten(np.asarray(buf[k], np.float64)) for k in
            ("obs", "actions", "episode_starts", "values", "log_probs", "advantages", "returns")}
    if recurrent:
        # (T, 2, N, H) -> per branch (T, N, H) -> (N*T, H)
        hs = {b: swap_and_flatten(np.asarray(buf["lstm_h"], np.float64)[:, b]) for b in (0, 1)}
        cs = {b: swap_and_flatten(np.asarray(buf["lstm_c"], np.float64)[:, b]) for b in (0, 1)}
        env_change = np.zeros((T, N))
        env_change[0, :] = 1.0
        env_change = swap_and_flatten(env_change).reshape(-1)
    names = list(w.keys())
    adam = adam or Adam(names, learning_rate)
    stats = []
    for order in epoch_orders:
        if recurrent:
            split = int(order)
            indices = np.arange(total)
            indices = np.concatenate((indices[split:], indices[:split]))
        else:
            indices = np.asarray(order)
        start = 0
        while start < total:
            bi = indices[start:start + batch_size]
            start += batch_size
            if recurrent:
                st, en = create_sequencers(flat["episode_starts"][bi].reshape(-1), env_change[bi])
                n_seq = len(st)
                P = lambda a: pad(st, en, a)  # noqa: E731
                PF = lambda a: pad_and_flatten(st, en, a.reshape(-1))  # noqa: E731
                obs = torch.tensor(P(flat["obs"][bi]).reshape(-1, flat["obs"].shape[-1]))
                acts = torch.tensor(P(flat["actions"][bi].reshape(-1)).reshape(-1)).long()
                old_lp = torch.tensor(PF(flat["log_probs"][bi]))
                adv = torch.tensor(PF(flat["advantages"][bi]))
                ret = torch.tensor(PF(flat["returns"][bi]))
                starts = torch.tensor(PF(flat["episode_starts"][bi]))
                mask = torch.tensor(PF(np.ones(len(bi)))) > 1e-8
                lstm = tuple((torch.tensor(hs[b][bi][st]), torch.tensor(cs[b][bi][st])) for b in (0, 1))
            else:
                n_seq = None
                obs = torch.tensor(flat["obs"][bi])
                acts = torch.tensor(flat["actions"][bi].reshape(-1)).long()
                old_lp = torch.tensor(flat["log_probs"][bi].reshape(-1))
                adv = torch.tensor(flat["advantages"][bi].reshape(-1))
                ret = torch.tensor(flat["returns"][bi].reshape(-1))
                starts = None
                mask = torch.ones(len(bi), dtype=torch.bool)
                lstm = None
            params = {k: v.clone().requires_grad_(True) for k, v in w.items()}
            values, log_prob, entropy = evaluate_actions(params, obs, acts, lstm, starts, n_seq)
            if normalize_advantage and (recurrent or len(adv) > 1):
                adv = (adv - adv[mask].mean()) / (adv[mask].std() + 1e-8)
            ratio = torch.exp(log_prob - old_lp)
            l1 = adv * ratio
            l2 = adv * torch.clamp(ratio, 1 - clip_range, 1 + clip_range)
            policy_loss = -torch.mean(torch.min(l1, l2)[mask])
            value_loss = torch.mean(((ret - values) ** 2)[mask])
            entropy_loss = -torch.mean(entropy[mask])
            loss = policy_loss + ent_coef * entropy_loss + vf_coef * value_loss
            with torch.no_grad():
                log_ratio = log_prob - old_lp
                approx_kl = torch.mean(((torch.exp(log_ratio) - 1) - log_ratio)[mask])
                clip_frac = torch.mean((torch.abs(ratio - 1) > clip_range).double()[mask])
            grads = torch.autograd.grad(loss, [params[k] for k in names], allow_unused=True)
            grads = {k: (g if g is not None else torch.zeros_like(w[k])) for k, g in zip(names, grads)}
            grads, gnorm = clip_grad_norm(grads, max_grad_norm)
            adam.step(w, grads)
            stats.append(dict(policy_loss=float(policy_loss.detach()), value_loss=float(value_loss.detach()),
                              entropy_loss=float(entropy_loss.detach()), loss=float(loss.detach()),
                              approx_kl=float(approx_kl),
                              clip_fraction=float(clip_frac), grad_norm=gnorm, n_seq=n_seq or 0))
    return {k: v.numpy() for k, v in w.items()}, stats, adam
