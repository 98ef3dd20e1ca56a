"""PPO learner on the collector's device buffers.

Restates the update the reference runs through ``model.learn``
(train/Grid_Train.py:228; RecurrentPPO with the hyperparameters of
train/Grid_Train.py:84-86: lr 3e-4, batch_size 64, n_epochs 10, clip 0.2,
ent_coef 0.01, vf_coef 0.5; SB3 defaults max_grad_norm 0.5,
normalize_advantage True, Adam eps 1e-5):

* sb3_contrib ``RecurrentPPO.train`` for ``RecurrentActorCriticPolicy``:
  per epoch the env-major flattened buffer (``swap_and_flatten``) is rolled
  by a random split index and cut into minibatches of ``batch_size``
  samples; each minibatch is split into sequences at episode starts and env
  changes (``create_sequencers``), padded, and both LSTMs are re-run from
  the buffer's stored states at the sequence starts (``_process_sequence``);
  clipped surrogate + value MSE + entropy over the unpadded positions,
  advantages normalised per minibatch, grad-norm clip, Adam.
* SB3 ``PPO.train`` for ``ActorCriticPolicy``: a random permutation per
  epoch, same losses without sequences.

Everything stays on the device: minibatch rows are gathered straight from
the collector's ``[T, N]``-major buffers by index arithmetic (no flattened
copies), sequences are packed with one scatter, and both LSTMs run together
over the padded batch (``voxnav.lstm_seq.dual_lstm``: one fused
matrix-core launch per step, csrc/voxnav_learn_f32.hip, forward and
backward), which equals sb3's masked per-step loop because a sequence can only begin
with an episode start.
The one host round-trip per recurrent minibatch is the (n_seq, max_len)
pair that sizes the padded tensor (none in the row layout,
``voxnav.lstm_seq.dual_lstm_rows``).  From the MLP latents on, the heads,
the advantage normalisation, the three losses and their gradient run in the
fused loss kernel (``learn_ops.ppo_loss``, csrc/voxnav_ppo_loss.hip); the
latents' gradient is backpropagated through the MLP and LSTM kernels.

With ``process_group`` set, gradients are averaged over the ranks (one
flattened all-reduce per minibatch, RCCL over xGMI with the nccl backend)
before the clip -- data-parallel training over agent shards.

The minibatch order is drawn from ``numpy.random.default_rng(seed)``
(sb3 uses the global numpy generator) or passed explicitly as
``epoch_orders`` (what the parity tests do with ``oracle/ppo_oracle.py``).
"""
from __future__ import annotations

import os
from contextlib import nullcontext as _nullctx
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as Fn

from . import learn_ops, lstm_seq
from .lstm_seq import dual_lstm
from .policy import ActorCriticPolicy, RecurrentActorCriticPolicy


class PPOLearner:
    def __init__(self, policy, learning_rate: float = 3e-4, n_epochs: int = 10, batch_size: int = 64,
                 clip_range: float = 0.2, ent_coef: float = 0.01, vf_coef: float = 0.5, max_grad_norm: float = 0.5,
                 normalize_advantage: bool = True, seed: int = 0, process_group=None):
        if not isinstance(policy, (ActorCriticPolicy, RecurrentActorCriticPolicy)):
            raise TypeError("policy must be an ActorCriticPolicy or RecurrentActorCriticPolicy")
        if batch_size < 1 or n_epochs < 1:
            raise ValueError("batch_size and n_epochs must be >= 1")
        self.policy = policy
        self.recurrent = bool(getattr(policy, "recurrent", False))
        self.lr = float(learning_rate)
        self.n_epochs = int(n_epochs)
        self.batch_size = int(batch_size)
        self.clip_range = float(clip_range)
        self.ent_coef = float(ent_coef)
        self.vf_coef = float(vf_coef)
        self.max_grad_norm = float(max_grad_norm)
        self.normalize_advantage = bool(normalize_advantage)
        self.rng = np.random.default_rng(seed)
        self.group = process_group
        self.params = [p for p in policy.parameters() if p.requires_grad]
        # on the GPU one fused Adam kernel over all parameters (sb3's Adam, same
        # update; torch's per-tensor foreach path costs ~9 launches per step)
        fused = bool(self.params) and all(p.is_cuda for p in self.params)
        self.optimizer = torch.optim.Adam(self.params, lr=self.lr, eps=1e-5, fused=fused or None)
        self.n_updates = 0
        # heads + losses + their gradient in one fused kernel family on the GPU
        # (learn_ops.ppo_loss); VOXNAV_FUSED_LOSS=0: torch's ops and autograd (A/B knob)
        self.fused_loss = os.environ.get("VOXNAV_FUSED_LOSS", "1") != "0"
        # the Adam step on the library's kernel (learn_ops.adam_step, the optimizer's
        # own state tensors); VOXNAV_NATIVE_ADAM=0: torch's fused Adam
        self.native_adam = os.environ.get("VOXNAV_NATIVE_ADAM", "1") != "0"
        # the row-layout LSTM keeps all its blocks resident and hands states over
        # inside the launch: with another rank's grid on the same device that
        # co-residency is not guaranteed, so such ranks take the packed path
        self._rows_off = self.recurrent and process_group is not None and _ranks_share_device(process_group,
                                                                                             self.params)

    # ------------------------------------------------------------ helpers
    def _orders(self, total: int) -> List:
        if self.recurrent:
            return [int(self.rng.integers(total)) for _ in range(self.n_epochs)]
        return [self.rng.permutation(total) for _ in range(self.n_epochs)]

    def _allreduce_grads(self):
        """Average the gradients over the group (one flattened all-reduce).
        The recurrent learner appends its row-layout error word (1.0 when an
        in-launch hand-off of this rank timed out) to the same buffer, and every
        rank takes the reduced word as its own: if any rank's gradients are
        garbage, every rank skips the Adam step and every rank raises in
        ``update_many`` (no rank applies a corrupted average, no rank runs on
        into the next collective alone)."""
        import torch.distributed as dist
        grads = [p.grad for p in self.params if p.grad is not None]
        parts = [g.reshape(-1) for g in grads]
        err = lstm_seq._rows_err(grads[0].device) if self.recurrent else None
        if err is not None:
            parts.append((err != 0).to(grads[0].dtype).view(1))
        flat = torch.cat(parts)
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
        if err is not None:
            err.copy_((flat[-1:] != 0).to(err.dtype))
            flat = flat[:-1]
        flat /= dist.get_world_size(self.group)
        o = 0
        for g in grads:
            n = g.numel()
            g.copy_(flat[o:o + n].view_as(g))
            o += n

    def _heads(self, lat_pi, lat_vf, actions, lat_pair=None):
        pol = self.policy
        # both MLP branches layer by layer and the heads on the f32 matrix
        # cores (voxnav/learn_ops.py; torch's own ops on the CPU)
        ex = pol.mlp_extractor
        h_pi, h_vf = learn_ops.mlp_pair(ex.policy_net, ex.value_net, lat_pi, None if lat_vf is lat_pi else lat_vf,
                                        x_pair=lat_pair)
        logits = learn_ops.linear(h_pi, pol.action_net)
        values = learn_ops.linear(h_vf, pol.value_net).flatten()
        logp_all = torch.log_softmax(logits, dim=-1)
        log_prob = logp_all.gather(1, actions.view(-1, 1)).flatten()
        entropy = -(logp_all.exp() * logp_all).sum(-1)
        return values, log_prob, entropy

    def _pack_begin(self, buf, idx: torch.Tensor, window: bool = False) -> dict:
        """The sequence structure of minibatch rows ``idx`` (env-major flat
        ids): sequences start at episode starts and env changes
        (sb3_contrib create_sequencers).  Everything but the padded size
        (n_seq, max_len) stays on the device; on CUDA the structure is
        computed on a side stream and the size copied to pinned host memory,
        so the one host read per minibatch can wait for it while the previous
        minibatch's update still runs (``update_many``).

        ``window``: the caller guarantees ``idx`` is one contiguous window of
        the rolled env-major order (``(idx[0] + i) mod T N``, what ``train``
        cuts) -- the row layout's mapping is only valid for such minibatches;
        any other index set takes the packed per-sequence path."""
        T, N = buf.actions.shape
        dev = idx.device
        side = None
        if dev.type == "cuda":
            if getattr(self, "_side", None) is None:
                self._side = torch.cuda.Stream(dev)
            side = self._side
            side.wait_stream(torch.cuda.current_stream(dev))
        n = idx.numel()
        rows = n // T if (window and dev.type == "cuda" and n % T == 0 and n // T <= N) else 0
        if rows and not self._rows_ok(buf.obs.shape[-1], rows):
            rows = 0
        with torch.cuda.stream(side) if side is not None else _nullctx():
            env = idx // T
            t = idx - env * T
            src = t * N + env                                         # row in the [T, N]-major buffers
            es = buf.episode_starts.reshape(-1)[src]
            if rows:
                # row layout (csrc/voxnav_learn_rows.hip): row r = env e0 + r over all T
                # steps; the last env of a minibatch that starts mid-rollout (steps
                # t < t0) shares row 0 with the first (steps >= t0)
                r = torch.remainder(env - env[0], N)
                r = torch.where(r == rows, torch.zeros_like(r), r)
                pos = t * rows + r
                t0 = t[0]
                st = (t == 0) | (es > 0.5) | ((r == 0) & (t == t0) & (t0 > 0))
                src_rows = torch.empty_like(src)
                src_rows[pos] = src
                grid = dict(src=src_rows,
                            env=torch.empty(n, dtype=torch.int32, device=dev).index_put_((pos,), env.to(torch.int32)),
                            start=torch.empty(n, dtype=torch.uint8, device=dev).index_put_((pos,), st.to(torch.uint8)),
                            keep=torch.empty(n, dtype=torch.float32, device=dev).index_put_((pos,), 1.0 - es))
                pk = dict(idx=idx, rows=rows, **grid)
                if side is not None:
                    ev = torch.cuda.Event()
                    ev.record(side)
                    pk["ev"] = ev
        if rows:
            if side is not None:
                main = torch.cuda.current_stream(dev)
                for v in pk.values():
                    if isinstance(v, torch.Tensor) and v.is_cuda:
                        v.record_stream(main)
            return pk
        with torch.cuda.stream(side) if side is not None else _nullctx():
            seq_start = (es > 0.5) | (t == 0)                         # episode start or env change
            seq_start[0] = True
            seq_id = torch.cumsum(seq_start.to(torch.int64), 0) - 1
            ar = torch.arange(idx.numel(), device=dev)
            # position in the sequence: distance to the last start at or before (a running max, no sync)
            pos = ar - torch.cummax(torch.where(seq_start, ar, torch.zeros_like(ar)), 0).values
            size = torch.stack([seq_id[-1] + 1, pos.max() + 1])
            pk = dict(idx=idx, env=env, t=t, src=src, es=es, seq_start=seq_start, seq_id=seq_id, pos=pos)
            if side is not None:
                host = torch.empty(2, dtype=torch.int64, pin_memory=True)
                host.copy_(size, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(side)
                pk.update(host=host, ev=ev)
            else:
                pk.update(host=size)
        if side is not None:
            main = torch.cuda.current_stream(dev)
            for v in pk.values():
                if isinstance(v, torch.Tensor) and v.is_cuda:
                    v.record_stream(main)            # made on the side stream, used on the main one
        return pk

    def _rows_ok(self, D: int, rows: int) -> bool:
        """The row-layout LSTM kernels take (D, rows) for this policy (cached host query)."""
        cache = self.__dict__.setdefault("_rows_cache", {})
        # the layout knobs the library reads at every launch are part of the key,
        # so the cached answer is always the one for the layout actually launched
        key = (D, rows, os.environ.get("VOXNAV_ROWS_V1"), os.environ.get("VOXNAV_ROWS_V2"),
               os.environ.get("VOXNAV_LSTM_ROWS"))
        if key not in cache:
            # VOXNAV_LSTM_ROWS=0: the per-sequence packed path (A/B knob)
            cache[key] = (not self._rows_off and os.environ.get("VOXNAV_LSTM_ROWS", "1") != "0"
                          and lstm_seq.rows_supported(self.policy, D, rows))
        return cache[key]

    def _evaluate_rows(self, buf, pk: dict):
        """evaluate_actions in the row layout: both LSTMs over [T, rows] in one
        persistent launch each (no host read, no padding)."""
        T, N = buf.actions.shape
        rows = pk["rows"]
        if "ev" in pk:
            torch.cuda.current_stream(pk["idx"].device).wait_event(pk["ev"])
        src = pk["src"]
        D = buf.obs.shape[-1]
        x = buf.obs.reshape(T * N, D)[src].view(T, rows, D)
        out = lstm_seq.dual_lstm_rows_pair(self.policy, x, pk["env"], pk["start"], pk["keep"], buf.lstm_h,
                                           buf.lstm_c)                       # [2, T, rows, H]: actor, critic
        H = out.shape[-1]
        lat = out.view(2, T * rows, H)
        return (lat[0], lat[1], lat), src

    def _evaluate_recurrent(self, buf, pk: dict):
        """evaluate_actions on a packed minibatch (``_pack_begin``)."""
        T, N = buf.actions.shape
        if "rows" in pk:
            return self._evaluate_rows(buf, pk)
        if "ev" in pk:
            pk["ev"].synchronize()                                # the minibatch's size only
            torch.cuda.current_stream(pk["idx"].device).wait_event(pk["ev"])
        n_seq, max_len = (int(v) for v in pk["host"].tolist())
        src, es, seq_start, seq_id, pos, t, env = (pk[k] for k in ("src", "es", "seq_start", "seq_id", "pos", "t",
                                                                   "env"))
        dev = src.device
        first = (torch.nonzero_static(seq_start, size=n_seq).flatten() if dev.type == "cuda"
                 else torch.nonzero(seq_start, as_tuple=True)[0])   # position of each sequence start
        D = buf.obs.shape[-1]
        x = torch.zeros((max_len, n_seq, D), dtype=torch.float32, device=dev)
        x[pos, seq_id] = buf.obs.reshape(T * N, D)[src]
        keep = (1.0 - es[first]).view(1, n_seq, 1)               # (1 - episode_start) at the sequence start
        tf, ef = t[first], env[first]
        h0 = buf.lstm_h[tf, :, ef].permute(1, 0, 2) * keep        # stored states [T, 2, N, H] -> [2, n_seq, H]
        c0 = buf.lstm_c[tf, :, ef].permute(1, 0, 2) * keep
        out_pi, out_vf = dual_lstm(self.policy, x, h0, c0)
        lat_pi = out_pi[pos, seq_id]
        lat_vf = out_vf[pos, seq_id]
        return (lat_pi, lat_vf, None), src

    def _evaluate_ff(self, buf, idx: torch.Tensor):
        T, N = buf.actions.shape
        if idx.is_cuda and buf.obs.shape[-1] % 4 == 0 and buf.obs.is_contiguous():
            src, obs = learn_ops.minibatch_rows(idx.contiguous(), T, N, buf.obs)   # one launch
            return (obs, obs, None), src
        env = idx // T
        src = (idx - env * T) * N + env
        obs = buf.obs.reshape(T * N, -1)[src]
        return (obs, obs, None), src

    def update(self, buf, idx: torch.Tensor, packed: Optional[dict] = None) -> torch.Tensor:
        """One minibatch (env-major flat ids ``idx``): losses, backward,
        (all-reduce), clip, Adam.  Returns the logged values as a device
        tensor (no host sync beyond the recurrent minibatch's size)."""
        if self.recurrent:
            (lat_pi, lat_vf, lat_pair), src = self._evaluate_recurrent(buf, packed or self._pack_begin(buf, idx))
        else:
            (lat_pi, lat_vf, lat_pair), src = self._evaluate_ff(buf, idx)
        norm = self.normalize_advantage and (self.recurrent or src.numel() > 1)
        if lat_pi.is_cuda and self.fused_loss:
            pol = self.policy
            ex = pol.mlp_extractor
            F = ex.latent_dim_pi
            if F == ex.latent_dim_vf and learn_ops.ppo_loss_supported(pol.action_net, pol.value_net, F):
                h = learn_ops.mlp_pair(ex.policy_net, ex.value_net, lat_pi, None if lat_vf is lat_pi else lat_vf,
                                       x_pair=lat_pair, stacked=True)
                if h is not None:
                    return self._update_fused(buf, h, src, norm)
        values, log_prob, entropy = self._heads(lat_pi, lat_vf, buf.actions.reshape(-1)[src].long(), lat_pair)
        adv = buf.advantages.reshape(-1)[src]
        if norm:
            adv = (adv - adv.mean()) / (adv.std() + 1e-8)
        old_lp = buf.log_probs.reshape(-1)[src]
        ret = buf.returns.reshape(-1)[src]
        ratio = torch.exp(log_prob - old_lp)
        l1 = adv * ratio
        l2 = adv * torch.clamp(ratio, 1 - self.clip_range, 1 + self.clip_range)
        policy_loss = -torch.min(l1, l2).mean()
        value_loss = Fn.mse_loss(ret, values)
        entropy_loss = -entropy.mean()
        loss = policy_loss + self.ent_coef * entropy_loss + self.vf_coef * value_loss
        self.optimizer.zero_grad(set_to_none=True)
        loss.backward()
        if self.group is not None:
            self._allreduce_grads()
        gnorm = self._clip_step()
        with torch.no_grad():
            log_ratio = log_prob - old_lp
            return torch.stack([policy_loss.detach().double(), value_loss.detach().double(),
                                entropy_loss.detach().double(), loss.detach().double(),
                                ((torch.exp(log_ratio) - 1) - log_ratio).mean().double(),
                                (torch.abs(ratio - 1) > self.clip_range).double().mean(),
                                gnorm.detach().double()])

    def _update_fused(self, buf, h: torch.Tensor, src: torch.Tensor, norm: bool) -> torch.Tensor:
        """``update`` from the MLP latents h [2, M, F] on: the heads, losses and
        their gradient in the fused loss kernel (learn_ops.ppo_loss), the
        latents' gradient backpropagated through the MLP and LSTM kernels,
        the head gradients assigned; then (all-reduce), clip, Adam."""
        pol = self.policy
        dh, grads, stats = learn_ops.ppo_loss(h, pol.action_net, pol.value_net, src, buf.actions.reshape(-1),
                                              buf.advantages.reshape(-1), buf.log_probs.reshape(-1),
                                              buf.returns.reshape(-1), self.clip_range, self.ent_coef, self.vf_coef,
                                              norm)
        self.optimizer.zero_grad(set_to_none=True)
        h.backward(dh)
        for prm, g in zip((pol.action_net.weight, pol.action_net.bias, pol.value_net.weight, pol.value_net.bias),
                          grads):
            if prm.requires_grad:
                prm.grad = g
        if self.group is not None:
            self._allreduce_grads()
        gnorm = self._clip_step()
        return torch.cat([stats, gnorm.detach().double().view(1)])

    def _clip_step(self) -> torch.Tensor:
        """clip_grad_norm_ + Adam step.  On the GPU: the norm in two launches
        (learn_ops.grad_norm_scale) and the step in one (learn_ops.adam_step),
        the clip applied by the step as its divisor of the gradients; else
        torch's clip and step."""
        fused = self.optimizer.param_groups[0].get("fused")
        if fused and self.params[0].is_cuda:
            gnorm, scale = learn_ops.grad_norm_scale(self.params, self.max_grad_norm)
            if self.native_adam:
                # the recurrent learner's row-layout launches set a device error word
                # when an in-launch hand-off times out; the step is skipped on the
                # device while it is set (rows_check raises after the minibatches)
                skip = lstm_seq.rows_err_word(self.params[0].device) if self.recurrent else None
                learn_ops.adam_step(self.optimizer, scale, skip=skip)
            else:
                self.optimizer.grad_scale = scale
                try:
                    self.optimizer.step()
                finally:
                    self.optimizer.grad_scale = None
        else:
            gnorm = torch.nn.utils.clip_grad_norm_(self.params, self.max_grad_norm)
            err = lstm_seq.rows_err_word(self.params[0].device) if self.recurrent else None
            if err is not None and err.device.type == "cpu" and int(err.item()) != 0:
                return gnorm                # a rank's hand-off timed out (the reduced word): no step anywhere
            self.optimizer.step()
        self.n_updates += 1
        return gnorm

    def update_many(self, buf, idxs: Sequence[torch.Tensor], windows: bool = False) -> torch.Tensor:
        """``update`` over consecutive minibatches, the next minibatch's
        sequence structure computed (side stream) while this one's update is
        queued, so the host read of its size does not idle the GPU.
        ``windows``: every ``idx`` is a contiguous window of the rolled
        env-major order (``train``'s minibatches), which lets whole-rollout
        minibatches take the row-layout LSTM.  Returns the stacked logs [n, 7]."""
        idxs = list(idxs)
        if not idxs:
            return torch.zeros((0, 7), dtype=torch.float64)
        nxt = self._pack_begin(buf, idxs[0], windows) if self.recurrent else None
        n0 = self.n_updates
        logs = []
        for i, idx in enumerate(idxs):
            cur = nxt
            if self.recurrent and i + 1 < len(idxs):
                nxt = self._pack_begin(buf, idxs[i + 1], windows)
            logs.append(self.update(buf, idx, packed=cur))
        if self.recurrent:
            try:
                lstm_seq.rows_check(self.params[0].device)   # a timed-out row-layout launch raises
            except Exception:
                # the skipped Adam steps did not advance the device step counters:
                # n_updates counts the steps actually applied, and the host mirror
                # of the step count is re-read on the next step
                cache = getattr(self.optimizer, "_vn_adam_t", None)
                if cache is not None:
                    t_dev = int(round(float(cache[0].item())))
                    self.n_updates = n0 + max(0, t_dev - (cache[1] - len(idxs)))
                self.optimizer._vn_adam_t = None
                raise
        return torch.stack(logs)

    # ------------------------------------------------------------ train
    def train(self, buf, epoch_orders: Optional[Sequence] = None) -> Dict[str, float]:
        """One ``train()`` over a collector ``RolloutBuffer`` (n_epochs passes).
        Returns the means of sb3's logged quantities."""
        T, N = buf.actions.shape
        total = T * N
        dev = buf.actions.device
        if self.recurrent and (buf.lstm_h is None or buf.lstm_c is None):
            raise ValueError("the recurrent learner needs the buffer's LSTM states (store_lstm_states=True)")
        orders = list(epoch_orders) if epoch_orders is not None else self._orders(total)
        acc = torch.zeros(7, dtype=torch.float64, device=dev)
        n_mb = 0
        self.policy.train()
        for order in orders:
            if self.recurrent:
                perm = torch.roll(torch.arange(total, device=dev), -int(order))
            else:
                perm = torch.as_tensor(np.asarray(order), dtype=torch.int64, device=dev)
            logs = self.update_many(buf, [perm[s:s + self.batch_size] for s in range(0, total, self.batch_size)],
                                    windows=self.recurrent)
            acc += logs.sum(0)
            n_mb += logs.shape[0]
        m = (acc / max(1, n_mb)).tolist()
        with torch.no_grad():
            v, r = buf.values.reshape(-1), buf.returns.reshape(-1)
            var_r = torch.var(r)
            ev = float("nan") if float(var_r) == 0 else float(1 - torch.var(r - v) / var_r)
        return dict(policy_gradient_loss=m[0], value_loss=m[1], entropy_loss=m[2], loss=m[3], approx_kl=m[4],
                    clip_fraction=m[5], grad_norm=m[6], explained_variance=ev, n_minibatches=n_mb,
                    n_updates=self.n_updates)


def _ranks_share_device(group, params) -> bool:
    """Whether another rank of ``group`` drives the same GPU as this one (one
    all-gather of (host, device uuid) at construction; False off the GPU)."""
    if not params or not params[0].is_cuda:
        return False
    import socket
    import torch.distributed as dist
    dev = params[0].device
    me = (socket.gethostname(), str(torch.cuda.get_device_properties(dev).uuid))
    allk = [None] * dist.get_world_size(group)
    dist.all_gather_object(allk, me, group=group)
    return allk.count(me) > 1


def learn(collector, learner: PPOLearner, total_timesteps: int, callback=None) -> List[Dict[str, float]]:
    """``model.learn(total_timesteps, callback=...)`` (OnPolicyAlgorithm.learn):
    alternate ``collector.collect()`` and ``learner.train()`` until
    ``total_timesteps`` env steps (agents x steps, summed over this rank)
    were collected, pushing the updated weights into the collector after
    every update.

    ``callback``: one callback or a list.  Objects with ``on_rollout_end``
    (``voxnav.evaluate.EvalCallback``, Grid_Train.py:218-226) run after each
    rollout, before the update -- the weights the rollout was collected
    with; plain callables ``callback(iteration, num_timesteps, stats)`` run
    after the update, returning False stops early (SB3 semantics).

    Returns the per-iteration stats: the train losses, ``num_timesteps``,
    the Monitor's ``ep_rew_mean`` / ``ep_len_mean`` over the last 100
    finished episodes (SB3's ``rollout/`` logger keys, when any episode has
    finished) and the evaluation's ``eval/*`` keys when one ran."""
    if collector.policy is not learner.policy:
        raise ValueError("collector and learner must share the policy module")
    cbs = [] if callback is None else (list(callback) if isinstance(callback, (list, tuple)) else [callback])
    per_rollout = collector.n_steps * collector.N
    done, it, history = 0, 0, []
    while done < total_timesteps:
        buf = collector.collect()
        done += per_rollout
        it += 1
        evals = {}
        for cb in cbs:
            if hasattr(cb, "on_rollout_end"):
                evals.update(cb.on_rollout_end(learner.policy, done, collector.n_steps, learner.optimizer) or {})
        st = learner.train(buf)
        collector.sync_weights()
        st["num_timesteps"] = done
        mon = getattr(collector, "monitor", None)
        if mon is not None and mon.ep_info_buffer:
            st["ep_rew_mean"] = mon.ep_rew_mean()
            st["ep_len_mean"] = mon.ep_len_mean()
        st.update(evals)
        history.append(st)
        stop = False
        for cb in cbs:
            if not hasattr(cb, "on_rollout_end") and callable(cb) and cb(it, done, st) is False:
                stop = True
        if stop:
            break
    return history
