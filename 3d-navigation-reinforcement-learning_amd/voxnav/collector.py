"""On-device PPO rollout collector (policy in the loop) around BatchedGridEnv.

Restates sb3_contrib ``RecurrentPPO.collect_rollouts`` (and SB3
``OnPolicyAlgorithm.collect_rollouts`` for the feed-forward policy), which
train/Grid_Train.py reaches through ``model.learn`` (:228) with
``n_steps=2048, gamma=0.99, gae_lambda=0.95`` (:84-85), for N agents on one
GPU with nothing crossing PCIe per step (one 4-byte count per rollout):

per step t
  1. policy forward on obs[t] (states already zeroed for agents whose
     previous step ended an episode), on the library's own f32 matrix-core
     kernels (csrc/voxnav_policy_f32.hip): ``vn_lstm_fused_f32`` (both
     LSTMs' ``[x | h] @ [W_ih | W_hh]^T`` with the cell update as epilogue,
     the episode-start mask applied on read, (h, c) stored into the buffer)
     and ``vn_mlp_head_f32`` (both Tanh MLPs, the action and value heads,
     the Categorical draw and its log-prob in one launch).  Policies outside
     those kernels' shapes take ``vn_linear_f32`` + ``vn_policy_head``;
     torch.mm (library GEMMs) remains only for the bf16 option and for f32
     shapes the f32 kernels do not take ("Collector paths")
  2. ``BatchedGridEnv.step_into`` -> obs[t+1], reward[t], terminated,
     truncated, terminal_obs (SB3 auto-reset inside the env kernel)
  3. ``vn_collect_post_step`` (one launch) -> episode_starts[t+1] = done;
     the SB3 Monitor's per-agent episode return (f64) / length and the
     episodes that ended at step t (voxnav.monitor); the truncated agents
     (SB3: ``done and info["TimeLimit.truncated"]``) append their terminal
     obs and critic state after step t to a device stash (the count never
     leaves the GPU); the (h, c) of finished agents zeroed where the next
     step reads the state arrays (``_process_sequence``'s
     ``(1 - episode_start)`` mask; the f32 buffer path masks on read)

after T steps: the stashed terminal values V(terminal_obs; critic state)
in one batch (equal to the per-step values up to the GEMMs' rounding), added
as ``rewards[t, a] += gamma * V`` (``vn_collect_bootstrap``); V(obs[T])
under the current critic states; then the GAE scan
(``vn_gae``) -> advantages, returns; the finished episodes go to
``monitor.ep_info_buffer`` (``ep_rew_mean`` / ``ep_len_mean``).

``policy_dtype="bf16"`` runs the policy GEMMs in bf16 (f32 accumulation,
bf16 activations; LSTM cell state, heads, sampling and everything after
them stay f32) -- the reference's SB3 policy is f32, which stays the
default.

Build-defined (documented in DESIGN.md): the Categorical draw uses a
counter-based Philox stream keyed by (sample_seed, global agent id, global
step) instead of torch's global generator, so a rollout is reproducible and
independent of how agents are sharded over GPUs.
"""
from __future__ import annotations

import ctypes as C
import os
import numpy as np
from dataclasses import dataclass
from typing import Optional

import torch

from . import _native
from .env import OBS_DIM, BatchedGridEnv
from .monitor import EpisodeMonitor
from .policy import ActorCriticPolicy, RecurrentActorCriticPolicy


def _p(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


@dataclass
class RolloutBuffer:
    """SB3 (Recurrent)RolloutBuffer fields, [T, N]-major, on the GPU.

    ``obs[t]`` is the observation the policy acted on at step t;
    ``episode_starts[t]`` is SB3's ``_last_episode_starts`` at step t;
    ``lstm_h / lstm_c [T, 2, N, H]`` are the (actor, critic) states entering
    step t, before the episode-start mask (SB3 stores ``_last_lstm_states``).
    """
    obs: torch.Tensor
    actions: torch.Tensor
    rewards: torch.Tensor
    episode_starts: torch.Tensor
    values: torch.Tensor
    log_probs: torch.Tensor
    advantages: torch.Tensor
    returns: torch.Tensor
    lstm_h: Optional[torch.Tensor] = None
    lstm_c: Optional[torch.Tensor] = None
    last_values: Optional[torch.Tensor] = None
    dones: Optional[torch.Tensor] = None


class _Weights:
    """The policy's parameters laid out for the collector's GEMMs/kernels.

    GEMM operands (weights, MLP biases) are in ``dtype`` (f32, or bf16 for
    the bf16 policy path); LSTM biases and the head weights stay f32 (they
    are applied inside the HIP kernels in f32)."""

    def __init__(self, policy, device, dtype=torch.float32):
        f = lambda t: t.detach().to(device=device, dtype=torch.float32).contiguous()  # noqa: E731
        g = lambda t: t.detach().to(device=device, dtype=dtype).contiguous()  # noqa: E731
        self.dtype = dtype
        self.recurrent = bool(getattr(policy, "recurrent", False))
        if self.recurrent:
            la, lc = policy.lstm_actor, policy.lstm_critic
            if la.num_layers != 1 or lc.num_layers != 1:
                raise NotImplementedError("one LSTM layer (Grid_Train's n_lstm_layers=1)")
            self.H = la.hidden_size
            self.w_ih_cat = torch.cat([g(la.weight_ih_l0), g(lc.weight_ih_l0)], 0)      # [2*4H, 80]
            self.w_hh = [g(la.weight_hh_l0), g(lc.weight_hh_l0)]                       # [4H, H]
            self.w_ih_vf = g(lc.weight_ih_l0)
            self.b_ih = torch.stack([f(la.bias_ih_l0), f(lc.bias_ih_l0)])               # [2, 4H]
            self.b_hh = torch.stack([f(la.bias_hh_l0), f(lc.bias_hh_l0)])
            # fused MFMA LSTM step (bf16 path, H % 64 == 0): [W_ih | W_hh] packed
            # K-contiguous, x part padded to a multiple of 8, K to a multiple of 64
            self.fused = dtype == torch.bfloat16 and self.H % 64 == 0
            if self.fused:
                od = la.weight_ih_l0.shape[1]
                self.kx = (od + 7) // 8 * 8
                self.Kp = (self.kx + self.H + 63) // 64 * 64
                wc = torch.zeros((2, 4 * self.H, self.Kp), dtype=torch.float32, device=device)
                for b, m in enumerate((la, lc)):
                    wc[b, :, :od] = f(m.weight_ih_l0)
                    wc[b, :, self.kx:self.kx + self.H] = f(m.weight_hh_l0)
                self.w_cat = wc.to(torch.bfloat16).contiguous()
                self.bias = (self.b_ih + self.b_hh).contiguous()
        ext = policy.mlp_extractor
        self.pi = [(g(m.weight), g(m.bias)) for m in ext.linears("pi")]
        self.vf = [(g(m.weight), g(m.bias)) for m in ext.linears("vf")]
        # f32 policy path on the f32 matrix cores (csrc/voxnav_policy_f32.hip):
        # the LSTM step as one kernel (vn_lstm_fused_f32) and the MLP layers as
        # Linear+Tanh kernels (vn_linear_f32, both branches per launch); needs
        # H % 64 == 0, layer widths % 128 and inputs % 16, pi and vf the same widths
        widths = [w.shape[0] for w, _ in self.pi]
        self.f32mlp = (dtype == torch.float32 and widths == [w.shape[0] for w, _ in self.vf]
                       and all(w.shape[0] % 128 == 0 and w.shape[1] % 16 == 0 for w, _ in self.pi + self.vf))
        self.fused32 = self.recurrent and self.f32mlp and self.H % 64 == 0
        if self.f32mlp:
            self.pi_packed = [pack_linear_f32(w) for w, _ in self.pi]
            self.vf_packed = [pack_linear_f32(w) for w, _ in self.vf]
        if self.fused32:
            od = la.weight_ih_l0.shape[1]
            self.Kp32 = (od + 15) // 16 * 16 + self.H
            self.lstm_packed = pack_lstm_f32([f(la.weight_ih_l0), f(lc.weight_ih_l0)],
                                             [f(la.weight_hh_l0), f(lc.weight_hh_l0)])
            self.bias32 = (self.b_ih + self.b_hh).contiguous()
        self.wa, self.ba = f(policy.action_net.weight), f(policy.action_net.bias)
        self.wv, self.bv = f(policy.value_net.weight).reshape(-1), f(policy.value_net.bias)
        self.A = self.wa.shape[0]
        self.P = self.wa.shape[1]
        if self.wv.shape[0] != self.P:
            raise NotImplementedError("pi and vf latents must have the same width")
        # the MLPs and heads in one launch (vn_mlp_head_f32): layer widths 128 / 256,
        # at most 4 layers, inputs % 16 <= 256, at most 8 actions; W^T per layer.
        # VOXNAV_MLP_HEAD=0: the per-layer kernels + vn_policy_head (A/B knob)
        k0 = self.pi[0][0].shape[1] if self.pi else 0
        self.mlp_head = (self.f32mlp and 1 <= len(self.pi) <= 4 and all(w.shape[0] in (128, 256) for w, _ in self.pi)
                         and k0 % 16 == 0 and 16 <= k0 <= 256 and self.P == widths[-1] and self.A <= 8
                         and os.environ.get("VOXNAV_MLP_HEAD", "1") != "0")
        if self.mlp_head:
            self.widths = widths
            self.mh_wt = [pack_mlp_head_f32(w) for w, _ in self.pi] + [pack_mlp_head_f32(w) for w, _ in self.vf]
            self.mh_b = [b for _, b in self.pi] + [b for _, b in self.vf]


def pack_lstm_f32(w_ih, w_hh) -> torch.Tensor:
    """[W_ih | 0 | W_hh] of each LSTM in vn_lstm_fused_f32's layout
    [n_lstm][H/64][Kp][4][64] (include/voxnav.h): element [b][ub][k][g][uu] =
    Wcat_b[g*H + 64*ub + uu][k], W_ih in columns [0, obs_dim), W_hh in
    [kx, kx + H), kx = obs_dim rounded up to 16."""
    nl = len(w_ih)
    G, od = w_ih[0].shape
    H = w_hh[0].shape[1]
    kx = (od + 15) // 16 * 16
    Kp = kx + H
    wc = torch.zeros((nl, G, Kp), dtype=torch.float32, device=w_ih[0].device)
    for b in range(nl):
        wc[b, :, :od] = w_ih[b]
        wc[b, :, kx:kx + H] = w_hh[b]
    return wc.view(nl, 4, H // 64, 64, Kp).permute(0, 2, 4, 1, 3).contiguous()


def pack_linear_f32(w: torch.Tensor) -> torch.Tensor:
    """W [Nout, K] in vn_linear_f32's layout [Nout/128][K][128]."""
    n, k = w.shape
    return w.detach().to(torch.float32).reshape(n // 128, 128, k).permute(0, 2, 1).contiguous()


def pack_mlp_head_f32(w: torch.Tensor) -> torch.Tensor:
    """W [N, K] in vn_mlp_head_f32's per-lane layout [N/32][Kp/8][64][4], K
    zero-padded to Kp = a multiple of 16: element [cb][kg][lane][s] =
    W[32 cb + lane % 32][8 kg + 4 (lane // 32) + s]."""
    n, k = w.shape
    kp = (k + 15) // 16 * 16
    w = torch.nn.functional.pad(w.detach().to(torch.float32), (0, kp - k))
    return w.reshape(n // 32, 32, kp // 8, 2, 4).permute(0, 2, 3, 1, 4).contiguous()


def _mlp(layers, x):
    for w, b in layers:
        x = torch.addmm(b, x, w.t())
        x.tanh_()
    return x


class RolloutCollector:
    """``collect()`` fills a RolloutBuffer of ``n_steps`` x ``env.num_agents``.

    ``policy``: ``RecurrentActorCriticPolicy`` (PPO-LSTM, Grid_Train) or
    ``ActorCriticPolicy`` (PPO-MLP).  Its parameters are read at
    construction and again by ``sync_weights()`` (after a learner update).
    """

    def __init__(self, env: BatchedGridEnv, policy, n_steps: int = 128, gamma: float = 0.99, gae_lambda: float = 0.95,
                 sample_seed: int = 42, deterministic: bool = False, store_lstm_states: bool = True,
                 reset_seed: int = 42, policy_dtype: str = "f32", monitor: bool = True):
        if not isinstance(policy, (ActorCriticPolicy, RecurrentActorCriticPolicy)):
            raise TypeError("policy must be an ActorCriticPolicy or RecurrentActorCriticPolicy")
        if getattr(policy, "obs_dim", OBS_DIM) != env.obs_dim:
            raise ValueError(f"policy obs_dim {policy.obs_dim} != env obs_dim {env.obs_dim}")
        self.env = env
        self.lib = env.lib
        self.device = env.device
        self.policy = policy
        self.n_steps = int(n_steps)
        self.gamma = float(gamma)
        self.gae_lambda = float(gae_lambda)
        self.sample_seed = int(sample_seed)
        self.deterministic = bool(deterministic)
        self.N = env.num_agents
        self.t_global = 0
        if policy_dtype not in ("f32", "bf16"):
            raise ValueError("policy_dtype must be 'f32' (the reference's) or 'bf16'")
        self.bf16 = policy_dtype == "bf16"
        self.cdt = torch.bfloat16 if self.bf16 else torch.float32
        self._sp = None
        self.sync_weights()
        T, N, dev = self.n_steps, self.N, self.device
        z = lambda *s, dt=torch.float32: torch.zeros(s, dtype=dt, device=dev)  # noqa: E731
        self._obs = z(T + 1, N, env.obs_dim)
        self._starts = z(T + 1, N)
        self.actions = z(T, N, dt=torch.int32)
        self.rewards = z(T, N)
        self.values = z(T, N)
        self.log_probs = z(T, N)
        self._term = z(N, dt=torch.uint8)
        self._trunc = z(N, dt=torch.uint8)
        self._tobs = z(N, env.obs_dim)
        self._last_values = z(N)
        self.recurrent = self.w.recurrent
        # the f32 MLP kernels' per-layer outputs, [branch][rows][width]; sized
        # for the larger of N and the bootstrap stash (the critic runs on it)
        if self.recurrent:
            H = self.w.H
            self.h = z(2, N, H)
            self.c = z(2, N, H)
            if not self.w.fused32:     # gate pre-activations of the library-GEMM path
                self._gx = z(N, 2 * 4 * H, dt=self.cdt)
                self._gh = z(2, N, 4 * H, dt=self.cdt)
            self.h_bf = z(2, N, H, dt=torch.bfloat16) if self.bf16 else None   # GEMM copy of h
            self.fused = self.bf16 and self.w.fused
            self.h_bf2 = z(2, N, H, dt=torch.bfloat16) if self.fused else None  # fused step's output (ping-pong)
            self.store = bool(store_lstm_states)
            self._no_start = z(N)                                              # step 0's mask (none)
            self._hs = z(T + 1, 2, N, H) if self.store else None
            self._cs = z(T + 1, 2, N, H) if self.store else None
        # truncation bootstrap stash (vn_collect_stash): the truncated agents'
        # terminal obs and critic state, appended on the device each step and
        # bootstrapped every `_flush_every` steps (one host read each; once per
        # rollout unless the rooms are small).  An episode truncates when its
        # step count reaches the room's free-cell count, so an agent truncates
        # at most (F - 1) // min_free + 1 times in F steps; F = min(T, 4 min_free)
        # keeps the stash at <= 4 rows per agent (obs + critic h, c: 4 (80 + 2H) B
        # a row) whatever n_steps is.
        fmin = max(1, int(np.min(env.total_free_cells)))
        self._flush_every = min(T, 4 * fmin)
        self._stash_cap = N * ((self._flush_every - 1) // fmin + 1)
        cap = self._stash_cap
        self._stash_cnt = z(1, dt=torch.int32)       # stash rows used (vn_collect_post_step's running count)
        self._stash_obs = z(cap, env.obs_dim)
        self._stash_flat = z(cap, dt=torch.int32)
        if self.recurrent:
            self._stash_h = z(cap, self.w.H, dt=torch.bfloat16 if self.fused else torch.float32)
            self._stash_c = z(cap, self.w.H)
        # SB3 Monitor on every worker (train/Grid_Train.py:125): it sums the env's
        # f64 rewards, so the env step also writes them (voxnav.monitor)
        if self.w.f32mlp and not self.w.mlp_head:
            rows = max(N, self._stash_cap)
            self._lat32 = [z(2, rows, wt.shape[0]) for wt, _ in self.w.vf]
        if self.recurrent and self.w.fused32:
            self._h_alt = z(2, N, self.w.H)           # ping-pong partner of self.h outside collect()
            self._crit_h = z(max(N, self._stash_cap), self.w.H)   # critic-only LSTM output (bootstrap, last values)
        # per-rollout buffers allocated once (the returned RolloutBuffer views
        # them until the next collect()): no allocator traffic between rollouts
        self._adv = z(T, N)
        self._ret = z(T, N)
        self._tv = z(max(N, self._stash_cap))
        self._zero = torch.zeros((), device=dev)
        if self.recurrent:
            self._crit_hin = z(N, self.w.H, dt=torch.bfloat16 if self.fused else torch.float32)
            self._crit_c = z(N, self.w.H)
        self.monitor = EpisodeMonitor(self.lib, N, T, dev) if monitor else None
        self._r64 = z(N, dt=torch.float64) if monitor else None
        # learn() start: reset every env, episode_starts = ones, zero states
        self._obs[0] = env.reset(seed=reset_seed)
        self._starts[0].fill_(1.0)
        self._carry = False

    def sync_weights(self):
        self.w = _Weights(self.policy, self.device, self.cdt)

    def _stream(self):
        if self._sp is not None:       # inside collect(): the stream it started on
            return self._sp
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    # -------------------------------------------------------------- policy
    def _cell(self, gx, gx_row, gh, b_ih, b_hh, h, c, h_bf, hs, cs, nl, M):
        if self.bf16:
            _native.check(self.lib.vn_lstm_cell_bf16(_p(gx), gx_row, _p(gh), _p(b_ih), _p(b_hh), _p(h), _p(c),
                                                     _p(h_bf), _p(hs), _p(cs), nl, M, self.w.H, self._stream()),
                          "vn_lstm_cell_bf16")
        else:
            _native.check(self.lib.vn_lstm_cell(_p(gx), gx_row, _p(gh), _p(b_ih), _p(b_hh), _p(h), _p(c), _p(hs),
                                                _p(cs), nl, M, self.w.H, self._stream()), "vn_lstm_cell")

    def _head(self, lat_pi, lat_vf, M, t, actions, values, log_probs):
        w = self.w
        fn = self.lib.vn_policy_head_bf16 if self.bf16 else self.lib.vn_policy_head
        pi = lat_pi is not None
        _native.check(fn(_p(lat_pi), _p(lat_vf), M, w.P, _p(w.wa) if pi else None, _p(w.ba) if pi else None,
                         w.A if pi else 0, _p(w.wv), _p(w.bv), self.sample_seed if pi else 0, t if pi else 0,
                         self.env.agent_id_base if pi else 0, int(self.deterministic) if pi else 0, _p(actions),
                         _p(values), _p(log_probs), self._stream()), "vn_policy_head")

    def _fused(self, obs, h_in, c, h_out, hs, cs, nl, M, b0):
        w = self.w
        _native.check(self.lib.vn_lstm_fused_bf16(_p(obs), obs.shape[1], _p(h_in), _p(w.w_cat[b0:b0 + nl]), w.Kp,
                                                  _p(w.bias[b0:b0 + nl]), _p(c), _p(h_out), None, _p(hs), _p(cs), nl,
                                                  M, w.H, self._stream()), "vn_lstm_fused_bf16")

    def _fused_rollout(self, obs, t):
        """The fused step inside collect(): c read from the buffer's lstm_c[t]
        (the episode-start mask applied on read; step 0 reads the current,
        already masked state) and written only to lstm_c[t+1]."""
        w = self.w
        c_in, start = (self.c, self._no_start) if t == 0 else (self._cs[t], self._starts[t])
        _native.check(self.lib.vn_lstm_fused_bf16_masked(_p(obs), obs.shape[1], _p(self.h_bf), _p(w.w_cat), w.Kp,
                                                         _p(w.bias), _p(c_in), _p(start), _p(self._cs[t + 1]),
                                                         _p(self.h_bf2), _p(self._hs[t + 1]), 2, self.N, w.H,
                                                         self._stream()), "vn_lstm_fused_bf16_masked")

    def _lstm32(self, obs, h_in, c_in, start, c_out, h_out, nl, M, b0):
        w = self.w
        _native.check(self.lib.vn_lstm_fused_f32(_p(obs), obs.shape[1], _p(h_in), _p(w.lstm_packed[b0:b0 + nl]),
                                                 w.Kp32, _p(w.bias32[b0:b0 + nl]), _p(c_in), _p(start), _p(c_out),
                                                 _p(h_out), nl, M, w.H, self._stream()), "vn_lstm_fused_f32")

    def _mlp32(self, x_pi, x_vf, M):
        """Both MLP branches (or the value branch alone when x_pi is None),
        layer by layer through vn_linear_f32 into the collector's latent
        buffers; returns (lat_pi, lat_vf)."""
        w = self.w
        if getattr(self, "_lat32", None) is None:      # (not allocated when the fused head is the default)
            rows = max(self.N, self._stash_cap)
            self._lat32 = [torch.zeros((2, rows, wt.shape[0]), dtype=torch.float32, device=self.device)
                           for wt, _ in w.vf]
        br = [(x_pi, w.pi_packed, w.pi, 0)] if x_pi is not None else []
        br.append((x_vf, w.vf_packed, w.vf, 1))
        xs = [b[0] for b in br]
        for li, (wt, _) in enumerate(w.vf):
            nout, k = wt.shape
            ys = [self._lat32[li][b[3]][:M] for b in br]
            arr = lambda ts: (C.c_void_p * 2)(*[t.data_ptr() for t in ts])  # noqa: E731
            _native.check(self.lib.vn_linear_f32(len(br), arr(xs), xs[0].stride(0), arr([b[1][li] for b in br]),
                                                 arr([b[2][li][1] for b in br]), arr(ys), M, k, nout, 1,
                                                 self._stream()), "vn_linear_f32")
            xs = ys
        return (xs[0] if x_pi is not None else None), xs[-1]

    def _mlp_head32(self, x_pi, x_vf, M, t, actions, values, log_probs):
        """Both MLP branches and the heads in one launch (vn_mlp_head_f32); the
        value branch alone when x_pi is None (values only)."""
        w = self.w
        xs = [x_pi, x_vf] if x_pi is not None else [x_vf]
        nb, nl = len(xs), len(w.widths)
        if nb == 2 and x_pi.stride(0) != x_vf.stride(0):
            raise ValueError("pi and vf inputs must share a row stride")
        wt = w.mh_wt if nb == 2 else w.mh_wt[nl:]
        bs = w.mh_b if nb == 2 else w.mh_b[nl:]
        arr = lambda ts: (C.c_void_p * len(ts))(*[x.data_ptr() for x in ts])  # noqa: E731
        pi = nb == 2
        _native.check(self.lib.vn_mlp_head_f32(nb, arr(xs), xs[0].stride(0), xs[0].shape[1], nl,
                                               (C.c_int32 * nl)(*w.widths), arr(wt), arr(bs),
                                               _p(w.wa) if pi else None, _p(w.ba) if pi else None, w.A if pi else 0,
                                               _p(w.wv), _p(w.bv), self.sample_seed if pi else 0, t if pi else 0,
                                               self.env.agent_id_base if pi else 0,
                                               int(self.deterministic) if pi else 0, _p(actions), _p(log_probs),
                                               _p(values), M, self._stream()), "vn_mlp_head_f32")

    def hidden_state(self):
        """(h, c) f32 [2, N, H] of the (actor, critic) LSTMs after the last step
        (h from its bf16 copy on the fused bf16 path)."""
        h = self.h_bf.float() if self.fused else self.h
        return h, self.c

    def _forward(self, obs: torch.Tensor, t: int, in_rollout: bool = False):
        """Policy step on obs [N, 80] into actions/values/log_probs[t]."""
        w, N = self.w, self.N
        if self.recurrent and self.fused:
            if in_rollout and self.store:
                self._fused_rollout(obs, t)
            else:
                hs = self._hs[t + 1] if self.store else None
                cs = self._cs[t + 1] if self.store else None
                self._fused(obs, self.h_bf, self.c, self.h_bf2, hs, cs, 2, N, 0)
            self.h_bf, self.h_bf2 = self.h_bf2, self.h_bf
            lat_pi = _mlp(w.pi, self.h_bf[0])
            lat_vf = _mlp(w.vf, self.h_bf[1])
            self._head(lat_pi, lat_vf, N, self.t_global, self.actions[t], self.values[t], self.log_probs[t])
            return
        if self.recurrent and self.w.fused32:
            # f32 on the matrix cores: the LSTM step (gates in registers) and the
            # Linear+Tanh layers; inside collect() (h, c) live in the buffer only
            # and the kernel applies the episode-start mask on read; step 0
            # reads the current, already masked state
            if in_rollout and self.store:
                hin, c_in, start = (self.h, self.c, None) if t == 0 else (self._hs[t], self._cs[t], self._starts[t])
                h_out, c_out = self._hs[t + 1], self._cs[t + 1]
                self._lstm32(obs, hin, c_in, start, c_out, h_out, 2, N, 0)
            else:
                h_out = self._h_alt
                self._lstm32(obs, self.h, self.c, None, self.c, h_out, 2, N, 0)
                if self.store:
                    self._hs[t + 1].copy_(h_out)
                    self._cs[t + 1].copy_(self.c)
                self.h, self._h_alt = h_out, self.h
            if w.mlp_head:
                self._mlp_head32(h_out[0], h_out[1], N, self.t_global, self.actions[t], self.values[t],
                                 self.log_probs[t])
                return
            lat_pi, lat_vf = self._mlp32(h_out[0], h_out[1], N)
            self._head(lat_pi, lat_vf, N, self.t_global, self.actions[t], self.values[t], self.log_probs[t])
            return
        x = obs if not self.bf16 else obs.to(self.cdt)
        if self.recurrent and in_rollout and self.store and not self.bf16:
            # f32 inside collect(): (h, c) live in the buffer only; the products
            # use the unmasked lstm_h[t] and the cell kernel applies the
            # episode-start mask (vn_lstm_cell_masked); step 0 reads the
            # current, already masked state
            H = w.H
            hin, c_in, start = (self.h, self.c, self._no_start) if t == 0 else \
                (self._hs[t], self._cs[t], self._starts[t])
            torch.mm(x, w.w_ih_cat.t(), out=self._gx)
            torch.mm(hin[0], w.w_hh[0].t(), out=self._gh[0])
            torch.mm(hin[1], w.w_hh[1].t(), out=self._gh[1])
            h_out = self._hs[t + 1]
            _native.check(self.lib.vn_lstm_cell_masked(_p(self._gx), 8 * H, _p(self._gh), _p(w.b_ih), _p(w.b_hh),
                                                       _p(c_in), _p(start), _p(h_out), _p(self._cs[t + 1]), 2, N, H,
                                                       self._stream()), "vn_lstm_cell_masked")
            x_pi, x_vf = h_out[0], h_out[1]
        elif self.recurrent:
            H = w.H
            hin = self.h_bf if self.bf16 else self.h
            torch.mm(x, w.w_ih_cat.t(), out=self._gx)
            torch.mm(hin[0], w.w_hh[0].t(), out=self._gh[0])
            torch.mm(hin[1], w.w_hh[1].t(), out=self._gh[1])
            hs = self._hs[t + 1] if self.store else None
            cs = self._cs[t + 1] if self.store else None
            self._cell(self._gx, 8 * H, self._gh, w.b_ih, w.b_hh, self.h, self.c, self.h_bf, hs, cs, 2, N)
            x_pi, x_vf = (self.h_bf[0], self.h_bf[1]) if self.bf16 else (self.h[0], self.h[1])
        else:
            x_pi = x_vf = x
        if w.mlp_head:
            self._mlp_head32(x_pi.contiguous(), x_vf.contiguous(), N, self.t_global, self.actions[t], self.values[t],
                             self.log_probs[t])
            return
        if w.f32mlp:
            lat_pi, lat_vf = self._mlp32(x_pi, x_vf, N)
        else:
            lat_pi = _mlp(w.pi, x_pi)
            lat_vf = _mlp(w.vf, x_vf)
        self._head(lat_pi, lat_vf, N, self.t_global, self.actions[t], self.values[t], self.log_probs[t])

    def _critic(self, obs: torch.Tensor, h: Optional[torch.Tensor], c: Optional[torch.Tensor], out: torch.Tensor):
        """predict_values: one critic step from state (h, c) [M, H] (consumed), value -> out [M].
        On the fused bf16 path h is the bf16 copy."""
        w, M = self.w, obs.shape[0]
        if self.recurrent and self.fused:
            h_out = torch.empty((M, w.H), dtype=torch.bfloat16, device=self.device)
            self._fused(obs.contiguous(), h.contiguous(), c, h_out, None, None, 1, M, 1)
            self._head(None, _mlp(w.vf, h_out), M, 0, None, out, None)
            return
        if self.recurrent and w.fused32:
            h_out = self._crit_h[:M]
            self._lstm32(obs.contiguous(), h.contiguous(), c, None, c, h_out, 1, M, 1)
            if w.mlp_head:
                self._mlp_head32(None, h_out, M, 0, None, out, None)
            else:
                self._head(None, self._mlp32(None, h_out, M)[1], M, 0, None, out, None)
            return
        if not self.recurrent and w.f32mlp:
            if w.mlp_head:
                self._mlp_head32(None, obs.contiguous(), M, 0, None, out, None)
            else:
                self._head(None, self._mlp32(None, obs.contiguous(), M)[1], M, 0, None, out, None)
            return
        x = obs if not self.bf16 else obs.to(self.cdt)
        if self.recurrent:
            H = w.H
            gx = torch.mm(x, w.w_ih_vf.t())
            gh = torch.mm(h if not self.bf16 else h.to(self.cdt), w.w_hh[1].t())
            h_bf = torch.empty((M, H), dtype=torch.bfloat16, device=self.device) if self.bf16 else None
            self._cell(gx, 4 * H, gh, w.b_ih[1], w.b_hh[1], h, c, h_bf, None, None, 1, M)
            x = h_bf if self.bf16 else h
        lat = _mlp(w.vf, x)
        self._head(None, lat, M, 0, None, out, None)

    @torch.no_grad()
    def act(self, obs: torch.Tensor) -> torch.Tensor:
        """``model.predict(obs, state)`` for all agents: one policy step on obs
        [N, obs_dim] that advances the collector's recurrent state; returns
        the actions [N] int32 (a view, valid until the next call).  Argmax
        when the collector was built with ``deterministic=True``."""
        self._forward(obs.contiguous(), 0)
        self.t_global += 1
        return self.actions[0]

    # -------------------------------------------------------------- rollout
    @torch.no_grad()
    def collect(self) -> RolloutBuffer:
        """One rollout of n_steps.  The returned buffer views the collector's
        storage: it stays valid until the next ``collect()``."""
        T, N, lib = self.n_steps, self.N, self.lib
        self._sp = None
        self._sp = self._stream()
        try:
            return self._collect(T, N, lib)
        finally:
            self._sp = None

    def _collect(self, T, N, lib):
        s = self._stream
        if self._carry:
            self._carry_over()
        mon = self.monitor
        if mon is not None:
            mon.begin()
        self._stash_cnt.zero_()
        rec = self.recurrent
        # with the buffer, the fused bf16 step keeps the cell state in lstm_c
        # only (vn_lstm_fused_bf16_masked) and the f32 step both h and c in
        # lstm_h / lstm_c (vn_lstm_cell_masked); self.c (and the f32 self.h)
        # are brought up to date after T
        csbuf = rec and self.store and (self.fused or not self.bf16)
        hbuf = csbuf and not self.fused
        for t in range(T):
            self._forward(self._obs[t], t, in_rollout=True)
            self.env.step_into(self.actions[t], self._obs[t + 1], self.rewards[t], self._term, self._trunc,
                               self._tobs, reward64=self._r64)
            # after the step, in one launch: episode_starts[t+1], the Monitor, the
            # truncated agents' terminal obs and critic state (before the
            # episode-start mask) into the bootstrap stash -- no host read -- and
            # the (h, c) rows of finished agents zeroed only where the next step
            # reads the state arrays themselves (the f32 buffer path reads
            # lstm_h / lstm_c[t+1] and masks on read).  The fused path's h_bf is
            # a ping-pong pair: read it after this step's swap
            hsrc = (self._hs[t + 1] if hbuf else self.h_bf if self.fused else self.h) if rec else None
            zs = rec and not hbuf
            _native.check(lib.vn_collect_post_step(
                _p(self._term), _p(self._trunc), N, t, _p(self._starts[t + 1]),
                _p(self._r64) if mon is not None else None, None,
                _p(mon.ep_return) if mon is not None else None, _p(mon.ep_length) if mon is not None else None,
                _p(mon.rec_return[t]) if mon is not None else None, _p(mon.rec_length[t]) if mon is not None else None,
                _p(self._tobs), self.env.obs_dim,
                _p(hsrc[1]) if rec else None, hsrc.element_size() if rec else 0,
                _p(self._cs[t + 1][1] if csbuf else self.c[1]) if rec else None, self.w.H if rec else 0,
                _p(self._stash_obs), _p(self._stash_h) if rec else None, _p(self._stash_c) if rec else None,
                _p(self._stash_flat), self._stash_cap, _p(self._stash_cnt),
                _p(self.h) if zs else None, _p(self.c) if zs else None, _p(self.h_bf) if zs else None,
                2 if zs else 0, s()), "vn_collect_post_step")
            self.t_global += 1
            if (t + 1) % self._flush_every == 0 and t + 1 < T:
                self._bootstrap(self._stash_cnt)   # bounded stash: flush, restart at row 0
                self._stash_cnt.zero_()
        if csbuf:   # the current (masked) state: lstm_c[T] (lstm_h[T]) with the episode-start mask
            done = self._starts[T][None, :, None] != 0
            torch.where(done, self._zero, self._cs[T], out=self.c)      # no rollout-sized temporaries
            if hbuf:
                torch.where(done, self._zero, self._hs[T], out=self.h)
        # the truncation bootstrap of the rest of the rollout
        self._bootstrap(self._stash_cnt)
        # V(last obs) under the current (masked) critic state
        if self.recurrent:
            hsrc = self.h_bf if self.fused else self.h
            self._crit_hin.copy_(hsrc[1])
            self._crit_c.copy_(self.c[1])
            self._critic(self._obs[T], self._crit_hin, self._crit_c, self._last_values)
        else:
            self._critic(self._obs[T], None, None, self._last_values)
        adv, ret = self._adv, self._ret
        _native.check(lib.vn_gae(_p(self.rewards), _p(self.values), _p(self._starts), _p(self._last_values),
                                 _p(self._starts[T]), T, N, self.gamma, self.gae_lambda, _p(adv), _p(ret), s()),
                      "vn_gae")
        self._carry = True
        if mon is not None:
            mon.harvest()
        hs = self._hs[:T] if self.recurrent and self.store else None
        cs = self._cs[:T] if self.recurrent and self.store else None
        return RolloutBuffer(obs=self._obs[:T], actions=self.actions, rewards=self.rewards,
                             episode_starts=self._starts[:T], values=self.values, log_probs=self.log_probs,
                             advantages=adv, returns=ret, lstm_h=hs, lstm_c=cs, last_values=self._last_values,
                             dones=self._starts[T])

    def _bootstrap(self, count: torch.Tensor):
        """V(terminal obs) from the stashed critic states, rewards[t, a] +=
        gamma * V for the stash's first ``count`` rows (one host read)."""
        M = int(count.item())
        if M > self._stash_cap:     # cannot happen: at most (F-1)//min_free+1 truncations per agent in F steps
            raise RuntimeError(f"bootstrap stash overflow: {M} > {self._stash_cap}")
        if M:
            tv = self._tv[:M]
            if self.recurrent:
                self._critic(self._stash_obs[:M], self._stash_h[:M], self._stash_c[:M], tv)
            else:
                self._critic(self._stash_obs[:M], None, None, tv)
            _native.check(self.lib.vn_collect_bootstrap(_p(self._stash_flat), _p(tv), M, self.gamma,
                                                        _p(self.rewards), self._stream()), "vn_collect_bootstrap")

    def _carry_over(self):
        # the previous rollout's last obs / episode starts / lstm states become
        # this rollout's first (_last_obs, _last_episode_starts, _last_lstm_states)
        T = self.n_steps
        self._obs[0].copy_(self._obs[T])
        self._starts[0].copy_(self._starts[T])
        if self.recurrent and self.store:
            self._hs[0].copy_(self._hs[T])
            self._cs[0].copy_(self._cs[T])
        self._carry = False
