"""BatchedGridEnv: N CubicEnv agents on one MI355X behind libvoxnav.

This replaces, for the hot path, what train/Grid_Train.py builds with
``SubprocVecEnv([make_env_fn(...) for i in range(NUM_ENVS)])``
(train/Grid_Train.py:120-126, :191-192): N independent ``GridAgent``
envs (envs/CubicEnv.py:15) with SB3 VecEnv auto-reset.  Inputs and outputs
are torch tensors resident on the GPU; nothing crosses PCIe per step.

Seeds.  ``reset(seed)`` with an int seeds agent i (global id
``agent_id_base + i``) with ``seed + gid``, the ``seed=42+i`` pattern of
Grid_Train's workers (:122-125).  After an auto-reset an agent's next
episode uses ``previous_seed + seed_stride`` (default: the global agent
count), all modulo 2**32, so every episode of every agent is reproducible
and identical for any sharding of the agents over GPUs.  (SB3 auto-resets
with ``seed=None``, i.e. OS entropy; the build pins the schedule instead.)
"""
from __future__ import annotations

import ctypes as C
import os
from typing import NamedTuple, Optional, Sequence, Union

import numpy as np
import torch

from . import _native
from .rooms import RoomSet, as_room_set

OBS_DIM = _native.VN_OBS_DIM
NUM_ACTIONS = 6
FINISH_PERCENTAGE = 0.84   # envs/CubicEnv.py:12
SEED_LIMIT = 2 ** 32       # np.random.seed range (envs/CubicEnv.py:80)


class StepResult(NamedTuple):
    obs: torch.Tensor            # f32 [N, obs_dim]  (post-reset obs for finished agents)
    reward: torch.Tensor         # f32 [N]  (or f64 with reward_f64=True)
    terminated: torch.Tensor     # bool [N]
    truncated: torch.Tensor      # bool [N]
    terminal_obs: Optional[torch.Tensor]  # f32 [N, obs_dim], rows valid where terminated|truncated


class Rollout(NamedTuple):
    obs: torch.Tensor            # f32 [K, N, obs_dim]
    reward: torch.Tensor         # f32 [K, N]
    terminated: torch.Tensor     # bool [K, N]
    truncated: torch.Tensor      # bool [K, N]
    actions: Optional[torch.Tensor]  # i32 [K, N]


def _variant_code(v) -> int:
    if isinstance(v, str):
        try:
            return {"cubic": _native.VN_VARIANT_CUBIC, "simple": _native.VN_VARIANT_SIMPLE}[v.lower()]
        except KeyError:
            raise ValueError(f"variant must be 'cubic' or 'simple', got {v!r}") from None
    if int(v) not in (_native.VN_VARIANT_CUBIC, _native.VN_VARIANT_SIMPLE):
        raise ValueError(f"variant must be 0 (cubic) or 1 (simple), got {v!r}")
    return int(v)


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream_ptr(device: torch.device):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class BatchedGridEnv:
    """N GridAgents (envs/CubicEnv.py) stepping together on one GPU.

    Parameters mirror ``GridAgent.__init__`` (envs/CubicEnv.py:17-29):
    ``room_path`` (or an explicit ``rooms`` RoomSet), ``width/depth/height``
    for the ctor box used when no room path is given, ``local_map_length``
    and ``crash_penalty``.  ``num_agents`` is the batch, ``autoreset`` the
    VecEnv behaviour.  ``variant="simple"`` selects the goal-seeking
    envs/simpleEnv.py GridAgent (obs 6L+7) instead
    of envs/CubicEnv.py.
    """

    def __init__(self, num_agents: int = 1, room_path=None, rooms: Optional[RoomSet] = None,
                 local_map_length: int = 4, crash_penalty: float = -2.0, width: int = 20, depth: int = 20,
                 height: int = 12, autoreset: bool = True, device: Union[int, str, torch.device, None] = None,
                 agent_id_base: int = 0, seed_stride: Optional[int] = None,
                 finish_percentage: float = FINISH_PERCENTAGE, variant: Union[int, str] = "cubic", lib=None):
        if not torch.cuda.is_available():
            raise _native.VoxnavError("BatchedGridEnv needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.lib = lib if lib is not None else _native.load()
        self.room_set = as_room_set(rooms, room_path, width, depth, height)
        self.num_agents = int(num_agents)
        self.local_map_length = int(local_map_length)
        if not 1 <= self.local_map_length <= _native.VN_MAX_L:
            raise ValueError(f"local_map_length must be in 1..{_native.VN_MAX_L}")
        self.crash_penalty = float(crash_penalty)
        self.autoreset = bool(autoreset)
        dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        if dev.type != "cuda":
            raise ValueError(f"device must be a GPU, got {dev}")
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.agent_id_base = int(agent_id_base)
        self.seed_stride = int(seed_stride) if seed_stride is not None else self.num_agents
        self.variant = _variant_code(variant)
        whd, walls, fs, gl = self.room_set.pack(self.variant)
        rs = _native.VnRoomSet(len(self.room_set), whd.ctypes.data, walls.ctypes.data, fs.ctypes.data,
                               gl.ctypes.data)
        cfg = _native.VnConfig(self.local_map_length, int(self.room_set.use_room_draw), int(self.autoreset),
                               self.variant, self.crash_penalty, float(finish_percentage), self.agent_id_base,
                               self.seed_stride)
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            _native.check(self.lib.vn_create(C.byref(rs), self.num_agents, C.byref(cfg), self.device.index,
                                             C.byref(h)), "vn_create")
        self._h = h
        info = _native.VnInfo()
        _native.check(self.lib.vn_get_info(self._h, C.byref(info)), "vn_get_info")
        self.info = info
        self.obs_dim = int(info.obs_dim)
        self.total_free_cells = np.asarray([r.total_free_cells_for(self.variant) for r in self.room_set.rooms],
                                           dtype=np.int64)
        self._was_reset = False
        self._t = 0   # global step counter for the random policy stream

    # ------------------------------------------------------------------ utils
    def close(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            self.lib.vn_destroy(h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        return _stream_ptr(self.device)

    def _seeds_tensor(self, seed) -> torch.Tensor:
        N = self.num_agents
        if seed is None:
            s = np.frombuffer(os.urandom(8 * N), dtype=np.uint64) % np.uint64(SEED_LIMIT)
            arr = s.astype(np.int64)
        elif isinstance(seed, (int, np.integer)):
            arr = int(seed) + self.agent_id_base + np.arange(N, dtype=np.int64)
        else:
            arr = np.asarray(seed.cpu() if isinstance(seed, torch.Tensor) else seed, dtype=np.int64).reshape(-1)
            if arr.size != N:
                raise ValueError(f"expected {N} seeds, got {arr.size}")
        if (arr < 0).any() or (arr >= SEED_LIMIT).any():
            raise ValueError("Seed must be between 0 and 2**32 - 1")   # np.random.seed (envs/CubicEnv.py:80)
        return torch.as_tensor(arr, dtype=torch.int64).to(self.device)

    # ------------------------------------------------------------------ API
    def reset(self, seed=None, mask: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None):
        """GridAgent.reset(seed) for all agents (or those with mask[i]).

        Returns obs f32 [N, obs_dim] (rows of unmasked agents are left as in
        ``out`` / zero).
        """
        seeds = self._seeds_tensor(seed)
        if out is None:
            out = torch.zeros((self.num_agents, self.obs_dim), dtype=torch.float32, device=self.device)
        m = None
        if mask is not None:
            m = mask.to(device=self.device, dtype=torch.uint8).contiguous()
        _native.check(self.lib.vn_reset(self._h, _ptr(seeds), _ptr(m), _ptr(out), self._stream()), "vn_reset")
        self._was_reset = True
        return out

    def step(self, actions, reward_f64: bool = False, terminal_obs: bool = True) -> StepResult:
        """GridAgent.step(a) for every agent + SB3 auto-reset (envs/CubicEnv.py:110-132)."""
        if not self._was_reset:
            raise RuntimeError("call reset() before step()")
        N = self.num_agents
        a = torch.as_tensor(actions, device=self.device).to(torch.int32).reshape(N).contiguous()
        obs = torch.empty((N, self.obs_dim), dtype=torch.float32, device=self.device)
        rew = torch.empty(N, dtype=torch.float64 if reward_f64 else torch.float32, device=self.device)
        te = torch.empty(N, dtype=torch.uint8, device=self.device)
        tr = torch.empty(N, dtype=torch.uint8, device=self.device)
        tob = torch.zeros((N, self.obs_dim), dtype=torch.float32, device=self.device) if (terminal_obs and self.autoreset) else None
        _native.check(self.lib.vn_step(self._h, _ptr(a), _ptr(obs), None if reward_f64 else _ptr(rew),
                                       _ptr(rew) if reward_f64 else None, _ptr(te), _ptr(tr), _ptr(tob),
                                       self._stream()), "vn_step")
        return StepResult(obs, rew, te.bool(), tr.bool(), tob)

    def step_into(self, actions: torch.Tensor, obs: torch.Tensor, reward: torch.Tensor, terminated: torch.Tensor,
                  truncated: torch.Tensor, terminal_obs: Optional[torch.Tensor] = None,
                  reward64: Optional[torch.Tensor] = None):
        """``step`` writing into caller-owned device buffers (no allocation):
        actions i32 [N], obs f32 [N, obs_dim], reward f32 (or f64) [N],
        terminated / truncated u8 [N], terminal_obs f32 [N, obs_dim] or None;
        ``reward64`` (f64 [N], with an f32 ``reward``) also receives the exact
        f64 reward (what the Monitor sums)."""
        if not self._was_reset:
            raise RuntimeError("call reset() before step()")
        N = self.num_agents
        for name, t, dt, shape in (("actions", actions, torch.int32, (N,)), ("obs", obs, torch.float32, (N, self.obs_dim)),
                                   ("terminated", terminated, torch.uint8, (N,)),
                                   ("truncated", truncated, torch.uint8, (N,))):
            if t.dtype != dt or tuple(t.shape) != shape or not t.is_contiguous() or t.device != self.device:
                raise ValueError(f"{name}: expected contiguous {dt} {shape} on {self.device}")
        if reward.dtype not in (torch.float32, torch.float64) or tuple(reward.shape) != (N,) or not reward.is_contiguous():
            raise ValueError("reward: expected contiguous f32/f64 [N]")
        f64 = reward.dtype == torch.float64
        if reward64 is not None:
            if f64 or reward64.dtype != torch.float64 or tuple(reward64.shape) != (N,) or not reward64.is_contiguous():
                raise ValueError("reward64: expected contiguous f64 [N] next to an f32 reward")
        r64 = reward if f64 else reward64
        _native.check(self.lib.vn_step(self._h, _ptr(actions), _ptr(obs), None if f64 else _ptr(reward),
                                       _ptr(r64), _ptr(terminated), _ptr(truncated),
                                       _ptr(terminal_obs), self._stream()), "vn_step")

    def step_random(self, k_steps: int, policy_seed: int = 42, t0: Optional[int] = None, record_actions: bool = False,
                    reward_f64: bool = False, out: Optional[Rollout] = None) -> Rollout:
        """k fused steps under the build's Philox uniform random policy."""
        if not self._was_reset:
            raise RuntimeError("call reset() before step_random()")
        K, N = int(k_steps), self.num_agents
        if t0 is None:
            t0 = self._t
        if out is None:
            obs = torch.empty((K, N, self.obs_dim), dtype=torch.float32, device=self.device)
            rew = torch.empty((K, N), dtype=torch.float64 if reward_f64 else torch.float32, device=self.device)
            te = torch.empty((K, N), dtype=torch.uint8, device=self.device)
            tr = torch.empty((K, N), dtype=torch.uint8, device=self.device)
            act = torch.empty((K, N), dtype=torch.int32, device=self.device) if record_actions else None
        else:
            self._check_rollout(out, K, reward_f64)
            obs, rew, te, tr, act = out
        _native.check(self.lib.vn_step_random(self._h, int(policy_seed), int(t0), K, _ptr(act), _ptr(obs),
                                              None if reward_f64 else _ptr(rew), _ptr(rew) if reward_f64 else None,
                                              _ptr(te), _ptr(tr), None, self._stream()), "vn_step_random")
        self._t = int(t0) + K
        return Rollout(obs, rew, te, tr, act)

    def _check_rollout(self, out: Rollout, K: int, reward_f64: bool):
        """A caller-owned [K, N, ...] rollout chunk: the kernel writes all K
        steps, so a short or mistyped buffer is refused here."""
        N, dev = self.num_agents, self.device
        obs, rew, te, tr, act = out
        rdt = torch.float64 if reward_f64 else torch.float32
        for name, t, dt, shape in (("obs", obs, torch.float32, (K, N, self.obs_dim)), ("reward", rew, rdt, (K, N)),
                                   ("terminated", te, torch.uint8, (K, N)), ("truncated", tr, torch.uint8, (K, N))):
            if t.dtype != dt or tuple(t.shape) != shape or not t.is_contiguous() or t.device != dev:
                raise ValueError(f"out.{name}: expected contiguous {dt} {shape} on {dev}")
        if act is not None and (act.dtype != torch.int32 or tuple(act.shape) != (K, N) or not act.is_contiguous()
                                or act.device != dev):
            raise ValueError(f"out.actions: expected contiguous int32 {(K, N)} on {dev}")

    def step_random_launcher(self, k_steps: int, policy_seed: int, t0: int, out: Rollout, reward_f64: bool = False):
        """``step_random(k_steps, policy_seed, t0, out=out)`` prepared: the
        argument checks and conversions happen here, and the returned
        zero-argument callable is one C call on the current stream (for timed
        loops whose host overhead per launch should be the launch itself)."""
        if not self._was_reset:
            raise RuntimeError("call reset() before step_random()")
        K = int(k_steps)
        self._check_rollout(out, K, reward_f64)
        obs, rew, te, tr, act = out
        args = (self._h, int(policy_seed), int(t0), K, _ptr(act), _ptr(obs), None if reward_f64 else _ptr(rew),
                _ptr(rew) if reward_f64 else None, _ptr(te), _ptr(tr), None, self._stream())
        fn = self.lib.vn_step_random
        t_end = int(t0) + K

        def launch():
            rc = fn(*args)
            if rc:
                _native.check(rc, "vn_step_random")
            self._t = t_end          # a later step_random() without t0 continues after this launch
        launch.out = out             # args holds raw device pointers: keep the tensors alive with the callable
        return launch

    def kernel_label(self, k_steps: int = 16, explicit_actions: bool = False, fast: bool = True) -> str:
        """Name of the kernel instantiation a step call of this shape launches
        (``k_steps=0``: reset; ``fast``: the rollout-buffer call)."""
        buf = C.create_string_buffer(160)
        _native.check(self.lib.vn_kernel_label(self._h, int(k_steps), int(bool(explicit_actions)), int(bool(fast)),
                                               buf, 160), "vn_kernel_label")
        return buf.value.decode()

    def export_state(self) -> torch.Tensor:
        out = torch.empty((self.num_agents, _native.VN_STATE_FIELDS), dtype=torch.int64, device=self.device)
        _native.check(self.lib.vn_export_state(self._h, _ptr(out), self._stream()), "vn_export_state")
        return out

    def state(self) -> dict:
        s = self.export_state().cpu().numpy()
        return {f: s[:, i] for i, f in enumerate(_native.STATE_FIELDS)}

    def belief(self) -> torch.Tensor:
        """int8 [N, pad_w, pad_d, pad_h], the reference's internal_grid values
        (CubicEnv: counts saturate at 63; simpleEnv: -1/0/1/2); -128 outside
        the agent's room."""
        i = self.info
        out = torch.empty((self.num_agents, i.pad_w, i.pad_d, i.pad_h), dtype=torch.int8, device=self.device)
        _native.check(self.lib.vn_export_belief(self._h, _ptr(out), self._stream()), "vn_export_belief")
        return out
