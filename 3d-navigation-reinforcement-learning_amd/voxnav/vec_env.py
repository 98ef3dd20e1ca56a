"""``VoxnavVecEnv``: SB3's VecEnv contract over ``BatchedGridEnv`` -- the
literal drop-in at the reference's call site.

train/Grid_Train.py builds its training env as
``SubprocVecEnv([make_env_fn(train_path, ray_len, i) for i in range(NUM_ENVS)])``
(:191-192), each worker a ``Monitor(GridEnv(...))`` reset once with
``seed=BASE_SEED + i`` (:120-126), and hands it to
``RecurrentPPO("MlpLstmPolicy", env, ...)`` (:199-205).  This class is what
that line becomes::

    train_env = VoxnavVecEnv(NUM_ENVS, room_path=train_path, local_map_length=ray_len, seed=BASE_SEED)

It keeps SB3's ``VecEnv`` surface (stable_baselines3/common/vec_env/
base_vec_env.py + subproc_vec_env.py; SB3 is not installed here, so the
contract is restated in SURVEY.md Appendix D.1 and tested against the CPU
oracle's auto-reset replay):

* ``num_envs``, ``observation_space`` (Box f32[80] in [-1, 1], CubicEnv.py:58-62;
  6L+7 for the simpleEnv variant), ``action_space`` (Discrete(6), :56),
  ``render_mode``;
* ``reset() -> obs`` f32 [N, obs_dim] (numpy), ``reset_infos``;
* ``step_async(actions)`` / ``step_wait() -> (obs, rewards, dones, infos)``:
  ``rewards`` f64 [N] (``np.stack`` of the workers' np.float64 rewards),
  ``dones`` bool [N] (terminated or truncated), and per env an info dict
  with ``"TimeLimit.truncated"`` (truncated and not terminated), on done
  ``"terminal_observation"`` (the last obs of the finished episode; ``obs``
  then holds the next episode's first one) and the Monitor's
  ``"episode": {"r": round(sum of f64 rewards, 6), "l": length,
  "t": round(seconds since the monitor started, 6)}``;
* ``seed``, ``close``, ``get_attr`` / ``set_attr`` / ``env_method`` /
  ``env_is_wrapped`` for the attributes SB3 and Grid_Train read
  (``visited_count``, ``bump_count``, ``total_free_cells``, ``done``,
  ``render_mode``; ``env_is_wrapped(Monitor)`` is True with the monitor on).

The step runs on the GPU (``vn_step`` + ``vn_monitor_step``); the VecEnv
contract then costs one device->host copy of obs / rewards / flags per
step and N info dicts built on the host, as SubprocVecEnv's pipes did.
The policy-in-the-loop collector (``voxnav.RolloutCollector``) is the path
with nothing on the host per step.

Seeds: the first ``reset()`` seeds env i with ``seed + agent_id_base + i``
(``make_env_fn``'s ``BASE_SEED + i``); ``seed(s)`` sets the seeds of the
next ``reset()`` to ``s + i`` (SB3's ``VecEnv.seed``).  Auto-reset seeds
follow the pinned schedule of ``BatchedGridEnv`` (SB3 auto-resets with
``seed=None``).
"""
from __future__ import annotations

import time
from typing import Any, List, Optional, Sequence, Union

import numpy as np
import torch

from .env import NUM_ACTIONS, BatchedGridEnv
from .monitor import EpisodeMonitor
from .spaces import Box, Discrete

try:  # pragma: no cover - only where stable-baselines3 is installed
    from stable_baselines3.common.vec_env.base_vec_env import VecEnv as _VecEnvBase  # type: ignore
    HAVE_SB3 = True
except Exception:  # noqa: BLE001
    _VecEnvBase = object
    HAVE_SB3 = False

# GridEnv / GridAgent attributes get_attr serves from the device state
_STATE_ATTRS = ("visited_count", "bump_count", "step_count", "done", "facing", "last_action", "x", "y", "z",
                "near_wall", "was_near_wall", "last_bump", "cells_insight_down")
_BOOL_ATTRS = ("done", "near_wall", "was_near_wall", "last_bump")


def build_infos(terminated: np.ndarray, truncated: np.ndarray, terminal_obs: Optional[np.ndarray],
                ep_return: Optional[np.ndarray], ep_length: Optional[np.ndarray], elapsed: float) -> List[dict]:
    """The per-env info dicts of one VecEnv step (SURVEY.md Appendix D.1 and
    SB3's Monitor.step): ``TimeLimit.truncated`` for every env; for the envs
    whose episode ended, ``terminal_observation`` and (monitor on) ``episode``."""
    n = int(terminated.shape[0])
    tl = (truncated & ~terminated).tolist()
    infos: List[dict] = [{"TimeLimit.truncated": v} for v in tl]
    done_idx = np.flatnonzero(terminated | truncated)
    if done_idx.size:
        t = round(float(elapsed), 6)
        for i in done_idx.tolist():
            d = infos[i]
            if ep_return is not None:
                d["episode"] = {"r": round(float(ep_return[i]), 6), "l": int(ep_length[i]), "t": t}
            if terminal_obs is not None:
                d["terminal_observation"] = terminal_obs[i]
    assert len(infos) == n
    return infos


class VoxnavVecEnv(_VecEnvBase):
    """``SubprocVecEnv([Monitor(GridEnv(...)) ...])`` for ``num_envs`` agents on one GPU."""

    metadata = {"render_modes": []}

    def __init__(self, num_envs: int, room_path=None, rooms=None, local_map_length: int = 4,
                 crash_penalty: float = -2.0, seed: int = 42, device=None, monitor: bool = True,
                 variant: Union[int, str] = "cubic", agent_id_base: int = 0, seed_stride: Optional[int] = None,
                 width: int = 20, depth: int = 20, height: int = 12):
        self.env = BatchedGridEnv(num_agents=num_envs, room_path=room_path, rooms=rooms,
                                  local_map_length=local_map_length, crash_penalty=crash_penalty, width=width,
                                  depth=depth, height=height, autoreset=True, device=device,
                                  agent_id_base=agent_id_base, seed_stride=seed_stride, variant=variant)
        n, od = self.env.num_agents, self.env.obs_dim
        obs_space = Box(low=np.full(od, -1.0, dtype=np.float32), high=np.full(od, 1.0, dtype=np.float32),
                        dtype=np.float32)
        act_space = Discrete(NUM_ACTIONS)
        if HAVE_SB3:  # pragma: no cover
            super().__init__(n, obs_space, act_space)
        else:
            self.num_envs = n
            self.observation_space = obs_space
            self.action_space = act_space
        self.render_mode = None
        self.reset_infos: List[dict] = [{} for _ in range(n)]
        dev = self.env.device
        z = lambda *s, dt=torch.float32: torch.zeros(s, dtype=dt, device=dev)  # noqa: E731
        self._actions = z(n, dt=torch.int32)
        self._obs = z(n, od)
        self._rew = z(n)
        self._rew64 = z(n, dt=torch.float64)
        self._term = z(n, dt=torch.uint8)
        self._trunc = z(n, dt=torch.uint8)
        self._tobs = z(n, od)
        self.monitor = EpisodeMonitor(self.env.lib, n, 1, dev) if monitor else None
        self._base_seed = int(seed)
        self._reset_done = False
        self._next_seeds: Optional[np.ndarray] = None
        self._waiting = False
        self.closed = False

    # ------------------------------------------------------------------ VecEnv API
    def seed(self, seed: Optional[int] = None) -> Sequence[Optional[int]]:
        """SB3 ``VecEnv.seed``: the next ``reset()`` seeds env i with ``seed + i``."""
        if seed is None:
            self._next_seeds = None
            return [None] * self.num_envs
        self._next_seeds = int(seed) + np.arange(self.num_envs, dtype=np.int64)
        return self._next_seeds.tolist()

    def reset(self) -> np.ndarray:
        # SB3 resets its workers with seed=None after the first reset, so an
        # env's RNG continues: here the first reset takes the base seed (or
        # the seeds from seed()), later ones each agent's next seed of the
        # pinned auto-reset schedule (the state's next_seed field), so no
        # reset replays an earlier episode.  The Monitor's t_start stays at
        # construction, as Monitor's does.
        if self._next_seeds is not None:
            seeds = self._next_seeds
        elif not self._reset_done:
            seeds = self._base_seed
        else:
            seeds = self.env.export_state()[:, 15].to(torch.int64)
        self.env.reset(seed=seeds, out=self._obs)
        self._next_seeds = None
        self._reset_done = True
        if self.monitor is not None:
            self.monitor.ep_return.zero_()
            self.monitor.ep_length.zero_()
        self.reset_infos = [{} for _ in range(self.num_envs)]
        return self._obs.cpu().numpy()

    def step_async(self, actions) -> None:
        a = torch.as_tensor(np.asarray(actions) if not isinstance(actions, torch.Tensor) else actions)
        if a.numel() != self.num_envs:
            raise ValueError(f"expected {self.num_envs} actions, got {a.numel()}")
        a = a.reshape(self.num_envs)
        if a.is_floating_point() or (a.numel() and (int(a.min()) < 0 or int(a.max()) >= NUM_ACTIONS)):
            raise KeyError("actions must be integers in 0..5")   # GridAgent's action_map lookup (CubicEnv.py:153)
        self._actions.copy_(a.to(torch.int32))
        self._waiting = True

    def step_wait(self):
        if not self._waiting:
            raise RuntimeError("step_wait() without step_async()")
        self._waiting = False
        self.env.step_into(self._actions, self._obs, self._rew, self._term, self._trunc, self._tobs,
                           reward64=self._rew64)
        mon = self.monitor
        if mon is not None:
            mon.step(0, self._term, self._trunc, reward64=self._rew64)
        obs = self._obs.cpu().numpy()
        rew = self._rew64.cpu().numpy()
        te = self._term.cpu().numpy().astype(bool)
        tr = self._trunc.cpu().numpy().astype(bool)
        done = te | tr
        tobs = self._tobs.cpu().numpy() if done.any() else None
        ep_r = mon.rec_return[0].cpu().numpy() if mon is not None else None
        ep_l = mon.rec_length[0].cpu().numpy() if mon is not None else None
        infos = build_infos(te, tr, tobs, ep_r, ep_l, time.time() - mon.t_start if mon is not None else 0.0)
        if mon is not None and done.any():
            for i in np.flatnonzero(done).tolist():
                mon.ep_info_buffer.append(infos[i]["episode"])
            mon.total_episodes += int(done.sum())
        return obs, rew, done, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def close(self) -> None:
        if not self.closed:
            self.env.close()
            self.closed = True

    def render(self, mode: Optional[str] = None):
        return None

    def get_images(self) -> Sequence[Optional[np.ndarray]]:
        return [None] * self.num_envs

    # ------------------------------------------------------------------ attribute access
    def _indices(self, indices) -> List[int]:
        if indices is None:
            return list(range(self.num_envs))
        if isinstance(indices, (int, np.integer)):
            return [int(indices)]
        return [int(i) for i in indices]

    def get_attr(self, attr_name: str, indices=None) -> List[Any]:
        idx = self._indices(indices)
        if attr_name in _STATE_ATTRS:
            col = self.env.state()[attr_name]
            return [bool(col[i]) if attr_name in _BOOL_ATTRS else int(col[i]) for i in idx]
        if attr_name == "total_free_cells":
            room = self.env.state()["room"]
            return [int(self.env.total_free_cells[room[i]]) for i in idx]
        if attr_name == "local_map_length":
            return [self.env.local_map_length] * len(idx)
        if attr_name in ("render_mode", "observation_space", "action_space", "metadata"):
            return [getattr(self, attr_name)] * len(idx)
        raise AttributeError(f"VoxnavVecEnv envs have no attribute {attr_name!r}")

    def set_attr(self, attr_name: str, value: Any, indices=None) -> None:
        if attr_name == "render_mode":
            self.render_mode = value
            return
        raise AttributeError(f"VoxnavVecEnv cannot set {attr_name!r} (env state lives on the GPU)")

    def env_method(self, method_name: str, *method_args, indices=None, **method_kwargs) -> List[Any]:
        idx = self._indices(indices)
        if method_name == "get_position":
            st = self.env.state()
            return [(int(st["x"][i]), int(st["y"][i]), int(st["z"][i])) for i in idx]
        if method_name == "render":
            return [None] * len(idx)
        raise AttributeError(f"VoxnavVecEnv envs have no method {method_name!r}")

    def env_is_wrapped(self, wrapper_class, indices=None) -> List[bool]:
        name = getattr(wrapper_class, "__name__", str(wrapper_class))
        return [name == "Monitor" and self.monitor is not None] * len(self._indices(indices))

    def getattr_depth_check(self, name: str, already_found: bool):
        return type(self) if (hasattr(self, name) and already_found) else None

    @property
    def unwrapped(self):
        return self

    def __len__(self):
        return self.num_envs

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

