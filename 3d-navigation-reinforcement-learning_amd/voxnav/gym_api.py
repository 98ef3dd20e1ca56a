"""``GridAgent``: the reference's single-env gymnasium API on the HIP path.

Same constructor, ``reset``/``step`` signatures, spaces and the attributes
callers read (``visited_count``, ``bump_count``, ``total_free_cells``,
``done``, ``get_position()`` -- train/Grid_Train.py:114-116,
train/evaluate_grid.py:210-218) as ``envs/CubicEnv.GridAgent``
(envs/CubicEnv.py:15-538), backed by a one-agent ``BatchedGridEnv``
without auto-reset.  The reward is returned as a Python/NumPy float64
exactly as the reference computes it.

``SimpleGridAgent`` is the same facade for the goal-seeking variant
``envs/simpleEnv.GridAgent`` (envs/simpleEnv.py:13-521).

Differences kept deliberately small:
  * rooms are parsed once at construction (the reference re-reads the file
    at every reset); the room list is sorted by file name;
  * ``internal_grid`` visit counts saturate at 63 (observationally exact:
    the obs clips at 20 and the reward caps at 25);
  * ``render_mode="matplotlib"`` is not provided (text render only).
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from .env import BatchedGridEnv
from .spaces import Box, Discrete, EnvBase


class GridAgent(EnvBase):
    metadata = {"render_modes": ["human"]}

    def __init__(self, grid=None, max_steps=2000, width: int = 20, depth: int = 20, height: int = 12,
                 cell_size: float = 0.25, local_map_length=4, room_path=None, render_mode: Optional[str] = None,
                 crash_penalty: float = -2.0, device=None, rooms=None):
        self.width, self.depth, self.height = int(width), int(depth), int(height)
        self.cell_size = cell_size
        self.local_map_length = int(local_map_length)
        self.max_steps = max_steps
        self.crash_penalty = crash_penalty
        self.render_mode = render_mode
        self.valid_facings = {0: "north", 1: "east", 2: "south", 3: "west"}
        self.action_space = Discrete(6)
        self.observation_space = Box(low=np.full(80, -1.0, dtype=np.float32), high=np.full(80, 1.0, dtype=np.float32),
                                     dtype=np.float32)
        self._env = BatchedGridEnv(num_agents=1, room_path=room_path, rooms=rooms,
                                   local_map_length=self.local_map_length, crash_penalty=crash_penalty,
                                   width=width, depth=depth, height=height, autoreset=False, device=device)
        self.rooms = [r.name for r in self._env.room_set.rooms] if self._env.room_set.use_room_draw else None
        self.total_free_cells = 1
        self._st = None

    # ------------------------------------------------------------------ gym API
    def reset(self, seed: Optional[int] = None, options: Optional[dict] = None):
        obs = self._env.reset(seed=None if seed is None else [int(seed)])
        self._refresh()
        room = self._env.room_set.rooms[self._st["room"]]
        self.width, self.depth, self.height = room.shape
        self.total_free_cells = room.total_free_cells
        self.max_steps = self.total_free_cells
        out = obs[0].cpu().numpy()
        if self.render_mode == "human":
            self.render()
        return out, {}

    def step(self, action):
        if not self.action_space.contains(action):
            raise KeyError(action)   # the reference's action_map lookup (envs/CubicEnv.py:153)
        res = self._env.step([int(action)], reward_f64=True, terminal_obs=False)
        obs = res.obs[0].cpu().numpy()
        reward = np.float64(res.reward[0].item())
        self._refresh()
        if self.render_mode == "human":
            self.render()
        return obs, reward, bool(res.terminated[0].item()), bool(res.truncated[0].item()), {}

    def close(self):
        self._env.close()

    # ------------------------------------------------------------------ attributes
    def _refresh(self):
        s = self._env.export_state()[0].cpu().numpy()
        from ._native import STATE_FIELDS
        self._st = {f: int(v) for f, v in zip(STATE_FIELDS, s)}

    def __getattr__(self, name):
        st = self.__dict__.get("_st")
        if st is not None:
            alias = {"done": "done", "visited_count": "visited_count", "bump_count": "bump_count",
                     "step_count": "step_count", "facing": "facing", "last_action": "last_action",
                     "x": "x", "y": "y", "z": "z", "near_wall": "near_wall", "was_near_wall": "was_near_wall",
                     "last_bump": "last_bump", "cells_insight_down": "cells_insight_down"}
            if name in alias:
                v = st[alias[name]]
                return bool(v) if name in ("done", "near_wall", "was_near_wall", "last_bump") else v
        raise AttributeError(name)

    def get_position(self):
        return (self.x, self.y, self.z)

    @property
    def internal_grid(self) -> np.ndarray:
        b = self._env.belief()[0].cpu().numpy().astype(np.int64)
        return b[: self.width, : self.depth, : self.height]

    @property
    def grid(self) -> np.ndarray:
        return self._env.room_set.rooms[self._st["room"]].grid()

    # ------------------------------------------------------------------ render
    def render(self):
        if self.render_mode == "human":
            self._render_text()

    def _render_text(self):
        ig = self.internal_grid
        print(f"--- Step: {self.step_count}, Pos: ({self.x}, {self.y}, {self.z}), "
              f"Facing: {self.valid_facings[self.facing]} ---")
        g = ig[:, :, self.z].copy()
        g[self.x, self.y] = 9
        for y in range(self.depth):
            row = ""
            for x in range(self.width):
                v = g[x, y]
                row += "A " if v == 9 else "# " if v == -2 else ". " if v >= 1 else "o " if v == 0 else "? "
            print(row)
        print("-" * (self.width * 2))


class SimpleGridAgent(EnvBase):
    """``envs/simpleEnv.GridAgent`` (goal-seeking variant) on the HIP path;
    a ``gymnasium.Env`` when gymnasium is importable, as the reference's
    (envs/simpleEnv.py:13).

    Same constructor, spaces, ``reset`` (returns None, :79-107), ``step``
    (:109-150) and ``get_obs`` as the reference.  The reference's reset
    draws from the global ``random`` without seeding; here ``reset(seed)``
    seeds the draws with ``random.seed(seed)`` (``seed=None``: OS entropy).
    ``get_obs()`` returns the observation of the last reset/step (the
    reference re-senses; sensing twice from the same cell only differs in
    the edge-of-room quirk at :311-319)."""

    metadata = {"render_modes": ["human"]}

    def __init__(self, grid=None, max_steps=2000, width: int = 20, depth: int = 20, height: int = 12,
                 cell_size: float = 0.25, local_map_length=4, room_path=None, render_mode: Optional[str] = None,
                 device=None, rooms=None):
        self.width, self.depth, self.height = int(width), int(depth), int(height)
        self.cell_size = cell_size
        self.local_map_length = L = int(local_map_length)
        self.max_steps = max_steps
        self.render_mode = render_mode
        self.valid_facings = {0: "north", 1: "east", 2: "south", 3: "west"}
        self.action_space = Discrete(6)
        self.observation_space = Box(                                   # :60-67
            low=np.array([-1] * (6 * L) + [0] * 6 + [0], dtype=np.float32),
            high=np.array([2] * (6 * L) + [np.inf] * 6 + [5], dtype=np.float32), dtype=np.float32)
        self._env = BatchedGridEnv(num_agents=1, room_path=room_path, rooms=rooms, local_map_length=L,
                                   width=width, depth=depth, height=height, autoreset=False, device=device,
                                   variant="simple")
        self.rooms = [r.name for r in self._env.room_set.rooms] if self._env.room_set.use_room_draw else None
        self.total_free_cells = 1
        self._st = None
        self._obs = None

    def reset(self, seed: Optional[int] = None, options: Optional[dict] = None):
        obs = self._env.reset(seed=None if seed is None else [int(seed)])
        self._refresh()
        room = self._env.room_set.rooms[self._st["room"]]
        self.width, self.depth, self.height = room.shape
        self.total_free_cells = room.total_free_cells_for(1)
        self.max_steps = self.total_free_cells
        self._obs = obs[0].cpu().numpy()
        return None

    def get_obs(self):
        if self._obs is None:
            raise RuntimeError("call reset() first")
        return self._obs.copy()

    def step(self, action):
        if not self.action_space.contains(action):
            raise KeyError(action)   # self.action_map[action] (envs/simpleEnv.py:161)
        res = self._env.step([int(action)], reward_f64=True, terminal_obs=False)
        self._obs = res.obs[0].cpu().numpy()
        reward = np.float64(res.reward[0].item())
        self._refresh()
        if self.render_mode == "human":
            self.render()
        return self._obs.copy(), reward, bool(res.terminated[0].item()), bool(res.truncated[0].item()), {}

    def close(self):
        self._env.close()

    def _refresh(self):
        s = self._env.export_state()[0].cpu().numpy()
        self._st = {"x": int(s[0]), "y": int(s[1]), "z": int(s[2]), "facing": int(s[3]), "last_action": int(s[4]),
                    "step_count": int(s[5]), "visited_count": int(s[6]), "bump_count": int(s[7]),
                    "done": bool(s[8]), "gx": int(s[9]), "gy": int(s[10]), "gz": int(s[11]), "room": int(s[13])}

    def __getattr__(self, name):
        st = self.__dict__.get("_st")
        if st is not None and name in st and name != "room":
            return st[name]
        raise AttributeError(name)

    def get_position(self):
        return (self.x, self.y, self.z)

    @property
    def internal_grid(self) -> np.ndarray:
        b = self._env.belief()[0].cpu().numpy().astype(np.int64)
        return b[: self.width, : self.depth, : self.height]

    @property
    def grid(self) -> np.ndarray:
        """simpleEnv's self.grid: 2 = wall (the -2 tokens of a file read 0 here)."""
        room = self._env.room_set.rooms[self._st["room"]]
        return np.where(room.walls_for(1), 2, 0).astype(np.int64)

    def render(self):
        if self.render_mode == "human":
            ig = self.internal_grid
            print(f"--- Step: {self.step_count}, Pos: ({self.x}, {self.y}, {self.z}), "
                  f"Facing: {self.valid_facings[self.facing]} ---")
            g = ig[:, :, self.z].copy()
            g[self.x, self.y] = 9
            for y in range(self.depth):
                print("".join("A " if v == 9 else "# " if v == 2 else ". " if v == 1 else "o " if v == 0 else "? "
                              for v in (g[x, y] for x in range(self.width))))
            print("-" * (self.width * 2))
