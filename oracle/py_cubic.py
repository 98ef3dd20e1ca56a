"""Per-agent Python/NumPy restatement of envs/CubicEnv.GridAgent -- TEST
INFRASTRUCTURE / CPU BASELINE ONLY.

Only ``tests/`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module; the product package never does.

This is the "reference's Python/NumPy CPU step loop" that BASELINE.json's
``north_star`` asks to time on the GPU box's host cores.  The reference
source cannot travel to the box, so this is a from-scratch restatement of
the same per-agent algorithm in the same idiom (one env object, NumPy
belief map, Python loops over rays and the 4x4x4 window, CPython
``random`` for the reset draws):

* ``reset``         -- envs/CubicEnv.py:77-108, room / start draw :402-466
* ``step``          -- :110-132 (near-wall transfer, truncation, action,
                       obs, reward, last_action)
* ``_move``         -- ``do_action`` :134-166 + ``_mark_visited`` :322-343
* ``_ray``          -- ``_sense_direction`` :345-397
* ``_observe``      -- ``get_obs`` :254-312 + ``_get_3d_local_map`` :229-251
* ``_reward``       -- ``compute_reward`` :169-224 (f64, same op order)

Pinned by tests/test_py_cubic.py against every golden trajectory the
unmodified reference produced (tests/golden/traj_*.npz): obs bytes, f64
reward, flags and the 13 state fields, step by step.

``python -m oracle.py_cubic --room 32x32x8 --L 10 --start-at T --stop-at T2``
runs one env under a random policy between two wall-clock instants and
prints ``{"steps": n}``: bench.py starts P of these (the SubprocVecEnv
shape, Grid_Train.py:191-192: one env per process) for the CPU baseline.
"""
from __future__ import annotations

import random
from typing import Optional, Sequence

import numpy as np

FINISH_PERCENTAGE = 0.84          # envs/CubicEnv.py:12
WALL = -2
UNKNOWN = -1

# horizontal moves by (relative action, facing): envs/CubicEnv.py:135-140
_MOVES = (
    ((0, 1, 0), (1, 0, 0), (0, -1, 0), (-1, 0, 0)),    # forward
    ((1, 0, 0), (0, -1, 0), (-1, 0, 0), (0, 1, 0)),    # right
    ((0, -1, 0), (-1, 0, 0), (0, 1, 0), (1, 0, 0)),    # backward
    ((-1, 0, 0), (0, 1, 0), (1, 0, 0), (0, -1, 0)),    # left
)
# sensing order of get_obs (:256-266): forward, left, right, backward, up, down
_RAY_REL = (0, 3, 1, 2)


def _heading(v) -> int:
    """Facing after a horizontal move (:148-151)."""
    if v[1] == 1:
        return 0
    if v[0] == 1:
        return 1
    if v[1] == -1:
        return 2
    return 3


class PyCubicAgent:
    """One CubicEnv agent.  ``rooms`` are OracleRoom-like objects (``.grid``
    int64 [W, D, H], walls == -2, optional ``.start``); ``use_room_draw``
    False is the ctor box (no room draw, :440-448)."""

    def __init__(self, rooms: Sequence, local_map_length: int = 4, crash_penalty: float = -2.0,
                 use_room_draw: bool = True):
        self.rooms = list(rooms)
        self.L = int(local_map_length)
        self.crash_penalty = float(crash_penalty)
        self.use_room_draw = bool(use_room_draw)
        self._starts = []
        for r in self.rooms:
            W, D, H = r.grid.shape
            free = [(x, y, z) for x in range(1, W - 1) for y in range(1, D - 1) for z in range(1, H - 1)
                    if r.grid[x, y, z] != WALL]
            self._starts.append(free)

    # ------------------------------------------------------------- reset
    def reset(self, seed: Optional[int] = None) -> np.ndarray:
        rng = random.Random(seed)
        k = rng.choice(range(len(self.rooms))) if self.use_room_draw else 0
        room = self.rooms[k]
        self.room_index = k
        self.grid = room.grid
        self.W, self.D, self.H = self.grid.shape
        starts = self._starts[k]
        self.total_free_cells = len(starts)
        self.max_steps = self.total_free_cells
        s = getattr(room, "start", None)
        if s is None:
            s = rng.choice(starts)
        if self.grid[s] == WALL:
            s = rng.choice(starts)
        self.x, self.y, self.z = s
        self.belief = np.full(self.grid.shape, UNKNOWN, dtype=np.int64)
        self.belief[s] = 1
        self.visited_count = 1
        self.step_count = 0
        self.bump_count = 0
        self.facing = 0
        self.last_action = 0
        self.done = self.explored = self.bumped = self.last_bump = False
        self.near_wall = self.was_near_wall = False
        self.cells_insight_down = 0
        return self._observe()

    # -------------------------------------------------------------- step
    def step(self, action: int):
        action = int(action)
        if self.near_wall:
            self.near_wall = False
            self.was_near_wall = True
        self.step_count += 1
        truncated = self.step_count >= self.max_steps
        self._move(action)
        obs = self._observe()
        reward = self._reward(action, truncated)
        self.last_action = action
        return obs, reward, self.done, truncated

    def _inside(self, x, y, z) -> bool:
        return 0 <= x < self.W and 0 <= y < self.D and 0 <= z < self.H

    def _move(self, a: int):
        if a < 4:
            v = _MOVES[a][self.facing]
            self.facing = _heading(v)
        else:
            v = (0, 0, 1) if a == 4 else (0, 0, -1)
        nx, ny, nz = self.x + v[0], self.y + v[1], self.z + v[2]
        b = self.belief
        if self._inside(nx, ny, nz) and self.grid[nx, ny, nz] != WALL:
            c = b[nx, ny, nz]
            if c == 0:
                b[nx, ny, nz] = 1
                self.visited_count += 1
                self.explored = True
            elif c > 0:
                b[nx, ny, nz] = c + 1
            self.x, self.y, self.z = nx, ny, nz
        else:
            self.bumped = True
        if self._inside(self.x, self.y, self.z) and self.grid[self.x, self.y, self.z] != WALL:
            b[self.x, self.y, self.z] += 1

    def _ray(self, d) -> int:
        free = 0
        x, y, z = self.x, self.y, self.z
        g, b = self.grid, self.belief
        for s in range(1, self.L + 1):
            x += d[0]
            y += d[1]
            z += d[2]
            if not self._inside(x, y, z):
                break
            if g[x, y, z] == WALL:
                b[x, y, z] = WALL
                if s == 1:
                    self.near_wall = True
                break           # cells behind the first wall are never touched
            free += 1
            if b[x, y, z] == UNKNOWN:
                b[x, y, z] = 0
        return free

    def _observe(self) -> np.ndarray:
        f = self.facing
        for rel in _RAY_REL:
            self._ray(_MOVES[rel][f])
        self._ray((0, 0, 1))
        self.cells_insight_down = self._ray((0, 0, -1))
        win = np.full(64, UNKNOWN, dtype=np.float32)
        b = self.belief
        i = 0
        for dx in (-2, -1, 0, 1):
            for dy in (-2, -1, 0, 1):
                for dz in (-2, -1, 0, 1):
                    px, py, pz = self.x + dx, self.y + dy, self.z + dz
                    if self._inside(px, py, pz):
                        win[i] = b[px, py, pz]
                    i += 1
        win = (np.clip(win, -2, 20.0) + 2) / np.float32(22.0)
        obs = np.zeros(80, dtype=np.float32)
        obs[:64] = win
        obs[64 + f] = 1.0
        obs[68] = self.last_action / 5.0
        obs[69] = float(self.was_near_wall)
        obs[70] = float(self.last_bump)
        obs[71] = self.cells_insight_down / self.L
        obs[72] = self.visited_count / self.total_free_cells
        return obs

    def _reward(self, a: int, truncated: bool) -> float:
        r = -0.05
        r -= min(int(self.belief[self.x, self.y, self.z]) * 0.02, 0.5)
        if self.bumped:
            self.bumped = False
            self.last_bump = True
            self.bump_count += 1
            r += self.crash_penalty
        else:
            self.last_bump = False
            if self.was_near_wall:
                self.was_near_wall = False
                r += 0.15
            if self.last_action != 2 and a == self.last_action and self.last_action < 4:
                r += 0.05
            if self.last_action == 2 and a == 2:
                r -= 0.5
        if self.explored:
            self.explored = False
            r += 1.0
        if self.visited_count / self.total_free_cells >= FINISH_PERCENTAGE:
            self.done = True
            r += 100.0
        if truncated:
            r += -5.0
        return r

    def state(self) -> dict:
        return dict(x=self.x, y=self.y, z=self.z, facing=self.facing, last_action=self.last_action,
                    step_count=self.step_count, visited_count=self.visited_count, bump_count=self.bump_count,
                    done=int(self.done), last_bump=int(self.last_bump), near_wall=int(self.near_wall),
                    was_near_wall=int(self.was_near_wall), cells_insight_down=self.cells_insight_down)


def _run_timed(room_whd, L, seed, start_at, stop_at):
    """One env under a uniform random policy, stepped from wall-clock
    ``start_at`` until ``stop_at`` (VecEnv auto-reset on done)."""
    import time
    from oracle.oracle import parse_room_text
    W, D, H = room_whd
    lines = [f"Size={W},{D},{H}"]
    for z in range(H):
        lines.append(f"Layer z={z}")
        for y in range(D):
            lines.append(" ".join("2" if (x in (0, W - 1) or y in (0, D - 1) or z in (0, H - 1)) else "0"
                                  for x in range(W)))
    env = PyCubicAgent([parse_room_text("\n".join(lines))], local_map_length=L, use_room_draw=True)
    acts = np.random.default_rng(seed).integers(0, 6, size=1 << 16)
    env.reset(seed)
    episodes = 0
    while time.time() < start_at:
        time.sleep(0.001)
    n = 0
    while True:
        for a in acts[(n & 0xFFFF):(n & 0xFFFF) + 256]:
            _, _, te, tr = env.step(a)
            if te or tr:
                episodes += 1
                env.reset(seed + episodes * 1_000_003)
        n += 256
        if time.time() >= stop_at:
            break
    return n, episodes


if __name__ == "__main__":
    import argparse
    import json
    ap = argparse.ArgumentParser()
    ap.add_argument("--room", default="32x32x8")
    ap.add_argument("--L", type=int, default=10)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--start-at", type=float, required=True)
    ap.add_argument("--stop-at", type=float, required=True)
    a = ap.parse_args()
    whd = tuple(int(v) for v in a.room.split("x"))
    n, ep = _run_timed(whd, a.L, a.seed, a.start_at, a.stop_at)
    print(json.dumps({"steps": n, "episodes": ep}), flush=True)
