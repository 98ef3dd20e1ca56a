"""CPU oracle for the voxnav hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module.  The product package
(``voxnav``) never imports it.

Two pieces:

* ``parse_room_text`` -- a from-scratch restatement of the reference's
  room-file parser ``GridAgent.load_room`` (envs/CubicEnv.py:402-438),
  including its quirks (numpy-style negative layer indices,
  ``2 -> -2`` mapping at :434, width check at :435-436), and of the
  walled fallback box (:440-448).
* ``OracleEnv`` -- ctypes wrapper around ``lib/libvoxnav_oracle.so``
  (``voxnav_oracle.c``), the C restatement of reset/step/get_obs/reward
  (envs/CubicEnv.py:77-224, :229-397) with CPython ``random`` draws.

Parity pinning: tests/test_oracle_golden.py checks both pieces against
golden vectors produced by the unmodified reference env
(tests/golden/gen_golden.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass
from pathlib import Path
from typing import Optional, Sequence

import numpy as np

_HERE = Path(__file__).resolve().parent
_LIB_PATH = _HERE / "lib" / "libvoxnav_oracle.so"

OBS_DIM = 80
STATE_FIELDS = (
    "x", "y", "z", "facing", "last_action", "step_count", "visited_count", "bump_count",
    "done", "last_bump", "near_wall", "was_near_wall", "cells_insight_down", "room",
    "max_steps", "next_seed",
)


# --------------------------------------------------------------------------
# room parsing (envs/CubicEnv.py:402-448)
# --------------------------------------------------------------------------
@dataclass
class OracleRoom:
    name: str
    grid: np.ndarray                 # int64 [W, D, H], walls == -2  (CubicEnv's self.grid)
    start: Optional[tuple] = None    # "Start position" line, if any
    goal: Optional[tuple] = None     # "Goal" line, if any
    tokens: Optional[np.ndarray] = None   # raw file values (simpleEnv's self.grid, walls == 2)

    @property
    def whd(self):
        return tuple(int(v) for v in self.grid.shape)

    @property
    def walls(self) -> np.ndarray:
        return (self.grid == -2).astype(np.uint8)

    @property
    def simple_walls(self) -> np.ndarray:
        """simpleEnv walls: file value 2 only; a -2 token is free there (envs/simpleEnv.py:282, :381)."""
        t = self.tokens if self.tokens is not None else np.where(self.grid == -2, 2, self.grid)
        return (t == 2).astype(np.uint8)

    def walls_for(self, variant: int) -> np.ndarray:
        return self.simple_walls if variant else self.walls

    def interior_free(self):
        """(total_free_cells, start list) -- envs/CubicEnv.py:450-457."""
        W, D, H = self.grid.shape
        cells = []
        for x in range(1, W - 1):
            for y in range(1, D - 1):
                for z in range(1, H - 1):
                    if self.grid[x, y, z] != -2:
                        cells.append((x, y, z))
        return len(cells), cells


def parse_room_text(text: str, name: str = "<room>") -> OracleRoom:
    """Restates load_room's text branch, envs/CubicEnv.py:408-438."""
    grid = None
    tokens = None
    start = goal = None
    row = 0
    z = None
    for raw in text.splitlines(keepends=True):
        line = raw.strip()
        if not line:
            continue
        if line.startswith("Start position"):
            start = tuple(int(v) for v in line.split("=")[1].split(","))
        elif line.startswith("Goal"):
            goal = tuple(int(v) for v in line.split("=")[1].split(","))
        elif line.startswith("Size"):
            d = line.split("=")[1].split(",")
            W, D, H = int(d[0]), int(d[1]), int(d[2])
            grid = np.zeros((W, D, H), dtype=np.int64)
            tokens = np.zeros((W, D, H), dtype=np.int64)
        elif line.startswith("Layer"):
            z = int(line.split("=")[1])
            row = 0
        else:
            raw = [int(v) for v in line.split()]
            vals = [v if v != 2 else -2 for v in raw]
            if len(vals) != grid.shape[0]:
                raise ValueError(f"Line '{line}' has {len(vals)} values, but width is {grid.shape[0]}")
            grid[:, row, z] = vals          # numpy indexing: negative z wraps, row >= D raises
            tokens[:, row, z] = raw         # simpleEnv keeps the raw values (envs/simpleEnv.py:381)
            row += 1
    return OracleRoom(name=name, grid=grid, start=start, goal=goal, tokens=tokens)


def parse_room_file(path) -> OracleRoom:
    p = Path(path)
    return parse_room_text(p.read_text(), name=p.name)


def walled_box(W: int, D: int, H: int) -> OracleRoom:
    """room_path=None fallback box, envs/CubicEnv.py:440-448."""
    g = np.zeros((W, D, H), dtype=np.int64)
    g[0, :, :] = -2
    g[-1, :, :] = -2
    g[:, 0, :] = -2
    g[:, -1, :] = -2
    g[:, :, 0] = -2
    g[:, :, -1] = -2
    return OracleRoom(name=f"box_{W}x{D}x{H}", grid=g)


def room_set_from_dir(path) -> list:
    """Path(room_path).glob('*.txt') (envs/CubicEnv.py:66), sorted by name."""
    return [parse_room_file(p) for p in sorted(Path(path).glob("*.txt"), key=lambda p: p.name)]


# --------------------------------------------------------------------------
# C oracle
# --------------------------------------------------------------------------
def build_oracle_lib(force: bool = False) -> Path:
    if force or not _LIB_PATH.exists() or _LIB_PATH.stat().st_mtime < (_HERE / "voxnav_oracle.c").stat().st_mtime:
        subprocess.run(["make", "-s", "-C", str(_HERE)], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build_oracle_lib()
        L = ctypes.CDLL(str(_LIB_PATH))
        c = ctypes
        P = c.c_void_p
        L.or_create.restype = P
        L.or_create.argtypes = [c.c_int, P, P, P, c.c_int, c.c_int, c.c_double, c.c_int]
        L.or_create2.restype = P
        L.or_create2.argtypes = [c.c_int, P, P, P, P, c.c_int, c.c_int, c.c_double, c.c_int, c.c_int]
        L.or_obs_dim.argtypes = [P]
        L.or_obs_dim.restype = c.c_int
        L.or_destroy.argtypes = [P]
        L.or_reset.argtypes = [P, c.c_int, c.c_int64, P]
        L.or_reset.restype = c.c_int
        L.or_step.argtypes = [P, c.c_int, c.c_int, P, P, P, P]
        L.or_step.restype = c.c_int
        L.or_get_state.argtypes = [P, c.c_int, P]
        L.or_get_belief.argtypes = [P, c.c_int, P]
        L.or_get_belief.restype = c.c_int
        L.or_room_total_free.argtypes = [P, c.c_int]
        L.or_room_total_free.restype = c.c_int
        L.or_reset_draw.argtypes = [P, c.c_int64, P]
        L.or_reset_draw.restype = c.c_int
        L.or_mt_outputs.argtypes = [c.c_int64, c.c_int, P]
        L.or_philox4x32_10.argtypes = [P, P, P]
        L.or_random_action.argtypes = [c.c_uint64, c.c_uint64, c.c_uint64]
        L.or_random_action.restype = c.c_int32
        L.or_run_random.argtypes = [P, P, c.c_int, c.c_int64, c.c_uint64, c.c_uint64, c.c_uint64, c.c_int,
                                    c.c_int, P, P, P, P, P, P, P, c.c_int, P]
        L.or_run_random.restype = c.c_int64
        L.or_gae.argtypes = [P, P, P, P, P, c.c_int, c.c_int, c.c_double, c.c_double, P, P]
        _lib = L
    return _lib


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class OracleEnv:
    """N independent CubicEnv (variant 0) or simpleEnv (variant 1) agents on
    the CPU (restated semantics)."""

    def __init__(self, rooms: Sequence[OracleRoom], n_agents: int = 1, local_map_length: int = 4,
                 crash_penalty: float = -2.0, use_room_draw: bool = True, variant: int = 0):
        self.rooms = list(rooms)
        self.n_agents = int(n_agents)
        self.L = int(local_map_length)
        self.variant = int(variant)
        whd = np.array([r.whd for r in self.rooms], dtype=np.int32).reshape(-1)
        walls = np.concatenate([r.walls_for(self.variant).reshape(-1) for r in self.rooms]).astype(np.uint8)
        fs = np.array([r.start if r.start is not None else (-1, -1, -1) for r in self.rooms],
                      dtype=np.int32).reshape(-1)
        gl = np.array([r.goal if r.goal is not None else (-1, -1, -1) for r in self.rooms],
                      dtype=np.int32).reshape(-1)
        self._keep = (whd, walls, fs, gl)
        self._h = lib().or_create2(len(self.rooms), _ptr(whd), _ptr(walls), _ptr(fs), _ptr(gl),
                                   int(bool(use_room_draw)), self.L, float(crash_penalty), self.n_agents,
                                   self.variant)
        self.obs_dim = int(lib().or_obs_dim(self._h))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().or_destroy(h)
            self._h = None

    def reset(self, agent: int, seed: int) -> np.ndarray:
        obs = np.zeros(self.obs_dim, np.float32)
        lib().or_reset(self._h, agent, int(seed), _ptr(obs))
        return obs

    def step(self, agent: int, action: int):
        obs = np.zeros(self.obs_dim, np.float32)
        r = np.zeros(1, np.float64)
        te = np.zeros(1, np.uint8)
        tr = np.zeros(1, np.uint8)
        rc = lib().or_step(self._h, agent, int(action), _ptr(obs), _ptr(r), _ptr(te), _ptr(tr))
        if rc != 0:
            raise ValueError(f"bad action {action}")
        return obs, float(r[0]), bool(te[0]), bool(tr[0])

    def state(self, agent: int) -> dict:
        out = np.zeros(16, np.int64)
        lib().or_get_state(self._h, agent, _ptr(out))
        return dict(zip(STATE_FIELDS, (int(v) for v in out)))

    def belief(self, agent: int) -> np.ndarray:
        st = self.state(agent)
        W, D, H = self.rooms[st["room"]].whd
        out = np.zeros(W * D * H, np.int32)
        lib().or_get_belief(self._h, agent, _ptr(out))
        return out.reshape(W, D, H)

    def reset_draw(self, seed: int):
        out = np.zeros(4, np.int32)
        draws = lib().or_reset_draw(self._h, int(seed), _ptr(out))
        return int(out[0]), (int(out[1]), int(out[2]), int(out[3])), int(draws)

    def run_random(self, seeds, policy_seed: int, K: int, t0: int = 0, gid_base: int = 0,
                   seed_stride: Optional[int] = None, autoreset: bool = True, initial_reset: bool = True,
                   record: bool = True, threads: int = 0, actions=None, terminal_obs: bool = False, gids=None):
        """K batched steps (Philox random policy, or `actions` [K, N]) with SB3-style autoreset.
        Agent i's random-policy stream is keyed by ``gids[i]`` when given (a
        sample of a larger batch), else by ``gid_base + i``."""
        N = self.n_agents
        seeds = np.ascontiguousarray(np.asarray(seeds, dtype=np.int64).reshape(N))
        stride = N if seed_stride is None else int(seed_stride)
        if record:
            obs = np.zeros((K, N, self.obs_dim), np.float32)
            rew = np.zeros((K, N), np.float64)
            te = np.zeros((K, N), np.uint8)
            tr = np.zeros((K, N), np.uint8)
            act = np.zeros((K, N), np.int32)
        else:
            obs = rew = te = tr = act = None
        tob = np.zeros((K, N, self.obs_dim), np.float32) if terminal_obs else None
        ain = None if actions is None else np.ascontiguousarray(np.asarray(actions, np.int32).reshape(K, N))
        gid = None if gids is None else np.ascontiguousarray(np.asarray(gids, np.int64).reshape(N))
        resets = lib().or_run_random(self._h, _ptr(seeds), int(bool(initial_reset)), stride, int(gid_base),
                                     int(policy_seed), int(t0), int(K), int(bool(autoreset)), _ptr(obs),
                                     _ptr(rew), _ptr(te), _ptr(tr), _ptr(act), _ptr(tob), _ptr(ain), int(threads),
                                     _ptr(gid))
        return dict(obs=obs, reward=rew, terminated=te, truncated=tr, actions=act, terminal_obs=tob,
                    resets=int(resets))


def mt_outputs(seed: int, n: int) -> np.ndarray:
    out = np.zeros(n, np.uint32)
    lib().or_mt_outputs(int(seed), int(n), _ptr(out))
    return out


def philox4x32_10(ctr, key) -> np.ndarray:
    c = np.asarray(ctr, dtype=np.uint32).reshape(4).copy()
    k = np.asarray(key, dtype=np.uint32).reshape(2).copy()
    o = np.zeros(4, np.uint32)
    lib().or_philox4x32_10(_ptr(c), _ptr(k), _ptr(o))
    return o


def random_action(policy_seed: int, gid: int, t: int) -> int:
    return int(lib().or_random_action(int(policy_seed), int(gid), int(t)))


def gae(rewards, values, episode_starts, last_values, dones, gamma=0.99, gae_lambda=0.95):
    r = np.ascontiguousarray(rewards, np.float32)
    v = np.ascontiguousarray(values, np.float32)
    s = np.ascontiguousarray(episode_starts, np.float32)
    lv = np.ascontiguousarray(last_values, np.float32)
    d = np.ascontiguousarray(dones, np.float32)
    T, N = r.shape
    adv = np.zeros((T, N), np.float32)
    ret = np.zeros((T, N), np.float32)
    lib().or_gae(_ptr(r), _ptr(v), _ptr(s), _ptr(lv), _ptr(d), T, N, float(gamma), float(gae_lambda),
                 _ptr(adv), _ptr(ret))
    return adv, ret
