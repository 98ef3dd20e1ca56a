"""Generate golden vectors from the UNMODIFIED reference env.

Runs only in the build container, where the reference is mounted read-only at
/root/reference (the GPU box never has it).  It imports
``envs/CubicEnv.py`` and ``envs/simpleEnv.py`` behind a ~20-line in-memory
``gymnasium`` stub (gymnasium is not installed; the envs only use
``gym.Env`` and ``spaces.Discrete/Box`` -- envs/CubicEnv.py:2-3,56-62), runs
them, and writes the observed inputs/outputs as compressed ``.npz`` data
under tests/golden/.  Nothing from the reference source is stored: only
actions, seeds and the env's observed state/obs/reward per step.

Usage:  python tests/golden/gen_golden.py  [--quick]
"""
from __future__ import annotations

import argparse
import contextlib
import hashlib
import importlib.util
import io
import os
import random
import shutil
import sys
import tempfile
import types
from collections import deque
from pathlib import Path

import numpy as np

REF = Path(os.environ.get("VOXNAV_REFERENCE", "/root/reference"))
OUT = Path(__file__).resolve().parent
REPO = OUT.parent.parent
sys.path.insert(0, str(REPO))
from oracle.oracle import random_action  # noqa: E402  (Philox stream, build-defined)

FIELDS = ("x", "y", "z", "facing", "last_action", "step_count", "visited_count", "bump_count",
          "done", "last_bump", "near_wall", "was_near_wall", "cells_insight_down")


def _install_gym_stub():
    gym = types.ModuleType("gymnasium")
    spaces = types.ModuleType("gymnasium.spaces")

    class Env:
        def reset(self, seed=None, options=None):
            return None

    class Discrete:
        def __init__(self, n):
            self.n = n

    class Box:
        def __init__(self, low=None, high=None, shape=None, dtype=None):
            self.low, self.high, self.shape, self.dtype = low, high, shape, dtype

    spaces.Discrete, spaces.Box = Discrete, Box
    gym.Env, gym.spaces = Env, spaces
    sys.modules["gymnasium"] = gym
    sys.modules["gymnasium.spaces"] = spaces


def _load(modname, relpath):
    sys.dont_write_bytecode = True
    os.environ.setdefault("MPLBACKEND", "Agg")
    spec = importlib.util.spec_from_file_location(modname, REF / relpath)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def grid_hash(a: np.ndarray) -> np.uint64:
    h = hashlib.blake2b(np.ascontiguousarray(a, dtype=np.int64).tobytes(), digest_size=8).digest()
    return np.frombuffer(h, dtype=np.uint64)[0]


def state_row(env):
    return [int(getattr(env, f)) for f in FIELDS]


# relative move tables (the action semantics of envs/CubicEnv.py:135-140)
_DIRS = [[(0, 1, 0), (1, 0, 0), (0, -1, 0), (-1, 0, 0)],
         [(1, 0, 0), (0, -1, 0), (-1, 0, 0), (0, 1, 0)],
         [(0, -1, 0), (-1, 0, 0), (0, 1, 0), (1, 0, 0)],
         [(-1, 0, 0), (0, 1, 0), (1, 0, 0), (0, -1, 0)]]


def explorer_action(env):
    """Greedy BFS explorer (golden-vector policy only): shortest path over
    true free cells to the nearest cell the agent has not visited."""
    W, D, H = env.width, env.depth, env.height
    start = (env.x, env.y, env.z)
    prev = {start: None}
    q = deque([start])
    goal = None
    while q:
        c = q.popleft()
        if c != start and env.internal_grid[c] <= 0:
            goal = c
            break
        for d in ((1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1)):
            n = (c[0] + d[0], c[1] + d[1], c[2] + d[2])
            if 0 <= n[0] < W and 0 <= n[1] < D and 0 <= n[2] < H and n not in prev and env.grid[n] != -2:
                prev[n] = c
                q.append(n)
    if goal is None:
        return 0
    c = goal
    while prev[c] != start:
        c = prev[c]
    d = (c[0] - start[0], c[1] - start[1], c[2] - start[2])
    if d == (0, 0, 1):
        return 4
    if d == (0, 0, -1):
        return 5
    for a in range(4):
        if _DIRS[a][env.facing] == d:
            return a
    raise AssertionError(d)


def seek_action(env):
    """Goal-seeking BFS (simpleEnv golden vectors only): shortest path over
    the true free cells (simpleEnv walls are 2) to the goal or one of the 4
    cells above it (envs/simpleEnv.py:201-206)."""
    W, D, H = env.width, env.depth, env.height
    targets = {(env.gx, env.gy, env.gz + i) for i in range(5)}
    start = (env.x, env.y, env.z)
    prev = {start: None}
    q = deque([start])
    goal = None
    while q:
        c = q.popleft()
        if c in targets and c != start:
            goal = c
            break
        for d in ((1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1)):
            n = (c[0] + d[0], c[1] + d[1], c[2] + d[2])
            if 0 <= n[0] < W and 0 <= n[1] < D and 0 <= n[2] < H and n not in prev and env.grid[n] != 2:
                prev[n] = c
                q.append(n)
    if goal is None:
        return 0
    c = goal
    while prev[c] != start:
        c = prev[c]
    d = (c[0] - start[0], c[1] - start[1], c[2] - start[2])
    if d == (0, 0, 1):
        return 4
    if d == (0, 0, -1):
        return 5
    for a in range(4):
        if _DIRS[a][env.facing] == d:
            return a
    raise AssertionError(d)


def run_trajectory(env, seeds, steps, policy, policy_seed, eps, full_dumps=(), simple=False):
    """Step `env`, resetting (seed from `seeds`, in order) at start and after
    every terminated/truncated step (SB3 VecEnv auto-reset order)."""
    seeds = list(seeds)
    coin = random.Random(policy_seed)      # private stream; never touches the env's global `random`
    rec = {k: [] for k in ("actions", "state", "reward", "terminated", "truncated", "obs", "belief_hash",
                           "reset_obs", "reset_state", "reset_at", "room_hash", "belief_dump", "dump_at")}
    si = 0

    def do_reset():
        nonlocal si
        s = seeds[si]
        si += 1
        if simple:
            random.seed(s)
            env.reset()
            obs = env.get_obs()
        else:
            obs, _ = env.reset(seed=s)
        rec["reset_obs"].append(np.asarray(obs, np.float32))
        rec["reset_state"].append(state_row(env) if not simple else [env.x, env.y, env.z, env.gx, env.gy, env.gz])
        rec["room_hash"].append(grid_hash(env.grid))

    with contextlib.redirect_stdout(io.StringIO()):
        do_reset()
        rec["reset_at"].append(0)
        for t in range(steps):
            if policy == "random" or coin.random() < eps:
                a = random_action(policy_seed, 0, t)
            elif policy == "seek":
                a = seek_action(env)
            else:
                a = explorer_action(env)
            obs, r, term, trunc, _ = env.step(a)
            rec["actions"].append(a)
            rec["reward"].append(float(r))
            rec["terminated"].append(bool(term))
            rec["truncated"].append(bool(trunc))
            rec["obs"].append(np.asarray(obs, np.float32))
            if not simple:
                rec["state"].append(state_row(env))
            else:
                rec["state"].append([env.x, env.y, env.z, env.facing, env.last_action, env.step_count,
                                     env.visited_count, env.bump_count, int(env.done)])
            rec["belief_hash"].append(grid_hash(env.internal_grid))
            if t in full_dumps:
                rec["belief_dump"].append(np.asarray(env.internal_grid, np.int32).copy())
                rec["dump_at"].append(t)
            if term or trunc:
                do_reset()
                rec["reset_at"].append(t + 1)
    out = dict(
        seeds=np.asarray(seeds[:si], np.int64),
        actions=np.asarray(rec["actions"], np.int32),
        state=np.asarray(rec["state"], np.int64),
        reward=np.asarray(rec["reward"], np.float64),
        terminated=np.asarray(rec["terminated"], np.uint8),
        truncated=np.asarray(rec["truncated"], np.uint8),
        obs=np.asarray(rec["obs"], np.float32),
        belief_hash=np.asarray(rec["belief_hash"], np.uint64),
        reset_obs=np.asarray(rec["reset_obs"], np.float32),
        reset_state=np.asarray(rec["reset_state"], np.int64),
        reset_at=np.asarray(rec["reset_at"], np.int64),
        room_hash=np.asarray(rec["room_hash"], np.uint64),
        dump_at=np.asarray(rec["dump_at"], np.int64),
    )
    for i, d in enumerate(rec["belief_dump"]):
        out[f"belief_dump_{i}"] = d
    return out


def write_box_room(dirpath: Path, W, D, H):
    """A walled box in the reference's room-file grammar (README.md:9-19)."""
    lines = [f"Size={W},{D},{H}"]
    for z in range(H):
        lines.append(f"Layer z={z}")
        for y in range(D):
            row = []
            for x in range(W):
                wall = x in (0, W - 1) or y in (0, D - 1) or z in (0, H - 1)
                row.append("2" if wall else "0")
            lines.append(" ".join(row))
        lines.append("")
    p = dirpath / f"box_{W}x{D}x{H}.txt"
    p.write_text("\n".join(lines) + "\n")
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--only", choices=["all", "simple"], default="all",
                    help="'simple': regenerate only the simpleEnv trajectories (section 4)")
    args = ap.parse_args()
    if not (REF / "envs" / "CubicEnv.py").exists():
        raise SystemExit(f"reference not found at {REF}")
    _install_gym_stub()
    cubic = _load("ref_cubic_env", "envs/CubicEnv.py")
    simple = _load("ref_simple_env", "envs/simpleEnv.py")
    rooms = REF / "rooms"
    tmp = Path(tempfile.mkdtemp(prefix="voxnav_golden_"))

    def single_room_dir(rel):
        d = tmp / ("single_" + hashlib.md5(rel.encode()).hexdigest()[:8])
        d.mkdir(exist_ok=True)
        shutil.copy(rooms / rel, d / Path(rel).name)
        return d

    def make_env(room_path=None, L=4, whd=None, cls=None):
        cls = cls or cubic.GridAgent
        kw = dict(local_map_length=L, room_path=str(room_path) if room_path else None)
        if whd:
            kw.update(width=whd[0], depth=whd[1], height=whd[2])
        env = cls(**kw)
        if env.rooms is not None:
            env.rooms = sorted(env.rooms)      # glob order is unspecified (envs/CubicEnv.py:66)
        return env

    if args.only == "all":
        # ---------------- 1. parsed-room fixtures (all room files) -------------
        names, dims, free, hashes, bfree = [], [], [], [], []
        with contextlib.redirect_stdout(io.StringIO()):
            for p in sorted(rooms.glob("P*/*.txt")):
                env = make_env(room_path=None)
                env.rooms = [p]
                env.reset(seed=0)
                g = env.grid
                names.append(str(p.relative_to(rooms)))
                dims.append(g.shape)
                free.append(env.total_free_cells)
                hashes.append(grid_hash(g))
                bnd = np.ones(g.shape, bool)
                bnd[1:-1, 1:-1, 1:-1] = False
                bfree.append(int(((g != -2) & bnd).sum()))
        np.savez_compressed(OUT / "rooms_parsed.npz", names=np.asarray(names), whd=np.asarray(dims, np.int32),
                            total_free=np.asarray(free, np.int64), grid_hash=np.asarray(hashes, np.uint64),
                            boundary_free=np.asarray(bfree, np.int64))
        print(f"rooms_parsed: {len(names)} files")

        # ---------------- 2. reset tables --------------------------------------
        n_seeds = 300 if args.quick else 2000
        # the reference also calls np.random.seed(seed) (envs/CubicEnv.py:80): seeds must lie in [0, 2**32)
        seed_list = list(range(n_seeds)) + [2 ** 32 - 1, 2 ** 31 + 5, 2 ** 31 - 1, 4000000000, 99991]
        reset_sets = {"P1_training": rooms / "P1_training", "P2_training": rooms / "P2_training",
                      "P3_training": rooms / "P3_training", "P2_evaluate": rooms / "P2_evaluate"}
        for tag, d in reset_sets.items():
            env = make_env(room_path=d, L=10)
            room_hashes = []
            with contextlib.redirect_stdout(io.StringIO()):
                for p in env.rooms:
                    e2 = make_env(room_path=None)
                    e2.rooms = [p]
                    e2.reset(seed=0)
                    room_hashes.append(grid_hash(e2.grid))
                rows = []
                for s in seed_list:
                    env.reset(seed=s)
                    ri = room_hashes.index(grid_hash(env.grid))
                    rows.append((ri, env.x, env.y, env.z))
            np.savez_compressed(OUT / f"reset_table_{tag}.npz", seeds=np.asarray(seed_list, np.int64),
                                draws=np.asarray(rows, np.int32), room_names=np.asarray([p.name for p in env.rooms]))
            print(f"reset_table_{tag}: {len(rows)} seeds")
        # box (room_path=None): a single start draw, no room draw
        env = make_env(room_path=None, L=10, whd=(32, 32, 8))
        rows = []
        with contextlib.redirect_stdout(io.StringIO()):
            for s in seed_list:
                env.reset(seed=s)
                rows.append((0, env.x, env.y, env.z))
        np.savez_compressed(OUT / "reset_table_box32x32x8.npz", seeds=np.asarray(seed_list, np.int64),
                            draws=np.asarray(rows, np.int32), room_names=np.asarray(["<ctor box>"]))

    # ---------------- 3. trajectories --------------------------------------
    box_dir = tmp / "boxes"
    box_dir.mkdir()
    scen = []
    for (W, D, H) in ((8, 8, 4), (16, 16, 8), (32, 32, 8)):
        sub = box_dir / f"{W}x{D}x{H}"
        sub.mkdir()
        write_box_room(sub, W, D, H)
    steps_scale = 0.3 if args.quick else 1.0
    S = lambda n: max(20, int(n * steps_scale))  # noqa: E731
    scen += [
        ("box8x8x4_ctor_L4_random", "ctor:8x8x4", 4, S(300), "random", 0.0),
        ("box8x8x4_file_L4_explore", "box:8x8x4", 4, S(400), "explore", 0.15),
        ("box8x8x4_file_L10_random", "box:8x8x4", 10, S(200), "random", 0.0),
        ("box16x16x8_file_L4_random", "box:16x16x8", 4, S(1300), "random", 0.0),
        ("box16x16x8_file_L4_explore", "box:16x16x8", 4, S(1300), "explore", 0.1),
        ("box32x32x8_file_L10_random", "box:32x32x8", 10, S(800), "random", 0.0),
        ("box32x32x8_ctor_L10_explore", "ctor:32x32x8", 10, S(1500), "explore", 0.1),
        ("kitchen2_L10_explore", "file:P3_training/kitchen2.txt", 10, S(1200), "explore", 0.1),
        ("maze8x8s22_L10_explore", "file:P2_training/maze_8x8_seed22.txt", 10, S(1200), "explore", 0.2),
        ("tightcorridor_L4_random", "file:P2_training/tightcorridor.txt", 4, S(700), "random", 0.0),
        ("maze3dtunnels_L10_explore", "file:P3_training/maze_3d_tunnels.txt", 10, S(600), "explore", 0.1),
        ("apartment48_L10_random", "file:P1_training/7x7x7_empty_appartment.txt", 10, S(500), "random", 0.0),
        ("P2_training_L10_random", "set:P2_training", 10, S(800), "random", 0.0),
        ("P3_training_L10_explore", "set:P3_training", 10, S(1500), "explore", 0.1),
        ("P1_training_L4_random", "set:P1_training", 4, S(400), "random", 0.0),
    ]

    def resolve(src):
        kind, arg = src.split(":", 1)
        if kind == "ctor":
            return None, tuple(int(v) for v in arg.split("x"))
        if kind == "box":
            return box_dir / arg, None
        if kind == "file":
            return single_room_dir(arg), None
        return rooms / arg, None

    rng_dump = lambda n: tuple(sorted({0, n // 3, n // 2, n - 1}))  # noqa: E731
    for i, (name, src, L, steps, policy, eps) in enumerate(scen if args.only == "all" else []):
        rp, whd = resolve(src)
        env = make_env(room_path=rp, L=L, whd=whd)
        seeds = [42 + 1000 * i + 7 * k for k in range(64)]
        t = run_trajectory(env, seeds, steps, policy, policy_seed=9000 + i, eps=eps, full_dumps=rng_dump(steps))
        meta = dict(L=np.int64(L), policy=np.asarray(policy), use_room_draw=np.int64(rp is not None),
                    crash_penalty=np.float64(-2.0), room_source=np.asarray(src))
        np.savez_compressed(OUT / f"traj_{name}.npz", **t, **meta)
        print(f"traj_{name}: {len(t['actions'])} steps, {len(t['reset_at'])} episodes, "
              f"term={int(t['terminated'].sum())} trunc={int(t['truncated'].sum())}")

    # ---------------- 4. simpleEnv (goal-seeking variant) --------------------
    # (the reference's reset does not seed `random`; the build seeds it with
    #  random.seed(seed) before every reset and calls get_obs() after it)
    for i, (name, src, L, steps, policy, eps) in enumerate([
        ("P2_training_L4", "set:P2_training", 4, S(600), "random", 0.0),
        ("maze8x8s22_L4", "file:P2_training/maze_8x8_seed22.txt", 4, S(400), "random", 0.0),
        ("box8x8x4_L4_random", "box:8x8x4", 4, S(400), "random", 0.0),
        ("maze8x8s22_L10_seek", "file:P2_training/maze_8x8_seed22.txt", 10, S(900), "seek", 0.25),
        ("kitchen2_L10_seek", "file:P3_training/kitchen2.txt", 10, S(700), "seek", 0.2),
        ("P3_training_L10_seek", "set:P3_training", 10, S(1200), "seek", 0.15),
        ("P2_training_L4_seek", "set:P2_training", 4, S(1000), "seek", 0.3),
    ]):
        rp, _ = resolve(src)
        env = make_env(room_path=rp, L=L, cls=simple.GridAgent)
        seeds = [77 + 31 * k for k in range(64)]
        t = run_trajectory(env, seeds, steps, policy, policy_seed=5000 + i, eps=eps, simple=True)
        np.savez_compressed(OUT / f"simple_{name}.npz", **t, L=np.int64(L), room_source=np.asarray(src),
                            policy=np.asarray(policy))
        print(f"simple_{name}: {len(t['actions'])} steps, {len(t['reset_at'])} episodes, "
              f"term={int(t['terminated'].sum())} trunc={int(t['truncated'].sum())}")
    shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
