#!/usr/bin/env python3
"""Access-pattern statistics of the byte-mark env kernel (PCM 3) on the
reference's training rooms, from the CPU oracle (test infrastructure; not a
test, not the product path).  Replays agents under a uniform random policy
(the P-set bench legs' policy) and counts, per env-step after a 32-step
warmup, what the kernel would load / store for it:

  * entering window columns (a horizontal move brings in 4) and how many of
    them already hold a known cell -- i.e. would NOT be all-zero in HBM, so a
    "never touched" bitmap could skip only the rest;
  * plane-row changes (the x row (y, z) / y row (x, z) the sensing marks)
    and the misses / dirty evictions of a direct-mapped LDS row cache of
    16 or 8 slots per axis;
  * blind byte marks (cells newly known outside the 4 x 4 window).

  python tests/analysis_pset_access.py P3_training 40 1056
Reference: envs/CubicEnv.py:229-251 (window), :322-343 (marks), :345-397
(rays); rooms per train/Grid_Train.py:50-55.  DESIGN.md 7.14 quotes the
output.
"""
import random
import sys
import tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "3d-navigation-reinforcement-learning_amd"))
from oracle.oracle import OracleEnv, room_set_from_dir  # noqa: E402
import voxnav.rooms as vr  # noqa: E402


def slot(a, z, mode):
    return ((a & 3) << 2) | (z & 3) if mode == 16 else ((a & 1) << 2) | (z & 3)


def main():
    name, nag, T = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    W0 = 32
    root = vr.extract_archive(tempfile.mkdtemp())
    env = OracleEnv(room_set_from_dir(root / name), n_agents=1, local_map_length=10)
    rng = random.Random(1)
    st = dict(steps=0, shifts=0, ent=0, ent_touched=0, row_changes=0, blind=0)
    cache = {16: dict(miss=0, wb=0), 8: dict(miss=0, wb=0)}
    for a in range(nag):
        env.reset(0, 1000 + a)
        cs = {m: [dict(), dict()] for m in cache}
        prev = [None, None]
        for t in range(T):
            s0 = env.state(0)
            b0 = env.belief(0)
            _, _, te, tr = env.step(0, rng.randrange(6))
            if te or tr:
                env.reset(0, rng.randrange(1 << 30))
                cs = {m: [dict(), dict()] for m in cache}
                prev = [None, None]
                continue
            s1 = env.state(0)
            x0, y0 = s0["x"], s0["y"]
            x, y, z = s1["x"], s1["y"], s1["z"]
            keys = [(y, z), (x, z)]
            timed = t >= W0
            if timed:
                st["steps"] += 1
                W, D, _ = b0.shape
                if (x, y) != (x0, y0):
                    st["shifts"] += 1
                    if x != x0:
                        ex = x + 1 if x > x0 else x - 2
                        ents = [(ex, y + q - 2) for q in range(4)]
                    else:
                        ey = y + 1 if y > y0 else y - 2
                        ents = [(x + q - 2, ey) for q in range(4)]
                    for cx, cy in ents:
                        if 0 <= cx < W and 0 <= cy < D:
                            st["ent"] += 1
                            st["ent_touched"] += int((b0[cx, cy, :] != -1).any())
                st["row_changes"] += sum(int(prev[k] != keys[k]) for k in range(2))
                b1 = env.belief(0)
                new = (b0 == -1) & (b1 != -1)
                new[max(0, x - 2):x + 2, max(0, y - 2):y + 2, :] = False
                st["blind"] += int(new.sum())
            for k in range(2):
                for m in cache:
                    c = cs[m][k]
                    sl = slot(keys[k][0], keys[k][1], m)
                    e = c.get(sl)
                    if (e is None or e != keys[k]) and timed:
                        cache[m]["miss"] += 1
                        cache[m]["wb"] += int(e is not None)
                    c[sl] = keys[k]
                prev[k] = keys[k]
    n = st["steps"]
    print(f"{name}: {nag} agents x {T} steps (first {W0} untimed), {n} timed env-steps")
    print(f"  horizontal moves {st['shifts'] / n:.3f}, entering columns {st['ent'] / n:.3f}, "
          f"of which already hold a known cell {st['ent_touched'] / n:.3f} "
          f"({100 * st['ent_touched'] / max(1, st['ent']):.1f} %)")
    print(f"  plane-row changes {st['row_changes'] / n:.3f}, blind byte marks {st['blind'] / n:.3f}")
    for m, d in cache.items():
        print(f"  direct-mapped row cache, {m} slots per axis: misses {d['miss'] / n:.3f}, "
              f"dirty evictions {d['wb'] / n:.3f}")


if __name__ == "__main__":
    main()
