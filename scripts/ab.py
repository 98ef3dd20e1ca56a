#!/usr/bin/env python3
"""Interleaved A/B timing of library variants in ONE process (same device,
same state), e.g.  python scripts/ab.py --variants base:path.so,lb4:other.so
A variant may add environment settings read at env creation:
  --variants pc:lib.so:VOXNAV_PCACHE=1,nopc:lib.so:VOXNAV_PCACHE=0

Ablation variants (VN_ABLATE bits, diagnostics only) are separate builds:
  python -c "import voxnav._build as b; b.build_variant('noobs', ['VN_ABLATE=16u'])"
(run with 3d-navigation-reinforcement-learning_amd on sys.path)."""
import argparse
import os
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "3d-navigation-reinforcement-learning_amd"))
import torch  # noqa: E402

from voxnav import _native  # noqa: E402
from voxnav.env import BatchedGridEnv, Rollout  # noqa: E402
from voxnav.rooms import box_room, load_archive_set, single_room_set  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", required=True)
    ap.add_argument("--configs", default="65536:32x32x8:10:16")
    ap.add_argument("--steps", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    libs, envs = {}, {}
    loaded = {}
    for v in a.variants.split(","):
        name, path, *kv = v.split(":")
        if path not in loaded:
            loaded[path] = _native.load_variant(REPO / path if not path.startswith("/") else path)
        libs[name] = loaded[path]
        envs[name] = dict(x.split("=", 1) for x in kv)
    cfgs = [c.split(":") for c in a.configs.split(",")]
    # One env alive at a time, created and destroyed per measurement, so every
    # variant gets the same device allocations (HBM placement shifts the
    # throughput of the same code by 10-15 % between allocations).
    outs = {}
    for c in cfgs:
        n, F = int(c[0]), int(c[3])
        od = 80 if len(c) < 5 or c[4] == "cubic" else 6 * int(c[2]) + 7
        outs[tuple(c)] = Rollout(torch.empty((F, n, od), device="cuda:0"), torch.empty((F, n), device="cuda:0"),
                                 torch.empty((F, n), dtype=torch.uint8, device="cuda:0"),
                                 torch.empty((F, n), dtype=torch.uint8, device="cuda:0"), None)
    res = {(name, tuple(c)): [] for name in libs for c in cfgs}
    for r in range(a.rounds):
        for c in cfgs:
            n, room, L, F = int(c[0]), c[1], int(c[2]), int(c[3])
            variant = c[4] if len(c) > 4 else "cubic"      # config field 5: cubic | simple
            rs = load_archive_set(room) if room.startswith("P") else single_room_set(box_room(*map(int, room.split("x"))))
            names = list(libs) if r % 2 == 0 else list(libs)[::-1]
            for name in names:
                saved = {k: os.environ.get(k) for k in envs[name]}
                os.environ.update(envs[name])
                e = BatchedGridEnv(num_agents=n, rooms=rs, local_map_length=L, autoreset=True, device="cuda:0",
                                   lib=libs[name], variant=variant)
                for k, old in saved.items():
                    if old is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = old
                e.reset(seed=42)
                o = outs[tuple(c)]
                for _ in range(max(2, 64 // F)):
                    e.step_random(F, out=o)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(max(1, a.steps // F)):
                    e.step_random(F, out=o)
                torch.cuda.synchronize()
                res[(name, tuple(c))].append(n * max(1, a.steps // F) * F / (time.perf_counter() - t0))
                e.close()
                del e
    for k, v in res.items():
        v = sorted(v)
        print(json.dumps({"variant": k[0], "config": ":".join(k[1]), "Gsteps_median": round(v[len(v) // 2] / 1e9, 3),
                          "Gsteps_max": round(v[-1] / 1e9, 3)}))


if __name__ == "__main__":
    main()
