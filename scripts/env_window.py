#!/usr/bin/env python3
"""One env window and nothing else (for rocprofv3 passes over a single
kernel configuration): reset, `warmup` untimed steps, `steps` steps in
F-step launches, with the library at --lib (a diagnostics variant) or the
product's.  Prints the host-timed rate.

  python scripts/env_window.py --room P3_training --F 128 --warmup 32 --steps 1024 [--lib path.so]
"""
import argparse
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
    ap.add_argument("--lib", default=None)
    ap.add_argument("--N", type=int, default=65536)
    ap.add_argument("--room", default="32x32x8")
    ap.add_argument("--L", type=int, default=10)
    ap.add_argument("--F", type=int, default=128)
    ap.add_argument("--warmup", type=int, default=32)
    ap.add_argument("--steps", type=int, default=1024)
    a = ap.parse_args()
    lib = _native.load_variant(REPO / a.lib) if a.lib else None
    rs = load_archive_set(a.room) if a.room.startswith("P") else single_room_set(box_room(*map(int, a.room.split("x"))))
    kw = {"lib": lib} if lib is not None else {}
    e = BatchedGridEnv(num_agents=a.N, rooms=rs, local_map_length=a.L, autoreset=True, device="cuda:0", **kw)
    e.reset(seed=42)
    F = a.F
    o = Rollout(torch.empty((F, a.N, 80), device="cuda:0"), torch.empty((F, a.N), device="cuda:0"),
                torch.empty((F, a.N), dtype=torch.uint8, device="cuda:0"),
                torch.empty((F, a.N), dtype=torch.uint8, device="cuda:0"), None)

    def run(total):
        while total > 0:
            k = min(F, total)
            e.step_random(k, policy_seed=42, out=Rollout(o.obs[:k], o.reward[:k], o.terminated[:k], o.truncated[:k],
                                                        None))
            total -= k

    run(a.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(a.steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"room": a.room, "F": F, "warmup": a.warmup, "steps": a.steps, "lib": a.lib or "product",
                      "kernel": e.kernel_label(F), "Gsteps": round(a.N * a.steps / el / 1e9, 3)}), flush=True)
    e.close()


if __name__ == "__main__":
    main()
