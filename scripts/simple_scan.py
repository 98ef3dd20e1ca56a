#!/usr/bin/env python3
"""Throughput scan of the simpleEnv kernels (bit-plane vs dense map) over
agent counts: python scripts/simple_scan.py --n 65536,262144 --dense 0,1"""
import argparse
import os
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "3d-navigation-reinforcement-learning_amd"))
import torch  # noqa: E402

from voxnav.env import BatchedGridEnv, Rollout  # noqa: E402
from voxnav.rooms import box_room, load_archive_set, single_room_set  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="65536,262144")
    ap.add_argument("--dense", default="0,1")
    ap.add_argument("--room", default="32x32x8")
    ap.add_argument("--L", type=int, default=4)
    ap.add_argument("--F", type=int, default=16)
    ap.add_argument("--steps", type=int, default=512)
    ap.add_argument("--autoreset", default="1", help="comma list of 0/1")
    ap.add_argument("--lib", default=None, help="another build of the library (e.g. -DVN_SIMPLE_PROF=1)")
    ap.add_argument("--ablate", default="0", help="ignored: ablations are compile-time VN_ABLATE builds (see scripts/ab.py)")
    a = ap.parse_args()
    lib = raw = None
    if a.lib:
        import ctypes
        from voxnav import _native
        lib = _native.load_variant(a.lib)
        raw = ctypes.CDLL(a.lib)
    rs = (load_archive_set(a.room) if a.room.startswith("P")
          else single_room_set(box_room(*map(int, a.room.split("x")))))
    for n in map(int, a.n.split(",")):
        for dense, abl, ar in [(d, b, r) for d in a.dense.split(",") for b in a.ablate.split(",")
                               for r in a.autoreset.split(",")]:
            os.environ["VOXNAV_SIMPLE_DENSE"] = dense
            os.environ["VOXNAV_ABLATE"] = abl
            e = BatchedGridEnv(num_agents=n, rooms=rs, local_map_length=a.L, autoreset=ar == "1", device="cuda:0",
                               variant="simple", **({"lib": lib} if lib is not None else {}))
            e.reset(seed=42)
            F = a.F
            o = Rollout(torch.empty((F, n, e.obs_dim), device="cuda:0"), torch.empty((F, n), device="cuda:0"),
                        torch.empty((F, n), dtype=torch.uint8, device="cuda:0"),
                        torch.empty((F, n), dtype=torch.uint8, device="cuda:0"), None)
            for _ in range(4):
                e.step_random(F, out=o)
            torch.cuda.synchronize()
            prof = None
            if raw is not None and hasattr(raw, "vn_debug_simple_prof"):
                import ctypes
                prof = (ctypes.c_ulonglong * 16)()
                raw.vn_debug_simple_prof(prof, 1)
            t0 = time.perf_counter()
            launches = max(1, a.steps // F)
            for _ in range(launches):
                e.step_random(F, out=o)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            st = launches * F
            if prof is not None:
                raw.vn_debug_simple_prof(prof, 1)
                waves = max(1, prof[7])
                names = ["action", "move+rows", "observe", "reward+stores", "reset", "flush"]
                print("  cycles/step/wave: " + ", ".join(f"{nm}={prof[q] / waves / F:.0f}" for q, nm in enumerate(names))
                      + f" | max wave cycles/launch={prof[6]}, max wave reset cycles/launch={prof[9]},"
                      f" resets/launch={prof[8] / launches:.0f}, wave reset events/launch={prof[10] / launches:.0f}",
                      flush=True)
            print(f"N={n} dense={dense} ablate={abl} autoreset={ar} F={F}: {el / st * 1e6:.2f} us/step  {n * st / el / 1e9:.3f} G env-steps/s",
                  flush=True)
            e.close()
            del e, o
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
