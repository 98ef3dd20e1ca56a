#!/usr/bin/env python3
"""Per-section shader-clock profile of the simpleEnv stepping wave
(simple_pipe_kernel; diagnostics build with -DVN_SIMPLE_PROF=1:
scripts/build_variants.py sprof:VN_SIMPLE_PROF=1): cycles per stepping wave
per step in each section, over a bench-shaped window (65,536 agents,
32x32x8, L=4, 128-step launches)."""
import argparse
import ctypes
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "3d-navigation-reinforcement-learning_amd"))
import torch  # noqa: E402

from voxnav import _native  # noqa: E402
from voxnav.env import BatchedGridEnv, Rollout  # noqa: E402
from voxnav.rooms import box_room, single_room_set  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default="3d-navigation-reinforcement-learning_amd/voxnav/_lib/variants/libvoxnav_sprof.so")
ap.add_argument("--N", type=int, default=65536)
ap.add_argument("--room", default="32x32x8")
ap.add_argument("--L", type=int, default=4)
ap.add_argument("--F", type=int, default=128)
ap.add_argument("--steps", type=int, default=2048)
a = ap.parse_args()
lib = _native.load_variant(REPO / a.lib)
raw = lib.raw if hasattr(lib, "raw") else lib
rs = single_room_set(box_room(*map(int, a.room.split("x"))))
e = BatchedGridEnv(num_agents=a.N, rooms=rs, local_map_length=a.L, autoreset=True, device="cuda:0", lib=lib,
                   variant="simple")
e.reset(seed=42)
F, od = a.F, 6 * a.L + 7
o = Rollout(torch.empty((F, a.N, od), device="cuda:0"), torch.empty((F, a.N), device="cuda:0"),
            torch.empty((F, a.N), dtype=torch.uint8, device="cuda:0"),
            torch.empty((F, a.N), dtype=torch.uint8, device="cuda:0"), None)
e.step_random(F, out=o)
torch.cuda.synchronize()
prof = (ctypes.c_ulonglong * 16)()
fn = getattr(raw, "vn_debug_simple_prof", None) or getattr(raw, "_lib").vn_debug_simple_prof
fn(prof, 1)
n = a.steps // F
t0 = time.perf_counter()
for _ in range(n):
    e.step_random(F, out=o)
torch.cuda.synchronize()
el = time.perf_counter() - t0
fn(prof, 1)
waves = max(1, prof[8])
names = ["commit", "premove+evict", "marks", "observe", "reward+stage", "reset", "handoff"]
tot = sum(prof[k] for k in range(7))
print(f"simple {a.room} L={a.L} F={F}: {a.N * n * F / el / 1e9:.3f} G env-steps/s (instrumented); "
      f"per stepping-wave step, s_memtime ticks:")
for k, nm in enumerate(names):
    print(f"  {nm:14s} {prof[k] / waves / F:9.1f}  ({100 * prof[k] / max(1, tot):5.1f} %)")
print(f"  loop total     {prof[7] / waves / F:9.1f}; waves x launches = {waves}")
