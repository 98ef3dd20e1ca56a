#!/usr/bin/env python3
"""Per-section shader-clock profile of the CubicEnv step loop (diagnostics
build with -DVN_ENV_PROF=1, scripts/build_variants.py eprof:VN_ENV_PROF=1):
cycles per wave per step in each section, over a bench-shaped window."""
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
from voxnav.rooms import box_room, single_room_set, load_archive_set  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default="3d-navigation-reinforcement-learning_amd/voxnav/_lib/variants/libvoxnav_eprof.so")
ap.add_argument("--N", type=int, default=65536)
ap.add_argument("--room", default="32x32x8")
ap.add_argument("--F", type=int, default=16)
ap.add_argument("--steps", type=int, default=5408)
ap.add_argument("--warmup", type=int, default=0, help="steps after each reset before the timed launch (0: whole-window mode)")
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
lib = _native.load_variant(REPO / a.lib)
raw = lib.raw if hasattr(lib, "raw") else lib
rs = load_archive_set(a.room) if a.room.startswith("P") else single_room_set(box_room(*map(int, a.room.split("x"))))
e = BatchedGridEnv(num_agents=a.N, rooms=rs, local_map_length=10, autoreset=True, device="cuda:0", lib=lib)
e.reset(seed=42)
F = a.F
Fb = max(F, a.warmup)   # the buffer also takes the warmup launch
ob = Rollout(torch.empty((Fb, a.N, 80), device="cuda:0"), torch.empty((Fb, a.N), device="cuda:0"),
             torch.empty((Fb, a.N), dtype=torch.uint8, device="cuda:0"),
             torch.empty((Fb, a.N), dtype=torch.uint8, device="cuda:0"), None)
o = Rollout(ob.obs[:F], ob.reward[:F], ob.terminated[:F], ob.truncated[:F], None)
prof = (ctypes.c_ulonglong * 16)()
fn = getattr(raw, "vn_debug_env_prof", None) or getattr(raw, "_lib").vn_debug_env_prof
if a.warmup:
    # the driver's window: reset, `warmup` steps, then one F-step launch (profiled), repeated
    wo = Rollout(ob.obs[:a.warmup], ob.reward[:a.warmup], ob.terminated[:a.warmup], ob.truncated[:a.warmup], None)
    n = a.reps
    el = 0.0
    acc = [0] * 16
    for r in range(a.reps):
        e.reset(seed=42 + r)
        e.step_random(a.warmup, policy_seed=7, t0=0, out=wo)
        torch.cuda.synchronize()
        fn(prof, 1)                       # drop the reset / warmup launches
        t0 = time.perf_counter()
        e.step_random(F, policy_seed=7, t0=a.warmup, out=o)
        torch.cuda.synchronize()
        el += time.perf_counter() - t0
        fn(prof, 1)
        for k in range(16):
            acc[k] = max(acc[k], prof[k]) if k == 11 else acc[k] + prof[k]
    for k in range(16):
        prof[k] = acc[k]
else:
    e.step_random(F, out=o)
    torch.cuda.synchronize()
    fn(prof, 1)
    n = a.steps // F
    t0 = time.perf_counter()
    for _ in range(n):
        e.step_random(F, out=o)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    fn(prof, 1)
waves = max(1, prof[8])
names = ["move+issue", "shift-commit", "sense+stage", "reward-ev", "reset", "obs-flush", "reward-store"]
tot = sum(prof[k] for k in range(7))
print(f"{a.room} F={F} warmup={a.warmup}: {a.N * n * F / el / 1e9:.3f} G env-steps/s (instrumented, host-timed); "
      f"per wave-step cycles:")
for k, nm in enumerate(names):
    print(f"  {nm:13s} {prof[k] / waves / F:9.1f}  ({100 * prof[k] / max(1, tot):5.1f} %)")
print(f"  loop total    {prof[7] / waves / F:9.1f}; waves x launches = {waves}")
print(f"  per launch: prologue {prof[9] / waves:9.1f}, loop {prof[7] / waves:9.1f}, epilogue {prof[10] / waves:9.1f}, "
      f"longest wave {prof[11]:9.1f} cycles")
# the last profiled launch's per-wave start / end (100-MHz clock): how long the tail is
wfn = getattr(raw, "vn_debug_env_wavetimes", None) or getattr(getattr(raw, "_lib", raw), "vn_debug_env_wavetimes", None)
if wfn is not None:
    import numpy as np
    nw = min(8192, (a.N * 4 + 63) // 64)
    t = (ctypes.c_ulonglong * (8192 * 2))()
    ids = (ctypes.c_uint * (8192 * 2))()
    wfn(t, ids)
    tt = np.frombuffer(t, dtype=np.uint64)[:2 * nw].reshape(nw, 2).astype(np.int64)
    ii = np.frombuffer(ids, dtype=np.uint32)[:2 * nw].reshape(nw, 2)
    t0 = tt[:, 0].min()
    st, en = (tt[:, 0] - t0) / 100.0, (tt[:, 1] - t0) / 100.0   # us
    span = en.max()
    print(f"  last launch, per wave (us from the first start): start p50 {np.median(st):.2f} max {st.max():.2f}; "
          f"end p10 {np.percentile(en, 10):.2f} p50 {np.median(en):.2f} p90 {np.percentile(en, 90):.2f} max {span:.2f}")
    print(f"  waves done at 80 / 90 / 95 % of the launch: {np.mean(en <= 0.8 * span):.3f} / "
          f"{np.mean(en <= 0.9 * span):.3f} / {np.mean(en <= 0.95 * span):.3f}")
    xcc = ii[:, 1] & 0xF
    simd = (ii[:, 0] >> 4) & 3
    for x in range(8):
        m = xcc == x
        if m.any():
            print(f"    XCC {x}: {m.sum():4d} waves, end p50 {np.median(en[m]):.2f} max {en[m].max():.2f}")
    # waves per SIMD slot: the last wave on each SIMD
    key = (ii[:, 1].astype(np.int64) << 32) | (ii[:, 0] >> 4).astype(np.int64)
    _, inv = np.unique(key, return_inverse=True)
    last = np.zeros(inv.max() + 1)
    np.maximum.at(last, inv, en)
    print(f"  per SIMD, its last wave's end: p10 {np.percentile(last, 10):.2f} p50 {np.median(last):.2f} max {last.max():.2f}")
