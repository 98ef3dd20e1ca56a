#!/usr/bin/env python3
"""Each wave's start / end of one CubicEnv launch (diagnostics build with
-DVN_ENV_WT=1: two clock reads and four stores per wave, nothing else): how
long a launch's tail is, by XCD and by SIMD."""
import argparse
import ctypes
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "3d-navigation-reinforcement-learning_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from voxnav import _native  # noqa: E402
from voxnav.env import BatchedGridEnv, Rollout  # noqa: E402
from voxnav.rooms import box_room, single_room_set, load_archive_set  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default="3d-navigation-reinforcement-learning_amd/voxnav/_lib/variants/libvoxnav_wt.so")
ap.add_argument("--N", type=int, default=65536)
ap.add_argument("--room", default="32x32x8")
ap.add_argument("--F", type=int, default=20)
ap.add_argument("--warmup", type=int, default=5)
a = ap.parse_args()
lib = _native.load_variant(REPO / a.lib)
raw = lib.raw if hasattr(lib, "raw") else lib
wfn = getattr(raw, "vn_debug_env_wavetimes", None) or getattr(getattr(raw, "_lib", raw), "vn_debug_env_wavetimes")
rs = load_archive_set(a.room) if a.room.startswith("P") else single_room_set(box_room(*map(int, a.room.split("x"))))
e = BatchedGridEnv(num_agents=a.N, rooms=rs, local_map_length=10, autoreset=True, device="cuda:0", lib=lib)
F = a.F
Fb = max(F, a.warmup, 1)
ob = Rollout(torch.empty((Fb, a.N, 80), device="cuda:0"), torch.empty((Fb, a.N), device="cuda:0"),
             torch.empty((Fb, a.N), dtype=torch.uint8, device="cuda:0"),
             torch.empty((Fb, a.N), dtype=torch.uint8, device="cuda:0"), None)
sl = lambda n: Rollout(ob.obs[:n], ob.reward[:n], ob.terminated[:n], ob.truncated[:n], None)  # noqa: E731
for rep in range(3):
    e.reset(seed=42)
    if a.warmup:
        e.step_random(a.warmup, policy_seed=7, t0=0, out=sl(a.warmup))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e.step_random(F, policy_seed=7, t0=a.warmup, out=sl(F))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    nw = min(8192, (a.N * 4 + 63) // 64)
    t = (ctypes.c_ulonglong * (8192 * 2))()
    ids = (ctypes.c_uint * (8192 * 2))()
    wfn(t, ids)
    tt = np.frombuffer(t, dtype=np.uint64)[:2 * nw].reshape(nw, 2).astype(np.int64)
    ii = np.frombuffer(ids, dtype=np.uint32)[:2 * nw].reshape(nw, 2)
    t0c = tt[:, 0].min()
    st, en = (tt[:, 0] - t0c) / 100.0, (tt[:, 1] - t0c) / 100.0
    span = en.max()
    print(f"{a.room} F={F} after {a.warmup}: host {el * 1e6:.1f} us; per wave (us from the first start): start p50 "
          f"{np.median(st):.2f} max {st.max():.2f}; end p10 {np.percentile(en, 10):.2f} p50 {np.median(en):.2f} "
          f"p90 {np.percentile(en, 90):.2f} max {span:.2f}; done at 80/90/95 %: {np.mean(en <= 0.8 * span):.3f} / "
          f"{np.mean(en <= 0.9 * span):.3f} / {np.mean(en <= 0.95 * span):.3f}", flush=True)
    if rep == 2:
        blk = np.arange(nw) // 4
        nb = (nw + 3) // 4
        rank = blk // max(1, nb // 4)          # dispatch rank of the block on its CU (4 blocks per CU)
        print("  by dispatch rank blockIdx // (grid / 4) (end p10 / p50 / p90): " + ", ".join(
            f"{r}: {np.percentile(en[rank == r], 10):.1f}/{np.median(en[rank == r]):.1f}/{np.percentile(en[rank == r], 90):.1f}"
            for r in range(4)))
        wib = np.arange(nw) % 4
        print("  by wave in block (end p50): " + ", ".join(f"{w}: {np.median(en[wib == w]):.1f}" for w in range(4)))
        xcc = ii[:, 1] & 0xF
        print("  by XCC (end p50 / max): " + ", ".join(
            f"{x}: {np.median(en[xcc == x]):.1f}/{en[xcc == x].max():.1f}" for x in range(8) if (xcc == x).any()))
        key = (ii[:, 1].astype(np.int64) << 32) | (ii[:, 0] >> 4).astype(np.int64)
        _, inv = np.unique(key, return_inverse=True)
        cnt = np.bincount(inv)
        last = np.zeros(inv.max() + 1)
        np.maximum.at(last, inv, en)
        first = np.full(inv.max() + 1, 1e18)
        np.minimum.at(first, inv, en)
        print(f"  {len(cnt)} SIMDs, waves per SIMD {np.bincount(cnt)[1:]}; per SIMD last end p10 "
              f"{np.percentile(last, 10):.1f} p50 {np.median(last):.1f} max {last.max():.1f}; first end p50 "
              f"{np.median(first):.1f}")
