#!/usr/bin/env python3
"""Placement and per-step clocks of the two-per-CU row forward
(vn_lstm_rows_set_diag, diagnostics): which blocks share a CU, which groups
they belong to, and each group's step durations."""
import ctypes as C
import os
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "3d-navigation-reinforcement-learning_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from types import SimpleNamespace  # noqa: E402

from voxnav import _native, lstm_seq  # noqa: E402


def group_of(bid, NT, mp=0):
    G = 2 * NT
    half = 8 * G
    second = bid >= half
    b = bid - half if second else bid
    ub = b // G + (8 if second else 0)
    g = b % G
    if second:
        g = (g + NT) % G
    return ub, g


def run(B, mp, L=128):
    dev = "cuda:0"
    os.environ["VOXNAV_ROWS_V2"] = "1"
    D, H, N = 80, 256, max(B, 64)
    NT = -(-B // 32)
    grid = 2 * 16 * NT
    torch.manual_seed(0)
    la, lc = torch.nn.LSTM(D, H).to(dev), torch.nn.LSTM(D, H).to(dev)
    pol = SimpleNamespace(lstm_actor=la, lstm_critic=lc)
    x = torch.randn((L, B, D), device=dev)
    env = torch.randint(0, N, (L, B), device=dev, dtype=torch.int32)
    start = torch.zeros((L, B), device=dev, dtype=torch.uint8)
    start[0] = 1
    keep = torch.ones((L, B), device=dev)
    hs = 0.5 * torch.randn((L, 2, N, H), device=dev)
    cs = 0.5 * torch.randn((L, 2, N, H), device=dev)
    lib = _native.load()
    lib.vn_lstm_rows_set_diag.argtypes = [C.c_void_p]
    diag = torch.zeros(2 * grid + grid * L * 8, dtype=torch.int32, device=dev)
    with torch.no_grad():
        lstm_seq.dual_lstm_rows_pair(pol, x, env, start, keep, hs, cs)   # warm
        torch.cuda.synchronize()
        lib.vn_lstm_rows_set_diag(C.c_void_p(diag.data_ptr()))
        lstm_seq.dual_lstm_rows_pair(pol, x, env, start, keep, hs, cs)
        torch.cuda.synchronize()
        lib.vn_lstm_rows_set_diag(None)
    lstm_seq.rows_check(torch.device(dev))
    d = diag.cpu().numpy().astype(np.uint32)
    hw, xcc = d[0:2 * grid:2], d[1:2 * grid:2]
    mk = d[2 * grid:].reshape(grid, L, 8).astype(np.int64)
    mk = mk - mk[:, :, :7].min()
    clk = mk[:, :, 6]
    sec = np.diff(mk[:, 1:, :7], axis=2) * 10 / 1000.0   # us, steps 1..
    names = ["x part", "wait", "h loads", "h mfma+gts", "epilogue", "barrier+add"]
    print("  sections (median us over blocks, steps >= 1):",
          ", ".join(f"{n} {np.median(sec[:, :, i]):.2f}" for i, n in enumerate(names)),
          f"| 6->next 0 {np.median((mk[:, 2:, 0] - mk[:, 1:-1, 6]) * 10 / 1000.0):.2f}")
    print("  sections p90:", ", ".join(f"{n} {np.percentile(sec[:, :, i], 90):.2f}" for i, n in enumerate(names)))
    cu = [(int(xcc[b]) & 0xF, (int(hw[b]) >> 8) & 0xFF) for b in range(grid)]
    members = defaultdict(list)
    for b in range(grid):
        members[cu[b]].append(b)
    occ = defaultdict(int)
    for k, v in members.items():
        occ[len(v)] += 1
    print(f"B={B} grid={grid}: CUs used {len(members)}, blocks per CU {dict(occ)}")
    rel = defaultdict(int)
    for k, v in members.items():
        if len(v) == 2:
            (u0, g0), (u1, g1) = group_of(v[0], NT, mp), group_of(v[1], NT, mp)
            rel["same group" if g0 == g1 else ("other LSTM same tile" if g0 % NT == g1 % NT else "other group")] += 1
            rel[f"bid diff {abs(v[1] - v[0])}"] += 1
    print("  pair relations:", dict(sorted(rel.items(), key=lambda kv: -kv[1])[:8]))
    print("  first CUs:", [(k, v) for k, v in list(members.items())[:6]])
    G = 2 * NT
    gend = np.zeros((G, L), dtype=np.int64)
    for b in range(grid):
        _, g = group_of(b, NT, mp)
        gend[g] = np.maximum(gend[g], clk[b])
    dur = np.diff(gend, axis=1) * 10 / 1000.0   # us (100 MHz clock)
    print(f"  group step us: median {np.median(dur):.2f}  p10 {np.percentile(dur, 10):.2f}  p90 {np.percentile(dur, 90):.2f}"
          f"  per-group medians {np.round(np.median(dur, axis=1)[:8], 2)}")
    # phase of LSTM 1's groups against LSTM 0's (same row tile), by step
    ph = (gend[NT:] - gend[:NT]) * 10 / 1000.0
    print("  LSTM1 - LSTM0 step-end offset us, median over tiles, steps 0,1,2,4,8,16,64,127:",
          [round(float(np.median(ph[:, t])), 2) for t in (0, 1, 2, 4, 8, 16, 64, 127)])
    t0 = mk[:, 0, 0] * 10 / 1000.0
    l_of = np.array([group_of(b, NT, mp)[1] // NT for b in range(grid)])
    print(f"  step-0 start us: LSTM0 {np.median(t0[l_of == 0]):.2f}  LSTM1 {np.median(t0[l_of == 1]):.2f}")
    # spread of the blocks of one group at the end of a step (us)
    spread = []
    for g in range(G):
        bl = [b for b in range(grid) if group_of(b, NT, mp)[1] == g]
        spread.append(np.median(clk[bl].max(0) - clk[bl].min(0)) * 10 / 1000.0)
    print(f"  within-group finish spread us (median over steps): {np.round(spread[:8], 2)}")
    print(f"  total {clk.max() * 10 / 1e6:.3f} ms; group step us by step quarter:",
          [round(float(np.median(dur[:, i * (L // 4):(i + 1) * (L // 4) - 1])), 2) for i in range(4)])


if __name__ == "__main__":
    for B in (256, 512):
        run(B, 0)
