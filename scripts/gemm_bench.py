#!/usr/bin/env python3
"""The learner's f32 matrix-core products at the bench minibatch (65,536
samples; csrc/voxnav_gemm_f32.hip through its C-ABI), each timed alone with
HIP events: microseconds and TF/s per shape.
python scripts/gemm_bench.py [reps]"""
import ctypes as C
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "3d-navigation-reinforcement-learning_amd"))
import torch  # noqa: E402

from voxnav import _native, learn_ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = "cuda:0"
lib = _native.load()
torch.manual_seed(0)
M = 65536


def p(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def st():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def timeit(name, flops, fn):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    print(f"{name:46s} {us:9.1f} us  {flops / us / 1e6:7.1f} TF/s", flush=True)


for K, N in ((80, 256), (256, 256), (256, 128)):
    x = torch.randn((2, M, K), device=dev)
    w = torch.randn((2, N, K), device=dev) * 0.05
    b = torch.randn((2, N), device=dev)
    y = torch.empty((2, M, N), device=dev)
    timeit(f"linear+tanh pair  M{M} K{K} N{N}", 2 * 2 * M * K * N,
           lambda: _native.check(lib.vn_gemm_f32_linear(p(x), K, M * K, p(w), K, N * K, p(b), N, p(y), N, M * N, M,
                                                        N, K, 2, 1, st())))
    dy = torch.randn((2, M, N), device=dev)
    yy = torch.tanh(torch.randn((2, M, N), device=dev))
    dx = torch.empty((2, M, K), device=dev)
    timeit(f"dX (tanh bwd) pair M{M} N{N} -> K{K}", 2 * 2 * M * K * N,
           lambda: _native.check(lib.vn_gemm_f32_dx(p(dy), p(yy), N, M * N, p(w), K, N * K, p(dx), K, M * K, M, K, N,
                                                    2, st())))
    timeit(f"dW (tanh bwd) pair [{N}x{K}] over {M}", 2 * 2 * M * K * N,
           lambda: learn_ops.mm_tn(dy, x, y=yy, colsum=True))

G, H, D = 1024, 256, 80
dG = torch.randn((2, M, G), device=dev)
hp = torch.randn((2, M, H), device=dev)
xx = torch.randn((1, M, D), device=dev).expand(2, M, D)
timeit(f"LSTM dW_hh [{G}x{H}] x2 over {M}", 2 * 2 * M * G * H, lambda: learn_ops.mm_tn(dG, hp))
timeit(f"LSTM dW_ih [{G}x{D}] x2 over {M} (+colsum)", 2 * 2 * M * G * D, lambda: learn_ops.mm_tn(dG, xx, colsum=True))
