#!/usr/bin/env python3
"""Time vn_lstm_fused_bf16 (both LSTMs, N=65536, H=256, obs 80) vs the
unfused bf16 path (library GEMMs + vn_lstm_cell_bf16), HIP events."""
import ctypes as C
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "3d-navigation-reinforcement-learning_amd"))
import torch  # noqa: E402

from voxnav import _native  # noqa: E402


def main():
    lib = _native.load() if len(sys.argv) < 2 else _native.load_variant(sys.argv[1])
    dev = "cuda:0"
    B, N, H, od = 2, 65536, 256, 80
    kx = (od + 7) // 8 * 8
    Kp = (kx + H + 63) // 64 * 64
    x = torch.rand((N, od), device=dev)
    hin = (torch.rand((B, N, H), device=dev) - 0.5).bfloat16()
    hout = torch.empty_like(hin)
    w = ((torch.rand((B, 4 * H, Kp), device=dev) - 0.5) * 0.1).bfloat16()
    bias = torch.zeros((B, 4 * H), device=dev)
    c = torch.zeros((B, N, H), device=dev)
    hs = torch.empty((B, N, H), device=dev)
    cs = torch.empty((B, N, H), device=dev)
    p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731

    def fused():
        assert lib.vn_lstm_fused_bf16(p(x), od, p(hin), p(w), Kp, p(bias), p(c), p(hout), None, p(hs), p(cs), B, N, H,
                                      None) == 0
    start = (torch.rand(N, device=dev) < 0.02).float()   # ~2 % of the agents start an episode
    c_out = torch.empty_like(c)

    def masked():   # the collector's rollout entry: c_in -> c_out, mask on read, no c_store
        assert lib.vn_lstm_fused_bf16_masked(p(x), od, p(hin), p(w), Kp, p(bias), p(c), p(start), p(c_out), p(hout),
                                             p(hs), B, N, H, None) == 0
    wih = w[:, :, :od].reshape(B * 4 * H, od).contiguous()
    whh = [w[b, :, kx:kx + H].contiguous() for b in range(B)]
    gx = torch.empty((N, B * 4 * H), dtype=torch.bfloat16, device=dev)
    gh = torch.empty((B, N, 4 * H), dtype=torch.bfloat16, device=dev)
    h32 = torch.empty((B, N, H), device=dev)

    def unfused():
        torch.mm(x.bfloat16(), wih.t(), out=gx)
        for b in range(B):
            torch.mm(hin[b], whh[b].t(), out=gh[b])
        assert lib.vn_lstm_cell_bf16(p(gx), 8 * H, p(gh), p(bias), p(bias), p(h32), p(c), p(hout), p(hs), p(cs), B,
                                     N, H, None) == 0
    variants = [("fused", fused), ("unfused", unfused)]
    if hasattr(lib, "vn_lstm_fused_bf16_masked"):
        variants.insert(1, ("fused_masked", masked))
    for name, fn in variants:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        print(f"{name}: {ms * 1e3:.1f} us  ({2 * B * N * (od + H) * 4 * H / ms / 1e9:.1f} TFLOP/s)")


if __name__ == "__main__":
    main()
