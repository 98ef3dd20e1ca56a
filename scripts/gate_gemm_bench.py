"""f32 gate GEMMs of the PPO-LSTM collector step (65,536 agents, obs 80,
H 256, actor + critic): today's three products (x @ W_ih_cat^T into gx
[N, 8H], h_b @ W_hh_b^T into gh [2, N, 4H]) vs per-LSTM contiguous gates
(x @ W_ih_b^T into g[b], then g[b] += h_b @ W_hh_b^T with beta = 1), which
would let the cell kernel read one gate array.  GEMM time only, HIP events."""
import json

import torch


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dev = "cuda"
    N, od, H = 65536, 80, 256
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand(N, od, device=dev, generator=g)
    h = torch.randn(2, N, H, device=dev, generator=g) * 0.3
    wih = torch.randn(2, 4 * H, od, device=dev, generator=g) * 0.05
    whh = torch.randn(2, 4 * H, H, device=dev, generator=g) * 0.05
    wih_cat = wih.reshape(8 * H, od).contiguous()
    gx = torch.empty(N, 8 * H, device=dev)
    gh = torch.empty(2, N, 4 * H, device=dev)
    gates = torch.empty(2, N, 4 * H, device=dev)

    def three():
        torch.mm(x, wih_cat.t(), out=gx)
        torch.mm(h[0], whh[0].t(), out=gh[0])
        torch.mm(h[1], whh[1].t(), out=gh[1])

    def acc():
        for b in range(2):
            torch.mm(x, wih[b].t(), out=gates[b])
            gates[b].addmm_(h[b], whh[b].t())

    three()
    acc()
    err = max(float((gates[b] - gx[:, b * 4 * H:(b + 1) * 4 * H] - gh[b]).abs().max()) for b in range(2))
    for name, fn in (("three_products", three), ("per_lstm_accumulate", acc)):
        print(json.dumps({"variant": name, "us": round(timeit(fn), 1), "max_abs_diff": err}), flush=True)


if __name__ == "__main__":
    main()
