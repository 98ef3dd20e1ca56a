"""Timing of the collector's policy MLP layer shapes (65,536 rows, 256 -> 256
-> 256 -> 128, Tanh; actor and critic) as two separate addmm chains vs one
batched chain over both heads.  Prints one JSON line per variant."""
import json
import time

import torch


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    dev = "cuda"
    N, dims = 65536, [256, 256, 256, 128]
    for dt in (torch.float32, torch.bfloat16):
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(2, N, dims[0], device=dev, dtype=dt, generator=g)
        W = [torch.randn(2, dims[i + 1], dims[i], device=dev, dtype=dt, generator=g) * 0.05 for i in range(3)]
        B = [torch.randn(2, dims[i + 1], device=dev, dtype=dt, generator=g) * 0.05 for i in range(3)]
        Wt = [w.transpose(1, 2).contiguous() for w in W]

        def sep():
            outs = []
            for h in range(2):
                y = x[h]
                for w, b in zip(W, B):
                    y = torch.addmm(b[h], y, w[h].t())
                    y.tanh_()
                outs.append(y)
            return outs

        def bat():
            y = x
            for wt, b in zip(Wt, B):
                y = torch.baddbmm(b[:, None, :], y, wt)
                y.tanh_()
            return y

        def bat2():
            y = x
            for wt, b in zip(Wt, B):
                y = torch.bmm(y, wt)
                y.add_(b[:, None, :]).tanh_()
            return y

        ref = sep()
        got = bat()
        err = max((ref[h].float() - got[h].float()).abs().max().item() for h in range(2))
        for name, fn in (("separate_addmm", sep), ("baddbmm", bat), ("bmm_add_tanh", bat2)):
            print(json.dumps({"dtype": str(dt), "variant": name, "us": round(timeit(fn), 1), "max_err_vs_sep": err}),
                  flush=True)


if __name__ == "__main__":
    main()
