"""The collector's f32 GEMM shapes (65,536 rows) under torch's two ROCm BLAS
backends (hipBLASLt, the default; "hipblas", i.e. rocBLAS; and CK): MLP layers 256 -> 256 and
256 -> 128 with bias (addmm), the recurrent product 256 -> 1024 and the
input projection 80 -> 2048 (mm).  HIP events, one JSON line per case."""
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
    N = 65536
    g = torch.Generator(device=dev).manual_seed(0)
    cases = {"mlp_256_256": (256, 256, True), "mlp_256_128": (256, 128, True), "w_hh_256_1024": (256, 1024, False),
             "w_ih_80_2048": (80, 2048, False)}
    for dt in (torch.float32, torch.bfloat16):
        for name, (k, n, bias) in cases.items():
            x = torch.randn(N, k, device=dev, generator=g).to(dt)
            w = (torch.randn(n, k, device=dev, generator=g) * 0.05).to(dt)
            b = torch.randn(n, device=dev, generator=g).to(dt)
            out = torch.empty(N, n, device=dev, dtype=dt)
            fn = (lambda: torch.addmm(b, x, w.t(), out=out)) if bias else (lambda: torch.mm(x, w.t(), out=out))
            res = {}
            for lib in ("hipblaslt", "hipblas", "ck"):
                try:
                    torch.backends.cuda.preferred_blas_library(lib)
                    res[lib] = round(timeit(fn), 1)
                except Exception as e:  # noqa: BLE001
                    res[lib] = f"error: {e}"
            torch.backends.cuda.preferred_blas_library("hipblaslt")
            print(json.dumps({"dtype": str(dt), "case": name, "us": res}), flush=True)


if __name__ == "__main__":
    main()
