#!/usr/bin/env python3
"""Host-side overhead around one timed env launch (the driver's
--steps 20 --warmup 5 window): wall time of synchronize -> launch ->
synchronize with and without the HIP events bench.py records, against the
kernel time those events measure."""
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "3d-navigation-reinforcement-learning_amd"))
import torch  # noqa: E402

from voxnav.env import BatchedGridEnv, Rollout  # noqa: E402
from voxnav.rooms import box_room, single_room_set  # noqa: E402


def main():
    N, F, K = 65536, 128, 20
    dev = torch.device("cuda:0")
    out = Rollout(torch.empty((F, N, 80), device=dev), torch.empty((F, N), device=dev),
                  torch.empty((F, N), dtype=torch.uint8, device=dev), torch.empty((F, N), dtype=torch.uint8, device=dev),
                  None)
    view = Rollout(out.obs[:K], out.reward[:K], out.terminated[:K], out.truncated[:K], None)
    res = {"events": [], "plain": [], "kernel_us": []}
    for rep in range(6):
        env = BatchedGridEnv(num_agents=N, rooms=single_room_set(box_room(32, 32, 8)), local_map_length=10,
                             device=dev)
        env.reset(seed=42)
        env.step_random(5, policy_seed=42, out=Rollout(out.obs[:5], out.reward[:5], out.terminated[:5],
                                                       out.truncated[:5], None))
        fn = env.step_random_launcher(K, 42, 5, view)
        stream = torch.cuda.current_stream(dev)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        if rep % 2 == 0:
            a.record(stream)
            fn()
            b.record(stream)
        else:
            fn()
        torch.cuda.synchronize(dev)
        el = (time.perf_counter() - t0) * 1e6
        if rep % 2 == 0:
            res["events"].append(round(el, 1))
            res["kernel_us"].append(round(a.elapsed_time(b) * 1e3, 1))
        else:
            res["plain"].append(round(el, 1))
        env.close()
    print(res)


if __name__ == "__main__":
    main()
