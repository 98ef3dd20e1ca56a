"""Calibrate the CPU baseline: time the UNMODIFIED reference env
(envs/CubicEnv.py, behind gen_golden.py's in-memory gymnasium stub) and
the from-scratch restatement oracle/py_cubic.py on the same workload, one
process each, in this build container (the reference cannot travel to the
GPU box, so bench.py times the restatement there).

Workload: 32x32x8 walled box (room_path=None ctor box), L=10, uniform
random actions, auto-reset on done.  The reference prints a line per
episode end (:214, :220); stdout is swallowed for both.

Usage:  python tests/golden/calibrate_py_baseline.py [--seconds 10]
Writes profiles/py_baseline_calibration.json.
"""
from __future__ import annotations

import argparse
import contextlib
import io
import json
import platform
import sys
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(HERE))


def run(env, reset, seconds):
    acts = np.random.default_rng(42).integers(0, 6, size=1 << 16)
    reset(env, 42)
    n = ep = 0
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(io.StringIO()):
        while time.perf_counter() - t0 < seconds:
            for a in acts[(n & 0xFFFF):(n & 0xFFFF) + 256]:
                _, _, te, tr, *_ = env.step(int(a))
                if te or tr:
                    ep += 1
                    reset(env, 42 + ep)
            n += 256
    return n / (time.perf_counter() - t0), ep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=10.0)
    a = ap.parse_args()
    import gen_golden
    gen_golden._install_gym_stub()
    ref = gen_golden._load("ref_cubic_env", "envs/CubicEnv.py")
    from oracle.oracle import walled_box
    from oracle.py_cubic import PyCubicAgent
    renv = ref.GridAgent(width=32, depth=32, height=8, local_map_length=10)
    r_rate, r_ep = run(renv, lambda e, s: e.reset(seed=s), a.seconds)
    penv = PyCubicAgent([walled_box(32, 32, 8)], local_map_length=10, use_room_draw=False)
    p_rate, p_ep = run(penv, lambda e, s: e.reset(s), a.seconds)
    cpu = next((l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")), "?")
    out = {"workload": "32x32x8 ctor box, L=10, uniform random actions, 1 env, 1 process",
           "reference_envs_CubicEnv_steps_per_s": round(r_rate, 1),
           "restatement_oracle_py_cubic_steps_per_s": round(p_rate, 1),
           "restatement_over_reference": round(p_rate / r_rate, 3),
           "seconds_each": a.seconds, "episodes": [r_ep, p_ep], "cpu_model": cpu,
           "python": platform.python_version(), "numpy": np.__version__}
    dst = REPO / "profiles" / "py_baseline_calibration.json"
    dst.write_text(json.dumps(out, indent=1) + "\n")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
