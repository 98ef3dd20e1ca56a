"""bench.py's launch path and window bookkeeping on CPU (no GPU).

* ``--gpus 2`` starts two ranks itself (torch.distributed.run child, gloo in
  the --dry-run rehearsal) and rank 0 prints one JSON line with n_gpus 2;
* the timed window is exactly --steps steps (F-step launches, remainder
  last), so the line's ``steps``/``warmup`` equal the flags;
* the Python/NumPy CPU baseline runs P processes x 1 env.
"""
import json
import subprocess
import sys

import pytest

from helpers import REPO

sys.path.insert(0, str(REPO))
import bench  # noqa: E402


def test_launch_sizes_cover_exactly():
    assert bench.launches(20, 16) == [16, 4]
    assert bench.launches(5, 16) == [5]
    assert bench.launches(5408, 16) == [16] * 338
    assert bench.launches(0, 16) == []
    for k in (1, 15, 16, 17, 100, 5408):
        assert sum(bench.launches(k, 16)) == k


def test_gpus2_launches_two_ranks_dry_run():
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--dry-run"], cwd=str(REPO),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["ranks"] == [0, 1] and rec["dry_run"] is True


def test_world_size_mismatch_is_rejected():
    env = {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}
    import os
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--dry-run"], cwd=str(REPO),
                       capture_output=True, text=True, timeout=120, env={**os.environ, **env})
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr


def test_python_numpy_baseline_runs_processes():
    v, steps, _ = bench.python_numpy_baseline("8x8x4", 4, 1.0, 2)
    assert steps >= 512 and v > 0
