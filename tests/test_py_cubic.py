"""Pin the per-agent Python/NumPy restatement (oracle/py_cubic.py, the CPU
baseline bench.py times) against the golden trajectories of the unmodified
reference env (envs/CubicEnv.py, tests/golden/gen_golden.py)."""
import numpy as np
import pytest

from helpers import STATE13, golden_trajectories, grid_hash, load_golden, source_texts
from oracle.oracle import parse_room_text, walled_box
from oracle.py_cubic import PyCubicAgent


def py_env(src: str, L: int, crash_penalty: float):
    texts, draw, whd = source_texts(src)
    rooms = [walled_box(*whd)] if whd else [parse_room_text(t, n) for n, t in texts]
    return PyCubicAgent(rooms, local_map_length=L, crash_penalty=crash_penalty, use_room_draw=draw)


@pytest.mark.parametrize("path", golden_trajectories(), ids=lambda p: p.stem)
def test_py_restatement_replays_golden(path):
    d = load_golden(path)
    env = py_env(str(d["room_source"]), int(d["L"]), float(d["crash_penalty"]))
    seeds = [int(s) for s in d["seeds"]]
    obs = env.reset(seeds[0])
    si, ri = 1, 1
    assert obs.tobytes() == d["reset_obs"][0].tobytes()
    assert [env.state()[f] for f in STATE13] == list(d["reset_state"][0])
    for t, a in enumerate(d["actions"]):
        obs, r, te, tr = env.step(int(a))
        assert obs.tobytes() == d["obs"][t].tobytes(), f"obs mismatch at step {t}"
        assert r == float(d["reward"][t]), f"reward mismatch at step {t}"
        assert (bool(te), bool(tr)) == (bool(d["terminated"][t]), bool(d["truncated"][t])), t
        assert [env.state()[f] for f in STATE13] == list(d["state"][t]), f"state mismatch at step {t}"
        assert grid_hash(env.belief) == int(d["belief_hash"][t]), f"belief mismatch at step {t}"
        if te or tr:
            obs = env.reset(seeds[si])
            si += 1
            assert obs.tobytes() == d["reset_obs"][ri].tobytes()
            ri += 1
    assert si == len(seeds)


def test_py_restatement_timed_runner_steps():
    import time
    from oracle.py_cubic import _run_timed
    t = time.time()
    n, _ = _run_timed((8, 8, 4), 4, 7, t, t + 0.3)
    assert n >= 256
