"""The SB3 VecEnv adapter (voxnav.vec_env.VoxnavVecEnv) against the CPU
oracle's auto-reset replay (``done = term or trunc``,
``info["TimeLimit.truncated"] = trunc and not term``, on done
``info["terminal_observation"] = obs`` and ``obs = reset()``; the Monitor's
``info["episode"] = {"r": round(sum(rewards), 6), "l": len, "t": ...}``).

SB3 is not installed, so the contract is the restatement; the env outputs
are bit-exact against the oracle, the episode returns are the f64 sums of
the oracle's rewards in step order.
"""
import numpy as np
import pytest

from helpers import oracle_env, product_room_set


def test_build_infos_contract():
    """Host-side info building (no GPU)."""
    pytest.importorskip("torch")
    from voxnav.vec_env import build_infos
    te = np.array([0, 1, 0, 1, 0], bool)
    tr = np.array([0, 0, 1, 1, 0], bool)
    tobs = np.arange(5 * 3, dtype=np.float32).reshape(5, 3)
    r = np.array([0.0, 1.25, -2.5, 3.0000004, 0.0])
    ln = np.array([0, 7, 9, 11, 0], np.int32)
    infos = build_infos(te, tr, tobs, r, ln, 1.23456789)
    assert [d["TimeLimit.truncated"] for d in infos] == [False, False, True, False, False]
    assert [("terminal_observation" in d) for d in infos] == [False, True, True, True, False]
    assert infos[2]["episode"] == {"r": -2.5, "l": 9, "t": 1.234568}
    assert infos[3]["episode"]["r"] == 3.0
    np.testing.assert_array_equal(infos[1]["terminal_observation"], tobs[1])
    no_mon = build_infos(te, tr, tobs, None, None, 0.0)
    assert all("episode" not in d for d in no_mon)


@pytest.mark.gpu
def test_vec_env_matches_oracle_autoreset_replay():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from voxnav.vec_env import VoxnavVecEnv
    src, L, N, K = "box:8x8x4", 4, 96, 230          # 72-step episodes: three truncations per agent
    venv = VoxnavVecEnv(N, rooms=product_room_set(src), local_map_length=L, seed=42, device="cuda:0")
    assert venv.num_envs == N and venv.observation_space.shape == (80,) and venv.action_space.n == 6
    assert venv.env_is_wrapped(type("Monitor", (), {})) == [True] * N
    obs = venv.reset()
    oenv = oracle_env(src, L, n_agents=N)
    seeds = 42 + np.arange(N)
    ref0 = np.stack([oracle_env(src, L).reset(0, int(s)) for s in seeds])
    assert obs.dtype == np.float32 and obs.tobytes() == ref0.tobytes()
    acts = np.random.default_rng(3).integers(0, 6, size=(K, N))
    orc = oenv.run_random(seeds, 0, K, seed_stride=N, actions=acts.astype(np.int32), terminal_obs=True)
    ret = np.zeros(N)
    length = np.zeros(N, np.int64)
    n_eps = 0
    for k in range(K):
        obs, rew, dones, infos = venv.step(acts[k])
        assert obs.tobytes() == orc["obs"][k].tobytes(), f"obs at step {k}"
        assert rew.dtype == np.float64 and np.array_equal(rew, orc["reward"][k])
        te, tr = orc["terminated"][k].astype(bool), orc["truncated"][k].astype(bool)
        np.testing.assert_array_equal(dones, te | tr)
        ret += orc["reward"][k]
        length += 1
        for i in range(N):
            d = infos[i]
            assert d["TimeLimit.truncated"] == bool(tr[i] and not te[i])
            if te[i] or tr[i]:
                assert d["terminal_observation"].tobytes() == orc["terminal_obs"][k][i].tobytes()
                assert d["episode"]["r"] == round(float(ret[i]), 6) and d["episode"]["l"] == int(length[i])
                assert d["episode"]["t"] >= 0.0
                ret[i], length[i] = 0.0, 0
                n_eps += 1
            else:
                assert "terminal_observation" not in d and "episode" not in d
    assert n_eps >= 3 * N
    assert len(venv.monitor.ep_info_buffer) == 100
    # attributes Grid_Train / evaluate_grid read, from the device state
    st = oenv.state(5)
    assert venv.get_attr("visited_count", 5) == [st["visited_count"]]
    assert venv.get_attr("bump_count", [5]) == [st["bump_count"]]
    assert venv.get_attr("total_free_cells", 0) == [72]
    assert venv.env_method("get_position", indices=[5]) == [(st["x"], st["y"], st["z"])]
    with pytest.raises(KeyError):
        venv.step(np.full(N, 6))
    # seed(): the next reset seeds env i with s + i
    venv.seed(1000)
    obs = venv.reset()
    ref = np.stack([oracle_env(src, L).reset(0, 1000 + i) for i in range(N)])
    assert obs.tobytes() == ref.tobytes()
    # a reset without seed() continues each env's pinned seed schedule (SB3
    # resets with seed=None): env i's next seed is 1000 + i + N, no replay
    t_start = venv.monitor.t_start
    obs = venv.reset()
    ref2 = np.stack([oracle_env(src, L).reset(0, 1000 + N + i) for i in range(N)])
    assert obs.tobytes() == ref2.tobytes()
    assert venv.monitor.t_start == t_start          # Monitor keeps t_start from construction
    venv.close()
