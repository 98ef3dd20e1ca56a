"""SB3 Monitor statistics (voxnav.monitor, train/Grid_Train.py:125) and the
EvalCallback cadence (voxnav.evaluate.EvalCallback, Grid_Train.py:218-226).

Monitor bar: every finished episode's return equals the f64 sum, in step
order, of the oracle's f64 rewards for that agent (bit-exact), its length
and the (step, agent) order equal the oracle replay's; ep_rew_mean /
ep_len_mean are SB3's safe_mean over the last 100 episodes.
"""
import numpy as np
import pytest

from helpers import box_text

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

BOXES = [(8, 8, 4), (6, 6, 4), (7, 5, 5), (5, 5, 4)]


@pytest.fixture(scope="module")
def voxnav():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import voxnav
    voxnav.load_library()
    return voxnav


def _small_policy(recurrent=True):
    from voxnav.policy import ActorCriticPolicy, RecurrentActorCriticPolicy
    torch.manual_seed(4)
    arch = dict(pi=[32, 16], vf=[32, 16])
    pol = RecurrentActorCriticPolicy(lstm_hidden_size=16, net_arch=arch) if recurrent else \
        ActorCriticPolicy(net_arch=arch)
    return pol.to("cuda:0")


@pytest.mark.parametrize("recurrent", [True, False], ids=["lstm", "mlp"])
def test_monitor_episodes_match_oracle_replay(voxnav, recurrent):
    from oracle.oracle import OracleEnv, parse_room_text
    from voxnav.collector import RolloutCollector
    from voxnav.env import BatchedGridEnv
    from voxnav.rooms import RoomSet, parse_room
    N, L, T, R = 96, 4, 40, 3
    texts = [(f"box{w}x{d}x{h}.txt", box_text(w, d, h)) for (w, d, h) in BOXES]
    prod = RoomSet([parse_room(t, n) for n, t in texts], use_room_draw=True, source="boxes")
    env = BatchedGridEnv(num_agents=N, rooms=prod, local_map_length=L, device="cuda:0")
    col = RolloutCollector(env, _small_policy(recurrent), n_steps=T, sample_seed=3, reset_seed=42)
    oenv = OracleEnv([parse_room_text(t, n) for n, t in texts], n_agents=N, local_map_length=L)
    seeds = 42 + np.arange(N)
    run_ret = np.zeros(N, np.float64)
    run_len = np.zeros(N, np.int64)
    all_r = []
    for r in range(R):
        buf = col.collect()
        acts = buf.actions.cpu().numpy()
        rr = oenv.run_random(seeds, 0, T, t0=r * T, seed_stride=N, initial_reset=(r == 0), actions=acts)
        want = []
        for t in range(T):
            for a in range(N):
                run_ret[a] = run_ret[a] + rr["reward"][t, a]      # Monitor: sum(rewards) in step order
                run_len[a] += 1
                if rr["terminated"][t, a] or rr["truncated"][t, a]:
                    want.append((t, a, run_ret[a], run_len[a]))
                    run_ret[a] = 0.0
                    run_len[a] = 0
        got = col.monitor.last_episodes
        assert got["step"].tolist() == [w[0] for w in want]
        assert got["agent"].tolist() == [w[1] for w in want]
        assert got["length"].tolist() == [int(w[3]) for w in want]
        assert got["return"].cpu().numpy().tobytes() == np.array([w[2] for w in want], np.float64).tobytes()
        all_r += [round(float(w[2]), 6) for w in want]
    assert len(all_r) > 100
    assert col.monitor.total_episodes == len(all_r)
    assert col.monitor.ep_rew_mean() == float(np.mean(all_r[-100:]))
    env.close()


def test_learn_reports_monitor_and_eval_callback(voxnav, tmp_path):
    """learn() history carries ep_rew_mean / ep_len_mean; EvalCallback runs at
    the SB3 cadence, logs evaluations.npz and saves best_model.zip whose
    weights reproduce the best evaluation."""
    from voxnav.checkpoint import load_checkpoint
    from voxnav.collector import RolloutCollector
    from voxnav.env import BatchedGridEnv
    from voxnav.evaluate import EvalCallback, evaluate_policy
    from voxnav.ppo import PPOLearner, learn
    from voxnav.rooms import RoomSet, parse_room
    pol = _small_policy(True)
    rooms = RoomSet([parse_room(box_text(w, d, h), f"b{w}{d}{h}.txt") for (w, d, h) in BOXES], use_room_draw=True,
                    source="boxes")
    env = BatchedGridEnv(num_agents=64, rooms=rooms, local_map_length=10, device="cuda:0")
    T = 32
    col = RolloutCollector(env, pol, n_steps=T)
    ln = PPOLearner(pol, n_epochs=1, batch_size=1024, seed=1)
    eval_rooms = RoomSet([parse_room(box_text(w, d, h), f"e{w}{d}{h}.txt") for (w, d, h) in ((9, 7, 4), (6, 8, 5))],
                         use_room_draw=True, source="eval-boxes")
    cb = EvalCallback(eval_rooms, eval_freq=48, n_eval_episodes=10, best_model_save_path=tmp_path / "best",
                      log_path=tmp_path / "log", local_map_length=10)
    hist = learn(col, ln, total_timesteps=5 * T * 64, callback=cb)
    assert len(hist) == 5
    # calls 32, 64, 96, 128, 160: multiples of 48 crossed after rollouts 2 (48), 3 (96), 5 (144)
    evaluated = [i for i, h in enumerate(hist) if "eval/mean_reward" in h]
    assert evaluated == [1, 2, 4]
    assert cb.evaluations_timesteps == [2 * T * 64, 3 * T * 64, 5 * T * 64]
    z = np.load(tmp_path / "log" / "evaluations.npz")
    assert z["results"].shape == (3, 10) and z["ep_lengths"].shape == (3, 10)
    assert np.array_equal(z["timesteps"], cb.evaluations_timesteps)
    assert cb.best_mean_reward == max(float(np.mean(r)) for r in z["results"])
    pol2, data = load_checkpoint(tmp_path / "best" / "best_model.zip", device="cuda:0")
    k = int(np.argmax([float(np.mean(r)) for r in z["results"]]))
    assert data["num_timesteps"] == cb.evaluations_timesteps[k]
    again = evaluate_policy(pol2, eval_rooms, n_episodes=10, local_map_length=10, seed=cb.seed + k * 10)
    assert [round(e["score"], 6) for e in again["episodes"]] == list(z["results"][k])
    with_mon = [h for h in hist if "ep_rew_mean" in h]
    assert with_mon, "episodes finish within 5 rollouts in the <= 72-cell boxes"
    assert all(np.isfinite(h["ep_rew_mean"]) and h["ep_len_mean"] > 0 for h in with_mon)
    env.close()
