"""Evaluation metrics (train/evaluate_grid.py) and checkpoint layout/naming
(train/Grid_Train.py:229-233) -- SURVEY.md 8(f) row 3.

GPU parity: ``evaluate_policy`` episodes replayed through the CPU oracle
env with the recorded actions give the same score (f64 sum, exact), steps,
bumps, discovered cells and finished flag; the recorded actions are the
argmax of the f64 policy oracle wherever the top-2 logit margin exceeds
1e-3 (f32 vs f64 policy arithmetic).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from helpers import oracle_env, product_room_set  # noqa: E402


def _policies():
    from voxnav.policy import ActorCriticPolicy, RecurrentActorCriticPolicy
    torch.manual_seed(3)
    arch = dict(pi=[64, 32], vf=[64, 32])
    return dict(lstm=RecurrentActorCriticPolicy(lstm_hidden_size=32, net_arch=arch),
                mlp=ActorCriticPolicy(net_arch=arch))


# ------------------------------------------------------------------ CPU
def test_checkpoint_name_matches_grid_train():
    from voxnav.checkpoint import checkpoint_name, eval_phase_for_steps
    arch = dict(pi=[256, 256, 128], vf=[256, 256, 128])
    assert (checkpoint_name(0, arch, 256, 250000, 10)
            == "rppo_hp1_arch_pi[256, 256, 128]_vf[256, 256, 128]_lstm_h256l1_shared_s250000_view10.zip")
    assert [eval_phase_for_steps(s) for s in (1_000_000, 1_000_001, 21_000_000, 21_000_001)] == \
        ["P1_empty", "P2_small", "P2_small", "P3_large"]


@pytest.mark.parametrize("kind", ["lstm", "mlp"])
def test_checkpoint_round_trip(tmp_path, kind):
    from voxnav.checkpoint import load_checkpoint, load_optimizer_state, save_checkpoint
    pol = _policies()[kind]
    opt = torch.optim.Adam(pol.parameters(), lr=3e-4, eps=1e-5)
    loss = sum((p * p).sum() for p in pol.parameters())
    loss.backward()
    opt.step()
    path = save_checkpoint(tmp_path / "ck", pol, opt, num_timesteps=1234, hyperparams=dict(batch_size=64))
    assert path.suffix == ".zip"
    import zipfile
    with zipfile.ZipFile(path) as z:
        assert {"data", "policy.pth", "policy.optimizer.pth", "pytorch_variables.pth",
                "_stable_baselines3_version"} <= set(z.namelist())
    pol2, data = load_checkpoint(path)
    assert data["num_timesteps"] == 1234 and data["hyperparams"]["batch_size"] == 64
    assert type(pol2) is type(pol)
    for (k, a), (k2, b) in zip(pol.state_dict().items(), pol2.state_dict().items()):
        assert k == k2 and torch.equal(a, b)
    opt2 = torch.optim.Adam(pol2.parameters(), lr=3e-4, eps=1e-5)
    assert load_optimizer_state(path, opt2)
    s1, s2 = opt.state_dict()["state"], opt2.state_dict()["state"]
    assert all(torch.equal(s1[i]["exp_avg"], s2[i]["exp_avg"]) for i in s1)


def test_results_table_row_format():
    from voxnav.evaluate import RESULTS_HEADER, results_table_row
    r = dict(avg_score=12.345, avg_bumps=3.0, finished_pct=40.0, avg_discovered=55.5, avg_steps=72.0)
    row = results_table_row("m", r)
    assert row == f"{'m':<40} | {12.35:>12.2f} | {3.0:>12.2f} | {40.0:>14.1f}% | {55.5:>18.2f} | {72.0:>12.2f}"
    assert len(row) == len(RESULTS_HEADER)


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["lstm", "mlp"])
def test_evaluate_policy_matches_oracle_replay(kind):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle.collector_oracle import PolicyOracle
    from voxnav.evaluate import evaluate_policy
    from voxnav.policy import numpy_weights
    pol = _policies()[kind]
    with torch.no_grad():
        pol.action_net.weight.mul_(300.0)      # decisive logits: argmax robust to f32 vs f64
    pol = pol.to("cuda:0")
    src, L, n, seed = "set:P1_training", 4, 12, 100
    r = evaluate_policy(pol, product_room_set(src), n_episodes=n, local_map_length=L, seed=seed,
                        device="cuda:0", record_actions=True)
    acts = r["actions"]
    po = PolicyOracle(numpy_weights(pol))
    oenv = oracle_env(src, L, n_agents=n)
    checked = 0
    for i in range(n):
        obs = oenv.reset(i, seed + i)
        H = po.H
        h = np.zeros((2, 1, H))
        c = np.zeros((2, 1, H))
        score, steps = 0.0, 0
        for t in range(acts.shape[0]):
            logits, _, h2, c2 = po.forward(obs[None], h, c, np.array([1.0 if t == 0 else 0.0]))
            if po.recurrent:
                h, c = h2, c2
            srt = np.sort(logits[0])
            if srt[-1] - srt[-2] > 1e-3:
                assert int(np.argmax(logits[0])) == int(acts[t, i]), (i, t)
                checked += 1
            obs, rew, te, tr = oenv.step(i, int(acts[t, i]))
            score += rew
            steps += 1
            if te or tr:
                break
        e = r["episodes"][i]
        st = oenv.state(i)
        assert (e["steps"], e["bumps"], e["discovered_cells"], e["finished"]) == \
            (steps, st["bump_count"], st["visited_count"], bool(st["done"])), i
        assert e["score"] == pytest.approx(score, rel=0, abs=1e-9), i
    assert checked > n * 10
    assert r["avg_steps"] == pytest.approx(np.mean([e["steps"] for e in r["episodes"]]))
