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


def test_eval_cadence_counts_crossed_multiples():
    from voxnav.evaluate import evals_due
    assert evals_due(0, 32, 48) == 0 and evals_due(32, 64, 48) == 1 and evals_due(64, 96, 48) == 1
    assert evals_due(0, 128, 1) == 128 and evals_due(5, 6, 0) == 0
    # Grid_Train: eval_freq = max(100_000 // NUM_ENVS, 1) vectorized steps
    assert evals_due(0, 12500, max(100_000 // 8, 1)) == 1


def test_learn_callback_plumbing_cpu():
    from voxnav.ppo import learn

    class Col:
        n_steps, N, monitor = 4, 2, None

        def __init__(self, pol):
            self.policy = pol

        def collect(self):
            return None

        def sync_weights(self):
            pass

    class Ln:
        optimizer = None

        def __init__(self, pol):
            self.policy = pol

        def train(self, buf):
            return {"loss": 0.0}

    seen = []

    class Hook:
        def on_rollout_end(self, policy, num_timesteps, n_steps, optimizer=None):
            seen.append((num_timesteps, n_steps))
            return {"eval/mean_reward": 1.0} if num_timesteps == 16 else None

    pol = object()
    calls = []
    hist = learn(Col(pol), Ln(pol), total_timesteps=40, callback=[Hook(), lambda i, n, st: calls.append(n)])
    assert [h["num_timesteps"] for h in hist] == [8, 16, 24, 32, 40]
    assert seen == [(8, 4), (16, 4), (24, 4), (32, 4), (40, 4)]
    assert calls == [8, 16, 24, 32, 40]
    assert "eval/mean_reward" in hist[1] and "eval/mean_reward" not in hist[0]


def _sb3_style_zip(path, policy):
    """An SB3-layout zip (the reference's model.save, Grid_Train.py:233): a
    `data` member whose fields SB3 serializes as base64 cloudpickle blobs
    (never decoded here) and the policy state_dict under SB3's key names."""
    import io
    import json
    import zipfile
    data = {"policy_class": {":type:": "<class 'abc.ABCMeta'>", ":serialized:": "gAWVOw=="},
            "num_timesteps": 1234, "policy_kwargs": {":type:": "<class 'dict'>", ":serialized:": "gAWV"}}
    b = io.BytesIO()
    torch.save({k: v.detach().cpu() for k, v in policy.state_dict().items()}, b)
    with zipfile.ZipFile(path, "w") as z:
        z.writestr("data", json.dumps(data))
        z.writestr("policy.pth", b.getvalue())
        z.writestr("_stable_baselines3_version", "2.3.2")
    return path


@pytest.mark.parametrize("kind", ["lstm", "mlp"])
def test_load_reference_sb3_zip_infers_architecture(tmp_path, kind):
    from voxnav.checkpoint import load_checkpoint
    from voxnav.policy import ActorCriticPolicy, RecurrentActorCriticPolicy
    torch.manual_seed(2)
    arch = dict(pi=[64, 32], vf=[48, 32])
    pol = (RecurrentActorCriticPolicy(lstm_hidden_size=32, net_arch=arch) if kind == "lstm"
           else ActorCriticPolicy(net_arch=arch))
    p = _sb3_style_zip(tmp_path / "rppo_hp1_s1234_view10.zip", pol)
    got, data = load_checkpoint(p)
    assert data == {"sb3": True, "sb3_version": "2.3.2"} and type(got) is type(pol)
    sd, sd2 = pol.state_dict(), got.state_dict()
    assert sd.keys() == sd2.keys() and all(torch.equal(sd[k], sd2[k]) for k in sd)


def test_unknown_voxnav_checkpoint_format_is_refused(tmp_path):
    """A voxnav zip of another format version fails loudly instead of
    loading through the SB3 shape-inference route (which would drop
    num_timesteps, hyperparameters and policy_kwargs)."""
    import json
    import zipfile
    from voxnav.checkpoint import load_checkpoint, save_checkpoint
    from voxnav.policy import ActorCriticPolicy
    torch.manual_seed(3)
    pol = ActorCriticPolicy(net_arch=dict(pi=[16], vf=[16]))
    p = tmp_path / "a.zip"
    save_checkpoint(p, pol, num_timesteps=7)
    q = tmp_path / "b.zip"
    with zipfile.ZipFile(p) as zi, zipfile.ZipFile(q, "w") as zo:
        for n in zi.namelist():
            b = zi.read(n)
            if n == "data":
                d = json.loads(b)
                d["format"] = "voxnav-sb3-layout-999"
                b = json.dumps(d).encode()
            zo.writestr(n, b)
    with pytest.raises(ValueError, match="format"):
        load_checkpoint(q)
    r = tmp_path / "c.zip"                                   # neither voxnav nor SB3
    with zipfile.ZipFile(p) as zi, zipfile.ZipFile(r, "w") as zo:
        zo.writestr("data", json.dumps({"x": 1}))
        zo.writestr("policy.pth", zi.read("policy.pth"))
    with pytest.raises(ValueError, match="neither"):
        load_checkpoint(r)


def test_policy_state_load_is_strict():
    from voxnav.checkpoint import load_policy_state
    from voxnav.policy import RecurrentActorCriticPolicy
    torch.manual_seed(0)
    arch = dict(pi=[16], vf=[16])
    pol = RecurrentActorCriticPolicy(lstm_hidden_size=8, net_arch=arch)
    sd = {k: v.clone() for k, v in pol.state_dict().items()}
    load_policy_state(pol, {**sd, "features_extractor.flatten.dummy": torch.zeros(1)})   # allow-listed prefix
    bad = dict(sd)
    bad["lstm_actor.weight_ih_l1"] = bad.pop("lstm_actor.weight_ih_l0")                 # renamed key
    with pytest.raises(RuntimeError):
        load_policy_state(pol, bad)
    missing = dict(sd)
    missing.pop("action_net.bias")
    with pytest.raises(RuntimeError):
        load_policy_state(pol, missing)


def test_gridagent_is_a_gym_env_class():
    from voxnav.gym_api import GridAgent
    from voxnav.spaces import EnvBase
    assert issubclass(GridAgent, EnvBase)
