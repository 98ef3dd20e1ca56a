"""PPO learner (voxnav.ppo) against the float64
restatement of sb3_contrib RecurrentPPO.train / SB3 PPO.train in
oracle/ppo_oracle.py (parity unpinned by the reference: SB3 is absent).

Tolerances: parameters after a train() call within 2e-5 absolute + 1e-4
relative of the f64 oracle (the learner runs in f32; a few Adam steps of
lr 3e-4 move parameters by ~1e-3); logged losses within 1e-4 relative.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import ppo_oracle as po  # noqa: E402


# ------------------------------------------------------------------ sequencers
def test_create_sequencers_known_answer():
    # 2 envs x 4 steps, env-major flat order: env0 t0..3, env1 t0..3
    starts = np.array([0, 0, 1, 0, 0, 1, 0, 0], float)
    env_change = np.array([1, 0, 0, 0, 1, 0, 0, 0], float)
    st, en = po.create_sequencers(starts, env_change)
    assert st.tolist() == [0, 2, 4, 5]
    assert en.tolist() == [1, 3, 4, 8]
    padded = po.pad(st, en, np.arange(8, dtype=float))
    assert padded.tolist() == [[0, 1, 0], [2, 3, 0], [4, 0, 0], [5, 6, 7]]
    # a minibatch cut mid-sequence starts a sequence at its first row
    st2, _ = po.create_sequencers(starts[3:], env_change[3:])
    assert st2.tolist() == [0, 1, 2]


def test_swap_and_flatten_is_env_major():
    a = np.arange(12).reshape(3, 4)          # [T=3, N=4]
    assert po.swap_and_flatten(a).reshape(-1).tolist() == [0, 4, 8, 1, 5, 9, 2, 6, 10, 3, 7, 11]


# ------------------------------------------------------------------ learner
def _policy(recurrent, seed=0, full=False):
    from voxnav.policy import ActorCriticPolicy, RecurrentActorCriticPolicy
    torch.manual_seed(seed)
    if full:   # the reference's policy: LSTM 256 (actor + critic), pi/vf [256, 256, 128] (Grid_Train.py:68-80)
        return RecurrentActorCriticPolicy() if recurrent else ActorCriticPolicy()
    arch = dict(pi=[32, 16], vf=[32, 16])
    if recurrent:
        return RecurrentActorCriticPolicy(obs_dim=80, lstm_hidden_size=16, net_arch=arch)
    return ActorCriticPolicy(obs_dim=80, net_arch=arch)


def _buffer(T, N, H, recurrent, seed=1, p_start=0.15):
    rng = np.random.default_rng(seed)
    b = dict(
        obs=rng.random((T, N, 80), dtype=np.float32),
        actions=rng.integers(0, 6, (T, N)).astype(np.int32),
        episode_starts=(rng.random((T, N)) < p_start).astype(np.float32),
        values=rng.normal(0, 1, (T, N)).astype(np.float32),
        log_probs=(np.log(1 / 6) + rng.normal(0, 0.15, (T, N))).astype(np.float32),
        advantages=rng.normal(0, 2, (T, N)).astype(np.float32),
        returns=rng.normal(0, 2, (T, N)).astype(np.float32),
    )
    b["episode_starts"][0, :2] = 1.0
    if recurrent:
        b["lstm_h"] = rng.normal(0, 0.3, (T, 2, N, H)).astype(np.float32)
        b["lstm_c"] = rng.normal(0, 0.3, (T, 2, N, H)).astype(np.float32)
    return b


def _as_rollout(b, device):
    from voxnav.collector import RolloutBuffer
    t = {k: torch.as_tensor(v, device=device) for k, v in b.items()}
    return RolloutBuffer(obs=t["obs"], actions=t["actions"], rewards=torch.zeros_like(t["values"]),
                         episode_starts=t["episode_starts"], values=t["values"], log_probs=t["log_probs"],
                         advantages=t["advantages"], returns=t["returns"], lstm_h=t.get("lstm_h"),
                         lstm_c=t.get("lstm_c"))


def _run_parity(device, recurrent, T=12, N=5, batch_size=16, epochs=2, full=False, p_start=0.15, atol=2e-5,
                rtol=1e-4, want_rows=None):
    from voxnav.policy import numpy_weights
    from voxnav.ppo import PPOLearner
    pol = _policy(recurrent, full=full).to(device)
    w0 = numpy_weights(pol)
    H = 256 if full else 16
    b = _buffer(T, N, H, recurrent, p_start=p_start)
    rng = np.random.default_rng(7)
    orders = ([int(rng.integers(T * N)) for _ in range(epochs)] if recurrent
              else [rng.permutation(T * N) for _ in range(epochs)])
    ln = PPOLearner(pol, n_epochs=epochs, batch_size=batch_size)
    st = ln.train(_as_rollout(b, device), epoch_orders=orders)
    if want_rows is not None:      # which LSTM re-run the minibatches took
        assert any(ln.__dict__.get("_rows_cache", {}).values()) == want_rows
    w1, ost, _ = po.train(w0, b, orders, batch_size=batch_size)
    got = numpy_weights(pol)
    moved = 0.0
    for k in w1:
        np.testing.assert_allclose(got[k], w1[k], atol=atol, rtol=rtol, err_msg=k)
        moved = max(moved, float(np.abs(w1[k] - w0[k]).max()))
    assert moved > 1e-4                                 # the update did something
    n = len(ost)
    assert st["n_minibatches"] == n == epochs * -(-T * N // batch_size)
    for key, okey in (("policy_gradient_loss", "policy_loss"), ("value_loss", "value_loss"),
                      ("entropy_loss", "entropy_loss"), ("approx_kl", "approx_kl"),
                      ("clip_fraction", "clip_fraction")):
        ref = np.mean([s[okey] for s in ost])
        assert abs(st[key] - ref) <= 1e-4 * max(1.0, abs(ref)), (key, st[key], ref)
    if recurrent:
        assert sum(s["n_seq"] for s in ost) > n        # sequences were actually split
    return ost


@pytest.mark.parametrize("recurrent", [True, False], ids=["lstm", "mlp"])
def test_learner_matches_oracle_cpu(recurrent):
    _run_parity("cpu", recurrent)


@pytest.mark.gpu
@pytest.mark.parametrize("recurrent", [True, False], ids=["lstm", "mlp"])
def test_learner_matches_oracle_gpu(recurrent):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run_parity("cuda:0", recurrent)


@pytest.mark.gpu
@pytest.mark.parametrize("recurrent", [True, False], ids=["lstm", "mlp"])
def test_learner_full_size_matches_oracle_gpu(recurrent):
    """The reference's policy size (LSTM 256 actor + critic, pi/vf
    [256, 256, 128]) on 128-step sequences (T=128, rare episode starts so
    most sequences run the whole rollout; BASELINE configs C3/C4), two
    epochs of 512-sample minibatches, against the f64 restatement.
    Tolerance 5e-5 + 1e-3 relative: Adam normalises each update by the
    gradient's running RMS, so parameters whose gradient is near zero move
    by up to ~lr x (f32 gradient noise / |g|) -- larger than the small-policy
    case's 2e-5 because the f32 sums run over 128 steps x 256 units."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ost = _run_parity("cuda:0", recurrent, T=128, N=8, batch_size=512, epochs=2, full=True, p_start=0.004,
                      atol=5e-5, rtol=1e-3)
    if recurrent:   # long sequences: on average >= 24 steps each (most run whole 128-step rollouts)
        assert 24 * sum(s["n_seq"] for s in ost) <= 2 * 128 * 8


@pytest.mark.gpu
@pytest.mark.parametrize("recurrent", [True, False], ids=["lstm", "mlp"])
def test_learner_bench_shape_minibatch_matches_oracle_gpu(recurrent):
    """One minibatch at the learner bench's own shape -- 65,536 samples = 512
    env rollouts x 128 steps (the row-layout LSTM with every one of its 256
    blocks resident; the MLP / loss / norm / Adam kernels at M = 65,536), the
    reference's policy -- against the f64 restatement: one train() call of
    one epoch, one Adam step.  Tolerance as the full-size test."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _run_parity("cuda:0", recurrent, T=128, N=512, batch_size=65536, epochs=1, full=True, p_start=0.004,
                atol=5e-5, rtol=1e-3, want_rows=True if recurrent else None)


@pytest.mark.gpu
def test_row_layout_error_word_skips_the_update():
    """A row-layout launch whose in-launch hand-off timed out (device error
    word set) must not update the parameters: the Adam step is gated on the
    word on the device, train() raises, and after the raise the learner
    trains normally with the step count re-read from the device."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from voxnav import _native, lstm_seq
    from voxnav.ppo import PPOLearner
    dev = "cuda:0"
    pol = _policy(True, full=True).to(dev)
    T, N = 16, 8
    b = _buffer(T, N, 256, True, p_start=0.05)
    ln = PPOLearner(pol, n_epochs=1, batch_size=T * N)
    buf = _as_rollout(b, dev)
    ln.train(buf, epoch_orders=[3])                      # a good step first: moments and step = 1
    assert any(ln._rows_cache.values()), "the row layout must be the path under test"
    w0 = [p.detach().clone() for p in pol.parameters()]
    m0 = [ln.optimizer.state[p]["exp_avg"].clone() for p in pol.parameters()]
    lstm_seq._rows_err(torch.device(dev)).fill_(1)       # as a timed-out hand-off leaves it
    with pytest.raises(_native.VoxnavError):
        ln.train(buf, epoch_orders=[5])
    for p, w, m in zip(pol.parameters(), w0, m0):
        assert torch.equal(p.detach(), w) and torch.equal(ln.optimizer.state[p]["exp_avg"], m)
    assert all(float(ln.optimizer.state[p]["step"]) == 1.0 for p in pol.parameters())
    ln.train(buf, epoch_orders=[5])                      # the word was cleared by the raise
    assert all(float(ln.optimizer.state[p]["step"]) == 2.0 for p in pol.parameters())
    assert any(not torch.equal(p.detach(), w) for p, w in zip(pol.parameters(), w0))


@pytest.mark.gpu
def test_optimizer_resume_keeps_fused_step(tmp_path):
    """A learner resumed from a checkpoint stays on the fused step: the
    loaded groups keep fused=True and the step counters are f32 device
    scalars, and the next update equals the one of the never-saved learner."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from voxnav.checkpoint import load_optimizer_state, save_checkpoint
    from voxnav.ppo import PPOLearner
    dev = "cuda:0"
    b = _buffer(12, 5, 16, True)
    pol = _policy(True).to(dev)
    ln = PPOLearner(pol, n_epochs=1, batch_size=16)
    ln.train(_as_rollout(b, dev), epoch_orders=[4])
    path = save_checkpoint(tmp_path / "r", pol, ln.optimizer)
    pol2 = _policy(True).to(dev)
    pol2.load_state_dict(pol.state_dict())
    ln2 = PPOLearner(pol2, n_epochs=1, batch_size=16)
    assert load_optimizer_state(path, ln2.optimizer)
    assert ln2.optimizer.param_groups[0]["fused"] is True
    for p in pol2.parameters():
        s = ln2.optimizer.state[p]["step"]
        assert s.device == p.device and s.dtype == torch.float32
    ln.train(_as_rollout(b, dev), epoch_orders=[7])
    ln2.train(_as_rollout(b, dev), epoch_orders=[7])
    for p, q in zip(pol.parameters(), pol2.parameters()):
        assert torch.equal(p, q)


@pytest.mark.gpu
def test_dual_lstm_bias_grads_are_distinct_tensors():
    """Regression for the round-1 learner flake: the dual-LSTM
    backward must give b_ih and b_hh separate gradient tensors, or autograd
    can keep one tensor as both leaves' .grad and in-place clipping scales it
    twice.  Asserts the cause directly: no shared storage after backward,
    and clip_grad_norm_ scales every gradient exactly once."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from voxnav.lstm_seq import dual_lstm
    from voxnav.policy import RecurrentActorCriticPolicy
    dev = torch.device("cuda:0")
    torch.manual_seed(3)
    pol = RecurrentActorCriticPolicy().to(dev)
    x = torch.randn(16, 64, 80, device=dev)
    h0 = 0.5 * torch.randn(2, 64, 256, device=dev)
    c0 = 0.5 * torch.randn(2, 64, 256, device=dev)
    a, c = dual_lstm(pol, x, h0, c0)
    (100.0 * (a.sum() + c.sum())).backward()
    for lstm in (pol.lstm_actor, pol.lstm_critic):
        gi, gh = lstm.bias_ih_l0.grad, lstm.bias_hh_l0.grad
        assert gi is not None and gh is not None
        assert gi.untyped_storage().data_ptr() != gh.untyped_storage().data_ptr()
        assert torch.equal(gi, gh)          # same values (d pre / d b), separate tensors
    params = [p for p in pol.parameters() if p.grad is not None]
    before = [p.grad.clone() for p in params]
    norm = torch.nn.utils.clip_grad_norm_(params, 0.5)
    coef = torch.clamp(0.5 / (norm + 1e-6), max=1.0)
    assert float(coef) < 1.0
    for p, g in zip(params, before):
        assert torch.equal(p.grad, g * coef)


def test_learner_batch_larger_than_buffer_and_defaults():
    from voxnav.ppo import PPOLearner
    pol = _policy(True)
    b = _buffer(6, 3, 16, True)
    ln = PPOLearner(pol, n_epochs=1, batch_size=1000, seed=3)
    st = ln.train(_as_rollout(b, "cpu"))
    assert st["n_minibatches"] == 1 and np.isfinite(st["loss"])
    with pytest.raises(ValueError):
        PPOLearner(pol, batch_size=0)


@pytest.mark.gpu
def test_learn_loop_end_to_end_gpu(tmp_path):
    """collect -> train -> sync_weights -> evaluate -> checkpoint on the GPU."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from helpers import product_room_set
    from voxnav.checkpoint import load_checkpoint, save_checkpoint
    from voxnav.collector import RolloutCollector
    from voxnav.env import BatchedGridEnv
    from voxnav.evaluate import evaluate_policy
    from voxnav.ppo import PPOLearner, learn
    pol = _policy(True).to("cuda:0")
    rooms = product_room_set("set:P2_training")
    env = BatchedGridEnv(num_agents=256, rooms=rooms, local_map_length=10, device="cuda:0")
    col = RolloutCollector(env, pol, n_steps=32)
    ln = PPOLearner(pol, n_epochs=2, batch_size=2048, seed=1)
    w0 = torch.cat([p.detach().reshape(-1).clone() for p in pol.parameters()])
    hist = learn(col, ln, total_timesteps=3 * 32 * 256)
    assert len(hist) == 3 and hist[-1]["num_timesteps"] == 3 * 32 * 256
    assert all(np.isfinite(h["loss"]) and h["n_minibatches"] == 8 for h in hist)
    w1 = torch.cat([p.detach().reshape(-1) for p in pol.parameters()])
    assert float((w1 - w0).abs().max()) > 1e-4
    # the collector acts with the updated weights
    assert torch.equal(col.w.pi[0][0], pol.mlp_extractor.policy_net[0].weight.detach())
    r = evaluate_policy(pol, rooms, n_episodes=8, local_map_length=10, seed=5, max_steps=300)
    assert len(r["episodes"]) == 8
    path = save_checkpoint(tmp_path / "m.zip", pol, ln.optimizer, num_timesteps=hist[-1]["num_timesteps"])
    pol2, data = load_checkpoint(path, device="cuda:0")
    assert data["num_timesteps"] == 3 * 32 * 256
    assert torch.equal(torch.cat([p.reshape(-1) for p in pol2.parameters()]), w1)
    env.close()


# ------------------------------------------------------------------ learner LSTM kernels
@pytest.mark.gpu
@pytest.mark.parametrize("L,B", [(1, 8), (7, 33), (128, 256)])
def test_dual_lstm_matches_nn_lstm_gpu(L, B):
    """voxnav.lstm_seq.dual_lstm (library GEMMs + csrc/voxnav_learn.hip cell
    kernels) against plain PyTorch fp32 nn.LSTM on the same device: outputs
    within 2e-5 absolute, parameter gradients within 1e-4 relative of their
    scale (f32 accumulation orders differ over L*B terms)."""
    from voxnav.lstm_seq import dual_lstm
    from voxnav.policy import RecurrentActorCriticPolicy
    dev = torch.device("cuda:0")
    torch.manual_seed(L * 1000 + B)
    pol = RecurrentActorCriticPolicy().to(dev)
    x = torch.randn(L, B, 80, device=dev)
    h0 = 0.5 * torch.randn(2, B, 256, device=dev)
    c0 = 0.5 * torch.randn(2, B, 256, device=dev)
    wpi = torch.randn(L, B, 256, device=dev)
    wvf = torch.randn(L, B, 256, device=dev)
    params = list(pol.lstm_actor.parameters()) + list(pol.lstm_critic.parameters())

    a, c = dual_lstm(pol, x, h0, c0)
    ga = torch.autograd.grad((a * wpi).sum() + (c * wvf).sum(), params)
    ra, _ = pol.lstm_actor(x, (h0[0:1].contiguous(), c0[0:1].contiguous()))
    rc, _ = pol.lstm_critic(x, (h0[1:2].contiguous(), c0[1:2].contiguous()))
    gr = torch.autograd.grad((ra * wpi).sum() + (rc * wvf).sum(), params)
    assert (a - ra).abs().max().item() < 2e-5
    assert (c - rc).abs().max().item() < 2e-5
    for g, r in zip(ga, gr):
        scale = r.abs().max().item() + 1e-6
        assert (g - r).abs().max().item() <= 1e-4 * scale, (g - r).abs().max().item() / scale
