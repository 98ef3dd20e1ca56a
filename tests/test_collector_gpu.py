"""Parity of the on-device rollout collector (voxnav.collector) on the GPU.

Env outputs (obs bytes, terminated/truncated, f32 rewards before the
bootstrap) are bit-exact against the C oracle replaying the collector's
actions; the float policy quantities are compared with the float64 oracle
(oracle/collector_oracle.py) within stated tolerances:

  values, log-probs, LSTM states       |gpu - f64| <= 1e-4 + 1e-4 |f64|
  bootstrapped rewards                  |gpu - f64| <= 1e-4 + 1e-5 |f64|
  advantages / returns (f64 GAE)        |gpu - f64| <= 2e-3 + 1e-4 |f64|
  sampled actions                       equal, or u within 1e-5 of a cdf
                                        boundary (f32 vs f64 rounding)
With policy_dtype="bf16" (bf16 GEMM operands, f32 accumulation and cell
state) the float bounds are 6e-2 + 6e-2|f64| (advantages 0.6 + 6e-2|f64|)
and up to 6 % of the draws may flip within 0.08 of a CDF boundary.  The
GAE kernel is bit-exact against the f32 oracle on the GPU's own
rewards/values.  The kernels alone are compared with the plain-PyTorch f32
policy (voxnav.policy.forward_torch) at 2e-5.
"""
import numpy as np
import pytest

from helpers import box_text

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

BOXES = [(8, 8, 4), (6, 6, 4), (7, 5, 5), (5, 5, 4)]     # 72 / 32 / 45 / 18 free cells


@pytest.fixture(scope="module")
def voxnav():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import voxnav
    voxnav.load_library()
    return voxnav


def _rooms():
    from voxnav.rooms import RoomSet, parse_room
    from oracle.oracle import parse_room_text
    texts = [(f"box{w}x{d}x{h}.txt", box_text(w, d, h)) for (w, d, h) in BOXES]
    prod = RoomSet([parse_room(t, n) for n, t in texts], use_room_draw=True, source="test-boxes")
    orc = [parse_room_text(t, n) for n, t in texts]
    return prod, orc


def _close(a, b, atol, rtol, what):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    bad = np.abs(a - b) > atol + rtol * np.abs(b)
    assert not bad.any(), f"{what}: {bad.sum()} of {bad.size} out of tolerance, max err {np.abs(a - b).max():.3g}"


def _policy(kind):
    from voxnav.policy import ActorCriticPolicy, RecurrentActorCriticPolicy
    torch.manual_seed(7)
    pol = RecurrentActorCriticPolicy() if kind == "lstm" else ActorCriticPolicy()
    # larger head weights than SB3's 0.01 init so the draws are not ~uniform
    with torch.no_grad():
        pol.action_net.weight.mul_(100.0)
        pol.action_net.bias.uniform_(-0.5, 0.5)
        pol.value_net.bias.fill_(0.3)
    return pol


def _set_rooms(name):
    from helpers import product_room_set, set_members
    from oracle.oracle import parse_room_text
    return product_room_set(f"set:{name}"), [parse_room_text(t, n) for n, t in set_members(name)]


# BASELINE C5: 524,288 agents as 8 shards of 65,536; the last shard (rank 7)
# has global ids 458,752.. and its seeds advance by 524,288 per episode
C5_SHARD = (7 * 65536, 8 * 65536)

COLLECT_CASES = [
    # (policy, T, rollouts, dtype, rooms, L, N, (agent_id_base, seed_stride) or None)
    # T=96 / 80 > 4 x 18 (the smallest box's free cells): the bootstrap stash
    # is flushed once inside the rollout (collector._flush_every = 72)
    ("lstm", 96, 2, "f32", "boxes", 4, 64, None), ("mlp", 80, 1, "f32", "boxes", 4, 64, None),
    ("lstm", 48, 2, "bf16", "boxes", 4, 64, None), ("mlp", 48, 1, "bf16", "boxes", 4, 64, None),
    # BASELINE configs at the reference's settings, a few hundred agents:
    # C4 = PPO-LSTM on P3_training (L=10, n_steps 128), C3 = PPO-MLP on P2_training
    ("lstm", 128, 2, "f32", "P3_training", 10, 192, None), ("mlp", 128, 3, "f32", "P2_training", 10, 256, None),
    # C4 through the bf16 policy path the bench also reports (its stated bounds)
    ("lstm", 128, 2, "bf16", "P3_training", 10, 192, None),
    # C5: the last shard's collector -- Philox draws keyed by global id, seeds
    # on the 524,288 stride (the bench's N>1 path)
    ("lstm", 128, 2, "f32", "P3_training", 10, 192, C5_SHARD),
]


def _case_id(c):
    return f"{c[0]}-{c[3]}-{c[4]}-T{c[1]}" + ("-C5shard" if c[7] else "")


@pytest.mark.parametrize("kind,T,rollouts,dtype,rooms,L,N,shard", COLLECT_CASES, ids=[_case_id(c) for c in COLLECT_CASES])
def test_collector_matches_oracle(voxnav, kind, T, rollouts, dtype, rooms, L, N, shard):
    from oracle import collector_oracle as co
    from oracle.oracle import OracleEnv, gae as gae32
    from voxnav.collector import RolloutCollector
    from voxnav.env import BatchedGridEnv
    from voxnav.policy import numpy_weights
    prod, orooms = _rooms() if rooms == "boxes" else _set_rooms(rooms)
    pol = _policy(kind)
    gid_base, stride = shard if shard else (0, N)
    env = BatchedGridEnv(num_agents=N, rooms=prod, local_map_length=L, device="cuda:0", agent_id_base=gid_base,
                         seed_stride=stride)
    col = RolloutCollector(env, pol.to("cuda:0"), n_steps=T, sample_seed=1234, reset_seed=42, policy_dtype=dtype)
    # f32: the reference's dtype, tight bounds; bf16 GEMM operands (8-bit
    # mantissa): looser bounds and some draws flip near a CDF boundary
    tol = dict(v=(1e-4, 1e-4), r=(1e-4, 1e-5), adv=(2e-3, 1e-4), flip=1e-5, nflip=2) if dtype == "f32" else \
        dict(v=(6e-2, 6e-2), r=(6e-2, 6e-2), adv=(0.6, 6e-2), flip=0.08, nflip=int(0.06 * T * N))
    orc = co.PolicyOracle(numpy_weights(pol))
    oenv = OracleEnv(orooms, n_agents=N, local_map_length=L)
    seeds = 42 + gid_base + np.arange(N)
    # reset observations
    ref = OracleEnv(orooms, n_agents=N, local_map_length=L)
    obs0 = np.stack([ref.reset(i, int(seeds[i])) for i in range(N)])
    assert col._obs[0].cpu().numpy().tobytes() == obs0.tobytes()
    starts0 = np.ones(N, np.float32)
    h = c = None
    total_boot = 0
    run_ret, run_len = np.zeros(N), np.zeros(N, np.int64)     # the Monitor's running sums (f64, step order)
    for r in range(rollouts):
        buf = col.collect()
        torch.cuda.synchronize()
        acts = buf.actions.cpu().numpy()
        rr = oenv.run_random(seeds, 0, T, t0=r * T, seed_stride=stride, initial_reset=(r == 0), actions=acts,
                             terminal_obs=True, gid_base=gid_base)
        gobs = buf.obs.cpu().numpy()
        assert gobs[1:].tobytes() == rr["obs"][:-1].tobytes(), "env obs"
        assert col._obs[T].cpu().numpy().tobytes() == rr["obs"][-1].tobytes()
        out = co.collect(orc, rr, gobs[0], starts0, acts, gamma=0.99, h0=h, c0=c, sample_seed=1234, t0=r * T,
                         gid_base=gid_base)
        h, c, starts0 = out["h"], out["c"], out["dones"]
        te, tr = rr["terminated"].astype(bool), rr["truncated"].astype(bool)
        total_boot += int((tr & ~te).sum())
        # Monitor episodes: the env step's exact f64 rewards (the FAST kernel
        # stores them with the f32 ones), summed in step order
        want = []
        for t in range(T):
            run_ret += rr["reward"][t]
            run_len += 1
            for a in np.nonzero(te[t] | tr[t])[0]:
                want.append((t, a, run_ret[a], run_len[a]))
                run_ret[a], run_len[a] = 0.0, 0
        got = col.monitor.last_episodes
        assert got["agent"].tolist() == [w[1] for w in want] and got["step"].tolist() == [w[0] for w in want]
        assert got["return"].cpu().numpy().tobytes() == np.array([w[2] for w in want], np.float64).tobytes()
        np.testing.assert_array_equal(buf.episode_starts.cpu().numpy(), out["episode_starts"])
        np.testing.assert_array_equal(buf.dones.cpu().numpy(), out["dones"])
        _close(buf.values.cpu(), out["values"], *tol["v"], "values")
        _close(buf.log_probs.cpu(), out["log_probs"], *tol["v"], "log_probs")
        _close(buf.rewards.cpu(), out["rewards"], *tol["r"], "rewards")
        _close(buf.last_values.cpu(), out["last_values"], *tol["v"], "last_values")
        # unbootstrapped rewards are the env's f32 rewards exactly
        plain = ~(tr & ~te)
        assert np.array_equal(buf.rewards.cpu().numpy()[plain], rr["reward"].astype(np.float32)[plain])
        mism = acts != out["oracle_actions"]
        assert np.all(out["margins"][mism] < tol["flip"]), f"{mism.sum()} action draws differ away from a cdf boundary"
        assert mism.sum() <= tol["nflip"]
        # GAE: bit-exact vs the f32 restatement on the GPU's own inputs; close to f64
        a32, r32 = gae32(buf.rewards.cpu().numpy(), buf.values.cpu().numpy(), buf.episode_starts.cpu().numpy(),
                         buf.last_values.cpu().numpy(), buf.dones.cpu().numpy())
        assert buf.advantages.cpu().numpy().tobytes() == a32.tobytes()
        assert buf.returns.cpu().numpy().tobytes() == r32.tobytes()
        a64, r64 = co.gae64(out["rewards"].astype(np.float64), out["values"], out["episode_starts"],
                            out["last_values"], out["dones"])
        _close(buf.advantages.cpu(), a64, *tol["adv"], "advantages")
        _close(buf.returns.cpu(), r64, *tol["adv"], "returns")
        if kind == "lstm":
            gh, gc = col.hidden_state()
            _close(gh.cpu(), h, *tol["v"], "h")
            _close(gc.cpu(), c, *tol["v"], "c")
            # stored states entering step t: zero at learn() start
            if r == 0:
                assert float(buf.lstm_h[0].abs().max()) == 0.0
    assert total_boot > 0, "the test rooms must produce truncations inside the rollout"


def test_kernels_match_torch_fp32(voxnav):
    """vn_lstm_cell + vn_policy_head (through the collector's forward) vs nn.LSTM/nn.Linear."""
    from voxnav.collector import RolloutCollector
    from voxnav.env import BatchedGridEnv
    N = 300
    prod, _ = _rooms()
    pol = _policy("lstm").to("cuda:0")
    env = BatchedGridEnv(num_agents=N, rooms=prod, local_map_length=4, device="cuda:0")
    col = RolloutCollector(env, pol, n_steps=4)
    g = torch.Generator(device="cuda:0").manual_seed(5)
    obs = torch.rand((N, 80), device="cuda:0", generator=g)
    h = torch.randn((2, N, 256), device="cuda:0", generator=g) * 0.5
    c = torch.randn((2, N, 256), device="cuda:0", generator=g) * 0.5
    col.h.copy_(h)
    col.c.copy_(c)
    col._forward(obs, 0)
    lg, v, h2, c2 = pol.forward_torch(obs, h, c)
    lsm = torch.log_softmax(lg, 1)
    a = col.actions[0].long()
    _close(col.values[0].cpu(), v.cpu(), 2e-5, 2e-5, "values")
    _close(col.log_probs[0].cpu(), lsm.gather(1, a[:, None])[:, 0].cpu(), 2e-5, 2e-5, "log_probs")
    _close(col.h.cpu(), h2.cpu(), 2e-5, 2e-5, "h")
    _close(col.c.cpu(), c2.cpu(), 2e-5, 2e-5, "c")
    # deterministic mode = argmax of the logits
    col.deterministic = True
    col.h.copy_(h)
    col.c.copy_(c)
    col._forward(obs, 1)
    assert torch.equal(col.actions[1].long(), lg.argmax(1))
    # the rollout entry (vn_lstm_cell_masked): a step from the buffer's
    # unmasked lstm_h / lstm_c[t] with episode_starts[t] is bitwise the step
    # from the masked state through vn_lstm_cell
    col.deterministic = False
    start = (torch.rand(N, device="cuda:0", generator=g) < 0.3).float()
    keep = (start == 0)[None, :, None]
    col._hs[1].copy_(h)
    col._cs[1].copy_(c)
    col._starts[1].copy_(start)
    col._forward(obs, 1, in_rollout=True)
    hm, cm = col._hs[2].clone(), col._cs[2].clone()
    assert torch.equal(col._hs[1], h) and torch.equal(col._cs[1], c)     # inputs not written
    col.h.copy_(torch.where(keep, h, 0.0))
    col.c.copy_(torch.where(keep, c, 0.0))
    col._forward(obs, 2)
    assert torch.equal(hm, col.h) and torch.equal(cm, col.c)


def test_compaction_and_episode_start(voxnav):
    import ctypes as C
    lib = voxnav.load_library()
    rng = np.random.default_rng(11)
    for N in (1, 63, 1000, 70001):
        te = torch.from_numpy((rng.random(N) < 0.05).astype(np.uint8)).cuda()
        tr = torch.from_numpy((rng.random(N) < 0.1).astype(np.uint8)).cuda()
        idx = torch.full((N,), -1, dtype=torch.int32, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
        p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
        assert lib.vn_collect_compact(p(te), p(tr), N, p(idx), p(cnt), None) == 0
        want = np.nonzero((tr.cpu().numpy() == 1) & (te.cpu().numpy() == 0))[0]
        M = int(cnt.item())
        assert M == len(want)
        assert np.array_equal(idx[:M].cpu().numpy(), want)
        H = 8
        h = torch.ones((2, N, H), device="cuda")
        c = torch.ones((2, N, H), device="cuda")
        st = torch.full((N,), 7.0, device="cuda")
        assert lib.vn_episode_start(p(te), p(tr), N, p(st), p(h), p(c), None, 2, H, None) == 0
        done = (te | tr).bool().cpu().numpy()
        assert np.array_equal(st.cpu().numpy(), done.astype(np.float32))
        assert float(h[:, done].abs().sum()) == 0.0 and bool((h[:, ~done] == 1).all())
        assert float(c[:, done].abs().sum()) == 0.0 and bool((c[:, ~done] == 1).all())
        # bootstrap add: two f32 roundings
        rew = torch.from_numpy(rng.standard_normal(N).astype(np.float32)).cuda()
        tv = torch.from_numpy(rng.standard_normal(max(M, 1)).astype(np.float32)).cuda()
        want_r = rew.cpu().numpy().copy()
        gv = (np.float32(0.99) * tv.cpu().numpy()[:M]).astype(np.float32)
        want_r[want] = (want_r[want] + gv).astype(np.float32)
        assert lib.vn_collect_bootstrap(p(idx), p(tv), M, C.c_double(0.99), p(rew), None) == 0
        assert rew.cpu().numpy().tobytes() == want_r.tobytes()


@pytest.mark.parametrize("N,hb", [(1, 4), (1000, 4), (70001, 4), (3000, 2)])
def test_collect_post_step(voxnav, N, hb):
    """vn_collect_post_step against its definition: episode starts, the
    Monitor step, the truncated agents' stash rows (as a set keyed by the flat
    reward index: rows are claimed atomically), and the zeroed state rows."""
    import ctypes as C
    lib = voxnav.load_library()
    rng = np.random.default_rng(N + hb)
    p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    dev = "cuda"
    t, od, H = 5, 80, 16
    te = torch.from_numpy((rng.random(N) < 0.05).astype(np.uint8)).to(dev)
    tr = torch.from_numpy((rng.random(N) < 0.1).astype(np.uint8)).to(dev)
    tobs = torch.from_numpy(rng.standard_normal((N, od)).astype(np.float32)).to(dev)
    hdt = torch.float32 if hb == 4 else torch.bfloat16
    hc = torch.from_numpy(rng.standard_normal((N, H)).astype(np.float32)).to(dev).to(hdt)
    cc = torch.from_numpy(rng.standard_normal((N, H)).astype(np.float32)).to(dev)
    r64 = torch.from_numpy(rng.standard_normal(N)).to(dev)
    ep_ret0 = torch.from_numpy(rng.standard_normal(N)).to(dev)
    ep_len0 = torch.from_numpy(rng.integers(0, 100, N).astype(np.int32)).to(dev)
    ep_ret, ep_len = ep_ret0.clone(), ep_len0.clone()
    rec_ret = torch.full((N,), 9.0, dtype=torch.float64, device=dev)
    rec_len = torch.full((N,), 9, dtype=torch.int32, device=dev)
    starts = torch.full((N,), 7.0, device=dev)
    cap = N
    st_obs = torch.zeros((cap, od), device=dev)
    st_h = torch.zeros((cap, H), dtype=hdt, device=dev)
    st_c = torch.zeros((cap, H), device=dev)
    st_flat = torch.full((cap,), -1, dtype=torch.int32, device=dev)
    cnt = torch.full((1,), 3, dtype=torch.int32, device=dev)     # a running count carried from earlier steps
    zh = torch.ones((2, N, H), device=dev)
    zc = torch.ones((2, N, H), device=dev)
    assert lib.vn_collect_post_step(p(te), p(tr), N, t, p(starts), p(r64), None, p(ep_ret), p(ep_len), p(rec_ret),
                                    p(rec_len), p(tobs), od, p(hc), hb, p(cc), H, p(st_obs), p(st_h), p(st_c),
                                    p(st_flat), cap, p(cnt), p(zh), p(zc), None, 2, None) == 0
    torch.cuda.synchronize()
    ten, trn = te.cpu().numpy().astype(bool), tr.cpu().numpy().astype(bool)
    done = ten | trn
    assert np.array_equal(starts.cpu().numpy(), done.astype(np.float32))
    r = ep_ret0.cpu().numpy() + r64.cpu().numpy()
    l = ep_len0.cpu().numpy() + 1
    assert np.array_equal(rec_ret.cpu().numpy(), np.where(done, r, 0.0))
    assert np.array_equal(rec_len.cpu().numpy(), np.where(done, l, 0))
    assert np.array_equal(ep_ret.cpu().numpy(), np.where(done, 0.0, r))
    assert np.array_equal(ep_len.cpu().numpy(), np.where(done, 0, l))
    want = np.nonzero(trn & ~ten)[0]
    M = int(cnt.item()) - 3
    assert M == len(want)
    flat = st_flat[3:3 + M].cpu().numpy()
    assert sorted(flat.tolist()) == sorted((t * N + want).tolist())
    agents = flat - t * N
    assert np.array_equal(st_obs[3:3 + M].cpu().numpy(), tobs.cpu().numpy()[agents])
    assert torch.equal(st_h[3:3 + M].cpu(), hc.cpu()[agents])
    assert np.array_equal(st_c[3:3 + M].cpu().numpy(), cc.cpu().numpy()[agents])
    assert float(zh[:, done].abs().sum()) == 0.0 and bool((zh[:, ~done] == 1).all())
    assert float(zc[:, done].abs().sum()) == 0.0 and bool((zc[:, ~done] == 1).all())


def test_fused_mfma_lstm_exact_mapping(voxnav):
    """vn_lstm_fused_bf16 against a float64 restatement on data that bf16
    holds exactly (multiples of 1/8), so the gate sums are exact in f32 and
    any row/column/gate mix-up in the MFMA operand or accumulator maps shows."""
    import ctypes as C
    lib = voxnav.load_library()
    rng = np.random.default_rng(21)
    B, N, H, od = 2, 200, 128, 80          # N not a multiple of 64: tail rows
    kx = (od + 7) // 8 * 8
    Kp = (kx + H + 63) // 64 * 64
    x = (rng.integers(-4, 5, size=(N, od)) / 8.0).astype(np.float32)
    h_in = (rng.integers(-4, 5, size=(B, N, H)) / 8.0).astype(np.float32)
    W = (rng.integers(-3, 4, size=(B, 4 * H, od + H)) / 8.0).astype(np.float32)
    bias = (rng.integers(-8, 9, size=(B, 4 * H)) / 8.0).astype(np.float32)
    c0 = rng.standard_normal((B, N, H)).astype(np.float32)
    wc = np.zeros((B, 4 * H, Kp), np.float32)
    wc[:, :, :od] = W[:, :, :od]
    wc[:, :, kx:kx + H] = W[:, :, od:]
    dev = "cuda:0"
    t = lambda a, dt=torch.float32: torch.as_tensor(a, dtype=dt, device=dev).contiguous()  # noqa: E731
    tx, th, tw, tb, tc = t(x), t(h_in, torch.bfloat16), t(wc, torch.bfloat16), t(bias), t(c0)
    hout = torch.zeros((B, N, H), dtype=torch.bfloat16, device=dev)
    hst = torch.zeros((B, N, H), device=dev)
    cst = torch.zeros((B, N, H), device=dev)
    p = lambda a: C.c_void_p(a.data_ptr())  # noqa: E731
    assert lib.vn_lstm_fused_bf16(p(tx), od, p(th), p(tw), Kp, p(tb), p(tc), p(hout), None, p(hst), p(cst), B, N, H,
                                  None) == 0
    torch.cuda.synchronize()
    xh = np.concatenate([np.broadcast_to(x, (B, N, od)), h_in], -1).astype(np.float64)
    pre = np.einsum("bnk,bgk->bng", xh, W.astype(np.float64)) + bias[:, None, :]
    sg = lambda v: 1.0 / (1.0 + np.exp(-v))  # noqa: E731
    i, f, g, o = (pre[..., k * H:(k + 1) * H] for k in range(4))
    c1 = sg(f) * c0 + sg(i) * np.tanh(g)
    h1 = sg(o) * np.tanh(c1)
    np.testing.assert_allclose(tc.cpu().numpy(), c1, atol=2e-6, rtol=2e-6)
    np.testing.assert_allclose(hst.cpu().numpy(), h1, atol=2e-6, rtol=2e-6)
    np.testing.assert_array_equal(cst.cpu().numpy(), tc.cpu().numpy())
    np.testing.assert_allclose(hout.float().cpu().numpy(), h1, atol=4e-3, rtol=4e-3)   # bf16 rounding of h
    # the same sizes through the unfused bf16 path (library GEMMs + vn_lstm_cell_bf16) agree
    gx = (t(x, torch.bfloat16) @ t(W[:, :, :od].reshape(B * 4 * H, od), torch.bfloat16).t())
    gh = torch.stack([th[b] @ t(W[b, :, od:], torch.bfloat16).t() for b in range(B)])
    h2 = torch.zeros((B, N, H), device=dev)
    c2 = t(c0)
    assert lib.vn_lstm_cell_bf16(p(gx), 8 * H, p(gh), p(tb), p(torch.zeros_like(tb)), p(h2), p(c2), None, None, None,
                                 B, N, H, None) == 0
    np.testing.assert_allclose(c2.cpu().numpy(), c1, atol=3e-2, rtol=3e-2)
    # the rollout entry (vn_lstm_fused_bf16_masked): c read from c_in with the
    # episode-start mask applied on read, written only to c_out -- bitwise the
    # same step as vn_lstm_fused_bf16 on the masked state
    start = (rng.random(N) < 0.3).astype(np.float32)
    ts = t(start)
    cm = t(np.where(start[None, :, None] != 0, 0.0, c0).astype(np.float32))
    h_a = torch.zeros((B, N, H), dtype=torch.bfloat16, device=dev)
    hs_a = torch.zeros((B, N, H), device=dev)
    assert lib.vn_lstm_fused_bf16(p(tx), od, p(th), p(tw), Kp, p(tb), p(cm), p(h_a), None, p(hs_a), None, B, N, H,
                                  None) == 0
    c_in = t(c0)
    c_out = torch.full((B, N, H), float("nan"), device=dev)
    h_b = torch.zeros((B, N, H), dtype=torch.bfloat16, device=dev)
    hs_b = torch.zeros((B, N, H), device=dev)
    assert lib.vn_lstm_fused_bf16_masked(p(tx), od, p(th), p(tw), Kp, p(tb), p(c_in), p(ts), p(c_out), p(h_b),
                                         p(hs_b), B, N, H, None) == 0
    torch.cuda.synchronize()
    assert torch.equal(c_out, cm) and torch.equal(h_b, h_a) and torch.equal(hs_b, hs_a)
    assert torch.equal(c_in, t(c0))                      # the input state is not written
    assert lib.vn_lstm_fused_bf16_masked(p(tx), od, p(th), p(tw), Kp, p(tb), p(c_in), None, p(c_in), p(h_b),
                                         None, B, N, H, None) != 0     # c_in == c_out refused


def test_fused_bf16_truncation_bootstrap_uses_post_step_state(voxnav):
    """The fused bf16 collector's truncation bootstrap: rewards[t, a] - r_env
    == gamma * V(terminal obs; critic state after step t), recomputed here
    from the rollout buffer's stored states lstm_h / lstm_c[t+1] through the
    same kernels.  (The fused step's h is a ping-pong pair, so the stash must
    read the buffer the step just wrote, at every t.)"""
    from oracle.oracle import OracleEnv
    from voxnav.collector import RolloutCollector
    from voxnav.env import BatchedGridEnv
    prod, orooms = _rooms()
    N, T, L = 64, 48, 4
    env = BatchedGridEnv(num_agents=N, rooms=prod, local_map_length=L, device="cuda:0")
    col = RolloutCollector(env, _policy("lstm").to("cuda:0"), n_steps=T, sample_seed=1234, reset_seed=42,
                           policy_dtype="bf16")
    assert col.fused and col.store
    oenv = OracleEnv(orooms, n_agents=N, local_map_length=L)
    seeds = 42 + np.arange(N)
    n_boot, parity = 0, set()
    for r in range(2):
        buf = col.collect()
        torch.cuda.synchronize()
        acts = buf.actions.cpu().numpy()
        rr = oenv.run_random(seeds, 0, T, t0=r * T, seed_stride=N, initial_reset=(r == 0), actions=acts,
                             terminal_obs=True)
        te, tr = rr["terminated"].astype(bool), rr["truncated"].astype(bool)
        ts, ag = np.nonzero(tr & ~te)
        it, ia = torch.as_tensor(ts + 1, device="cuda:0"), torch.as_tensor(ag, device="cuda:0")
        h = col._hs[it, 1, ia].to(torch.bfloat16)
        c = col._cs[it, 1, ia].clone()
        tobs = torch.as_tensor(rr["terminal_obs"][ts, ag], device="cuda:0")
        v = torch.empty(len(ts), device="cuda:0")
        col._critic(tobs, h, c, v)
        got = buf.rewards.cpu().numpy()[ts, ag].astype(np.float64) - rr["reward"].astype(np.float32)[ts, ag]
        np.testing.assert_allclose(got, 0.99 * v.cpu().numpy().astype(np.float64), atol=2e-5, rtol=1e-5)
        n_boot += len(ts)
        parity |= set((ts % 2).tolist())
    assert n_boot > 0 and parity == {0, 1}, "truncations at both even and odd steps"


@pytest.mark.parametrize("N,od,masked,inplace", [(300, 80, False, False), (257, 80, True, False),
                                                 (130, 31, True, False), (128, 80, False, True)])
def test_fused_f32_lstm_exact_mapping(voxnav, N, od, masked, inplace):
    """vn_lstm_fused_f32 (v_mfma_f32_32x32x2_f32) against a float64
    restatement on small-integer / 8 data, so the f32 gate sums are exact and
    any row / unit / gate / k mix-up in the operand, packing or accumulator
    maps shows; row tails (N % 128), obs_dim % 4 != 0 (scalar x loads), the
    episode-start mask (h rows and c of starting agents read as zero) and the
    in-place state (c_in == c_out)."""
    import ctypes as C
    from voxnav.collector import pack_lstm_f32
    lib = voxnav.load_library()
    rng = np.random.default_rng(23 + N)
    B, H = 2, 128
    x = (rng.integers(-4, 5, size=(N, od)) / 8.0).astype(np.float32)
    h_in = (rng.integers(-4, 5, size=(B, N, H)) / 8.0).astype(np.float32)
    w_ih = (rng.integers(-3, 4, size=(B, 4 * H, od)) / 8.0).astype(np.float32)
    w_hh = (rng.integers(-3, 4, size=(B, 4 * H, H)) / 8.0).astype(np.float32)
    bias = (rng.integers(-8, 9, size=(B, 4 * H)) / 8.0).astype(np.float32)
    c0 = rng.standard_normal((B, N, H)).astype(np.float32)
    start = (rng.random(N) < 0.3).astype(np.float32)
    dev = "cuda:0"
    t = lambda a: torch.as_tensor(a, device=dev).contiguous()  # noqa: E731
    wp = pack_lstm_f32([t(w_ih[b]) for b in range(B)], [t(w_hh[b]) for b in range(B)])
    Kp = (od + 15) // 16 * 16 + H
    tc_in = t(c0)
    tc_out = tc_in if inplace else torch.full((B, N, H), float("nan"), device=dev)
    th_out = torch.full((B, N, H), float("nan"), device=dev)
    p = lambda a: None if a is None else C.c_void_p(a.data_ptr())  # noqa: E731
    tx, th = t(x), t(h_in)
    assert lib.vn_lstm_fused_f32(p(tx), od, p(th), p(wp), Kp, p(t(bias)), p(tc_in), p(t(start)) if masked else None,
                                 p(tc_out), p(th_out), B, N, H, None) == 0
    torch.cuda.synchronize()
    keep = (start == 0)[None, :, None] if masked else np.ones((1, N, 1), bool)
    hm = np.where(keep, h_in, 0.0)
    cm = np.where(keep, c0, 0.0)
    pre = (np.einsum("nk,bgk->bng", x.astype(np.float64), w_ih.astype(np.float64))
           + np.einsum("bnk,bgk->bng", hm.astype(np.float64), w_hh.astype(np.float64)) + bias[:, None, :])
    sg = lambda v: 1.0 / (1.0 + np.exp(-v))  # noqa: E731
    i, f, g, o = (pre[..., k * H:(k + 1) * H] for k in range(4))
    c1 = sg(f) * cm + sg(i) * np.tanh(g)
    h1 = sg(o) * np.tanh(c1)
    np.testing.assert_allclose(tc_out.cpu().numpy(), c1, atol=2e-6, rtol=2e-6)
    np.testing.assert_allclose(th_out.cpu().numpy(), h1, atol=2e-6, rtol=2e-6)
    if not inplace:
        assert torch.equal(tc_in, t(c0)) and torch.equal(th, t(h_in))     # inputs not written
    assert lib.vn_lstm_fused_f32(p(tx), od, p(th), p(wp), Kp, p(t(bias)), p(tc_in), None, p(tc_out), p(th), B, N, H,
                                 None) != 0                                  # h_in == h_out refused


@pytest.mark.parametrize("M,K,nout,nb", [(65, 256, 256, 2), (300, 80, 128, 1), (1024, 256, 384, 2)])
def test_linear_f32_exact_mapping(voxnav, M, K, nout, nb):
    """vn_linear_f32 (bias + Tanh epilogue, one or two branches per launch)
    against float64 on exact data; the identity-activation form is bitwise
    the exact sum."""
    import ctypes as C
    from voxnav.collector import pack_linear_f32
    lib = voxnav.load_library()
    rng = np.random.default_rng(M + K)
    dev = "cuda:0"
    xs = [(rng.integers(-4, 5, size=(M, K)) / 8.0).astype(np.float32) for _ in range(nb)]
    ws = [(rng.integers(-3, 4, size=(nout, K)) / 16.0).astype(np.float32) for _ in range(nb)]
    bs = [(rng.integers(-8, 9, size=nout) / 8.0).astype(np.float32) for _ in range(nb)]
    tx = [torch.as_tensor(a, device=dev) for a in xs]
    tw = [pack_linear_f32(torch.as_tensor(w, device=dev)) for w in ws]
    tb = [torch.as_tensor(b, device=dev) for b in bs]
    arr = lambda ts: (C.c_void_p * 2)(*[t.data_ptr() for t in ts])  # noqa: E731
    for act in (1, 0):
        ty = [torch.full((M, nout), float("nan"), device=dev) for _ in range(nb)]
        assert lib.vn_linear_f32(nb, arr(tx), K, arr(tw), arr(tb), arr(ty), M, K, nout, act, None) == 0
        torch.cuda.synchronize()
        for i in range(nb):
            ref = xs[i].astype(np.float64) @ ws[i].astype(np.float64).T + bs[i]
            got = ty[i].cpu().numpy()
            if act:
                np.testing.assert_allclose(got, np.tanh(ref), atol=1e-6, rtol=1e-5)   # hardware exp / rcp
            else:
                np.testing.assert_array_equal(got, ref.astype(np.float32))


# ---------------------------------------------------------------- bench shapes
# The collector bench (C4: 65,536 agents, H = 256) runs the persistent fused
# LSTM kernel with n_items = ceil(N / 128) x 2 LSTMs x H / 64 far above its
# 2-blocks-per-CU slots, so every block walks several items and the K-chunk
# stream runs on across them; these cases take that branch (and an N % 128
# tail) on exact data, with the float64 restatement computed on the device.
def _f64_lstm_ref(x, h_in, c0, w_ih, w_hh, bias, start):
    keep = (start == 0).view(1, -1, 1) if start is not None else None
    hm = h_in if keep is None else torch.where(keep, h_in, 0.0)
    cm = c0 if keep is None else torch.where(keep, c0, 0.0)
    d = torch.float64
    pre = (torch.einsum("nk,bgk->bng", x.to(d), w_ih.to(d)) + torch.einsum("bnk,bgk->bng", hm.to(d), w_hh.to(d))
           + bias.to(d)[:, None, :])
    i, f, g, o = pre.chunk(4, dim=-1)
    c1 = torch.sigmoid(f) * cm.to(d) + torch.sigmoid(i) * torch.tanh(g)
    return torch.sigmoid(o) * torch.tanh(c1), c1


@pytest.mark.parametrize("N,masked", [(65536 + 77, True), (65536, False)])
def test_fused_f32_lstm_bench_shape(voxnav, N, masked):
    """vn_lstm_fused_f32 at the collector bench's shape (H = 256, both LSTMs,
    65,536 agents and a ragged 65,613) -- the multi-item persistent path --
    against float64 on exact small-integer / 8 data: every row of h and c
    within 2e-6 (the gate sums are exact; only the hardware exp / rcp of the
    nonlinearities round)."""
    import ctypes as C
    from voxnav.collector import pack_lstm_f32
    lib = voxnav.load_library()
    dev = "cuda:0"
    B, H, od = 2, 256, 80
    g = torch.Generator(device=dev).manual_seed(N)
    ri = lambda lo, hi, shape, den: (torch.randint(lo, hi + 1, shape, generator=g, device=dev) / den).float()  # noqa: E731
    x = ri(-4, 4, (N, od), 8.0)
    h_in = ri(-4, 4, (B, N, H), 8.0)
    w_ih = ri(-3, 3, (B, 4 * H, od), 8.0)
    w_hh = ri(-3, 3, (B, 4 * H, H), 8.0)
    bias = ri(-8, 8, (B, 4 * H), 8.0)
    c0 = torch.randn((B, N, H), generator=g, device=dev)
    start = (torch.rand(N, generator=g, device=dev) < 0.3).float() if masked else None
    wp = pack_lstm_f32([w_ih[b].contiguous() for b in range(B)], [w_hh[b].contiguous() for b in range(B)])
    Kp = (od + 15) // 16 * 16 + H
    c_out = torch.full((B, N, H), float("nan"), device=dev)
    h_out = torch.full((B, N, H), float("nan"), device=dev)
    p = lambda a: None if a is None else C.c_void_p(a.data_ptr())  # noqa: E731
    assert lib.vn_lstm_fused_f32(p(x), od, p(h_in), p(wp), Kp, p(bias), p(c0), p(start), p(c_out), p(h_out), B, N, H,
                                 None) == 0
    torch.cuda.synchronize()
    h1, c1 = _f64_lstm_ref(x, h_in, c0, w_ih, w_hh, bias, start)
    for got, ref, what in ((c_out, c1, "c"), (h_out, h1, "h")):
        err = (got.double() - ref).abs() - 2e-6 * ref.abs()
        bad = err > 2e-6
        assert not bool(bad.any()), f"{what}: {int(bad.sum())} of {bad.numel()} out of tolerance, " \
                                    f"rows {torch.nonzero(bad.any(-1).any(0)).flatten()[:8].tolist()}"


@pytest.mark.parametrize("M,K,nout", [(65536 + 33, 256, 256), (65536 + 33, 256, 128), (65536, 80, 256)])
def test_linear_f32_bench_shape(voxnav, M, K, nout):
    """vn_linear_f32 at the collector bench's row count (65,536 agents and a
    ragged 65,569; the MLP layers 80->256, 256->256, 256->128 of both
    branches in one launch) against float64 on exact data: the identity form
    bitwise, the Tanh form within 1e-6 + 1e-5 |y|."""
    import ctypes as C
    from voxnav.collector import pack_linear_f32
    lib = voxnav.load_library()
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(M + K + nout)
    ri = lambda lo, hi, shape, den: (torch.randint(lo, hi + 1, shape, generator=g, device=dev) / den).float()  # noqa: E731
    xs = [ri(-4, 4, (M, K), 8.0) for _ in range(2)]
    ws = [ri(-3, 3, (nout, K), 16.0) for _ in range(2)]
    bs = [ri(-8, 8, (nout,), 8.0) for _ in range(2)]
    tw = [pack_linear_f32(w) for w in ws]
    arr = lambda ts: (C.c_void_p * 2)(*[t.data_ptr() for t in ts])  # noqa: E731
    for act in (1, 0):
        ty = [torch.full((M, nout), float("nan"), device=dev) for _ in range(2)]
        assert lib.vn_linear_f32(2, arr(xs), K, arr(tw), arr(bs), arr(ty), M, K, nout, act, None) == 0
        torch.cuda.synchronize()
        for i in range(2):
            ref = xs[i].double() @ ws[i].double().T + bs[i].double()
            if act:
                ref = torch.tanh(ref)
                bad = (ty[i].double() - ref).abs() > 1e-6 + 1e-5 * ref.abs()
                assert not bool(bad.any()), f"branch {i}: {int(bad.sum())} out of tolerance"
            else:
                assert torch.equal(ty[i], ref.float()), f"branch {i}: identity form not exact"


def _philox_u(seed, gids, t):
    """The sampler's uniform (collector_oracle.sample_uniform) for many agents at once (numpy)."""
    m = np.uint64(0xFFFFFFFF)
    gids = np.asarray(gids, np.uint64)
    hi = (int(t) | (1 << 63)) & ((1 << 64) - 1)
    c0, c1 = gids & m, gids >> np.uint64(32)
    c2 = np.full_like(gids, hi & 0xFFFFFFFF)
    c3 = np.full_like(gids, hi >> 32)
    k0, k1 = np.uint64(seed & 0xFFFFFFFF), np.uint64((seed >> 32) & 0xFFFFFFFF)
    for r in range(10):
        if r:
            k0 = (k0 + np.uint64(0x9E3779B9)) & m
            k1 = (k1 + np.uint64(0xBB67AE85)) & m
        p0 = np.uint64(0xD2511F53) * c0
        p1 = np.uint64(0xCD9E8D57) * c2
        c0, c1, c2, c3 = (p1 >> np.uint64(32)) ^ c1 ^ k0, p1 & m, (p0 >> np.uint64(32)) ^ c3 ^ k1, p0 & m
    return (c0 >> np.uint64(8)).astype(np.float64) / 16777216.0


def _mlp_head_ref(xs, layers, wa, ba, wv, bv):
    """float64 restatement of the pi / vf MLPs (Linear + Tanh) and the heads."""
    d = torch.float64
    hs = []
    for x, ls in zip(xs, layers):
        h = x.to(d)
        for w, b in ls:
            h = torch.tanh(h @ w.to(d).T + b.to(d))
        hs.append(h)
    logits = hs[0] @ wa.to(d).T + ba.to(d) if wa is not None else None
    value = hs[-1] @ wv.to(d) + bv.to(d)
    return logits, value


@pytest.mark.parametrize("M,K0,widths,nb", [(65536 + 33, 256, (256, 256, 128), 2), (77, 80, (256, 256, 128), 2),
                                            (300, 80, (128, 256), 2), (1000, 256, (256, 256, 128), 1),
                                            (65536, 80, (256, 256, 128), 2)])
def test_mlp_head_f32_matches_float64(voxnav, M, K0, widths, nb):
    """vn_mlp_head_f32 (both MLP branches + heads in one launch, activations in
    LDS) against float64: values and log-probs within 2e-5 + 2e-5 |x| (the
    hardware exp / rcp of the Tanh), the Philox draw equal to the draw the
    float64 probabilities give except within 1e-5 of a CDF boundary, argmax in
    deterministic mode; value-only launches (n_branch 1); ragged M, the
    collector bench's 65,536 rows, K0 = 80 (PPO-MLP) and 256 (after the LSTM),
    a 128-wide first layer."""
    import ctypes as C
    lib = voxnav.load_library()
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(M + K0 + nb)
    rn = lambda *s, sc=1.0: (torch.randn(s, generator=g, device=dev) * sc).contiguous()  # noqa: E731
    xs = [rn(M, K0), rn(M, K0)][:nb] if nb == 2 else [rn(M, K0)]
    layers = []
    for _ in range(nb):
        ls, k = [], K0
        for n in widths:
            ls.append((rn(n, k, sc=1.0 / k ** 0.5), rn(n, sc=0.1)))
            k = n
        layers.append(ls)
    P, A = widths[-1], 6
    wa, ba = rn(A, P, sc=3.0 / P ** 0.5), rn(A, sc=0.5)
    wv, bv = rn(P, sc=1.0 / P ** 0.5), rn(1)
    from voxnav.collector import pack_mlp_head_f32
    wt = [pack_mlp_head_f32(w) for ls in layers for w, _ in ls]
    bs = [b for ls in layers for _, b in ls]
    arr = lambda ts: (C.c_void_p * len(ts))(*[t.data_ptr() for t in ts])  # noqa: E731
    p = lambda t: None if t is None else C.c_void_p(t.data_ptr())  # noqa: E731
    nl = len(widths)
    ref_lg, ref_v = _mlp_head_ref(xs, layers, wa if nb == 2 else None, ba, wv, bv)
    for det in (0, 1):
        acts = torch.full((M,), -1, dtype=torch.int32, device=dev)
        lps = torch.full((M,), float("nan"), device=dev)
        vals = torch.full((M,), float("nan"), device=dev)
        assert lib.vn_mlp_head_f32(nb, arr(xs), K0, K0, nl, (C.c_int32 * nl)(*widths), arr(wt), arr(bs),
                                   p(wa) if nb == 2 else None, p(ba) if nb == 2 else None, A if nb == 2 else 0, p(wv),
                                   p(bv), 1234, 77, 1000, det, p(acts) if nb == 2 else None,
                                   p(lps) if nb == 2 else None, p(vals), M, None) == 0
        torch.cuda.synchronize()
        bad = (vals.double() - ref_v).abs() > 2e-5 + 2e-5 * ref_v.abs()
        assert not bool(bad.any()), f"values: {int(bad.sum())} out of tolerance"
        if nb == 1:
            assert int((acts == -1).sum()) == M and bool(torch.isnan(lps).all())     # pi outputs untouched
            break
        lsm = torch.log_softmax(ref_lg, -1)
        if det:
            srt = ref_lg.sort(-1, descending=True).values
            clear = (srt[:, 0] - srt[:, 1]) > 1e-5
            assert torch.equal(acts.long()[clear], ref_lg.argmax(-1)[clear])
        else:
            # the draw the float64 probabilities give for the same uniform
            from oracle.collector_oracle import sample_uniform
            un = _philox_u(1234, 1000 + np.arange(M, dtype=np.uint64), 77)
            assert all(un[i] == sample_uniform(1234, 1000 + i, 77) for i in (0, 1, M - 1))
            u = torch.as_tensor(un, dtype=torch.float64, device=dev)
            cdf = lsm.exp().cumsum(-1)
            want = (u[:, None] < cdf[:, :A - 1]).to(torch.int64)
            want = torch.where(want.any(-1), want.argmax(-1), torch.full_like(want[:, 0], A - 1))
            margin = (cdf[:, :A - 1] - u[:, None]).abs().min(-1).values
            diff = acts.long() != want
            assert bool((margin[diff] < 1e-5).all()), f"{int(diff.sum())} draws differ away from a cdf boundary"
        lp_ref = lsm.gather(1, acts.long()[:, None])[:, 0]
        bad = (lps.double() - lp_ref).abs() > 2e-5 + 2e-5 * lp_ref.abs()
        assert not bool(bad.any()), f"log_probs: {int(bad.sum())} out of tolerance"
