"""Parity of the HIP env (through the C-ABI) with the golden vectors and the oracle.

Bar: bit-exact obs (f32 bytes), exact f64 reward, identical
terminated/truncated flags, integer agent state and belief map (visit counts
compared as min(count, 127), the device's saturating int8) -- on the
reference's golden trajectories, and against the CPU oracle for batched
random-policy rollouts with SB3 auto-reset, at sizes the oracle finishes in
seconds.  Size-independent properties cover the full BASELINE shape.
"""
import numpy as np
import pytest

from helpers import (GOLDEN, STATE13, golden_trajectories, grid_hash, load_golden, oracle_env,
                     product_room_set)

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

STATE_IDX = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12]


@pytest.fixture(scope="module")
def voxnav():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import voxnav
    voxnav.load_library()
    return voxnav


def make_env(voxnav, src, L, n=1, autoreset=False, **kw):
    from voxnav.env import BatchedGridEnv
    return BatchedGridEnv(num_agents=n, rooms=product_room_set(src), local_map_length=L, autoreset=autoreset,
                          device="cuda:0", **kw)


def belief_of(env, agent, whd):
    W, D, H = whd
    return env.belief()[agent, :W, :D, :H].cpu().numpy().astype(np.int64)


@pytest.mark.parametrize("path", golden_trajectories(), ids=lambda p: p.stem)
def test_golden_trajectory_on_gpu(voxnav, path):
    d = load_golden(path)
    src = str(d["room_source"])
    env = make_env(voxnav, src, int(d["L"]), crash_penalty=float(d["crash_penalty"]))
    rooms = env.room_set.rooms
    seeds = [int(s) for s in d["seeds"]]
    si = 0

    def do_reset(ri):
        nonlocal si
        obs = env.reset(seed=[seeds[si]]).cpu().numpy()[0]
        si += 1
        assert obs.tobytes() == d["reset_obs"][ri].tobytes(), f"reset obs {ri}"
        st = env.export_state()[0].cpu().numpy()
        assert list(st[STATE_IDX]) == list(d["reset_state"][ri]), f"reset state {ri}"
        room = rooms[int(st[13])]
        assert grid_hash(room.grid()) == int(d["room_hash"][ri])
        return room

    room = do_reset(0)
    ri = 1
    dumps = {int(t): i for i, t in enumerate(d["dump_at"])}
    acts = torch.as_tensor(d["actions"], dtype=torch.int32, device="cuda:0")
    for t in range(len(d["actions"])):
        res = env.step(acts[t:t + 1], reward_f64=True, terminal_obs=False)
        obs = res.obs.cpu().numpy()[0]
        if obs.tobytes() != d["obs"][t].tobytes():
            idx = np.nonzero(obs.view(np.uint32) != d["obs"][t].view(np.uint32))[0]
            st = env.export_state()[0].cpu().numpy()
            raise AssertionError(f"obs mismatch at step {t} (action {d['actions'][t]}): idx {idx.tolist()} "
                                 f"got {obs[idx].tolist()} want {d['obs'][t][idx].tolist()}; "
                                 f"state got {st[STATE_IDX].tolist()} want {d['state'][t].tolist()}")
        assert float(res.reward[0].item()) == float(d["reward"][t]), f"reward at step {t}"
        te, tr = bool(res.terminated[0].item()), bool(res.truncated[0].item())
        assert (te, tr) == (bool(d["terminated"][t]), bool(d["truncated"][t])), t
        st = env.export_state()[0].cpu().numpy()
        assert list(st[STATE_IDX]) == list(d["state"][t]), f"state mismatch at step {t}"
        if t in dumps or t % 97 == 0:
            b = belief_of(env, 0, room.shape)
            if t in dumps:
                ref = np.minimum(d[f"belief_dump_{dumps[t]}"].astype(np.int64), 127)
                assert (b == ref).all(), f"belief dump at step {t}"
            if b.max() < 127:
                assert grid_hash(b) == int(d["belief_hash"][t]), f"belief hash at step {t}"
        if te or tr:
            room = do_reset(ri)
            ri += 1
    assert si == len(seeds)


ROLLOUT_CASES = [
    # (room source, L, agents, steps)
    ("box:8x8x4", 4, 512, 300),
    ("ctor:8x8x4", 10, 256, 200),
    ("box:16x16x8", 4, 512, 400),
    ("ctor:32x32x8", 10, 1024, 150),
    ("set:P2_training", 10, 1024, 200),
    ("set:P3_training", 10, 1024, 200),
    ("set:P1_training", 4, 256, 200),
    ("file:P3_training/maze_3d_tunnels.txt", 10, 512, 400),
    ("file:P2_training/tightcorridor.txt", 7, 300, 300),
    ("file:P3_training/kitchen2.txt", 16, 256, 200),
]


@pytest.mark.parametrize("src,L,N,K", ROLLOUT_CASES, ids=[f"{c[0]}-L{c[1]}" for c in ROLLOUT_CASES])
def test_random_rollout_matches_oracle(voxnav, src, L, N, K):
    env = make_env(voxnav, src, L, n=N, autoreset=True)
    seeds = 42 + np.arange(N, dtype=np.int64)
    env.reset(seed=42)
    ro = env.step_random(K, policy_seed=7, t0=0, record_actions=True, reward_f64=True)
    orc = oracle_env(src, L, n_agents=N).run_random(seeds, policy_seed=7, K=K, seed_stride=N)
    np.testing.assert_array_equal(ro.actions.cpu().numpy(), orc["actions"])
    np.testing.assert_array_equal(ro.terminated.cpu().numpy(), orc["terminated"])
    np.testing.assert_array_equal(ro.truncated.cpu().numpy(), orc["truncated"])
    np.testing.assert_array_equal(ro.reward.cpu().numpy(), orc["reward"])
    got = ro.obs.cpu().numpy()
    bad = np.argwhere((got.view(np.uint32) != orc["obs"].view(np.uint32)).any(-1))
    assert bad.size == 0, f"obs mismatch at (step, agent) {bad[:5].tolist()}"


FAST_CASES = [("ctor:32x32x8", 10, 1024, 160), ("set:P3_training", 10, 1000, 120), ("box:8x8x4", 4, 333, 200)]


@pytest.mark.parametrize("src,L,N,K", FAST_CASES, ids=[f"{c[0]}-N{c[2]}" for c in FAST_CASES])
def test_rollout_buffer_call_matches_oracle(voxnav, src, L, N, K):
    """The rollout-buffer call (f32 reward, flags, no action record / f64
    reward) runs its own kernel instantiation: bit-exact against the oracle,
    including agent counts that leave a partly filled wave (N % 16 != 0)."""
    env = make_env(voxnav, src, L, n=N, autoreset=True)
    env.reset(seed=42)
    ro = env.step_random(K, policy_seed=7, t0=0)
    orc = oracle_env(src, L, n_agents=N).run_random(42 + np.arange(N, dtype=np.int64), policy_seed=7, K=K,
                                                    seed_stride=N)
    np.testing.assert_array_equal(ro.terminated.cpu().numpy(), orc["terminated"])
    np.testing.assert_array_equal(ro.truncated.cpu().numpy(), orc["truncated"])
    np.testing.assert_array_equal(ro.reward.cpu().numpy(), orc["reward"].astype(np.float32))
    assert ro.obs.cpu().numpy().tobytes() == orc["obs"].tobytes()


def test_step_with_actions_f32_matches_oracle(voxnav):
    """vn_step with explicit actions, f32 reward, terminal_obs (the collector's call)."""
    src, L, N, K = "box:8x8x4", 4, 400, 100
    env = make_env(voxnav, src, L, n=N, autoreset=True)
    env.reset(seed=1000)
    acts = np.random.default_rng(5).integers(0, 6, size=(K, N)).astype(np.int32)
    orc = oracle_env(src, L, n_agents=N).run_random(1000 + np.arange(N), policy_seed=0, K=K, seed_stride=N,
                                                    actions=acts, terminal_obs=True)
    at = torch.as_tensor(acts, device="cuda:0")
    for k in range(K):
        res = env.step(at[k], reward_f64=False, terminal_obs=True)
        np.testing.assert_array_equal(res.obs.cpu().numpy(), orc["obs"][k])
        np.testing.assert_array_equal(res.reward.cpu().numpy(), orc["reward"][k].astype(np.float32))
        te, tr = res.terminated.cpu().numpy(), res.truncated.cpu().numpy()
        np.testing.assert_array_equal(te, orc["terminated"][k].astype(bool))
        np.testing.assert_array_equal(tr, orc["truncated"][k].astype(bool))
        done = te | tr
        np.testing.assert_array_equal(res.terminal_obs.cpu().numpy()[done], orc["terminal_obs"][k][done])


def test_step_random_refuses_short_rollout_buffers(voxnav):
    """A caller-owned rollout chunk shorter than k_steps (or mistyped) is
    refused before the launch: the kernel writes all K steps."""
    from voxnav.env import Rollout
    N = 64
    env = make_env(voxnav, "box:8x8x4", 4, n=N, autoreset=True)
    env.reset(seed=3)
    dev = env.device

    def chunk(K, rdt=torch.float32):
        return Rollout(torch.empty((K, N, 80), device=dev), torch.empty((K, N), dtype=rdt, device=dev),
                       torch.empty((K, N), dtype=torch.uint8, device=dev),
                       torch.empty((K, N), dtype=torch.uint8, device=dev), None)
    with pytest.raises(ValueError):
        env.step_random(5, out=chunk(1))
    with pytest.raises(ValueError):
        env.step_random(2, out=chunk(2, torch.float64))
    with pytest.raises(ValueError):
        env.step_random_launcher(3, 7, 0, chunk(2))
    env.step_random(2, out=chunk(2))          # the right shape runs
    torch.cuda.synchronize()


def test_step_with_actions_autoreset_terminal_obs(voxnav):
    """vn_step with explicit actions: obs/terminal_obs/flags vs oracle (SB3 semantics)."""
    src, L, N, K = "box:8x8x4", 4, 384, 160
    env = make_env(voxnav, src, L, n=N, autoreset=True)
    env.reset(seed=1000)
    rng = np.random.default_rng(3)
    acts = rng.integers(0, 6, size=(K, N)).astype(np.int32)
    orc = oracle_env(src, L, n_agents=N).run_random(1000 + np.arange(N), policy_seed=0, K=K, seed_stride=N,
                                                    actions=acts, terminal_obs=True)
    at = torch.as_tensor(acts, device="cuda:0")
    ended = 0
    for k in range(K):
        res = env.step(at[k], reward_f64=True, terminal_obs=True)
        np.testing.assert_array_equal(res.obs.cpu().numpy(), orc["obs"][k])
        np.testing.assert_array_equal(res.reward.cpu().numpy(), orc["reward"][k])
        te, tr = res.terminated.cpu().numpy(), res.truncated.cpu().numpy()
        np.testing.assert_array_equal(te, orc["terminated"][k].astype(bool))
        np.testing.assert_array_equal(tr, orc["truncated"][k].astype(bool))
        done = te | tr
        ended += int(done.sum())
        np.testing.assert_array_equal(res.terminal_obs.cpu().numpy()[done], orc["terminal_obs"][k][done])
    assert ended >= N  # every agent finished at least one 72-step episode


@pytest.mark.parametrize("tag", ["P1_training", "P2_training", "P3_training", "P2_evaluate", "box32x32x8"])
def test_reset_draws_match_reference_on_gpu(voxnav, tag):
    z = load_golden(GOLDEN / f"reset_table_{tag}.npz")
    src = "ctor:32x32x8" if tag.startswith("box") else f"set:{tag}"
    seeds = z["seeds"].astype(np.int64)
    env = make_env(voxnav, src, 10, n=len(seeds))
    env.reset(seed=seeds)
    st = env.export_state().cpu().numpy()
    got = np.stack([st[:, 13], st[:, 0], st[:, 1], st[:, 2]], axis=1)
    np.testing.assert_array_equal(got, z["draws"])


def test_reset_many_rejections_slow_path(voxnav):
    """Seeds whose reset needs > 8 MT words exercise the device slow path."""
    src = "set:P2_evaluate"   # 7 rooms: k=3 bits, reject 1/8
    orc = oracle_env(src, 4)
    found = []
    for s in range(200000):
        room, xyz, draws = orc.reset_draw(s)
        if draws >= 6:
            found.append((s, room, xyz, draws))
        if len(found) >= 64:
            break
    assert max(f[3] for f in found) >= 9, "no seed needing > 8 draws found"
    seeds = np.array([f[0] for f in found], np.int64)
    env = make_env(voxnav, src, 4, n=len(seeds))
    env.reset(seed=seeds)
    st = env.export_state().cpu().numpy()
    for i, (s, room, xyz, draws) in enumerate(found):
        assert (st[i, 13], st[i, 0], st[i, 1], st[i, 2]) == (room, *xyz), (s, draws)


def test_sharding_is_bitwise_invariant(voxnav):
    """Two shards (agent_id_base 0 and N/2) == one env of N agents."""
    src, L, N, K = "set:P3_training", 10, 512, 120
    full = make_env(voxnav, src, L, n=N, autoreset=True)
    full.reset(seed=42)
    a = full.step_random(K, policy_seed=5, t0=0)
    parts = []
    for base in (0, N // 2):
        sh = make_env(voxnav, src, L, n=N // 2, autoreset=True, agent_id_base=base, seed_stride=N)
        sh.reset(seed=42)
        parts.append(sh.step_random(K, policy_seed=5, t0=0))
    obs = torch.cat([parts[0].obs, parts[1].obs], dim=1)
    assert torch.equal(obs, a.obs)
    assert torch.equal(torch.cat([parts[0].reward, parts[1].reward], 1), a.reward)


def test_fused_k_equals_single_steps(voxnav):
    src, L, N = "set:P2_training", 10, 640
    e1 = make_env(voxnav, src, L, n=N, autoreset=True)
    e2 = make_env(voxnav, src, L, n=N, autoreset=True)
    e1.reset(seed=9)
    e2.reset(seed=9)
    a = e1.step_random(64, policy_seed=11, t0=100)
    for k in range(64):
        b = e2.step_random(1, policy_seed=11, t0=100 + k)
        assert torch.equal(a.obs[k], b.obs[0]), k
        assert torch.equal(a.reward[k], b.reward[0]), k


def test_full_size_properties(voxnav):
    """BASELINE config at full size (65536 agents, 32x32x8, L=10): a sampled
    subset of agents against the oracle + size-independent invariants."""
    N, L, K = 65536, 10, 64
    env = make_env(voxnav, "box:32x32x8", L, n=N, autoreset=True)
    env.reset(seed=42)
    ro = env.step_random(K, policy_seed=42, t0=0, reward_f64=True)
    obs = ro.obs.cpu().numpy()
    # window values lie on the (v+2)/22 lattice, facing one-hot sums to 1
    lattice = (np.arange(23, dtype=np.float32) / np.float32(22.0)).astype(np.float32)
    assert np.isin(obs[:, :, :64], lattice).all()
    np.testing.assert_array_equal(obs[:, :, 64:68].sum(-1), 1.0)
    assert (obs[:, :, 73:] == 0).all()
    # sampled agents replayed alone through the oracle (agents are independent)
    rng = np.random.default_rng(0)
    for g in rng.choice(N, size=24, replace=False):
        orc = oracle_env("box:32x32x8", L, n_agents=1).run_random(
            [42 + int(g)], policy_seed=42, K=K, gid_base=int(g), seed_stride=N)
        assert obs[:, g].tobytes() == orc["obs"][:, 0].tobytes(), g
        np.testing.assert_array_equal(ro.reward[:, g].cpu().numpy(), orc["reward"][:, 0])


def test_full_size_p3_sampled_belief(voxnav):
    """P3_training at the bench's agent count (65536, byte-mark kernel with
    deferred plane marks), one 128-step launch: sampled agents replayed alone
    through the oracle -- obs, f64 rewards, flags and the final belief map."""
    src, N, L, K = "set:P3_training", 65536, 10, 128
    env = make_env(voxnav, src, L, n=N, autoreset=True)
    env.reset(seed=42)
    ro = env.step_random(K, policy_seed=42, t0=0, reward_f64=True)
    rng = np.random.default_rng(1)
    picks = rng.choice(N, size=16, replace=False)
    sel = torch.as_tensor(picks, device=env.device)
    b = env.belief().index_select(0, sel).cpu().numpy().astype(np.int64)
    st = env.export_state().cpu().numpy()
    obs = ro.obs.index_select(1, sel).cpu().numpy()
    rew = ro.reward.index_select(1, sel).cpu().numpy()
    te = ro.terminated.index_select(1, sel).cpu().numpy()
    rooms = env.room_set.rooms
    for j, g in enumerate(picks):
        orc_env = oracle_env(src, L, n_agents=1)
        orc = orc_env.run_random([42 + int(g)], policy_seed=42, K=K, gid_base=int(g), seed_stride=N)
        assert obs[:, j].tobytes() == orc["obs"][:, 0].tobytes(), g
        np.testing.assert_array_equal(rew[:, j], orc["reward"][:, 0])
        np.testing.assert_array_equal(te[:, j], orc["terminated"][:, 0])
        W, D, H = rooms[int(st[g, 13])].shape
        np.testing.assert_array_equal(b[j, :W, :D, :H], np.minimum(orc_env.belief(0), 63), err_msg=f"agent {g}")


@pytest.mark.parametrize("src", ["set:P3_training", "set:P2_training"])
def test_full_batch_room_set_sampled_blocks_through_autoreset(voxnav, src):
    """The room-set bench workload as the bench runs it: 65,536 agents, f32
    reward into a caller-owned rollout, five 128-step launches (640 steps).
    One agent from every 64-agent block is replayed through the oracle launch
    by launch -- obs bytes, reward, terminated / truncated -- across
    auto-resets.  The sampled agent of a block is one whose first room has at
    most 600 free cells when the block has such an agent (an episode truncates
    when its step count reaches the room's free cells, so each of those
    certainly ends an episode and restarts in a newly drawn room inside the
    window); the test asserts that at least 90 % of the sample is of that kind
    and that every one of them reset.  Belief maps of every 8th sampled agent
    are compared after the first and the last launch."""
    from voxnav.env import Rollout
    N, L, F, K_TOTAL = 65536, 10, 128, 640
    env = make_env(voxnav, src, L, n=N, autoreset=True)
    dev = env.device
    env.reset(seed=42)
    room0 = env.export_state().cpu().numpy()[:, 13]
    short = env.total_free_cells[room0] <= 600                  # certainly truncate within the window
    blocks = np.arange(N // 64, dtype=np.int64)
    rot = (blocks[:, None] * 41 + 17 + np.arange(64)[None, :]) % 64     # per block, a rotated scan order
    cand = blocks[:, None] * 64 + rot
    first = np.argmax(short[cand], axis=1)                      # first short-room agent in scan order (0 if none)
    sample = cand[blocks, first]
    sure = short[sample]
    assert sure.mean() >= 0.9, f"{src}: only {sure.sum()} of {len(sample)} sampled agents in a short room"
    dump = sample[::8]
    idx = torch.as_tensor(sample, device=dev)
    orc_env = oracle_env(src, L, n_agents=len(sample))
    out = Rollout(torch.empty((F, N, 80), dtype=torch.float32, device=dev),
                  torch.empty((F, N), dtype=torch.float32, device=dev),
                  torch.empty((F, N), dtype=torch.uint8, device=dev),
                  torch.empty((F, N), dtype=torch.uint8, device=dev), None)
    env.reset(seed=42)                                          # again: the same draws (seeded)
    rooms = env.room_set.rooms
    resets = np.zeros(len(sample), dtype=np.int64)
    for t in range(0, K_TOTAL, F):
        env.step_random(F, policy_seed=42, t0=t, out=out)
        orc = orc_env.run_random(42 + sample, policy_seed=42, K=F, t0=t, seed_stride=N, initial_reset=(t == 0),
                                 gids=sample, threads=8)
        obs = out.obs.index_select(1, idx).cpu().numpy()
        if obs.tobytes() != orc["obs"].tobytes():
            bad = np.argwhere((obs.view(np.uint32) != orc["obs"].view(np.uint32)).any(-1))
            raise AssertionError(f"{src}: obs mismatch at (step, sampled agent) {(bad[:5] + [t, 0]).tolist()}")
        np.testing.assert_array_equal(out.reward.index_select(1, idx).cpu().numpy(),
                                      orc["reward"].astype(np.float32), err_msg=f"{src} reward, steps {t}..{t + F}")
        te = out.terminated.index_select(1, idx).cpu().numpy()
        tr = out.truncated.index_select(1, idx).cpu().numpy()
        np.testing.assert_array_equal(te, orc["terminated"], err_msg=f"{src} terminated, steps {t}..{t + F}")
        np.testing.assert_array_equal(tr, orc["truncated"], err_msg=f"{src} truncated, steps {t}..{t + F}")
        resets += (te | tr).sum(0).astype(np.int64)
        if t == 0 or t + F == K_TOTAL:
            st = env.export_state().cpu().numpy()
            b = env.belief().index_select(0, torch.as_tensor(dump, device=dev)).cpu().numpy().astype(np.int64)
            for j, g in enumerate(dump):
                W, D, H = rooms[int(st[g, 13])].shape
                np.testing.assert_array_equal(b[j, :W, :D, :H], np.minimum(orc_env.belief(8 * j), 63),
                                              err_msg=f"{src}: belief of agent {g} after step {t + F}")
    assert (resets[sure] > 0).all(), f"{src}: {(resets[sure] == 0).sum()} short-room agents did not reset"
    assert (resets > 0).mean() >= 0.9, f"{src}: only {(resets > 0).sum()} of {len(sample)} sampled agents reset"
    env.close()


def test_gae_matches_oracle(voxnav):
    from oracle.oracle import gae as oracle_gae
    from voxnav.gae import compute_gae
    T, N = 128, 3000
    rng = np.random.default_rng(1)
    r = rng.normal(size=(T, N)).astype(np.float32)
    v = rng.normal(size=(T, N)).astype(np.float32)
    s = (rng.random((T, N)) < 0.05).astype(np.float32)
    s[0] = 1
    lv = rng.normal(size=N).astype(np.float32)
    dn = (rng.random(N) < 0.1).astype(np.float32)
    adv, ret = compute_gae(*(torch.as_tensor(a, device="cuda:0") for a in (r, v, s, lv, dn)))
    ea, er = oracle_gae(r, v, s, lv, dn)
    np.testing.assert_array_equal(adv.cpu().numpy(), ea)
    np.testing.assert_array_equal(ret.cpu().numpy(), er)


def test_gridagent_facade_matches_golden(voxnav):
    from voxnav.gym_api import GridAgent
    d = load_golden(GOLDEN / "traj_box8x8x4_file_L4_explore.npz")
    ag = GridAgent(local_map_length=4, rooms=product_room_set("box:8x8x4").rooms)
    obs, info = ag.reset(seed=int(d["seeds"][0]))
    assert obs.dtype == np.float32 and obs.shape == (80,) and info == {}
    assert obs.tobytes() == d["reset_obs"][0].tobytes()
    si = 1
    for t, a in enumerate(d["actions"][:150]):
        obs, r, te, tr, info = ag.step(int(a))
        assert isinstance(r, np.float64) and r == d["reward"][t]
        assert obs.tobytes() == d["obs"][t].tobytes()
        assert ag.visited_count == d["state"][t][6] and ag.bump_count == d["state"][t][7]
        if te or tr:
            ag.reset(seed=int(d["seeds"][si]))
            si += 1
    ag.close()

MIX_CASES = [("box:32x32x8", 10, 96), ("box:8x8x4", 4, 40), ("box:16x16x8", 7, 50), ("set:P3_training", 10, 64),
             ("box:100x40x8", 10, 48)]
# belief modes: (VOXNAV_PCACHE, VOXNAV_DEFER)
MIX_MODES = [("0", "1"), ("0", "0"), ("1", "1"), ("2", "1")]


@pytest.mark.parametrize("pcache,defer", MIX_MODES, ids=[f"pc{a}-df{b}" for a, b in MIX_MODES])
@pytest.mark.parametrize("src,L,N", MIX_CASES, ids=[c[0] for c in MIX_CASES])
def test_launch_mix_belief_matches_oracle(voxnav, monkeypatch, pcache, defer, src, L, N):
    """Launches of 16, 1, 5, 3 and 30 fused steps on one env in each belief
    mode (VOXNAV_PCACHE: 0 byte marks, 1 plane sets in u64 LDS rows, 2 in u32
    rows -- marks outside the window then live only in the marked-bit planes
    and reach a column's bytes when it enters the window; VOXNAV_DEFER 1: in
    byte-mark mode with plane rows of <= 2 words a sensing pass's plane marks
    are applied at the start of the next step or at the launch's end):
    obs, f64 rewards, flags and every agent's exported belief map equal the
    oracle's after 120 steps with auto-resets."""
    if pcache != "0" and src.startswith(("set:", "box:100")):
        pytest.skip("plane-set modes need PH-8 rooms of <= 64 x 64")
    monkeypatch.setenv("VOXNAV_PCACHE", pcache)
    monkeypatch.setenv("VOXNAV_DEFER", defer)
    env = make_env(voxnav, src, L, n=N, autoreset=True)
    env.reset(seed=42)
    ks = [16, 1, 5, 16, 3, 16, 16, 1, 16, 30]
    obs, rew, te, tr = [], [], [], []
    for k in ks:
        ro = env.step_random(k, policy_seed=7, reward_f64=True)
        obs.append(ro.obs.cpu().numpy())
        rew.append(ro.reward.cpu().numpy())
        te.append(ro.terminated.cpu().numpy())
        tr.append(ro.truncated.cpu().numpy())
    orc_env = oracle_env(src, L, n_agents=N)
    orc = orc_env.run_random(42 + np.arange(N, dtype=np.int64), policy_seed=7, K=sum(ks), seed_stride=N)
    assert np.concatenate(obs).tobytes() == orc["obs"].tobytes()
    np.testing.assert_array_equal(np.concatenate(rew), orc["reward"])
    np.testing.assert_array_equal(np.concatenate(te), orc["terminated"])
    np.testing.assert_array_equal(np.concatenate(tr), orc["truncated"])
    b = env.belief().cpu().numpy().astype(np.int64)
    st = env.export_state().cpu().numpy()
    rooms = env.room_set.rooms
    for a in range(N):
        W, D, H = rooms[int(st[a, 13])].shape
        np.testing.assert_array_equal(b[a, :W, :D, :H], np.minimum(orc_env.belief(a), 63), err_msg=f"agent {a}")


WREC_CASES = [("box:32x32x8", 10, 64, "2"), ("box:16x16x8", 7, 48, "0"), ("set:P3_training", 10, 64, "3"),
              ("box:100x40x8", 10, 32, "0")]
# window record settings: (VOXNAV_ENV_WREC: launches of at most this many steps write it, VOXNAV_ENV_WREC_EARLY)
WREC_MODES = [("1", "1"), ("8", "1"), ("8", "0"), ("0", "1")]


@pytest.mark.parametrize("wrec,early", WREC_MODES, ids=[f"wrec{a}-early{b}" for a, b in WREC_MODES])
@pytest.mark.parametrize("src,L,N,pcache", WREC_CASES, ids=[f"{c[0]}-pc{c[3]}" for c in WREC_CASES])
def test_window_record_launch_mix_matches_oracle(voxnav, monkeypatch, wrec, early, src, L, N, pcache):
    """The window record (csrc/voxnav_env.hip wrec_fill): a step launch of at
    most VOXNAV_ENV_WREC steps stores the agent's 16 window columns and the
    next launch fills its window from them (loaded beside the state with
    VOXNAV_ENV_WREC_EARLY=1).  Runs of one-step launches (record -> record),
    short launches that write it and long ones that do not (their next launch
    falls back to the map; the P3 set's small rooms end episodes inside the
    76 steps, so auto-resets run between records): obs, f64 rewards, flags
    and every agent's belief map equal the oracle's, in each belief mode
    (pcache "3": the mode the room set selects; "0" forces byte marks)."""
    monkeypatch.setenv("VOXNAV_ENV_WREC", wrec)
    monkeypatch.setenv("VOXNAV_ENV_WREC_EARLY", early)
    if pcache != "3":
        monkeypatch.setenv("VOXNAV_PCACHE", pcache)
    env = make_env(voxnav, src, L, n=N, autoreset=True)
    env.reset(seed=42)
    ks = [1, 1, 1, 5, 1, 1, 16, 1, 2, 1, 1, 8, 1, 30, 1, 1]
    obs, rew, te, tr = [], [], [], []
    for k in ks:
        ro = env.step_random(k, policy_seed=7, reward_f64=True)
        obs.append(ro.obs.cpu().numpy())
        rew.append(ro.reward.cpu().numpy())
        te.append(ro.terminated.cpu().numpy())
        tr.append(ro.truncated.cpu().numpy())
    orc_env = oracle_env(src, L, n_agents=N)
    orc = orc_env.run_random(42 + np.arange(N, dtype=np.int64), policy_seed=7, K=sum(ks), seed_stride=N)
    assert np.concatenate(obs).tobytes() == orc["obs"].tobytes()
    np.testing.assert_array_equal(np.concatenate(rew), orc["reward"])
    np.testing.assert_array_equal(np.concatenate(te), orc["terminated"])
    np.testing.assert_array_equal(np.concatenate(tr), orc["truncated"])
    b = env.belief().cpu().numpy().astype(np.int64)
    st = env.export_state().cpu().numpy()
    rooms = env.room_set.rooms
    for a in range(N):
        W, D, H = rooms[int(st[a, 13])].shape
        np.testing.assert_array_equal(b[a, :W, :D, :H], np.minimum(orc_env.belief(a), 63), err_msg=f"agent {a}")


@pytest.mark.parametrize("src", ["box:32x32x8", "box:16x16x8"])
def test_masked_reset_mid_episode_matches_fresh_env(voxnav, src):
    """vn_reset with a mask in the middle of an episode (plane-set mode with
    the stood-column map for these rooms): the reset agents then step exactly
    like a fresh env reset with the same seeds, and the others exactly like an
    env that was never partly reset -- obs, f64 rewards, flags and belief maps,
    over launches of 1 and 7 steps.  Covers the per-agent stood rows and
    nonzero-set masks a reset must clear (envs/CubicEnv.py:77-108)."""
    N, L = 64, 10
    rng = np.random.default_rng(5)
    a_pre = rng.integers(0, 6, size=(37, N)).astype(np.int32)
    a_post = rng.integers(0, 6, size=(41, N)).astype(np.int32)
    odd = torch.zeros(N, dtype=torch.uint8)
    odd[1::2] = 1
    new_seeds = 1000 + np.arange(N, dtype=np.int64) * 7

    def run(env, steps):
        out = []
        for t in range(steps.shape[0]):
            r = env.step(torch.as_tensor(steps[t]), reward_f64=True)
            out.append((r.obs.cpu().numpy(), r.reward.cpu().numpy(), r.terminated.cpu().numpy(),
                        r.truncated.cpu().numpy()))
        return out

    A = make_env(voxnav, src, L, n=N)
    C = make_env(voxnav, src, L, n=N)
    B = make_env(voxnav, src, L, n=N)
    for e in (A, C):
        e.reset(seed=42)
        run(e, a_pre)
        e.step_random(7, policy_seed=3, t0=0)          # a fused launch in the middle
    A.reset(seed=new_seeds, mask=odd)
    B.reset(seed=new_seeds)
    ra, rb, rc = run(A, a_post), run(B, a_post), run(C, a_post)
    o, e_ = odd.numpy().astype(bool), ~odd.numpy().astype(bool)
    for t in range(len(ra)):
        for k in range(4):
            assert ra[t][k][o].tobytes() == rb[t][k][o].tobytes(), (t, k)
            assert ra[t][k][e_].tobytes() == rc[t][k][e_].tobytes(), (t, k)
    ba, bb, bc = (x.belief().cpu().numpy() for x in (A, B, C))
    np.testing.assert_array_equal(ba[o], bb[o])
    np.testing.assert_array_equal(ba[e_], bc[e_])
    sa, sb, sc = (x.export_state().cpu().numpy() for x in (A, B, C))
    np.testing.assert_array_equal(sa[o], sb[o])
    np.testing.assert_array_equal(sa[e_], sc[e_])
    for e in (A, B, C):
        e.close()
