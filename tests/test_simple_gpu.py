"""Parity of the simpleEnv variant (envs/simpleEnv.py)
on the GPU, through the C-ABI.

Bar: bit-exact obs (f32 bytes, 6L+7 floats), exact f64 reward, identical
terminated / truncated flags, integer agent state, goal and belief map --
on the reference's golden simpleEnv trajectories (tests/golden/simple_*.npz,
reset seeded with random.seed(seed) then get_obs(), see gen_golden.py) and
against the CPU oracle for batched random-policy rollouts with SB3
auto-reset.
"""
import numpy as np
import pytest

from helpers import grid_hash, load_golden, oracle_env, product_room_set, simple_golden_trajectories

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

STATE9 = [0, 1, 2, 3, 4, 5, 6, 7, 8]   # x y z facing last_action step visited bumps done


@pytest.fixture(scope="module")
def voxnav():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import voxnav
    voxnav.load_library()
    return voxnav


def make_env(src, L, n=1, autoreset=False, **kw):
    from voxnav.env import BatchedGridEnv
    return BatchedGridEnv(num_agents=n, rooms=product_room_set(src), local_map_length=L, autoreset=autoreset,
                          device="cuda:0", variant="simple", **kw)


@pytest.mark.parametrize("path", simple_golden_trajectories(), ids=lambda p: p.stem)
def test_simple_golden_trajectory_on_gpu(voxnav, path):
    d = load_golden(path)
    L = int(d["L"])
    env = make_env(str(d["room_source"]), L)
    assert env.obs_dim == 6 * L + 7
    seeds = [int(s) for s in d["seeds"]]
    si = 0

    def do_reset(ri):
        nonlocal si
        obs = env.reset(seed=[seeds[si]]).cpu().numpy()[0]
        si += 1
        assert obs.tobytes() == d["reset_obs"][ri].tobytes(), f"reset obs {ri}"
        st = env.export_state()[0].cpu().numpy()
        assert [st[0], st[1], st[2], st[9], st[10], st[11]] == list(d["reset_state"][ri]), f"reset/goal {ri}"
        return env.room_set.rooms[int(st[13])]

    room = do_reset(0)
    ri = 1
    acts = torch.as_tensor(d["actions"], dtype=torch.int32, device="cuda:0")
    for t in range(len(d["actions"])):
        res = env.step(acts[t:t + 1], reward_f64=True, terminal_obs=False)
        obs = res.obs.cpu().numpy()[0]
        assert obs.tobytes() == d["obs"][t].tobytes(), f"obs mismatch at step {t}"
        assert float(res.reward[0].item()) == float(d["reward"][t]), f"reward at step {t}"
        te, tr = bool(res.terminated[0].item()), bool(res.truncated[0].item())
        assert (te, tr) == (bool(d["terminated"][t]), bool(d["truncated"][t])), t
        st = env.export_state()[0].cpu().numpy()
        assert list(st[STATE9]) == list(d["state"][t]), f"state mismatch at step {t}"
        if t % 23 == 0 or te or tr:
            W, D, H = room.shape
            b = env.belief()[0, :W, :D, :H].cpu().numpy().astype(np.int64)
            assert grid_hash(b) == int(d["belief_hash"][t]), f"belief hash at step {t}"
        if te or tr:
            room = do_reset(ri)
            ri += 1
    assert si == len(seeds)


SIMPLE_CASES = [
    ("box:8x8x4", 4, 512, 300),
    ("ctor:12x10x6", 10, 256, 200),
    ("set:P2_training", 4, 1024, 250),
    ("set:P3_training", 10, 1024, 200),
    ("file:P2_training/maze_8x8_seed22.txt", 10, 300, 300),
    ("file:P3_training/kitchen2.txt", 16, 256, 200),
    ("set:P1_training", 7, 200, 150),
]


@pytest.mark.parametrize("src,L,N,K", SIMPLE_CASES, ids=[f"{c[0]}-L{c[1]}" for c in SIMPLE_CASES])
def test_simple_random_rollout_matches_oracle(voxnav, src, L, N, K):
    _rollout_vs_oracle(src, L, N, K)


# the word-layout pipelined kernel (simple_pipe_kernel: the default for rooms
# higher than 8 or wider / deeper than 32) on rooms the line layout takes by default
PIPE_CASES = [("box:8x8x4", 4, 300, 200), ("set:P2_training", 4, 1024, 250), ("ctor:12x10x6", 10, 256, 200)]


@pytest.mark.parametrize("src,L,N,K", PIPE_CASES, ids=[f"{c[0]}-L{c[1]}" for c in PIPE_CASES])
def test_simple_word_layout_kernel_matches_oracle(voxnav, monkeypatch, src, L, N, K):
    monkeypatch.setenv("VOXNAV_SIMPLE_LINE", "0")
    env = make_env(src, L, n=8)
    assert env.kernel_label(16).startswith("simple_pipe_kernel<")
    env.close()
    _rollout_vs_oracle(src, L, N, K)


# the dense int8 map kernel: rooms wider or deeper than 64 cells, or forced
# with VOXNAV_SIMPLE_DENSE=1 (the bit-plane kernel covers the cases above)
DENSE_CASES = [
    ("ctor:70x9x5", 4, 256, 200, False),
    ("ctor:10x66x5", 6, 128, 150, False),
    ("set:P3_training", 10, 512, 150, True),
    ("box:8x8x4", 4, 256, 200, True),
]


@pytest.mark.parametrize("src,L,N,K,force", DENSE_CASES, ids=[f"{c[0]}-L{c[1]}" for c in DENSE_CASES])
def test_simple_dense_layout_matches_oracle(voxnav, monkeypatch, src, L, N, K, force):
    if force:
        monkeypatch.setenv("VOXNAV_SIMPLE_DENSE", "1")
    _rollout_vs_oracle(src, L, N, K)


def _rollout_vs_oracle(src, L, N, K):
    env = make_env(src, L, n=N, autoreset=True)
    seeds = 42 + np.arange(N, dtype=np.int64)
    obs0 = env.reset(seed=42).cpu().numpy()
    oenv = oracle_env(src, L, n_agents=N, variant=1)
    ref0 = np.stack([oracle_env(src, L, variant=1).reset(0, int(s)) for s in seeds[:8]])
    assert obs0[:8].tobytes() == ref0.tobytes()
    ro = env.step_random(K, policy_seed=7, t0=0, record_actions=True, reward_f64=True)
    orc = oenv.run_random(seeds, policy_seed=7, K=K, seed_stride=N)
    np.testing.assert_array_equal(ro.actions.cpu().numpy(), orc["actions"])
    np.testing.assert_array_equal(ro.terminated.cpu().numpy(), orc["terminated"])
    np.testing.assert_array_equal(ro.truncated.cpu().numpy(), orc["truncated"])
    np.testing.assert_array_equal(ro.reward.cpu().numpy(), orc["reward"])
    got = ro.obs.cpu().numpy()
    bad = np.argwhere((got.view(np.uint32) != orc["obs"].view(np.uint32)).any(-1))
    assert bad.size == 0, f"obs mismatch at (step, agent) {bad[:5].tolist()}"
    st = env.export_state().cpu().numpy()
    for i in range(0, N, max(1, N // 16)):
        o = oenv.state(i)
        assert [o[f] for f in ("x", "y", "z", "facing", "last_action", "step_count", "visited_count",
                               "bump_count", "done", "room")] == [int(v) for v in st[i, [0, 1, 2, 3, 4, 5, 6, 7,
                                                                                       8, 13]]]
        assert (o["last_bump"], o["near_wall"], o["was_near_wall"]) == tuple(int(v) for v in st[i, 9:12])  # goal
        W, D, H = oenv.rooms[o["room"]].whd
        b = env.belief()[i, :W, :D, :H].cpu().numpy().astype(np.int64)
        np.testing.assert_array_equal(b, oenv.belief(i))


def _bench_shaped_run(N, sample, K, F=128, src="box:32x32x8", L=4, policy_seed=42,
                      label="simple_line_kernel<4, false>"):
    """The bench's simpleEnv call: ``step_random(out=...)`` in F-step launches
    into a reused [F, N, 6L+7] chunk, f32 reward, no action record; the
    sampled agents compared with the oracle launch by launch (the per-agent
    reset draw-ahead is carried across launches)."""
    from voxnav.env import Rollout
    env = make_env(src, L, n=N, autoreset=True)
    assert env.kernel_label(F) == label
    dev = env.device
    D = env.obs_dim
    out = Rollout(torch.empty((F, N, D), dtype=torch.float32, device=dev),
                  torch.empty((F, N), dtype=torch.float32, device=dev),
                  torch.empty((F, N), dtype=torch.uint8, device=dev),
                  torch.empty((F, N), dtype=torch.uint8, device=dev), None)
    idx = torch.as_tensor(sample, device=dev)
    gids = np.asarray(sample, dtype=np.int64)
    oenv = oracle_env(src, L, n_agents=len(sample), variant=1)
    env.reset(seed=42)
    t, ends = 0, {"terminated": 0, "truncated": 0}
    while t < K:
        k = min(F, K - t)
        env.step_random(k, policy_seed=policy_seed, t0=t,
                        out=Rollout(out.obs[:k], out.reward[:k], out.terminated[:k], out.truncated[:k], None))
        orc = oenv.run_random(42 + gids, policy_seed=policy_seed, K=k, t0=t, seed_stride=N, initial_reset=(t == 0),
                              gids=gids, threads=8)
        got = out.obs[:k].index_select(1, idx).cpu().numpy()
        bad = np.argwhere((got.view(np.uint32) != orc["obs"].view(np.uint32)).any(-1))
        assert bad.size == 0, f"obs mismatch at (step, sampled agent) {(bad[:5] + [t, 0]).tolist()}"
        np.testing.assert_array_equal(out.reward[:k].index_select(1, idx).cpu().numpy(),
                                      orc["reward"].astype(np.float32), err_msg=f"reward, steps {t}..{t + k}")
        for f in ends:
            g = getattr(out, f)[:k].index_select(1, idx).cpu().numpy()
            np.testing.assert_array_equal(g, orc[f], err_msg=f"{f}, steps {t}..{t + k}")
            ends[f] += int(g.sum())
        t += k
    st = env.export_state().index_select(0, idx).cpu().numpy()
    bel = env.belief()
    for j in range(0, len(sample), max(1, len(sample) // 32)):
        o = oenv.state(j)
        assert [o[f] for f in ("x", "y", "z", "facing", "last_action", "step_count", "visited_count", "bump_count",
                               "done")] == [int(v) for v in st[j, :9]], f"state of agent {sample[j]}"
        W, D_, H = oenv.rooms[o["room"]].whd
        b = bel[int(sample[j]), :W, :D_, :H].cpu().numpy().astype(np.int64)
        np.testing.assert_array_equal(b, oenv.belief(j), err_msg=f"belief of agent {sample[j]}")
    env.close()
    return ends


def test_simple_bench_instantiation_all_agents(voxnav):
    """The benched simpleEnv instantiation (simple_line_kernel<4, false>: 32x32x8,
    L=4, 128-step launches, f32 reward) with 256 agents checked in full over
    2,560 steps: goal terminations (a goal-seeking episode ends every ~2k
    steps per agent under the random policy) and resets from the draw-ahead
    inside and across launches."""
    N = 256
    ends = _bench_shaped_run(N, np.arange(N, dtype=np.int64), 2560)
    assert ends["terminated"] > 0


def test_simple_bench_instantiation_full_batch_sampled(voxnav):
    """The bench's full batch (65,536 agents) in the same launches: one
    sampled agent from every 64-agent block of the kernel (position varied),
    2,560 steps."""
    N = 65536
    blocks = np.arange(N // 64, dtype=np.int64)
    sample = blocks * 64 + (blocks * 41 + 9) % 64
    ends = _bench_shaped_run(N, sample, 2560)
    assert ends["terminated"] > 0


def test_simple_word_layout_bench_shape_sampled(voxnav, monkeypatch):
    """The word-layout kernel (VOXNAV_SIMPLE_LINE=0) in the bench's launches:
    4,096 agents, one sampled per 64-agent block, 1,280 steps."""
    monkeypatch.setenv("VOXNAV_SIMPLE_LINE", "0")
    N = 4096
    blocks = np.arange(N // 64, dtype=np.int64)
    _bench_shaped_run(N, blocks * 64 + (blocks * 23 + 5) % 64, 1280, label="simple_pipe_kernel<4, false>")


def test_simple_step_actions_terminal_obs(voxnav):
    src, L, N, K = "box:8x8x4", 4, 200, 160
    env = make_env(src, L, n=N, autoreset=True)
    env.reset(seed=500)
    rng = np.random.default_rng(5)
    acts = rng.integers(0, 6, size=(K, N)).astype(np.int32)
    orc = oracle_env(src, L, n_agents=N, variant=1).run_random(500 + np.arange(N), policy_seed=0, K=K,
                                                               seed_stride=N, actions=acts, terminal_obs=True)
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
    assert ended >= N


def test_simple_sharding_and_fusion_invariance(voxnav):
    src, L, N, K = "set:P3_training", 10, 512, 96
    full = make_env(src, L, n=N, autoreset=True)
    full.reset(seed=42)
    a = full.step_random(K, policy_seed=5, t0=0)
    parts = []
    for base in (0, N // 2):
        sh = make_env(src, L, n=N // 2, autoreset=True, agent_id_base=base, seed_stride=N)
        sh.reset(seed=42)
        parts.append(sh.step_random(K, policy_seed=5, t0=0))
    assert torch.equal(torch.cat([parts[0].obs, parts[1].obs], dim=1), a.obs)
    single = make_env(src, L, n=N, autoreset=True)
    single.reset(seed=42)
    steps = [single.step_random(1, policy_seed=5, t0=k) for k in range(K)]
    assert torch.equal(torch.cat([s.obs for s in steps], 0), a.obs)
    assert torch.equal(torch.cat([s.reward for s in steps], 0), a.reward)


def test_simple_gridagent_facade_matches_golden(voxnav):
    from voxnav.gym_api import SimpleGridAgent
    d = load_golden(sorted(p for p in simple_golden_trajectories() if "kitchen2" in p.name)[0])
    ag = SimpleGridAgent(local_map_length=int(d["L"]), rooms=product_room_set(str(d["room_source"])).rooms)
    assert ag.reset(seed=int(d["seeds"][0])) is None          # the reference's reset returns None
    assert ag.get_obs().tobytes() == d["reset_obs"][0].tobytes()
    assert ag.observation_space.shape == (6 * int(d["L"]) + 7,)
    assert (ag.gx, ag.gy, ag.gz) == tuple(int(v) for v in d["reset_state"][0][3:])
    si = 1
    for t, a in enumerate(d["actions"][:200]):
        obs, r, te, tr, info = ag.step(int(a))
        assert isinstance(r, np.float64) and r == d["reward"][t]
        assert obs.tobytes() == d["obs"][t].tobytes()
        assert (ag.visited_count, ag.bump_count, ag.done) == (d["state"][t][6], d["state"][t][7], bool(d["state"][t][8]))
        if te or tr:
            ag.reset(seed=int(d["seeds"][si]))
            si += 1
    ag.close()
