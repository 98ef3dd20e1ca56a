"""Full-episode parity of the benched kernel instantiations at the headline
room (32x32x8 box, L=10) -- every agent crosses the 5,400-step truncation
and the SB3 auto-reset (plane clear at full u32 row width, wall-image
re-copy), against the CPU oracle (oracle/voxnav_oracle.c, pinned to the
reference's golden trajectories by tests/test_oracle_golden.py).

* the bench's call: ``step_random(out=...)`` in F=16 and F=128 (the bench
  default) launches, f32 reward, no action record ->
  ``env_kernel<8, false, true, false, 2>``;
* the collector's call: ``step_into`` with explicit actions, f32 reward,
  one step per launch -> ``env_kernel<8, true, true, false, 2>``;
* the full BASELINE batch (65,536 agents) with one sampled agent from every
  64-agent block, through a whole episode (also as C5's last shard);
* BASELINE C2 at its size (4,096 agents, 16x16x8, L=10) through its
  1,176-step truncation and auto-reset.

Bar: obs bytes, f32 reward (the oracle's f64 reward rounded), terminated /
truncated flags bit-exact at every step; exported belief maps equal the
oracle's (visit counts saturating at 63) at three points of the episode.
"""
import numpy as np
import pytest

from helpers import oracle_env, product_room_set

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

SRC, L = "box:32x32x8", 10
EPISODE = 5400                 # total_free_cells of the 32x32x8 box
K_TOTAL = 5504                 # 344 launches of 16: the truncation at 5,400 and 104 steps of the next episode
BELIEF_AT = (2000, 5408, K_TOTAL)


@pytest.fixture(scope="module")
def voxnav():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import voxnav
    voxnav.load_library()
    return voxnav


def make_env(n, **kw):
    from voxnav.env import BatchedGridEnv
    return BatchedGridEnv(num_agents=n, rooms=product_room_set(SRC), local_map_length=L, autoreset=True,
                          device="cuda:0", **kw)


def check_beliefs(env, orc_env, sample, step):
    b = env.belief()
    b = b.index_select(0, torch.as_tensor(sample, device=b.device)).cpu().numpy().astype(np.int64)
    for j in range(len(sample)):
        ref = np.minimum(orc_env.belief(j), 63)
        W, D, H = ref.shape
        np.testing.assert_array_equal(b[j, :W, :D, :H], ref, err_msg=f"belief of agent {sample[j]} at step {step}")


def run_random_episode(env, N, sample, F=16, gid_base=0, seed_stride=None, src=SRC, k_total=K_TOTAL,
                       belief_at=BELIEF_AT, L=L):
    """Bench-shaped launches; compare the sampled agents launch by launch.
    ``sample`` are local agent indices; the shard's global ids start at
    ``gid_base`` and its seeds advance by ``seed_stride`` (the global count)."""
    seed_stride = N if seed_stride is None else seed_stride
    from voxnav.env import Rollout
    dev = env.device
    out = Rollout(torch.empty((F, N, 80), dtype=torch.float32, device=dev),
                  torch.empty((F, N), dtype=torch.float32, device=dev),
                  torch.empty((F, N), dtype=torch.uint8, device=dev),
                  torch.empty((F, N), dtype=torch.uint8, device=dev), None)
    # (", true": the deferred-flush instantiation, VOXNAV_ENV_DFLUSH bit 1)
    assert env.kernel_label(F) in ("env_kernel<8, false, true, false, 2>", "env_kernel<8, false, true, false, 2, true>")
    idx = torch.as_tensor(sample, device=dev)
    orc_env = oracle_env(src, L, n_agents=len(sample))
    gids = gid_base + np.asarray(sample, dtype=np.int64)
    seeds = 42 + gids
    env.reset(seed=42)
    t = 0
    truncations = 0
    while t < k_total:
        k = min(F, k_total - t)
        env.step_random(k, policy_seed=42, t0=t,
                        out=Rollout(out.obs[:k], out.reward[:k], out.terminated[:k], out.truncated[:k], None))
        orc = orc_env.run_random(seeds, policy_seed=42, K=k, t0=t, seed_stride=seed_stride,
                                 initial_reset=(t == 0), gids=gids, threads=8)
        obs = out.obs[:k].index_select(1, idx).cpu().numpy()
        if obs.tobytes() != orc["obs"].tobytes():
            bad = np.argwhere((obs.view(np.uint32) != orc["obs"].view(np.uint32)).any(-1))
            raise AssertionError(f"obs mismatch at (step, sampled agent) {(bad[:5] + [t, 0]).tolist()}")
        np.testing.assert_array_equal(out.reward[:k].index_select(1, idx).cpu().numpy(),
                                      orc["reward"].astype(np.float32), err_msg=f"reward, steps {t}..{t + k}")
        np.testing.assert_array_equal(out.terminated[:k].index_select(1, idx).cpu().numpy(), orc["terminated"])
        tr = out.truncated[:k].index_select(1, idx).cpu().numpy()
        np.testing.assert_array_equal(tr, orc["truncated"])
        truncations += int(tr.sum())
        t += k
        if t in belief_at:
            check_beliefs(env, orc_env, sample, t)
    return truncations


def test_bench_kernel_full_episode_matches_oracle(voxnav):
    """The benched instantiation, 256 agents, 5,504 steps: every agent's
    5,400-step episode truncates and auto-resets inside the run."""
    N = 256
    env = make_env(N)
    tr = run_random_episode(env, N, np.arange(N, dtype=np.int64))
    assert tr == N        # each agent truncated exactly once, at step 5,400
    env.close()


def test_full_batch_sampled_blocks_full_episode(voxnav):
    """65,536 agents (the headline batch): one agent from every 64-agent
    block (each block of the kernel), position varied, through the whole
    episode and the auto-reset."""
    N = 65536
    blocks = np.arange(N // 64, dtype=np.int64)
    sample = blocks * 64 + (blocks * 37 + 11) % 64
    env = make_env(N)
    tr = run_random_episode(env, N, sample)
    assert tr == len(sample)
    env.close()


def test_c5_last_shard_env_full_episode_at_bench_launch_size(voxnav):
    """The env half of BASELINE C5's last shard (rank 7 of 8: global ids
    458,752..524,287, seeds advancing by 524,288 per episode) under the
    random policy on the headline box, in the bench's 128-step launches,
    one sampled agent from every 64-agent block through the whole episode
    and the auto-reset.  (The PPO-LSTM collector of the same shard on
    P3_training: tests/test_collector_gpu.py, case lstm-f32-P3_training-C5shard.)"""
    N, WORLD, RANK = 65536, 8, 7
    blocks = np.arange(N // 64, dtype=np.int64)
    sample = blocks * 64 + (blocks * 29 + 5) % 64
    env = make_env(N, agent_id_base=RANK * N, seed_stride=WORLD * N)
    tr = run_random_episode(env, N, sample, F=128, gid_base=RANK * N, seed_stride=WORLD * N)
    assert tr == len(sample)
    env.close()


C2_SRC, C2_EPISODE = "box:16x16x8", 1176   # BASELINE C2: 4,096 agents, one 16x16x8 room (1,176 free cells)


def test_c2_config_through_truncation_and_autoreset(voxnav):
    """BASELINE config C2 at its size: 4,096 agents, 16x16x8 box, L=10,
    random policy, in the bench's 128-step launches for 1,280 steps -- every
    agent's 1,176-step episode truncates and auto-resets inside the window.
    256 sampled agents (every 16th, offset varied) step-by-step bit-exact,
    belief maps of the sample at steps 640 and 1,280 (the truncation at
    1,176 falls inside the tenth launch, 1,152 + 24)."""
    from voxnav.env import BatchedGridEnv
    N = 4096
    env = BatchedGridEnv(num_agents=N, rooms=product_room_set(C2_SRC), local_map_length=10, autoreset=True,
                         device="cuda:0")
    blocks = np.arange(N // 16, dtype=np.int64)
    sample = blocks * 16 + (blocks * 7 + 3) % 16
    tr = run_random_episode(env, N, sample, F=128, src=C2_SRC, k_total=1280, belief_at=(640, 1280))
    assert tr == len(sample)          # each sampled agent truncated exactly once, at step 1,176
    env.close()


def test_step_into_full_episode_matches_oracle(voxnav):
    """The collector's call (explicit actions, one step per launch, f32
    reward, terminal_obs) over a whole 32x32x8 episode and its auto-reset."""
    N, K, CH = 128, 5410, 541
    env = make_env(N)
    dev = env.device
    assert env.kernel_label(1, explicit_actions=True) == "env_kernel<8, true, true, false, 2>"
    acts = np.random.default_rng(17).integers(0, 6, size=(K, N)).astype(np.int32)
    at = torch.as_tensor(acts, device=dev)
    obs = torch.empty((CH, N, 80), dtype=torch.float32, device=dev)
    rew = torch.empty((CH, N), dtype=torch.float32, device=dev)
    te = torch.empty((CH, N), dtype=torch.uint8, device=dev)
    tr = torch.empty((CH, N), dtype=torch.uint8, device=dev)
    tob = torch.zeros((CH, N, 80), dtype=torch.float32, device=dev)
    orc_env = oracle_env(SRC, L, n_agents=N)
    seeds = 42 + np.arange(N, dtype=np.int64)
    env.reset(seed=42)
    ended = 0
    for c0 in range(0, K, CH):
        for j in range(CH):
            env.step_into(at[c0 + j], obs[j], rew[j], te[j], tr[j], tob[j])
        orc = orc_env.run_random(seeds, policy_seed=0, K=CH, t0=c0, seed_stride=N, initial_reset=(c0 == 0),
                                 actions=acts[c0:c0 + CH], terminal_obs=True, threads=8)
        assert obs.cpu().numpy().tobytes() == orc["obs"].tobytes(), f"obs, steps {c0}..{c0 + CH}"
        np.testing.assert_array_equal(rew.cpu().numpy(), orc["reward"].astype(np.float32))
        np.testing.assert_array_equal(te.cpu().numpy(), orc["terminated"])
        trn = tr.cpu().numpy()
        np.testing.assert_array_equal(trn, orc["truncated"])
        done = (te.cpu().numpy() | trn).astype(bool)
        ended += int(done.sum())
        np.testing.assert_array_equal(tob.cpu().numpy()[done], orc["terminal_obs"][done])
    assert ended == N
    check_beliefs(env, orc_env, np.arange(N), K)
    env.close()
