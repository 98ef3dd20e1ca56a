"""Pin the CPU oracle against golden vectors from the unmodified reference.

The goldens (tests/golden/*.npz) were produced by tests/golden/gen_golden.py
running envs/CubicEnv.py itself.  If these pass, the oracle is a faithful
restatement of the reference on: every room file's parse, the reset draws
(CPython MT19937 room/start choice) for thousands of seeds, and per-step
state / obs bits / f64 reward / belief map over random-policy and
explorer-policy trajectories in boxes, real rooms and room sets.
"""
import random

import numpy as np
import pytest

from helpers import (GOLDEN, STATE13, archive_texts, golden_trajectories, grid_hash, load_golden, oracle_env,
                     simple_golden_trajectories,
                     set_members)
from oracle import oracle as O


def test_mt_matches_cpython_random():
    for s in [0, 1, 42, 4242, 2 ** 31 - 1, 2 ** 32 - 1, 2 ** 32 + 17, -9, 10 ** 15]:
        random.seed(s)
        ref = [random.getrandbits(32) for _ in range(1300)]   # crosses two twists
        assert list(O.mt_outputs(s, 1300)) == ref, s


def test_philox_known_answers():
    # Random123 kat_vectors for philox4x32_10
    assert [int(v) for v in O.philox4x32_10([0, 0, 0, 0], [0, 0])] == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c,
                                                                          0x9b00dbd8]
    assert [int(v) for v in O.philox4x32_10([0xffffffff] * 4, [0xffffffff] * 2)] == [0x408f276d, 0x41c83b0e,
                                                                                      0xa20bc7c6, 0x6d5451fd]
    assert [int(v) for v in O.philox4x32_10([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344],
                                            [0xa4093822, 0x299f31d0])] == [0xd16cfe09, 0x94fdcceb, 0x5001e420,
                                                                          0x24126ea1]


def test_random_action_range_and_uniformity():
    acts = np.array([O.random_action(42, g, t) for g in range(64) for t in range(200)])
    assert acts.min() == 0 and acts.max() == 5
    counts = np.bincount(acts, minlength=6)
    assert counts.min() > 0.8 * len(acts) / 6


def test_room_parse_matches_reference():
    z = load_golden(GOLDEN / "rooms_parsed.npz")
    texts = archive_texts()
    assert len(z["names"]) == 65
    for name, whd, tf, h, bf in zip(z["names"], z["whd"], z["total_free"], z["grid_hash"], z["boundary_free"]):
        r = O.parse_room_text(texts[str(name)], str(name))
        assert r.whd == tuple(int(v) for v in whd), name
        assert grid_hash(r.grid) == int(h), name
        assert r.interior_free()[0] == int(tf), name
        bnd = np.ones(r.grid.shape, bool)
        bnd[1:-1, 1:-1, 1:-1] = False
        assert int(((r.grid != -2) & bnd).sum()) == int(bf), name


def test_room_parse_quirks():
    # negative layer index wraps like numpy; layer 2 of kitchen2 is never written
    r = O.parse_room_text(archive_texts()["P3_training/kitchen2.txt"])
    assert (r.grid[:, :, 2] == 0).all()
    with pytest.raises(ValueError):
        O.parse_room_text("Size=3,3,3\nLayer z=0\n2 2\n")
    with pytest.raises(IndexError):
        O.parse_room_text("Size=2,1,3\nLayer z=0\n2 2\n2 2\n")


@pytest.mark.parametrize("tag", ["P1_training", "P2_training", "P3_training", "P2_evaluate", "box32x32x8"])
def test_reset_draws_match_reference(tag):
    z = load_golden(GOLDEN / f"reset_table_{tag}.npz")
    if tag.startswith("box"):
        env = oracle_env("ctor:32x32x8", 10)
    else:
        env = oracle_env(f"set:{tag}", 10)
        assert [n for n, _ in set_members(tag)] == [str(v) for v in z["room_names"]]
    for s, row in zip(z["seeds"], z["draws"]):
        room, xyz, _ = env.reset_draw(int(s))
        assert (room, *xyz) == tuple(int(v) for v in row), (tag, int(s))


def replay_oracle(d, env):
    """Replay a golden trajectory through the oracle; assert bit-exactness."""
    seeds = list(d["seeds"])
    si = 0
    obs = env.reset(0, int(seeds[si]))
    si += 1
    assert obs.tobytes() == d["reset_obs"][0].tobytes()
    st = env.state(0)
    assert [st[f] for f in STATE13] == list(d["reset_state"][0])
    ri = 1
    dumps = {int(t): i for i, t in enumerate(d["dump_at"])}
    for t, a in enumerate(d["actions"]):
        obs, r, te, tr = env.step(0, int(a))
        assert obs.tobytes() == d["obs"][t].tobytes(), f"obs mismatch at step {t}"
        assert r == float(d["reward"][t]), f"reward mismatch at step {t}: {r!r} vs {d['reward'][t]!r}"
        assert (te, tr) == (bool(d["terminated"][t]), bool(d["truncated"][t])), t
        st = env.state(0)
        assert [st[f] for f in STATE13] == list(d["state"][t]), f"state mismatch at step {t}"
        assert grid_hash(env.belief(0)) == int(d["belief_hash"][t]), f"belief mismatch at step {t}"
        if t in dumps:
            assert (env.belief(0) == d[f"belief_dump_{dumps[t]}"]).all()
        if te or tr:
            obs = env.reset(0, int(seeds[si]))
            si += 1
            assert obs.tobytes() == d["reset_obs"][ri].tobytes()
            st = env.state(0)
            assert [st[f] for f in STATE13] == list(d["reset_state"][ri])
            ri += 1
    assert si == len(seeds)


@pytest.mark.parametrize("path", golden_trajectories(), ids=lambda p: p.stem)
def test_oracle_replays_golden_trajectory(path):
    d = load_golden(path)
    env = oracle_env(str(d["room_source"]), int(d["L"]), crash_penalty=float(d["crash_penalty"]))
    replay_oracle(d, env)


def test_goldens_cover_the_edge_cases():
    """The fixture set must exercise termination, truncation, bumps, resets."""
    term = trunc = bumps = resets = 0
    for p in golden_trajectories():
        d = load_golden(p)
        term += int(d["terminated"].sum())
        trunc += int(d["truncated"].sum())
        bumps += int(d["state"][:, 7].max())
        resets += len(d["reset_at"]) - 1
    assert term >= 2 and trunc >= 2 and bumps > 50 and resets >= 4


def test_oracle_gae_known_answer():
    # hand-computed 3-step, 2-env case (gamma=0.5, lambda=0.5)
    r = np.array([[1, 0], [0, 1], [1, 1]], np.float32)
    v = np.array([[0.5, 0], [0.25, 0.5], [0, 1]], np.float32)
    s = np.array([[1, 1], [0, 1], [0, 0]], np.float32)
    lv = np.array([2.0, 0.0], np.float32)
    dn = np.array([0.0, 1.0], np.float32)
    adv, ret = O.gae(r, v, s, lv, dn, gamma=0.5, gae_lambda=0.5)
    # env0: t2: d=1+0.5*2-0=2 A=2; t1: d=0+0.5*0-0.25=-0.25 A=-0.25+0.25*2=0.25;
    #        t0: d=1+0.5*0.25-0.5=0.625 A=0.625+0.25*0.25=0.6875
    # env1: t2: done -> d=1-1=0 A=0; t1: start[2]=0 -> d=1+0.5*1-0.5=1 A=1; t0: start[1]=1 -> d=0-0=0 A=0
    np.testing.assert_array_equal(adv[:, 0], np.array([0.6875, 0.25, 2.0], np.float32))
    np.testing.assert_array_equal(adv[:, 1], np.array([0.0, 1.0, 0.0], np.float32))
    np.testing.assert_array_equal(ret, adv + v)


SIMPLE_STATE = ("x", "y", "z", "facing", "last_action", "step_count", "visited_count", "bump_count", "done")


def simple_state_row(env, agent=0):
    st = env.state(agent)
    return [st[f] for f in SIMPLE_STATE]


def simple_reset_row(env, agent=0):
    st = env.state(agent)
    # for the simpleEnv variant, state fields 9..11 hold the goal (gx, gy, gz)
    return [st["x"], st["y"], st["z"], st["last_bump"], st["near_wall"], st["was_near_wall"]]


def replay_simple_oracle(d, env):
    """Replay a golden simpleEnv trajectory (envs/simpleEnv.py, reset seeded
    with random.seed(seed) then get_obs(), as tests/golden/gen_golden.py ran it)."""
    seeds = list(d["seeds"])
    si = 0
    obs = env.reset(0, int(seeds[si]))
    si += 1
    assert obs.tobytes() == d["reset_obs"][0].tobytes()
    assert simple_reset_row(env) == list(d["reset_state"][0])
    ri = 1
    for t, a in enumerate(d["actions"]):
        obs, r, te, tr = env.step(0, int(a))
        assert obs.tobytes() == d["obs"][t].tobytes(), f"obs mismatch at step {t}"
        assert r == float(d["reward"][t]), f"reward mismatch at step {t}: {r!r} vs {d['reward'][t]!r}"
        assert (te, tr) == (bool(d["terminated"][t]), bool(d["truncated"][t])), t
        assert simple_state_row(env) == list(d["state"][t]), f"state mismatch at step {t}"
        assert grid_hash(env.belief(0)) == int(d["belief_hash"][t]), f"belief mismatch at step {t}"
        if te or tr:
            obs = env.reset(0, int(seeds[si]))
            si += 1
            assert obs.tobytes() == d["reset_obs"][ri].tobytes()
            assert simple_reset_row(env) == list(d["reset_state"][ri])
            ri += 1
    assert si == len(seeds)


@pytest.mark.parametrize("path", simple_golden_trajectories(), ids=lambda p: p.stem)
def test_oracle_replays_simple_golden(path):
    d = load_golden(path)
    env = oracle_env(str(d["room_source"]), int(d["L"]), variant=1)
    assert env.obs_dim == 6 * int(d["L"]) + 7
    replay_simple_oracle(d, env)
    # the room the golden ran in is the one the oracle parsed (raw tokens, walls == 2)
    st = env.state(0)
    assert grid_hash(env.rooms[st["room"]].tokens) in {int(h) for h in d["room_hash"]}
