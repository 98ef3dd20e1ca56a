"""CPU checks of the collector oracle (oracle/collector_oracle.py).

SB3 / sb3_contrib are not installed and not vendored, so
the collector's float semantics are "parity unpinned" by the reference;
the oracle is pinned here against the plain-PyTorch f32 policy module
(voxnav.policy, which mirrors SB3's layer structure) and against
hand-computed known answers.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import collector_oracle as co  # noqa: E402
from oracle.oracle import gae as gae32  # noqa: E402


def _policies():
    from voxnav.policy import ActorCriticPolicy, RecurrentActorCriticPolicy
    torch.manual_seed(0)
    return [RecurrentActorCriticPolicy(), ActorCriticPolicy()]


@pytest.mark.parametrize("kind", [0, 1], ids=["lstm", "mlp"])
def test_policy_oracle_matches_torch_fp32(kind):
    from voxnav.policy import numpy_weights
    pol = _policies()[kind]
    rng = np.random.default_rng(1)
    N = 32
    obs = rng.random((N, 80)).astype(np.float32)
    orc = co.PolicyOracle(numpy_weights(pol))
    if pol.recurrent:
        h = rng.standard_normal((2, N, 256)).astype(np.float32) * 0.3
        c = rng.standard_normal((2, N, 256)).astype(np.float32) * 0.3
        starts = (rng.random(N) < 0.3).astype(np.float32)
        lg, v, h2, c2 = pol.forward_torch(torch.from_numpy(obs), torch.from_numpy(h), torch.from_numpy(c),
                                          torch.from_numpy(starts))
        olg, ov, oh, oc = orc.forward(obs, h.astype(np.float64), c.astype(np.float64), starts)
        np.testing.assert_allclose(h2.numpy(), oh, atol=2e-6)
        np.testing.assert_allclose(c2.numpy(), oc, atol=2e-6)
    else:
        lg, v = pol.forward_torch(torch.from_numpy(obs))
        olg, ov, _, _ = orc.forward(obs)
    np.testing.assert_allclose(lg.numpy(), olg, atol=2e-6)
    np.testing.assert_allclose(v.numpy(), ov, atol=2e-6)


def test_sb3_init_gains():
    pol = _policies()[0]
    w = pol.action_net.weight.detach().double()
    # orthogonal rows scaled by 0.01 (action_net), zero biases
    np.testing.assert_allclose((w @ w.T).numpy(), 1e-4 * np.eye(6), atol=1e-9)
    assert float(pol.value_net.bias.detach().abs().max()) == 0.0
    w1 = pol.mlp_extractor.policy_net[0].weight.detach().double()   # 256x256, gain sqrt(2)
    np.testing.assert_allclose((w1 @ w1.T).numpy(), 2.0 * np.eye(256), atol=1e-5)


def test_categorical_draw_frequencies():
    lsm = co.log_softmax(np.array([[0.0, 1.0, -1.0, 0.5, 0.2, -2.0]]))[0]
    p = np.exp(lsm)
    n = 20000
    counts = np.zeros(6)
    for i in range(n):
        a, _ = co.categorical_draw(lsm, co.sample_uniform(42, i, 7))
        counts[a] += 1
    # 5 sigma of a binomial
    assert np.all(np.abs(counts / n - p) < 5 * np.sqrt(p * (1 - p) / n))


def test_sample_uniform_known_properties():
    u = [co.sample_uniform(42, g, t) for g in range(4) for t in range(4)]
    assert all(0.0 <= x < 1.0 for x in u)
    assert len(set(u)) == 16
    assert co.sample_uniform(42, 3, 5) == co.sample_uniform(42, 3, 5)
    assert co.sample_uniform(42, 3, 5) != co.sample_uniform(43, 3, 5)


def test_gae64_known_answer_and_f32_restatement():
    # two steps, one env, no episode boundary: hand-computed
    r = np.array([[1.0], [2.0]])
    v = np.array([[0.5], [0.25]])
    lv = np.array([0.75])
    g, lam = 0.9, 0.8
    d1 = 2.0 + g * 0.75 - 0.25
    d0 = 1.0 + g * 0.25 - 0.5
    adv, ret = co.gae64(r, v, np.zeros((2, 1)), lv, np.zeros(1), g, lam)
    np.testing.assert_allclose(adv[:, 0], [d0 + g * lam * d1, d1])
    np.testing.assert_allclose(ret, adv + v)
    rng = np.random.default_rng(3)
    T, N = 40, 16
    r, v = rng.standard_normal((T, N)), rng.standard_normal((T, N))
    s = (rng.random((T, N)) < 0.1).astype(np.float64)
    lv, dn = rng.standard_normal(N), (rng.random(N) < 0.5).astype(np.float64)
    a64, r64 = co.gae64(r, v, s, lv, dn)
    a32, r32 = gae32(r, v, s, lv, dn)
    np.testing.assert_allclose(a32, a64, atol=1e-4)
    np.testing.assert_allclose(r32, r64, atol=1e-4)
