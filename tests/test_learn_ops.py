"""The learner's matrix-core products (voxnav/learn_ops.py over
csrc/voxnav_gemm_f32.hip) against plain PyTorch fp32 on the same device:
the paired Linear+Tanh layers (forward and every gradient), the heads'
plain Linear, and the split-K weight-gradient product with column sums, at
the learner's minibatch size and at ragged / odd shapes.  Tolerances are
relative to each tensor's scale: f32 sums over up to 65,536 samples in a
different order."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _close(got, ref, rel=2e-5, floor=1e-6):
    err = (got - ref).abs().max().item()
    assert err <= rel * ref.abs().max().item() + floor, err


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("M,K,N,shared", [(65536 + 333, 256, 128, False), (65536, 80, 256, True), (77, 40, 6, False)])
def test_linear_tanh_pair_matches_torch(M, K, N, shared):
    from voxnav.learn_ops import linear_tanh_pair
    dev = "cuda:0"
    torch.manual_seed(M + K + N)
    la, lb = torch.nn.Linear(K, N).to(dev), torch.nn.Linear(K, N).to(dev)
    xa = torch.randn((M, K), device=dev, requires_grad=not shared)
    xb = xa if shared else torch.randn((M, K), device=dev, requires_grad=True)
    dy = torch.randn((2, M, N), device=dev)
    w = torch.stack([la.weight, lb.weight])
    b = torch.stack([la.bias, lb.bias])
    y = linear_tanh_pair(xa if shared else torch.stack([xa, xb]), w, b)
    (y * dy).sum().backward()
    got = [la.weight.grad.clone(), la.bias.grad.clone(), lb.weight.grad.clone(), lb.bias.grad.clone()]
    if not shared:
        got += [xa.grad.clone(), xb.grad.clone()]
    for p in [la.weight, la.bias, lb.weight, lb.bias, xa, xb]:
        p.grad = None
    ya, yb = torch.tanh(la(xa)), torch.tanh(lb(xb))
    ((ya * dy[0]).sum() + (yb * dy[1]).sum()).backward()
    _close(y[0], ya)
    _close(y[1], yb)
    ref = [la.weight.grad, la.bias.grad, lb.weight.grad, lb.bias.grad]
    if not shared:
        ref += [xa.grad, xb.grad]
    for g, r in zip(got, ref):
        _close(g, r)


@pytest.mark.parametrize("N", [6, 1, 130])
def test_head_linear_matches_torch(N):
    from voxnav.learn_ops import linear
    dev = "cuda:0"
    torch.manual_seed(N)
    lin = torch.nn.Linear(128, N).to(dev)
    x = torch.randn((4099, 128), device=dev, requires_grad=True)
    dy = torch.randn((4099, N), device=dev)
    y = linear(x, lin)
    (y * dy).sum().backward()
    got = [x.grad.clone(), lin.weight.grad.clone(), lin.bias.grad.clone()]
    x.grad = lin.weight.grad = lin.bias.grad = None
    y2 = lin(x)
    (y2 * dy).sum().backward()
    _close(y, y2)
    for g, r in zip(got, [x.grad, lin.weight.grad, lin.bias.grad]):
        _close(g, r)


@pytest.mark.parametrize("K,M,N,bt", [(65536, 1024, 256, 2), (65536 + 777, 1024, 80, 2), (1000, 6, 128, 1),
                                      (17, 33, 5, 1)])
def test_mm_tn_matches_torch(K, M, N, bt):
    from voxnav.learn_ops import mm_tn
    dev = "cuda:0"
    torch.manual_seed(K + M)
    a = torch.randn((bt, K, M), device=dev)
    y = 0.9 * torch.tanh(torch.randn((bt, K, M), device=dev))
    b = torch.randn((bt, K, N), device=dev)
    out, cs = mm_tn(a, b, colsum=True)
    _close(out, a.transpose(1, 2) @ b)
    _close(cs, a.sum(1))
    z = a * (1 - y * y)
    out2, cs2 = mm_tn(a, b, y=y, colsum=True)
    _close(out2, z.transpose(1, 2) @ b)
    _close(cs2, z.sum(1))
    # a batch-shared B (stride 0) and a strided batch of A
    bs = b[:1].expand(bt, K, N)
    out3, _ = mm_tn(a, bs)
    _close(out3, a.transpose(1, 2) @ bs)


@pytest.mark.parametrize("D,H,L,B", [(80, 256, 8, 512), (31, 64, 5, 300), (67, 16, 3, 70)])
def test_dual_lstm_matches_torch(D, H, L, B):
    """The learner's LSTM re-run (voxnav/lstm_seq.py over the fused per-step
    kernels of csrc/voxnav_learn_f32.hip) against two torch nn.LSTMs: outputs
    and every parameter / initial-state gradient, including input widths that
    are not multiples of 4 (simpleEnv's 6L + 7 observation, zero-padded)."""
    from types import SimpleNamespace
    from voxnav.lstm_seq import dual_lstm
    dev = "cuda:0"
    torch.manual_seed(D * H + L)
    la, lc = torch.nn.LSTM(D, H).to(dev), torch.nn.LSTM(D, H).to(dev)
    pol = SimpleNamespace(lstm_actor=la, lstm_critic=lc)
    x = torch.randn((L, B, D), device=dev)
    h0 = torch.randn((2, B, H), device=dev, requires_grad=True)
    c0 = torch.randn((2, B, H), device=dev, requires_grad=True)
    dy = torch.randn((2, L, B, H), device=dev)
    oa, oc = dual_lstm(pol, x, h0, c0)
    ((oa * dy[0]).sum() + (oc * dy[1]).sum()).backward()
    params = list(la.parameters()) + list(lc.parameters())
    got = [p.grad.clone() for p in params] + [h0.grad.clone(), c0.grad.clone()]
    for p in params + [h0, c0]:
        p.grad = None
    ra, _ = la(x, (h0[0:1], c0[0:1]))
    rc, _ = lc(x, (h0[1:2], c0[1:2]))
    ((ra * dy[0]).sum() + (rc * dy[1]).sum()).backward()
    _close(oa, ra)
    _close(oc, rc)
    ref = [p.grad for p in params] + [h0.grad, c0.grad]
    for g, r in zip(got, ref):
        _close(g, r, rel=1e-4)
