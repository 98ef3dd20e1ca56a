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


def _rows_reference(x, env, start, keep, hs, cs, lstm, l):
    """float64 restatement of one LSTM over the row layout: at a sequence start
    the state is the buffer's stored state x keep, else the row's previous."""
    L, B, _ = x.shape
    w_ih, w_hh = lstm.weight_ih_l0.double(), lstm.weight_hh_l0.double()
    b = (lstm.bias_ih_l0 + lstm.bias_hh_l0).double()
    h = torch.zeros((B, w_hh.shape[1]), dtype=torch.float64, device=x.device)
    c = torch.zeros_like(h)
    outs = []
    for t in range(L):
        st = start[t].bool().view(B, 1)
        k = keep[t].double().view(B, 1)
        h = torch.where(st, hs[t, l, env[t].long()].double() * k, h)
        c = torch.where(st, cs[t, l, env[t].long()].double() * k, c)
        gi, gf, gg, go = (x[t].double() @ w_ih.T + h @ w_hh.T + b).chunk(4, dim=1)
        c = torch.sigmoid(gf) * c + torch.sigmoid(gi) * torch.tanh(gg)
        h = torch.sigmoid(go) * torch.tanh(c)
        outs.append(h)
    return torch.stack(outs)


@pytest.mark.parametrize("layout", ["auto", "units16", "units32"])
@pytest.mark.parametrize("L,B,N,p_start", [(24, 512, 600, 0.03), (9, 37, 40, 0.2), (128, 64, 64, 0.01),
                                           (128, 512, 512, 0.004), (1, 1, 4, 0.5), (2, 33, 8, 0.5),
                                           (5, 289, 300, 1.0)])
def test_dual_lstm_rows_matches_float64(L, B, N, p_start, layout, monkeypatch):
    """The persistent row-layout LSTM (csrc/voxnav_learn_rows.hip: weights
    resident, in-launch h / partial-dh hand-offs between the unit blocks of a
    row tile) against a float64 restatement: outputs and the weight / bias
    gradients of both LSTMs, with sequence starts (stored states x keep) at t = 0,
    at random steps and mid-row; full 512-row tiles, a ragged last tile, a
    whole 128-step rollout, and the learner bench's own shape (512 rows x 128
    steps: every block of the launch resident, 128 hand-offs per direction);
    edge shapes: one step of one row, two steps of a 33-row batch (one full
    tile and a 1-row tile), and a batch where every row starts a sequence at
    every step (no state crosses a step: only the stored states).
    Both layouts, forced: 16 unit blocks of 16 units (VOXNAV_ROWS_V2=1; two
    blocks per CU at 512 rows) and 8 of 32 (VOXNAV_ROWS_V1=1), and the
    default pick per direction."""
    from types import SimpleNamespace
    from voxnav import lstm_seq
    monkeypatch.delenv("VOXNAV_ROWS_V1", raising=False)
    monkeypatch.delenv("VOXNAV_ROWS_V2", raising=False)
    if layout == "units32":
        monkeypatch.setenv("VOXNAV_ROWS_V1", "1")
    elif layout == "units16":
        monkeypatch.setenv("VOXNAV_ROWS_V2", "1")
    dev = "cuda:0"
    D, H = 80, 256
    torch.manual_seed(L * B + N)
    la, lc = torch.nn.LSTM(D, H).to(dev), torch.nn.LSTM(D, H).to(dev)
    pol = SimpleNamespace(lstm_actor=la, lstm_critic=lc)
    if not lstm_seq.rows_supported(pol, D, B):
        pytest.skip("row-layout kernels not co-resident on this device")
    x = torch.randn((L, B, D), device=dev)
    env = torch.randint(0, N, (L, B), device=dev, dtype=torch.int32)
    start = (torch.rand((L, B), device=dev) < p_start).to(torch.uint8)
    start[0] = 1
    keep = (torch.rand((L, B), device=dev) > 0.3).float()
    hs = 0.5 * torch.randn((L, 2, N, H), device=dev)
    cs = 0.5 * torch.randn((L, 2, N, H), device=dev)
    dy = torch.randn((2, L, B, H), device=dev)
    oa, oc = lstm_seq.dual_lstm_rows(pol, x, env, start, keep, hs, cs)
    ((oa * dy[0]).sum() + (oc * dy[1]).sum()).backward()
    params = list(la.parameters()) + list(lc.parameters())
    got = [p.grad.clone() for p in params]
    lstm_seq.rows_check(torch.device(dev))
    for p in params:
        p.grad = None
    ra = _rows_reference(x, env, start, keep, hs, cs, la, 0)
    rc = _rows_reference(x, env, start, keep, hs, cs, lc, 1)
    ((ra * dy[0].double()).sum() + (rc * dy[1].double()).sum()).backward()
    _close(oa, ra.float())
    _close(oc, rc.float())
    for g, p in zip(got, params):
        _close(g, p.grad, rel=1e-4)


def _ppo_loss_reference(h, wa, ba, wv, bv, act, adv, olp, ret, clip, ent_coef, vf_coef, norm):
    """sb3's heads + losses in float64 with autograd (RecurrentPPO.train /
    PPO.train, the block after evaluate_actions)."""
    h = h.detach().double().requires_grad_(True)
    P = [t.detach().double().requires_grad_(True) for t in (wa, ba, wv, bv)]
    logits = h[0] @ P[0].T + P[1]
    values = (h[1] @ P[2].T + P[3]).flatten()
    lp_all = torch.log_softmax(logits, -1)
    lp = lp_all.gather(1, act.long().view(-1, 1)).flatten()
    ent = -(lp_all.exp() * lp_all).sum(-1)
    adv = adv.double()
    if norm:
        adv = (adv - adv.mean()) / (adv.std() + 1e-8)
    ratio = torch.exp(lp - olp.double())
    pl = -torch.min(adv * ratio, adv * torch.clamp(ratio, 1 - clip, 1 + clip)).mean()
    vl = torch.nn.functional.mse_loss(ret.double(), values)
    el = -ent.mean()
    loss = pl + ent_coef * el + vf_coef * vl
    loss.backward()
    lr = lp - olp.double()
    stats = torch.stack([pl, vl, el, loss, ((torch.exp(lr) - 1) - lr).mean(),
                         ((ratio - 1).abs() > clip).double().mean()]).detach()
    return h.grad, [p.grad for p in P], stats


@pytest.mark.parametrize("M,F,A,gather,norm", [(65536, 128, 6, True, True), (77, 64, 3, False, True),
                                               (4099, 256, 8, True, False), (1, 128, 6, False, False)])
def test_ppo_loss_matches_float64(M, F, A, gather, norm):
    """The fused loss kernel (heads, advantage normalisation, clipped
    surrogate, value MSE, entropy; gradient to the latents and the head
    weights) against the same block in float64 autograd.  Old log-probs are
    spread so the ratio falls on both sides of the clip range and inside it
    (the min's tie, where torch splits the gradient)."""
    from voxnav.learn_ops import ppo_loss
    dev = "cuda:0"
    torch.manual_seed(M + F + A)
    an, vn = torch.nn.Linear(F, A).to(dev), torch.nn.Linear(F, 1).to(dev)
    h = torch.tanh(torch.randn((2, M, F), device=dev))
    R = M + 1000 if gather else M
    src = torch.randperm(R, device=dev)[:M].contiguous() if gather else None
    act = torch.randint(0, A, (R,), device=dev, dtype=torch.int32)
    adv = torch.randn(R, device=dev) * 3 + 0.5
    ret = torch.randn(R, device=dev)
    with torch.no_grad():
        lp_true = torch.log_softmax(h[0] @ an.weight.T + an.bias, -1)
    sel = src if gather else torch.arange(M, device=dev)
    olp = torch.randn(R, device=dev) - 1.5
    olp[sel] = lp_true.gather(1, act[sel].long().view(-1, 1)).flatten() + 0.3 * torch.randn(M, device=dev)
    clip, ent, vf = 0.2, 0.01, 0.5
    dh, grads, stats = ppo_loss(h, an, vn, src, act, adv, olp, ret, clip, ent, vf, norm)
    g = lambda t: t if src is None else t[src]  # noqa: E731
    rdh, rgrads, rstats = _ppo_loss_reference(h, an.weight, an.bias, vn.weight, vn.bias, g(act), g(adv), g(olp),
                                              g(ret), clip, ent, vf, norm)
    if M == 1 and norm:
        return
    _close(dh.double(), rdh, rel=2e-5, floor=1e-9)
    for a, b in zip(grads, rgrads):
        assert a.shape == b.shape
        _close(a.double(), b, rel=1e-4, floor=1e-9)
    _close(stats, rstats, rel=1e-5, floor=1e-7)


def test_grad_norm_scale_matches_clip_grad_norm():
    """The two-launch gradient norm (and the Adam grad_scale divisor) against
    torch.nn.utils.clip_grad_norm_ over tensors of ragged sizes and offsets;
    and the fused Adam step with that divisor against clip + step."""
    from voxnav.learn_ops import grad_norm_scale
    dev = "cuda:0"
    torch.manual_seed(3)
    shapes = [(1024, 256), (1024, 80), (1024,), (6, 128), (6,), (1, 128), (1,), (333, 7)]
    ps = [torch.nn.Parameter(torch.randn(s, device=dev)) for s in shapes]
    for p in ps:
        p.grad = torch.randn_like(p) * 0.05
    ref_ps = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    for r, p in zip(ref_ps, ps):
        r.grad = p.grad.clone()
    for max_norm in (0.5, 1e3):
        norm, scale = grad_norm_scale(ps, max_norm)
        ref = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(p.grad.double()) for p in ps])).float()
        _close(norm, ref, rel=1e-6)
        assert abs(scale.item() - max(1.0, (ref.item() + 1e-6) / max_norm)) <= 1e-6 * scale.item()
    opt = torch.optim.Adam(ps, lr=3e-4, eps=1e-5, fused=True)
    ref_opt = torch.optim.Adam(ref_ps, lr=3e-4, eps=1e-5, fused=True)
    norm, scale = grad_norm_scale(ps, 0.5)
    opt.grad_scale = scale
    opt.step()
    torch.nn.utils.clip_grad_norm_(ref_ps, 0.5)
    ref_opt.step()
    for p, r in zip(ps, ref_ps):
        _close(p.detach(), r.detach(), rel=1e-6, floor=1e-7)



def test_adam_step_matches_torch_fused_adam():
    """The library's Adam step (clip divisor applied on the way) against
    torch's fused Adam with the same grad_scale, over three steps from a
    fresh state, including a tensor whose size is not a multiple of 4; the
    optimizer state (step, moments) is torch's own."""
    from voxnav.learn_ops import adam_step, grad_norm_scale
    dev = "cuda:0"
    torch.manual_seed(5)
    shapes = [(1024, 336), (6, 128), (6,), (333, 7), (1,)]
    ps = [torch.nn.Parameter(torch.randn(s, device=dev)) for s in shapes]
    rs = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    opt = torch.optim.Adam(ps, lr=3e-4, eps=1e-5, fused=True)
    ref = torch.optim.Adam(rs, lr=3e-4, eps=1e-5, fused=True)
    for it in range(3):
        for p, r in zip(ps, rs):
            g = torch.randn_like(p) * 0.3
            p.grad, r.grad = g.clone(), g.clone()
        _, scale = grad_norm_scale(ps, 0.5)
        adam_step(opt, scale)
        ref.grad_scale = scale.clone()
        ref.step()
        ref.grad_scale = None
        for p, r in zip(ps, rs):
            _close(p.detach(), r.detach(), rel=1e-6, floor=1e-7)
            for k in ("exp_avg", "exp_avg_sq"):
                _close(opt.state[p][k], ref.state[r][k], rel=1e-5, floor=1e-12)
            assert float(opt.state[p]["step"]) == float(ref.state[r]["step"]) == it + 1


def test_minibatch_rows_matches_index_arithmetic():
    """The one-launch minibatch gather against the torch index arithmetic it
    replaces (env-major ids -> [T, N]-major rows), ragged M."""
    from voxnav.learn_ops import minibatch_rows
    dev = "cuda:0"
    T, N, D = 128, 1000, 80
    obs = torch.randn((T, N, D), device=dev)
    idx = torch.randperm(T * N, device=dev)[:4099].contiguous()
    src, rows = minibatch_rows(idx, T, N, obs)
    env = idx // T
    ref = (idx - env * T) * N + env
    assert torch.equal(src, ref)
    assert torch.equal(rows, obs.reshape(T * N, D)[ref])
