"""Split-K weight gradients of the learner (voxnav/splitk.py) against plain
products: mm_tn on CPU (the chunking arithmetic, including a ragged last
chunk), and on the GPU the split-K Linear's gradients against nn.Linear's
own autograd at the learner's minibatch size."""
import pytest
import torch

from voxnav import splitk


@pytest.mark.parametrize("K", [100, 8192, 65536, 65536 + 777])
def test_mm_tn_matches_plain_product_cpu(K):
    g = torch.Generator().manual_seed(K)
    a = torch.randn((K, 24), generator=g, dtype=torch.float64)
    b = torch.randn((K, 40), generator=g, dtype=torch.float64)
    ref = a.t() @ b
    out = splitk.mm_tn(a, b)
    assert out.shape == (24, 40)
    assert torch.allclose(out, ref, rtol=1e-12, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("rows", [65536, 65536 + 333])
def test_splitk_linear_grads_match_nn_linear_gpu(rows):
    torch.manual_seed(0)
    dev = "cuda:0"
    lin = torch.nn.Linear(256, 128).to(dev)
    x = torch.randn((rows, 256), device=dev, requires_grad=True)
    dy = torch.randn((rows, 128), device=dev)
    y = splitk.sequential(torch.nn.Sequential(lin, torch.nn.Tanh()), x)
    (y * dy).sum().backward()
    gw, gb, gx = lin.weight.grad.clone(), lin.bias.grad.clone(), x.grad.clone()
    lin.weight.grad = lin.bias.grad = x.grad = None
    y2 = torch.tanh(lin(x))
    (y2 * dy).sum().backward()
    assert torch.allclose(y, y2, rtol=1e-5, atol=1e-6)
    # f32 sums over 65,536 samples in a different order: relative to the scale
    for got, ref in ((gw, lin.weight.grad), (gb, lin.bias.grad), (gx, x.grad)):
        assert (got - ref).abs().max().item() <= 1e-5 * ref.abs().max().item() + 1e-6
