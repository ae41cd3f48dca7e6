"""The MLP kernels (csrc/field_x6.hip: bf16 matrix cores, fp32 operands split into three bf16
pieces, six products per term; chain / weight-gradient wave-pair backward) against fp64 and plain
PyTorch fp32 (NeRFSmall.forward, run_nerf_helpers.py:265-306): the path must be as accurate as fp32.

Bar: per output / per weight-gradient tensor, the kernel's error against fp64 is at most 2x the
error of the same computation in plain PyTorch fp32 (the reference's own arithmetic; max and RMS),
and within the fp32 summation bound 2e-5 * sum|terms| used by test_mlp_large_vs_torch_fp32. (The
split drops terms <= 2^-23 |ab| per product; fp32 products round at 2^-24 |ab|; both accumulate in
fp32.)
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(W, x):
    h = torch.relu(x[:, :32] @ W["sigma_net.0.weight"].t())
    o = h @ W["sigma_net.1.weight"].t()
    c = torch.relu(torch.cat([x[:, 32:], o[:, 1:]], -1) @ W["color_net.0.weight"].t())
    c = torch.relu(c @ W["color_net.1.weight"].t())
    return torch.cat([c @ W["color_net.2.weight"].t(), o[:, :1]], -1)


def _run(net, x, graw):
    for p in net.parameters():
        p.grad = None
    xx = x.clone().requires_grad_(True)
    raw = net(xx)
    (raw * graw).sum().backward()
    torch.cuda.synchronize()
    return raw.detach().double(), xx.grad.double(), {k: p.grad.double() for k, p in net.named_parameters()}


def _check_vs_fp64(net, x, graw):
    raw6, dx6, g6 = _run(net, x, graw)
    W64 = {k: p.detach().double().clone().requires_grad_(True) for k, p in net.named_parameters()}
    x64 = x.double().clone().requires_grad_(True)
    ref = _ref(W64, x64)
    (ref * graw.double()).sum().backward()
    torch.backends.cuda.matmul.allow_tf32 = False
    W32 = {k: p.detach().clone().requires_grad_(True) for k, p in net.named_parameters()}
    x32 = x.clone().requires_grad_(True)
    r32 = _ref(W32, x32)
    (r32 * graw).sum().backward()
    Wabs = {k: p.detach().double().abs().requires_grad_(True) for k, p in net.named_parameters()}
    refabs = _ref(Wabs, x.double().abs())
    (refabs * graw.double().abs()).sum().backward()

    fails = []

    def check(name, got6, got32, want, bound=None):
        e6, e32 = (got6 - want).abs(), (got32.double() - want).abs()
        rms = lambda e: e.pow(2).mean().sqrt().item()  # noqa: E731
        floor = 1e-12 + 1e-7 * want.abs().max().item()
        print(f"{name:22s} max x6 {e6.max().item():.3e} torch {e32.max().item():.3e}"
              f" | rms x6 {rms(e6):.3e} torch {rms(e32):.3e}")
        if e6.max().item() > 2 * e32.max().item() + floor or rms(e6) > 2 * rms(e32) + floor:
            fails.append(name)
        if bound is not None and not (e6 <= bound).all():
            fails.append(name + " (bound)")

    check("raw", raw6, r32.detach(), ref.detach())
    check("dx", dx6, x32.grad, x64.grad)
    for k in g6:
        check(k, g6[k], W32[k].grad, W64[k].grad, bound=2e-5 * Wabs[k].grad + 1e-6)
    return fails


@pytest.mark.parametrize("scale", [0.5, 0.05])
def test_x6_as_accurate_as_fp32(nerf, gpu, scale):
    torch.manual_seed(1)
    net = nerf.NeRFSmall(2, 64, 15, 3, 64, 32, 16).to(gpu)
    P = 65536
    x = torch.randn(P, 48, device=gpu) * scale
    graw = torch.randn(P, 4, device=gpu)
    fails = _check_vs_fp64(net, x, graw)
    assert not fails, fails


@pytest.mark.parametrize("P", [1, 31, 33, 1000, 4096 * 32 + 17, 300001])
def test_x6_ragged_sizes(nerf, gpu, P):
    """Ragged sizes: wave pairs with no tile, a partial last tile, more tiles than the persistent
    grid; same accuracy bar as above."""
    torch.manual_seed(2)
    net = nerf.NeRFSmall(2, 64, 15, 3, 64, 32, 16).to(gpu)
    x = torch.randn(P, 48, device=gpu) * 0.3
    graw = torch.randn(P, 4, device=gpu)
    fails = _check_vs_fp64(net, x, graw)
    assert not fails, fails
