"""The bf16x6 MLP kernels (csrc/field_x6.hip; bf16 matrix cores, operands split into three bf16
pieces, six products per term) against the f32-MFMA kernels (field_frag.hip, NERF_MLP=2) and an
fp64 reference: the x6 path must be as accurate as fp32. Both x6 backward kernels are checked:
NERF_MLP=3 (one wave per tile) and NERF_MLP=4 (the default: chain / weight-gradient wave pairs).

Bar: per output / per weight-gradient tensor, the x6 error against fp64 is at most 2x the error of
the same computation in plain PyTorch fp32 (the reference's own arithmetic; max and RMS), and
within the fp32 summation bound 2e-5 * sum|terms| used by test_mlp_large_vs_torch_fp32. (The split
drops terms <= 2^-23 |ab| per product; fp32 products round at 2^-24 |ab|; both accumulate in
fp32.) The f32-MFMA kernel's errors are printed beside them.
"""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(W, x):
    h = torch.relu(x[:, :32] @ W["sigma_net.0.weight"].t())
    o = h @ W["sigma_net.1.weight"].t()
    c = torch.relu(torch.cat([x[:, 32:], o[:, 1:]], -1) @ W["color_net.0.weight"].t())
    c = torch.relu(c @ W["color_net.1.weight"].t())
    return torch.cat([c @ W["color_net.2.weight"].t(), o[:, :1]], -1)


def _run(nerf, net, x, graw, version):
    old = os.environ.get("NERF_MLP")
    if version is None:
        os.environ.pop("NERF_MLP", None)
    else:
        os.environ["NERF_MLP"] = version
    try:
        for p in net.parameters():
            p.grad = None
        xx = x.clone().requires_grad_(True)
        raw = net(xx)
        (raw * graw).sum().backward()
        torch.cuda.synchronize()
        return raw.detach().double(), xx.grad.double(), {k: p.grad.double() for k, p in net.named_parameters()}
    finally:
        if old is None:
            os.environ.pop("NERF_MLP", None)
        else:
            os.environ["NERF_MLP"] = old


@pytest.mark.parametrize("version", ["3", "4"])
@pytest.mark.parametrize("scale", [0.5, 0.05])
def test_x6_as_accurate_as_f32_mfma(nerf, gpu, scale, version):
    torch.manual_seed(1)
    net = nerf.NeRFSmall(2, 64, 15, 3, 64, 32, 16).to(gpu)
    P = 65536
    x = torch.randn(P, 48, device=gpu) * scale
    graw = torch.randn(P, 4, device=gpu)
    raw6, dx6, g6 = _run(nerf, net, x, graw, version)
    raw2, dx2, g2 = _run(nerf, net, x, graw, "2")
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

    def check(name, got6, got2, got32, want, bound=None):
        e6, e2, e32 = (got6 - want).abs(), (got2 - want).abs(), (got32.double() - want).abs()
        rms = lambda e: e.pow(2).mean().sqrt().item()  # noqa: E731
        floor = 1e-12 + 1e-7 * want.abs().max().item()
        print(f"{name:22s} max x6 {e6.max().item():.3e} f32mfma {e2.max().item():.3e} torch {e32.max().item():.3e}"
              f" | rms x6 {rms(e6):.3e} f32mfma {rms(e2):.3e} torch {rms(e32):.3e}")
        if e6.max().item() > 2 * e32.max().item() + floor or rms(e6) > 2 * rms(e32) + floor:
            fails.append(name)
        if bound is not None and not (e6 <= bound).all():
            fails.append(name + " (bound)")

    check("raw", raw6, raw2, r32.detach(), ref.detach())
    check("dx", dx6, dx2, x32.grad, x64.grad)
    for k in g6:
        check(k, g6[k], g2[k], W32[k].grad, W64[k].grad, bound=2e-5 * Wabs[k].grad + 1e-6)
    assert not fails, fails


@pytest.mark.parametrize("P", [1, 31, 33, 1000, 4096 * 32 + 17, 300001])
def test_split_backward_matches_one_wave_backward(nerf, gpu, P):
    """The wave-pair backward (4) and the one-wave backward (3) do the same products per tile in the
    same order; only the block-level fp32 reductions differ. Ragged sizes: pairs with no tile, a
    partial last tile, more tiles than the persistent grid."""
    torch.manual_seed(2)
    net = nerf.NeRFSmall(2, 64, 15, 3, 64, 32, 16).to(gpu)
    x = torch.randn(P, 48, device=gpu) * 0.3
    graw = torch.randn(P, 4, device=gpu)
    raw3, dx3, g3 = _run(nerf, net, x, graw, "3")
    raw4, dx4, g4 = _run(nerf, net, x, graw, "4")
    assert torch.equal(raw3, raw4)
    assert torch.equal(dx3, dx4)    # per-point results: identical arithmetic
    for k in g3:
        scale = g3[k].abs().max().item() + 1e-30
        assert (g4[k] - g3[k]).abs().max().item() <= 1e-5 * scale, k
