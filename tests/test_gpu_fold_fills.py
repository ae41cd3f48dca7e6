"""The training step's zero fills folded into render()'s first launch (nerf_rays_pack_z,
_lib.defer_fill_zero): the dense part of a GradArena(defer_tables=True) zero and the TV loss
accumulator are stored by the rays_pack launch instead of two fill kernels. Against fills at once
(_lib.set_fold_fills(False)), deterministic backward, eager and replayed from a HIP graph: every
parameter, gradient and loss bit-identical after several steps (so the gradients were zeroed before
each backward), and no fill is left pending after a step."""
import pytest
import torch

from tables import blender_bbox, synthetic_rays

pytestmark = pytest.mark.gpu


def _run(nerf, gpu, fold, graphed, steps=4, R=1024):
    from indoor_nerf_amd import _lib
    from indoor_nerf_amd.graphs import GraphedTrainStep
    lo, hi = blender_bbox()
    args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), finest_res=1024, N_samples=64,
                          N_importance=128, white_bkgd=True, perturb=1.0, tv_loss_weight=1e-6)
    torch.manual_seed(0)
    kw, _, _, grad_vars, opt = nerf.create_nerf(args, device=gpu)
    kw.update(near=2.0, far=6.0)
    ro, rd = synthetic_rays(R, seed=31)
    rays = (torch.from_numpy(ro).to(gpu), torch.from_numpy(rd).to(gpu))
    target = torch.rand(R, 3, device=gpu, generator=torch.Generator(device=gpu).manual_seed(3))
    params = grad_vars + list(kw["embed_fn"].parameters())
    arena = nerf.GradArena(params, defer_tables=True)
    nerf.manual_seed(5)
    tv_gen = torch.Generator().manual_seed(7)
    losses = []
    _lib.set_fold_fills(fold)
    try:
        st = GraphedTrainStep(rays, target, kw, opt, args, tv_generator=tv_gen, zero_grad=arena.zero_) if graphed else None
        for it in range(1, steps + 1):
            if graphed:
                loss, _ = st(it)
            else:
                loss, _ = nerf.train_step(rays, target, kw, opt, args, it, tv_generator=tv_gen, zero_grad=arena.zero_)
            assert not any(_lib._ZERO_FILLS.values()), "a deferred fill outlived its step"
            losses.append(loss.detach().clone())
        torch.cuda.synchronize()
    finally:
        _lib.set_fold_fills(True)
    return [p.detach().clone() for p in params], [p.grad.clone() for p in params], torch.stack(losses)


@pytest.mark.parametrize("graphed", [False, True], ids=["eager", "graphed"])
def test_folded_fills_bitwise(nerf, gpu, graphed):
    nerf.set_deterministic(True)
    try:
        pa, ga, la = _run(nerf, gpu, True, graphed)
        pb, gb, lb = _run(nerf, gpu, False, graphed)
    finally:
        nerf.set_deterministic(False)
    assert torch.equal(la, lb)
    for i, (a, b) in enumerate(zip(pa, pb)):
        assert torch.equal(a, b), f"parameter {i}"
    for i, (a, b) in enumerate(zip(ga, gb)):
        assert torch.equal(a, b), f"gradient {i}"


def test_rays_pack_zero_ranges(nerf, gpu):
    """nerf_rays_pack_z stores zeros over its ranges (also with no rays, and ranges larger than the
    rays' grid) and packs exactly as nerf_rays_pack."""
    from indoor_nerf_amd import _lib
    g = torch.Generator(device=gpu).manual_seed(2)
    o, d = torch.randn(300, 3, device=gpu, generator=g), torch.randn(300, 3, device=gpu, generator=g)
    a, b = torch.empty(300, 11, device=gpu), torch.empty(300, 11, device=gpu)
    z1, z2 = torch.full((18_688,), 7.0, device=gpu), torch.full((5_000_000,), 3.0, device=gpu)
    zr = (_lib.ZeroRange * 2)(_lib.ZeroRange(z1.data_ptr(), z1.numel()), _lib.ZeroRange(z2.data_ptr(), z2.numel()))
    _lib.call("nerf_rays_pack_z", _lib.ptr(o), _lib.ptr(d), 300, 2.0, 6.0, 0, 0.0, 0.0, 1, _lib.ptr(a), zr, 2,
              _lib.stream())
    _lib.call("nerf_rays_pack", _lib.ptr(o), _lib.ptr(d), 300, 2.0, 6.0, 0, 0.0, 0.0, 1, _lib.ptr(b), _lib.stream())
    z3 = torch.full((1000,), 1.0, device=gpu)
    zr3 = (_lib.ZeroRange * 1)(_lib.ZeroRange(z3.data_ptr(), z3.numel()))
    _lib.call("nerf_rays_pack_z", None, None, 0, 2.0, 6.0, 0, 0.0, 0.0, 1, None, zr3, 1, _lib.stream())
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert not z1.any() and not z2.any() and not z3.any()
