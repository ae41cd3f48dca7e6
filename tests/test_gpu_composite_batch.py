"""The compositing backwards of a training iteration in one launch (nerf_composite_bwd_batch; render
.set_batched_composite_bwd defers the fine and the coarse CompositeFn backward to the pass's final
callback) against one nerf_composite_bwd per pass: bit-identical raw gradients at the ABI (every
supported pair of per-lane sample counts, either order, more than two jobs, the one-launch-per-job
fallback, empty jobs) and identical parameter gradients through render_rays — also when a loss
differentiates render_rays' raw output itself (the guard launches the deferred backward first)."""
import pytest
import torch

from tables import blender_bbox, synthetic_rays

pytestmark = pytest.mark.gpu


def _job(gpu, R, S, C, seed, white=1):
    from indoor_nerf_amd import _lib
    g = torch.Generator(device=gpu).manual_seed(seed)
    t = dict(raw=torch.randn(R, S, C, device=gpu, generator=g) * 2.0,
             z=torch.sort(2.0 + 4.0 * torch.rand(R, S, device=gpu, generator=g), -1).values,
             rays_d=torch.randn(R, 3, device=gpu, generator=g),
             noise=torch.randn(R, S, device=gpu, generator=g) if seed % 2 else None,
             g_rgb=torch.randn(R, 3, device=gpu, generator=g), g_disp=None,
             g_acc=torch.randn(R, device=gpu, generator=g), g_weights=None,
             g_depth=torch.randn(R, device=gpu, generator=g) if seed % 3 == 0 else None,
             g_entropy=torch.randn(R, device=gpu, generator=g),
             g_normal=torch.randn(R, 3, device=gpu, generator=g) if C == 7 else None)
    t["graw"] = torch.full((R, S, C), float("nan"), device=gpu)
    P = lambda k: _lib.ptr(t[k], k, allow_none=True)   # noqa: E731
    j = _lib.CompositeBwdJob(P("raw"), C, P("z"), P("rays_d"), P("noise"), R, S, white, P("g_rgb"), P("g_disp"),
                             P("g_acc"), P("g_weights"), P("g_depth"), P("g_entropy"), P("g_normal"), P("graw"))
    return j, t


def _single(gpu, t, C, R, S, white=1):
    from indoor_nerf_amd import _lib
    out = torch.full_like(t["graw"], float("nan"))
    P = lambda k: _lib.ptr(t[k], k, allow_none=True)   # noqa: E731
    _lib.call("nerf_composite_bwd", P("raw"), C, P("z"), P("rays_d"), P("noise"), R, S, white, P("g_rgb"),
              P("g_disp"), P("g_acc"), P("g_weights"), P("g_depth"), P("g_entropy"), P("g_normal"), _lib.ptr(out),
              _lib.stream())
    return out


@pytest.mark.parametrize("shapes", [
    [(4096, 192, 4), (4096, 64, 4)],     # the lego iteration (K 3 + 1)
    [(300, 64, 4), (511, 128, 7)],       # K 1 + 2, the heavier second (swapped inside), normals
    [(37, 64, 7), (5, 3, 4)],            # K 1 + 1, tiny
    [(65, 250, 4), (33, 100, 4)],        # K 4 + 2
    [(17, 192, 4), (9, 130, 4)],         # K 3 + 3
    [(40, 500, 4), (20, 64, 4)],         # K 8 + 1: no pair kernel, one launch per job
    [(70, 192, 4), (0, 64, 4), (30, 64, 4), (11, 128, 4)],   # an empty job; more than two jobs
])
def test_composite_bwd_batch_bitwise(nerf, gpu, shapes):
    from indoor_nerf_amd import _lib
    jobs = [_job(gpu, R, S, C, seed=i + 1) for i, (R, S, C) in enumerate(shapes)]
    _lib.call("nerf_composite_bwd_batch", (_lib.CompositeBwdJob * len(jobs))(*[j for j, _ in jobs]), len(jobs),
              _lib.stream())
    refs = [_single(gpu, t, C, R, S) for (_, t), (R, S, C) in zip(jobs, shapes)]
    torch.cuda.synchronize()
    for (_, t), ref in zip(jobs, refs):
        assert not torch.isnan(ref).any()
        assert torch.equal(t["graw"], ref)


def test_composite_bwd_batch_validates_before_launch(nerf, gpu):
    from indoor_nerf_amd import _lib
    (j0, t0), (j1, _) = _job(gpu, 64, 64, 4, 1), _job(gpu, 64, 64, 4, 2)
    j1.raw_channels = 5
    with pytest.raises(RuntimeError, match="raw_channels"):
        _lib.call("nerf_composite_bwd_batch", (_lib.CompositeBwdJob * 2)(j0, j1), 2, _lib.stream())
    torch.cuda.synchronize()
    assert torch.isnan(t0["graw"]).all()          # nothing ran
    _lib.call("nerf_composite_bwd_batch", None, 0, _lib.stream())


def _scene(nerf, gpu, R=1024):
    lo, hi = blender_bbox()
    args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), finest_res=1024, N_samples=64,
                          N_importance=128, white_bkgd=True, perturb=1.0)
    torch.manual_seed(0)
    kw, _, _, _, _ = nerf.create_nerf(args, device=gpu)
    kw = {k: v for k, v in kw.items() if k not in ("ndc", "use_viewdirs", "near", "far")}
    ro, rd = synthetic_rays(R, seed=13)
    ro, rd = torch.from_numpy(ro).to(gpu), torch.from_numpy(rd).to(gpu)
    vd = rd / torch.norm(rd, dim=-1, keepdim=True)
    rays = torch.cat([ro, rd, torch.full((R, 1), 2.0, device=gpu), torch.full((R, 1), 6.0, device=gpu), vd], -1)
    return kw, rays


def _pass(nerf, kw, rays, batched, raw_loss):
    from indoor_nerf_amd import _lib
    params = list(kw["embed_fn"].parameters()) + list(kw["network_fn"].parameters()) + list(kw["network_fine"].parameters())
    for p in params:
        p.grad = None
    prev = nerf.batched_composite_bwd()
    nerf.set_batched_composite_bwd(batched)
    nerf.manual_seed(21)
    _lib.set_timing(True)
    try:
        out = nerf.render_rays(rays, **kw, retraw=True)
        loss = ((out["rgb_map"] - 0.5) ** 2).mean() + ((out["rgb0"] - 0.5) ** 2).mean() + out["sparsity_loss"].mean()
        if raw_loss:
            loss = loss + 1e-3 * (out["raw"][..., 3] ** 2).mean()
        loss.backward()
        torch.cuda.synchronize()
        names = [n for n, _, _ in _lib.timing_records()]
    finally:
        _lib.set_timing(False)
        nerf.set_batched_composite_bwd(prev)
    return [p.grad.clone() for p in params], names


@pytest.mark.parametrize("raw_loss", [False, True], ids=["composite_only", "loss_on_raw_too"])
def test_render_rays_batched_composite_bwd_matches(nerf, gpu, raw_loss):
    """Deferred + batched vs immediate compositing backwards, same draws, deterministic backward:
    every parameter gradient bit-identical. Without a loss on raw the two passes' backwards are one
    nerf_composite_bwd_batch launch; with one (render_rays' guarded raw output), the deferred fine
    backward is launched when the raw gradient arrives, before autograd sums the two."""
    kw, rays = _scene(nerf, gpu)
    nerf.set_deterministic(True)
    try:
        g_a, names_a = _pass(nerf, kw, rays, True, raw_loss)
        g_b, names_b = _pass(nerf, kw, rays, False, raw_loss)
    finally:
        nerf.set_deterministic(False)
    for i, (a, b) in enumerate(zip(g_a, g_b)):
        assert torch.equal(a, b), i
    assert names_b.count("nerf_composite_bwd_batch") == 2
    assert names_a.count("nerf_composite_bwd_batch") == (2 if raw_loss else 1)
    assert "nerf_composite_bwd" not in names_a
