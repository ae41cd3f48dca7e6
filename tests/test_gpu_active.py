"""Active-point backward (csrc/active.hip, field.set_active_points): the MLP backward and the hash bins
walk only the samples whose raw gradient is not all zero. raw2outputs' autograd (run_nerf.py:364-386)
gives a sample with relu(sigma + noise) = 0 alpha = 0, weight 0 and a zero sigma gradient, and
NeRFSmall's backward is linear in the upstream gradient, so the skipped terms are exactly 0."""
import pytest
import torch

from tables import blender_bbox, synthetic_rays

pytestmark = pytest.mark.gpu


def test_active_rows_kernel(nerf, gpu):
    """nerf_active_rows against torch: the points whose graw row (through the row map, the reuse's
    point order) is nonzero, ascending; how many of them are below n_first; the zeroed rows of the
    inactive points at or above n_first. Also without a row map."""
    from indoor_nerf_amd import _lib
    g = torch.Generator(device=gpu).manual_seed(1)
    i32 = torch.int32
    for P in (1, 63, 4096, 4097, 100_003):
        for mapped in (True, False):
            graw = torch.randn(P, 4, device=gpu, generator=g)
            graw[torch.rand(P, device=gpu, generator=g) < 0.4] = 0.0
            graw[torch.rand(P, device=gpu, generator=g) < 0.05, 1:] = 0.0   # partly zero rows stay active
            gmap = torch.randperm(P, device=gpu, generator=g).to(i32) if mapped else None
            n_first = P // 3
            L = 16
            zero = torch.full((L, P, 2), 7.0, device=gpu)
            rows = torch.full((P,), -1, device=gpu, dtype=i32)
            counts = torch.zeros(2, device=gpu, dtype=i32)
            ws = torch.empty(int(_lib.load().nerf_active_rows_workspace_bytes(P)) // 4, device=gpu, dtype=i32)
            _lib.call("nerf_active_rows", _lib.ptr(graw), None, P, _lib.ptr(gmap, "graw_rows", i32, True), n_first,
                      _lib.ptr(rows, "rows", i32), _lib.ptr(counts, "counts", i32),
                      _lib.ptr(zero), 2 * P, L, _lib.ptr(ws, "ws", i32), ws.numel() * 4, _lib.stream())
            torch.cuda.synchronize()
            on = (graw[gmap.long()] if mapped else graw).ne(0).any(-1)
            want = torch.nonzero(on).flatten().to(i32)
            assert int(counts[0]) == want.numel()
            assert torch.equal(rows[:want.numel()], want)
            assert int(counts[1]) == int((want < n_first).sum())
            # zeroed: rows p >= n_first of the inactive points; every other row untouched
            zrow = torch.nonzero(~on).flatten()
            zrow = zrow[zrow >= n_first]
            expect = torch.full((L, P, 2), 7.0, device=gpu)
            expect[:, zrow, :] = 0.0
            assert torch.equal(zero, expect)


def _scene(nerf, gpu, R=512):
    lo, hi = blender_bbox()
    args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), finest_res=1024, N_samples=64,
                          N_importance=128, white_bkgd=True)
    torch.manual_seed(0)
    kw_train, _, _, _, _ = nerf.create_nerf(args, device=gpu)
    with torch.no_grad():
        g = torch.Generator().manual_seed(7)
        for e in kw_train["embed_fn"].embeddings:
            e.weight.copy_((torch.rand(e.weight.shape, generator=g) * 2 - 1) * 0.05)
    kw = {k: v for k, v in kw_train.items() if k not in ("ndc", "use_viewdirs", "near", "far")}
    ro, rd = synthetic_rays(R, seed=9)
    ro, rd = torch.from_numpy(ro).to(gpu), torch.from_numpy(rd).to(gpu)
    vd = rd / torch.norm(rd, dim=-1, keepdim=True)
    rays = torch.cat([ro, rd, torch.full((R, 1), 2.0, device=gpu), torch.full((R, 1), 6.0, device=gpu), vd], -1)
    target = torch.rand(R, 3, device=gpu, generator=torch.Generator(device=gpu).manual_seed(3))
    return kw, rays, target


def _params(kw):
    return (list(kw["embed_fn"].parameters()) + list(kw["network_fn"].parameters())
            + list(kw["network_fine"].parameters()))


def _grads(nerf, kw, rays, target, active, reuse, parts):
    nerf.set_active_points(active)
    nerf.set_coarse_reuse(reuse)
    try:
        for p in _params(kw):
            p.grad = None
        out = nerf.render_rays(rays, **kw, pytest=True)
        loss = sum(((out[k] - target) ** 2).mean() for k in parts)
        loss.backward()
        torch.cuda.synchronize()
        return [None if p.grad is None else p.grad.detach().clone() for p in _params(kw)]
    finally:
        nerf.set_active_points(False)
        nerf.set_coarse_reuse(True)


@pytest.mark.parametrize("reuse", [True, False], ids=["reuse", "no_reuse"])
@pytest.mark.parametrize("parts", [("rgb_map", "rgb0"), ("rgb_map",), ("rgb0",)],
                         ids=["both_passes", "fine_only", "coarse_only"])
def test_active_points_match_all_points(nerf, gpu, reuse, parts):
    """Active points vs every point, deterministic mode: table gradients within 1e-6 of the level's
    largest |gradient| (the same entries; runs may split at other wave boundaries, and each entry is
    rounded to fixed point on its own), MLP gradients within 1e-6 in norm (the same terms, summed in
    other tiles). Some points must be inactive for the test to mean anything."""
    kw, rays, target = _scene(nerf, gpu)
    nerf.set_deterministic(True)
    try:
        g_all = _grads(nerf, kw, rays, target, False, reuse, parts)
        g_act = _grads(nerf, kw, rays, target, True, reuse, parts)
    finally:
        nerf.set_deterministic(False)
    n_tab = kw["embed_fn"].n_levels
    for i, (a, b) in enumerate(zip(g_act, g_all)):
        assert (a is None) == (b is None), i
        if a is None:
            continue
        scale = float(b.abs().max())
        if i < n_tab:
            assert float((a - b).abs().max()) <= 1e-6 * scale + 1e-30, f"table {i}"
        else:
            assert float((a - b).norm()) <= 1e-6 * float(b.norm()) + 1e-30, f"mlp param {i - n_tab}"


def test_active_points_some_inactive(nerf, gpu):
    """The scene of the tests above has samples with an all-zero raw gradient (outside the box or
    relu(sigma) = 0), so the active-point path is exercised."""
    import importlib
    rmod = importlib.import_module("indoor_nerf_amd.render")
    kw, rays, target = _scene(nerf, gpu)
    seen = []
    orig = rmod.CompositeFn.backward

    def spy(ctx, *grads):
        out = orig(ctx, *grads)
        seen.append(float((out[0] == 0).all(-1).float().mean()))
        return out
    rmod.CompositeFn.backward = staticmethod(spy)
    try:
        out = nerf.render_rays(rays, **kw, pytest=True)
        ((out["rgb_map"] - target) ** 2).mean().add(((out["rgb0"] - target) ** 2).mean()).backward()
        torch.cuda.synchronize()
    finally:
        rmod.CompositeFn.backward = staticmethod(orig)
    assert len(seen) == 2 and all(0.0 < f < 1.0 for f in seen), seen
