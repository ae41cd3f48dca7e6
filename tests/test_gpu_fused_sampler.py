"""The coarse pass's compositing and the hierarchical sampler in one launch (nerf_composite_sample_fine,
render.set_fused_coarse_sampler) against the two launches it replaces (nerf_composite_fwd, then
nerf_sample_fine_rows on its weights): the fused kernel hands the weights to the sampler through LDS
instead of HBM, so every output is bit-identical — at the ABI on random inputs (with and without
normals, noise, row maps; deterministic, given and Philox uniforms; the two-launch fallback for
S > 128) and through render_rays' forward and backward."""
import pytest
import torch

from tables import blender_bbox, synthetic_rays

pytestmark = pytest.mark.gpu


def _inputs(gpu, R, S, C, seed):
    g = torch.Generator(device=gpu).manual_seed(seed)
    raw = torch.randn(R, S, C, device=gpu, generator=g) * 2.0
    z = torch.sort(2.0 + 4.0 * torch.rand(R, S, device=gpu, generator=g), -1).values
    rays = torch.rand(R, 11, device=gpu, generator=g)
    rays_d = rays[:, 3:6].contiguous()
    noise = torch.randn(R, S, device=gpu, generator=g)
    return raw, z, rays, rays_d, noise


def _run(nerf, gpu, fused, R, S, N, C, noise, det, uniforms, maps):
    from indoor_nerf_amd import _lib
    raw, z, rays, rays_d, nz = _inputs(gpu, R, S, C, seed=R + S + C)
    M = S + N
    f = dict(device=gpu, dtype=torch.float32)
    i32 = dict(device=gpu, dtype=torch.int32)
    comp = dict(rgb=torch.empty(R, 3, **f), disp=torch.empty(R, **f), acc=torch.empty(R, **f),
                weights=torch.empty(R, S, **f), depth=torch.empty(R, **f), ent=torch.empty(R, **f),
                normal=torch.empty(R, 3, **f) if C == 7 else None)
    samp = dict(z_fine=torch.empty(R, M, **f), pts=torch.empty(R, M, 3, **f), z_std=torch.empty(R, **f),
                samples=torch.empty(R, N, **f))
    if maps:
        samp.update(cr=torch.empty(R, S, **i32), ir=torch.empty(R, N, **i32), ip=torch.empty(R, N, 3, **f),
                    perm=torch.empty(R * M, **i32))
    t = torch.linspace(0, 1, N, device=gpu) if det else None
    u = torch.rand(R, N, device=gpu, generator=torch.Generator(device=gpu).manual_seed(4)) if uniforms else None
    P = lambda k: _lib.ptr(samp.get(k), k, torch.int32 if k in ("cr", "ir", "perm") else torch.float32, True)  # noqa: E731
    cargs = (_lib.ptr(raw), C, _lib.ptr(z), _lib.ptr(rays_d), _lib.ptr(nz if noise else None, allow_none=True), R, S, 1,
             *[_lib.ptr(comp[k], k, allow_none=True) for k in ("rgb", "disp", "acc", "weights", "depth", "ent", "normal")])
    sargs = (N, int(det), _lib.ptr(t, allow_none=True), _lib.ptr(u, allow_none=True), 1234, 77, None,
             P("z_fine"), P("pts"), P("z_std"), P("samples"), P("cr"), P("ir"), P("ip"), P("perm"))
    if fused:
        _lib.call("nerf_composite_sample_fine", *cargs, _lib.ptr(rays), 11, *sargs, _lib.stream())
    else:
        _lib.call("nerf_composite_fwd", *cargs, _lib.stream())
        _lib.call("nerf_sample_fine_rows", _lib.ptr(rays), 11, _lib.ptr(z), _lib.ptr(comp["weights"]), R, S, *sargs,
                  _lib.stream())
    torch.cuda.synchronize()
    return {k: v for d in (comp, samp) for k, v in d.items() if v is not None}


@pytest.mark.parametrize("R,S,N,C,noise,det,uniforms,maps", [
    (300, 64, 128, 4, False, False, False, True),     # the lego coarse pass (K = 1), Philox
    (37, 64, 128, 7, True, False, True, True),        # normals + noise, given uniforms
    (129, 128, 64, 4, False, True, False, False),     # K = 2, deterministic
    (5, 3, 7, 4, False, False, False, True),          # tiny rays
    (33, 100, 50, 7, True, False, False, False),      # ragged K = 2
    (17, 200, 64, 4, False, False, False, True),      # S > 128: the two-launch fallback inside the call
])
def test_fused_coarse_sampler_bitwise(nerf, gpu, R, S, N, C, noise, det, uniforms, maps):
    a = _run(nerf, gpu, True, R, S, N, C, noise, det, uniforms, maps)
    b = _run(nerf, gpu, False, R, S, N, C, noise, det, uniforms, maps)
    assert a.keys() == b.keys()
    for k in a:
        assert torch.equal(a[k], b[k]) or (torch.isnan(a[k]).equal(torch.isnan(b[k]))
                                           and torch.equal(a[k].nan_to_num(), b[k].nan_to_num())), k


def test_fused_coarse_sampler_empty_batch(nerf, gpu):
    from indoor_nerf_amd import _lib
    _lib.call("nerf_composite_sample_fine", None, 4, None, None, None, 0, 64, 0, *([None] * 7), None, 11, 128, 0,
              None, None, 0, 0, None, *([None] * 8), _lib.stream())


def _render(nerf, gpu, fused):
    lo, hi = blender_bbox()
    args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), finest_res=1024, N_samples=64,
                          N_importance=128, white_bkgd=True, perturb=1.0)
    torch.manual_seed(0)
    kw, _, _, _, _ = nerf.create_nerf(args, device=gpu)
    kw = {k: v for k, v in kw.items() if k not in ("ndc", "use_viewdirs", "near", "far")}
    R = 1024
    ro, rd = synthetic_rays(R, seed=13)
    ro, rd = torch.from_numpy(ro).to(gpu), torch.from_numpy(rd).to(gpu)
    vd = rd / torch.norm(rd, dim=-1, keepdim=True)
    rays = torch.cat([ro, rd, torch.full((R, 1), 2.0, device=gpu), torch.full((R, 1), 6.0, device=gpu), vd], -1)
    prev = nerf.fused_coarse_sampler()
    nerf.set_fused_coarse_sampler(fused)
    nerf.manual_seed(21)
    try:
        out = nerf.render_rays(rays, **kw)
        loss = ((out["rgb_map"] - 0.5) ** 2).mean() + ((out["rgb0"] - 0.5) ** 2).mean()
        loss.backward()
        torch.cuda.synchronize()
    finally:
        nerf.set_fused_coarse_sampler(prev)
    params = list(kw["embed_fn"].parameters()) + list(kw["network_fn"].parameters()) + list(kw["network_fine"].parameters())
    return {k: v.detach().clone() for k, v in out.items() if torch.is_tensor(v)}, [p.grad.clone() for p in params]


def test_render_rays_fused_coarse_sampler_matches(nerf, gpu):
    """render_rays with the fused launch vs the two launches on the same Philox draws (deterministic
    backward): every output and gradient bit-identical."""
    nerf.set_deterministic(True)
    try:
        out_a, g_a = _render(nerf, gpu, True)
        out_b, g_b = _render(nerf, gpu, False)
    finally:
        nerf.set_deterministic(False)
    assert out_a.keys() == out_b.keys()
    for k in out_a:
        assert torch.equal(out_a[k], out_b[k]), k
    for i, (a, b) in enumerate(zip(g_a, g_b)):
        assert torch.equal(a, b), i
