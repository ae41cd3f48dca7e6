"""Per-ray SH4 records (nerf_sample_stratified_sh writes SH4 of each ray's view direction once, with its
three exact bf16 pieces; the MLP kernels take them with sh_stride 0 instead of evaluating and splitting
SH per point, render.set_sh_rows) against the in-kernel evaluation: the same sh4_eval on the same
floats and the same split, so the MLP outputs and every gradient are bit-identical — at the ABI
(forward and backward, two-segment point order) and through render_rays."""
import pytest
import torch

from tables import blender_bbox, synthetic_rays

pytestmark = pytest.mark.gpu


def test_mlp_per_ray_sh_rows_bitwise(nerf, gpu):
    from indoor_nerf_amd import _lib
    from indoor_nerf_amd.field import _weights_struct
    R, S, N, L = 37, 64, 128, 16
    M = S + N
    P = R * M
    g = torch.Generator(device=gpu).manual_seed(3)
    rays = torch.rand(R, 11, device=gpu, generator=g)
    rays[:, 8:] = torch.nn.functional.normalize(torch.randn(R, 3, device=gpu, generator=g), dim=-1)
    t = torch.linspace(0, 1, S, device=gpu)
    z, pts = torch.empty(R, S, device=gpu), torch.empty(R, S, 3, device=gpu)
    vd, sh = torch.empty(R, 3, device=gpu), torch.empty(R, 40, device=gpu)
    _lib.call("nerf_sample_stratified_sh", _lib.ptr(rays), 11, R, S, _lib.ptr(t), 0, 0, None, 0, 0, None, _lib.ptr(z),
              _lib.ptr(pts), None, _lib.ptr(vd), _lib.ptr(sh), _lib.stream())
    ref = torch.empty(R, 16, device=gpu)
    _lib.call("nerf_sh4_fwd", _lib.ptr(vd), R, _lib.ptr(ref), _lib.stream())
    torch.cuda.synchronize()
    assert torch.equal(sh[:, :16], ref)
    # the record's bf16 pieces: exact (v0 + v1 + v2 == v) and each the RNE bf16 of the remainder
    pcs = sh[:, 16:].contiguous().view(torch.bfloat16).float().reshape(R, 3, 16)
    assert torch.equal(pcs[:, 0], ref.bfloat16().float())
    assert torch.equal(pcs[:, 1], (ref - pcs[:, 0]).bfloat16().float())
    assert torch.equal((pcs[:, 0] + pcs[:, 1]) + pcs[:, 2], ref)
    # the reuse's two-segment point order: importance rows (N per ray) then coarse rows (S per ray)
    ranks = torch.argsort(torch.rand(R, M, device=gpu, generator=g), -1) + (torch.arange(R, device=gpu) * M)[:, None]
    inv = torch.cat([ranks[:, :N].reshape(-1), ranks[:, N:].reshape(-1)]).to(torch.int32)
    order = _lib.PointOrder(_lib.ptr(inv, "inv", torch.int32).value, R * N, S)
    feat = torch.randn(L, P, 2, device=gpu, generator=g)
    keep = torch.rand(P, device=gpu, generator=g) < 0.9
    shapes = [(64, 32), (16, 64), (64, 31), (64, 64), (3, 64)]
    weights = [torch.randn(s, device=gpu, generator=g) * 0.2 for s in shapes]
    graw = torch.randn(P, 4, device=gpu, generator=g)
    ws = torch.empty(int(_lib.load().nerf_mlp_bwd_det_workspace_bytes()) // 4, device=gpu)

    def run(rows):
        view = (_lib.ptr(sh), 0, None) if rows else (None, 0, _lib.ptr(vd))
        raw, geo = torch.empty(P, 4, device=gpu), torch.empty(P, 16, device=gpu)
        _lib.call("nerf_mlp_fwd_ord", _lib.ptr(feat), 2, 2 * P, *view, N, _lib.ptr(keep, "keep", torch.bool), P,
                  _weights_struct(weights), _lib.ptr(raw), _lib.ptr(geo), None, None, 0, order, _lib.stream())
        grads = [torch.zeros_like(w) for w in weights]
        gs = _lib.MlpGrads()
        for name, tt in zip(("w0", "w1", "c0", "c1", "c2"), grads):
            setattr(gs, name, _lib.ptr(tt).value)
        dfeat = torch.empty(L, P, 2, device=gpu)
        j = _lib.MlpBwdJob()
        j.feat, j.feat_stride_point, j.feat_stride_level = _lib.ptr(feat), 2, 2 * P
        if rows:
            j.sh, j.sh_stride = _lib.ptr(sh), 0
        else:
            j.viewdirs = _lib.ptr(vd)
        j.samples_per_ray, j.keep, j.n_points = N, _lib.ptr(keep, "keep", torch.bool), P
        j.weights, j.graw, j.grads, j.dfeat, j.order = _weights_struct(weights), _lib.ptr(graw), gs, _lib.ptr(dfeat), order
        _lib.call("nerf_mlp_bwd_batch", (_lib.MlpBwdJob * 1)(j), 1, _lib.ptr(ws), ws.numel() * 4, _lib.stream())
        torch.cuda.synchronize()
        return [raw, geo, dfeat] + grads

    for a, b in zip(run(True), run(False)):
        assert torch.equal(a, b)


def _train(nerf, gpu, rows, R=1024):
    lo, hi = blender_bbox()
    args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), finest_res=1024, N_samples=64,
                          N_importance=128, white_bkgd=True, perturb=1.0)
    torch.manual_seed(0)
    kw, _, _, _, _ = nerf.create_nerf(args, device=gpu)
    kw = {k: v for k, v in kw.items() if k not in ("ndc", "use_viewdirs", "near", "far")}
    ro, rd = synthetic_rays(R, seed=17)
    ro, rd = torch.from_numpy(ro).to(gpu), torch.from_numpy(rd).to(gpu)
    vd = rd / torch.norm(rd, dim=-1, keepdim=True)
    rays = torch.cat([ro, rd, torch.full((R, 1), 2.0, device=gpu), torch.full((R, 1), 6.0, device=gpu), vd], -1)
    prev = nerf.sh_rows()
    nerf.set_sh_rows(rows)
    nerf.manual_seed(9)
    try:
        out = nerf.render_rays(rays, **kw)
        (((out["rgb_map"] - 0.5) ** 2).mean() + ((out["rgb0"] - 0.5) ** 2).mean()).backward()
        torch.cuda.synchronize()
    finally:
        nerf.set_sh_rows(prev)
    params = list(kw["embed_fn"].parameters()) + list(kw["network_fn"].parameters()) + list(kw["network_fine"].parameters())
    return {k: v.detach().clone() for k, v in out.items() if torch.is_tensor(v)}, [p.grad.clone() for p in params]


def test_render_rays_sh_rows_bitwise(nerf, gpu):
    nerf.set_deterministic(True)
    try:
        oa, ga = _train(nerf, gpu, True)
        ob, gb = _train(nerf, gpu, False)
    finally:
        nerf.set_deterministic(False)
    for k in oa:
        assert torch.equal(oa[k], ob[k]), k
    for i, (a, b) in enumerate(zip(ga, gb)):
        assert torch.equal(a, b), i
