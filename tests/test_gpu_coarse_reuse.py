"""The premise of DESIGN §8.5 (reusing the coarse pass's encoding in the fine pass), checked on the
HIP path: the fine point set of every ray contains each coarse point bit for bit, at the coarse
depth's rank in the merged sorted depths (run_nerf.py:512-513: torch.sort(cat([z_vals, z_samples]))
then rays_o + rays_d * z), and the hash features of those fine points equal the coarse pass's bit for
bit (one embedder serves both networks, run_nerf.py:225,275). Training perturbation through the
reference's pytest uniforms, so the coarse-only and the full call draw the same stratified depths."""
import pytest
import torch

from tables import blender_bbox, synthetic_rays

pytestmark = pytest.mark.gpu


def test_fine_set_contains_coarse_points_bitwise(nerf, gpu):
    lo, hi = blender_bbox()
    args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), finest_res=1024, N_samples=64,
                          N_importance=128, white_bkgd=True)
    torch.manual_seed(0)
    kw_train, _, _, _, _ = nerf.create_nerf(args, device=gpu)
    emb = kw_train["embed_fn"]
    with torch.no_grad():
        g = torch.Generator().manual_seed(7)
        for e in emb.embeddings:
            e.weight.copy_((torch.rand(e.weight.shape, generator=g) * 2 - 1) * 0.05)
    kw = {k: v for k, v in kw_train.items() if k not in ("ndc", "use_viewdirs", "near", "far")}
    R = 512
    ro, rd = synthetic_rays(R, seed=9)
    ro, rd = torch.from_numpy(ro).to(gpu), torch.from_numpy(rd).to(gpu)
    vd = rd / torch.norm(rd, dim=-1, keepdim=True)
    rays = torch.cat([ro, rd, torch.full((R, 1), 2.0, device=gpu), torch.full((R, 1), 6.0, device=gpu), vd], -1)
    with torch.no_grad():
        coarse = nerf.render_rays(rays, **(kw | {"N_importance": 0}), pytest=True)["pts"]          # [R, 64, 3]
        fine = nerf.render_rays(rays, **kw, pytest=True)["pts"]                                    # [R, 192, 3]
    torch.cuda.synchronize()
    assert coarse.shape == (R, 64, 3) and fine.shape == (R, 192, 3)
    eq = (fine[:, None, :, :] == coarse[:, :, None, :]).all(-1)                                    # [R, 64, 192]
    assert eq.any(-1).all().item(), "a coarse point is missing from its ray's fine set"
    # the first match of coarse point j sits at or after rank j, in increasing order along the ray
    pos = eq.float().argmax(-1)                                                                    # [R, 64]
    assert (pos[:, 1:] > pos[:, :-1]).all().item()
    assert (pos >= torch.arange(64, device=gpu)).all().item()
    picked = torch.gather(fine, 1, pos[..., None].expand(-1, -1, 3))
    assert torch.equal(picked, coarse)
    with torch.no_grad():
        f_coarse = emb(coarse.reshape(-1, 3))
        f_fine = emb(picked.reshape(-1, 3).contiguous())
    torch.cuda.synchronize()
    for a, b in zip(f_coarse, f_fine):   # (features [P, 32], keep mask)
        assert torch.equal(a, b)


# ---- the reuse itself (render.CoarseReuse): the fine pass gathers its importance samples only, into
# the head of the coarse pass's importance-first feature buffer; the backward bins each shared point once

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


def _train_pass(nerf, kw, rays, target, reuse, parts):
    nerf.set_coarse_reuse(reuse)
    try:
        for p in _params(kw):
            p.grad = None
        out = nerf.render_rays(rays, **kw, pytest=True)
        loss = sum(((out[k] - target) ** 2).mean() for k in parts)
        loss.backward()
        torch.cuda.synchronize()
        outs = {k: v.detach().clone() for k, v in out.items() if torch.is_tensor(v)}
        grads = [None if p.grad is None else p.grad.detach().clone() for p in _params(kw)]
        return outs, grads
    finally:
        nerf.set_coarse_reuse(True)


@pytest.mark.parametrize("R", [512, 4096])
@pytest.mark.parametrize("parts", [("rgb_map", "rgb0"), ("rgb_map",), ("rgb0",)],
                         ids=["both_passes", "fine_only", "coarse_only"])
def test_coarse_reuse_matches_reencoding(nerf, gpu, parts, R):
    """Reuse on vs off on the same draws (deterministic mode, so the MLP weight gradients are summed in
    a fixed order): every render output bit-identical; MLP gradients within 1e-6 in norm (the fine
    net's points are walked in the reuse's importance-first order, so its tiles hold other points and
    the fp32 sums associate differently; the reference's own order is autograd's matmul); table gradients
    within 1e-5 of the level's largest |gradient| (the shared points' fine and coarse d feat are summed
    in fp32 before the bin instead of binned as two entries). fine_only: the coarse pass is not
    differentiated, so the fine job bins the coarse points itself; coarse_only: no fine backward."""
    kw, rays, target = _scene(nerf, gpu, R=R)     # 4096: the bench's batch (786,432 fine points)
    nerf.set_deterministic(True)
    try:
        out_a, g_a = _train_pass(nerf, kw, rays, target, True, parts)
        out_b, g_b = _train_pass(nerf, kw, rays, target, False, parts)
    finally:
        nerf.set_deterministic(False)
    assert out_a.keys() == out_b.keys()
    for k in out_a:
        assert torch.equal(out_a[k], out_b[k]), k
    n_tab = kw["embed_fn"].n_levels
    for i, (a, b) in enumerate(zip(g_a, g_b)):
        assert (a is None) == (b is None), i
        if a is None:
            continue
        if i < n_tab:
            scale = float(b.abs().max())
            assert float((a - b).abs().max()) <= 1e-5 * scale + 1e-30, f"table {i}"
            assert scale > 0, f"table {i}: no gradient"
        else:
            assert float((a - b).norm()) <= 1e-6 * float(b.norm()) + 1e-30, f"mlp param {i - n_tab}"


def test_coarse_reuse_is_taken(nerf, gpu):
    """The training forward takes the reuse path: two hash gathers (R*S coarse points, R*N importance
    samples, not R*(S+N)) and the fine MLP in the reuse's point order (nerf_mlp_fwd_h3)."""
    import importlib
    from indoor_nerf_amd import _lib
    rmod = importlib.import_module("indoor_nerf_amd.render")
    hmod = importlib.import_module("indoor_nerf_amd.hashgrid")
    kw, rays, target = _scene(nerf, gpu, R=256)
    plans, gathered = [], []
    orig_init, orig_enc = rmod.CoarseReuse.__init__, hmod.HashEmbedder.encode_into

    def init(self, *a):
        orig_init(self, *a)
        plans.append(self)

    def enc(self, xyz, *a, **k):
        gathered.append(xyz.shape[0])
        return orig_enc(self, xyz, *a, **k)
    rmod.CoarseReuse.__init__, hmod.HashEmbedder.encode_into = init, enc
    _lib.set_timing(True)
    try:
        out = nerf.render_rays(rays, **kw, pytest=True)
        torch.cuda.synchronize()
        names = [n for n, _, _ in _lib.timing_records()]
    finally:
        _lib.set_timing(False)
        rmod.CoarseReuse.__init__, hmod.HashEmbedder.encode_into = orig_init, orig_enc
    assert names.count("nerf_hash_encode_fwd_q") == 2 and names.count("nerf_mlp_fwd_h3") == 2
    assert gathered == [256 * 64, 256 * 128]
    assert len(plans) == 1 and plans[0].used
    assert out["pts"].shape == (256, 192, 3)


@pytest.mark.parametrize("sorted_coarse", [True, False])
def test_fine_row_maps_partition_each_ray(nerf, gpu, sorted_coarse):
    """nerf_sample_fine_rows: per ray, the coarse rows and the importance rows are disjoint and cover
    the ray's S+N fine rows; z_fine at a coarse row is that coarse depth; importance rows ascend (the
    bitonic merge) — also through the rank-sort path taken for unsorted coarse depths."""
    from indoor_nerf_amd import _lib
    R, S, N = 300, 64, 128
    M = S + N
    g = torch.Generator(device=gpu).manual_seed(5)
    z = 2.0 + 4.0 * torch.rand(R, S, device=gpu, generator=g)
    if sorted_coarse:
        z = torch.sort(z, -1).values
    w = torch.rand(R, S, device=gpu, generator=g)
    rays = torch.rand(R, 11, device=gpu, generator=g)
    zf, pf = torch.empty(R, M, device=gpu), torch.empty(R, M, 3, device=gpu)
    cr = torch.empty(R, S, device=gpu, dtype=torch.int32)
    ir = torch.empty(R, N, device=gpu, dtype=torch.int32)
    ip = torch.empty(R, N, 3, device=gpu)
    perm = torch.empty(R * M, device=gpu, dtype=torch.int32)   # the maps' inverse, still offered by the ABI
    _lib.call("nerf_sample_fine_rows", _lib.ptr(rays), 11, _lib.ptr(z), _lib.ptr(w), R, S, N, 0, None, None, 11, 0,
              None, _lib.ptr(zf), _lib.ptr(pf), None, None, _lib.ptr(cr, "cr", torch.int32),
              _lib.ptr(ir, "ir", torch.int32), _lib.ptr(ip), _lib.ptr(perm, "perm", torch.int32), _lib.stream())
    torch.cuda.synchronize()
    base = (torch.arange(R, device=gpu) * M)[:, None]
    allr = torch.sort(torch.cat([cr, ir], 1).long() - base, 1).values
    assert torch.equal(allr, torch.arange(M, device=gpu).expand(R, M))
    assert torch.equal(zf.reshape(-1)[cr.long().reshape(-1)].reshape(R, S), z)
    assert torch.equal(pf.reshape(-1, 3)[ir.long().reshape(-1)], ip.reshape(-1, 3))   # same bits as pts_fine
    # perm: fine row -> importance-first position (importance k of ray r: r*N + k; coarse i: R*N + r*S + i)
    assert torch.equal(perm[ir.long().reshape(-1)].long(), torch.arange(R * N, device=gpu))
    assert torch.equal(perm[cr.long().reshape(-1)].long(), R * N + torch.arange(R * S, device=gpu))
    if sorted_coarse:
        assert (ir[:, 1:] > ir[:, :-1]).all().item()


@pytest.mark.parametrize("R,S,N", [(37, 64, 128), (5, 3, 7)])
def test_mlp_point_order_matches_merged(nerf, gpu, R, S, N):
    """nerf_mlp_fwd_ord / a batch job with a nerf_point_order against the plain kernels on the same
    points in the merged order: raw / geo at the io rows bit-identical, d feat at the io rows
    bit-identical (the per-point chain is order-free), weight gradients equal up to the order of the
    fp32 sums (other points share a tile), in deterministic mode."""
    from indoor_nerf_amd import _lib
    from indoor_nerf_amd.field import _weights_struct
    M, L = S + N, 16
    P = R * M
    g = torch.Generator(device=gpu).manual_seed(11)
    # inv: per ray, a random split of its M merged rows into N importance and S coarse positions
    ranks = torch.argsort(torch.rand(R, M, device=gpu, generator=g), -1) + (torch.arange(R, device=gpu) * M)[:, None]
    inv = torch.cat([ranks[:, :N].reshape(-1), ranks[:, N:].reshape(-1)]).to(torch.int32)
    feat_o = torch.randn(L, P, 2, device=gpu, generator=g)
    feat_m = torch.empty_like(feat_o)
    feat_m[:, inv.long()] = feat_o
    keep_o = torch.rand(P, device=gpu, generator=g) < 0.9
    keep_m = torch.empty_like(keep_o)
    keep_m[inv.long()] = keep_o
    vd = torch.nn.functional.normalize(torch.randn(R, 3, device=gpu, generator=g), dim=-1)
    shapes = [(64, 32), (16, 64), (64, 31), (64, 64), (3, 64)]
    weights = [torch.randn(s, device=gpu, generator=g) * 0.2 for s in shapes]
    order = _lib.PointOrder(_lib.ptr(inv, "inv", torch.int32).value, R * N, S)
    bool_ = torch.bool

    def fwd(feat, keep, spr, order):
        raw, geo = torch.empty(P, 4, device=gpu), torch.empty(P, 16, device=gpu)
        _lib.call("nerf_mlp_fwd_ord", _lib.ptr(feat), 2, 2 * P, None, 0, _lib.ptr(vd), spr,
                  _lib.ptr(keep, "keep", bool_), P, _weights_struct(weights), _lib.ptr(raw), _lib.ptr(geo), None, None,
                  0, order, _lib.stream())
        return raw, geo
    raw_m, geo_m = fwd(feat_m, keep_m, M, None)
    raw_o, geo_o = fwd(feat_o, keep_o, N, order)
    torch.cuda.synchronize()
    assert torch.equal(raw_o, raw_m) and torch.equal(geo_o, geo_m)

    graw = torch.randn(P, 4, device=gpu, generator=g)
    ws = torch.empty(int(_lib.load().nerf_mlp_bwd_det_workspace_bytes()) // 4, device=gpu)

    def bwd(feat, keep, spr, order):
        grads = [torch.zeros_like(w) for w in weights]
        gs = _lib.MlpGrads()
        for name, t in zip(("w0", "w1", "c0", "c1", "c2"), grads):
            setattr(gs, name, _lib.ptr(t).value)
        dfeat = torch.empty(L, P, 2, device=gpu)
        j = _lib.MlpBwdJob()
        j.feat, j.feat_stride_point, j.feat_stride_level = _lib.ptr(feat), 2, 2 * P
        j.viewdirs, j.samples_per_ray, j.keep, j.n_points = _lib.ptr(vd), spr, _lib.ptr(keep, "keep", bool_), P
        j.weights, j.graw, j.grads, j.dfeat = _weights_struct(weights), _lib.ptr(graw), gs, _lib.ptr(dfeat)
        if order is not None:
            j.order = order
        arr = (_lib.MlpBwdJob * 1)(j)
        _lib.call("nerf_mlp_bwd_batch", arr, 1, _lib.ptr(ws), ws.numel() * 4, _lib.stream())
        return dfeat, grads
    df_m, gr_m = bwd(feat_m, keep_m, M, None)
    df_o, gr_o = bwd(feat_o, keep_o, N, order)
    torch.cuda.synchronize()
    assert torch.equal(df_o, df_m[:, inv.long()])
    for a, b in zip(gr_o, gr_m):
        assert float((a - b).norm()) <= 1e-5 * float(b.norm()) + 1e-30
