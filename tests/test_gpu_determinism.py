"""Deterministic mode and the numerical check (needs an MI355X).

SURVEY.md §8(b) asks for a `deterministic` flag on the hash backward; the reference's render_rays
tests its outputs for NaN/Inf under DEBUG (run_nerf.py:40, :545-547).

* nerf_hash_encode_bwd_* with deterministic = 1: the owner pass sums in exact integer fixed point
  (csrc/hashgrid.hip hash_bwd_owner_kernel<12, 1024, true>) -> bit-identical across runs, and
  closer to the fp64 scatter than the fp32-rounded default path.
* nerf_mlp_bwd_batch with a deterministic workspace: per-block weight-gradient images reduced over
  blocks in a fixed order (mlp_wgrad_reduce_kernel).
* set_deterministic(True): a whole training iteration's gradients (render coarse + fine, loss head
  with TV, backward: the TV gradient is binned into the hash backward's owner pass) are bit-identical
  across runs.
"""
import numpy as np
import pytest
import torch

from tables import blender_bbox, closed_form_table, synthetic_rays

pytestmark = pytest.mark.gpu


def _ray_points(n_rays, S, seed):
    ro, rd = synthetic_rays(n_rays, seed=seed)
    rng = np.random.RandomState(seed)
    z = np.sort(2.0 + 4.0 * rng.rand(n_rays, S), axis=1).astype(np.float32)
    return (ro[:, None, :] + rd[:, None, :] * z[..., None]).reshape(-1, 3).astype(np.float32)


def test_hash_bwd_deterministic_bitwise_and_accurate(nerf, gpu, oracle):
    from indoor_nerf_amd import _lib
    lo, hi = blender_bbox()
    x = _ray_points(4096, 192, 31)
    P = x.shape[0]
    rng = np.random.RandomState(31)
    # gradients over six decades (dynamic range inside every row), one level all zero
    dfeat = (rng.randn(16, P, 2) * 10.0 ** rng.uniform(-6, 0, (16, P, 1))).astype(np.float32)
    dfeat[5] = 0.0
    emb = nerf.HashEmbedder((torch.from_numpy(lo), torch.from_numpy(hi)), finest_resolution=1024).to(gpu)
    meta = emb._meta
    xt, dt = torch.from_numpy(x).to(gpu), torch.from_numpy(dfeat).to(gpu)
    lib = _lib.load()

    def run(det):
        nbytes = int(lib.nerf_hash_encode_bwd_workspace_bytes(16, 19, P, det))
        ws = torch.empty(nbytes, dtype=torch.uint8, device=gpu)
        ws.fill_(0xA5)   # stale bytes must not matter
        g = [torch.zeros(1 << 19, 2, device=gpu) for _ in range(16)]
        _lib.call("nerf_hash_encode_bwd_ws", _lib.ptr(xt), P, meta["bmin"], meta["bmax"], meta["res"], 16, 19,
                  _lib.ptr(dt), 2, 2 * P, _lib.ptr_array(g), det, _lib.ptr(ws, dtype=torch.uint8), nbytes,
                  _lib.stream())
        torch.cuda.synchronize()
        return g

    a, b, plain = run(1), run(1), run(0)
    for lvl in range(16):
        assert torch.equal(a[lvl], b[lvl]), f"level {lvl}: deterministic runs differ"
    assert not a[5].any()
    xc = torch.from_numpy(x)
    bmin, bmax = torch.from_numpy(lo), torch.from_numpy(hi)
    for lvl in (0, 7, 15):
        vmin, vmax, idx, _ = oracle.voxel_corners(xc, bmin, bmax, torch.tensor(emb.level_res[lvl]), 19)
        w = ((xc - vmin) / (vmax - vmin)).double()
        wx, wy, wz = w[:, 0:1], w[:, 1:2], w[:, 2:3]
        gl = torch.from_numpy(dfeat[lvl]).double()
        contrib = []
        for c in range(8):
            i, j, k = (c >> 2) & 1, (c >> 1) & 1, c & 1
            contrib.append(gl * ((wz if k else 1 - wz) * (wy if j else 1 - wy) * (wx if i else 1 - wx)))
        contrib = torch.stack(contrib, 1).reshape(-1, 2)
        ref = torch.zeros(1 << 19, 2, dtype=torch.float64).index_add_(0, idx.reshape(-1), contrib)
        scale = torch.zeros(1 << 19, 2, dtype=torch.float64).index_add_(0, idx.reshape(-1), contrib.abs())
        for name, got in (("deterministic", a), ("default", plain)):
            err = (got[lvl].cpu().double() - ref).abs()
            bad = err > 2e-6 * scale + 1e-30
            assert not bool(bad.any()), f"{name} level {lvl}: {int(bad.sum())} rows off"
        # the fixed-point sums add no rounding of their own (~2^-75 of the level's largest entry);
        # what remains is the fp32 weight products and the in-wave run merge, shared with the default
        e_det = (a[lvl].cpu().double() - ref).abs().sum()
        e_def = (plain[lvl].cpu().double() - ref).abs().sum()
        assert float(e_det) <= 1.05 * float(e_def) + 1e-30, f"level {lvl}: {float(e_det):.3e} vs {float(e_def):.3e}"


def test_mlp_bwd_batch_deterministic(nerf, gpu):
    from indoor_nerf_amd import _lib, field
    torch.manual_seed(5)
    nets = [nerf.NeRFSmall(2, 64, 15, 3, 64, 32, 16).to(gpu) for _ in range(2)]
    sizes = (786432, 262144)
    feats = [torch.randn(16, P, 2, device=gpu) * 0.3 for P in sizes]
    spr = (192, 64)
    vd = torch.nn.functional.normalize(torch.randn(4096, 3, device=gpu), dim=-1)
    graws = [torch.randn(P, 4, device=gpu) for P in sizes]
    ws = torch.empty(int(_lib.load().nerf_mlp_bwd_det_workspace_bytes()) // 4, device=gpu)

    def run(det):
        for n in nets:
            for p in n.parameters():
                p.grad = None
        jobs = (_lib.MlpBwdJob * 2)()
        dfs = []
        for k, (n, P) in enumerate(zip(nets, sizes)):
            df = torch.empty(16, P, 2, device=gpu)
            dfs.append(df)
            j = jobs[k]
            j.feat, j.feat_stride_point, j.feat_stride_level = _lib.ptr(feats[k]), 2, 2 * P
            j.viewdirs, j.samples_per_ray, j.n_points = _lib.ptr(vd), spr[k], P
            j.weights = field._weights_struct(n.mlp_weights())
            j.graw = _lib.ptr(graws[k])
            j.grads = field._grads_struct(n.mlp_weights())
            j.dfeat = _lib.ptr(df)
        _lib.call("nerf_mlp_bwd_batch", jobs, 2, _lib.ptr(ws) if det else None, ws.numel() * 4 if det else 0,
                  _lib.stream())
        torch.cuda.synchronize()
        return [p.grad.clone() for n in nets for p in n.mlp_weights()], dfs

    g1, d1 = run(True)
    g2, d2 = run(True)
    g3, d3 = run(False)
    for x, y in zip(g1 + d1, g2 + d2):
        assert torch.equal(x, y)
    for x, y in zip(d1, d3):
        assert torch.equal(x, y)   # the input gradients never involve a cross-block sum
    for x, y in zip(g1, g3):
        torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-5 * float(y.abs().max()))


def test_mlp_bwd_batch_concurrent_streams_bitwise(nerf, gpu):
    """The C-ABI is stateless (SURVEY.md §8(b) Threading): two nerf_mlp_bwd_batch problems launched
    on two streams at once — small enough (96 blocks each) that their blocks run side by side on the
    256 CUs — give bit-identical results to the same launches run one after the other (deterministic
    mode, one reduction workspace per stream)."""
    from indoor_nerf_amd import _lib, field
    torch.manual_seed(11)
    sizes = (8192, 4096)
    spr = (192, 64)
    lib = _lib.load()

    def problem(seed):
        g = torch.Generator(device=gpu).manual_seed(seed)
        nets = [nerf.NeRFSmall(2, 64, 15, 3, 64, 32, 16).to(gpu) for _ in range(2)]
        feats = [torch.randn(16, P, 2, device=gpu, generator=g) * 0.3 for P in sizes]
        # ceil(P / spr) rays: 8192 points at 192 samples per ray end in a partial 43rd ray (a floor
        # here left its points reading past the view directions: garbage, and once a fault)
        vds = [torch.nn.functional.normalize(torch.randn(-(-P // s), 3, device=gpu, generator=g), dim=-1)
               for P, s in zip(sizes, spr)]
        graws = [torch.randn(P, 4, device=gpu, generator=g) for P in sizes]
        ws = torch.empty(int(lib.nerf_mlp_bwd_det_workspace_bytes()) // 4, device=gpu)
        return dict(nets=nets, feats=feats, vds=vds, graws=graws, ws=ws)

    def launch(pr, dfs, stream):
        jobs = (_lib.MlpBwdJob * 2)()
        for k, (n, P) in enumerate(zip(pr["nets"], sizes)):
            j = jobs[k]
            j.feat, j.feat_stride_point, j.feat_stride_level = _lib.ptr(pr["feats"][k]), 2, 2 * P
            j.viewdirs, j.samples_per_ray, j.n_points = _lib.ptr(pr["vds"][k]), spr[k], P
            j.weights = field._weights_struct(n.mlp_weights())
            j.graw = _lib.ptr(pr["graws"][k])
            j.grads = field._grads_struct(n.mlp_weights())
            j.dfeat = _lib.ptr(dfs[k])
        _lib.call("nerf_mlp_bwd_batch", jobs, 2, _lib.ptr(pr["ws"]), pr["ws"].numel() * 4,
                  _lib.c_vp(stream.cuda_stream))

    probs = [problem(100), problem(200)]

    def run(concurrent, reps=6):
        for pr in probs:
            for n in pr["nets"]:
                for p in n.parameters():
                    p.grad = None
        dfs = [[torch.empty(16, P, 2, device=gpu) for P in sizes] for _ in probs]
        # .grad buffers exist before the streams fork (accumulate_grad_buffers allocates them)
        for pr in probs:
            for n in pr["nets"]:
                field._grads_struct(n.mlp_weights())
        torch.cuda.synchronize()
        streams = [torch.cuda.Stream(device=gpu) for _ in probs]
        for _ in range(reps):
            if concurrent:
                for pr, df, s in zip(probs, dfs, streams):
                    launch(pr, df, s)
            else:
                for pr, df, s in zip(probs, dfs, streams):
                    launch(pr, df, s)
                    s.synchronize()
        torch.cuda.synchronize()
        return [p.grad.clone() for pr in probs for n in pr["nets"] for p in n.mlp_weights()] + \
            [d.clone() for df in dfs for d in df]

    serial = run(False)
    for _ in range(3):
        conc = run(True)
        for x, y in zip(serial, conc):
            assert torch.equal(x, y), "concurrent MLP backwards on two streams differ from serial execution"


def test_train_iteration_bitwise_reproducible(nerf, gpu):
    from indoor_nerf_amd import model
    lo, hi = blender_bbox()
    args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), finest_res=1024, N_samples=64,
                          N_importance=128, white_bkgd=True, tv_loss_weight=1e-6)
    torch.manual_seed(0)
    kw, _, _, grad_vars, opt = nerf.create_nerf(args, device=gpu)
    kw.update(near=2.0, far=6.0, pytest=True)
    with torch.no_grad():   # a trained-like table: sigma and the fine samples are not degenerate
        tab = closed_form_table(scale=0.2, salt=4)
        for i, e in enumerate(kw["embed_fn"].embeddings):
            e.weight.copy_(torch.from_numpy(tab[i]))
    ro, rd = synthetic_rays(4096, seed=12)
    rays = (torch.from_numpy(ro).to(gpu), torch.from_numpy(rd).to(gpu))
    target = torch.rand(4096, 3, device=gpu, generator=torch.Generator(device=gpu).manual_seed(3))

    def grads(det):
        nerf.set_deterministic(det)
        try:
            model.forward_backward(rays, target, kw, opt, args, 1, tv_generator=torch.Generator().manual_seed(5))
            torch.cuda.synchronize()
            return [p.grad.clone() for p in grad_vars + list(kw["embed_fn"].parameters())]
        finally:
            nerf.set_deterministic(False)

    a, b, c = grads(True), grads(True), grads(False)
    for i, (x, y) in enumerate(zip(a, b)):
        assert torch.equal(x, y), f"parameter {i}: deterministic iterations differ"
    for x, y in zip(a, c):
        assert float((x - y).norm()) <= 1e-3 * float(y.norm()) + 1e-12


def test_deferred_table_zero_bitwise(nerf, gpu):
    """GradArena(defer_tables=True): the tables' memset is skipped and the iteration's owner pass
    stores every row (NERF_OWNER_OVERWRITE). Deterministic mode, so the comparison is bitwise: the
    gradients equal the memset + accumulate path's, stale table gradients do not leak in, and a
    second backward without zeroing still accumulates."""
    from indoor_nerf_amd import model
    from indoor_nerf_amd.dist import GradArena
    lo, hi = blender_bbox()
    args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), finest_res=1024, N_samples=64,
                          N_importance=128, white_bkgd=True, tv_loss_weight=1e-6)
    torch.manual_seed(0)
    kw, _, _, grad_vars, opt = nerf.create_nerf(args, device=gpu)
    kw.update(near=2.0, far=6.0, pytest=True)
    with torch.no_grad():
        tab = closed_form_table(scale=0.2, salt=4)
        for i, e in enumerate(kw["embed_fn"].embeddings):
            e.weight.copy_(torch.from_numpy(tab[i]))
    ro, rd = synthetic_rays(2048, seed=13)
    rays = (torch.from_numpy(ro).to(gpu), torch.from_numpy(rd).to(gpu))
    target = torch.rand(2048, 3, device=gpu, generator=torch.Generator(device=gpu).manual_seed(4))
    params = [p for g in opt.param_groups for p in g["params"]]

    def grads(defer, passes):
        arena = GradArena(params, defer_tables=defer)
        arena.flat.fill_(7.0)             # stale gradients everywhere
        assert (len(arena.deferred) == 16) == defer
        for k in range(passes):           # the zero inside the first iteration's scope (_lib.zero_deferral)
            model.forward_backward(rays, target, kw, opt, args, 1, tv_generator=torch.Generator().manual_seed(5),
                                   zero_grad=arena.zero_ if k == 0 else (lambda: None))
        torch.cuda.synchronize()
        return [p.grad.clone() for p in params]

    nerf.set_deterministic(True)
    try:
        ref, got = grads(False, 1), grads(True, 1)
        ref2, got2 = grads(False, 2), grads(True, 2)
    finally:
        nerf.set_deterministic(False)
    from indoor_nerf_amd import hashgrid
    assert not hashgrid._DEFERRED
    for i, (x, y) in enumerate(zip(ref + ref2, got + got2)):
        assert torch.equal(x, y), f"gradient {i % len(params)} differs ({'two passes' if i >= len(params) else 'one pass'})"
    assert any(bool(g.any()) for g in got[-16:])


def test_deferred_table_zero_other_writers(nerf, gpu):
    """Deferred table gradients reaching a writer other than the binned owner pass are zeroed first:
    2^20-row tables have no binned plan (the memory-side atomic path accumulates), and a backward
    that never reaches the tables leaves them to hashgrid.materialize_zero()."""
    from indoor_nerf_amd import hashgrid
    from indoor_nerf_amd.dist import GradArena
    lo, hi = blender_bbox()
    emb = nerf.HashEmbedder((torch.from_numpy(lo), torch.from_numpy(hi)), finest_resolution=1024,
                            log2_hashmap_size=20).to(gpu)
    rng = np.random.RandomState(3)
    x = torch.from_numpy((lo + (hi - lo) * rng.rand(4096, 3)).astype(np.float32)).to(gpu)
    w = torch.from_numpy(rng.randn(4096, 32).astype(np.float32)).to(gpu)
    params = list(emb.parameters())
    ref_arena = GradArena(params)
    ref_arena.zero_()
    (emb(x)[0] * w).sum().backward()
    ref = [p.grad.clone() for p in params]
    from indoor_nerf_amd import _lib
    arena = GradArena(params, defer_tables=True)
    assert len(arena.deferred) == 16
    arena.flat.fill_(7.0)
    with _lib.zero_deferral():          # as inside a training iteration
        arena.zero_()
    assert len(hashgrid._DEFERRED) == 16
    (emb(x)[0] * w).sum().backward()
    torch.cuda.synchronize()
    for a, b in zip(ref, params):
        torch.testing.assert_close(b.grad, a, rtol=1e-5, atol=1e-7)
    assert not hashgrid._DEFERRED
    arena.flat.fill_(7.0)
    with _lib.zero_deferral():
        arena.zero_()                   # no backward reaches the tables this time
    hashgrid.materialize_zero()
    assert all(not bool(p.grad.any()) for p in params)


def test_arena_zero_outside_a_step_is_immediate(nerf, gpu):
    """GradArena(defer_tables=True).zero_() called by user code (outside model.forward_backward's
    zero_deferral scope) leaves no fill pending: the gradients read zero as soon as it returns, and no
    later launch on any device takes their ranges."""
    from indoor_nerf_amd import _lib, hashgrid
    from indoor_nerf_amd.dist import GradArena
    lo, hi = blender_bbox()
    emb = nerf.HashEmbedder((torch.from_numpy(lo), torch.from_numpy(hi)), finest_resolution=1024).to(gpu)
    net = nerf.NeRFSmall(2, 64, 15, 3, 64, 32, 16).to(gpu)
    params = list(net.parameters()) + list(emb.parameters())
    arena = GradArena(params, defer_tables=True)
    assert len(arena.deferred) == 16 and arena.zero_end > 0
    arena.flat.fill_(7.0)
    arena.zero_()
    assert not any(_lib._ZERO_FILLS.values()) and not hashgrid._DEFERRED
    assert all(not bool(p.grad.any()) for p in params)
    # inside a step's scope the same call defers: the dense part waits for render()'s first launch
    arena.flat.fill_(7.0)
    with _lib.zero_deferral():
        arena.zero_()
    assert sum(len(v) for v in _lib._ZERO_FILLS.values()) == 1 and len(hashgrid._DEFERRED) == 16
    hashgrid.materialize_zero()
    assert not any(_lib._ZERO_FILLS.values()) and not hashgrid._DEFERRED
    assert all(not bool(p.grad.any()) for p in params)


def test_check_numerics_flags_nan_and_inf(nerf, gpu):
    t = {"rgb_map": torch.rand(4096, 3, device=gpu), "depth_map": torch.rand(4096, device=gpu),
         "acc_map": torch.rand(1000, device=gpu), "weights": torch.zeros(0, device=gpu)}
    assert nerf.check_numerics(t) == []
    t["depth_map"][4000] = float("nan")
    t["acc_map"][3] = float("inf")
    assert nerf.check_numerics(t) == ["depth_map", "acc_map"]
    import importlib
    render = importlib.import_module("indoor_nerf_amd.render")   # the module (the package re-exports render())
    lo, hi = blender_bbox()
    args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), finest_res=1024, N_samples=64,
                          N_importance=64, white_bkgd=True)
    kw, _, _, _, _ = nerf.create_nerf(args, device=gpu)
    kw.update(near=2.0, far=6.0)
    ro, rd = synthetic_rays(256, seed=2)
    nerf.set_debug(True)
    assert render.DEBUG
    try:   # the hook runs inside render_rays (run_nerf.py:545-547) and reports nothing for finite outputs
        with torch.no_grad():
            out = nerf.render(800, 800, None, rays=(torch.from_numpy(ro).to(gpu), torch.from_numpy(rd).to(gpu)), **kw)
        assert nerf.check_numerics({"rgb_map": out[0], "acc_map": out[2]}) == []
    finally:
        nerf.set_debug(False)


def test_saved_h3_matches_recompute_bitwise(nerf, gpu):
    """The training forward's saved C1 outputs (nerf_mlp_fwd_h3, the backward job's h3) against the
    backward's own recompute of layer C1: one deterministic training iteration (both nets, coarse-
    feature reuse, TV) gives bit-identical gradients of every parameter, and the render outputs are
    the same bits (the forward's h3 is the same fwd_chain arithmetic as the recompute's)."""
    from indoor_nerf_amd import field, model
    lo, hi = blender_bbox()
    args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), finest_res=1024, N_samples=64,
                          N_importance=128, white_bkgd=True, tv_loss_weight=1e-6)
    torch.manual_seed(0)
    kw, _, _, grad_vars, opt = nerf.create_nerf(args, device=gpu)
    kw.update(near=2.0, far=6.0, pytest=True)
    with torch.no_grad():
        tab = closed_form_table(scale=0.2, salt=4)
        for i, e in enumerate(kw["embed_fn"].embeddings):
            e.weight.copy_(torch.from_numpy(tab[i]))
    ro, rd = synthetic_rays(4096, seed=13)
    rays = (torch.from_numpy(ro).to(gpu), torch.from_numpy(rd).to(gpu))
    target = torch.rand(4096, 3, device=gpu, generator=torch.Generator(device=gpu).manual_seed(3))
    calls = []
    orig = nerf._lib.call

    def spy(name, *a):
        if name == "nerf_mlp_bwd_batch":   # the jobs' h3 pointers
            calls.append([bool(a[0][k].h3) for k in range(a[1])])
        return orig(name, *a)

    def run(save):
        field.set_save_h3(save)
        nerf.set_deterministic(True)
        nerf._lib.call = spy
        try:
            loss = model.forward_backward(rays, target, kw, opt, args, 1,
                                          tv_generator=torch.Generator().manual_seed(5))[0]
            torch.cuda.synchronize()
            return float(loss), [p.grad.clone() for p in grad_vars + list(kw["embed_fn"].parameters())]
        finally:
            nerf._lib.call = orig
            nerf.set_deterministic(False)
            field.set_save_h3(True)

    la, a = run(True)
    assert calls == [[True, True]]          # both nets' backward read the saved h3
    lb, b = run(False)
    assert calls[1:] == [[False, False]]
    assert la == lb
    for i, (x, y) in enumerate(zip(a, b)):
        assert torch.equal(x, y), f"parameter {i}: saved-h3 backward differs from the recompute"


@pytest.mark.parametrize("det", [True, False], ids=["deterministic", "default"])
def test_tv_bins_in_hash_bin_launch(nerf, gpu, det):
    """The pass's TV bins inside the hash bin launch (nerf_hash_encode_bwd_bin_batch_tv, the TV blocks in
    front) against their own nerf_tv_bwd_bin launch: same workspace chunks, so one training iteration
    (both nets, coarse-feature reuse, TV) gives bit-identical gradients in deterministic mode, and
    gradients within the owner's summation-order rounding (fp64 LDS sums, one fp32 rounding: 1e-6 of
    each table's largest) in the default mode."""
    from indoor_nerf_amd import hashgrid, model
    lo, hi = blender_bbox()
    args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), finest_res=1024, N_samples=64,
                          N_importance=128, white_bkgd=True, tv_loss_weight=1e-2)
    torch.manual_seed(0)
    kw, _, _, grad_vars, opt = nerf.create_nerf(args, device=gpu)
    kw.update(near=2.0, far=6.0, pytest=True)
    with torch.no_grad():
        tab = closed_form_table(scale=0.2, salt=4)
        for i, e in enumerate(kw["embed_fn"].embeddings):
            e.weight.copy_(torch.from_numpy(tab[i]))
    ro, rd = synthetic_rays(4096, seed=13)
    rays = (torch.from_numpy(ro).to(gpu), torch.from_numpy(rd).to(gpu))
    target = torch.rand(4096, 3, device=gpu, generator=torch.Generator(device=gpu).manual_seed(3))
    calls = []
    orig = nerf._lib.call

    def spy(name, *a):
        if name in ("nerf_hash_encode_bwd_bin_batch_tv", "nerf_tv_bwd_bin", "nerf_hash_encode_bwd_bin_batch"):
            calls.append(name)
        return orig(name, *a)

    def run(fused):
        hashgrid.set_tv_in_bins(fused)
        nerf.set_deterministic(det)
        nerf._lib.call = spy
        calls.clear()
        try:
            loss = model.forward_backward(rays, target, kw, opt, args, 1,
                                          tv_generator=torch.Generator().manual_seed(5))[0]
            torch.cuda.synchronize()
            return float(loss), list(calls), [p.grad.clone() for p in grad_vars + list(kw["embed_fn"].parameters())]
        finally:
            nerf._lib.call = orig
            nerf.set_deterministic(False)
            hashgrid.set_tv_in_bins(True)

    la, ca, a = run(True)
    assert ca == ["nerf_hash_encode_bwd_bin_batch_tv"]
    lb, cb, b = run(False)
    assert cb == ["nerf_tv_bwd_bin", "nerf_hash_encode_bwd_bin_batch"]
    # the loss: the TV forward's per-level block sums meet in float atomics (either mode)
    assert abs(la - lb) <= 1e-6 * abs(lb)
    for i, (x, y) in enumerate(zip(a, b)):
        if det:
            assert torch.equal(x, y), f"parameter {i}: TV bins in the hash bin launch differ"
        else:   # default mode: the MLP's weight-gradient atomics and the owner's fp64 LDS sums are unordered
            m = float(y.abs().max())
            assert float((x - y).abs().max()) <= 1e-6 * m, f"parameter {i}"
