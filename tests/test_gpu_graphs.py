"""The training iteration replayed from HIP graphs (graphs.GraphedTrainStep) against the eager
iteration (model.train_step) on identical models, rays and random streams.

Both paths draw the same Philox seeds (stratified jitter, importance uniforms) and TV cuboids in
the same order; the captured launches read them from device slots refreshed before each replay.
The only differences are fp32 atomics inside the backward kernels (summation order): losses agree
to 1e-5 relative, and each parameter tensor's distance from the eager one is ≤ 1e-3 of how far
RAdam moved it (Adam's m/sqrt(v) turns a rounding-level gradient difference on a near-zero-grad
table row into an O(lr) step, so an elementwise bound would measure the atomics, not the graph;
two eager runs differ the same way). The TV switch-off at iteration 1000 (run_nerf.py:1036-1037)
forces a re-capture that is checked the same way.
"""
import numpy as np
import pytest
import torch

from tables import blender_bbox, synthetic_rays

pytestmark = pytest.mark.gpu


def _setup(nerf, gpu, R=1024, **extra):
    lo, hi = blender_bbox()
    args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), finest_res=1024, N_samples=64,
                          N_importance=128, white_bkgd=True, perturb=1.0, **{"tv_loss_weight": 1e-6, **extra})
    torch.manual_seed(0)
    kw, _, _, grad_vars, opt = nerf.create_nerf(args, device=gpu)
    kw.update(near=2.0, far=6.0)
    with torch.no_grad():
        g = torch.Generator().manual_seed(5)
        for e in kw["embed_fn"].embeddings:
            e.weight.copy_((torch.rand(e.weight.shape, generator=g) * 2 - 1) * 0.05)
    ro, rd = synthetic_rays(R, seed=21)
    rays = (torch.from_numpy(ro).to(gpu), torch.from_numpy(rd).to(gpu))
    target = torch.rand(R, 3, device=gpu, generator=torch.Generator(device=gpu).manual_seed(3))
    params = grad_vars + list(kw["embed_fn"].parameters())
    arena = nerf.GradArena(params)
    return args, kw, opt, rays, target, params, arena


def _run(nerf, gpu, graphed, steps, **extra):
    from indoor_nerf_amd.graphs import GraphedTrainStep
    args, kw, opt, rays, target, params, arena = _setup(nerf, gpu, **extra)
    p0 = [p.detach().clone() for p in params]
    nerf.manual_seed(99)
    tv_gen = torch.Generator().manual_seed(7)
    losses = []
    if graphed:
        st = GraphedTrainStep(rays, target, kw, opt, args, tv_generator=tv_gen, zero_grad=arena.zero_)
        for it in steps:
            loss, _ = st(it)
            losses.append(loss.clone())
    else:
        st = None
        for it in steps:
            loss, _ = nerf.train_step(rays, target, kw, opt, args, it, tv_generator=tv_gen, zero_grad=arena.zero_)
            losses.append(loss.clone())
    torch.cuda.synchronize()
    return [float(l) for l in losses], [(p.detach().clone(), q) for p, q in zip(params, p0)], st, opt


def _check_params(pg, pe, rel=1e-3):
    for (a, a0), (b, b0) in zip(pg, pe):
        assert torch.equal(a0, b0)
        moved = float((b - b0).norm())
        d = float((a - b).norm())
        assert d <= rel * moved + 1e-7, (tuple(a.shape), d, moved)


def test_graphed_train_step_matches_eager(nerf, gpu):
    steps = list(range(1, 9))
    le, pe, _, oe = _run(nerf, gpu, False, steps)
    lg, pg, st, og = _run(nerf, gpu, True, steps)
    assert st.captures == 1, st.captures
    np.testing.assert_allclose(lg, le, rtol=1e-5)
    _check_params(pg, pe)
    # optimizer host state advanced identically (RAdam step count drives N_sma / step size)
    for ga, gb in zip(og.param_groups, oe.param_groups):
        for pa, pb in zip(ga["params"], gb["params"]):
            assert og.state[pa]["step"] == oe.state[pb]["step"] == len(steps)


def test_graphed_train_step_recaptures_at_tv_switch_off(nerf, gpu):
    steps = list(range(996, 1006))        # TV on through 1000, off afterwards
    le, pe, _, _ = _run(nerf, gpu, False, steps)
    lg, pg, st, _ = _run(nerf, gpu, True, steps)
    assert st.captures == 2, st.captures
    np.testing.assert_allclose(lg, le, rtol=1e-5)
    _check_params(pg, pe)


def test_graphed_tv_forward_fused_matches_eager(nerf, gpu):
    """The captured step runs its TV forward inside the fine pass's compositing launch
    (nerf_composite_fwd_tv; corners from the device slots, drawn after render as in the eager step)
    and no nerf_tv_fwd launch; with a TV weight that makes the TV a large share of the loss, the
    replays' losses and parameters match the eager steps (which launch nerf_tv_fwd after render)."""
    calls = []
    orig = nerf._lib.call

    def spy(name, *a):
        calls.append(name)
        return orig(name, *a)
    steps = list(range(1, 5))
    le, pe, _, _ = _run(nerf, gpu, False, steps, tv_loss_weight=1e-2)
    nerf._lib.call = spy
    try:
        lg, pg, st, _ = _run(nerf, gpu, True, steps, tv_loss_weight=1e-2)
    finally:
        nerf._lib.call = orig
    assert st.captures == 1
    assert "nerf_composite_fwd_tv" in calls and "nerf_tv_fwd" not in calls[calls.index("nerf_composite_fwd_tv"):]
    np.testing.assert_allclose(lg, le, rtol=1e-5)
    _check_params(pg, pe)


def test_timing_refused_inside_capture(nerf, gpu):
    """bench.py's HIP-event timing is eager-only: a capture with timing on fails loudly."""
    from indoor_nerf_amd import _lib
    from indoor_nerf_amd.graphs import GraphedTrainStep
    args, kw, opt, rays, target, params, arena = _setup(nerf, gpu, R=256)
    st = GraphedTrainStep(rays, target, kw, opt, args, zero_grad=arena.zero_, warmup=1)
    st(1)
    _lib.set_timing(True)
    try:
        with pytest.raises(RuntimeError):
            st(2)
    finally:
        _lib.set_timing(False)


def test_graph_replay_after_workspace_growth(nerf, gpu):
    """A captured iteration keeps the hash backward's bin workspace address in its kernel arguments:
    a larger eager backward in between grows the workspace, and the old one must stay valid (it is
    retired, never freed). Deterministic configuration (perturb 0, no TV): the replayed backward's
    gradients equal an eager backward's at the same parameters up to fp32 atomics order."""
    from indoor_nerf_amd.graphs import GraphedTrainStep
    from indoor_nerf_amd.model import forward_backward
    args, kw, opt, rays, target, params, arena = _setup(nerf, gpu, R=512)
    kw["perturb"] = 0.0
    args.tv_loss_weight = 0.0
    st = GraphedTrainStep(rays, target, kw, opt, args, zero_grad=arena.zero_)
    for it in range(1, 5):
        st(it)
    assert st.captures == 1
    # a 16x larger eager backward: the bin workspace grows past the captured one
    ro, rd = synthetic_rays(8192, seed=33)
    big = (torch.from_numpy(ro).to(gpu), torch.from_numpy(rd).to(gpu))
    big_t = torch.rand(8192, 3, device=gpu)
    forward_backward(big, big_t, kw, opt, args, 5, zero_grad=arena.zero_)
    junk = [torch.full((1 << 26,), 1e30, device=gpu) for _ in range(8)]   # grab freed blocks
    torch.cuda.synchronize()
    st.scalars.upload()
    st.graphs[0].replay()
    torch.cuda.synchronize()
    g_graph = arena.flat.clone()
    forward_backward(rays, target, kw, opt, args, 6, zero_grad=arena.zero_)
    torch.cuda.synchronize()
    g_eager = arena.flat.clone()
    del junk
    assert torch.isfinite(g_graph).all()
    scale = float(g_eager.abs().max())
    assert scale > 0
    assert float((g_graph - g_eager).abs().max()) <= 1e-4 * scale
