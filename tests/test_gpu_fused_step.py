"""The hash tables' RAdam step fused into the iteration's owner pass (nerf_hash_encode_bwd_owner_step,
hashgrid.fused_table_step, RAdam.table_step) against the owner pass + the optimizer's own launch
(radam.py:28-94 restated in csrc/optim.hip). Both apply the same elementwise update (radam_elem,
hash_common.h) to the same fp32 gradient rows, so in deterministic mode (fixed-order MLP gradient sums,
fixed-point owner sums) every parameter, moment and step count is bit-identical after RAdam's moment-only
steps (1-5) and its adaptive ones (6+), eagerly and replayed from a HIP graph."""
import pytest
import torch

from tables import blender_bbox, synthetic_rays

pytestmark = pytest.mark.gpu


def _run(nerf, gpu, fused, graphed, steps, R=1024):
    from indoor_nerf_amd import hashgrid
    from indoor_nerf_amd.graphs import GraphedTrainStep
    lo, hi = blender_bbox()
    args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), finest_res=1024, N_samples=64,
                          N_importance=128, white_bkgd=True, perturb=1.0, tv_loss_weight=1e-6)
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
    p0 = [p.detach().clone() for p in params]
    arena = nerf.GradArena(params, defer_tables=True)     # the owner pass stores the tables' gradients
    nerf.manual_seed(99)
    tv_gen = torch.Generator().manual_seed(7)
    prev = hashgrid.fused_table_step_enabled()
    hashgrid.set_fused_table_step(fused)
    try:
        if graphed:
            st = GraphedTrainStep(rays, target, kw, opt, args, tv_generator=tv_gen, zero_grad=arena.zero_)
            for it in steps:
                st(it)
        else:
            for it in steps:
                nerf.train_step(rays, target, kw, opt, args, it, tv_generator=tv_gen, zero_grad=arena.zero_)
        torch.cuda.synchronize()
    finally:
        hashgrid.set_fused_table_step(prev)
    tabs = kw["embed_fn"].tables()
    state = [(opt.state[p]["step"], opt.state[p]["exp_avg"].clone(), opt.state[p]["exp_avg_sq"].clone()) for p in tabs]
    return [p.detach().clone() for p in params], [p.grad.clone() for p in tabs], state, p0


@pytest.mark.parametrize("graphed", [False, True], ids=["eager", "graphed"])
def test_fused_table_step_bitwise(nerf, gpu, graphed):
    nerf.set_deterministic(True)
    try:
        steps = list(range(1, 9))
        pa, ga, sa, p0 = _run(nerf, gpu, True, graphed, steps)
        pb, gb, sb, _ = _run(nerf, gpu, False, graphed, steps)
    finally:
        nerf.set_deterministic(False)
    for i, (a, b) in enumerate(zip(pa, pb)):
        assert torch.equal(a, b), f"parameter {i}"
    for a, b in zip(ga, gb):
        assert torch.equal(a, b)                       # .grad stays in place after the step
    for (na, ma, va), (nb, mb, vb) in zip(sa, sb):
        assert na == nb == len(steps)
        assert torch.equal(ma, mb) and torch.equal(va, vb)
    # the tables moved (RAdam's adaptive steps start at step 6)
    assert all(not torch.equal(a, b) for a, b in zip(pa[-16:], p0[-16:]))


def test_fused_table_step_is_taken(nerf, gpu):
    """train_step with the deferred table zero launches the owner pass with the step (the optimizer's
    own launch then covers the MLP tensors only) and advances the tables' step count once."""
    from indoor_nerf_amd import _lib, optim
    seen = []
    orig = optim.RAdam.table_step

    def spy(self, tables):
        s = orig(self, tables)
        seen.append(s is not None)
        return s
    optim.RAdam.table_step = spy
    try:
        _lib.set_timing(True)
        _run(nerf, gpu, True, False, [1, 2])
        names = [n for n, _, _ in _lib.timing_records()]
    finally:
        _lib.set_timing(False)
        optim.RAdam.table_step = orig
    assert seen == [True, True]
    assert names.count("nerf_hash_encode_bwd_owner_step") == 2 and names.count("nerf_radam_step") == 2


def _unfused_reference(nerf, opt, tables, pre, step, lr):
    """RAdam's own launch (nerf_radam_step) applied to the pre-step clones `pre` = [(p, m, v)] with the
    gradient rows the fused owner pass stored in the tables' .grad, at optimizer step `step` and the
    learning rate of that step (train_step's lr_schedule has moved the group's lr on since)."""
    from indoor_nerf_amd import _lib
    group = next(g for g in opt.param_groups if any(q is tables[0] for q in g["params"]))
    n_sma, step_size = opt._scalars(group, step)
    mode = 2 if n_sma >= 5 else (1 if step_size > 0 else 0)
    dc, stc = opt._coefs({**group, "lr": lr}, mode, step_size)
    beta1, beta2 = group["betas"]
    segs = []
    for t, (cp, cm, cv) in zip(tables, pre):
        s = _lib.RAdamSegment()
        s.p, s.g, s.m, s.v = (_lib.ptr(x).value for x in (cp, t.grad, cm, cv))
        s.n = t.numel()
        s.beta1, s.beta2, s.one_minus_beta1, s.one_minus_beta2 = beta1, beta2, 1 - beta1, 1 - beta2
        s.eps, s.decay_coef, s.step_coef, s.mode = group["eps"], dc, stc, mode
        segs.append(s)
    arr = (_lib.RAdamSegment * len(segs))(*segs)
    _lib.call("nerf_radam_step", arr, len(segs), None, _lib.stream())
    torch.cuda.synchronize()
    return mode


@pytest.mark.parametrize("log2_T", [19, 12], ids=["T2^19", "T2^12"])
@pytest.mark.parametrize("graphed", [False, True], ids=["eager", "graphed"])
def test_fused_table_step_default_mode_matches_radam_launch(nerf, gpu, graphed, log2_T):
    """Default (non-deterministic) mode, the production path: the owner pass's prefetching table step
    (hash_bwd_owner_kernel with the step on; with 2^12-row tables the partial-slice owner_table_step)
    against RAdam's own launch applied to clones of the pre-step parameters and moments with the very
    gradient rows the fused launch stored in .grad: parameters and both moments bit-identical, through
    the moment-only steps (1-5) and the adaptive ones (6+)."""
    from indoor_nerf_amd import hashgrid
    from indoor_nerf_amd.graphs import GraphedTrainStep
    lo, hi = blender_bbox()
    args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), finest_res=1024, N_samples=64,
                          N_importance=128, white_bkgd=True, perturb=1.0, tv_loss_weight=1e-6,
                          log2_hashmap_size=log2_T)
    torch.manual_seed(0)
    kw, _, _, grad_vars, opt = nerf.create_nerf(args, device=gpu)
    kw.update(near=2.0, far=6.0)
    with torch.no_grad():
        g = torch.Generator().manual_seed(5)
        for e in kw["embed_fn"].embeddings:
            e.weight.copy_((torch.rand(e.weight.shape, generator=g) * 2 - 1) * 0.05)
    R = 1024
    ro, rd = synthetic_rays(R, seed=21)
    rays = (torch.from_numpy(ro).to(gpu), torch.from_numpy(rd).to(gpu))
    target = torch.rand(R, 3, device=gpu, generator=torch.Generator(device=gpu).manual_seed(3))
    params = grad_vars + list(kw["embed_fn"].parameters())
    arena = nerf.GradArena(params, defer_tables=True)
    nerf.manual_seed(99)
    tv_gen = torch.Generator().manual_seed(7)
    tabs = kw["embed_fn"].tables()
    prev = hashgrid.fused_table_step_enabled()
    hashgrid.set_fused_table_step(True)
    modes = set()
    try:
        st = GraphedTrainStep(rays, target, kw, opt, args, tv_generator=tv_gen, zero_grad=arena.zero_) if graphed \
            else None
        for it in range(1, 10):
            torch.cuda.synchronize()
            pre = None
            lr = next(g for g in opt.param_groups if any(q is tabs[0] for q in g["params"]))["lr"]
            if it >= 2:   # state exists from the first step on
                pre = [(p.detach().clone(), opt.state[p]["exp_avg"].clone(), opt.state[p]["exp_avg_sq"].clone())
                       for p in tabs]
            if st is not None:
                st(it)
            else:
                nerf.train_step(rays, target, kw, opt, args, it, tv_generator=tv_gen, zero_grad=arena.zero_)
            torch.cuda.synchronize()
            if pre is None:
                continue
            assert hashgrid.last_fused_table_step() or graphed
            modes.add(_unfused_reference(nerf, opt, tabs, pre, opt.state[tabs[0]]["step"], lr))
            for lvl, (p, (cp, cm, cv)) in enumerate(zip(tabs, pre)):
                assert torch.equal(p.detach(), cp), f"iteration {it} level {lvl}: parameters"
                assert torch.equal(opt.state[p]["exp_avg"], cm), f"iteration {it} level {lvl}: exp_avg"
                assert torch.equal(opt.state[p]["exp_avg_sq"], cv), f"iteration {it} level {lvl}: exp_avg_sq"
    finally:
        hashgrid.set_fused_table_step(prev)
    assert modes == {0, 2}, modes   # moment-only steps and adaptive steps both covered
