"""create_nerf (PocketNeRF/run_nerf.py:218-344) and the training iteration of train()
(run_nerf.py:1007-1035, :1161-1162, :1289-1293) on this package's modules.

create_nerf keeps the reference's return value (render_kwargs_train, render_kwargs_test, start,
grad_vars, optimizer), dict keys, RAdam param groups and checkpoint reload; it fixes the HEAD bugs
listed in SURVEY.md §0.3 (predict_normals / use_quantization kwargs) by accepting the arguments.
"""
import os
from types import SimpleNamespace

import numpy as np
import torch

from .field import NeRFSmall, run_network
from .hashgrid import HashEmbedder, SHEncoder
from .losses import total_variation_all, train_loss, tv_accumulator, tv_forward_early
from .optim import RAdam
from .render import render
from . import _lib, hashgrid

DEFAULTS = dict(multires=10, i_embed=1, i_embed_views=2, multires_views=4, use_viewdirs=True, N_importance=0,
                N_samples=64, netchunk=1024 * 64, finest_res=512, log2_hashmap_size=19, lrate=5e-4,
                lrate_decay=250, perturb=1., white_bkgd=False, raw_noise_std=0., predict_normals=False,
                use_quantization=False, quantization_bits=8, use_acaq=False, target_metric=None, bit_penalty=1e-3,
                acaq_start_iter=1000, dataset_type="blender", no_ndc=False, lindisp=False,
                basedir="./logs/", expname="", ft_path=None, no_reload=True, sparse_loss_weight=1e-10,
                tv_loss_weight=1e-6, chunk=1024 * 32,
                # structural priors (run_nerf.py:683-703)
                use_structural_priors=False, depth_prior_weight=0.01, planarity_weight=0.005,
                manhattan_weight=0.002, normal_consistency_weight=0.001, structural_loss_start_iter=2000,
                structural_loss_ramp_iters=1000, overfitting_threshold=8.0, min_structural_weight=0.0001)


def make_args(**kw):
    d = dict(DEFAULTS)
    d.update(kw)
    return SimpleNamespace(**d)


def create_nerf(args, device=None):
    device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    get = lambda k: getattr(args, k, DEFAULTS.get(k))  # noqa: E731
    if get("i_embed") != 1 or get("i_embed_views") != 2:
        raise NotImplementedError("create_nerf: only the hash-grid (i_embed=1) + SH (i_embed_views=2) model is "
                                  "built on the HIP path (the positional-encoding NeRF is out of scope)")
    if get("use_structural_priors") and not get("predict_normals"):
        args.predict_normals = True     # run_nerf.py:723-727: the priors need the normals head
    use_q, q_bits = get("use_quantization"), get("quantization_bits")
    embed_fn = HashEmbedder(bounding_box=args.bounding_box, log2_hashmap_size=get("log2_hashmap_size"),
                            finest_resolution=get("finest_res"), use_quantization=use_q,
                            quantization_bits=q_bits).to(device)
    embedding_params = list(embed_fn.parameters())
    embeddirs_fn = SHEncoder() if get("use_viewdirs") else None
    input_ch, input_ch_views = embed_fn.out_dim, (embeddirs_fn.out_dim if embeddirs_fn else 0)
    model = NeRFSmall(num_layers=2, hidden_dim=64, geo_feat_dim=15, num_layers_color=3, hidden_dim_color=64,
                      input_ch=input_ch, input_ch_views=input_ch_views, use_quantization=use_q,
                      quantization_bits=q_bits).to(device)
    grad_vars = list(model.parameters())
    model_fine = None
    if get("N_importance") > 0:
        model_fine = NeRFSmall(num_layers=2, hidden_dim=64, geo_feat_dim=15, num_layers_color=3, hidden_dim_color=64,
                               input_ch=input_ch, input_ch_views=input_ch_views, use_quantization=use_q,
                               quantization_bits=q_bits, predict_normals=get("predict_normals")).to(device)
        grad_vars += list(model_fine.parameters())
    netchunk = get("netchunk")
    network_query_fn = lambda inputs, viewdirs, network_fn: run_network(  # noqa: E731
        inputs, viewdirs, network_fn, embed_fn=embed_fn, embeddirs_fn=embeddirs_fn, netchunk=netchunk)
    optimizer = RAdam([{"params": grad_vars, "weight_decay": 1e-6},
                       {"params": embedding_params, "eps": 1e-15}], lr=get("lrate"), betas=(0.9, 0.99))
    start = 0
    basedir, expname = get("basedir"), get("expname")
    ft_path = get("ft_path")
    if ft_path is not None and ft_path != "None":
        ckpts = [ft_path]
    elif basedir and expname and os.path.isdir(os.path.join(basedir, expname)):
        ckpts = [os.path.join(basedir, expname, f) for f in sorted(os.listdir(os.path.join(basedir, expname)))
                 if "tar" in f]
    else:
        ckpts = []
    if len(ckpts) > 0 and not get("no_reload"):
        ckpt = torch.load(ckpts[-1], map_location=device, weights_only=True)
        start = ckpt["global_step"]
        optimizer.load_state_dict(ckpt["optimizer_state_dict"])
        model.load_state_dict(ckpt["network_fn_state_dict"])
        if model_fine is not None:
            model_fine.load_state_dict(ckpt["network_fine_state_dict"])
        embed_fn.load_state_dict(ckpt["embed_fn_state_dict"])
    render_kwargs_train = {
        "network_query_fn": network_query_fn, "perturb": get("perturb"), "N_importance": get("N_importance"),
        "network_fine": model_fine, "N_samples": get("N_samples"), "network_fn": model, "embed_fn": embed_fn,
        "use_viewdirs": get("use_viewdirs"), "white_bkgd": get("white_bkgd"), "raw_noise_std": get("raw_noise_std"),
        "predict_normals": get("predict_normals"),
    }
    if get("dataset_type") != "llff" or get("no_ndc"):
        render_kwargs_train["ndc"] = False
        render_kwargs_train["lindisp"] = get("lindisp")
    render_kwargs_test = dict(render_kwargs_train)
    render_kwargs_test["perturb"] = False
    render_kwargs_test["raw_noise_std"] = 0.
    return render_kwargs_train, render_kwargs_test, start, grad_vars, optimizer


def save_checkpoint(path, global_step, render_kwargs_train, optimizer, sharded=None, write_rank=0):
    """The reference's checkpoint dict (run_nerf.py:1345-1362), written by one process.

    With a dist.ShardedOptimizer this is a COLLECTIVE call: EVERY rank must call it (the moment
    shards are assembled into full tensors with one all-reduce first), and only rank `write_rank`
    writes the file; a call on one rank alone would wait forever for the others. Without sharding
    any rank may call it on its own. Returns True on the rank that wrote."""
    rank = 0
    if sharded is not None:
        import torch.distributed as dist
        if sharded.world > 1 and not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("save_checkpoint(sharded=...): torch.distributed is not initialised")
        sharded.consolidate_state()
        rank = sharded.rank
    if rank != write_rank:
        return False
    fine = render_kwargs_train["network_fine"]
    torch.save({"global_step": global_step,
                "network_fn_state_dict": render_kwargs_train["network_fn"].state_dict(),
                "network_fine_state_dict": fine.state_dict() if fine is not None else None,
                "embed_fn_state_dict": render_kwargs_train["embed_fn"].state_dict(),
                "optimizer_state_dict": optimizer.state_dict()}, path)
    return True


def acaq_quantizers(render_kwargs_train):
    """The quantizers the A-CAQ loop adjusts, in the reference's order (run_nerf.py:1184-1194): the
    embedder's 16 levels, then the COARSE network's activation and weight quantizers."""
    qs = []
    emb, net = render_kwargs_train["embed_fn"], render_kwargs_train["network_fn"]
    if getattr(emb, "quantizers", None) is not None:
        qs.extend(emb.quantizers)
    if getattr(net, "sigma_act_quantizers", None) is not None:
        qs.extend(net.sigma_act_quantizers)
    if getattr(net, "sigma_weight_quantizer", None) is not None:
        qs.append(net.sigma_weight_quantizer)
    return qs


def acaq_update(i, img_loss, render_kwargs_train, args):
    """A-CAQ bit-width controller of train() (run_nerf.py:1182-1250), after optimizer.step():
    from acaq_start_iter, every 10th iteration each quantizer's soft_bits moves by a loss-driven
    delta minus a bit penalty (csrc/quant.hip acaq_update_kernel; no host sync). The best img_loss
    of the MDL mode (the reference's train.best_loss) lives on the device next to the embedder.
    Returns the device report [target, loss_ratio] of an update, else None."""
    get = lambda k, d=None: getattr(args, k, DEFAULTS.get(k, d))  # noqa: E731
    if not (get("use_acaq", False) and get("use_quantization") and i >= get("acaq_start_iter", 1000)):
        return None
    if i % 10 != 0:
        return None
    qs = acaq_quantizers(render_kwargs_train)
    if not qs:
        return None
    from .quantization import _descriptors
    emb = render_kwargs_train["embed_fn"]
    dev = img_loss.device
    if getattr(emb, "_acaq_best", None) is None or emb._acaq_best.device != dev:
        emb._acaq_best = torch.full((1,), float("nan"), dtype=torch.float64, device=dev)
    report = torch.empty(2, dtype=torch.float64, device=dev)
    tm = get("target_metric", None)
    loss32 = img_loss.detach().reshape(()).float().contiguous().clone()
    from .dist import allreduce_mean_
    allreduce_mean_(loss32)        # DP: every replica's controller sees the global batch's loss
    _lib.call("nerf_acaq_update", _descriptors(qs), len(qs), _lib.ptr(loss32, "img_loss"),
              _lib.ptr(emb._acaq_best, "best_loss", dtype=torch.float64), int(tm is not None),
              float(tm) if tm is not None else 0.0, float(get("bit_penalty", 1e-3)),
              _lib.ptr(report, "report", dtype=torch.float64), _lib.stream())
    for q in qs:
        torch.autograd.graph.increment_version(q.soft_bits)
    return report


def forward_backward(batch_rays, target_s, render_kwargs_train, optimizer, args, global_step, H=0, W=0, K=None,
                     loss_scale_sparsity=1.0, tv_generator=None, zero_grad=None, schedule=True, spatial_coords=None):
    """render (coarse+fine), zero grads, img/img0 MSE + sparsity + TV (run_nerf.py:1007-1037),
    backward. Returns (loss, img_loss, psnr) device tensors (no host sync)."""
    with _lib.zero_deferral():
        return _forward_backward(batch_rays, target_s, render_kwargs_train, optimizer, args, global_step, H, W, K,
                                 loss_scale_sparsity, tv_generator, zero_grad, schedule, spatial_coords)


def _forward_backward(batch_rays, target_s, render_kwargs_train, optimizer, args, global_step, H, W, K,
                      loss_scale_sparsity, tv_generator, zero_grad, schedule, spatial_coords):
    get = lambda k: getattr(args, k, DEFAULTS.get(k))  # noqa: E731
    # the gradient zero and the TV loss accumulator first: a GradArena(defer_tables=True) zero and the
    # accumulator's fill are then stores in render()'s first launch (_lib.defer_fill_zero), not fills.
    # Equivalent to the reference's render -> zero_grad order: the forward touches no gradient
    if zero_grad is None:
        optimizer.zero_grad()
    else:
        zero_grad()
    tv_w = get("tv_loss_weight")
    tv_acc = tv_accumulator(render_kwargs_train["embed_fn"]) if tv_w > 0 else None
    # a captured step's TV forward runs inside the fine compositing launch (corners drawn after render)
    tv_early = tv_forward_early(render_kwargs_train["embed_fn"], tv_acc) if tv_w > 0 else None
    rgb, depth, acc, extras = render(H, W, K, chunk=get("chunk"), rays=batch_rays, retraw=True,
                                     **render_kwargs_train)
    # run_nerf.py:1011-1037 (img2mse x2, sparsity, TV, mse2psnr) fused into one launch (csrc/loss.hip)
    tv = (total_variation_all(render_kwargs_train["embed_fn"], generator=tv_generator, out=tv_acc, early=tv_early)
          if tv_w > 0 else None)
    loss, img_loss, psnr = train_loss(rgb, extras.get("rgb0"), target_s, extras.get("sparsity_loss"),
                                      extras.get("sparsity_loss0"), tv, get("sparse_loss_weight") * loss_scale_sparsity,
                                      tv_w if tv_w > 0 else 0.0)
    if schedule and global_step > 1000:
        args.tv_loss_weight = 0.0
    if get("use_structural_priors") and global_step >= get("structural_loss_start_iter"):
        loss = structural_loss(depth, extras, args, global_step, spatial_coords, addend=loss)
    _lib.flush_zero_fills()       # fills no launch took (render() without rays to pack)
    loss.backward(_unit_seed(loss))
    hashgrid.materialize_zero()   # table gradients whose deferred zero no owner pass consumed
    return loss, img_loss, psnr


_SEEDS = {}


def _unit_seed(loss):
    """d loss / d loss = 1 from a persistent device tensor: loss.backward() would launch a fill
    kernel for it every iteration (and capture one into the step graph)."""
    key = (loss.device, loss.dtype, tuple(loss.shape))
    seed = _SEEDS.get(key)
    if seed is None:
        seed = _SEEDS[key] = torch.ones_like(loss, memory_format=torch.contiguous_format)
    return seed


def fused_priors_eligible(args, n_rays):
    """True when structural_loss takes the device path (priors.fused_structural_losses): no host
    synchronisation, so graphs.GraphedTrainStep may capture the iteration. The one test both use:
    args.fused_priors (default True), the normals head present (predict_normals) and
    1 <= n_rays <= PRIORS_MAX_RAYS; anything else runs the eager torch path, which branches on host
    counts and cannot be captured."""
    get = lambda k: getattr(args, k, DEFAULTS.get(k))  # noqa: E731
    return (bool(getattr(args, "fused_priors", True)) and bool(get("predict_normals"))
            and 1 <= int(n_rays) <= _lib.PRIORS_MAX_RAYS)


def structural_loss(depth, extras, args, global_step, spatial_coords=None, addend=None):
    """run_nerf.py:1068-1131: the structural-prior weights ramp from 10 % to 100 % over
    structural_loss_ramp_iters, then combine_structural_losses_v2 on the fine pass's depth and normal
    maps. Default: the device path (priors.fused_structural_losses, csrc/priors_fused.hip: no host
    synchronisation, so graphs.GraphedTrainStep captures these iterations too; the ramp is a device
    scalar, a per-step graph slot under capture). args.fused_priors = False selects the eager torch
    path (priors.combine_structural_losses_v2, the reference's RNG draws; its estimators persist
    across iterations, run_nerf.py:939-940). The overfitting-driven weight reduction (:1073-1094)
    needs train()'s test-set PSNR history and is left to the caller. Failures are swallowed as in
    the reference (:1144-1148). addend (the iteration's other losses): returns addend + the structural
    loss (the device path forms the sum in its loss launch)."""
    from . import graphs
    from .priors import (ManhattanFrameEstimator, SemanticPlaneDetector, combine_structural_losses_v2,
                         fused_structural_losses)
    get = lambda k: getattr(args, k, DEFAULTS.get(k))  # noqa: E731
    start = get("structural_loss_start_iter")
    ramp_of = lambda step: 0.1 + 0.9 * min(1.0, (step - start) / get("structural_loss_ramp_iters"))  # noqa: E731
    base = {"depth_prior": get("depth_prior_weight"), "planarity": get("planarity_weight"),
            "manhattan": get("manhattan_weight"), "normal_consistency": get("normal_consistency_weight")}
    normals = extras.get("normal_map", None) if get("predict_normals") else None
    if normals is not None and fused_priors_eligible(args, depth.shape[0]):
        sc = graphs.active()
        if sc is not None:   # captured: the ramp of the replayed step, written before every replay
            import weakref
            off, ptr = sc.alloc_f32(1)
            sc_ref = weakref.ref(sc)   # no StepScalars <-> filler cycle: the ring is freed with its graph

            def fill(hi, hf, off=off):
                hf[off] = ramp_of(sc_ref().step)
            sc.add_filler(fill)
            scale = sc.dev_f[off:off + 1]
        else:
            scale = torch.full((1,), ramp_of(global_step), device=depth.device)
        total, _ = fused_structural_losses(depth, normals, spatial_coords, base, 0.4, 0.5, scale=scale, addend=addend)
        return total
    if getattr(args, "_priors", None) is None:
        args._priors = (ManhattanFrameEstimator(confidence_threshold=0.4), SemanticPlaneDetector(normal_threshold=0.5))
    ramp = ramp_of(global_step)
    weights = {k: v * ramp for k, v in base.items()}
    try:
        total, _ = combine_structural_losses_v2(depth, normals, extras.get("rays_d"), spatial_coords, weights,
                                                *args._priors)
    except Exception as e:   # noqa: BLE001 - the reference's policy
        print(f"  ⚠️  Structural priors V2 failed: {e}")
        total = 0.0
    return total if addend is None else addend + total


def structural_overfit_update(args, global_step, psnr_list):
    """train()'s overfitting-driven reduction of the structural-prior weights (run_nerf.py:1072-1094),
    a host-side step of the training loop: every 500 iterations from structural_loss_start_iter + 500
    on, when more than 50 training PSNRs are recorded and the mean of the last 20 exceeds
    args._last_test_psnr by more than args.overfitting_threshold, the four weights are multiplied by
    0.7 (floored at args.min_structural_weight). Returns True when it reduced them. The reference
    reads args._last_test_psnr only through hasattr and never sets it, so in its own train() this
    never fires; a caller that records its test PSNR there gets the reduction. Under
    graphs.GraphedTrainStep the weights are part of the launch-structure key: a reduction re-captures."""
    get = lambda k: getattr(args, k, DEFAULTS.get(k))  # noqa: E731
    i = global_step
    if not (i > get("structural_loss_start_iter") + 500 and i % 500 == 0 and len(psnr_list) > 50):
        return False
    recent = float(np.mean(psnr_list[-20:]))
    if not hasattr(args, "_last_test_psnr") or recent - args._last_test_psnr <= get("overfitting_threshold"):
        return False
    floor = get("min_structural_weight")
    for k in ("depth_prior_weight", "planarity_weight", "manhattan_weight", "normal_consistency_weight"):
        setattr(args, k, max(floor, get(k) * 0.7))
    return True


def optimizer_update(optimizer):
    optimizer.step()


def lr_schedule(optimizer, args, global_step):
    """TV switch-off after 1000 iterations (run_nerf.py:1036-1037) and lr decay (:1289-1293)."""
    get = lambda k: getattr(args, k, DEFAULTS.get(k))  # noqa: E731
    if global_step > 1000:
        args.tv_loss_weight = 0.0
    decay_steps = get("lrate_decay") * 1000
    new_lrate = get("lrate") * (0.1 ** (global_step / decay_steps))
    for g in optimizer.param_groups:
        g["lr"] = new_lrate


def holds_owner(grad_hook):
    """True when grad_hook runs the step's held owner pass itself (dist.ShardedOptimizer.reduce_grads
    with overlap: the owner pass is launched bucket by bucket beside the reduce-scatters)."""
    return bool(getattr(getattr(grad_hook, "__self__", None), "overlap", False))


def train_step(batch_rays, target_s, render_kwargs_train, optimizer, args, global_step, H=0, W=0, K=None,
               grad_hook=None, loss_scale_sparsity=1.0, tv_generator=None, zero_grad=None, spatial_coords=None,
               post_hook=None):
    """One iteration of train() without host bookkeeping: render (coarse+fine), img/img0 MSE,
    sparsity, TV (run_nerf.py:1007-1037), backward, [grad_hook, e.g. DP all-reduce or reduce-scatter],
    RAdam step, [post_hook, e.g. the sharded optimizer's parameter all-gather], A-CAQ bit widths,
    lr decay (:1182-1250, :1289-1293). Returns (loss, psnr) as device tensors (no host sync).
    graphs.GraphedTrainStep replays the same iteration from HIP graphs."""
    with hashgrid.hold_owner(target_s.device, holds_owner(grad_hook)), \
            hashgrid.fused_table_step(target_s.device, optimizer, render_kwargs_train["embed_fn"].tables(),
                                      enabled=grad_hook is None):
        loss, img_loss, psnr = forward_backward(batch_rays, target_s, render_kwargs_train, optimizer, args,
                                                global_step, H=H, W=W, K=K, loss_scale_sparsity=loss_scale_sparsity,
                                                tv_generator=tv_generator, zero_grad=zero_grad,
                                                spatial_coords=spatial_coords)
    if grad_hook is not None:
        grad_hook()
    optimizer_update(optimizer)
    if post_hook is not None:
        post_hook()
    acaq_update(global_step, img_loss, render_kwargs_train, args)
    lr_schedule(optimizer, args, global_step)
    return loss.detach(), psnr.detach()
