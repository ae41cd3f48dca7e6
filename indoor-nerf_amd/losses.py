"""Losses of the training step on the HIP kernels.

total_variation_loss mirrors PocketNeRF/loss.py:11-43 (one random hashed cuboid per level; the
cuboid corner is drawn with torch.randint on the host, like the reference). total_variation_all
runs all levels of a HashEmbedder in one forward and one backward launch (csrc/optim.hip).
sigma_sparsity_loss mirrors loss.py:45-47 (plain torch; unused by the reference's training loop).
"""
import math

import torch

from . import _lib, hashgrid
from .hashgrid import accumulate_grad_buffers


def tv_cube(level, min_resolution, max_resolution, n_levels):
    """Resolution and cuboid edge of loss.py:13-22 (python-double b, float32 product, floor)."""
    b = math.exp((math.log(float(max_resolution)) - math.log(float(min_resolution))) / (n_levels - 1))
    res = int(torch.floor(torch.as_tensor(min_resolution).cpu() * b ** level).item())
    min_cube = int(min_resolution) - 1
    if min_cube > 50:
        raise ValueError("total_variation_loss: min cuboid size greater than max (loss.py:19-21)")
    cube = int(torch.floor(torch.clip(torch.tensor(res) / 10.0, min_cube, 50)).item())
    return res, cube


class TVFn(torch.autograd.Function):
    """min_vertex: host [L,3] cuboid corners, or an int device address of [L,3] int64 slots that a
    captured step refreshes before every replay (graphs.StepScalars)."""
    @staticmethod
    def forward(ctx, min_vertex, cubes, log2_T, out, early, *tables):
        L = len(tables)
        if isinstance(min_vertex, int):
            mv, dmv = None, _lib.c_vp(min_vertex)
        else:
            mv, dmv = (_lib.c_i64 * (3 * L))(*[int(v) for v in min_vertex.reshape(-1).tolist()]), None
        cb = (_lib.c_int * L)(*[int(c) for c in cubes])
        dev = tables[0].device
        if early is not None and early.launched:   # already run inside the fine compositing launch
            ctx.save_for_backward(*tables)
            ctx.mv, ctx.dmv, ctx.cb, ctx.log2_T, ctx.verts = mv, dmv, cb, log2_T, early.verts
            return early.out
        # the cuboid vertices' rows, gathered once here: the backward's stencil reads them densely
        verts = (early.verts if early is not None else
                 torch.empty(2 * sum((int(c) + 1) ** 3 for c in cubes), device=dev, dtype=torch.float32))
        if out is None:
            loss = torch.zeros(L, device=dev, dtype=torch.float32)
        else:   # a zeroed accumulator (tv_accumulator: its fill rides along in render()'s first launch)
            _lib.flush_zero_fills([out])
            loss = out
        hashgrid.join_tables(dev)     # a pending parameter all-gather of the upper levels (dist.py)
        _lib.call("nerf_tv_fwd", _lib.ptr_array(tables), L, log2_T, mv, dmv, cb, _lib.ptr(loss, "loss"),
                  _lib.ptr(verts, "tv_verts"), _lib.stream())
        ctx.save_for_backward(*tables)
        ctx.mv, ctx.dmv, ctx.cb, ctx.log2_T, ctx.verts = mv, dmv, cb, log2_T, verts
        return loss

    @staticmethod
    def backward(ctx, g):
        tables = ctx.saved_tensors
        if g is not None and any(t.requires_grad for t in tables):
            grads = accumulate_grad_buffers(tables)
            g = g.contiguous()
            L = len(tables)
            n_ch = int(_lib.load().nerf_tv_bwd_bin_chunks(L, ctx.cb))
            det = int(hashgrid.deterministic())
            binned = n_ch > 0 and int(_lib.load().nerf_hash_encode_bwd_workspace_bytes(L, ctx.log2_T, 1, det)) > 0
            if binned:
                job = TVBinJob(tables, grads, g, ctx.mv, ctx.dmv, ctx.cb, ctx.log2_T, n_ch, ctx.verts)
                if torch._C._current_graph_task_id() != -1:
                    # summed by the pass's owner launch with the hash backwards (field._PendingField)
                    from .field import _pending_field
                    _pending_field(g.device).add(job)
                else:
                    pb = hashgrid.pending_bins(g.device)
                    pb.reserve(n_ch)
                    pb.add_tv(job, queue=False)
                    pb.flush()
            else:
                if det:
                    raise NotImplementedError(f"deterministic TV backward: no binned path for log2_T {ctx.log2_T}")
                hashgrid.materialize_zero(grads)
                _lib.call("nerf_tv_bwd", _lib.ptr_array(tables), L, ctx.log2_T, ctx.mv, ctx.dmv, ctx.cb,
                          _lib.ptr(g, "grad_loss"), _lib.ptr_array(grads, "grad_tables"), _lib.stream())
        return (None, None, None, None, None) + (None,) * len(tables)


class TVBinJob:
    """A TV backward awaiting its bin launch (csrc/hashgrid.hip tv_bwd_bin_kernel): binned into the
    iteration's hash-backward workspace and summed by the same owner pass (no float atomics; exact
    under the deterministic mode)."""

    def __init__(self, tables, grads, g, mv, dmv, cb, log2_T, n_chunks, verts=None):
        self.tables, self.grads, self.g, self.verts = tables, grads, g, verts
        self.mv, self.dmv, self.cb, self.log2_T, self.n_chunks = mv, dmv, cb, log2_T, n_chunks
        self.stream = torch.cuda.current_stream() if g.is_cuda else None


def draw_min_vertices(embedder, generator=None):
    """One cuboid corner per level: torch.randint(0, res - cube, (3,)) (loss.py:25)."""
    mvs, cubes = [], []
    for lvl in range(embedder.n_levels):
        res, cube = tv_cube(lvl, embedder.base_resolution, embedder.finest_resolution, embedder.n_levels)
        mvs.append(torch.randint(0, res - cube, (3,), generator=generator))
        cubes.append(cube)
    return torch.stack(mvs), cubes


def tv_accumulator(embedder):
    """The [L] loss accumulator of a later total_variation_all(..., out=), its zero fill deferred to the
    next render()'s first launch (_lib.defer_fill_zero): a training step allocates it before render."""
    acc = torch.empty(embedder.n_levels, device=embedder.tables()[0].device, dtype=torch.float32)
    _lib.defer_fill_zero(acc)
    return acc


def tv_forward_early(embedder, out):
    """Before render() of a captured step: have the step's TV forward launched inside the fine pass's
    compositing (hashgrid.EarlyTV, nerf_composite_fwd_tv) instead of as a launch of its own after
    render. Only the corner slots and the vertex buffer are allocated here; the corners are still drawn
    after render (total_variation_all registers their filler), so the host draw order is unchanged.
    Returns the job for total_variation_all(..., early=), or None (not capturing, no accumulator, off)."""
    from . import graphs
    sc = graphs.active()
    if sc is None or out is None or not hashgrid._TV_FWD_FUSED["on"]:
        return None
    L = embedder.n_levels
    off, ptr = sc.alloc_i64(3 * L)
    cubes = [tv_cube(l, embedder.base_resolution, embedder.finest_resolution, L)[1] for l in range(L)]
    verts = torch.empty(2 * sum((c + 1) ** 3 for c in cubes), device=out.device, dtype=torch.float32)
    job = hashgrid.EarlyTV(embedder.tables(), _lib.c_vp(ptr), off, cubes, embedder.log2_hashmap_size, out, verts)
    hashgrid.register_early_tv(job)
    return job


def total_variation_all(embedder, min_vertex=None, generator=None, out=None, early=None):
    """Per-level TV losses [L] of all levels of `embedder` (sum them for the reference's TV_loss).
    out: an accumulator from tv_accumulator (None: a fresh zeroed one). early: tv_forward_in_hash's job
    (its forward may already have run inside the coarse hash forward)."""
    from . import graphs
    sc = graphs.active()
    if early is not None:
        hashgrid.take_early_tv(early.out.device)
    if sc is not None and min_vertex is None:
        # captured step: the corners are drawn by the same host code before every replay
        L = embedder.n_levels
        if early is not None:
            off, ptr = early.slot_off, early.dmv.value
        else:
            off, ptr = sc.alloc_i64(3 * L)

        def fill(hi, hf, off=off):
            mv, _ = draw_min_vertices(embedder, generator)
            hi[off:off + 3 * L] = mv.reshape(-1).numpy()
        sc.add_filler(fill)
        cubes = [tv_cube(l, embedder.base_resolution, embedder.finest_resolution, L)[1] for l in range(L)]
        return TVFn.apply(ptr, cubes, embedder.log2_hashmap_size, out, early, *embedder.tables())
    if min_vertex is None:
        min_vertex, cubes = draw_min_vertices(embedder, generator)
    else:
        cubes = [tv_cube(l, embedder.base_resolution, embedder.finest_resolution, embedder.n_levels)[1]
                 for l in range(embedder.n_levels)]
    return TVFn.apply(torch.as_tensor(min_vertex), cubes, embedder.log2_hashmap_size, out, None, *embedder.tables())


def total_variation_loss(embeddings, min_resolution, max_resolution, level, log2_hashmap_size, n_levels=16,
                         min_vertex=None):
    """loss.py:11-43 for one level's nn.Embedding."""
    res, cube = tv_cube(level, min_resolution, max_resolution, n_levels)
    if min_vertex is None:
        min_vertex = torch.randint(0, res - cube, (3,))
    return TVFn.apply(torch.as_tensor(min_vertex).reshape(1, 3), [cube], log2_hashmap_size, None, None,
                      embeddings.weight)[0]


class TrainLossFn(torch.autograd.Function):
    """run_nerf.py:1011-1037 in one launch (csrc/loss.hip): returns (loss, img_loss, psnr[1])."""
    @staticmethod
    def forward(ctx, rgb, rgb0, target, sp, sp0, tv, sparse_w, tv_w):
        ctx.set_materialize_grads(False)     # img_loss / psnr carry no gradient: no zero fills
        R = rgb.shape[0]
        f = dict(device=rgb.device, dtype=torch.float32)
        rgb, target = rgb.contiguous(), target.contiguous().float()
        rgb0 = rgb0.contiguous() if rgb0 is not None else None
        loss, img, psnr = torch.empty((), **f), torch.empty((), **f), torch.empty(1, **f)
        n_tv = 0 if tv is None else tv.numel()
        _lib.call("nerf_train_loss_fwd", _lib.ptr(rgb, "rgb"), _lib.ptr(rgb0, "rgb0", allow_none=True),
                  _lib.ptr(target, "target"), R, _lib.ptr(sp, "sparsity", allow_none=True),
                  _lib.ptr(sp0, "sparsity0", allow_none=True), float(sparse_w), _lib.ptr(tv, "tv", allow_none=True),
                  n_tv, float(tv_w), _lib.ptr(loss), _lib.ptr(img), _lib.ptr(psnr), _lib.stream())
        ctx.save_for_backward(rgb, rgb0, target)
        ctx.meta = (R, float(sparse_w), n_tv, float(tv_w), sp is not None, sp0 is not None)
        ctx.mark_non_differentiable(img, psnr)
        return loss, img, psnr

    @staticmethod
    def backward(ctx, g, _g_img, _g_psnr):
        rgb, rgb0, target = ctx.saved_tensors
        if g is None:
            return (None,) * 8
        R, sparse_w, n_tv, tv_w, has_sp, has_sp0 = ctx.meta
        f = dict(device=rgb.device, dtype=torch.float32)
        d_rgb = torch.empty_like(rgb)
        d_rgb0 = torch.empty_like(rgb0) if (rgb0 is not None and ctx.needs_input_grad[1]) else None
        d_sp = torch.empty(R, **f) if has_sp and ctx.needs_input_grad[3] else None
        d_sp0 = torch.empty(R, **f) if has_sp0 and ctx.needs_input_grad[4] else None
        d_tv = torch.empty(n_tv, **f) if n_tv and ctx.needs_input_grad[5] else None
        _lib.call("nerf_train_loss_bwd", _lib.ptr(rgb, "rgb"), _lib.ptr(rgb0, "rgb0", allow_none=True),
                  _lib.ptr(target, "target"), R, sparse_w, n_tv, tv_w, _lib.ptr(g.contiguous(), "grad_loss"),
                  _lib.ptr(d_rgb), _lib.ptr(d_rgb0, allow_none=True), _lib.ptr(d_sp, allow_none=True),
                  _lib.ptr(d_sp0, allow_none=True), _lib.ptr(d_tv, allow_none=True), _lib.stream())
        return d_rgb, d_rgb0, None, d_sp, d_sp0, d_tv, None, None


def train_loss(rgb, rgb0, target, sparsity, sparsity0, tv, sparse_w, tv_w):
    """Fused loss of one training iteration (see TrainLossFn); any of rgb0/sparsity/sparsity0/tv may be None."""
    return TrainLossFn.apply(rgb, rgb0, target, sparsity, sparsity0, tv, sparse_w, tv_w)


def sigma_sparsity_loss(sigmas):
    """loss.py:45-47 (Cauchy sparsity)."""
    return torch.log(1.0 + 2 * sigmas ** 2).sum(dim=-1)
