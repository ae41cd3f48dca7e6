"""Volumetric renderer on the HIP kernels.

API mirror of PocketNeRF/run_nerf.py:71-151, :347-549 (batchify_rays, render, raw2outputs,
render_rays) and PocketNeRF/run_nerf_helpers.py:10-13, :311-397 (img2mse, mse2psnr, to8b,
get_rays, get_rays_np, ndc_rays, sample_pdf). Sampling, compositing and the hierarchical
resampling run in libnerfhip (csrc/sampling.hip, csrc/composite.hip); the field query goes
through network_query_fn (field.run_network -> the fused hash-grid + MLP kernels).

Randomness: pytest=True reproduces the reference's np.random.seed(0) draws exactly; otherwise
stratified jitter and importance uniforms are drawn in-kernel (Philox4x32-10) from a seed taken
from torch's CPU generator, and raw noise uses torch.randn like the reference.
"""
import ctypes
import os

import numpy as np
import torch

from . import _lib
from .hashgrid import early_tv

img2mse = lambda x, y: torch.mean((x - y) ** 2)  # noqa: E731
# The reference divides by torch.log(torch.Tensor([10.])) (a [1] float32 tensor): same value and shape
# here without creating a device tensor from host data (that copy would synchronise the stream).
mse2psnr = lambda x: (-10. * torch.log(x) / _LOG10_F32).reshape(1)  # noqa: E731
_LOG10_F32 = float(np.float32(np.log(10.0)))
to8b = lambda x: (255 * np.clip(x, 0, 1)).astype(np.uint8)  # noqa: E731

_LINSPACE = {}
_SEED_GEN = None

# run_nerf.py:40 DEBUG: when True, render_rays tests every returned tensor for NaN/Inf (one fused
# device count, csrc/checks.hip, and one host read per call) and prints the reference's message.
# The package namespace re-exports the render() function under this module's name, so set it with
# set_debug() (or on the module: importlib.import_module("indoor_nerf_amd.render").DEBUG).
DEBUG = False


def set_debug(enabled=True):
    """run_nerf.py:40's module flag (DEBUG = True) for this package."""
    global DEBUG
    DEBUG = bool(enabled)


def check_numerics(ret):
    """run_nerf.py:545-547 over the tensors of `ret`; returns the keys that hold NaN/Inf."""
    items = [(k, v) for k, v in ret.items() if torch.is_tensor(v) and v.dtype == torch.float32 and v.is_cuda]
    bad = []
    for i in range(0, len(items), _lib.MAX_CHECK):
        part = items[i:i + _lib.MAX_CHECK]
        ts = [v.contiguous() for _, v in part]
        counts = torch.empty(len(ts), dtype=torch.int32, device=ts[0].device)
        sizes = (_lib.c_i64 * len(ts))(*[t.numel() for t in ts])
        _lib.call("nerf_count_nonfinite", _lib.ptr_array(ts, "ret"), sizes, len(ts),
                  _lib.ptr(counts, "counts", dtype=torch.int32), _lib.stream())
        bad += [k for (k, _), c in zip(part, counts.tolist()) if c]
    for k in bad:
        print(f"! [Numerical Error] {k} contains nan or inf.")
    return bad


def _linspace(n, device):
    key = (n, str(device))
    if key not in _LINSPACE:
        _LINSPACE[key] = torch.linspace(0., 1., steps=n).to(device)   # CPU linspace values, as the reference
    return _LINSPACE[key]


def _draw_seed():
    global _SEED_GEN
    if _SEED_GEN is None:
        _SEED_GEN = torch.Generator().manual_seed(torch.initial_seed() & ((1 << 63) - 1))
    s = torch.randint(0, 2 ** 62, (2,), generator=_SEED_GEN)
    return int(s[0]), int(s[1])


def _rng():
    """(seed, offset, d_rng) for an in-kernel Philox draw. Eager: a fresh host seed. While a
    training step is being captured (graphs.GraphedTrainStep): two device slots that a filler
    refreshes with a fresh seed before every replay."""
    from . import graphs
    sc = graphs.active()
    if sc is None:
        s, o = _draw_seed()
        return s, o, None
    off, ptr = sc.alloc_i64(2)

    def fill(hi, hf, off=off):
        s, o = _draw_seed()
        hi[off], hi[off + 1] = s, o
    sc.add_filler(fill)
    return 0, 0, _lib.c_vp(ptr)


def manual_seed(seed):
    """Seed the in-kernel Philox draws (stratified jitter, importance uniforms)."""
    global _SEED_GEN
    _SEED_GEN = torch.Generator().manual_seed(int(seed))


_PYTEST_SHARD = (0, 1)


def pytest_shard(rank, world):
    """pytest=True draws for a data-parallel shard: every draw then takes the reference's
    np.random.seed(0) uniforms for the GLOBAL batch (world x this rank's rays, run_nerf.py:482-486,
    run_nerf_helpers.py:368-377) and keeps this rank's contiguous rows, so that G shards see exactly
    the draws one process sees for the whole batch (tests/test_gpu_dist.py). (0, 1) = off."""
    global _PYTEST_SHARD
    if not (0 <= rank < world):
        raise ValueError(f"pytest_shard: rank {rank} of {world}")
    _PYTEST_SHARD = (int(rank), int(world))


def _pytest_uniforms(shape, device):
    np.random.seed(0)
    rank, world = _PYTEST_SHARD
    if world == 1:
        return torch.from_numpy(np.random.rand(*shape).astype(np.float32)).to(device)
    full = np.random.rand(shape[0] * world, *shape[1:]).astype(np.float32)
    return torch.from_numpy(full[rank * shape[0]:(rank + 1) * shape[0]]).to(device)


# ---------------------------------------------------------------- compositing

class CompositeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, raw, z, rays_d, noise, white_bkgd, sampler=None, defer=False):
        if z.requires_grad or rays_d.requires_grad:
            raise NotImplementedError("raw2outputs: gradients w.r.t. z_vals / rays_d are not implemented "
                                      "(the reference detaches both)")
        ctx.set_materialize_grads(False)
        raw = raw.contiguous()
        z = z.contiguous().float()
        rays_d = rays_d.contiguous().float()
        R, S, C = raw.shape
        dev = raw.device
        f = dict(device=dev, dtype=torch.float32)
        rgb, disp, acc = torch.empty(R, 3, **f), torch.empty(R, **f), torch.empty(R, **f)
        weights, depth, ent = torch.empty(R, S, **f), torch.empty(R, **f), torch.empty(R, **f)
        normal = torch.empty(R, 3, **f) if C == 7 else None
        cargs = (_lib.ptr(raw, "raw"), C, _lib.ptr(z, "z_vals"), _lib.ptr(rays_d, "rays_d"),
                 _lib.ptr(noise, "noise", allow_none=True), R, S, int(bool(white_bkgd)), _lib.ptr(rgb, "rgb"),
                 _lib.ptr(disp, "disp"), _lib.ptr(acc, "acc"), _lib.ptr(weights, "weights"), _lib.ptr(depth, "depth"),
                 _lib.ptr(ent, "entropy"), _lib.ptr(normal, "normal", allow_none=True))
        tv = early_tv(dev) if sampler is None else None
        if tv is not None:   # a captured step's TV forward in the same launch (losses.tv_forward_early)
            from .hashgrid import join_tables
            join_tables(dev)                    # a pending all-gather of table levels (dist.py): TV reads them all
            _lib.flush_zero_fills([tv.out])     # its accumulator's fill: normally done by nerf_rays_pack_z
            job = _lib.TVFwdJob(_lib.c_vp(ctypes.addressof(tv.ptrs)), None, tv.dmv, _lib.c_vp(ctypes.addressof(tv.cb)),
                                _lib.ptr(tv.out, "tv_loss"), _lib.ptr(tv.verts, "tv_verts"))
            _lib.call("nerf_composite_fwd_tv", *cargs, ctypes.byref(job), len(tv.tables), tv.log2_T, _lib.stream())
            tv.launched = True
        elif sampler is None:
            _lib.call("nerf_composite_fwd", *cargs, _lib.stream())
        else:   # the coarse pass: the hierarchical sampler on these weights in the same launch
            _lib.call("nerf_composite_sample_fine", *cargs, *sampler, _lib.stream())
        ctx.save_for_backward(raw, z, rays_d, noise)
        ctx.white, ctx.defer = int(bool(white_bkgd)), defer
        outs = (rgb, disp, acc, weights, depth, ent)
        return outs + ((normal,) if normal is not None else ())

    @staticmethod
    def backward(ctx, *grads):
        raw, z, rays_d, noise = ctx.saved_tensors
        R, S, C = raw.shape
        names = ["g_rgb", "g_disp", "g_acc", "g_weights", "g_depth", "g_entropy", "g_normal"]
        gs = [None if g is None else g.contiguous().float() for g in grads] + [None] * (7 - len(grads))
        graw = torch.empty_like(raw)
        job = _lib.CompositeBwdJob(_lib.ptr(raw, "raw"), C, _lib.ptr(z, "z_vals"), _lib.ptr(rays_d, "rays_d"),
                                   _lib.ptr(noise, "noise", allow_none=True), R, S, ctx.white,
                                   *[_lib.ptr(g, n, allow_none=True) for g, n in zip(gs, names)],
                                   _lib.ptr(graw, "grad_raw"))
        task = torch._C._current_graph_task_id()
        if ctx.defer and _DEFER["on"] and task != -1 and task != _DEFER["off_task"]:
            # graw is read only by the field's (deferred) backward: launched with the pass's other
            # compositing backward as the pass's final callback (field._PendingField)
            from .field import _pending_field
            _pending_field(raw.device).add(CompositeJob(job, (raw, z, rays_d, noise, gs, graw)))
        else:
            _lib.call("nerf_composite_bwd_batch", (_lib.CompositeBwdJob * 1)(job), 1, _lib.stream())
        return graw, None, None, None, None, None, None


class CompositeJob:
    """A compositing backward awaiting its launch (nerf_composite_bwd_batch: the fine and the coarse
    pass's in one launch); `refs` keeps its inputs and output alive until then."""

    def __init__(self, job, refs):
        self.job, self.refs = job, refs
        self.stream = torch.cuda.current_stream()


def run_composite_jobs(jobs):
    if jobs:
        _lib.call("nerf_composite_bwd_batch", (_lib.CompositeBwdJob * len(jobs))(*[j.job for j in jobs]), len(jobs),
                  _lib.stream())


_DEFER = {"on": True, "off_task": None}


def set_batched_composite_bwd(enabled=True):
    """Defer the compositing backward of a field's raw output to the pass's final callback, where the
    fine and the coarse pass's run as one launch (on by default). Taken only for raw straight from the
    fused field without a normals head (the field's own backward is deferred too, so nothing else reads
    the raw gradient before the launch); a render_rays raw output that is itself differentiated
    (retraw) flushes the deferred launch first (_RawGuardFn)."""
    _DEFER["on"] = bool(enabled)


def batched_composite_bwd():
    return _DEFER["on"]


class _RawGuardFn(torch.autograd.Function):
    """render_rays' raw output (retraw) when the compositing backward of the same raw may be deferred:
    identity forward; a gradient through it (a loss on raw itself) launches any deferred compositing
    backward at once and turns deferral off for the rest of the pass, so autograd's sum of the two
    raw gradients reads a written buffer."""

    @staticmethod
    def forward(ctx, raw):
        return raw.view_as(raw)

    @staticmethod
    def backward(ctx, g):
        _DEFER["off_task"] = torch._C._current_graph_task_id()
        from .field import _pending_field
        _pending_field(g.device).flush_composites()
        return g


_FUSED_SAMPLER = {"on": True}
_SH_ROWS = {"on": True}


def set_sh_rows(enabled=True):
    """render_rays writes each ray's SH4 view encoding once (nerf_sample_stratified_sh) and the fused
    field's MLP kernels load it instead of evaluating SH per point (on by default; bit-identical)."""
    _SH_ROWS["on"] = bool(enabled)


def sh_rows():
    return _SH_ROWS["on"]


def set_fused_coarse_sampler(enabled=True):
    """render_rays' coarse compositing and hierarchical sampler in one launch (nerf_composite_sample_fine,
    on by default; bit-identical to nerf_composite_fwd + nerf_sample_fine_rows)."""
    _FUSED_SAMPLER["on"] = bool(enabled)


def fused_coarse_sampler():
    return _FUSED_SAMPLER["on"]


def raw2outputs(raw, z_vals, rays_d, raw_noise_std=0, white_bkgd=False, pytest=False, predict_normals=False,
                _sampler=None, _defer=False):
    """run_nerf.py:347-411 -> (rgb_map, disp_map, acc_map, weights, depth_map, sparsity_loss[, normal_map]).
    Internal (render_rays): _sampler = its nerf_sample_fine_rows arguments after d_weights' group;
    _defer = raw reaches nothing but this call and render_rays' guarded raw output."""
    R, S = raw.shape[0], raw.shape[1]
    noise = None
    if raw_noise_std > 0.:
        if pytest:
            noise = _pytest_uniforms((R, S), raw.device) * raw_noise_std
        else:
            # torch.randn(R, S) * raw_noise_std (run_nerf.py) in one launch: normal_'s transform z * std + 0
            # rounds like the product, from the same generator draws (tests/test_gpu_parity.py)
            noise = torch.empty(R, S, device=raw.device).normal_(0.0, raw_noise_std)
    if raw.shape[-1] not in (4, 7):
        raise ValueError(f"raw2outputs: raw must have 4 or 7 channels, got {raw.shape[-1]}")
    if not predict_normals and raw.shape[-1] == 7:
        raw = raw[..., :4]      # the reference reads channels 0..3 only
    defer = _defer and bool(getattr(raw, "_nerf_field_raw", False)) and raw.dtype == torch.float32
    outs = CompositeFn.apply(raw.float(), z_vals, rays_d, noise, white_bkgd, _sampler, defer)
    if predict_normals:
        if raw.shape[-1] == 4:
            # the reference slices raw[..., 4:7] of a 4-channel raw (the coarse net has no normals
            # head, run_nerf.py:240-247 vs :260-268): an empty [R, 0] normal map (run_nerf.py:361,407)
            return outs + (raw.new_zeros(R, 0),)
        return outs
    return outs[:6]


# ---------------------------------------------------------------- coarse-feature reuse

_REUSE = {"on": True}


def set_coarse_reuse(enabled=True):
    """the fine pass of render_rays encodes only its importance samples and takes
    the hash features of its coarse points from the coarse pass (on by default; off = re-encode all
    of them, as the reference does). Features are bit-identical either way."""
    _REUSE["on"] = bool(enabled)


def coarse_reuse():
    return _REUSE["on"]


def last_reuse_used():
    """Whether the last render_rays call's fine pass took the coarse features (bench.py's pricing)."""
    return _REUSE.get("last", False)


class CoarseReuse:
    """Hand-over of one render_rays call's coarse hash encoding to its fine pass.

    The reference merges the coarse depths into the fine ones (run_nerf.py:512-516: torch.sort of
    cat([z_vals, z_samples]), then rays_o + rays_d * z) and queries both networks through ONE
    embedder (run_nerf.py:225,275), so 64 of a ray's 192 fine points are the coarse points bit for
    bit and, the tables being unchanged inside an iteration, so are their 16-level features.
    render_rays attaches this object to the coarse and then the fine point tensors
    (`pts._nerf_reuse`); field.FieldFn (the fused run_network) encodes the coarse points into the tail
    rows of one feature buffer [L, R*(S+N), 2] laid out in importance-first order (importance sample k
    of ray r at row r*N + k, then coarse sample i at R*N + r*S + i), and the fine pass gathers only its
    importance samples, into the head rows: no copy, no scattered writes. The fine MLP walks that order
    (nerf_point_order: raw / geo / graw / dgeo stay in the merged order at rows inv, = the sampler's
    importance rows then its coarse rows), so its d feat is importance-first too: the fine bin reads
    the importance samples' rows contiguously and the coarse bin adds the coarse points' fine d feat
    (the tail rows) to their coarse d feat (nerf_hash_encode_bwd_bin_rows): each shared point is binned
    once. Any other network_query_fn ignores the attribute."""

    def __init__(self, R, S, N):
        self.R, self.S, self.N = R, S, N
        self.state = "armed"          # -> "recorded" (coarse FieldFn) -> "rows" (sample_fine) -> "used"
        self.feat = self.keep = self.pts = self.embedder = self.versions = None
        self.inv = self.imp_pts = None

    def alloc(self, n_levels, device):
        """The shared feature / keep buffers; returns them and the coarse pass's first row."""
        P = self.R * (self.S + self.N)
        self.feat = torch.empty(n_levels, P, 2, device=device, dtype=torch.float32)
        self.keep = torch.empty(P, device=device, dtype=torch.bool)
        return self.feat, self.keep, self.R * self.N

    def record(self, pts, embedder, tables):
        self.pts, self.embedder = pts, embedder
        self.versions = [t._version for t in tables]
        self.state = "recorded"

    def matches(self, embedder, tables, P):
        return (self.state == "rows" and embedder is self.embedder and P == self.R * (self.S + self.N)
                and [t._version for t in tables] == self.versions)

    @property
    def used(self):
        return self.state == "used"

    def release_forward(self):
        """After the fine forward: only the row maps and the coarse points stay (the backward's)."""
        self.feat = self.keep = self.embedder = None


# ---------------------------------------------------------------- sampling

def sample_pdf(bins, weights, N_samples, det=False, pytest=False):
    """run_nerf_helpers.py:354-397 (no gradient: the reference detaches its samples)."""
    bins = bins.detach().contiguous().float()
    weights = weights.detach().contiguous().float()
    R, nb = bins.shape
    if weights.shape != (R, nb - 1):
        raise ValueError(f"sample_pdf: weights {tuple(weights.shape)} must be [R, n_bins - 1] = [{R}, {nb - 1}]")
    out = torch.empty(R, N_samples, device=bins.device, dtype=torch.float32)
    t_imp = _linspace(N_samples, bins.device) if det else None
    u = _pytest_uniforms((R, N_samples), bins.device) if (pytest and not det) else None
    seed, off, rng = _rng()
    _lib.call("nerf_sample_pdf", _lib.ptr(bins, "bins"), nb, _lib.ptr(weights, "weights"), nb - 1, R, nb, N_samples,
              int(det), _lib.ptr(t_imp, "t", allow_none=True), _lib.ptr(u, "u", allow_none=True), seed, off, rng,
              _lib.ptr(out, "samples"), _lib.stream())
    return out


def render_rays(ray_batch, network_fn, network_query_fn, N_samples, embed_fn=None, retraw=False, lindisp=False,
                perturb=0., N_importance=0, network_fine=None, white_bkgd=False, raw_noise_std=0., verbose=False,
                pytest=False, predict_normals=False):
    """run_nerf.py:414-549."""
    rays = ray_batch.detach().float().contiguous()
    R, C = rays.shape
    dev = rays.device
    f = dict(device=dev, dtype=torch.float32)
    # contiguous copies of the directions (compositing) and view directions (field), written by the
    # sampler launch instead of two slicing copies
    viewdirs = torch.empty(R, 3, **f) if C > 8 else None
    rays_d = torch.empty(R, 3, **f)

    z = torch.empty(R, N_samples, **f)
    pts = torch.empty(R, N_samples, 3, **f)
    u = _pytest_uniforms((R, N_samples), dev) if (perturb > 0. and pytest) else None
    seed, off, rng = (0, 0, None) if (u is not None or not perturb > 0.) else _rng()
    # the view directions' SH4 rows, once per ray (the fused field reads them instead of evaluating
    # SH per point, field.FieldFn): attached to the viewdirs tensor the field receives
    # [R, 40]: 16 fp32 coefficients + their three bf16 pieces (the MLP's pre-split C0 operand)
    sh_rays = torch.empty(R, 40, **f) if (viewdirs is not None and _SH_ROWS["on"]) else None
    _lib.call("nerf_sample_stratified_sh", _lib.ptr(rays, "ray_batch"), C, R, N_samples,
              _lib.ptr(_linspace(N_samples, dev)), int(bool(lindisp)), int(perturb > 0.), _lib.ptr(u, "u", allow_none=True),
              seed, off, rng, _lib.ptr(z, "z"), _lib.ptr(pts, "pts"), _lib.ptr(rays_d, "rays_d"),
              _lib.ptr(viewdirs, "viewdirs", allow_none=True), _lib.ptr(sh_rays, "sh_rows", allow_none=True),
              _lib.stream())
    if sh_rays is not None:
        viewdirs._nerf_sh = sh_rays

    reuse = CoarseReuse(R, N_samples, N_importance) if (N_importance > 0 and _REUSE["on"] and R > 0) else None
    if reuse is not None:
        pts._nerf_reuse = reuse       # the fused run_network records the coarse encoding in it
    raw = network_query_fn(pts, viewdirs, network_fn)
    if reuse is not None:
        del pts._nerf_reuse
        if reuse.state != "recorded" or R * (N_samples + N_importance) > 2 ** 31 - 1:
            reuse = None
    ret = {}
    if N_importance > 0:
        det = perturb == 0.
        M = N_samples + N_importance
        z_fine = torch.empty(R, M, **f)
        pts_fine = torch.empty(R, M, 3, **f)
        z_std = torch.empty(R, **f)
        t_imp = _linspace(N_importance, dev) if det else None
        u_imp = _pytest_uniforms((R, N_importance), dev) if (pytest and not det) else None
        seed, off, rng = (0, 0, None) if (det or u_imp is not None) else _rng()
        i32 = dict(device=dev, dtype=torch.int32)
        if reuse is not None:
            # inv = [importance rows | coarse rows]: the merged row of each importance-first position
            reuse.inv, reuse.imp_pts = torch.empty(R * M, **i32), torch.empty(R, N_importance, 3, **f)
            reuse.state = "rows"
        inv = None if reuse is None else reuse.inv
        # nerf_sample_fine_rows' arguments after (d_z, d_weights, n_rays, n_samples)
        samp = (N_importance, int(det), _lib.ptr(t_imp, "t", allow_none=True), _lib.ptr(u_imp, "u", allow_none=True),
                seed, off, rng, _lib.ptr(z_fine, "z_fine"), _lib.ptr(pts_fine, "pts_fine"), _lib.ptr(z_std, "z_std"),
                None, None if inv is None else _lib.ptr_at(inv, R * N_importance, "coarse_rows", torch.int32),
                _lib.ptr(inv, "imp_rows", torch.int32, True),
                _lib.ptr(None if reuse is None else reuse.imp_pts, "imp_pts", allow_none=True), None)
        fused = _FUSED_SAMPLER["on"]
        outs = raw2outputs(raw, z, rays_d, raw_noise_std, white_bkgd, pytest=pytest, predict_normals=predict_normals,
                           _sampler=(_lib.ptr(rays, "ray_batch"), C) + samp if fused else None, _defer=True)
        weights = outs[3]
        if not fused:
            _lib.call("nerf_sample_fine_rows", _lib.ptr(rays, "ray_batch"), C, _lib.ptr(z, "z"),
                      _lib.ptr(weights.detach().contiguous(), "weights"), R, N_samples, *samp, _lib.stream())
        rgb_map_0, _, acc_map_0, _, depth_map_0, sparsity_loss_0 = outs[:6]
        normal_map_0 = outs[6] if predict_normals else None
        z, pts = z_fine, pts_fine
        run_fn = network_fn if network_fine is None else network_fine
        if reuse is not None:
            pts._nerf_reuse = reuse
        raw = network_query_fn(pts, viewdirs, run_fn)
        if reuse is not None:
            del pts._nerf_reuse
            reuse.release_forward()
        _REUSE["last"] = reuse is not None and reuse.used
        outs = raw2outputs(raw, z, rays_d, raw_noise_std, white_bkgd, pytest=pytest, predict_normals=predict_normals,
                           _defer=True)
        rgb_map, disp_map, acc_map, weights, depth_map, sparsity_loss = outs[:6]
        normal_map = outs[6] if predict_normals else None
        ret.update(rgb0=rgb_map_0, depth0=depth_map_0, acc0=acc_map_0, sparsity_loss0=sparsity_loss_0, z_std=z_std)
        if predict_normals:
            ret["normal0"] = normal_map_0
    else:
        outs = raw2outputs(raw, z, rays_d, raw_noise_std, white_bkgd, pytest=pytest, predict_normals=predict_normals,
                           _defer=True)
        rgb_map, disp_map, acc_map, weights, depth_map, sparsity_loss = outs[:6]
        normal_map = outs[6] if predict_normals else None

    ret.update(rgb_map=rgb_map, depth_map=depth_map, acc_map=acc_map, sparsity_loss=sparsity_loss, pts=pts,
               rays_d=rays_d)
    if predict_normals:
        ret["normal_map"] = normal_map
    if retraw:
        ret["raw"] = _RawGuardFn.apply(raw) if getattr(raw, "_nerf_field_raw", False) else raw
    if DEBUG:
        check_numerics(ret)
    return ret


def batchify_rays(rays_flat, chunk=1024 * 32, **kwargs):
    """run_nerf.py:71-83."""
    all_ret = {}
    for i in range(0, rays_flat.shape[0], chunk):
        ret = render_rays(rays_flat[i:i + chunk], **kwargs)
        for k in ret:
            all_ret.setdefault(k, []).append(ret[k])
    return {k: (v[0] if len(v) == 1 else torch.cat(v, 0)) for k, v in all_ret.items()}


def camera(K, c2w):
    """nerf_camera of a float64 (or float32) K and a [3,4] pose: the float32 values get_rays'
    tensor ops see (run_nerf_helpers.py:311-320)."""
    cam = _lib.Camera()
    pose = torch.as_tensor(c2w, dtype=torch.float32).detach().cpu().reshape(-1, 4)[:3]
    for k, v in enumerate(pose.reshape(-1).tolist()):
        cam.c2w[k] = v
    Kf = [[float(np.float32(float(K[r][c]))) for c in range(3)] for r in range(2)]
    cam.fx, cam.fy, cam.cx, cam.cy = Kf[0][0], Kf[1][1], Kf[0][2], Kf[1][2]
    return cam


def get_rays(H, W, K, c2w, device=None):
    """run_nerf_helpers.py:311-320 -> rays_o, rays_d [H, W, 3] on the device (csrc/rays.hip,
    one launch; the pose is read on the host)."""
    device = torch.device(device) if device is not None else (c2w.device if torch.is_tensor(c2w) else
                                                               torch.device("cuda"))
    H, W = int(H), int(W)
    rays_o = torch.empty(H, W, 3, device=device, dtype=torch.float32)
    rays_d = torch.empty(H, W, 3, device=device, dtype=torch.float32)
    _lib.call("nerf_sample_rays", camera(K, c2w), H, W, 0, 0, H, W, H * W, 0, 0, 0, None, 0,
              _lib.ptr(rays_o, "rays_o"), _lib.ptr(rays_d, "rays_d"), None, None, _lib.stream())
    return rays_o, rays_d


def get_rays_np(H, W, K, c2w):
    """run_nerf_helpers.py:323-330."""
    i, j = np.meshgrid(np.arange(W, dtype=np.float32), np.arange(H, dtype=np.float32), indexing="xy")
    dirs = np.stack([(i - K[0][2]) / K[0][0], -(j - K[1][2]) / K[1][1], -np.ones_like(i)], -1)
    rays_d = np.sum(dirs[..., np.newaxis, :] * c2w[:3, :3], -1)
    rays_o = np.broadcast_to(c2w[:3, -1], np.shape(rays_d))
    return rays_o, rays_d


def ndc_rays(H, W, focal, near, rays_o, rays_d):
    """run_nerf_helpers.py:333-350."""
    t = -(near + rays_o[..., 2]) / rays_d[..., 2]
    rays_o = rays_o + t[..., None] * rays_d
    o0 = -1. / (W / (2. * focal)) * rays_o[..., 0] / rays_o[..., 2]
    o1 = -1. / (H / (2. * focal)) * rays_o[..., 1] / rays_o[..., 2]
    o2 = 1. + 2. * near / rays_o[..., 2]
    d0 = -1. / (W / (2. * focal)) * (rays_d[..., 0] / rays_d[..., 2] - rays_o[..., 0] / rays_o[..., 2])
    d1 = -1. / (H / (2. * focal)) * (rays_d[..., 1] / rays_d[..., 2] - rays_o[..., 1] / rays_o[..., 2])
    d2 = -2. * near / rays_o[..., 2]
    return torch.stack([o0, o1, o2], -1), torch.stack([d0, d1, d2], -1)


def _pack_rays(H, W, K, rays_o, rays_d, near, far, ndc, use_viewdirs):
    """render()'s prologue (run_nerf.py:115-140) in one launch (csrc/rays.hip nerf_rays_pack):
    viewdirs = d/|d|, ndc_rays (near plane 1), [o, d, near, far, viewdir] per ray."""
    o = torch.reshape(rays_o, [-1, 3]).float().contiguous()
    d = torch.reshape(rays_d, [-1, 3]).float().contiguous()
    n = d.shape[0]
    out = torch.empty(n, 11 if use_viewdirs else 8, device=d.device, dtype=torch.float32)
    cw = ch = 0.0
    if ndc:
        focal = K[0][0]
        # -1./(W/(2.*focal)) is a python double in the reference; torch rounds it to float32
        cw = float(np.float32(-1. / (W / (2. * float(focal)))))
        ch = float(np.float32(-1. / (H / (2. * float(focal)))))
    zeros, nz, keep = _lib.take_zero_fills(d.device)   # a training step's zero fills ride along (_lib.defer_fill_zero)
    _lib.call("nerf_rays_pack_z", _lib.ptr(o, "rays_o"), _lib.ptr(d, "rays_d"), n, float(near), float(far),
              int(bool(ndc)), cw, ch, int(bool(use_viewdirs)), _lib.ptr(out, "rays"), zeros, nz, _lib.stream())
    del keep
    return out


def render(H, W, K, chunk=1024 * 32, rays=None, c2w=None, ndc=True, near=0., far=1., use_viewdirs=False,
           c2w_staticcam=None, **kwargs):
    """run_nerf.py:86-151 -> [rgb_map, depth_map, acc_map, extras]."""
    if c2w is not None:
        rays_o, rays_d = get_rays(H, W, K, c2w)
    else:
        rays_o, rays_d = rays
    sh = rays_d.shape
    if use_viewdirs and c2w_staticcam is not None:
        # viewdirs from the moving camera, rays from the static one (run_nerf.py:115-126)
        vd = rays_d / torch.norm(rays_d, dim=-1, keepdim=True)
        rays_o, rays_d = get_rays(H, W, K, c2w_staticcam)
        rays = _pack_rays(H, W, K, rays_o, rays_d, near, far, ndc, False)
        rays = torch.cat([rays, torch.reshape(vd, [-1, 3]).float()], -1)
    else:
        rays = _pack_rays(H, W, K, rays_o, rays_d, near, far, ndc, use_viewdirs)
    all_ret = batchify_rays(rays, chunk, **kwargs)
    for k in all_ret:
        all_ret[k] = torch.reshape(all_ret[k], list(sh[:-1]) + list(all_ret[k].shape[1:]))
    k_extract = ["rgb_map", "depth_map", "acc_map"]
    return [all_ret[k] for k in k_extract] + [{k: all_ret[k] for k in all_ret if k not in k_extract}]


def render_path(render_poses, hwf, K, chunk, render_kwargs, gt_imgs=None, savedir=None, render_factor=0):
    """run_nerf.py:154-215: full frames along a camera path through render() (device ray generation,
    chunked fused field, compositing) -> (rgbs [N,H,W,3], depths [N,H,W] normalised to [0,1]) as
    numpy. With gt_imgs (and render_factor 0) the per-view PSNR -10 log10(mean((rgb - gt)^2)) is
    printed and its average pickled to savedir, as the reference does; savedir also receives each
    view as 8-bit PNGs ({i:03d}.png colour, {i:03d}_depth.png depth) instead of the reference's
    matplotlib figure. As the reference, render_factor shrinks H, W and focal but passes K unchanged
    to render()."""
    H, W, focal = hwf
    near, far = render_kwargs["near"], render_kwargs["far"]
    if render_factor != 0:
        H, W, focal = H // render_factor, W // render_factor, focal / render_factor
    rgbs, depths, psnrs = [], [], []
    dev = next(render_kwargs["network_fn"].parameters()).device     # the reference's default CUDA tensors
    for i, c2w in enumerate(render_poses):
        c2w = (c2w if torch.is_tensor(c2w) else torch.as_tensor(np.asarray(c2w, np.float32))).to(dev)
        with torch.no_grad():
            rgb, depth, acc, _ = render(H, W, K, chunk=chunk, c2w=c2w[:3, :4], **render_kwargs)
        rgb_np = rgb.cpu().numpy()
        rgbs.append(rgb_np)
        depths.append(((depth - near) / (far - near)).cpu().numpy())
        if gt_imgs is not None and render_factor == 0:
            gt = gt_imgs[i].cpu().numpy() if torch.is_tensor(gt_imgs[i]) else np.asarray(gt_imgs[i])
            p = -10. * np.log10(np.mean(np.square(rgb_np - gt)))
            print(p)
            psnrs.append(p)
        if savedir is not None:
            from PIL import Image
            os.makedirs(savedir, exist_ok=True)
            Image.fromarray(to8b(rgbs[-1])).save(os.path.join(savedir, f"{i:03d}.png"))
            Image.fromarray(to8b(np.clip(depths[-1], 0, 1))).save(os.path.join(savedir, f"{i:03d}_depth.png"))
    rgbs, depths = np.stack(rgbs, 0), np.stack(depths, 0)
    if gt_imgs is not None and render_factor == 0:
        avg = sum(psnrs) / len(psnrs)
        print("Avg PSNR over Test set: ", avg)
        if savedir is not None:
            import pickle
            with open(os.path.join(savedir, "test_psnrs_avg{:0.2f}.pkl".format(avg)), "wb") as fp:
                pickle.dump(psnrs, fp)
    return rgbs, depths
