"""Radiance field: NeRFSmall and run_network on the fused HIP MLP.

API mirror of PocketNeRF/run_nerf_helpers.py:169-306 (NeRFSmall, same constructor arguments, same
parameters `sigma_net.{0,1}.weight`, `color_net.{0,1,2}.weight`) and run_network / batchify
(PocketNeRF/run_nerf.py:43-68). When run_network is handed this package's HashEmbedder, SHEncoder
and NeRFSmall it runs the fused path (FieldFn): hash encoding in a level-major layout, SH of each
ray's view direction computed once per point inside the MLP kernel's prologue, and the
sigma := 0 mask in its epilogue — no [P,48] concat and no per-sample SH tensor.
"""
import os

import torch
import torch.nn as nn

from . import _lib
from .hashgrid import HashEmbedder, SHEncoder, accumulate_grad_buffers, bin_chunks, hash_encode_bwd, pending_bins
from .quantization import LearnedBitwidthQuantizer, calibrate_from_stats, new_stats, quant_records


def _weights_struct(weights, w0q=None):
    """Kernel weight pointers; with the A-CAQ weight quantizer, layer 0 reads the quantized W0."""
    w = _lib.MlpWeights()
    for name, t in zip(("w0", "w1", "c0", "c1", "c2"), weights):
        setattr(w, name, _lib.ptr(t.detach(), name).value)
    if w0q is not None:
        w.w0 = _lib.ptr(w0q, "w0_quantized").value
    return w


def _fake_quant(x, rec):
    y = torch.empty_like(x)
    _lib.call("nerf_fake_quant", _lib.ptr(x.detach(), "x"), x.numel(), _lib.ptr(rec, "record"), _lib.ptr(y, "y"),
              _lib.stream())
    return y


def _act_calibration(feat_args, P, weights, w0q, n_calib):
    """Calibration-only MLP launch: (min, max) of relu(x W0q^T) over the first n_calib points."""
    st = new_stats(1, w0q.device)
    _lib.call("nerf_mlp_fwd_q", *feat_args, P, _weights_struct(weights, w0q), None, None, None,
              _lib.ptr(st, "stats", dtype=torch.int32), n_calib, _lib.stream())
    return st


def _grads_struct(weights):
    g = _lib.MlpGrads()
    for name, t in zip(("w0", "w1", "c0", "c1", "c2"), accumulate_grad_buffers(weights)):
        setattr(g, name, _lib.ptr(t, "grad_" + name).value)
    return g


def _head_struct(head):
    h = _lib.NormalHead()
    for name, t in zip(("n0", "b0", "n1", "b1"), head):
        setattr(h, name, _lib.ptr(t.detach(), "normal_net." + name).value)
    return h


def _head_forward(o16, raw4, keep, head, rows=None):
    """raw [P,7] = [raw4, normals] (csrc/normals.hip); keep masks n_z like run_network. rows (int32):
    keep is in a source order whose point q sits at merged row rows[q]; then returns (raw7, the keep
    flags scattered to the merged rows), else raw7."""
    P = raw4.shape[0]
    raw7 = torch.empty(P, 7, device=raw4.device, dtype=torch.float32)
    if rows is None:
        _lib.call("nerf_normal_head_fwd", _lib.ptr(o16, "geo"), _lib.ptr(raw4, "raw4"),
                  _lib.ptr(keep, "keep", dtype=torch.bool, allow_none=True), P, _head_struct(head),
                  _lib.ptr(raw7, "raw7"), _lib.stream())
        return raw7
    if rows.shape[0] < P:
        raise ValueError(f"normal head: {rows.shape[0]} rows for {P} points")
    keep_m = torch.empty_like(keep)
    _lib.call("nerf_normal_head_fwd_rows", _lib.ptr(o16, "geo"), _lib.ptr(raw4, "raw4"),
              _lib.ptr(keep, "keep", dtype=torch.bool), _lib.ptr(rows, "rows", torch.int32), P, _head_struct(head),
              _lib.ptr(raw7, "raw7"), _lib.ptr(keep_m, "keep_out", dtype=torch.bool), _lib.stream())
    return raw7, keep_m


def _head_backward(o16, keep, head, g7, needs):
    """-> (graw4 [P,4], dgeo [P,16]); the head's weight gradients are ACCUMULATED into .grad by the
    kernel (csrc/normals.hip sums them over the points in-kernel), for those of (N0, b0, N1, b1) that
    require grad (the others go to scratch)."""
    P = o16.shape[0]
    f = dict(device=o16.device, dtype=torch.float32)
    graw4, dgeo = torch.empty(P, 4, **f), torch.empty(P, 16, **f)
    g = _lib.NormalHeadGrads()
    bufs = [accumulate_grad_buffers([t])[0] if need else torch.zeros_like(t) for t, need in zip(head, needs)]
    for name, t in zip(("n0", "b0", "n1", "b1"), bufs):
        setattr(g, name, _lib.ptr(t, "grad_normal_net." + name).value)
    ws = _head_workspace(o16.device)
    _lib.call("nerf_normal_head_bwd", _lib.ptr(o16, "geo"), _lib.ptr(keep, "keep", dtype=torch.bool, allow_none=True),
              P, _head_struct(head), _lib.ptr(g7.contiguous(), "grad_raw"), _lib.ptr(graw4), _lib.ptr(dgeo), g,
              _lib.ptr(ws, "head_workspace"), ws.numel() * 4, _lib.stream())
    return graw4, dgeo


_HEAD_WS = {}


def _head_workspace(device):
    """Per-block partial sums of the head's weight gradients (one per device, fixed size; a captured
    graph keeps its address, so it is never replaced)."""
    key = str(device)
    if key not in _HEAD_WS:
        _HEAD_WS[key] = torch.empty(int(_lib.load().nerf_normal_head_bwd_workspace_bytes()) // 4, device=device)
    return _HEAD_WS[key]


class MLPFn(torch.autograd.Function):
    """x [P, 48] = [hash feat 32 | SH 16] -> raw [P, 4] (or [P, 7] with the normals head). MLP weight
    grads accumulate into .grad; the head's are returned to autograd."""

    @staticmethod
    def forward(ctx, x, net, *params):
        weights, head = params[:5], params[5:]
        x = x.contiguous()
        P = x.shape[0]
        raw = torch.empty(P, 4, device=x.device, dtype=torch.float32)
        o16 = torch.empty(P, 16, device=x.device, dtype=torch.float32) if head else None
        xp = _lib.ptr(x, "x")
        sh_ptr = _lib.c_vp(x.data_ptr() + 32 * 4) if P > 0 else xp
        feat_args = (xp, 48, 2, sh_ptr, 48, None, 1, None)
        w0q, arec = net.quant_state(lambda w0q: _act_calibration(feat_args, P, weights, w0q, P))
        _lib.call("nerf_mlp_fwd_q", *feat_args, P, _weights_struct(weights, w0q), _lib.ptr(raw, "raw"),
                  _lib.ptr(o16, "geo", allow_none=True), _lib.ptr(arec, "act_record", allow_none=True), None, 0,
                  _lib.stream())
        if head:
            raw = _head_forward(o16, raw, None, head)
        ctx.save_for_backward(x, o16, w0q, arec, *params)
        ctx.n_head = len(head)
        ctx.eval_quant = net.use_quantization and not net.training
        return raw

    @staticmethod
    def backward(ctx, g_raw):
        x, o16, w0q, arec, *params = ctx.saved_tensors
        weights, head = params[:5], params[5:]
        P = x.shape[0]
        _no_eval_quant_grad(ctx)
        g = g_raw.contiguous()
        head_grads, dgeo = (None,) * ctx.n_head, None
        if head:
            g, dgeo = _head_backward(o16, None, head, g, ctx.needs_input_grad[7:11])
        need_x = ctx.needs_input_grad[0]
        dx = torch.zeros_like(x) if need_x else None
        if any(w.requires_grad for w in weights) or need_x:
            grads = _grads_struct(weights) if any(w.requires_grad for w in weights) else _scratch_grads(weights)
            xp = _lib.ptr(x, "x")
            sh_ptr = _lib.c_vp(x.data_ptr() + 32 * 4) if P > 0 else xp
            dfeat = _lib.ptr(dx, "dx") if need_x else None
            dsh = None
            if need_x:
                dsh_t = torch.empty(P, 16, device=x.device, dtype=torch.float32)
                dsh = _lib.ptr(dsh_t, "dsh")
            _lib.call("nerf_mlp_bwd_q", xp, 48, 2, sh_ptr, 48, None, 1, None, P, _weights_struct(weights, w0q),
                      _lib.ptr(g, "grad_raw"), grads, dfeat, dsh, _lib.ptr(dgeo, "dgeo", allow_none=True),
                      _lib.ptr(arec, "act_record", allow_none=True), _lib.stream())
            if need_x:
                dx[:, 32:] = dsh_t
        return (dx, None) + (None,) * len(weights) + tuple(head_grads)


def _no_eval_quant_grad(ctx):
    if ctx.eval_quant:
        raise NotImplementedError("NeRFSmall: backward through eval-mode A-CAQ quantizers (round(.) with a zero "
                                  "gradient) is not implemented; train in training mode as the reference does")


def _scratch_grads(weights):
    g = _lib.MlpGrads()
    for name, t in zip(("w0", "w1", "c0", "c1", "c2"), weights):
        setattr(g, name, _lib.ptr(torch.zeros_like(t), "scratch").value)
    return g


def _point_order(order):
    """nerf_point_order of (io_rows, seg_split, spr2), or None (the identity)."""
    if order is None:
        return None
    rows, split, spr2 = order
    return _lib.PointOrder(_lib.ptr(rows, "io_rows", torch.int32).value, split, spr2)


class FieldFn(torch.autograd.Function):
    """Fused run_network: pts [P,3], viewdirs [R,3] (P = R*S) -> raw [P,4] ([P,7] with normals)."""

    @staticmethod
    def forward(ctx, pts, viewdirs, samples_per_ray, embedder, net, netchunk, reuse, *params):
        if pts.requires_grad or viewdirs.requires_grad:
            raise NotImplementedError("run_network: gradients w.r.t. positions/directions are not implemented")
        n_tab = embedder.n_levels
        tables, weights, head = params[:n_tab], params[n_tab:n_tab + 5], params[n_tab + 5:]
        pts = pts.contiguous()
        sh_rays = getattr(viewdirs, "_nerf_sh", None)   # render_rays' per-ray SH4 rows (sh_stride 0)
        viewdirs = viewdirs.contiguous()
        P = pts.shape[0]
        dev = pts.device
        # the activation quantizer calibrates on the first netchunk points (run_nerf.py:43-50, :64)
        n_calib = P if netchunk is None else min(P, netchunk)
        # coarse-feature reuse (render.CoarseReuse): plain fp32 tables with a binned backward
        plain = not embedder.quantization_active() and embedder.binned_backward()
        ctx.reuse = order = None
        spr = samples_per_ray
        if (reuse is not None and plain and reuse.matches(embedder, tables, P)
                and (not net.use_quantization or n_calib >= P)):   # calibration over all points: any order
            # fine pass: the importance samples are gathered into the head rows of the reuse buffer, whose
            # tail holds the coarse pass's features; the MLP walks that importance-first order
            feat, keep, row0 = reuse.feat, reuse.keep, 0
            embedder.encode_into(reuse.imp_pts.view(-1, 3), feat, 2, 2 * P, keep)
            order = (reuse.inv, reuse.R * reuse.N, reuse.S)
            spr = reuse.N
            reuse.state = "used"
            ctx.reuse = ("fine", reuse)
        elif reuse is not None and plain and reuse.state == "armed" and P == reuse.R * reuse.S:
            feat, keep, row0 = reuse.alloc(n_tab, dev)      # coarse pass: the tail rows of the reuse buffer
            embedder.encode_into(pts, feat, 2, 2 * feat.shape[1], keep, row0=row0)
            reuse.record(pts, embedder, tables)
            ctx.reuse = ("coarse", reuse)
        else:
            feat = torch.empty(n_tab, P, 2, device=dev, dtype=torch.float32)
            keep, row0 = torch.empty(P, device=dev, dtype=torch.bool), 0
            embedder.encode_into(pts, feat, 2, 2 * P, keep)
        sl = 2 * feat.shape[1]
        keep = keep[row0:row0 + P]                   # the MLP's keep flags, in its point order
        raw = torch.empty(P, 4, device=dev, dtype=torch.float32)
        o16 = torch.empty(P, 16, device=dev, dtype=torch.float32) if head else None
        # with the normals head, run_network's mask lands on n_z, not sigma (run_nerf.py:66); the head
        # runs in the merged order of raw / geo
        keep_arg = None if head else _lib.ptr(keep, "keep", dtype=torch.bool)
        if sh_rays is not None:
            view_args = (_lib.ptr(sh_rays, "sh_rows"), 0, None)
        else:
            view_args = (None, 0, _lib.ptr(viewdirs, "viewdirs"))
        feat_args = (_lib.ptr_at(feat, 2 * row0, "feat"), 2, sl, *view_args, spr, keep_arg)
        w0q, arec = net.quant_state(lambda w0q: _act_calibration(feat_args, P, weights, w0q, n_calib))
        # a training forward keeps layer C1's outputs for the backward (nerf_mlp_fwd_h3: 256 B per point;
        # the backward then skips C1's recompute) — not with the activation quantizer (its backward
        # recomputes) or active-point lists (the backward walks other tiles)
        h3 = None
        if (_SAVE_H3["on"] and arec is None and not _ACTIVE["on"] and P > 0
                and any(ctx.needs_input_grad[7:7 + n_tab + 5])):
            h3 = torch.empty(int(_lib.load().nerf_mlp_h3_bytes(P)) // 4, device=dev, dtype=torch.float32)
        _lib.call("nerf_mlp_fwd_h3", *feat_args, P, _weights_struct(weights, w0q), _lib.ptr(raw, "raw"),
                  _lib.ptr(o16, "geo", allow_none=True), _lib.ptr(arec, "act_record", allow_none=True), None, 0,
                  _point_order(order), _lib.ptr(h3, "h3", allow_none=True), _lib.stream())
        ctx.h3 = h3
        if head and order is not None:   # keep scattered to the merged rows by the head's own launch
            raw, keep = _head_forward(o16, raw, keep, head, rows=order[0])
        elif head:
            raw = _head_forward(o16, raw, keep, head)
        ctx.save_for_backward(pts, viewdirs, feat, keep, o16, w0q, arec, *params)
        ctx.spr, ctx.embedder, ctx.n_tab, ctx.n_head = spr, embedder, n_tab, len(head)
        ctx.sh_rays = sh_rays
        ctx.frow0, ctx.order = row0, order
        ctx.eval_quant = net.use_quantization and not net.training
        ctx.zero_tab_grad = embedder.quantization_active() and not embedder.training
        return raw

    @staticmethod
    def backward(ctx, g_raw):
        pts, viewdirs, feat, keep, o16, w0q, arec, *params = ctx.saved_tensors
        n_tab = ctx.n_tab
        tables, weights, head = params[:n_tab], params[n_tab:n_tab + 5], params[n_tab + 5:]
        P = pts.shape[0]
        _no_eval_quant_grad(ctx)
        g = g_raw.contiguous()
        head_grads, dgeo = (None,) * ctx.n_head, None
        if head:
            g, dgeo = _head_backward(o16, keep, head, g, ctx.needs_input_grad[7 + n_tab + 5:])
        need_tab = any(t.requires_grad for t in tables) and not ctx.zero_tab_grad
        need_w = any(w.requires_grad for w in weights)
        if need_w or need_tab:
            job = _FieldJob(pts, viewdirs, feat, keep, head, w0q, arec, weights, tables, g, dgeo, ctx, need_w,
                            need_tab)
            if torch._C._current_graph_task_id() != -1:
                _pending_field(pts.device).add(job)   # launched with the pass's other FieldFn backwards
            else:
                _run_field_jobs([job])
        return (None,) * (7 + n_tab + len(weights)) + tuple(head_grads)


class _FieldJob:
    """Everything one FieldFn backward needs after its autograd node has returned."""

    def __init__(self, pts, viewdirs, feat, keep, head, w0q, arec, weights, tables, g, dgeo, ctx, need_w, need_tab):
        self.pts, self.viewdirs, self.feat, self.keep, self.head = pts, viewdirs, feat, keep, head
        self.w0q, self.arec, self.weights, self.tables, self.g, self.dgeo = w0q, arec, weights, tables, g, dgeo
        self.spr, self.meta, self.need_w, self.need_tab = ctx.spr, ctx.embedder._meta, need_w, need_tab
        self.sh_rays = ctx.sh_rays
        self.reuse = ctx.reuse     # (role, render.CoarseReuse) or None
        self.frow0, self.order = ctx.frow0, ctx.order   # feature rows from frow0 of feat; the MLP's point order
        self.h3 = getattr(ctx, "h3", None)               # the forward's saved C1 outputs (or None: recompute)
        self.stream = torch.cuda.current_stream()

    def alloc(self):
        P = self.pts.shape[0]
        self.dfeat = torch.empty(self.feat.shape[0], P, 2, device=self.feat.device) if self.need_tab else None

    def mlp_job(self):
        P = self.pts.shape[0]
        j = _lib.MlpBwdJob()
        j.feat = _lib.ptr_at(self.feat, 2 * self.frow0, "feat")
        j.feat_stride_point, j.feat_stride_level = 2, 2 * self.feat.shape[1]
        j.dfeat_stride_point, j.dfeat_stride_level = 2, 2 * P
        if self.order is not None:
            j.order = _point_order(self.order)
        if self.sh_rays is not None:   # per-ray SH rows (sh_stride 0)
            j.sh, j.sh_stride, j.viewdirs = _lib.ptr(self.sh_rays, "sh_rows"), 0, None
        else:
            j.viewdirs = _lib.ptr(self.viewdirs, "viewdirs")
        j.samples_per_ray = self.spr
        j.keep = None if self.head else _lib.ptr(self.keep, "keep", dtype=torch.bool)
        j.n_points = P
        j.weights = _weights_struct(self.weights, self.w0q)
        j.graw = _lib.ptr(self.g, "grad_raw")
        j.grads = _grads_struct(self.weights) if self.need_w else _scratch_grads(self.weights)
        j.dfeat = _lib.ptr(self.dfeat, "dfeat", allow_none=True)
        j.dgeo = _lib.ptr(self.dgeo, "dgeo", allow_none=True)
        j.act_qrec = _lib.ptr(self.arec, "act_record", allow_none=True)
        if getattr(self, "act", None) is not None:
            j.rows = _lib.ptr(self.act[0], "active_rows", torch.int32)
            j.d_count = self.count_ptr(0)
        elif self.h3 is not None:
            j.h3 = _lib.ptr(self.h3, "h3")
        return j

    def find_active(self, jobs):
        """The active points of this backward (nerf_active_rows: points whose upstream gradient row is not
        all zero), in the MLP's point order, before its MLP backward: self.act = (rows, counts) and
        j.rows / j.d_count of the MLP job (counts[1]: the active importance samples of a reuse fine pass,
        the list's prefix). Feature-gradient rows that a bin reads but the active-point backward does not
        write are zeroed here: the coarse points' rows of a reuse pair (the merged coarse bin walks every
        coarse point)."""
        P = self.pts.shape[0]
        self.act = None
        if not _ACTIVE["on"] or P == 0:
            return
        role, plan = self.reuse if (self.reuse is not None and self.reuse[1].used) else (None, None)
        partner = None if plan is None else next(
            (k for k in jobs if k is not self and k.reuse is not None and k.reuse[1] is plan), None)
        dev = self.pts.device
        i32 = dict(device=dev, dtype=torch.int32)
        rows, counts = torch.empty(P, **i32), torch.empty(2, **i32)
        graw_rows = zero = None
        n_first = 0
        if role == "fine":   # the MLP walks the importance-first order; graw / dgeo are in the merged one
            graw_rows, n_first = self.order[0], plan.R * plan.N
            zero = self.dfeat if self.need_tab else None
        elif self.need_tab and role == "coarse" and partner is not None and partner.need_tab:
            zero = self.dfeat
        ws = torch.empty(int(_lib.load().nerf_active_rows_workspace_bytes(P)) // 4, **i32)
        _lib.call("nerf_active_rows", _lib.ptr(self.g, "grad_raw"), _lib.ptr(self.dgeo, "dgeo", allow_none=True), P,
                  _lib.ptr(graw_rows, "graw_rows", torch.int32, True), n_first, _lib.ptr(rows, "rows", torch.int32),
                  _lib.ptr(counts, "counts", torch.int32), _lib.ptr(zero, "zero_feat", allow_none=True), 2 * P,
                  len(self.tables), _lib.ptr(ws, "workspace", torch.int32), ws.numel() * 4, _lib.stream())
        self.act = (rows, counts)
        # the points the bins walk: a reuse pair's coarse bin walks every coarse point (zeroed rows), the
        # fine one the active importance samples; otherwise the active rows
        binned = "all" if (role == "coarse" and zero is not None) else ("first" if role == "fine" else "rows")
        _LAST_ACTIVE.append((counts, P, binned))

    def count_ptr(self, k):
        """Device pointer of counts[k] of the active lists."""
        return _lib.c_vp(self.act[1].data_ptr() + 4 * k)


_DETERMINISTIC = {"on": False, "ws": {}}
_SAVE_H3 = {"on": os.environ.get("NERF_SAVE_H3", "1") != "0"}   # the env switch: A/B runs


def set_save_h3(enabled=True):
    """Keep layer C1's outputs of a training forward for the backward (default on: 256 B per point,
    the backward skips C1's recompute, bit-identical); off = recompute (tests, A/B)."""
    _SAVE_H3["on"] = bool(enabled)
_BIN_BATCH = {"on": True}


def set_bin_batch(enabled=True):
    """The hash bins of a backward pass (fine + coarse) as one launch (nerf_hash_encode_bwd_bin_batch;
    default on, the same workspace contents as one launch each)."""
    _BIN_BATCH["on"] = bool(enabled)
_ACTIVE = {"on": False}
_LAST_ACTIVE = []    # (device counts, points) of the last field backward's jobs (bench.py reports them)


def last_active_units():
    """Of the last field backward (a host sync; None without active lists): the fraction of its points
    that were active, the points its MLP backward walked and the points its hash bins walked."""
    if not _LAST_ACTIVE:
        return None
    mlp = sum(int(c[0]) for c, _, _ in _LAST_ACTIVE)
    binned = sum(P if b == "all" else int(c[1]) if b == "first" else int(c[0]) for c, P, b in _LAST_ACTIVE)
    return {"fraction": mlp / max(1, sum(P for _, P, _ in _LAST_ACTIVE)), "mlp_points": mlp, "hash_points": binned}


def set_active_points(enabled=True):
    """Walk only the active points in the field backward (nerf_active_rows): the MLP backward and the
    hash bins skip the samples whose raw gradient is all zero (relu(sigma + noise) = 0: no alpha, no
    weight, no sigma gradient, run_nerf.py:364-386), whose terms in every gradient sum are exactly 0.
    Off by default: the two compaction launches cost ~32 us per lego step, which pays once more than
    ~7 % of the samples are inactive — a trained scene's empty space — but the bench's synthetic
    training has every sample active after ~10 iterations (tools/grad_sparsity.py)."""
    _ACTIVE["on"] = bool(enabled)


def active_points():
    return _ACTIVE["on"]


def set_deterministic(enabled=True):
    """Bitwise-reproducible backward (the `deterministic` flag of SURVEY.md §8(b)'s hash_encode_bwd):
    MLP weight gradients reduced over blocks in a fixed order and the hash-table gradients summed in
    exact integer fixed point (csrc/field_x6.hip mlp_wgrad_reduce, csrc/hashgrid.hip owner<DET>)."""
    from . import hashgrid
    _DETERMINISTIC["on"] = bool(enabled)
    hashgrid.set_deterministic(enabled)
    if enabled and torch.cuda.is_available():   # allocated now, not inside a later HIP-graph capture
        _det_workspace(torch.device("cuda", torch.cuda.current_device()))


def deterministic():
    return _DETERMINISTIC["on"]


def _det_workspace(device):
    if not _DETERMINISTIC["on"]:
        return None
    key = str(device)
    ws = _DETERMINISTIC["ws"].get(key)
    if ws is None:
        n = int(_lib.load().nerf_mlp_bwd_det_workspace_bytes()) // 4
        ws = _DETERMINISTIC["ws"][key] = torch.empty(n, device=device, dtype=torch.float32)
    return ws


def _run_field_jobs(jobs):
    """MLP backwards of up to two nets per launch (nerf_mlp_bwd_batch), then the hash backwards (and
    the pass's TV backwards, losses.TVBinJob) binned side by side and summed by one owner pass."""
    from .render import CompositeJob, run_composite_jobs
    run_composite_jobs([j for j in jobs if isinstance(j, CompositeJob)])    # the fields' raw gradients
    tv_jobs = [j for j in jobs if not isinstance(j, (_FieldJob, CompositeJob))]
    jobs = [j for j in jobs if isinstance(j, _FieldJob)]
    if jobs:
        ws = _det_workspace(jobs[0].pts.device)
        for j in jobs:
            j.alloc()
        _LAST_ACTIVE.clear()
        for j in jobs:
            j.find_active(jobs)
        for k in range(0, len(jobs), _lib.MLP_MAX_JOBS):
            part = jobs[k:k + _lib.MLP_MAX_JOBS]
            arr = (_lib.MlpBwdJob * len(part))(*[j.mlp_job() for j in part])
            _lib.call("nerf_mlp_bwd_batch", arr, len(part), _lib.ptr(ws, "det_workspace", allow_none=True),
                      0 if ws is None else ws.numel() * 4, _lib.stream())
    tab_jobs = [j for j in jobs if j.need_tab]
    if tab_jobs or tv_jobs:
        dev = (tab_jobs[0].pts if tab_jobs else tv_jobs[0].g).device
        pb = pending_bins(dev)
        bins = [b for j in tab_jobs for b in _bin_items(j, tab_jobs)]
        pb.reserve(sum(bin_chunks(b["n"]) for b in bins) + sum(j.n_chunks for j in tv_jobs))
        if _BIN_BATCH["on"]:
            pb.begin_batch()  # the pass's bins as one launch (nerf_hash_encode_bwd_bin_batch_tv: TV bins in front)
        try:
            for j in tv_jobs:
                pb.add_tv(j, queue=False)
            for b in bins:
                j = b.pop("job")
                hash_encode_bwd(b.pop("xyz"), j.meta, b.pop("dfeat"), 2, b.pop("sl"), accumulate_grad_buffers(j.tables),
                                defer=True, queue=False, **b)
        finally:
            if _BIN_BATCH["on"]:
                pb.end_batch()
        pb.flush()
    for j in jobs:
        j.dfeat = None


def _bin_items(j, jobs):
    """The bin launches of one FieldFn backward (hash_encode_bwd keyword sets). With the coarse-feature
    reuse (render.CoarseReuse) the fine job bins its importance samples only (the head rows of its
    importance-first d feat), and the fine d feat of the coarse points (its tail rows) is added to the
    coarse job's own (dfeat2):
    each point shared by the two passes is binned once with the sum of both gradients. Without the
    coarse job in this batch (its output was not differentiated), the fine job bins the coarse points
    itself with the fine d feat alone."""
    P = j.pts.shape[0]
    plain = dict(job=j, xyz=j.pts, dfeat=j.dfeat, sl=2 * P, n=P)
    act = getattr(j, "act", None)
    # with active lists: the bin walks the active rows only (count on the device)
    listed = dict(plain, rows=act[0], count=j.count_ptr(0)) if act is not None else plain
    if j.reuse is None or not j.reuse[1].used:
        return [listed]
    role, plan = j.reuse
    partner = next((k for k in jobs if k is not j and k.reuse is not None and k.reuse[1] is plan), None)
    n_imp = plan.R * plan.N    # the fine d feat is in importance-first order: [importance | coarse points]
    if role == "coarse":
        if partner is None:
            return [listed]
        # every coarse point: its inactive rows were zeroed (find_active), and so were the fine ones
        return [dict(plain, dfeat2=partner.dfeat, dfeat2_row0=n_imp, sl2=2 * partner.pts.shape[0])]
    if act is not None:   # the active importance samples: the prefix of the active list
        out = [dict(plain, xyz=plan.imp_pts, n=n_imp, rows=act[0], count=j.count_ptr(1))]
    else:
        out = [dict(plain, xyz=plan.imp_pts, n=n_imp)]
    if partner is None:
        Pc = plan.R * plan.S
        out.append(dict(job=j, xyz=plan.pts, dfeat=None, sl=2 * Pc, n=Pc, dfeat2=j.dfeat, dfeat2_row0=n_imp, sl2=2 * P))
    return out


class _PendingField:
    """FieldFn backwards of the running autograd pass (per device). The coarse and the fine field of a
    training iteration are independent autograd subgraphs whose MLP backwards are both ready once
    autograd reaches the first of them; they are queued here and launched together as the pass's
    final callback (one nerf_mlp_bwd_batch launch for both nets, then one owner pass for both hash
    backwards). Under a HIP-graph capture the callback is captured like the rest of the backward."""

    def __init__(self):
        self.jobs = []

    def add(self, job):
        if not self.jobs:
            torch.autograd.Variable._execution_engine.queue_callback(self.flush)
        self.jobs.append(job)

    def flush_composites(self):
        """Launch the queued compositing backwards now (render._RawGuardFn)."""
        from .render import CompositeJob, run_composite_jobs
        comp = [j for j in self.jobs if isinstance(j, CompositeJob)]
        if comp:
            self.jobs = [j for j in self.jobs if not isinstance(j, CompositeJob)]
            with torch.cuda.stream(comp[0].stream):
                run_composite_jobs(comp)

    def flush(self):
        jobs, self.jobs = self.jobs, []
        if not jobs:
            return
        stream = jobs[0].stream
        for j in jobs[1:]:
            if j.stream != stream:
                stream.wait_stream(j.stream)
        with torch.cuda.stream(stream):
            _run_field_jobs(jobs)
        cur = torch.cuda.current_stream()
        if cur != stream:
            cur.wait_stream(stream)


_PENDING_FIELD = {}


def _pending_field(device):
    return _PENDING_FIELD.setdefault(str(device), _PendingField())


class NeRFSmall(nn.Module):
    """run_nerf_helpers.py:169-306 on the fused MFMA MLP. create_nerf builds it with
    num_layers=2, hidden_dim=64, geo_feat_dim=15, num_layers_color=3, hidden_dim_color=64,
    input_ch=32 (hash), input_ch_views=16 (SH) — the only shape the kernel implements."""

    def __init__(self, num_layers=3, hidden_dim=64, geo_feat_dim=15, num_layers_color=4, hidden_dim_color=64,
                 input_ch=3, input_ch_views=3, use_quantization=False, quantization_bits=8, predict_normals=False):
        super().__init__()
        shape = (num_layers, hidden_dim, geo_feat_dim, num_layers_color, hidden_dim_color, input_ch, input_ch_views)
        if shape != (2, 64, 15, 3, 64, 32, 16):
            raise NotImplementedError(f"NeRFSmall{shape}: the HIP MLP implements create_nerf's configuration "
                                      "(2, 64, 15, 3, 64, 32, 16)")
        self.input_ch = input_ch
        self.input_ch_views = input_ch_views
        self.use_quantization = use_quantization
        self.num_layers = num_layers
        self.geo_feat_dim = geo_feat_dim
        self.num_layers_color = num_layers_color
        self.predict_normals = predict_normals
        self.sigma_net = nn.ModuleList([nn.Linear(input_ch, hidden_dim, bias=False),
                                        nn.Linear(hidden_dim, 1 + geo_feat_dim, bias=False)])
        if use_quantization:   # run_nerf_helpers.py:207-233
            self.sigma_act_quantizers = nn.ModuleList([
                LearnedBitwidthQuantizer(init_bits=float(quantization_bits), min_bits=2.0, max_bits=32.0,
                                         symmetric=False) for _ in range(num_layers - 1)])
            self.sigma_weight_quantizer = LearnedBitwidthQuantizer(init_bits=float(quantization_bits), min_bits=2.0,
                                                                   max_bits=32.0, symmetric=True)
        else:
            self.sigma_act_quantizers = None
            self.sigma_weight_quantizer = None
        self.color_net = nn.ModuleList([nn.Linear(input_ch_views + geo_feat_dim, hidden_dim_color, bias=False),
                                        nn.Linear(hidden_dim_color, hidden_dim_color, bias=False),
                                        nn.Linear(hidden_dim_color, 3, bias=False)])
        if predict_normals:   # run_nerf_helpers.py:259-263
            self.normal_net = nn.Sequential(nn.Linear(geo_feat_dim, hidden_dim // 2), nn.ReLU(),
                                            nn.Linear(hidden_dim // 2, 3))

    def quant_state(self, act_calibration):
        """(W0q, activation record) for one forward, or (None, None) without quantization.
        run_nerf_helpers.py:272-284: W0 goes through sigma_weight_quantizer (symmetric) and the
        layer-0 ReLU output through sigma_act_quantizers[0] (asymmetric), both calibrating on their
        first training call. act_calibration(W0q) -> stats runs the calibration-only MLP launch."""
        if not self.use_quantization:
            return None, None
        wq, aq = self.sigma_weight_quantizer, self.sigma_act_quantizers[0]
        W0 = self.sigma_net[0].weight
        if self.training and not wq.calibrated:
            wq.calibrate(W0)
        if self.training and not aq.calibrated:
            w0q = _fake_quant(W0, wq.record())
            calibrate_from_stats([aq], act_calibration(w0q))
            return w0q, aq.record()
        recs = quant_records([wq, aq], self.training)
        return _fake_quant(W0, recs[0]), recs[1]

    def mlp_weights(self):
        return [self.sigma_net[0].weight, self.sigma_net[1].weight, self.color_net[0].weight,
                self.color_net[1].weight, self.color_net[2].weight]

    def head_params(self):
        """Normals head parameters (N0, b0, N1, b1), or [] without the head."""
        if not self.predict_normals:
            return []
        return [self.normal_net[0].weight, self.normal_net[0].bias, self.normal_net[2].weight,
                self.normal_net[2].bias]

    def field_params(self):
        return self.mlp_weights() + self.head_params()

    @property
    def raw_channels(self):
        return 7 if self.predict_normals else 4

    def forward(self, x):
        for w in self.field_params():
            if not w.is_contiguous():
                raise ValueError("NeRFSmall: weights must be contiguous")
        return MLPFn.apply(x.float(), self, *self.field_params())


def batchify(fn, chunk):
    """run_nerf.py:43-50."""
    if chunk is None:
        return fn

    def ret(inputs):
        return torch.cat([fn(inputs[i:i + chunk]) for i in range(0, inputs.shape[0], chunk)], 0)
    return ret


def run_network(inputs, viewdirs, fn, embed_fn, embeddirs_fn, netchunk=1024 * 64):
    """run_nerf.py:53-68. inputs [..., S, 3], viewdirs [R, 3]. Fused when the modules are ours;
    netchunk is then only a memory knob the fused kernels do not need."""
    fused = (isinstance(embed_fn, HashEmbedder) and isinstance(fn, NeRFSmall)
             and isinstance(embeddirs_fn, SHEncoder) and viewdirs is not None and inputs.dim() == 3)
    if fused:
        if embed_fn.training:
            embed_fn.current_step += 1
        R, S = inputs.shape[0], inputs.shape[1]
        reuse = getattr(inputs, "_nerf_reuse", None)     # render.CoarseReuse of this render_rays call
        raw = FieldFn.apply(inputs.reshape(-1, 3), viewdirs, S, embed_fn, fn, netchunk, reuse,
                            *embed_fn.tables(), *fn.field_params())
        out = raw.reshape(R, S, fn.raw_channels)
        # without a normals head FieldFn's backward only queues its job: raw2outputs may then defer the
        # compositing backward too (render.CompositeJob)
        out._nerf_field_raw = fn.raw_channels == 4
        return out
    inputs_flat = torch.reshape(inputs, [-1, inputs.shape[-1]])
    embedded, keep_mask = embed_fn(inputs_flat)
    if viewdirs is not None:
        input_dirs = viewdirs[:, None].expand(inputs.shape)
        embedded = torch.cat([embedded, embeddirs_fn(torch.reshape(input_dirs, [-1, input_dirs.shape[-1]]))], -1)
    outputs_flat = batchify(fn, netchunk)(embedded)
    outputs_flat = outputs_flat.clone()
    outputs_flat[~keep_mask, -1] = 0
    return torch.reshape(outputs_flat, list(inputs.shape[:-1]) + [outputs_flat.shape[-1]])
