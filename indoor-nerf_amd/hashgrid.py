"""Multi-resolution hash encoding and SH view encoding on the HIP kernels.

API mirror of PocketNeRF/hash_encoding.py: HashEmbedder (:11-107) and SHEncoder (:110-191), same
constructor arguments, attributes, parameters (`embeddings.{i}.weight`, nn.Embedding(2^log2T, 2))
and return values. Forward and backward run in libnerfhip (csrc/hashgrid.hip, csrc/field.hip).
"""
import ctypes
import os

import torch
import torch.nn as nn

from . import _lib
from .quantization import LearnedBitwidthQuantizer, calibrate_from_stats, new_stats, quant_records


def level_resolutions(base_resolution, finest_resolution, n_levels):
    """floor(base * b**i) in float32 with b = exp((ln F - ln B)/(L-1)) (hash_encoding.py:28, :89),
    evaluated with the reference's tensor dtypes (int64 base/finest, float32 b) on the CPU."""
    b_res = torch.as_tensor(base_resolution).cpu()
    f_res = torch.as_tensor(finest_resolution).cpu()
    b = torch.exp((torch.log(f_res) - torch.log(b_res)) / (n_levels - 1))
    return [float(torch.floor(b_res * b ** i)) for i in range(n_levels)], b


def _bbox_floats(bounding_box):
    lo, hi = bounding_box
    lo = torch.as_tensor(lo, dtype=torch.float32).detach().cpu().reshape(3)
    hi = torch.as_tensor(hi, dtype=torch.float32).detach().cpu().reshape(3)
    return [float(v) for v in lo], [float(v) for v in hi]


# Deferred zero of hash-table gradients (GradArena(defer_tables=True).zero_): instead of a 64 MiB
# memset before the step, the iteration's binned owner pass STORES every table row
# (NERF_OWNER_OVERWRITE: the same bits as memset + accumulate, minus the memset and the owner's row
# loads). A deferred gradient's contents are stale until then; any other writer or reader
# materialises the zero first (materialize_zero), and train steps do so for whatever is still
# deferred after backward().
_DEFERRED = {}   # data_ptr -> gradient tensor


def defer_zero(grads):
    for g in grads:
        _DEFERRED[g.data_ptr()] = g


def materialize_zero(grads=None):
    """Zero deferred gradients now: the given ones (those of them that are deferred), or all (and every
    pending dense fill, _lib.defer_fill_zero)."""
    _lib.flush_zero_fills(grads)
    keys = list(_DEFERRED) if grads is None else [g.data_ptr() for g in grads if g.data_ptr() in _DEFERRED]
    for k in keys:
        _DEFERRED.pop(k).zero_()


def forget_deferred(grads):
    """Drop pending deferred zeros of these gradients (their owner zeroed them itself)."""
    for g in grads:
        _DEFERRED.pop(g.data_ptr(), None)


def take_deferred(grads):
    """True (and no longer deferred) when every gradient of an owner launch is deferred: the launch
    overwrites them. Otherwise any deferred ones among them are zeroed now and the launch adds."""
    if grads and all(g.data_ptr() in _DEFERRED for g in grads):
        for g in grads:
            del _DEFERRED[g.data_ptr()]
        return True
    materialize_zero(grads)
    return False


# Parameter-gather gates (dist.ShardedOptimizer(overlap=True).gather_params): the
# all-gather of each table bucket after the first runs on a side stream and is joined only where the
# next iteration first reads those levels. The hash forward launches the levels below a gate, joins
# it, then launches the levels from it on (encode_into); any other reader of the tables joins every
# pending gate first (join_tables). Under graph capture the gated forward is cut into graph segments
# at the same levels instead (split_next_forward), and the replay joins the gates between the segments.
class TableGate:
    """Levels [level, L) of a device's tables are being written by a side-stream collective: join()
    runs `finish` on the host once (the gloo rehearsal's wait + host->device copy; None on RCCL) and
    makes `stream` wait for `event`."""

    def __init__(self, level, event, finish=None):
        self.level, self.event, self.finish = int(level), event, finish

    def join(self, stream):
        if self.finish is not None:
            f, self.finish = self.finish, None
            f()
        stream.wait_event(self.event)


_GATES = {}    # str(device) -> [TableGate], ascending levels
_SPLITS = {}   # str(device) -> (levels, callback): the next hash forward is cut into graph segments


def gate_tables(device, gates):
    """Register the pending table gates of `device` (an older set is joined first)."""
    join_tables(device)
    if gates:
        _GATES[str(device)] = sorted(gates, key=lambda g: g.level)


def join_tables(device):
    """Make the current stream wait for every pending table gate of `device` (no-op without one)."""
    for g in _GATES.pop(str(device), ()):
        g.join(torch.cuda.current_stream(device))


def take_gates(device):
    """Remove and return the pending gates of `device` (the caller joins them)."""
    return _GATES.pop(str(device), [])


def split_next_forward(device, levels, split):
    """During a graph capture: cut the next hash forward on `device` before each of `levels`, calling
    split(level) there (graphs.GraphedTrainStep ends one graph segment and begins the next)."""
    if levels:
        _SPLITS[str(device)] = (sorted(int(v) for v in levels), split)
    else:
        _SPLITS.pop(str(device), None)


def accumulate_grad_buffers(params):
    """The fused backward kernels ACCUMULATE straight into .grad (like a fused optimizer's bucket):
    create zero grads where they are missing and return them."""
    out = []
    for p in params:
        if p.grad is None:
            p.grad = torch.zeros_like(p, memory_format=torch.contiguous_format)
        out.append(p.grad)
    return out


class HashEncodeFn(torch.autograd.Function):
    """xyz [P,3] -> (feat, keep). feat is [P, 2L] (layout 'point') or [L, P, 2] (layout 'level')."""

    @staticmethod
    def forward(ctx, xyz, embedder, layout, *tables):
        meta = embedder._meta
        if xyz.requires_grad:
            raise NotImplementedError("HashEmbedder: gradients w.r.t. positions are not implemented "
                                      "(the reference never back-propagates into sample positions)")
        xyz = xyz.contiguous()
        P, L = xyz.shape[0], len(tables)
        if layout == "point":
            feat = torch.empty(P, 2 * L, device=xyz.device, dtype=torch.float32)
            sp, sl = 2 * L, 2
        else:
            feat = torch.empty(L, P, 2, device=xyz.device, dtype=torch.float32)
            sp, sl = 2, 2 * P
        keep = torch.empty(P, device=xyz.device, dtype=torch.bool)
        embedder.encode_into(xyz, feat, sp, sl, keep)
        ctx.save_for_backward(xyz, *tables)
        ctx.meta, ctx.sp, ctx.sl = meta, sp, sl
        # eval-mode quantizers return (round(.) - zp) * scale: zero gradient w.r.t. the tables
        ctx.zero_grad = embedder.quantization_active() and not embedder.training
        ctx.mark_non_differentiable(keep)
        return feat, keep

    @staticmethod
    def backward(ctx, g_feat, g_keep):
        xyz, *tables = ctx.saved_tensors
        if g_feat is not None and any(t.requires_grad for t in tables):
            grads = accumulate_grad_buffers(tables)
            if not ctx.zero_grad:
                hash_encode_bwd(xyz, ctx.meta, g_feat.contiguous(), ctx.sp, ctx.sl, grads)
        return (None, None, None) + (None,) * len(tables)


_DET = {"on": False}


def set_deterministic(enabled=True):
    """Bitwise-reproducible hash-table gradients: the binned backward's owner pass sums in exact
    integer fixed point (nerf_hash_encode_bwd_* with deterministic = 1)."""
    _DET["on"] = bool(enabled)


def deterministic():
    return _DET["on"]


_BWD_WORKSPACE = {}
# Workspaces replaced by a larger one are never freed: a HIP graph captured earlier (graphs.
# GraphedTrainStep) keeps their addresses in its kernel arguments, and the caching allocator would
# hand the memory to someone else before the next replay. They are kept alive here instead (the
# workspace only grows, so this holds a few buffers at most).
_RETIRED = []


def bwd_workspace(n_levels, log2_T, n_points, device):
    """Device workspace of nerf_hash_encode_bwd_ws (the binned backward's per-chunk regions), one per
    device, grown to the largest (n_levels, n_points) seen; calls that share it run in stream order
    (autograd's backward stream). None when the binned path does not apply (log2_T > 19)."""
    det = int(_DET["on"])
    need = int(_lib.load().nerf_hash_encode_bwd_workspace_bytes(n_levels, log2_T, n_points, det))
    if need == 0:
        if det:
            raise NotImplementedError(f"deterministic hash backward: no binned path for log2_T {log2_T} (<= 19)")
        return None, 0
    key = str(device)
    hit = _BWD_WORKSPACE.get(key)
    if hit is None or hit[1] < need:
        old = _BWD_WORKSPACE.pop(key, None)
        if old is not None:
            _RETIRED.append(old[0])
        hit = _BWD_WORKSPACE[key] = (torch.empty(need, dtype=torch.uint8, device=device), need)
    return hit


class _PendingBins:
    """Binned hash backwards of the running autograd pass that await their owner pass (per device).
    The fine and the coarse pass of a training iteration are two HashEncode nodes scattering into
    the same tables: both bin into one workspace, side by side, and ONE owner launch sums them, queued
    as the pass's final callback (it runs before backward() returns, so .grad is complete, and under
    a HIP-graph capture it is captured like the rest of the backward)."""

    def __init__(self):
        self.ws, self.cap, self.used, self.peak = None, 0, 0, 0
        self.tag = self.grads = self.stream = None
        self.hold = False     # hold_owner(): the pass's owner launch is left to the caller (HeldOwner)
        self.held = None
        self.step_plan = None  # fused_table_step(): (optimizer, tables) whose step the owner pass runs
        self.batch = None      # begin_batch(): bin launches collected for one nerf_hash_encode_bwd_bin_batch

    def flush(self, final=True):
        """Launch (or hold) the owner pass of the open workspace. final=False: an early flush that makes
        room for more bins of the same pass (_slot) — its gradients are partial, so it never runs a fused
        table step."""
        if self.batch:
            self._drain_batch()           # collected bins of this workspace run before its owner pass
        if self.used == 0:
            return
        L, log2_T, _, det = self.tag
        flags = det | (OWNER_OVERWRITE if take_deferred(self.grads) else 0)
        step = None
        plan = self.step_plan
        if (plan is not None and final and not self.hold and (flags & OWNER_OVERWRITE)
                and [g.data_ptr() for g in self.grads] == [p.grad.data_ptr() for p in plan[1]]):
            self.step_plan = None          # one owner pass per plan
            step = plan[0].table_step(plan[1])
        _FUSED_STEP["last"] = step is not None
        held = HeldOwner(L, log2_T, self.used, self.cap, self.grads, flags, self.ws, step)
        self.last = (self.tag, self.used, self.cap)
        self.used, self.tag, self.grads = 0, None, None
        if self.hold:
            self.held = held
            return
        with torch.cuda.stream(self.stream):
            held.run(0, L)
        cur = torch.cuda.current_stream()
        if cur != self.stream:
            cur.wait_stream(self.stream)

    def take_held(self):
        """The owner pass held back by hold_owner() (HeldOwner), or None. It stays valid for replays of a
        captured step (same workspace, tables and chunk counts)."""
        return self.held

    def last_entry_count(self):
        """Entries the bins of the last owner pass's workspace emitted (nerf_hash_bwd_entry_count;
        a host sync — measurement only, e.g. bench.py's pricing of the hash backward), or None."""
        if getattr(self, "last", None) is None or self.ws is None:
            return None
        (L, log2_T, _, det), used, cap = self.last
        out = torch.zeros(1, dtype=torch.int64, device=self.ws.device)
        _lib.call("nerf_hash_bwd_entry_count", L, log2_T, used, cap, det,
                  _lib.ptr(self.ws, "workspace", dtype=torch.uint8), self.ws.numel(),
                  _lib.ptr(out, "count", dtype=torch.int64), _lib.stream())
        return int(out.item())

    def reserve(self, n_chunks):
        """Size the next workspace for n_chunks chunks, so that a batch whose total is known up front
        bins into ONE workspace and is summed by ONE owner pass (the sums then do not depend on the
        workspace history: the deterministic mode's results are reproducible from the first call)."""
        self.peak = max(self.peak, n_chunks)

    def _slot(self, L, log2_T, grad_tables, n_ch, device, queue):
        """Chunks [base, base + n_ch) of the open workspace for a bin launch into grad_tables: opens
        a workspace (flushing the previous one if it is for other tables or too small)."""
        lib = _lib.load()
        det = int(_DET["on"])
        tag = (L, log2_T, tuple(g.data_ptr() for g in grad_tables), det)
        total = (self.used if self.tag == tag else 0) + n_ch
        self.peak = max(self.peak, total)     # the next pass sizes its workspace for this
        if self.used and (self.tag != tag or total > self.cap):
            self.flush(final=False)
        if self.used == 0:
            cap = max(self.peak, n_ch)
            C = int(lib.nerf_hash_bwd_chunk_points())
            need = int(lib.nerf_hash_encode_bwd_workspace_bytes(L, log2_T, C * cap, det))
            if self.ws is None or self.ws.numel() < need:
                if self.ws is not None:
                    _RETIRED.append(self.ws)     # a captured graph may still bin into it
                self.ws = torch.empty(need, dtype=torch.uint8, device=device)
            self.cap = cap
            self.tag, self.grads, self.stream = tag, list(grad_tables), torch.cuda.current_stream()
            if queue:
                torch.autograd.Variable._execution_engine.queue_callback(self.flush)
        base = self.used
        self.used += n_ch
        return base, det

    def add(self, xyz, meta, dfeat, sp, sl, grad_tables, queue=True, n=None, rows=None, dfeat2=None, rows2=None,
            sp2=2, sl2=0, dfeat2_row0=0, count=None):
        """Bin n points (default: every row of xyz). rows / dfeat2 / rows2: the row maps of
        nerf_hash_encode_bwd_bin_rows (coarse-feature reuse); dfeat2_row0: dfeat2's rows start at that
        row of the tensor; count: device pointer of the number of listed rows (active points)."""
        d2 = _lib.ptr(dfeat2, "grad_feat2", allow_none=True)
        if d2 is not None:
            d2 = _lib.c_vp(d2.value + 4 * sp2 * int(dfeat2_row0))
        L, log2_T = len(grad_tables), meta["log2_T"]
        P = xyz.shape[0] if n is None else n
        base, det = self._slot(L, log2_T, grad_tables, bin_chunks(P), xyz.device, queue)
        job = _lib.BinJob(_lib.ptr(xyz, "xyz"), _lib.ptr(rows, "rows", torch.int32, True), count, P,
                          _lib.ptr(dfeat, "grad_feat", allow_none=True), sp, sl, d2,
                          _lib.ptr(rows2, "rows2", torch.int32, True), sp2, sl2, base)
        common = (meta["bmin"], meta["bmax"], meta["res"], L, log2_T)
        if self.batch is not None:
            key = (id(self.ws), self.cap, det, L, log2_T, id(meta["bmin"]), id(meta["bmax"]), id(meta["res"]))
            if self.batch and self.batch[0][1] != key:
                self._drain_batch()
            self.batch.append((job, key, common, det, (xyz, rows, dfeat, dfeat2, rows2)))
            return
        self._launch_bins([job], common, det)

    def _launch_bins(self, jobs, common, det, tv=None):
        if tv is not None:   # the pass's TV bins in the same launch (nerf_hash_encode_bwd_bin_batch_tv)
            _lib.call("nerf_hash_encode_bwd_bin_batch_tv", (_lib.BinJob * len(jobs))(*jobs), len(jobs), *common, self.cap,
                      det, _lib.ptr(self.ws, "workspace", dtype=torch.uint8), self.ws.numel(), tv[0], _lib.stream())
            return
        _lib.call("nerf_hash_encode_bwd_bin_batch", (_lib.BinJob * len(jobs))(*jobs), len(jobs), *common, self.cap, det,
                  _lib.ptr(self.ws, "workspace", dtype=torch.uint8), self.ws.numel(), _lib.stream())

    def begin_batch(self):
        """Collect the following add() / add_tv() calls of one workspace into one
        nerf_hash_encode_bwd_bin_batch(_tv) (end_batch; the fine and the coarse bins of an iteration and
        its TV bins then run as one launch)."""
        self.batch, self.batch_tv = [], None

    def _drain_batch(self):
        """Launch the collected bins (they target the open workspace) and keep collecting."""
        tv, self.batch_tv = getattr(self, "batch_tv", None), None
        if self.batch:
            _, _, common, det, _ = self.batch[0]
            self._launch_bins([b[0] for b in self.batch], common, det, tv)
            self.batch = []
        elif tv is not None:   # no hash bins in this workspace: the TV launch alone
            self._launch_tv(tv[1], tv[2])

    def end_batch(self):
        self._drain_batch()
        self.batch = None

    def add_tv(self, job, queue=True):
        """Bin a TV backward (losses.TVBinJob) into the open workspace: its gradient is summed by the
        same owner pass as the hash backwards of the iteration. Inside begin_batch() (with the forward's
        vertex rows) it rides in the batch's first hash bin launch, else it is a launch of its own."""
        L = len(job.tables)
        base, det = self._slot(L, job.log2_T, job.grads, job.n_chunks, job.tables[0].device, queue)
        if self.batch is not None and job.verts is not None and _TV_IN_BINS["on"]:
            if getattr(self, "batch_tv", None) is not None:
                self._drain_batch()           # one TV job per launch
            tabs = _lib.ptr_array(job.tables)
            ctv = _lib.TVBinJob(_lib.c_vp(ctypes.addressof(tabs)),
                                None if job.mv is None else _lib.c_vp(ctypes.addressof(job.mv)),
                                job.dmv, _lib.c_vp(ctypes.addressof(job.cb)), _lib.ptr(job.g, "grad_loss"),
                                _lib.ptr(job.verts, "tv_verts"), base)
            self.batch_tv = (ctv, job, base, tabs)   # tabs: the struct points into it
            return
        self._launch_tv(job, base)

    def _launch_tv(self, job, base):
        det = self.tag[3]
        _lib.call("nerf_tv_bwd_bin", _lib.ptr_array(job.tables), len(job.tables), job.log2_T, job.mv, job.dmv, job.cb,
                  _lib.ptr(job.g, "grad_loss"), _lib.ptr(job.verts, "tv_verts", allow_none=True), base, self.cap, det,
                  _lib.ptr(self.ws, "workspace", dtype=torch.uint8), self.ws.numel(), _lib.stream())


class HeldOwner:
    """An owner pass of a binned backward, launched by the caller, level range by level range
    (nerf_hash_encode_bwd_owner_range): a data-parallel step starts the reduce-scatter of each gradient
    bucket once its levels are summed (dist.ShardedOptimizer). `flags` (deterministic, overwrite) were
    fixed when the pass was held."""

    def __init__(self, L, log2_T, used, cap, grads, flags, ws, step=None):
        self.L, self.log2_T, self.used, self.cap, self.grads = L, log2_T, used, cap, list(grads)
        self.flags, self.ws, self.step = flags, ws, step

    def run(self, level_begin, level_end):
        """Launch the levels [level_begin, level_end) on the CURRENT stream (the caller's: after a replayed
        graph the capture stream is not ordered behind the replay); with a fused table step
        (fused_table_step) the tables' optimizer update runs in the same launch."""
        _lib.call("nerf_hash_encode_bwd_owner_step", self.L, level_begin, level_end, self.log2_T, self.used,
                  self.cap, _lib.ptr_array(self.grads, "grad_tables"), self.flags,
                  _lib.ptr(self.ws, "workspace", dtype=torch.uint8), self.ws.numel(), self.step, _lib.stream())


class hold_owner:
    """Context manager: inside it, the binned backwards' owner passes are not launched at the end of
    the autograd pass but held (pending_bins(device).take_held()) for the caller to run by level range.
    Only the caller that runs them may use it (dist.ShardedOptimizer.reduce_grads does)."""

    def __init__(self, device, enabled=True):
        self.pb, self.enabled = pending_bins(device), bool(enabled)

    def __enter__(self):
        self.prev, self.pb.hold = self.pb.hold, self.enabled or self.pb.hold
        if self.enabled:
            self.pb.held = None
        return self.pb

    def __exit__(self, *exc):
        self.pb.hold = self.prev
        return False


class EarlyTV:
    """A captured training step's TV forward (losses.tv_forward_early) awaiting the step's fine-pass
    compositing, which launches it (render.CompositeFn, nerf_composite_fwd_tv: the TV blocks beside the
    one-wave rays); total_variation_all takes it back after render. dmv: the device
    corner slots (drawn before every replay by a filler registered after render: the draw order of
    the separate launch); out: the zeroed [L] loss accumulator; verts: the vertex rows for the
    backward."""

    def __init__(self, tables, dmv, slot_off, cubes, log2_T, out, verts):
        self.tables, self.dmv, self.slot_off, self.cubes, self.log2_T = list(tables), dmv, slot_off, cubes, log2_T
        self.out, self.verts, self.launched = out, verts, False
        self.ptrs = _lib.ptr_array(self.tables)
        self.cb = (_lib.c_int * len(cubes))(*cubes)


_EARLY_TV = {}
_TV_FWD_FUSED = {"on": os.environ.get("NERF_TV_FWD_FUSED", "1") != "0"}   # the env switch: A/B runs


def set_tv_fwd_fused(enabled=True):
    """Launch a captured step's TV forward inside its fine-pass compositing launch (default on)."""
    _TV_FWD_FUSED["on"] = bool(enabled)


def early_tv(device):
    """The pending EarlyTV of `device` not launched yet, or None."""
    job = _EARLY_TV.get(torch.device(device).index)
    return job if job is not None and not job.launched else None


def register_early_tv(job):
    _EARLY_TV[job.out.device.index] = job


def take_early_tv(device):
    return _EARLY_TV.pop(torch.device(device).index, None)


_FUSED_STEP = {"on": True}
_TV_IN_BINS = {"on": os.environ.get("NERF_TV_IN_BINS", "1") != "0"}   # the env switch: A/B runs


def set_tv_in_bins(enabled=True):
    """Run a pass's binned TV backward inside its hash bin launch (default on; bit-identical)."""
    _TV_IN_BINS["on"] = bool(enabled)


def set_fused_table_step(enabled=True):
    """Fuse the hash tables' RAdam step into the iteration's owner pass (nerf_hash_encode_bwd_owner_step;
    on by default): model.train_step / graphs.GraphedTrainStep without a gradient hook (one process)
    and with the deferred table-gradient zero. Bit-identical to the owner pass + the optimizer's own
    launch; off = the two launches."""
    _FUSED_STEP["on"] = bool(enabled)


def fused_table_step_enabled():
    return _FUSED_STEP["on"]


def last_fused_table_step():
    """Whether the last owner pass launched (or captured) ran the tables' optimizer step (bench.py)."""
    return _FUSED_STEP.get("last", False)


class fused_table_step:
    """Context manager around an iteration's forward + backward: the owner pass of the tables' binned
    backward also applies `optimizer`'s step to them (RAdam.table_step), and optimizer.step() then
    skips them. Inactive (a no-op) when disabled, when the optimizer has no table_step, or when the
    pass is held for a gradient hook (data parallel: the gradients are reduced first)."""

    def __init__(self, device, optimizer, tables, enabled=True):
        self.pb = pending_bins(device)
        self.plan = ((optimizer, list(tables)) if (enabled and _FUSED_STEP["on"] and tables
                                                     and hasattr(optimizer, "table_step")) else None)

    def __enter__(self):
        self.pb.step_plan = self.plan
        return self

    def __exit__(self, *exc):
        self.pb.step_plan = None
        return False


def bin_chunks(n_points):
    """Chunks of the binned backward's workspace that n_points occupy (csrc/hashgrid.hip kChunkPts)."""
    C = int(_lib.load().nerf_hash_bwd_chunk_points())
    return (n_points + C - 1) // C


_PENDING = {}
OWNER_OVERWRITE = 2   # include/nerf_hip.h NERF_OWNER_OVERWRITE


def pending_bins(device):
    return _PENDING.setdefault(str(device), _PendingBins())


def hash_encode_bwd(xyz, meta, dfeat, sp, sl, grad_tables, defer=None, queue=True, **rows):
    """Scatter-add d feat into the gradient tables (hash_encoding.py:82-107 autograd; csrc/hashgrid.hip).
    defer (default: inside an autograd backward pass) bins now and leaves the owner pass to the end
    of the pass (_PendingBins), shared with the other hash backwards of the pass; queue=False leaves
    the owner pass to the caller (pending_bins(device).flush()). rows: n / rows / dfeat2 / rows2 / sl2
    of _PendingBins.add (binned path only)."""
    L, log2_T = len(grad_tables), meta["log2_T"]
    P = xyz.shape[0] if rows.get("n") is None else rows["n"]
    if defer is None:
        defer = torch._C._current_graph_task_id() != -1
    det = int(_DET["on"])
    if defer and P > 0 and int(_lib.load().nerf_hash_encode_bwd_workspace_bytes(L, log2_T, P, det)) > 0:
        pending_bins(xyz.device).add(xyz, meta, dfeat, sp, sl, grad_tables, queue=queue, **rows)
        return
    if any(rows.get(k) is not None for k in ("rows", "dfeat2", "count")):
        raise NotImplementedError("hash_encode_bwd: row maps need the binned path (log2_T <= 19, a deferred pass)")
    materialize_zero(grad_tables)
    ws, nbytes = bwd_workspace(len(grad_tables), meta["log2_T"], xyz.shape[0], xyz.device)
    _lib.call("nerf_hash_encode_bwd_ws", _lib.ptr(xyz, "xyz"), xyz.shape[0], meta["bmin"], meta["bmax"],
              meta["res"], len(grad_tables), meta["log2_T"], _lib.ptr(dfeat, "grad_feat"), sp, sl,
              _lib.ptr_array(grad_tables, "grad_tables"), det,
              _lib.ptr(ws, "workspace", dtype=torch.uint8, allow_none=True), nbytes, _lib.stream())


class HashEmbedder(nn.Module):
    """hash_encoding.py:11-107 on MI355X. forward(x [P,3]) -> (feat [P, L*F], keep [P] bool)."""

    def __init__(self, bounding_box, n_levels=16, n_features_per_level=2, log2_hashmap_size=19,
                 base_resolution=16, finest_resolution=512, use_quantization=False, quantization_bits=8):
        super().__init__()
        if n_features_per_level != 2:
            raise NotImplementedError("HashEmbedder: the HIP kernels implement n_features_per_level == 2")
        if not 1 <= n_levels <= _lib.MAX_LEVELS:
            raise ValueError(f"HashEmbedder: n_levels must be 1..{_lib.MAX_LEVELS}")
        self.bounding_box = bounding_box
        self.n_levels = n_levels
        self.n_features_per_level = n_features_per_level
        self.log2_hashmap_size = log2_hashmap_size
        self.base_resolution = torch.tensor(base_resolution)
        self.finest_resolution = torch.tensor(finest_resolution)
        self.out_dim = n_levels * n_features_per_level
        self.use_quantization = use_quantization
        self._packed = None
        self.warmup_steps = 500
        self.current_step = 0
        res, self.b = level_resolutions(self.base_resolution, self.finest_resolution, n_levels)
        self.embeddings = nn.ModuleList([nn.Embedding(2 ** log2_hashmap_size, n_features_per_level)
                                         for _ in range(n_levels)])
        for i, emb in enumerate(self.embeddings):
            nn.init.uniform_(emb.weight, a=-0.0001, b=0.0001)
            emb.weight._nerf_owner_grad = True   # every backward into it ends in an owner pass
            emb.weight._nerf_level = i           # dist.ShardedOptimizer's gather gates name levels
        # A-CAQ (hash_encoding.py:37-53): one asymmetric learned-bitwidth quantizer per level,
        # registered after the tables as in the reference (parameter order = optimizer state order)
        self.quantizers = nn.ModuleList([
            LearnedBitwidthQuantizer(init_bits=float(quantization_bits), min_bits=2.0, max_bits=32.0, symmetric=False)
            for _ in range(n_levels)]) if use_quantization else None
        bmin, bmax = _bbox_floats(bounding_box)
        self._meta = dict(res=_lib.host_f32(res), bmin=_lib.host_f32(bmin), bmax=_lib.host_f32(bmax),
                          log2_T=log2_hashmap_size)
        self.level_res = res

    def tables(self):
        return [e.weight for e in self.embeddings]

    # ---- A-CAQ ------------------------------------------------------------------------------
    def quantization_active(self):
        """hash_encoding.py:97-101: quantize unless training inside the warm-up window (the
        caller has already advanced current_step for this forward)."""
        return (self.use_quantization and self.quantizers is not None
                and not (self.training and self.current_step < self.warmup_steps))

    def level_records(self, xyz):
        """[L, 8] quantizer records for this forward. In training mode, quantizers not yet
        calibrated first calibrate on this batch's gathered corners (quantization.py:146-147):
        one gather-min/max launch over all levels."""
        qs = list(self.quantizers)
        if self.training:
            todo = [i for i, q in enumerate(qs) if not q.calibrated]
            if todo:
                join_tables(xyz.device)
                xyz = xyz.contiguous()
                st = new_stats(len(qs), xyz.device)
                meta = self._meta
                _lib.call("nerf_hash_gather_minmax", _lib.ptr(xyz, "xyz"), xyz.shape[0], meta["bmin"], meta["bmax"],
                          meta["res"], self.n_levels, meta["log2_T"], _lib.ptr_array(self.tables()),
                          _lib.ptr(st, "stats", dtype=torch.int32), _lib.stream())
                if len(todo) == len(qs):
                    calibrate_from_stats(qs, st)
                else:
                    for i in todo:
                        calibrate_from_stats([qs[i]], st[i:i + 1])
        return quant_records(qs, self.training)

    def train(self, mode=True):
        if self._packed is not None:
            self._packed["key"] = None       # repack everything on the next eval-mode forward
        return super().train(mode)

    def packed_tables(self):
        """Eval-mode int-packed tables (csrc/quant.hip): (buffer, records). No host sync: the
        records are computed on the device and a level is repacked only when its record changed
        (checked on the device) or when a table changed (torch version counters; HIP kernels that
        write tables in place bump them, see optim.RAdam)."""
        qs = list(self.quantizers)
        rec = quant_records(qs, False)
        tabs = self.tables()
        key = tuple((t.data_ptr(), t._version) for t in tabs)
        n, dev = self.n_levels, tabs[0].device
        join_tables(dev)
        st = self._packed
        if st is None or st["buf"].device != dev:
            nbytes = int(_lib.load().nerf_quant_packed_bytes(n, self.log2_hashmap_size))
            st = self._packed = dict(buf=torch.empty(nbytes, dtype=torch.uint8, device=dev),
                                     prev=torch.full((n, 8), float("nan"), device=dev),
                                     dirty=torch.empty(n, dtype=torch.int32, device=dev), key=None)
        _lib.call("nerf_quant_pack_tables", _lib.ptr_array(tabs), n, self.log2_hashmap_size, _lib.ptr(rec, "records"),
                  _lib.ptr(st["prev"], "prev_records"), int(st["key"] != key),
                  _lib.ptr(st["dirty"], "dirty", dtype=torch.int32), _lib.ptr(st["buf"], "packed", dtype=torch.uint8),
                  _lib.stream())
        st["key"] = key
        return st["buf"], rec

    def encode_into(self, xyz, feat, sp, sl, keep, row0=0):
        """Forward gather into caller-allocated feat/keep on the path this forward needs: plain,
        fake-quantized (training / STE) or int-packed (eval-mode quantizers). row0: the points land in
        rows row0 .. row0 + n of feat (level-major, point stride sp, level stride sl) and keep."""
        meta = self._meta
        P = xyz.shape[0]
        if P > 0 and ((row0 + P - 1) * sp + (self.n_levels - 1) * sl + 2 > feat.numel() or row0 + P > keep.numel()):
            raise ValueError("encode_into: rows out of the feature / keep buffers")
        fp = _lib.ptr_at(feat, sp * row0, "feat")
        kp = _lib.ptr_at(keep, row0, "keep", dtype=torch.bool)
        key, L = str(xyz.device), self.n_levels
        plain = not self.quantization_active()
        gates = _GATES.pop(key, []) if plain else []
        plan = _SPLITS.pop(key, None) if plain else None
        if not plain:
            join_tables(xyz.device)
        if self.quantization_active() and not self.training:
            buf, rec = self.packed_tables()
            _lib.call("nerf_hash_encode_fwd_packed", _lib.ptr(xyz, "xyz"), P, meta["bmin"], meta["bmax"], meta["res"],
                      self.n_levels, meta["log2_T"], _lib.ptr(buf, "packed", dtype=torch.uint8),
                      _lib.ptr(rec, "records"), fp, sp, sl, kp, _lib.stream())
            return
        rec = self.level_records(xyz) if self.quantization_active() else None
        if not gates and plan is None:
            _lib.call("nerf_hash_encode_fwd_q", _lib.ptr(xyz, "xyz"), P, meta["bmin"], meta["bmax"], meta["res"],
                      self.n_levels, meta["log2_T"], _lib.ptr_array(self.tables()),
                      _lib.ptr(rec, "records", allow_none=True), fp, sp, sl, kp, _lib.stream())
            return
        # gated (a pending parameter all-gather of the upper levels) or cut for a graph capture: the
        # levels below each cut first, then the wait / the segment boundary, then the next range.
        # Levels are independent (the keep flags come with level 0), so the features are the same bits.
        stream = torch.cuda.current_stream(xyz.device)
        cuts = [g.level for g in gates] if gates else plan[0]
        bounds = sorted({0, L} | {min(max(c, 0), L) for c in cuts})
        tabs = self.tables()
        for lb, le in zip(bounds[:-1], bounds[1:]):
            for g in [g for g in gates if g.level <= lb]:
                gates.remove(g)
                g.join(stream)
            if plan is not None and lb in plan[0] and lb > 0:
                plan[1](lb)
            res = self._level_slice(lb, le)
            _lib.call("nerf_hash_encode_fwd_q", _lib.ptr(xyz, "xyz"), P, meta["bmin"], meta["bmax"], res, le - lb,
                      meta["log2_T"], _lib.ptr_array(tabs[lb:le]), None,
                      _lib.ptr_at(feat, sp * row0 + sl * lb, "feat"), sp, sl, kp if lb == 0 else None, _lib.stream())
        for g in gates:           # cuts at or past the last level: nothing here reads them
            g.join(stream)

    def _level_slice(self, lb, le):
        """Host resolutions of levels [lb, le) (the whole-grid array for [0, L))."""
        if (lb, le) == (0, self.n_levels):
            return self._meta["res"]
        cache = self._meta.setdefault("res_slices", {})
        if (lb, le) not in cache:
            cache[(lb, le)] = _lib.host_f32(self.level_res[lb:le])
        return cache[(lb, le)]

    def binned_backward(self):
        """The binned backward exists for these tables (log2_T <= 19, plain and deterministic)."""
        lib = _lib.load()
        return all(int(lib.nerf_hash_encode_bwd_workspace_bytes(self.n_levels, self.log2_hashmap_size, 1, d)) > 0
                   for d in (0, 1))

    def encode(self, x, layout="point"):
        return HashEncodeFn.apply(x, self, layout, *self.tables())

    def forward(self, x):
        if self.training:
            self.current_step += 1
        return self.encode(x, "point")


class SHEncoder(nn.Module):
    """hash_encoding.py:110-191 (degree 4 only, the value create_nerf uses)."""

    def __init__(self, input_dim=3, degree=4):
        super().__init__()
        assert input_dim == 3
        if degree != 4:
            raise NotImplementedError("SHEncoder: the HIP kernel implements degree 4")
        self.input_dim = input_dim
        self.degree = degree
        self.out_dim = degree ** 2

    def forward(self, input, **kwargs):
        if input.requires_grad:
            raise NotImplementedError("SHEncoder: gradients w.r.t. directions are not implemented "
                                      "(the reference never back-propagates into view directions)")
        d = input.reshape(-1, 3).contiguous().float()
        out = torch.empty(d.shape[0], 16, device=d.device, dtype=torch.float32)
        _lib.call("nerf_sh4_fwd", _lib.ptr(d, "dirs"), d.shape[0], _lib.ptr(out, "sh"), _lib.stream())
        return out.reshape(*input.shape[:-1], 16)

