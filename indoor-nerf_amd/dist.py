"""Data parallelism for the training step: one process per GPU, rays sharded, parameters replicated,
gradients reduced with ONE all-reduce per step (RCCL over xGMI via torch.distributed 'nccl';
'gloo' on CPU for tests).

The reference has no distributed code; this is the build's DP layer (§8(e)).
All parameter gradients live in one flat GradArena buffer (p.grad are views into it), so the
fused backward kernels accumulate straight into the buffer that is all-reduced, zeroing is one
memset, and the collective is a single 67 MB bucket (16 x 2^19 x 2 table entries + 2 x 9,344
MLP weights) — large enough to run at per-link xGMI bandwidth with RCCL's multi-channel rings.
"""
import os

import torch
import torch.distributed as dist

from . import _lib


def env_rank_world():
    return int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(os.environ.get("LOCAL_RANK", 0))


def init_process_group(backend=None, force=False):
    """Init from torchrun's env (RANK/WORLD_SIZE/MASTER_*); no-op for a single process unless `force`
    (a one-rank process group: the multi-rank code path over RCCL on one GPU, bench.py NERF_DIST_FORCE)."""
    rank, world, local = env_rank_world()
    if (world == 1 and not force) or (dist.is_available() and dist.is_initialized()):
        return rank, world, local
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29517")
    if backend is None:
        # NERF_DIST_BACKEND=gloo: rehearse the multi-rank path on one GPU (ranks share cuda:0)
        backend = os.environ.get("NERF_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl":   # ranks beyond the visible GPUs (one-GPU rehearsals) wrap around
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world, local


def shard(t, rank, world, dim=0):
    """Contiguous equal shard `rank` of `world` along dim (strong scaling of one global batch)."""
    n = t.shape[dim]
    if n % world:
        raise ValueError(f"shard: size {n} is not divisible by world size {world}")
    step = n // world
    return t.narrow(dim, rank * step, step)


_ALIGN = 64      # elements: every rank's shard starts on a 256-B boundary (vectorised RAdam)


class GradArena:
    """One flat fp32 buffer holding the .grad of every parameter (views), in parameter order, each
    starting on a 256-B boundary (_ALIGN elements: the fused RAdam's float4 path needs 16-B aligned
    tensors, and a 3-element bias would otherwise misalign every gradient after it). pad_to: round
    the buffer up to a multiple of this many elements (the sharded optimizer needs world x _ALIGN)
    — the gaps and the tail are never a gradient and stay zero."""

    def __init__(self, params, pad_to=1, defer_tables=False, bucket_starts=()):
        # quantizer scalars (soft_bits, range_scale, v_max) never receive a gradient in the
        # reference (their uses are detached): they keep grad None, so the optimizer skips them
        self.params = [p for p in params if p.requires_grad and not getattr(p, "_nerf_no_grad", False)]
        # buckets: contiguous element ranges, each a multiple of pad_to long, split before the
        # parameters in bucket_starts (dist.ShardedOptimizer reduces them one by one)
        starts = {id(p) for p in bucket_starts}
        self.offsets, off, b0, self.buckets = [], 0, 0, []
        for p in self.params:
            if id(p) in starts and off > b0:
                off = -(-off // pad_to) * pad_to
                self.buckets.append((b0, off))
                b0 = off
            self.offsets.append(off)
            off += -(-p.numel() // _ALIGN) * _ALIGN
        self.numel = off
        total = -(-self.numel // pad_to) * pad_to
        self.buckets.append((b0, total))
        dev = self.params[0].device
        self.flat = torch.zeros(total, device=dev, dtype=torch.float32)
        self.views = [self.flat[o:o + p.numel()].view_as(p) for p, o in zip(self.params, self.offsets)]
        # defer_tables: the hash tables' gradients (a trailing run of the arena) are not memset by
        # zero_(); the iteration's owner pass overwrites them (hashgrid.defer_zero)
        self.deferred, self.zero_end = [], self.flat.numel()
        if defer_tables:
            tail = len(self.params)
            while tail > 0 and getattr(self.params[tail - 1], "_nerf_owner_grad", False):
                tail -= 1
            if tail < len(self.params):
                self.deferred = self.views[tail:]
                self.zero_end = self.offsets[tail]
        self.attach()

    def attach(self):
        for p, v in zip(self.params, self.views):
            p.grad = v

    def zero_(self):
        if self.deferred and _lib.zero_deferral_active():
            # inside a training iteration (model.forward_backward): the tables' zero by the iteration's
            # owner pass (it stores every row), the dense rest by render()'s first launch
            # (_lib.defer_fill_zero) or before the backward at the latest
            from .hashgrid import defer_zero
            _lib.defer_fill_zero(self.flat[:self.zero_end])
            defer_zero(self.deferred)
        else:
            # anywhere else the gradients read zero when zero_() returns
            if self.deferred:
                from .hashgrid import forget_deferred
                forget_deferred(self.deferred)
            _lib.flush_zero_fills([self.flat])
            self.flat.zero_()
        self.attach()

    def allreduce_mean(self, group=None):
        """Mean of the gradients over the process group (a one-rank group runs the collective too: the
        RCCL rehearsal of bench.py NERF_DIST_FORCE; no group: nothing to do)."""
        if not (dist.is_available() and dist.is_initialized()):
            return
        world = dist.get_world_size(group)
        h = _staged(self.flat)
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
        h.mul_(1.0 / world)
        if h is not self.flat:
            self.flat.copy_(h)


def _world():
    return dist.get_world_size() if (dist.is_available() and dist.is_initialized()) else 1


def _staged(t):
    """gloo collectives run on host memory: stage a device tensor through the CPU (rehearsals and
    tests only; 'nccl' = RCCL works on the device tensor itself)."""
    return t.cpu() if (t.is_cuda and dist.get_backend() == "gloo") else t


def _reduce_scatter(out, inp, group=None):
    """dist.reduce_scatter_tensor (sum) for every backend: 'nccl' (RCCL) on the device tensors, gloo
    (tests, one-GPU rehearsals) on host copies — the same call and the same shard indexing."""
    if dist.get_backend(group) == "gloo" and (out.is_cuda or inp.is_cuda):
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.reduce_scatter_tensor(h, inp.cpu(), op=dist.ReduceOp.SUM, group=group)
        out.copy_(h)
    else:
        dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=group)


def _all_gather(out, inp, group=None):
    """dist.all_gather_into_tensor for every backend (gloo on host copies); inp may be a view of out."""
    if dist.get_backend(group) == "gloo" and (out.is_cuda or inp.is_cuda):
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(h, inp.cpu(), group=group)
        out.copy_(h)
    else:
        dist.all_gather_into_tensor(out, inp, group=group)


def _all_gather_begin(out, inp, group, stream):
    """Start dist.all_gather_into_tensor on `stream` (the caller's side stream) and return
    (event, finish): `event` completes with the gathered `out` once finish() (None on device backends)
    has run on the host. RCCL: the collective is enqueued on the stream, the event recorded behind it.
    gloo (one-GPU rehearsals, tests): the shard goes to the host, the collective runs asynchronously in
    gloo's thread, and finish() waits for it and copies the result back on the stream — so the GPU
    runs the caller's next launches while the collective is in flight, as it would beside RCCL."""
    ev = torch.cuda.Event()
    if dist.get_backend(group) == "gloo" and (out.is_cuda or inp.is_cuda):
        with torch.cuda.stream(stream):
            h_in = inp.cpu()
        h = torch.empty(out.shape, dtype=out.dtype)
        work = dist.all_gather_into_tensor(h, h_in, group=group, async_op=True)

        def finish(keep=(h_in, h)):   # the collective's host buffers live until it has completed
            work.wait()
            with torch.cuda.stream(stream):
                out.copy_(h)
                ev.record(stream)
        return ev, finish
    with torch.cuda.stream(stream):
        dist.all_gather_into_tensor(out, inp, group=group)
        ev.record(stream)
    return ev, None


def _capturing(t):
    return t.is_cuda and torch.cuda.is_current_stream_capturing()


def allreduce_calibration_stats(stats):
    """A-CAQ calibration statistics [n, 2] int32 = order-preserving uint32 images of (min, max)
    (quantization.new_stats): the elementwise MIN / MAX over ranks, in place, so that every rank
    calibrates its quantizers on the statistics of the global batch and the replicas stay equal
    (quantization.py:97-119 run on one process's batch). No-op for a single process."""
    if _world() == 1 or _capturing(stats):
        return stats
    u = _staged(stats).to(torch.int64) & 0xFFFFFFFF          # the uint32 order, exactly, in int64
    lo, hi = u[:, 0].contiguous(), u[:, 1].contiguous()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    out = torch.stack([lo, hi], 1)
    out = torch.where(out >= 1 << 31, out - (1 << 32), out).to(torch.int32)
    stats.copy_(out.to(stats.device))
    return stats


def allreduce_mean_(t):
    """In-place mean over ranks of a small device tensor (the A-CAQ controller's img_loss)."""
    if _world() == 1 or _capturing(t):
        return t
    s = _staged(t)
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    s.mul_(1.0 / _world())
    if s is not t:
        t.copy_(s)
    return t


def shard_ranges(offsets, sizes, lo, hi):
    """Per parameter (flat offset, size): the part of [lo, hi) it holds, as a local element range
    (a, b), or None. The ranges of all ranks tile every parameter exactly once."""
    out = []
    for off, n in zip(offsets, sizes):
        a, b = max(lo, off), min(hi, off + n)
        out.append((a - off, b - off) if b > a else None)
    return out


class ShardedOptimizer:
    """Optimizer-state sharding for data parallelism (ZeRO stage 1).

    The parameters become views of one flat fp32 buffer laid out like the GradArena, padded to a
    multiple of world x _ALIGN, and in each of the arena's buckets (one, or the split made with
    GradArena(bucket_starts=...)) rank r owns the contiguous r-th 1/G of the bucket.
    Per iteration, instead of an all-reduce of the gradients and a dense RAdam pass over all 16.8 M
    elements on every rank:
      reduce_grads()   reduce-scatter (sum) of the gradient buffer into this rank's shard
      optimizer.step() RAdam on the shard only (the HIP kernel on sub-ranges of the tensors, reading
                       the summed gradient x 1/G: the mean without a pass of its own)
      gather_params()  all-gather of the updated parameter shards into every replica
    The collective bytes equal one all-reduce; the dense optimizer traffic drops by G. Elementwise
    RAdam on a shard is bit-identical to RAdam on the whole tensor (tests/test_gpu_dist.py).
    Exp_avg / exp_avg_sq are valid on the rank's own shard only; consolidate_state() assembles
    them for a checkpoint (model.save_checkpoint).

    overlap (with buckets): the step's hash-table owner pass is held back (hashgrid.hold_owner, set
    by model.train_step / graphs.GraphedTrainStep for this hook) and reduce_grads() runs it bucket by
    bucket — the levels of bucket 0, then those of bucket 1, ... — starting each bucket's
    reduce-scatter on a side stream as soon as its levels are summed, so the collective of the first
    buckets runs under the owner pass of the later ones.
    overlap_gather (default: overlap): gather_params() all-gathers the first bucket in stream order and
    every later bucket that holds only hash-table levels on the side stream, registering a gate
    (hashgrid.gate_tables) at the bucket's first level: the next iteration's hash forward launches
    the levels below it while the collective runs and waits only before the gated levels; any other
    reader of the tables (TV, A-CAQ calibration, the packed eval tables, reduce_grads,
    consolidate_state, wait_params) joins the gates first. Parameters of a gated bucket read through
    another path after gather_params() (e.g. a direct copy of the tensors) need wait_params() first."""

    def __init__(self, optimizer, arena, group=None, overlap=False, overlap_gather=None):
        self.opt, self.arena, self.group = optimizer, arena, group
        # grouped: a process group exists — its collectives run even at one rank (the one-GPU RCCL
        # rehearsal of the N > 1 path, bench.py NERF_DIST_FORCE=1); without one every hook is local
        self.grouped = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if self.grouped else 1
        self.rank = dist.get_rank(group) if self.grouped else 0
        n_flat = arena.flat.numel()
        if any((e - s) % (self.world * _ALIGN) for s, e in arena.buckets):
            raise ValueError("ShardedOptimizer: build the GradArena with pad_to=world*64")
        dev = arena.flat.device
        # parameters as views of one flat buffer (same layout as the gradients)
        self.pflat = torch.zeros(n_flat, device=dev, dtype=torch.float32)
        with torch.no_grad():
            for p, off in zip(arena.params, arena.offsets):
                view = self.pflat[off:off + p.numel()].view_as(p)
                view.copy_(p.data)
                p.data = view
        arena.attach()
        # per bucket (s, e): this rank owns [own_lo, own_hi), stored at gshard[g0, g0 + n/G)
        self.pieces, g0 = [], 0
        for s, e in arena.buckets:
            n = (e - s) // self.world
            self.pieces.append((s + self.rank * n, s + (self.rank + 1) * n, g0))
            g0 += n
        self.count = g0
        self.gshard = torch.zeros(self.count, device=dev, dtype=torch.float32)
        shard, self.ranges = {}, []
        for p, off in zip(arena.params, arena.offsets):
            r = None
            for lo, hi, gp in self.pieces:
                a, b = max(lo, off), min(hi, off + p.numel())
                if b > a:
                    r = (a - off, b - off)
                    shard[p] = (a - off, b - off, self.gshard[gp + a - lo:gp + b - lo])
            self.ranges.append(r)
        # the reduce-scatter leaves the SUM of the ranks' gradients; the RAdam launch reads it x 1/G
        # (nerf_radam_segment.grad_scale), so no pass over the shard forms the mean first
        optimizer.set_shard(shard if self.grouped else None, grad_scale=1.0 / self.world)
        self.overlap = bool(overlap) and len(arena.buckets) > 1 and dev.type == "cuda"
        self.side = torch.cuda.Stream(device=dev) if self.overlap else None
        self._levels = None
        og = self.overlap if overlap_gather is None else (bool(overlap_gather) and self.overlap)
        self._gates = self._gate_levels() if og else {}

    def _gate_levels(self):
        """{bucket index: first table level} for the buckets after the first that hold only hash-table
        levels (HashEmbedder tags each table with ._nerf_level), in ascending level order; the
        first bucket that breaks this ends the list (it and the later ones are gathered in order)."""
        out, last = {}, -1
        for k, (s, e) in enumerate(self.arena.buckets):
            if k == 0:
                continue
            held = [p for p, off in zip(self.arena.params, self.arena.offsets) if s <= off < e]
            lv = [getattr(p, "_nerf_level", None) for p in held]
            if not held or None in lv or min(lv) <= last:
                break
            out[k], last = min(lv), max(lv)
        return out

    def gate_levels(self):
        """The table levels at which gather_params() leaves a gate for the next forward (ascending)."""
        return sorted(self._gates.values())

    def wait_params(self):
        """Make the current stream wait for the side-stream all-gathers of the last gather_params()."""
        from .hashgrid import join_tables
        join_tables(self.pflat.device)

    def _level_ranges(self, held):
        """Per bucket, the level range [lb, le) of the held owner pass whose tables lie in it."""
        if self._levels is None or self._levels[0] is not held:
            base = self.arena.flat.data_ptr()
            bucket_of = []
            for g in held.grads:
                off = (g.data_ptr() - base) // 4
                bucket_of.append(next(k for k, (s, e) in enumerate(self.arena.buckets) if s <= off < e))
            if bucket_of != sorted(bucket_of):
                raise RuntimeError("ShardedOptimizer(overlap): table levels must lie in bucket order")
            ranges = [(bucket_of.index(k) if k in bucket_of else 0, len(bucket_of) - bucket_of[::-1].index(k)
                       if k in bucket_of else 0) for k in range(len(self.arena.buckets))]
            self._levels = (held, ranges)
        return self._levels[1]

    def reduce_grads(self):
        """Reduce-scatter of each gradient bucket: this rank's shard of the summed gradient (RAdam
        reads it x 1/G). The same collective on every backend (RCCL on the device buffers; gloo on
        host copies of them). With overlap and a held owner pass: every bucket's levels are summed and recorded first, then each
        bucket's reduce-scatter waits on the side stream for its own levels only."""
        from .hashgrid import pending_bins
        self.wait_params()      # the last all-gather wrote the parameter shards the update reads
        held = pending_bins(self.arena.flat.device).take_held() if self.overlap else None
        if not self.grouped:
            if held is not None:
                held.run(0, held.L)
            return
        flat, events = self.arena.flat, []
        if held is not None:
            for lb, le in self._level_ranges(held):
                held.run(lb, le)
                ev = torch.cuda.Event()
                ev.record()
                events.append(ev)
        for k, ((s, e), (lo, hi, g0)) in enumerate(zip(self.arena.buckets, self.pieces)):
            out = self.gshard[g0:g0 + hi - lo]
            if events:
                self.side.wait_event(events[k])
                with torch.cuda.stream(self.side):
                    _reduce_scatter(out, flat[s:e], self.group)
            else:
                _reduce_scatter(out, flat[s:e], self.group)
        if events:
            torch.cuda.current_stream(flat.device).wait_stream(self.side)

    def gather_params(self):
        """All-gather of each bucket's updated parameter shards (in place: the shard is a view of the
        output); with overlap_gather the table-only buckets after the first on the side stream,
        behind gates the next forward joins (class docstring)."""
        if not self.grouped:
            return
        from .hashgrid import TableGate, gate_tables
        dev = self.pflat.device
        self.wait_params()
        gates = []
        for k, ((s, e), (lo, hi, _)) in enumerate(zip(self.arena.buckets, self.pieces)):
            if k not in self._gates:
                _all_gather(self.pflat[s:e], self.pflat[lo:hi], self.group)
                continue
            if not gates:
                self.side.wait_stream(torch.cuda.current_stream(dev))   # the update wrote the shards
            ev, finish = _all_gather_begin(self.pflat[s:e], self.pflat[lo:hi], self.group, self.side)
            gates.append(TableGate(self._gates[k], ev, finish))
        gate_tables(dev, gates)
        for p in self.arena.params:       # the collective wrote the parameters in place
            torch.autograd.graph.increment_version(p)

    def consolidate_state(self):
        """COLLECTIVE: every rank must call it (model.save_checkpoint(sharded=...) does so on every
        rank and writes on one). Every rank's exp_avg / exp_avg_sq shards are summed into full
        tensors on every rank (each element is owned by exactly one rank; the others contribute
        zeros) with ONE all-reduce over both moments of every parameter laid out like the gradient
        arena, so the call count cannot differ between ranks whatever state each rank holds."""
        if not self.grouped:
            return
        self.wait_params()
        keys = ("exp_avg", "exp_avg_sq")
        n = self.arena.flat.numel()
        buf = torch.zeros(len(keys) * n, device=self.pflat.device, dtype=torch.float32)
        for p, off, r in zip(self.arena.params, self.arena.offsets, self.ranges):
            st = self.opt.state.get(p)
            if not st or r is None:
                continue
            for k, key in enumerate(keys):
                buf[k * n + off + r[0]:k * n + off + r[1]] = st[key].reshape(-1)[r[0]:r[1]]
        h = _staged(buf)
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=self.group)
        if h is not buf:
            buf.copy_(h)
        for p, off in zip(self.arena.params, self.arena.offsets):
            st = self.opt.state.get(p)
            if not st:
                continue
            for k, key in enumerate(keys):
                st[key].view(-1).copy_(buf[k * n + off:k * n + off + p.numel()])


def broadcast_params(params, src=0):
    """Make every rank start from rank `src`'s parameters."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    for p in params:
        h = _staged(p.data)
        dist.broadcast(h, src=src)
        if h is not p.data:
            p.data.copy_(h)
