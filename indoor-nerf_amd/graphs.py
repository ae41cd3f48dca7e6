"""The training iteration captured in HIP graphs (torch.cuda.CUDAGraph on ROCm = hipGraph).

A PocketNeRF iteration (run_nerf.py:1007-1037, :1161-1162, :1289-1293) is ~40 kernel launches of
which many are short; launched one by one from Python the GPU idles between them (the host spends
~0.2 ms per step in autograd and ctypes). GraphedTrainStep captures the iteration once — forward,
losses, backward and the RAdam update: one graph on one process, two (graph 1 = forward + backward,
graph 2 = the update) when a DP gradient hook runs between them — and replays it.

What changes from step to step without changing the launch structure lives in device memory and is
written before each replay (StepScalars): the Philox (seed, offset) of the stratified and
importance sampling kernels, the TV cuboid corners (drawn on the host with the same generator as
the eager path), and RAdam's per-step scalars (step count, N_sma, step size, lr decay). Those are
computed by the same host code as the eager path ("fillers" registered while capturing), written
into a ring of mapped host memory and fetched by the replay's own first launch.

The launch structure itself depends on host state that changes rarely: the TV term switches off
after iteration 1000 (run_nerf.py:1036-1037) and A-CAQ quantization switches on after the
embedder's warm-up; GraphedTrainStep re-captures when that key changes.
"""
import time
from contextlib import contextmanager

import torch

_ACTIVE = None


def active():
    """The StepScalars of the capture in progress, or None (eager execution)."""
    return _ACTIVE


@contextmanager
def capturing(scalars):
    global _ACTIVE
    prev, _ACTIVE = _ACTIVE, scalars
    try:
        yield scalars
    finally:
        _ACTIVE = prev


class StepScalars:
    """Device-resident per-step scalars of a captured step (int64 and float32 slots).

    The host writes each replay's values into the next slot of a ring of mapped host memory
    (nerf_host_ring_alloc); the captured step's first launch (nerf_scalars_fetch) copies that slot
    into the device slots, picking it with a device counter the launch advances, and publishes how
    many replays have fetched into the ring, so the host rewrites a slot only after its last reader
    without an event. Nothing is queued between two replays; the pinned copy + event it replaces
    cost 8 us per step (profiles/r04zf_ab_upload.jsonl)."""

    def __init__(self, device, n_i64=1024, n_f32=1024, ring=4):
        import ctypes
        import numpy as np
        from . import _lib
        if n_f32 % 2:
            raise ValueError("StepScalars: n_f32 must be even (the slot's last 8 bytes hold its replay tag)")
        self.n_i64, self.nb = n_i64, 8 * n_i64 + 4 * n_f32
        # [int64 slots | float32 slots] on the device; the ring holds `ring` copies of that layout
        self.dev = torch.zeros(self.nb, dtype=torch.uint8, device=device)
        self.dev_i = self.dev[:8 * n_i64].view(torch.int64)
        self.dev_f = self.dev[8 * n_i64:].view(torch.float32)
        self.ctl = torch.zeros(4, dtype=torch.int64, device=device)   # replays, words A, start B, words B
        h = ctypes.c_void_p()
        self.done_off = ring * self.nb           # int64 after the slots: fetches completed (device-written)
        _lib.call("nerf_host_ring_alloc", self.done_off + 64, ctypes.byref(h))
        self._ring = h.value
        buf = np.ctypeslib.as_array((ctypes.c_uint8 * (self.done_off + 64)).from_address(self._ring))
        self.pinned = [(buf[k * self.nb:k * self.nb + 8 * n_i64].view(np.int64),
                        buf[k * self.nb + 8 * n_i64:(k + 1) * self.nb].view(np.float32)) for k in range(ring)]
        self.done = buf[self.done_off:self.done_off + 8].view(np.int64)
        self.done[0] = 0
        # the fetch's sticky error word: replay index + 1 of a fetch whose slot carried another tag
        self.err = buf[self.done_off + 8:self.done_off + 16].view(np.int64)
        self.err[0] = 0
        # the last 8 bytes of each slot: the index of the replay the slot was written for
        self.tags = [buf[(k + 1) * self.nb - 8:(k + 1) * self.nb].view(np.int64) for k in range(ring)]
        self.issued = 0    # uploads so far = index of the replay the next upload prepares
        self.step = 0      # the global step of the replay being prepared (fillers may read it)
        self.ni = self.nf = 0
        self.fillers = []

    def close(self):
        """Free the ring now (outside any capture): after a synchronize no replay still reads it."""
        ring, self._ring = getattr(self, "_ring", None), None
        if ring:
            from . import _lib
            torch.cuda.synchronize(self.dev.device)
            _lib.call("nerf_host_ring_free", ring)

    def __del__(self):
        # fallback only (GraphedTrainStep closes the ring it replaces)
        try:
            self.close()
        except Exception:      # interpreter shutdown: the process's mappings go with it
            pass

    def alloc_i64(self, n):
        if self.ni + n > self.dev_i.numel():
            raise RuntimeError("StepScalars: int64 slots exhausted")
        off, self.ni = self.ni, self.ni + n
        return off, self.dev_i.data_ptr() + 8 * off

    def alloc_f32(self, n):
        if self.nf + n > self.dev_f.numel() - 2:     # the last two words: the slot's replay tag
            raise RuntimeError("StepScalars: float32 slots exhausted")
        off, self.nf = self.nf, self.nf + n
        return off, self.dev_f.data_ptr() + 4 * off

    def add_filler(self, fn):
        """fn(host_int64_numpy, host_float32_numpy) writes this step's values into its slots."""
        self.fillers.append(fn)

    def capture_fetch(self):
        """The fetch launch: first in the captured step, on the capture stream."""
        from . import _lib
        _lib.call("nerf_scalars_fetch", self._ring, self.nb, len(self.pinned), self.done_off,
                  _lib.ptr(self.ctl, "ctl", torch.int64), self.dev.data_ptr(), _lib.stream())

    def seal(self):
        """After the capture: the words the fetch copies (the slots the capture allocated)."""
        self.ctl.copy_(torch.tensor([0, 2 * self.ni, 2 * self.n_i64, self.nf], dtype=torch.int64))
        torch.cuda.synchronize(self.dev.device)
        self.done[0] = 0
        self.err[0] = 0
        self.issued = 0

    def check(self):
        """Raise if a replay fetched a slot written for another replay (the fetch kernel's tag check)."""
        e = int(self.err[0])
        if e:
            raise RuntimeError(f"StepScalars: replay {e - 1} fetched a ring slot written for another replay: the "
                               "uploads and the replays of the captured step have parted (a replay without its "
                               "upload(); each upload() must be followed by exactly one replay); re-seal() before "
                               "replaying again")

    def upload(self):
        """Run every filler into the ring slot the next replay fetches (call once before each replay)."""
        self.check()
        n, R = self.issued, len(self.pinned)
        if int(self.done[0]) < n - R + 1:        # replay n - R has not fetched this slot yet
            deadline = time.monotonic() + 60.0
            while int(self.done[0]) < n - R + 1:
                if time.monotonic() > deadline:
                    raise RuntimeError(f"StepScalars: replay {n - R} never fetched its scalars (each upload() "
                                       "must be followed by one replay of the captured step)")
                time.sleep(0)
        hi, hf = self.pinned[n % R]
        for fn in self.fillers:
            fn(hi, hf)
        self.tags[n % R][0] = n
        self.issued = n + 1


# "thread_local": only the capturing thread's unsafe calls (allocations, synchronisations) invalidate the
# capture. With the nccl (RCCL) process group a watchdog thread queries its collectives' events while
# a step is captured; the process-wide "global" mode would count those queries against the capture.
CAPTURE_MODE = "thread_local"


class _Segments:
    """Capture of one graph as a list of graphs cut at chosen points (split()): each segment is its own
    CUDAGraph on the same memory pool and capture stream, replayed in order with host work (event
    waits) between them. Used for graph 1 of a step whose hash forward is gated by a pending
    parameter all-gather (dist.ShardedOptimizer.gather_params): the segment boundary sits where the
    eager forward would wait (hashgrid.split_next_forward)."""

    def __init__(self, pool, stream):
        self.pool, self.stream, self.graphs, self.cuts = pool, stream, [], []

    def _begin(self):
        g = torch.cuda.CUDAGraph()
        g.capture_begin(self.pool, capture_error_mode=CAPTURE_MODE)
        self.graphs.append(g)

    def split(self, level):
        self.graphs[-1].capture_end()
        self.cuts.append(int(level))
        self._begin()

    def __enter__(self):
        torch.cuda.synchronize()
        self._ctx = torch.cuda.stream(self.stream)
        self._ctx.__enter__()
        self._begin()
        return self

    def __exit__(self, *exc):
        try:
            self.graphs[-1].capture_end()
        finally:
            self._ctx.__exit__(*exc)
        return False


class SegmentedGraph:
    """Graph 1 of a step as its captured segments (_Segments); replay() replays them in order on the
    current stream (GraphedTrainStep._replay_forward joins pending table gates between them)."""

    def __init__(self, graphs, cuts):
        self.segments, self.cuts = list(graphs), list(cuts)

    def replay(self):
        for g in self.segments:
            g.replay()

    def __len__(self):
        return len(self.segments)


def gate_levels(post_hook):
    """The table levels at which a post hook (dist.ShardedOptimizer.gather_params) leaves gates for the
    next forward; [] for any other hook."""
    fn = getattr(getattr(post_hook, "__self__", None), "gate_levels", None)
    return list(fn()) if callable(fn) else []


class GraphedTrainStep:
    """train_step (model.py) as captured graphs: one (forward + backward + RAdam) without a grad
    hook; with one, two graphs (forward + backward, RAdam) and the eager grad hook between them and
    the post hook after the second (the DP collectives stay outside the graphs). Call it like
    train_step(...) with the same arguments every iteration; it runs `warmup` eager iterations
    before the first capture (allocations, optimizer state, quantizer calibration)."""

    def __init__(self, batch_rays, target_s, render_kwargs_train, optimizer, args, H=0, W=0, K=None,
                 grad_hook=None, loss_scale_sparsity=1.0, tv_generator=None, zero_grad=None, warmup=2,
                 post_hook=None, sampler=None):
        self.rays, self.target = batch_rays, target_s
        # sampler (rays.RaySampler): every iteration draws a new batch into batch_rays / target_s first
        # (train()'s no_batching path, run_nerf.py:975-1004), inside the captured step
        self.sampler = sampler
        self.kw, self.opt, self.args = render_kwargs_train, optimizer, args
        self.H, self.W, self.K = H, W, K
        if zero_grad is None:
            # gradients must live at fixed addresses across replays: one flat arena, zeroed in place
            from .dist import GradArena
            arena = GradArena([p for g in optimizer.param_groups for p in g["params"]], defer_tables=True)
            zero_grad = arena.zero_
        self.hook, self.scale_sp, self.tv_gen, self.zero_grad = grad_hook, loss_scale_sparsity, tv_generator, zero_grad
        self.post_hook = post_hook
        self.warmup = warmup
        self.eager_steps = 0
        self.key = None
        self.graphs = None
        self.captures = 0

    def _n_forwards(self):
        return 2 if self.kw.get("network_fine") is not None else 1     # coarse + fine embedder calls

    def _structure_key(self, global_step):
        """Host state that changes the launch sequence of a step: the TV term (on until iteration
        1000), per embedder call of the step whether A-CAQ quantization is active, and whether the
        structural priors are on (with the weights baked into their launch)."""
        from .model import DEFAULTS
        get = lambda k: getattr(self.args, k, DEFAULTS.get(k))  # noqa: E731
        tv_w = get("tv_loss_weight")
        emb = self.kw["embed_fn"]
        quant = ()
        if getattr(emb, "use_quantization", False):
            quant = tuple(emb.current_step + k + 1 >= emb.warmup_steps for k in range(self._n_forwards()))
        priors = ()
        if self._priors_active(global_step):
            priors = (get("depth_prior_weight"), get("planarity_weight"), get("manhattan_weight"),
                      get("normal_consistency_weight"), get("structural_loss_start_iter"),
                      get("structural_loss_ramp_iters"))
        crop = self.sampler.crop_key(global_step) if self.sampler is not None else None
        return (tv_w > 0, quant, priors, crop)

    def _capture(self, global_step):
        from . import _lib, hashgrid
        from .model import forward_backward, holds_owner, optimizer_update
        if _lib.timing_enabled():
            raise RuntimeError("GraphedTrainStep: kernel timing is on; torch on ROCm cannot capture timing "
                               "events (time eager_step() instead)")
        dev = self.target.device
        hashgrid.join_tables(dev)          # the previous step's parameter all-gather, if still pending
        sc = StepScalars(dev)
        emb = self.kw["embed_fn"]
        step0 = emb.current_step           # the captured (not executed) forwards must not count
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        pool = torch.cuda.graph_pool_handle()
        # without a gradient hook between them (one process) the update joins the first graph: one
        # graph launch per iteration (a second launch left the GPU idle ~9 us between them)
        single = self.hook is None
        g2 = None if single else torch.cuda.CUDAGraph()
        # with an overlapping DP hook the owner pass stays out of graph 1: the hook runs it by level range
        # beside the bucket reduce-scatters (dist.ShardedOptimizer(overlap=True))
        with torch.cuda.stream(side), hashgrid.hold_owner(dev, holds_owner(self.hook)), \
                hashgrid.fused_table_step(dev, self.opt, emb.tables(), enabled=self.hook is None):
            with capturing(sc):
                # with a gated parameter all-gather behind the post hook, graph 1 is cut into segments
                # where the hash forward would wait for it (replayed with the waits between them)
                seg = _Segments(pool, side)
                try:
                    with seg:
                        hashgrid.split_next_forward(dev, gate_levels(self.post_hook), seg.split)
                        sc.capture_fetch()
                        if self.sampler is not None:
                            self.sampler.fill(global_step, self.rays[0], self.rays[1], self.target)
                        out = forward_backward(self.rays, self.target, self.kw, self.opt, self.args, global_step,
                                               H=self.H, W=self.W, K=self.K, loss_scale_sparsity=self.scale_sp,
                                               tv_generator=self.tv_gen, zero_grad=self.zero_grad, schedule=False)
                        if single:
                            optimizer_update(self.opt)
                finally:
                    hashgrid.split_next_forward(dev, None, None)
                if not single:
                    with torch.cuda.graph(g2, pool=pool, stream=side, capture_error_mode=CAPTURE_MODE):
                        optimizer_update(self.opt)
        torch.cuda.current_stream(dev).wait_stream(side)
        sc.seal()
        emb.current_step = step0
        old = getattr(self, "scalars", None)
        self.graphs = (SegmentedGraph(seg.graphs, seg.cuts), g2)
        self.cuts = seg.cuts
        self.out = out
        self.scalars = sc
        if old is not None:
            old.close()     # the replaced graph's ring (its graph is gone: no replay can read it)
        self.params = [p for g in self.opt.param_groups for p in g["params"] if p.grad is not None]
        self.captures += 1

    def eager_step(self, global_step):
        """The same iteration launched eagerly (same arguments, host state and gradient arena),
        e.g. to time its kernels with HIP events, which cannot be captured."""
        from .model import train_step
        if self.sampler is not None:
            self.sampler.fill(global_step, self.rays[0], self.rays[1], self.target)
        return train_step(self.rays, self.target, self.kw, self.opt, self.args, global_step, H=self.H, W=self.W,
                          K=self.K, grad_hook=self.hook, loss_scale_sparsity=self.scale_sp,
                          tv_generator=self.tv_gen, zero_grad=self.zero_grad, post_hook=self.post_hook)

    def _replay_forward(self):
        """Graph 1's segments in order; before each, the pending table gates (the last post hook's
        side-stream all-gathers) of the levels it reads: segment k reads levels below the next cut,
        the last one everything."""
        from . import hashgrid
        dev = self.target.device
        segs, gates = self.graphs[0].segments, hashgrid.take_gates(self.target.device)
        ends = list(self.cuts) + [float("inf")]
        stream = torch.cuda.current_stream(dev)
        for k, g in enumerate(segs):
            for gate in [x for x in gates if x.level < ends[k]]:
                gates.remove(gate)
                gate.join(stream)
            g.replay()

    def check(self):
        """A host sync point's check of the captured step's scalar ring (StepScalars.check): upload()
        checks before every replay, so a replay that fetched another replay's slot is otherwise seen
        only at the next upload — never after a run's final replay. Call it where the host waits for
        the device anyway (end of training, checkpoint save; bench.py after its timed region). When it
        raises, the flagged replay (and possibly the one after it) has already trained on that slot."""
        sc = getattr(self, "scalars", None)
        if sc is not None:
            torch.cuda.synchronize(self.target.device)
            sc.check()

    def _priors_active(self, global_step):
        from .model import DEFAULTS
        get = lambda k: getattr(self.args, k, DEFAULTS.get(k))  # noqa: E731
        return bool(get("use_structural_priors")) and global_step >= get("structural_loss_start_iter")

    def __call__(self, global_step):
        from .model import acaq_update, fused_priors_eligible, lr_schedule
        if self._priors_active(global_step) and not fused_priors_eligible(self.args, self.rays[0].shape[0]):
            # the eager priors path (args.fused_priors = False, no normals head, or more rays than the
            # device path takes) branches on host counts and draws host permutations: not capturable
            self.graphs, self.key = None, None
            return self.eager_step(global_step)
        key = self._structure_key(global_step)
        if key != self.key:                # new launch structure: eager steps first (allocations,
            self.key = key                 # quantizer calibration), then a fresh capture
            self.graphs = None
            self.eager_steps = 0
        if self.eager_steps < self.warmup:
            self.eager_steps += 1
            return self.eager_step(global_step)
        if self.graphs is None:
            self._capture(global_step)
        self.scalars.step = global_step
        try:
            self.scalars.upload()
            self._replay_forward()
        except BaseException:
            # an upload without its replay (or the reverse) would pair every later replay with another
            # step's slot: re-synchronise the host's and the device's replay counts
            self.scalars.seal()
            raise
        emb = self.kw["embed_fn"]
        if emb.training:
            emb.current_step += self._n_forwards()
        if self.hook is not None:
            self.hook()
        if self.graphs[1] is not None:
            self.graphs[1].replay()
        for p in self.params:              # the replayed RAdam wrote the parameters in place
            torch.autograd.graph.increment_version(p)
        if self.post_hook is not None:
            self.post_hook()
        loss, img_loss, psnr = self.out
        acaq_update(global_step, img_loss, self.kw, self.args)
        lr_schedule(self.opt, self.args, global_step)
        return loss.detach(), psnr.detach()
