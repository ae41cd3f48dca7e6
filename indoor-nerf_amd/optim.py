"""RAdam with a fused HIP step (PocketNeRF/radam.py:5-94).

Same constructor, param groups, state keys ('step', 'exp_avg', 'exp_avg_sq') and the 10-slot
step-size cache per group. The scalar algebra (N_sma, step_size) runs on the host in Python
doubles exactly as the reference does; the elementwise update of every parameter of every group
runs in ONE kernel launch (csrc/optim.hip) instead of ~8 eager ops per tensor.
"""
import ctypes
import math

import torch
from torch.optim.optimizer import Optimizer

from . import _lib

_MAX_SEGS = 32


class RAdam(Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, degenerated_to_sgd=False):
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameters: {betas}")
        self.degenerated_to_sgd = degenerated_to_sgd
        if isinstance(params, (list, tuple)) and len(params) > 0 and isinstance(params[0], dict):
            for param in params:
                if "betas" in param and (param["betas"][0] != betas[0] or param["betas"][1] != betas[1]):
                    param["buffer"] = [[None, None, None] for _ in range(10)]
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                        buffer=[[None, None, None] for _ in range(10)])
        super().__init__(params, defaults)
        self.shard = None
        self.grad_scale = 1.0
        self._fused = set()    # ids of the parameters whose step of this iteration the owner pass ran

    def set_shard(self, shard, grad_scale=1.0):
        """Data-parallel optimizer sharding (dist.ShardedOptimizer): `shard` maps a parameter to the
        (start, end, grad) element range this rank updates, `grad` a flat fp32 tensor of end - start
        reduced gradients (the rank's reduce-scatter output) or None for p.grad[start:end];
        parameters missing from the map are not updated here (their step count still advances, as
        on the rank that owns them). None = every element of every parameter (the default).
        grad_scale: the kernel reads every sharded gradient as g * grad_scale (1 / world: the
        reduce-scatter's sum becomes the mean inside the update, no separate pass)."""
        self.shard = shard
        self.grad_scale = float(grad_scale) if shard is not None else 1.0

    def _scalars(self, group, step):
        beta1, beta2 = group["betas"]
        buffered = group["buffer"][int(step % 10)]
        if step == buffered[0]:
            n_sma, step_size = buffered[1], buffered[2]
        else:
            buffered[0] = step
            beta2_t = beta2 ** step
            n_sma_max = 2 / (1 - beta2) - 1
            n_sma = n_sma_max - 2 * step * beta2_t / (1 - beta2_t)
            buffered[1] = n_sma
            if n_sma >= 5:
                step_size = math.sqrt((1 - beta2_t) * (n_sma - 4) / (n_sma_max - 4) * (n_sma - 2) / n_sma
                                      * n_sma_max / (n_sma_max - 2)) / (1 - beta1 ** step)
            elif self.degenerated_to_sgd:
                step_size = 1.0 / (1 - beta1 ** step)
            else:
                step_size = -1
            buffered[2] = step_size
        return n_sma, step_size

    def _range(self, p):
        """(start, end, grad pointer) of the elements of p this rank updates, or None."""
        if self.shard is None:
            return 0, p.numel(), _lib.ptr(p.grad, "grad").value
        r = self.shard.get(p)
        if r is None or r[1] <= r[0]:
            return None
        a, b, g = r
        gp = _lib.ptr(g, "grad_shard").value if g is not None else p.grad.data_ptr() + 4 * a
        return a, b, gp

    def _segment(self, group, p, mode, step_size, rng=None):
        beta1, beta2 = group["betas"]
        state = self.state[p]
        a, b, gp = rng if rng is not None else (0, p.numel(), _lib.ptr(p.grad, "grad").value)
        s = _lib.RAdamSegment()
        s.p = _lib.ptr(p, "param").value + 4 * a
        s.g = gp
        s.m = _lib.ptr(state["exp_avg"], "exp_avg").value + 4 * a
        s.v = _lib.ptr(state["exp_avg_sq"], "exp_avg_sq").value + 4 * a
        s.n = b - a
        s.beta1, s.beta2 = beta1, beta2
        s.one_minus_beta1, s.one_minus_beta2 = 1 - beta1, 1 - beta2
        s.eps = group["eps"]
        s.decay_coef, s.step_coef = self._coefs(group, mode, step_size)
        s.mode = mode
        s.grad_scale = self.grad_scale
        return s

    @staticmethod
    def _coefs(group, mode, step_size):
        wd = group["weight_decay"]
        decay_coef = -wd * group["lr"] if (wd != 0 and mode != 0) else 0.0
        step_coef = -step_size * group["lr"] if mode != 0 else 0.0
        return decay_coef, step_coef

    def _advance(self, group, p):
        """state['step'] += 1 and this step's (mode, step_size) (radam.py:49-79)."""
        state = self.state[p]
        state["step"] += 1
        n_sma, step_size = self._scalars(group, state["step"])
        mode = 2 if n_sma >= 5 else (1 if step_size > 0 else 0)
        return mode, step_size

    def _params(self):
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("RAdam does not support sparse gradients")
                if p.dtype != torch.float32 or not p.is_contiguous() or not p.grad.is_contiguous():
                    raise TypeError("RAdam (HIP): parameters and grads must be contiguous float32")
                state = self.state[p]
                if len(state) == 0:
                    state["step"] = 0
                    state["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                yield group, p

    def table_step(self, tables):
        """The hash tables' step of this iteration as a nerf_radam_table_step for the owner pass
        (hashgrid.fused_table_step), or None when it cannot be fused: the tables must share one
        parameter group and one step count, without data-parallel sharding. Eager: the scalars of the
        coming step (state['step'] advances in step(), which then skips the tables); under a HIP-graph
        capture: a device slot that a filler refreshes before every replay (and advances the count)."""
        from . import graphs
        if self.shard is not None or not tables:
            return None
        group = next((g for g in self.param_groups if any(q is tables[0] for q in g["params"])), None)
        if group is None or any(not any(q is p for q in group["params"]) for p in tables):
            return None
        for p in tables:
            if p.grad is None or p.dtype != torch.float32 or not p.is_contiguous():
                return None
            state = self.state[p]
            if len(state) == 0:
                state["step"] = 0
                state["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
        if len({self.state[p]["step"] for p in tables}) != 1:
            return None
        beta1, beta2 = group["betas"]
        s = _lib.RAdamTableStep()
        keep = [_lib.ptr_array(list(tables), "tables"),
                _lib.ptr_array([self.state[p]["exp_avg"] for p in tables], "exp_avg"),
                _lib.ptr_array([self.state[p]["exp_avg_sq"] for p in tables], "exp_avg_sq")]
        s.d_params, s.d_exp_avg, s.d_exp_avg_sq = keep
        s.beta1, s.beta2, s.one_minus_beta1, s.one_minus_beta2 = beta1, beta2, 1 - beta1, 1 - beta2
        s.eps = group["eps"]
        sc = graphs.active()
        if sc is None:
            n_sma, step_size = self._scalars(group, self.state[tables[0]]["step"] + 1)
            mode = 2 if n_sma >= 5 else (1 if step_size > 0 else 0)
            s.decay_coef, s.step_coef = self._coefs(group, mode, step_size)
            s.mode, s.d_coef = mode, None
        else:
            off, dptr = sc.alloc_f32(4)
            s.decay_coef = s.step_coef = 0.0
            s.mode, s.d_coef = 2, dptr

            def fill(hi, hf, off=off, group=group, tables=tuple(tables)):
                for p in tables:
                    mode, step_size = self._advance(group, p)
                dc, stc = self._coefs(group, mode, step_size)
                hf[off:off + 4] = (dc, stc, float(mode), 0.0)
            sc.add_filler(fill)
        self._fused = {id(p) for p in tables}
        s._keep = keep      # the pointer arrays live as long as the struct
        return s

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        from . import graphs
        sc = graphs.active()
        if sc is not None:
            self._capture_step(sc)
            return loss
        segs, updated = [], []
        fused, self._fused = self._fused, set()
        for group, p in self._params():
            if id(p) in fused:     # updated by the owner pass (table_step): the step count only
                self._advance(group, p)
                torch.autograd.graph.increment_version(p)
                continue
            mode, step_size = self._advance(group, p)
            rng = self._range(p)
            if rng is None:
                continue
            segs.append(self._segment(group, p, mode, step_size, rng))
            updated.append(p)
        for i in range(0, len(segs), _MAX_SEGS):
            chunk = segs[i:i + _MAX_SEGS]
            arr = (_lib.RAdamSegment * len(chunk))(*chunk)
            _lib.call("nerf_radam_step", arr, len(chunk), None, _lib.stream())
        # the kernel writes through raw pointers: bump the version counters the reference's
        # in-place tensor ops would have bumped (cache keys such as HashEmbedder.packed_tables)
        for p in updated:
            torch.autograd.graph.increment_version(p)
        return loss

    def _capture_step(self, sc):
        """Captured in a HIP graph (graphs.GraphedTrainStep): the launch reads (decay_coef,
        step_coef, mode) of each tensor from device slots that a filler computes before every
        replay with the same host algebra (state['step'] advances there, not at capture)."""
        fused, self._fused = self._fused, set()
        every = [(g, p) for g, p in self._params() if id(p) not in fused]   # the owner pass's (table_step)
        pairs = [(g, p) for g, p in every if self._range(p) is not None]
        others = [(g, p) for g, p in every if self._range(p) is None]
        if others:
            def advance(hi, hf, others=others):     # parameters another rank updates: step count only
                for g, p in others:
                    self._advance(g, p)
            sc.add_filler(advance)
        for i in range(0, len(pairs), _MAX_SEGS):
            chunk = pairs[i:i + _MAX_SEGS]
            off, dptr = sc.alloc_f32(4 * len(chunk))
            segs = [self._segment(g, p, 2, 0.0, self._range(p)) for g, p in chunk]
            arr = (_lib.RAdamSegment * len(chunk))(*segs)
            _lib.call("nerf_radam_step", arr, len(chunk), _lib.c_vp(dptr), _lib.stream())

            def fill(hi, hf, off=off, chunk=chunk):
                for j, (g, p) in enumerate(chunk):
                    mode, step_size = self._advance(g, p)
                    dc, stc = self._coefs(g, mode, step_size)
                    hf[off + 4 * j:off + 4 * j + 4] = (dc, stc, float(mode), 0.0)
            sc.add_filler(fill)
