"""A-CAQ quantizers on the HIP kernels (csrc/quant.hip).

API mirror of PocketNeRF/quantization.py: FakeQuantizer (:6-64), LearnedBitwidthQuantizer (:66-194),
PassthroughQuantizer (:198-210) and calculate_fqr (:213-227) — same constructor arguments, parameters
(`soft_bits`, `range_scale`, `v_max`), buffers (`running_min`, `running_max`), properties and
calibrate-on-first-training-call behaviour. The quantizer's scalar algebra (bit width, scale, zero
point) is evaluated on the device by nerf_quant_params, so no call syncs with the host; the values
are applied elementwise by nerf_fake_quant or fused into the hash-grid gather / MLP kernels
(hashgrid.HashEmbedder, field.NeRFSmall).
"""
import torch
import torch.nn as nn

from . import _lib


class FakeQuantFn(torch.autograd.Function):
    """y = Q(x) with the quantizer record `rec` [8]; in training mode Q is the STE form
    x + (deq - x).detach() (quantization.py:53-54, :176-181), whose gradient is the identity."""

    @staticmethod
    def forward(ctx, x, rec, ste=True):
        xc = x.contiguous()
        y = torch.empty_like(xc)
        _lib.call("nerf_fake_quant", _lib.ptr(xc, "x"), xc.numel(), _lib.ptr(rec, "record"), _lib.ptr(y, "y"),
                  _lib.stream())
        ctx.ste = ste
        return y

    @staticmethod
    def backward(ctx, g):
        # eval mode returns (round(.) - zp) * scale, whose gradient w.r.t. x is zero; the gradient
        # w.r.t. the quantizer's own scalars in eval mode is not propagated (the reference never
        # trains a module in eval mode)
        return (g if ctx.ste else torch.zeros_like(g)), None, None


def _descriptor(q):
    d = _lib.Quantizer()
    d.soft_bits = _lib.ptr(q.soft_bits.detach(), "soft_bits").value
    d.range_scale = _lib.ptr(q.range_scale.detach(), "range_scale").value
    d.v_max = _lib.ptr(q.v_max.detach(), "v_max").value if q.v_max is not None else None
    d.running_min = _lib.ptr(q.running_min, "running_min").value
    d.running_max = _lib.ptr(q.running_max, "running_max").value
    d.min_bits = float(q.min_bits)
    d.max_bits = float(q.max_bits)
    return d


_DESC_CACHE = {}


def _descriptors(quantizers):
    """ctypes array of nerf_quantizer for these modules, cached on the tensors' device addresses
    (rebuilding 16 descriptors per forward was a measurable share of a render step's host time)."""
    key = tuple((q.soft_bits.data_ptr(), q.range_scale.data_ptr(),
                 q.v_max.data_ptr() if q.v_max is not None else 0, q.running_min.data_ptr(),
                 q.running_max.data_ptr(), q.min_bits, q.max_bits) for q in quantizers)
    arr = _DESC_CACHE.get(key)
    if arr is None:
        if len(_DESC_CACHE) > 64:
            _DESC_CACHE.clear()
        arr = (_lib.Quantizer * len(quantizers))()
        for i, q in enumerate(quantizers):
            arr[i] = _descriptor(q)
        _DESC_CACHE[key] = arr
    return arr


def quant_records(quantizers, training):
    """[n, 8] device records {scale, scale+1e-8, zero_point, qmin, qmax, ste, bits, 0} of n
    LearnedBitwidthQuantizers in one launch (quantization.py:158-178)."""
    dev = quantizers[0].soft_bits.device
    rec = torch.empty(len(quantizers), 8, device=dev, dtype=torch.float32)
    _lib.call("nerf_quant_params", _descriptors(quantizers), len(quantizers), int(bool(training)),
              _lib.ptr(rec, "records"), _lib.stream())
    return rec


def new_stats(n, device):
    """Calibration statistics buffer: n (min, max) slots, reset to (+inf, -inf)."""
    st = torch.empty(n, 2, device=device, dtype=torch.int32)
    _lib.call("nerf_quant_minmax_reset", _lib.ptr(st, "stats", dtype=torch.int32), n, _lib.stream())
    return st


def calibrate_from_stats(quantizers, stats):
    """calibrate() (quantization.py:97-119) of each quantizer from its (min, max) row of `stats`.
    Under data parallelism the statistics are first reduced over ranks (dist.py), so every replica
    calibrates identically."""
    from .dist import allreduce_calibration_stats
    allreduce_calibration_stats(stats)
    _lib.call("nerf_quant_calibrate", _descriptors(quantizers), len(quantizers),
              _lib.ptr(stats, "stats", dtype=torch.int32), _lib.stream())
    for q in quantizers:
        q.calibrated = True


class LearnedBitwidthQuantizer(nn.Module):
    """quantization.py:66-194 (soft bit width, calibrated range) on the device."""

    def __init__(self, init_bits=8.0, min_bits=2.0, max_bits=32.0, symmetric=True):
        super().__init__()
        self.soft_bits = nn.Parameter(torch.tensor(float(init_bits)))
        self.min_bits = min_bits
        self.max_bits = max_bits
        self.symmetric = symmetric
        self.range_scale = nn.Parameter(torch.tensor(0.0002))
        if not symmetric:
            self.v_max = nn.Parameter(torch.tensor(0.0001))
        else:
            self.register_buffer("v_max", None)
        self.calibrated = False
        self.register_buffer("running_min", torch.tensor(float("inf")))
        self.register_buffer("running_max", torch.tensor(float("-inf")))
        for p in self.parameters(recurse=False):
            p._nerf_no_grad = True   # every use is detached (:176-181): no gradient ever reaches them

    def calibrate(self, x):
        """Fold x's min/max into the running range and reset range_scale / v_max (:97-119)."""
        with torch.no_grad():
            xc = x.detach().contiguous().float()
            st = new_stats(1, xc.device)
            _lib.call("nerf_quant_minmax", _lib.ptr(xc, "x"), xc.numel(), _lib.ptr(st, "stats", dtype=torch.int32),
                      _lib.stream())
            calibrate_from_stats([self], st)

    @property
    def bit_width(self):
        return torch.clamp(self.soft_bits, self.min_bits, self.max_bits)

    @property
    def integer_bit_width(self):
        return int(torch.round(self.bit_width).item())

    def get_quantization_params(self):
        B = self.integer_bit_width
        if self.symmetric:
            return -(2 ** (B - 1)), 2 ** (B - 1) - 1
        return 0, 2 ** B - 1

    def record(self, training=None):
        """This quantizer's [8] device record for the current mode."""
        return quant_records([self], self.training if training is None else training)[0]

    def forward(self, x):
        if self.training and not self.calibrated:
            self.calibrate(x)
        return FakeQuantFn.apply(x.float(), self.record(), self.training)

    def extra_repr(self):
        return (f"soft_bits={self.soft_bits.data:.2f}, range=[{self.min_bits}, {self.max_bits}], "
                f"symmetric={self.symmetric}, range_scale={self.range_scale.data:.6f}")


class FakeQuantizer(nn.Module):
    """quantization.py:6-64: fixed bit width, learnable scale (and zero point when asymmetric).
    The record is assembled from the device scalars with tensor ops; Q runs in nerf_fake_quant."""

    def __init__(self, num_bits=8, symmetric=True, initialize_scale=True):
        super().__init__()
        self.num_bits = num_bits
        self.symmetric = symmetric
        if symmetric:
            self.qmin, self.qmax = -(2 ** (num_bits - 1)), 2 ** (num_bits - 1) - 1
        else:
            self.qmin, self.qmax = 0, 2 ** num_bits - 1
        self.scale = nn.Parameter(torch.tensor(1.0))
        if not symmetric:
            self.zero_point = nn.Parameter(torch.tensor(0.0))
        else:
            self.register_buffer("zero_point", torch.tensor(0.0))

    def forward(self, x):
        s = self.scale.detach().reshape(1)
        zp = self.zero_point.detach().reshape(1) if not self.symmetric else torch.zeros_like(s)
        c = lambda v: torch.full_like(s, float(v))  # noqa: E731
        # x / scale (+ zero_point): no epsilon in this quantizer (:35-38)
        rec = torch.cat([s, s, zp, c(self.qmin), c(self.qmax), c(1.0 if self.training else 0.0),
                         c(self.num_bits), c(0.0)]).contiguous()
        return FakeQuantFn.apply(x.float(), rec, self.training)

    def extra_repr(self):
        return f"num_bits={self.num_bits}, symmetric={self.symmetric}"


class PassthroughQuantizer(nn.Module):
    """quantization.py:198-210."""

    def __init__(self, **kwargs):
        super().__init__()
        self.bit_width = 32.0
        self.integer_bit_width = 32

    def forward(self, x):
        return x

    def extra_repr(self):
        return "passthrough"


def calculate_fqr(quantizers):
    """Average bit width over the quantizers (quantization.py:213-227)."""
    if not quantizers:
        return 32.0
    total = 0
    for q in quantizers:
        if hasattr(q, "bit_width"):
            total += q.bit_width
        elif hasattr(q, "num_bits"):
            total += q.num_bits
        else:
            total += 32
    return total / len(quantizers)
