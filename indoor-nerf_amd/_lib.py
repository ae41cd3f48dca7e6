"""ctypes binding of libnerfhip.so (include/nerf_hip.h).

The product path has no fallback: if the library is missing, cannot be loaded, or a tensor is not a
contiguous float32 CUDA tensor, the call raises. Kernel errors raise RuntimeError with the
library's message (nerf_last_error).
"""
import contextlib
import ctypes
import os

import torch  # must be imported before the library so it binds torch's libamdhip64.so.7

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NERF_HIP_LIB", os.path.join(_HERE, "libnerfhip.so"))

c_f32p = ctypes.POINTER(ctypes.c_float)
c_i64 = ctypes.c_int64
c_vp = ctypes.c_void_p
c_int = ctypes.c_int
c_u64 = ctypes.c_uint64

MAX_LEVELS = 16


class MlpWeights(ctypes.Structure):
    _fields_ = [(n, c_vp) for n in ("w0", "w1", "c0", "c1", "c2")]


class MlpGrads(ctypes.Structure):
    _fields_ = [(n, c_vp) for n in ("w0", "w1", "c0", "c1", "c2")]


MLP_MAX_JOBS = 2   # NERF_MLP_MAX_JOBS
MAX_CHECK = 32     # NERF_MAX_CHECK


class PointOrder(ctypes.Structure):
    """nerf_point_order (include/nerf_hip.h)."""
    _fields_ = [("io_rows", c_vp), ("seg_split", c_i64), ("spr2", c_i64)]


class MlpBwdJob(ctypes.Structure):
    """nerf_mlp_bwd_job (include/nerf_hip.h): the arguments of nerf_mlp_bwd_q for one net."""
    _fields_ = [("feat", c_vp), ("feat_stride_point", c_i64), ("feat_stride_level", c_i64), ("sh", c_vp),
                ("sh_stride", c_i64), ("viewdirs", c_vp), ("samples_per_ray", c_i64), ("keep", c_vp),
                ("n_points", c_i64), ("weights", MlpWeights), ("graw", c_vp), ("grads", MlpGrads), ("dfeat", c_vp),
                ("dsh", c_vp), ("dgeo", c_vp), ("act_qrec", c_vp), ("order", PointOrder),
                ("dfeat_stride_point", c_i64), ("dfeat_stride_level", c_i64), ("rows", c_vp), ("d_count", c_vp),
                ("h3", c_vp)]


PRIORS_MAX_RAYS = 8192   # NERF_PRIORS_MAX_RAYS


class CompositeBwdJob(ctypes.Structure):
    _fields_ = [("raw", c_vp), ("raw_channels", c_int), ("z", c_vp), ("rays_d", c_vp), ("noise", c_vp),
                ("n_rays", c_i64), ("n_samples", c_int), ("white_bkgd", c_int),
                ("g_rgb", c_vp), ("g_disp", c_vp), ("g_acc", c_vp), ("g_weights", c_vp), ("g_depth", c_vp),
                ("g_entropy", c_vp), ("g_normal", c_vp), ("graw", c_vp)]


class BinJob(ctypes.Structure):
    """nerf_bin_job (include/nerf_hip.h)."""
    _fields_ = [("xyz", c_vp), ("rows", c_vp), ("count", c_vp), ("n_points", c_i64), ("dfeat", c_vp),
                ("feat_stride_point", c_i64), ("feat_stride_level", c_i64), ("dfeat2", c_vp), ("rows2", c_vp),
                ("feat2_stride_point", c_i64), ("feat2_stride_level", c_i64), ("chunk_base", c_i64)]


class TVBinJob(ctypes.Structure):
    """nerf_tv_bin_job (include/nerf_hip.h, ABI 11)."""
    _fields_ = [("d_tables", c_vp), ("min_vertex", c_vp), ("d_min_vertex", c_vp), ("cube", c_vp), ("d_scale", c_vp),
                ("d_verts", c_vp), ("chunk_base", c_i64)]


class TVFwdJob(ctypes.Structure):
    """nerf_tv_fwd_job (include/nerf_hip.h, ABI 11)."""
    _fields_ = [("d_tables", c_vp), ("min_vertex", c_vp), ("d_min_vertex", c_vp), ("cube", c_vp), ("d_loss", c_vp),
                ("d_verts", c_vp)]


class ZeroRange(ctypes.Structure):
    _fields_ = [("ptr", c_vp), ("n", c_i64)]


MAX_ZERO_RANGES = 4


class PriorsConfig(ctypes.Structure):
    """nerf_priors_config (include/nerf_hip.h)."""
    _fields_ = [("use_manhattan", c_int), ("use_planarity", c_int), ("use_consistency", c_int),
                ("w_manhattan", ctypes.c_float), ("w_planarity", ctypes.c_float), ("w_consistency", ctypes.c_float),
                ("d_scale", c_vp), ("confidence_threshold", ctypes.c_float), ("normal_threshold", ctypes.c_float),
                ("centres0", c_vp), ("perm", c_vp), ("idx1", c_vp), ("usv", c_vp), ("seed", c_u64),
                ("offset", c_u64), ("d_rng", c_vp)]


class NormalHead(ctypes.Structure):
    _fields_ = [("n0", c_vp), ("b0", c_vp), ("n1", c_vp), ("b1", c_vp)]


class NormalHeadGrads(ctypes.Structure):
    _fields_ = [("n0", c_vp), ("b0", c_vp), ("n1", c_vp), ("b1", c_vp)]


class RAdamSegment(ctypes.Structure):
    _fields_ = [("p", c_vp), ("g", c_vp), ("m", c_vp), ("v", c_vp), ("n", c_i64),
                ("beta1", ctypes.c_float), ("beta2", ctypes.c_float),
                ("one_minus_beta1", ctypes.c_float), ("one_minus_beta2", ctypes.c_float),
                ("eps", ctypes.c_float), ("decay_coef", ctypes.c_float), ("step_coef", ctypes.c_float),
                ("mode", c_int), ("grad_scale", ctypes.c_float)]


class RAdamTableStep(ctypes.Structure):
    """nerf_radam_table_step (include/nerf_hip.h): the tables' optimizer step fused into the owner pass."""
    _fields_ = [("d_params", ctypes.POINTER(c_vp)), ("d_exp_avg", ctypes.POINTER(c_vp)),
                ("d_exp_avg_sq", ctypes.POINTER(c_vp)),
                ("beta1", ctypes.c_float), ("beta2", ctypes.c_float),
                ("one_minus_beta1", ctypes.c_float), ("one_minus_beta2", ctypes.c_float),
                ("eps", ctypes.c_float), ("decay_coef", ctypes.c_float), ("step_coef", ctypes.c_float),
                ("mode", c_int), ("d_coef", c_vp)]


class Quantizer(ctypes.Structure):
    _fields_ = [("soft_bits", c_vp), ("range_scale", c_vp), ("v_max", c_vp), ("running_min", c_vp),
                ("running_max", c_vp), ("min_bits", ctypes.c_float), ("max_bits", ctypes.c_float)]


class Camera(ctypes.Structure):
    _fields_ = [("c2w", ctypes.c_float * 12), ("fx", ctypes.c_float), ("fy", ctypes.c_float),
                ("cx", ctypes.c_float), ("cy", ctypes.c_float)]


# name -> argtypes (restype is int for all but the two metadata calls)
SIGNATURES = {
    "nerf_hash_encode_fwd": [c_vp, c_i64, c_f32p, c_f32p, c_f32p, c_int, c_int, ctypes.POINTER(c_vp),
                             c_vp, c_i64, c_i64, c_vp, c_vp],
    "nerf_hash_encode_fwd_q": [c_vp, c_i64, c_f32p, c_f32p, c_f32p, c_int, c_int, ctypes.POINTER(c_vp), c_vp,
                               c_vp, c_i64, c_i64, c_vp, c_vp],
    "nerf_hash_encode_bwd": [c_vp, c_i64, c_f32p, c_f32p, c_f32p, c_int, c_int, c_vp, c_i64, c_i64,
                             ctypes.POINTER(c_vp), c_vp],
    "nerf_hash_encode_bwd_ws": [c_vp, c_i64, c_f32p, c_f32p, c_f32p, c_int, c_int, c_vp, c_i64, c_i64,
                                ctypes.POINTER(c_vp), c_int, c_vp, ctypes.c_size_t, c_vp],
    "nerf_hash_encode_bwd_bin": [c_vp, c_i64, c_f32p, c_f32p, c_f32p, c_int, c_int, c_vp, c_i64, c_i64, c_i64,
                                 c_i64, c_int, c_vp, ctypes.c_size_t, c_vp],
    "nerf_hash_encode_bwd_owner": [c_int, c_int, c_i64, c_i64, ctypes.POINTER(c_vp), c_int, c_vp, ctypes.c_size_t,
                                   c_vp],
    "nerf_hash_encode_bwd_bin_batch": [ctypes.POINTER(BinJob), c_int, c_f32p, c_f32p, c_f32p, c_int, c_int, c_i64,
                                       c_int, c_vp, ctypes.c_size_t, c_vp],
    "nerf_hash_encode_bwd_bin_batch_tv": [ctypes.POINTER(BinJob), c_int, c_f32p, c_f32p, c_f32p, c_int, c_int, c_i64,
                                          c_int, c_vp, ctypes.c_size_t, ctypes.POINTER(TVBinJob), c_vp],
    "nerf_hash_encode_bwd_bin_rows": [c_vp, c_vp, c_vp, c_i64, c_f32p, c_f32p, c_f32p, c_int, c_int, c_vp, c_i64,
                                      c_i64, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_int, c_vp, ctypes.c_size_t, c_vp],
    "nerf_active_rows": [c_vp, c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_i64, c_int, c_vp, ctypes.c_size_t, c_vp],
    "nerf_hash_bwd_entry_count": [c_int, c_int, c_i64, c_i64, c_int, c_vp, ctypes.c_size_t, c_vp, c_vp],
    "nerf_hash_encode_bwd_owner_step": [c_int, c_int, c_int, c_int, c_i64, c_i64, ctypes.POINTER(c_vp), c_int, c_vp,
                                        ctypes.c_size_t, ctypes.POINTER(RAdamTableStep), c_vp],
    "nerf_hash_encode_bwd_owner_range": [c_int, c_int, c_int, c_int, c_i64, c_i64, ctypes.POINTER(c_vp), c_int, c_vp,
                                         ctypes.c_size_t, c_vp],
    "nerf_sh4_fwd": [c_vp, c_i64, c_vp, c_vp],
    "nerf_mlp_fwd": [c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, ctypes.POINTER(MlpWeights),
                     c_vp, c_vp, c_vp],
    "nerf_mlp_bwd": [c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, ctypes.POINTER(MlpWeights),
                     c_vp, ctypes.POINTER(MlpGrads), c_vp, c_vp, c_vp, c_vp],
    "nerf_mlp_fwd_q": [c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, ctypes.POINTER(MlpWeights),
                       c_vp, c_vp, c_vp, c_vp, c_i64, c_vp],
    "nerf_mlp_fwd_ord": [c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, ctypes.POINTER(MlpWeights),
                         c_vp, c_vp, c_vp, c_vp, c_i64, ctypes.POINTER(PointOrder), c_vp],
    "nerf_mlp_fwd_h3": [c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, ctypes.POINTER(MlpWeights),
                        c_vp, c_vp, c_vp, c_vp, c_i64, ctypes.POINTER(PointOrder), c_vp, c_vp],
    "nerf_mlp_bwd_q": [c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64, ctypes.POINTER(MlpWeights),
                       c_vp, ctypes.POINTER(MlpGrads), c_vp, c_vp, c_vp, c_vp, c_vp],
    "nerf_count_nonfinite": [ctypes.POINTER(c_vp), ctypes.POINTER(c_i64), c_int, c_vp, c_vp],
    "nerf_priors_prep": [c_vp, c_vp, c_vp, c_i64, ctypes.POINTER(PriorsConfig), c_vp, ctypes.c_size_t, c_vp, c_vp],
    "nerf_priors_loss": [c_vp, c_vp, c_vp, c_i64, ctypes.POINTER(PriorsConfig), c_vp, ctypes.c_size_t, c_vp, c_vp,
                         c_vp],
    "nerf_priors_loss_add": [c_vp, c_vp, c_vp, c_i64, ctypes.POINTER(PriorsConfig), c_vp, ctypes.c_size_t, c_vp, c_vp,
                             c_vp, c_vp],
    "nerf_priors_bwd": [c_vp, c_vp, c_vp, c_i64, ctypes.POINTER(PriorsConfig), c_vp, ctypes.c_size_t, c_vp, c_vp,
                        c_vp, c_vp],
    "nerf_mlp_bwd_batch": [ctypes.POINTER(MlpBwdJob), c_int, c_vp, ctypes.c_size_t, c_vp],
    "nerf_normal_head_fwd": [c_vp, c_vp, c_vp, c_i64, ctypes.POINTER(NormalHead), c_vp, c_vp],
    "nerf_normal_head_fwd_rows": [c_vp, c_vp, c_vp, c_vp, c_i64, ctypes.POINTER(NormalHead), c_vp, c_vp, c_vp],
    "nerf_normal_head_bwd": [c_vp, c_vp, c_i64, ctypes.POINTER(NormalHead), c_vp, c_vp, c_vp,
                             ctypes.POINTER(NormalHeadGrads), c_vp, ctypes.c_size_t, c_vp],
    "nerf_composite_fwd": [c_vp, c_int, c_vp, c_vp, c_vp, c_i64, c_int, c_int,
                           c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "nerf_composite_fwd_tv": [c_vp, c_int, c_vp, c_vp, c_vp, c_i64, c_int, c_int,
                              c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, ctypes.POINTER(TVFwdJob), c_int, c_int, c_vp],
    "nerf_composite_bwd": [c_vp, c_int, c_vp, c_vp, c_vp, c_i64, c_int, c_int,
                           c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "nerf_composite_bwd_batch": [ctypes.POINTER(CompositeBwdJob), c_int, c_vp],
    "nerf_composite_sample_fine": [c_vp, c_int, c_vp, c_vp, c_vp, c_i64, c_int, c_int,
                                   c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                   c_vp, c_i64, c_int, c_int, c_vp, c_vp, c_u64, c_u64, c_vp,
                                   c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "nerf_sample_stratified": [c_vp, c_i64, c_i64, c_int, c_vp, c_int, c_int, c_vp, c_u64, c_u64, c_vp, c_vp, c_vp,
                               c_vp, c_vp, c_vp],
    "nerf_sample_stratified_sh": [c_vp, c_i64, c_i64, c_int, c_vp, c_int, c_int, c_vp, c_u64, c_u64, c_vp, c_vp, c_vp,
                                  c_vp, c_vp, c_vp, c_vp],
    "nerf_sample_pdf": [c_vp, c_i64, c_vp, c_i64, c_i64, c_int, c_int, c_int, c_vp, c_vp, c_u64, c_u64, c_vp, c_vp,
                        c_vp],
    "nerf_sample_fine": [c_vp, c_i64, c_vp, c_vp, c_i64, c_int, c_int, c_int, c_vp, c_vp, c_u64, c_u64, c_vp,
                         c_vp, c_vp, c_vp, c_vp, c_vp],
    "nerf_sample_fine_rows": [c_vp, c_i64, c_vp, c_vp, c_i64, c_int, c_int, c_int, c_vp, c_vp, c_u64, c_u64, c_vp,
                              c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp],
    "nerf_sample_rays": [ctypes.POINTER(Camera), c_int, c_int, c_int, c_int, c_int, c_int, c_i64, c_int, c_u64,
                         c_u64, c_vp, c_int, c_vp, c_vp, c_vp, c_vp, c_vp],
    "nerf_sample_rays_sel": [c_vp, c_vp, c_i64, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_i64, c_vp, c_vp,
                             c_vp, c_vp, c_vp, c_vp],
    "nerf_rays_pack_z": [c_vp, c_vp, c_i64, ctypes.c_float, ctypes.c_float, c_int, ctypes.c_float, ctypes.c_float,
                         c_int, c_vp, ctypes.POINTER(ZeroRange), c_int, c_vp],
    "nerf_rays_pack": [c_vp, c_vp, c_i64, ctypes.c_float, ctypes.c_float, c_int, ctypes.c_float, ctypes.c_float,
                       c_int, c_vp, c_vp],
    "nerf_radam_step": [ctypes.POINTER(RAdamSegment), c_int, c_vp, c_vp],
    "nerf_host_ring_alloc": [c_i64, ctypes.POINTER(c_vp)],
    "nerf_host_ring_free": [c_vp],
    "nerf_scalars_fetch": [c_vp, c_i64, c_int, c_i64, c_vp, c_vp, c_vp],
    "nerf_nearest_pixel": [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp],
    "nerf_tv_fwd": [ctypes.POINTER(c_vp), c_int, c_int, ctypes.POINTER(c_i64), c_vp, ctypes.POINTER(c_int), c_vp,
                    c_vp, c_vp],
    "nerf_tv_bwd": [ctypes.POINTER(c_vp), c_int, c_int, ctypes.POINTER(c_i64), c_vp, ctypes.POINTER(c_int), c_vp,
                    ctypes.POINTER(c_vp), c_vp],
    "nerf_tv_bwd_bin": [ctypes.POINTER(c_vp), c_int, c_int, ctypes.POINTER(c_i64), c_vp, ctypes.POINTER(c_int), c_vp,
                        c_vp, c_i64, c_i64, c_int, c_vp, ctypes.c_size_t, c_vp],
    "nerf_train_loss_fwd": [c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, ctypes.c_float, c_vp, c_int, ctypes.c_float,
                            c_vp, c_vp, c_vp, c_vp],
    "nerf_quant_params": [ctypes.POINTER(Quantizer), c_int, c_int, c_vp, c_vp],
    "nerf_quant_minmax_reset": [c_vp, c_int, c_vp],
    "nerf_quant_minmax": [c_vp, c_i64, c_vp, c_vp],
    "nerf_hash_gather_minmax": [c_vp, c_i64, c_f32p, c_f32p, c_f32p, c_int, c_int, ctypes.POINTER(c_vp), c_vp, c_vp],
    "nerf_quant_calibrate": [ctypes.POINTER(Quantizer), c_int, c_vp, c_vp],
    "nerf_fake_quant": [c_vp, c_i64, c_vp, c_vp, c_vp],
    "nerf_acaq_update": [ctypes.POINTER(Quantizer), c_int, c_vp, c_vp, c_int, ctypes.c_double, ctypes.c_double,
                         c_vp, c_vp],
    "nerf_quant_pack_tables": [ctypes.POINTER(c_vp), c_int, c_int, c_vp, c_vp, c_int, c_vp, c_vp, c_vp],
    "nerf_hash_encode_fwd_packed": [c_vp, c_i64, c_f32p, c_f32p, c_f32p, c_int, c_int, c_vp, c_vp, c_vp, c_i64,
                                    c_i64, c_vp, c_vp],
    "nerf_train_loss_bwd": [c_vp, c_vp, c_vp, c_i64, ctypes.c_float, c_int, ctypes.c_float, c_vp, c_vp, c_vp,
                            c_vp, c_vp, c_vp, c_vp],
}

_lib = None


def load():
    """Load libnerfhip.so once; raise if it is missing (no CPU fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libnerfhip.so not found at {LIB_PATH}: build it with `python -c "
                           f"'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
    lib = ctypes.CDLL(LIB_PATH)
    lib.nerf_last_error.restype = ctypes.c_char_p
    lib.nerf_last_error.argtypes = []
    lib.nerf_abi_version.restype = c_int
    lib.nerf_abi_version.argtypes = []
    lib.nerf_hash_bwd_chunk_points.restype = c_int
    lib.nerf_hash_bwd_chunk_points.argtypes = []
    lib.nerf_tv_bwd_bin_chunks.restype = c_i64
    lib.nerf_tv_bwd_bin_chunks.argtypes = [c_int, ctypes.POINTER(c_int)]
    lib.nerf_hash_encode_bwd_workspace_bytes.restype = ctypes.c_size_t
    lib.nerf_hash_encode_bwd_workspace_bytes.argtypes = [c_int, c_int, c_i64, c_int]
    lib.nerf_normal_head_bwd_workspace_bytes.restype = ctypes.c_size_t
    lib.nerf_normal_head_bwd_workspace_bytes.argtypes = []
    lib.nerf_priors_workspace_bytes.restype = ctypes.c_size_t
    lib.nerf_priors_workspace_bytes.argtypes = [c_i64]
    lib.nerf_mlp_bwd_det_workspace_bytes.restype = ctypes.c_size_t
    lib.nerf_mlp_bwd_det_workspace_bytes.argtypes = []
    lib.nerf_active_rows_workspace_bytes.restype = ctypes.c_size_t
    lib.nerf_active_rows_workspace_bytes.argtypes = [c_i64]
    lib.nerf_quant_packed_bytes.restype = ctypes.c_size_t
    lib.nerf_quant_packed_bytes.argtypes = [c_int, c_int]
    if hasattr(lib, "nerf_mlp_h3_bytes"):   # ABI 10 (an older A/B variant may lack it)
        lib.nerf_mlp_h3_bytes.restype = ctypes.c_size_t
        lib.nerf_mlp_h3_bytes.argtypes = [c_i64]
    for name, argtypes in SIGNATURES.items():
        # a library of an older tree (an A/B variant, tools/build_variant.py --rev) may lack newer
        # entries: they stay unbound and call() raises if one is used (test_abi holds the in-tree library
        # to every symbol of include/nerf_hip.h)
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.argtypes = argtypes
        fn.restype = c_int
    _lib = lib
    return lib


def exported_symbols():
    return ["nerf_last_error", "nerf_abi_version", "nerf_hash_bwd_chunk_points", "nerf_tv_bwd_bin_chunks",

            "nerf_hash_encode_bwd_workspace_bytes",
            "nerf_quant_packed_bytes", "nerf_mlp_bwd_det_workspace_bytes", "nerf_priors_workspace_bytes",
            "nerf_normal_head_bwd_workspace_bytes", "nerf_active_rows_workspace_bytes",
            "nerf_mlp_h3_bytes"] + list(SIGNATURES)


_TIMING = None   # when a list: (name, start_event, end_event) per launch, recorded on the current stream


def set_timing(enabled):
    """Record a pair of HIP events around every kernel call (bench.py's per-kernel timing)."""
    global _TIMING
    _TIMING = [] if enabled else None


def timing_enabled():
    return _TIMING is not None


def timing_records():
    return _TIMING or []


def call(name, *args):
    lib = load()
    if _TIMING is not None:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("kernel timing cannot be recorded inside a HIP-graph capture (torch on ROCm "
                               "refuses external events); time an eager step instead")
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        rc = getattr(lib, name)(*args)
        ev1.record()
        _TIMING.append((name, ev0, ev1))
    else:
        rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.nerf_last_error().decode(errors="replace")
        raise RuntimeError(f"{name} failed (code {rc}): {msg}")


def stream():
    return c_vp(torch.cuda.current_stream().cuda_stream)


# Zero fills folded into a later launch (nerf_rays_pack_z: render()'s first kernel): a training step
# (model.forward_backward, inside zero_deferral()) registers its MLP-gradient zero and its TV loss
# accumulator here before render(), and whoever needs one of them zero before that launch took it
# calls flush_zero_fills first. Pending fills are kept per device: a render() on one device takes only
# that device's ranges. Outside a training step's scope every fill is done at once, so public callers
# (GradArena.zero_() followed by a read of p.grad, or a backward of their own) never see stale values.
_ZERO_FILLS = {}   # device index -> [tensor]
_FOLD_FILLS = {"on": True}
_DEFER_SCOPE = [0]


def set_fold_fills(enabled=True):
    """Fold deferrable zero fills into render()'s first launch (default); off = fill at once."""
    _FOLD_FILLS["on"] = bool(enabled)


@contextlib.contextmanager
def zero_deferral():
    """Scope of one training iteration (model.forward_backward): zero fills and the tables' deferred
    gradient zero may wait for the launches that consume them."""
    _DEFER_SCOPE[0] += 1
    try:
        yield
    finally:
        _DEFER_SCOPE[0] -= 1


def zero_deferral_active():
    return _DEFER_SCOPE[0] > 0


def defer_fill_zero(t):
    """Zero the contiguous float32 CUDA tensor `t` in the next nerf_rays_pack_z launch on its device (or
    at flush_zero_fills, whichever comes first); at once outside zero_deferral()."""
    if not (_FOLD_FILLS["on"] and _DEFER_SCOPE[0] > 0 and t.is_cuda and t.dtype == torch.float32
            and t.is_contiguous()):
        t.zero_()
        return
    _ZERO_FILLS.setdefault(t.device.index, []).append(t)


def take_zero_fills(device):
    """Up to MAX_ZERO_RANGES pending fills of `device` as a ZeroRange array (ctypes) + count; they are
    done by the caller's launch."""
    pending = _ZERO_FILLS.get(torch.device(device).index, [])
    taken = pending[:MAX_ZERO_RANGES]
    del pending[:MAX_ZERO_RANGES]
    arr = (ZeroRange * max(1, len(taken)))(*[ZeroRange(t.data_ptr(), t.numel()) for t in taken])
    return arr, len(taken), taken


def flush_zero_fills(tensors=None):
    """Zero pending fills now: those overlapping the given tensors, or all (every device)."""
    todo = []
    if tensors is None:
        for pending in _ZERO_FILLS.values():
            todo += pending
            pending.clear()
    else:
        spans = [(t.device.index, t.data_ptr(), t.data_ptr() + t.numel() * t.element_size()) for t in tensors]

        def hit(z):
            a, b = z.data_ptr(), z.data_ptr() + z.numel() * 4
            return any(d == z.device.index and a < e and s < b for d, s, e in spans)
        for pending in _ZERO_FILLS.values():
            todo += [z for z in pending if hit(z)]
            pending[:] = [z for z in pending if not hit(z)]
    for z in todo:
        z.zero_()


def ptr(t, name="tensor", dtype=torch.float32, allow_none=False):
    """Device pointer of a contiguous CUDA tensor of the given dtype (None -> NULL if allowed)."""
    if t is None:
        if allow_none:
            return None
        raise ValueError(f"{name} must not be None")
    if not t.is_cuda:
        raise RuntimeError(f"{name}: indoor_nerf_amd kernels need CUDA (ROCm) tensors, got device {t.device}")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: tensor must be contiguous")
    return c_vp(t.data_ptr())


def ptr_at(t, elems, name="tensor", dtype=torch.float32):
    """ptr(t) advanced by `elems` elements (a row offset inside a contiguous buffer)."""
    p = ptr(t, name, dtype)
    if not 0 <= elems <= t.numel():
        raise ValueError(f"{name}: offset {elems} outside {t.numel()} elements")
    return c_vp((p.value or 0) + elems * t.element_size())


def host_f32(values):
    arr = (ctypes.c_float * len(values))(*[float(v) for v in values])
    return arr


def ptr_array(tensors, name="tables"):
    arr = (c_vp * len(tensors))()
    for i, t in enumerate(tensors):
        arr[i] = ptr(t, f"{name}[{i}]").value
    return arr
