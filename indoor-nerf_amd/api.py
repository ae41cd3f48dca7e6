"""Public API of indoor_nerf_amd: the reference's render_rays-path names (PocketNeRF/run_nerf.py,
run_nerf_helpers.py, hash_encoding.py, radam.py, loss.py) backed by libnerfhip."""
from . import _lib
from .dist import GradArena, ShardedOptimizer, broadcast_params, init_process_group, shard
from .field import NeRFSmall, active_points, batchify, deterministic, run_network, set_active_points, set_deterministic
from .hashgrid import HashEmbedder, SHEncoder, fused_table_step_enabled, level_resolutions, set_fused_table_step
from .losses import sigma_sparsity_loss, total_variation_all, total_variation_loss, train_loss
from .model import (acaq_quantizers, acaq_update, create_nerf, make_args, save_checkpoint, structural_overfit_update,
                    train_step)
from .optim import RAdam
from .quantization import FakeQuantizer, LearnedBitwidthQuantizer, PassthroughQuantizer, calculate_fqr
from .rays import RaySampler, crop_window
from .scene import get_bbox3d_for_blenderobj, get_bbox3d_for_llff
from .render import (batchify_rays, camera, check_numerics, set_debug, get_rays, get_rays_np, img2mse, manual_seed, mse2psnr, ndc_rays, raw2outputs,
                     render, render_path, render_rays, sample_pdf, set_coarse_reuse, coarse_reuse, to8b,
                     set_fused_coarse_sampler, fused_coarse_sampler, set_batched_composite_bwd,
                     batched_composite_bwd, set_sh_rows, sh_rows)
from .data import load_blender_data, load_llff_data, load_scannet_data, pose_spherical
from .priors import (ManhattanFrameEstimator, SemanticPlaneDetector, combine_structural_losses_v2, manhattan_sdf_loss,
                     spatial_normal_consistency_loss, structured_planarity_loss)

__all__ = ["HashEmbedder", "SHEncoder", "NeRFSmall", "RAdam", "run_network", "batchify", "batchify_rays", "render",
           "render_rays", "raw2outputs", "sample_pdf", "get_rays", "get_rays_np", "ndc_rays", "img2mse", "mse2psnr",
           "to8b", "create_nerf", "make_args", "save_checkpoint", "train_step", "total_variation_loss",
           "total_variation_all", "train_loss", "sigma_sparsity_loss", "level_resolutions", "GradArena", "ShardedOptimizer", "init_process_group",
           "shard", "broadcast_params", "manual_seed", "load_library", "LearnedBitwidthQuantizer", "FakeQuantizer",
           "PassthroughQuantizer", "calculate_fqr", "acaq_update", "acaq_quantizers", "structural_overfit_update", "RaySampler", "crop_window", "camera",
           "get_bbox3d_for_blenderobj", "get_bbox3d_for_llff", "render_path", "load_blender_data", "load_llff_data",
           "pose_spherical", "load_scannet_data", "ManhattanFrameEstimator", "SemanticPlaneDetector",
           "combine_structural_losses_v2", "manhattan_sdf_loss", "spatial_normal_consistency_loss",
           "structured_planarity_loss", "set_deterministic", "deterministic", "check_numerics", "set_debug",
           "set_coarse_reuse", "coarse_reuse", "set_fused_coarse_sampler", "fused_coarse_sampler",
           "set_batched_composite_bwd", "batched_composite_bwd", "set_sh_rows", "sh_rows", "set_active_points", "active_points", "set_fused_table_step",
           "fused_table_step_enabled"]


def load_library():
    """Load libnerfhip.so (raises if it is missing)."""
    return _lib.load()
