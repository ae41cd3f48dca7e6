"""render_path (run_nerf.py:154-215) on the HIP path: full frames from camera poses, per-view
PSNR against ground truth, normalised depth, saved PNGs; the frames agree with the CPU oracle's
render_rays on the same rays (eval mode: deterministic importance sampling, no noise).

Tolerance: rgb <= 1e-3 abs (the fine-pass bar of DESIGN.md §2: sample_pdf's thin-bin rule), PSNR
equal to -10 log10(mse) of the returned frame (same numbers, host-side)."""
import os

import numpy as np
import pytest
import torch

from tables import blender_bbox

pytestmark = pytest.mark.gpu


def test_render_path_vs_oracle(nerf, gpu, oracle, tmp_path):
    lo, hi = blender_bbox()
    args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), finest_res=512, N_samples=32,
                          N_importance=32, white_bkgd=True)
    torch.manual_seed(0)
    kw_train, kw_test, _, _, _ = nerf.create_nerf(args, device=gpu)
    kw_test.update(near=2.0, far=6.0)
    emb = kw_test["embed_fn"]
    with torch.no_grad():
        g = torch.Generator().manual_seed(3)
        for e in emb.embeddings:
            e.weight.copy_((torch.rand(e.weight.shape, generator=g) * 2 - 1) * 0.05)
    for m in (kw_test["network_fn"], kw_test["network_fine"], emb):
        m.eval()
    H, W = 12, 16
    focal = 0.5 * W / np.tan(0.5 * 0.6911112070083618)
    K = np.array([[focal, 0, 0.5 * W], [0, focal, 0.5 * H], [0, 0, 1]])
    poses = torch.stack([nerf.pose_spherical(a, -30.0, 4.0) for a in (-40.0, 75.0)])
    gt = np.random.default_rng(0).random((2, H, W, 3)).astype(np.float32)
    rgbs, depths = nerf.render_path(poses, [H, W, focal], K, 1024, kw_test, gt_imgs=gt, savedir=str(tmp_path))
    assert rgbs.shape == (2, H, W, 3) and depths.shape == (2, H, W)
    # saved views and the PSNR pickle
    assert os.path.exists(tmp_path / "000.png") and os.path.exists(tmp_path / "001_depth.png")
    psnrs = [-10. * np.log10(np.mean(np.square(rgbs[i] - gt[i]))) for i in range(2)]
    assert any(f.startswith("test_psnrs_avg{:0.2f}".format(sum(psnrs) / 2)) for f in os.listdir(tmp_path))
    # oracle on the same rays
    cw = {k: v.detach().cpu() for k, v in kw_test["network_fn"].state_dict().items()}
    fw = {k: v.detach().cpu() for k, v in kw_test["network_fine"].state_dict().items()}
    tabs = [e.weight.detach().cpu() for e in emb.embeddings]
    for i in range(2):
        ro, rd = nerf.get_rays_np(H, W, K, poses[i].numpy())
        ro_t = torch.from_numpy(np.ascontiguousarray(ro.reshape(-1, 3), np.float32))
        rd_t = torch.from_numpy(np.ascontiguousarray(rd.reshape(-1, 3), np.float32))
        ref = oracle.render_rays(ro_t, rd_t, oracle.viewdirs_of(rd_t), 2.0, 6.0, cw, fw, tabs, torch.from_numpy(lo),
                                 torch.from_numpy(hi), oracle.level_resolutions(16, 512), n_samples=32,
                                 n_importance=32, perturb=0.0)
        err = np.abs(rgbs[i].reshape(-1, 3) - ref["rgb_map"].numpy()).max()
        assert err < 1e-3, (i, err)
        d = (ref["depth_map"].numpy() - 2.0) / 4.0
        np.testing.assert_allclose(depths[i].reshape(-1), d, rtol=1e-3, atol=1e-3)
