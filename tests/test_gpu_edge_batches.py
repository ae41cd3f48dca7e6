"""Degenerate batch sizes through the product path (SURVEY §8(c) edge cases), on the HIP library.

* an empty ray batch through `render_rays` (coarse + fine, training perturbation) and the backward
  of a loss over its outputs: the reference's torch ops accept zero rays (run_nerf.py:414-549), so
  the drop-in must too — every C-ABI entry returns before launching, the outputs are empty with the
  reference's trailing shapes, and the parameter gradients stay zero;
* a single ray, and a ragged 37-ray batch (no multiple of a wave, a 32-point MLP tile or a 512-point
  bin chunk), against the same rays rendered inside a 4096-ray batch: per-ray results do not depend
  on the batch around them (eval mode: deterministic sampling, no noise), so the outputs must be
  bit-identical to the rows of the large batch.
(`render` itself raises on zero rays, as the reference's does: its batchify_rays leaves no outputs.)
"""
import pytest
import torch

from tables import blender_bbox, synthetic_rays

pytestmark = pytest.mark.gpu


def _model(nerf, gpu):
    lo, hi = blender_bbox()
    args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), finest_res=512, N_samples=64,
                          N_importance=128, white_bkgd=True)
    torch.manual_seed(0)
    kw_train, kw_test, _, grad_vars, _ = nerf.create_nerf(args, device=gpu)
    emb = kw_train["embed_fn"]
    with torch.no_grad():
        g = torch.Generator().manual_seed(5)
        for e in emb.embeddings:
            e.weight.copy_((torch.rand(e.weight.shape, generator=g) * 2 - 1) * 0.05)
    kw_test.update(near=2.0, far=6.0)
    return kw_train, kw_test, grad_vars


def test_render_rays_empty_batch(nerf, gpu):
    kw_train, _, grad_vars = _model(nerf, gpu)
    kw = {k: v for k, v in kw_train.items() if k not in ("ndc", "use_viewdirs", "near", "far")}
    rays = torch.empty(0, 11, device=gpu)
    ret = nerf.render_rays(rays, **kw)
    torch.cuda.synchronize()
    assert ret["rgb_map"].shape == (0, 3) and ret["rgb0"].shape == (0, 3)
    assert ret["depth_map"].shape == (0,) and ret["acc_map"].shape == (0,) and ret["z_std"].shape == (0,)
    assert ret["pts"].shape == (0, 192, 3)
    for p in grad_vars:
        p.grad = None
    loss = ret["rgb_map"].sum() + ret["rgb0"].sum() + ret["sparsity_loss"].sum()
    loss.backward()
    torch.cuda.synchronize()
    for p in grad_vars:
        assert p.grad is None or not p.grad.any().item()


@pytest.mark.parametrize("R", [1, 37])
def test_render_rays_small_batches_match_large(nerf, gpu, R):
    _, kw_test, _ = _model(nerf, gpu)
    ro, rd = synthetic_rays(4096, seed=4)
    ro, rd = torch.from_numpy(ro).to(gpu), torch.from_numpy(rd).to(gpu)
    with torch.no_grad():
        ref = nerf.render(800, 800, None, rays=(ro, rd), **kw_test)
        got = nerf.render(800, 800, None, rays=(ro[:R].contiguous(), rd[:R].contiguous()), **kw_test)
    torch.cuda.synchronize()
    for i, k in enumerate(("rgb_map", "depth_map", "acc_map")):
        assert got[i].shape[0] == R
        assert torch.equal(got[i], ref[i][:R]), k
    for k in ("rgb0", "z_std", "pts"):
        assert torch.equal(got[3][k], ref[3][k][:R]), k
