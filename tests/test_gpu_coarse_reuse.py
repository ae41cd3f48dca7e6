"""The premise of DESIGN §8.5 (reusing the coarse pass's encoding in the fine pass), checked on the
HIP path: the fine point set of every ray contains each coarse point bit for bit, at the coarse
depth's rank in the merged sorted depths (run_nerf.py:512-513: torch.sort(cat([z_vals, z_samples]))
then rays_o + rays_d * z), and the hash features of those fine points equal the coarse pass's bit for
bit (one embedder serves both networks, run_nerf.py:225,275). Training perturbation through the
reference's pytest uniforms, so the coarse-only and the full call draw the same stratified depths."""
import pytest
import torch

from tables import blender_bbox, synthetic_rays

pytestmark = pytest.mark.gpu


def test_fine_set_contains_coarse_points_bitwise(nerf, gpu):
    lo, hi = blender_bbox()
    args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), finest_res=1024, N_samples=64,
                          N_importance=128, white_bkgd=True)
    torch.manual_seed(0)
    kw_train, _, _, _, _ = nerf.create_nerf(args, device=gpu)
    emb = kw_train["embed_fn"]
    with torch.no_grad():
        g = torch.Generator().manual_seed(7)
        for e in emb.embeddings:
            e.weight.copy_((torch.rand(e.weight.shape, generator=g) * 2 - 1) * 0.05)
    kw = {k: v for k, v in kw_train.items() if k not in ("ndc", "use_viewdirs", "near", "far")}
    R = 512
    ro, rd = synthetic_rays(R, seed=9)
    ro, rd = torch.from_numpy(ro).to(gpu), torch.from_numpy(rd).to(gpu)
    vd = rd / torch.norm(rd, dim=-1, keepdim=True)
    rays = torch.cat([ro, rd, torch.full((R, 1), 2.0, device=gpu), torch.full((R, 1), 6.0, device=gpu), vd], -1)
    with torch.no_grad():
        coarse = nerf.render_rays(rays, **(kw | {"N_importance": 0}), pytest=True)["pts"]          # [R, 64, 3]
        fine = nerf.render_rays(rays, **kw, pytest=True)["pts"]                                    # [R, 192, 3]
    torch.cuda.synchronize()
    assert coarse.shape == (R, 64, 3) and fine.shape == (R, 192, 3)
    eq = (fine[:, None, :, :] == coarse[:, :, None, :]).all(-1)                                    # [R, 64, 192]
    assert eq.any(-1).all().item(), "a coarse point is missing from its ray's fine set"
    # the first match of coarse point j sits at or after rank j, in increasing order along the ray
    pos = eq.float().argmax(-1)                                                                    # [R, 64]
    assert (pos[:, 1:] > pos[:, :-1]).all().item()
    assert (pos >= torch.arange(64, device=gpu)).all().item()
    picked = torch.gather(fine, 1, pos[..., None].expand(-1, -1, 3))
    assert torch.equal(picked, coarse)
    with torch.no_grad():
        f_coarse = emb(coarse.reshape(-1, 3))
        f_fine = emb(picked.reshape(-1, 3).contiguous())
    torch.cuda.synchronize()
    for a, b in zip(f_coarse, f_fine):   # (features [P, 32], keep mask)
        assert torch.equal(a, b)
