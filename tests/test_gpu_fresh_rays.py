"""A new ray batch every iteration inside the captured training step (train()'s no_batching draw,
run_nerf.py:975-1004; bench.py's fresh-rays leg): nerf_sample_rays_sel (image, seed and offset read
on the device) against nerf_sample_rays with the same draw, and GraphedTrainStep(sampler=...) against
the same iterations launched eagerly (the sampler's draws happen in the same order in both)."""
import numpy as np
import pytest
import torch

from tables import blender_bbox

pytestmark = pytest.mark.gpu


def _rig(n_img, H, W, seed=0):
    from indoor_nerf_amd.synthetic import CAMERA_ANGLE_X, pose_spherical
    focal = 0.5 * W / np.tan(0.5 * CAMERA_ANGLE_X)
    K = np.array([[focal, 0, 0.5 * W], [0, focal, 0.5 * H], [0, 0, 1]])
    poses = np.stack([pose_spherical(t, -30.0, 4.0311) for t in np.linspace(-180, 180, n_img + 1)[:-1]])
    images = np.random.RandomState(seed).rand(n_img, H, W, 3).astype(np.float32)
    return images, poses, K


@pytest.mark.parametrize("crop", [False, True], ids=["whole", "precrop"])
def test_sample_rays_sel_matches_host_draw(nerf, gpu, crop):
    from indoor_nerf_amd import _lib
    H, W, n = 60, 80, 1000
    images, poses, K = _rig(5, H, W)
    s = nerf.RaySampler(images, poses, H, W, K, np.arange(5), n, precrop_iters=10 if crop else 0, device=gpu)
    r0, c0, h, w = nerf.crop_window(H, W, 3, s.precrop_iters, s.precrop_frac)
    for img_i, seed, off in ((0, 11, 3), (4, 2 ** 61 + 7, 12345), (2, 5, 0), (7, 9, 1)):   # 7: taken mod 5
        want, want_t, want_c = s.sample(3, img_i=img_i % 5, seed=seed, return_coords=True) if off == 3 + 0 else \
            (None, None, None)
        # host-argument launch with this (image, seed, offset)
        ro, rd, tg = (torch.empty(n, 3, device=gpu) for _ in range(3))
        co = torch.empty(n, 2, device=gpu, dtype=torch.int32)
        img = s.images[img_i % 5]
        _lib.call("nerf_sample_rays", s._camera(img_i % 5), H, W, r0, c0, h, w, n, 1, seed, off, _lib.ptr(img), 3,
                  _lib.ptr(ro), _lib.ptr(rd), _lib.ptr(tg), _lib.ptr(co, dtype=torch.int32), _lib.stream())
        sel = torch.tensor([img_i, seed, off], dtype=torch.int64, device=gpu)
        ro2, rd2, tg2 = (torch.empty(n, 3, device=gpu) for _ in range(3))
        co2 = torch.empty(n, 2, device=gpu, dtype=torch.int32)
        _lib.call("nerf_sample_rays_sel", _lib.ptr(s._device_cams(), dtype=torch.uint8), _lib.ptr(s.images), 5, H, W,
                  3, r0, c0, h, w, n, _lib.ptr(sel, dtype=torch.int64), _lib.ptr(ro2), _lib.ptr(rd2), _lib.ptr(tg2),
                  _lib.ptr(co2, dtype=torch.int32), _lib.stream())
        torch.cuda.synchronize()
        for a, b in ((ro, ro2), (rd, rd2), (tg, tg2), (co, co2)):
            assert torch.equal(a, b)
        c = co2.cpu().numpy()
        assert len(np.unique(c[:, 0] * W + c[:, 1])) == n
        assert c[:, 0].min() >= r0 and c[:, 0].max() < r0 + h and c[:, 1].min() >= c0 and c[:, 1].max() < c0 + w
        np.testing.assert_array_equal(tg2.cpu().numpy(), images[img_i % 5][c[:, 0], c[:, 1]])
        if want is not None:
            assert torch.equal(want[0], ro) and torch.equal(want[1], rd) and torch.equal(want_t, tg)


def _train(nerf, gpu, graphed, steps=6, R=1024):
    from indoor_nerf_amd.graphs import GraphedTrainStep
    lo, hi = blender_bbox()
    args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), finest_res=1024, N_samples=64,
                          N_importance=128, white_bkgd=True, perturb=1.0, tv_loss_weight=1e-6)
    torch.manual_seed(0)
    kw, _, _, grad_vars, opt = nerf.create_nerf(args, device=gpu)
    kw.update(near=2.0, far=6.0)
    H = W = 100
    images, poses, K = _rig(8, H, W, seed=3)
    np.random.seed(17)
    nerf.manual_seed(5)
    sampler = nerf.RaySampler(images, poses, H, W, K, np.arange(8), R, device=gpu)
    params = grad_vars + list(kw["embed_fn"].parameters())
    arena = nerf.GradArena(params, defer_tables=True)
    rays = (torch.empty(R, 3, device=gpu), torch.empty(R, 3, device=gpu))
    target = torch.empty(R, 3, device=gpu)
    st = GraphedTrainStep(rays, target, kw, opt, args, H=H, W=W, tv_generator=torch.Generator().manual_seed(7),
                          zero_grad=arena.zero_, sampler=sampler)
    losses, batches = [], []
    for it in range(1, steps + 1):
        loss, _ = st(it) if graphed else st.eager_step(it)
        torch.cuda.synchronize()
        losses.append(float(loss))
        batches.append((rays[0].clone(), rays[1].clone(), target.clone()))
    return losses, batches, st.captures


def test_graphed_fresh_rays_match_eager(nerf, gpu):
    """GraphedTrainStep(sampler=RaySampler): the captured step draws each replay's batch on the device
    from the replay's slot; the batches equal the eager draws bit for bit (same host draw order) and
    the losses follow the eager run (HIP-graph iteration tolerance); every batch differs."""
    la, ba, caps = _train(nerf, gpu, True)
    lb, bb, _ = _train(nerf, gpu, False)
    assert caps == 1
    for k, (x, y) in enumerate(zip(ba, bb)):
        for a, b in zip(x, y):
            assert torch.equal(a, b), f"batch {k}"
    assert all(not torch.equal(ba[k][1], ba[k + 1][1]) for k in range(len(ba) - 1))
    np.testing.assert_allclose(la, lb, rtol=1e-5)
