"""train()'s per-iteration ray batch on the device (PocketNeRF/run_nerf.py:973-1004).

RaySampler keeps the training images and poses resident in HBM and builds each iteration's
(batch_rays, target_s) with one nerf_sample_rays launch: N_rand distinct pixels of one image
(inside the precrop window for i < precrop_iters), their rays and target colours. The reference
re-uploads the image, builds all H*W rays and draws np.random.choice(H*W, N_rand, replace=False) on
the host every iteration. The image is still chosen with np.random.choice(i_train) like the
reference; the pixel subset comes from a keyed device permutation (same distribution: uniform
without replacement; not the same random stream).
"""
import numpy as np
import torch

from . import _lib
from .render import _draw_seed, camera


def crop_window(H, W, i, precrop_iters=0, precrop_frac=0.5):
    """(r0, c0, h, w) of the pixel grid train() samples from at iteration i (run_nerf.py:984-996):
    the centre crop of linspace(H//2 - dH, H//2 + dH - 1, 2 dH) x (same for W) while
    i < precrop_iters, else the whole image. Cell k of the window is pixel (r0 + k // w, c0 + k % w)."""
    if i < precrop_iters:
        dH = int(H // 2 * precrop_frac)
        dW = int(W // 2 * precrop_frac)
        return H // 2 - dH, W // 2 - dW, 2 * dH, 2 * dW
    return 0, 0, H, W


class RaySampler:
    """Device-resident (images [N,H,W,C], poses [N,3,4]) ray batches for train()'s no_batching path."""

    def __init__(self, images, poses, H, W, K, i_train, N_rand, precrop_iters=0, precrop_frac=0.5, device=None):
        device = torch.device(device or "cuda")
        if torch.is_tensor(images):    # e.g. already resident on the device
            self.images = images.to(device=device, dtype=torch.float32).contiguous()
        else:
            self.images = torch.as_tensor(np.asarray(images), dtype=torch.float32).to(device).contiguous()
        if self.images.dim() != 4 or self.images.shape[-1] < 3:
            raise ValueError("RaySampler: images must be [N, H, W, C>=3]")
        self.poses = np.asarray(poses, dtype=np.float32)[:, :3, :4]
        self.H, self.W, self.K = int(H), int(W), K
        self.i_train = np.asarray(i_train)
        self.N_rand = int(N_rand)
        self.precrop_iters, self.precrop_frac = precrop_iters, precrop_frac
        self.device = device
        self._cams = {}
        self._d_cams = None
        self._device_cams()     # every camera resident now: a captured step reads them (fill)

    def _camera(self, img_i):
        if img_i not in self._cams:
            self._cams[img_i] = camera(self.K, self.poses[img_i])
        return self._cams[img_i]

    def sample(self, i, img_i=None, seed=None, return_coords=False):
        """(batch_rays [2, N_rand, 3], target_s [N_rand, 3]) for iteration i."""
        if img_i is None:
            img_i = int(np.random.choice(self.i_train))
        r0, c0, h, w = crop_window(self.H, self.W, i, self.precrop_iters, self.precrop_frac)
        n = self.N_rand
        rays = torch.empty(2, n, 3, device=self.device, dtype=torch.float32)
        target = torch.empty(n, 3, device=self.device, dtype=torch.float32)
        coords = torch.empty(n, 2, device=self.device, dtype=torch.int32) if return_coords else None
        s0, s1 = _draw_seed() if seed is None else (int(seed), 0)
        img = self.images[img_i]
        _lib.call("nerf_sample_rays", self._camera(img_i), self.H, self.W, r0, c0, h, w, n, 1, s0, s1 + int(i),
                  _lib.ptr(img, "image"), int(img.shape[-1]), _lib.ptr(rays[0], "rays_o"), _lib.ptr(rays[1], "rays_d"),
                  _lib.ptr(target, "target"), _lib.ptr(coords, "coords", dtype=torch.int32, allow_none=True),
                  _lib.stream())
        return (rays, target, coords) if return_coords else (rays, target)

    def crop_key(self, i):
        """The launch structure of iteration i's draw (the precrop window is on or off): part of a
        captured step's re-capture key (graphs.GraphedTrainStep)."""
        return crop_window(self.H, self.W, i, self.precrop_iters, self.precrop_frac)

    def _device_cams(self):
        """Every image's nerf_camera, resident on the device (nerf_sample_rays_sel picks one)."""
        if self._d_cams is None:
            n = self.images.shape[0]
            arr = (_lib.Camera * n)(*[self._camera(k) for k in range(n)])
            raw = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
            self._d_cams = raw.to(self.device)
        return self._d_cams

    def fill(self, i, rays_o, rays_d, target):
        """Iteration i's batch into the caller's buffers (rays_o, rays_d [N_rand, 3], target
        [N_rand, 3]): the image with np.random.choice(i_train) and the pixels from a fresh seed, as
        sample() draws them. While a training step is captured (graphs.GraphedTrainStep(sampler=...))
        the (image, seed, offset) triple is a per-replay slot (graphs.StepScalars) that the captured
        nerf_sample_rays_sel launch reads, so every replay trains on a new batch (run_nerf.py:975-1004);
        the draws happen in the same order as eagerly, so the replayed batches equal the eager ones."""
        import weakref
        from . import graphs
        r0, c0, h, w = crop_window(self.H, self.W, i, self.precrop_iters, self.precrop_frac)
        n = self.N_rand
        for t, name in ((rays_o, "rays_o"), (rays_d, "rays_d"), (target, "target")):
            if tuple(t.shape) != (n, 3):
                raise ValueError(f"RaySampler.fill: {name} must be [{n}, 3], got {tuple(t.shape)}")
        sc = graphs.active()
        C = int(self.images.shape[-1])
        if sc is None:
            img_i = int(np.random.choice(self.i_train))
            s0, s1 = _draw_seed()
            img = self.images[img_i]
            _lib.call("nerf_sample_rays", self._camera(img_i), self.H, self.W, r0, c0, h, w, n, 1, s0, s1 + int(i),
                      _lib.ptr(img, "image"), C, _lib.ptr(rays_o, "rays_o"), _lib.ptr(rays_d, "rays_d"),
                      _lib.ptr(target, "target"), None, _lib.stream())
            return
        off, ptr = sc.alloc_i64(3)
        sc_ref = weakref.ref(sc)

        def fill(hi, hf, off=off):
            img_i = int(np.random.choice(self.i_train))
            s0, s1 = _draw_seed()
            hi[off], hi[off + 1], hi[off + 2] = img_i, s0, s1 + int(sc_ref().step)
        sc.add_filler(fill)
        _lib.call("nerf_sample_rays_sel", _lib.ptr(self._device_cams(), "cams", dtype=torch.uint8),
                  _lib.ptr(self.images, "images"), int(self.images.shape[0]), self.H, self.W, C, r0, c0, h, w, n,
                  _lib.c_vp(ptr), _lib.ptr(rays_o, "rays_o"), _lib.ptr(rays_d, "rays_d"), _lib.ptr(target, "target"),
                  None, _lib.stream())
