"""Scene bounding boxes for the hash grid (setup-time host code, run once per dataset).

API mirror of PocketNeRF/utils.py:27-92 (get_bbox3d_for_blenderobj, get_bbox3d_for_llff) with the
ray helpers they use from PocketNeRF/ray_utils.py:5-100 (get_ray_directions, get_rays,
get_ndc_rays). Same fp32 arithmetic as the reference: the box is the min/max over the four image
corners' rays at near/far of every camera, padded by 1.0 (Blender) or (0.1, 0.1, 1e-4) (LLFF, in
NDC space). Only the four corner pixels are evaluated (the reference builds all H*W directions and
reads those four rows). These return CPU tensors; HashEmbedder reads them once at construction.
"""
import numpy as np
import torch


def _corner_directions(H, W, focal):
    """get_ray_directions (ray_utils.py:5-28) at pixels 0, W-1, H*W-W, H*W-1 (row-major)."""
    i = torch.tensor([0.0, W - 1.0, 0.0, W - 1.0])
    j = torch.tensor([0.0, 0.0, H - 1.0, H - 1.0])
    return torch.stack([(i - W / 2) / focal, -(j - H / 2) / focal, -torch.ones_like(i)], -1)


def get_rays_world(directions, c2w):
    """ray_utils.get_rays (:31-56): normalised world directions, camera origin."""
    rays_d = directions @ c2w[:3, :3].T
    rays_d = rays_d / torch.norm(rays_d, dim=-1, keepdim=True)
    rays_o = c2w[:3, -1].expand(rays_d.shape)
    return rays_o.reshape(-1, 3), rays_d.reshape(-1, 3)


def get_ndc_rays(H, W, focal, near, rays_o, rays_d):
    """ray_utils.get_ndc_rays (:59-100)."""
    t = -(near + rays_o[..., 2]) / rays_d[..., 2]
    rays_o = rays_o + t[..., None] * rays_d
    ox_oz = rays_o[..., 0] / rays_o[..., 2]
    oy_oz = rays_o[..., 1] / rays_o[..., 2]
    o0 = -1. / (W / (2. * focal)) * ox_oz
    o1 = -1. / (H / (2. * focal)) * oy_oz
    o2 = 1. + 2. * near / rays_o[..., 2]
    d0 = -1. / (W / (2. * focal)) * (rays_d[..., 0] / rays_d[..., 2] - ox_oz)
    d1 = -1. / (H / (2. * focal)) * (rays_d[..., 1] / rays_d[..., 2] - oy_oz)
    d2 = 1 - o2
    return torch.stack([o0, o1, o2], -1), torch.stack([d0, d1, d2], -1)


def _bounds(points):
    lo = [100.0, 100.0, 100.0]
    hi = [-100.0, -100.0, -100.0]
    for pt in points:
        for a in range(3):
            v = float(pt[a])
            lo[a] = min(lo[a], v)
            hi[a] = max(hi[a], v)
    return lo, hi


def get_bbox3d_for_blenderobj(camera_transforms, H, W, near=2.0, far=6.0):
    """utils.py:27-58: camera_transforms is the transforms_*.json dict."""
    camera_angle_x = float(camera_transforms["camera_angle_x"])
    focal = 0.5 * W / np.tan(0.5 * camera_angle_x)
    dirs = _corner_directions(H, W, focal)
    pts = []
    for frame in camera_transforms["frames"]:
        c2w = torch.tensor(frame["transform_matrix"], dtype=torch.float32)
        ro, rd = get_rays_world(dirs, c2w)
        for k in range(4):
            pts += [ro[k] + near * rd[k], ro[k] + far * rd[k]]
    lo, hi = _bounds(pts)
    return torch.tensor(lo) - torch.tensor([1.0, 1.0, 1.0]), torch.tensor(hi) + torch.tensor([1.0, 1.0, 1.0])


def get_bbox3d_for_llff(poses, hwf, near=0.0, far=1.0):
    """utils.py:61-92: the box of the NDC rays (near plane 1) of every pose's image corners."""
    H, W, focal = hwf
    H, W = int(H), int(W)
    dirs = _corner_directions(H, W, focal)
    pts = []
    for pose in torch.tensor(np.asarray(poses), dtype=torch.float32):
        ro, rd = get_rays_world(dirs, pose)
        ro, rd = get_ndc_rays(H, W, focal, 1.0, ro, rd)
        for k in range(4):
            pts += [ro[k] + near * rd[k], ro[k] + far * rd[k]]
    lo, hi = _bounds(pts)
    return torch.tensor(lo) - torch.tensor([0.1, 0.1, 0.0001]), torch.tensor(hi) + torch.tensor([0.1, 0.1, 0.0001])
