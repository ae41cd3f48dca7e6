"""Synthetic Blender-rig inputs for bench.py and smoke tests (no dataset access on the GPU box).

The lego rig of SURVEY.md §8(d): spiral poses pose_spherical(theta, -30, 4.0311)
(PocketNeRF/load_blender.py:12-35), camera_angle_x = 0.6911112070083618, near 2, far 6, and the
scene AABB get_bbox3d_for_blenderobj returns for it (utils.py:27-58)."""
import numpy as np

CAMERA_ANGLE_X = 0.6911112070083618
BLENDER_BBOX = ((-3.8502, -3.8500, -3.3230), (3.8491, 3.8496, 2.6801))


def pose_spherical(theta_deg, phi_deg, radius):
    t = np.eye(4)
    t[2, 3] = radius
    ph, th = np.deg2rad(phi_deg), np.deg2rad(theta_deg)
    rot_phi = np.array([[1, 0, 0, 0], [0, np.cos(ph), -np.sin(ph), 0], [0, np.sin(ph), np.cos(ph), 0], [0, 0, 0, 1]])
    rot_theta = np.array([[np.cos(th), 0, -np.sin(th), 0], [0, 1, 0, 0], [np.sin(th), 0, np.cos(th), 0], [0, 0, 0, 1]])
    c2w = np.array([[-1, 0, 0, 0], [0, 0, 1, 0], [0, 1, 0, 0], [0, 0, 0, 1]]) @ (rot_theta @ rot_phi @ t)
    return c2w.astype(np.float32)


def blender_rays(n_rays, H=800, W=800, pose_index=3, seed=0):
    """n_rays pixels of one spiral pose (seeded permutation); returns rays_o, rays_d [n,3] float32."""
    focal = 0.5 * W / np.tan(0.5 * CAMERA_ANGLE_X)
    c2w = pose_spherical(np.linspace(-180, 180, 101)[:-1][pose_index], -30.0, 4.0311)
    pix = np.random.RandomState(seed).permutation(H * W)[:n_rays]
    i, j = (pix % W).astype(np.float32), (pix // W).astype(np.float32)
    dirs = np.stack([(i - 0.5 * W) / focal, -(j - 0.5 * H) / focal, -np.ones_like(i)], -1).astype(np.float32)
    rays_d = (dirs[:, None, :] * c2w[None, :3, :3]).sum(-1).astype(np.float32)
    rays_o = np.broadcast_to(c2w[:3, 3], rays_d.shape).astype(np.float32).copy()
    return rays_o, rays_d


def blender_bbox():
    return (np.array(BLENDER_BBOX[0], np.float32), np.array(BLENDER_BBOX[1], np.float32))


# Forward-facing LLFF rig (fern at factor 8: 504 x 378, SURVEY.md §8(d) "Fern: NDC, near 0 far 1"):
# three cameras looking down -z with small yaw / translation (tests/golden/make_golden.py llff_rig).
LLFF_HWF = (378, 504, 407.5)


def llff_poses():
    poses = []
    for yaw, tx in ((-4.0, -0.08), (0.0, 0.0), (5.0, 0.1)):
        a = np.deg2rad(yaw)
        R = np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]])
        poses.append(np.concatenate([R, np.array([[tx], [0.02 * yaw], [0.0]])], 1))
    return np.array(poses, np.float32)


def llff_rays(n_rays, pose_index=1, seed=0):
    """n_rays world-space rays of one LLFF camera (NDC conversion happens in render(ndc=True)).
    Returns rays_o, rays_d [n,3] float32 and (H, W, K) with K float64 as train() builds it."""
    H, W, focal = LLFF_HWF
    K = np.array([[focal, 0, 0.5 * W], [0, focal, 0.5 * H], [0, 0, 1]])
    c2w = llff_poses()[pose_index]
    pix = np.random.RandomState(seed).permutation(H * W)[:n_rays]
    i, j = (pix % W).astype(np.float32), (pix // W).astype(np.float32)
    dirs = np.stack([(i - K[0][2]) / K[0][0], -(j - K[1][2]) / K[1][1], -np.ones_like(i)], -1).astype(np.float32)
    rays_d = (dirs[:, None, :] * c2w[None, :3, :3]).sum(-1).astype(np.float32)
    rays_o = np.broadcast_to(c2w[:3, 3], rays_d.shape).astype(np.float32).copy()
    return rays_o, rays_d, (H, W, K)


def llff_bbox():
    """NDC box of the rig (scene.get_bbox3d_for_llff, utils.py:61-92)."""
    from .scene import get_bbox3d_for_llff
    lo, hi = get_bbox3d_for_llff(llff_poses(), LLFF_HWF, near=0.0, far=1.0)
    return lo.numpy(), hi.numpy()


# ScanNet-like indoor scene (configs/scannet_scene0000.txt: near 0.1, far 10): a 6 x 5 x 3 m room,
# the box the loader derives from the mesh bounds padded by 1 (load_scannet.py:100-104), and
# 640 x 480 cameras (ScanNet's colour intrinsics at that size: focal ~ 577.9) inside it.
SCANNET_BBOX = ((-1.0, -1.0, -1.0), (7.0, 6.0, 4.0))


def scannet_bbox():
    return (np.array(SCANNET_BBOX[0], np.float32), np.array(SCANNET_BBOX[1], np.float32))


def scannet_rays(n_rays, seed=0, H=480, W=640, focal=577.9):
    """n_rays rays of one camera standing in the room and looking horizontally, with the integer
    pixel coordinates they came from ([n, 2] row, col: train()'s select_coords)."""
    rng = np.random.default_rng(seed)
    yaw = rng.uniform(0, 2 * np.pi)
    c2w = np.eye(4, dtype=np.float64)
    # camera looks along -z_cam; world up is +z
    fwd = np.array([np.cos(yaw), np.sin(yaw), 0.0])
    right = np.array([np.sin(yaw), -np.cos(yaw), 0.0])
    up = np.array([0.0, 0.0, 1.0])
    c2w[:3, 0], c2w[:3, 1], c2w[:3, 2] = right, up, -fwd
    c2w[:3, 3] = rng.uniform([1.5, 1.5, 1.2], [4.5, 3.5, 1.8])
    flat = rng.choice(H * W, size=n_rays, replace=False)
    i, j = (flat % W).astype(np.float32), (flat // W).astype(np.float32)
    dirs = np.stack([(i - W * .5) / focal, -(j - H * .5) / focal, -np.ones_like(i)], -1)
    rays_d = (dirs @ c2w[:3, :3].T).astype(np.float32)
    rays_o = np.broadcast_to(c2w[:3, 3], rays_d.shape).astype(np.float32).copy()
    coords = np.stack([j, i], -1).astype(np.float32)
    return rays_o, rays_d, coords
