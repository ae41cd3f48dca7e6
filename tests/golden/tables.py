"""Deterministic synthetic inputs shared by the golden-vector generator and the tests.

Test infrastructure only. The golden fixtures must not carry a 64 MiB hash table, so the
"trained-like" table is a closed-form function of (level, row, feature) that numpy reproduces
bit-for-bit anywhere (uint64 integer hashing, then one float64 -> float32 rounding).
"""
import numpy as np

M32 = np.uint64(0xFFFFFFFF)


def _mix32(h):
    h = h & M32
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0x5BD1E995)) & M32
    h ^= h >> np.uint64(15)
    return h


def closed_form_table(n_levels=16, log2_T=19, n_feat=2, scale=0.05, salt=0):
    """[n_levels, 2**log2_T, n_feat] float32 table with values in [-scale, scale)."""
    T = 1 << log2_T
    rows = np.arange(T, dtype=np.uint64)
    out = np.empty((n_levels, T, n_feat), np.float32)
    for lvl in range(n_levels):
        for f in range(n_feat):
            h = rows * np.uint64(2654435761) + np.uint64(lvl * 40503 + f * 9973 + 12345 + salt * 7919)
            h = _mix32(h)
            out[lvl, :, f] = (((h.astype(np.float64) / 4294967296.0) * 2.0 - 1.0) * scale).astype(np.float32)
    return out


def blender_bbox():
    """Scene AABB of the synthetic Blender rig (measured with
    get_bbox3d_for_blenderobj near=2 far=6 on the lego poses)."""
    return (np.array([-3.8502, -3.8500, -3.3230], np.float32),
            np.array([3.8491, 3.8496, 2.6801], np.float32))


def pose_spherical(theta_deg, phi_deg, radius):
    """Camera-to-world of the Blender spiral rig (restated from load_blender.py:12-35)."""
    t = np.eye(4)
    t[2, 3] = radius
    ph = phi_deg / 180.0 * np.pi
    rot_phi = np.array([[1, 0, 0, 0], [0, np.cos(ph), -np.sin(ph), 0],
                        [0, np.sin(ph), np.cos(ph), 0], [0, 0, 0, 1]], np.float64)
    th = theta_deg / 180.0 * np.pi
    rot_theta = np.array([[np.cos(th), 0, -np.sin(th), 0], [0, 1, 0, 0],
                          [np.sin(th), 0, np.cos(th), 0], [0, 0, 0, 1]], np.float64)
    c2w = rot_theta @ rot_phi @ t
    c2w = np.array([[-1, 0, 0, 0], [0, 0, 1, 0], [0, 1, 0, 0], [0, 0, 0, 1]], np.float64) @ c2w
    return c2w.astype(np.float32)


def synthetic_rays(n_rays, H=800, W=800, pose_index=3, seed=0, skip=0):
    """Pinhole rays of one spiral pose, n_rays pixels chosen by a seeded permutation (entries
    skip .. skip + n_rays of it, so two calls with disjoint ranges give disjoint pixels).

    Returns rays_o, rays_d as float32 [n_rays, 3] (d unnormalised, as get_rays makes them)."""
    camera_angle_x = 0.6911112070083618
    focal = 0.5 * W / np.tan(0.5 * camera_angle_x)
    thetas = np.linspace(-180, 180, 101)[:-1]
    c2w = pose_spherical(thetas[pose_index], -30.0, 4.0311)
    rng = np.random.RandomState(seed)
    pix = rng.permutation(H * W)[skip:skip + n_rays]
    i = (pix % W).astype(np.float32)
    j = (pix // W).astype(np.float32)
    dirs = np.stack([(i - 0.5 * W) / focal, -(j - 0.5 * H) / focal, -np.ones_like(i)], -1).astype(np.float32)
    rays_d = (dirs[:, None, :] * c2w[None, :3, :3]).sum(-1).astype(np.float32)
    rays_o = np.broadcast_to(c2w[:3, 3], rays_d.shape).astype(np.float32).copy()
    return rays_o, rays_d


# ---- tiny on-disk datasets for the loader fixtures (F17) ---------------------------------------
BLENDER_SPLITS = {"train": [0.0, 40.0, 95.0], "val": [150.0, -120.0], "test": [10.0, 200.0, -60.0]}


def make_tiny_blender(root, H=10, W=12, seed=0):
    """transforms_{train,val,test}.json + RGBA PNGs (random pixels) in the nerf_synthetic layout."""
    import json
    import os

    from PIL import Image
    rng = np.random.default_rng(seed)
    for split, thetas in BLENDER_SPLITS.items():
        os.makedirs(os.path.join(root, split), exist_ok=True)
        frames = []
        for k, th in enumerate(thetas):
            name = f"./{split}/r_{k}"
            Image.fromarray(rng.integers(0, 256, (H, W, 4), dtype=np.uint8), "RGBA").save(
                os.path.join(root, name + ".png"))
            frames.append({"file_path": name, "transform_matrix": pose_spherical(th, -30.0, 4.0311).tolist()})
        with open(os.path.join(root, f"transforms_{split}.json"), "w") as fp:
            json.dump({"camera_angle_x": 0.6911112070083618, "frames": frames}, fp)


def make_tiny_llff(root, n_views=5, full=(32, 40), factor=4, seed=1):
    """poses_bounds.npy (LLFF [down, right, back] columns + hwf, near/far) + images/ and
    images_<factor>/ RGB PNGs (random pixels; the loader reads images_<factor>/ when present)."""
    import os

    from PIL import Image
    rng = np.random.default_rng(seed)
    H, W = full
    rows = []
    for k in range(n_views):
        yaw = 0.08 * (k - n_views / 2)
        c, s = np.cos(yaw), np.sin(yaw)
        right, up, back = np.array([c, 0, -s]), np.array([0.0, 1.0, 0.0]), np.array([s, 0, c])
        pos = np.array([0.3 * (k - 2), 0.05 * k, 0.1 * k])
        # LLFF stores [down, right, back, position, hwf]
        pose = np.stack([-up, right, back, pos, np.array([H, W, 35.0 + k])], 1)
        rows.append(np.concatenate([pose.reshape(-1), [1.5 + 0.1 * k, 9.0 + k]]))
    np.save(os.path.join(root, "poses_bounds.npy"), np.array(rows, np.float64))
    for sub, (h, w) in (("images", (H, W)), (f"images_{factor}", (H // factor, W // factor))):
        os.makedirs(os.path.join(root, sub), exist_ok=True)
        for k in range(n_views):
            Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8), "RGB").save(
                os.path.join(root, sub, f"IMG_{k:04d}.png"))


# ---- structural-prior inputs (F18) ------------------------------------------------------------
def priors_inputs(n, seed, with_small=True, spread=0.15):
    """A ray batch's depth [n] and normal map [n,3] (unit normals: floor-like, wall-like and random
    directions, plus zero / short normals of transparent rays), and distinct integer pixel
    coordinates [n,2] (train()'s select_coords) — float32 numpy."""
    rng = np.random.default_rng(seed)
    kind = rng.integers(0, 3, n)
    v = rng.normal(size=(n, 3))
    v[kind == 0] = v[kind == 0] * [spread, spread, 1.0]      # near +-z: floor
    v[kind == 1] = v[kind == 1] * [1.0, 1.0, spread * 0.67]  # near horizontal: walls
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    if with_small:
        v[rng.random(n) < 0.08] = 0.0                        # rays with zero weights
        short = rng.random(n) < 0.05
        v[short] *= 0.05
    depth = rng.uniform(0.5, 6.0, n)
    flat = rng.choice(64 * 80, size=n, replace=False)
    coords = np.stack([flat // 80, flat % 80], 1)
    return depth.astype(np.float32), v.astype(np.float32), coords.astype(np.float32)


def make_tiny_scannet(root, scene="scene0000_00", H=12, W=16, seed=2):
    """A ScanNet scene in the layout load_scannet.py reads: nerfstyle_<scene>/transforms_*.json +
    RGB PNGs (OpenCV-convention poses) and scans/<scene>/<scene>_vh_clean.ply (binary little-endian,
    float x y z + uchar colour), with the vertices also saved as vertices.npy (for the golden
    generator's pyvista stand-in)."""
    import json
    import os

    from PIL import Image
    rng = np.random.default_rng(seed)
    sdir = os.path.join(root, "nerfstyle_" + scene)
    for split, n in (("train", 12), ("val", 2), ("test", 3)):
        os.makedirs(os.path.join(sdir, split), exist_ok=True)
        frames = []
        for k in range(n):
            name = f"./{split}/{k}"
            Image.fromarray(rng.integers(0, 256, (H, W, 3), dtype=np.uint8), "RGB").save(
                os.path.join(sdir, name + ".png"))
            pose = np.eye(4)
            a = rng.uniform(0, 2 * np.pi)
            pose[:3, :3] = [[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]]
            pose[:3, 3] = rng.uniform([0, 0, 0.5], [6, 5, 2.5])
            frames.append({"file_path": name, "transform_matrix": pose.tolist()})
        with open(os.path.join(sdir, f"transforms_{split}.json"), "w") as fp:
            json.dump({"camera_angle_x": 1.0175, "frames": frames}, fp)
    mdir = os.path.join(root, "scans", scene)
    os.makedirs(mdir, exist_ok=True)
    verts = rng.uniform([-0.2, -0.1, -0.05], [6.3, 5.2, 3.1], (50, 3)).astype(np.float32)
    cols = rng.integers(0, 256, (50, 3), dtype=np.uint8)
    rec = np.zeros(50, dtype=[("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("red", "u1"), ("green", "u1"),
                              ("blue", "u1")])
    rec["x"], rec["y"], rec["z"] = verts[:, 0], verts[:, 1], verts[:, 2]
    rec["red"], rec["green"], rec["blue"] = cols[:, 0], cols[:, 1], cols[:, 2]
    header = ("ply\nformat binary_little_endian 1.0\nelement vertex 50\nproperty float x\nproperty float y\n"
              "property float z\nproperty uchar red\nproperty uchar green\nproperty uchar blue\n"
              "element face 0\nproperty list uchar int vertex_indices\nend_header\n")
    with open(os.path.join(mdir, f"{scene}_vh_clean.ply"), "wb") as f:
        f.write(header.encode("ascii"))
        f.write(rec.tobytes())
    np.save(os.path.join(mdir, "vertices.npy"), verts)


# ---- procedural scene for the convergence fixture (F19) ----------------------------------------
# Two opaque spheres inside the lego AABB; a ray's target colour is the colour at its first hit
# (inside near..far, in units of the unnormalised ray direction as render_rays samples z), else the
# white background the Blender configs composite onto.
SCENE_SPHERES = (((0.0, 0.0, 0.2), 1.1), ((1.3, 0.7, 0.4), 0.55))


def _sphere_colour(k, n):
    if k == 0:
        return np.clip(0.5 + 0.45 * n, 0.0, 1.0)
    return np.broadcast_to(np.array([0.9, 0.25, 0.1]), n.shape)


def procedural_targets(rays_o, rays_d, near=2.0, far=6.0):
    o, d = rays_o.astype(np.float64), rays_d.astype(np.float64)
    best = np.full(o.shape[0], np.inf)
    rgb = np.ones_like(o)
    for k, (c, r) in enumerate(SCENE_SPHERES):
        oc = o - np.array(c)
        a = (d * d).sum(-1)
        b = 2.0 * (oc * d).sum(-1)
        cc = (oc * oc).sum(-1) - r * r
        disc = b * b - 4 * a * cc
        ok = disc > 0
        t = np.where(ok, (-b - np.sqrt(np.maximum(disc, 0.0))) / (2 * a), np.inf)
        hit = ok & (t >= near) & (t <= far) & (t < best)
        n = (o + d * t[:, None] - np.array(c)) / r
        rgb[hit] = _sphere_colour(k, n[hit])
        best = np.where(hit, t, best)
    return rgb.astype(np.float32)


def convergence_rays(train_poses=(3, 15, 28, 40, 53, 65, 78, 90), n_per_pose=4096, n_eval_per_pose=256,
                     novel_pose=34, n_novel=1024, H=200, W=200):
    """Training pool (rays_o, rays_d, rgb [N,3]): n_per_pose pixels of each of eight spiral poses at
    a 200 x 200 sensor. Held-out set: n_eval_per_pose OTHER pixels of the same poses (interpolation,
    the PSNR the convergence test pins). Novel set: a pose between two training poses."""
    tr = [synthetic_rays(n_per_pose, H=H, W=W, pose_index=p, seed=100 + p) for p in train_poses]
    ev = [synthetic_rays(n_eval_per_pose, H=H, W=W, pose_index=p, seed=100 + p, skip=n_per_pose) for p in train_poses]
    ro, rd = np.concatenate([t[0] for t in tr]), np.concatenate([t[1] for t in tr])
    eo, ed = np.concatenate([t[0] for t in ev]), np.concatenate([t[1] for t in ev])
    no, nd = synthetic_rays(n_novel, H=H, W=W, pose_index=novel_pose, seed=99)
    return ((ro, rd, procedural_targets(ro, rd)), (eo, ed, procedural_targets(eo, ed)),
            (no, nd, procedural_targets(no, nd)))
