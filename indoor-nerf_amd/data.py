"""Dataset loaders on the caller side of the path: Blender (nerf_synthetic) and
LLFF (forward-facing) scenes, with the reference's return values so that train()/render_path()
consume them unchanged.

  load_blender_data  PocketNeRF/load_blender.py:38-91  (+ pose_spherical :11-35)
  load_llff_data     PocketNeRF/load_llff.py:244-319   (+ _load_data :63-123, poses_avg,
                     recenter_poses, render_path_spiral, spherify_poses :126-241)

Host-side numpy/PIL code, run once per dataset; the images end up as one [N, H, W, C] fp32 tensor
in HBM (rays.RaySampler). Deviations, all outside the numerical path:
  * image decoding uses PIL (imageio is not in this image); 8-bit PNG/JPEG decode identically;
  * the reference's _minify shells out to ImageMagick `mogrify` to build images_<factor>/ when it
    is missing. Here an existing images_<factor>/ is used exactly as the reference does, and a
    missing one is produced in memory with PIL's box filter (mogrify's resampling filter is not
    reproducible without ImageMagick; nothing is written to the dataset directory);
  * half_res Blender images: cv2.resize(INTER_AREA) at exactly 2x is the 2x2 box mean, computed
    here with numpy (fp32), returned as float64 like the reference's np.zeros buffer.
"""
import json
import os

import numpy as np
import torch
from PIL import Image

from .scene import get_bbox3d_for_blenderobj, get_bbox3d_for_llff

_IMG_EXT = ("JPG", "jpg", "png")


def _imread(path):
    """imageio.imread: uint8 array [H, W, C] (PNG gamma chunks ignored, as ignoregamma=True)."""
    with Image.open(path) as im:
        return np.asarray(im).copy()


# ---------------------------------------------------------------------------------- Blender
def _translate_z(t):
    m = torch.eye(4)
    m[2, 3] = t
    return m


def _rotation(axes, ang):
    """4x4 rotation in the plane of axes (a, b): [a,a] = [b,b] = cos, [a,b] = -sin, [b,a] = sin,
    the layout of load_blender.py's rot_phi (a, b = 1, 2) and rot_theta (0, 2); entries from
    np.cos/np.sin in float64, stored as float32 like torch.Tensor(...)."""
    a, b = axes
    m = torch.eye(4)
    c, s = float(np.cos(ang)), float(np.sin(ang))
    m[a, a] = c
    m[b, b] = c
    m[a, b] = -s
    m[b, a] = s
    return m


_BLENDER_FLIP = torch.tensor([[-1., 0., 0., 0.], [0., 0., 1., 0.], [0., 1., 0., 0.], [0., 0., 0., 1.]])


def pose_spherical(theta, phi, radius):
    """Camera-to-world of a camera on a sphere (load_blender.py:30-35), fp32, applied in the
    reference's order: translate, tilt by phi, turn by theta, swap to the Blender axes."""
    c2w = _translate_z(radius)
    c2w = _rotation((1, 2), phi / 180. * np.pi) @ c2w
    c2w = _rotation((0, 2), theta / 180. * np.pi) @ c2w
    return _BLENDER_FLIP @ c2w


def _box_half(img):
    """2x2 box mean = cv2.resize(..., INTER_AREA) at an exact factor 2."""
    H, W = img.shape[0] // 2, img.shape[1] // 2
    v = img[:2 * H, :2 * W].reshape(H, 2, W, 2, -1)
    return ((v[:, 0, :, 0] + v[:, 0, :, 1]) + (v[:, 1, :, 0] + v[:, 1, :, 1])) * np.float32(0.25)


def load_blender_data(basedir, half_res=False, testskip=1):
    """-> imgs [N,H,W,4] (fp32 RGBA in [0,1]; float64 when half_res), poses [N,4,4] fp32,
    render_poses [40,4,4], [H, W, focal], i_split (train/val/test index arrays), bounding_box."""
    metas = {}
    for split in ("train", "val", "test"):
        with open(os.path.join(basedir, f"transforms_{split}.json")) as fp:
            metas[split] = json.load(fp)
    img_blocks, pose_blocks, first = [], [], [0]
    for split in ("train", "val", "test"):
        step = testskip if (split != "train" and testskip != 0) else 1
        frames = metas[split]["frames"][::step]
        block = np.array([_imread(os.path.join(basedir, fr["file_path"] + ".png")) for fr in frames])
        img_blocks.append((block / 255.).astype(np.float32))
        pose_blocks.append(np.array([fr["transform_matrix"] for fr in frames]).astype(np.float32))
        first.append(first[-1] + len(frames))
    i_split = [np.arange(first[k], first[k + 1]) for k in range(3)]
    imgs = np.concatenate(img_blocks, 0)
    poses = np.concatenate(pose_blocks, 0)
    H, W = imgs[0].shape[:2]
    camera_angle_x = float(metas["test"]["camera_angle_x"])     # the last split read, as the reference
    focal = .5 * W / np.tan(.5 * camera_angle_x)
    render_poses = torch.stack([pose_spherical(a, -30.0, 4.0) for a in np.linspace(-180, 180, 41)[:-1]], 0)
    if half_res:
        H, W, focal = H // 2, W // 2, focal / 2.
        imgs = np.stack([_box_half(im) for im in imgs]).astype(np.float64)
    bounding_box = get_bbox3d_for_blenderobj(metas["train"], H, W, near=2.0, far=6.0)
    return imgs, poses, render_poses, [H, W, focal], i_split, bounding_box


# ------------------------------------------------------------------------------------- LLFF
def _image_files(d):
    return [os.path.join(d, f) for f in sorted(os.listdir(d)) if f.endswith(_IMG_EXT)]


def _load_data(basedir, factor=None, width=None, height=None, load_imgs=True):
    """load_llff.py:63-123: poses [3,5,N] (hwf column rewritten for the loaded resolution),
    bds [2,N], imgs [H,W,3,N] in [0,1]."""
    arr = np.load(os.path.join(basedir, "poses_bounds.npy"))
    poses = arr[:, :-2].reshape([-1, 3, 5]).transpose([1, 2, 0])
    bds = arr[:, -2:].transpose([1, 0])
    src = _image_files(os.path.join(basedir, "images"))
    full_shape = _imread(src[0]).shape
    if factor is not None:
        sfx, target = f"_{factor}", None
    elif height is not None:
        factor = full_shape[0] / float(height)
        width = int(full_shape[1] / factor)
        sfx, target = f"_{width}x{height}", (width, height)
    elif width is not None:
        factor = full_shape[1] / float(width)
        height = int(full_shape[0] / factor)
        sfx, target = f"_{width}x{height}", (width, height)
    else:
        sfx, target, factor = "", None, 1
    imgdir = os.path.join(basedir, "images" + sfx)
    if os.path.isdir(imgdir):
        files = _image_files(imgdir)
        reader = _imread
    else:   # in-memory stand-in for _minify (module docstring)
        files = src
        size = target or (int(round(full_shape[1] / factor)), int(round(full_shape[0] / factor)))

        def reader(f):
            with Image.open(f) as im:
                return np.asarray(im.convert("RGB").resize(size, Image.BOX))
    if poses.shape[-1] != len(files):
        print(f"Mismatch between imgs {len(files)} and poses {poses.shape[-1]} !!!!")
        return None
    shape = reader(files[0]).shape
    poses[:2, 4, :] = np.array(shape[:2]).reshape([2, 1])
    poses[2, 4, :] = poses[2, 4, :] * 1. / factor
    if not load_imgs:
        return poses, bds
    imgs = np.stack([reader(f)[..., :3] / 255. for f in files], -1)
    return poses, bds, imgs


def normalize(x):
    return x / np.linalg.norm(x)


def viewmatrix(z, up, pos):
    """3x4 camera frame looking along z with the given up hint (load_llff.py:129-135)."""
    z = normalize(z)
    x = normalize(np.cross(up, z))
    y = normalize(np.cross(z, x))
    return np.stack([x, y, z, pos], 1)


def ptstocam(pts, c2w):
    return np.matmul(c2w[:3, :3].T, (pts - c2w[:3, 3])[..., np.newaxis])[..., 0]


def poses_avg(poses):
    """Mean camera of a rig: centroid, summed view/up axes, the first pose's hwf (:141-151)."""
    centre = poses[:, :3, 3].mean(0)
    forward = normalize(poses[:, :3, 2].sum(0))
    up = poses[:, :3, 1].sum(0)
    return np.concatenate([viewmatrix(forward, up, centre), poses[0, :3, -1:]], 1)


def render_path_spiral(c2w, up, rads, focal, zdelta, zrate, rots, N):
    """N poses on an elliptical spiral around c2w, all looking at the point `focal` ahead (:154-164)."""
    scale = np.array(list(rads) + [1.])
    hwf = c2w[:, 4:5]
    target = np.dot(c2w[:3, :4], np.array([0, 0, -focal, 1.]))
    out = []
    for th in np.linspace(0., 2. * np.pi * rots, N + 1)[:-1]:
        centre = np.dot(c2w[:3, :4], np.array([np.cos(th), -np.sin(th), -np.sin(th * zrate), 1.]) * scale)
        out.append(np.concatenate([viewmatrix(normalize(centre - target), up, centre), hwf], 1))
    return out


def _homogeneous(p34):
    bottom = np.broadcast_to(np.array([0., 0., 0., 1.]), p34.shape[:-2] + (1, 4))
    return np.concatenate([p34[..., :3, :4], bottom], -2)


def recenter_poses(poses):
    """Express every pose in the frame of the rig's average camera (:167-181)."""
    out = poses + 0
    ref = _homogeneous(poses_avg(poses)[None])[0]
    out[:, :3, :4] = (np.linalg.inv(ref) @ _homogeneous(poses))[:, :3, :4]
    return out


def spherify_poses(poses, bds):
    """360-degree rigs (:185-241): centre on the point closest to all optical axes, scale the mean
    camera distance to 1, and a 120-pose circle at the rig's mean height."""
    dirs, origins = poses[:, :3, 2:3], poses[:, :3, 3:4]
    A = np.eye(3) - dirs * np.transpose(dirs, [0, 2, 1])
    b = -A @ origins
    centre = np.squeeze(-np.linalg.inv((np.transpose(A, [0, 2, 1]) @ A).mean(0)) @ b.mean(0))
    up0 = normalize((poses[:, :3, 3] - centre).mean(0))
    ax1 = normalize(np.cross([.1, .2, .3], up0))
    ax2 = normalize(np.cross(up0, ax1))
    frame = np.stack([ax1, ax2, up0, centre], 1)
    reset = np.linalg.inv(_homogeneous(frame[None])) @ _homogeneous(poses)
    rad = np.sqrt(np.mean(np.sum(np.square(reset[:, :3, 3]), -1)))
    sc = 1. / rad
    reset[:, :3, 3] *= sc
    bds *= sc
    rad *= sc
    zh = np.mean(reset[:, :3, 3], 0)[2]
    rc = np.sqrt(rad ** 2 - zh ** 2)
    circle = []
    for th in np.linspace(0., 2. * np.pi, 120):
        eye = np.array([rc * np.cos(th), rc * np.sin(th), zh])
        z = normalize(eye)
        x = normalize(np.cross(z, np.array([0, 0, -1.])))
        y = normalize(np.cross(z, x))
        circle.append(np.stack([x, y, z, eye], 1))
    circle = np.stack(circle, 0)
    hwf = poses[0, :3, -1:]
    circle = np.concatenate([circle, np.broadcast_to(hwf, circle[:, :3, -1:].shape)], -1)
    reset = np.concatenate([reset[:, :3, :4], np.broadcast_to(hwf, reset[:, :3, -1:].shape)], -1)
    return reset, circle, bds


def load_llff_data(basedir, factor=8, recenter=True, bd_factor=.75, spherify=False, path_zflat=False):
    """-> images [N,H,W,3] fp32, poses [N,3,5] fp32 (LLFF axes turned to x right / y up / z back),
    bds [N,2], render_poses [120 or 60,3,5], i_test (the view closest to the mean camera),
    bounding_box (of the NDC rays, utils.py:61-92)."""
    poses, bds, imgs = _load_data(basedir, factor=factor)
    # [down, right, back] -> [right, up, back]; views first
    poses = np.concatenate([poses[:, 1:2, :], -poses[:, 0:1, :], poses[:, 2:, :]], 1)
    poses = np.moveaxis(poses, -1, 0).astype(np.float32)
    images = np.moveaxis(imgs, -1, 0).astype(np.float32)
    bds = np.moveaxis(bds, -1, 0).astype(np.float32)
    sc = 1. if bd_factor is None else 1. / (bds.min() * bd_factor)
    poses[:, :3, 3] *= sc
    bds *= sc
    if recenter:
        poses = recenter_poses(poses)
    if spherify:
        poses, render_poses, bds = spherify_poses(poses, bds)
    else:
        c2w = poses_avg(poses)
        up = normalize(poses[:, :3, 1].sum(0))
        near_d, far_d = bds.min() * .9, bds.max() * 5.
        dt = .75
        focus = 1. / ((1. - dt) / near_d + dt / far_d)     # harmonic mix of the depth range
        zdelta = near_d * .2
        rads = np.percentile(np.abs(poses[:, :3, 3]), 90, 0)
        n_views, n_rots = 120, 2
        c2w_path = c2w
        if path_zflat:
            c2w_path[:3, 3] = c2w_path[:3, 3] + (-near_d * .1) * c2w_path[:3, 2]
            rads[2] = 0.
            n_rots, n_views = 1, n_views // 2   # the reference's N_views /= 2 makes a float that
                                                # np.linspace rejects (numpy >= 1.18): an int here
        render_poses = render_path_spiral(c2w_path, up, rads, focus, zdelta, zrate=.5, rots=n_rots, N=n_views)
    render_poses = np.array(render_poses).astype(np.float32)
    c2w = poses_avg(poses)
    i_test = np.argmin(np.sum(np.square(c2w[:3, 3] - poses[:, :3, 3]), -1))
    images = images.astype(np.float32)
    poses = poses.astype(np.float32)
    bounding_box = get_bbox3d_for_llff(poses[:, :3, :4], poses[0, :3, -1], near=0.0, far=1.0)
    return images, poses, bds, render_poses, i_test, bounding_box


# ----------------------------------------------------------------------------------- ScanNet
_PLY_TYPES = {"char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "i2", "int16": "i2",
              "ushort": "u2", "uint16": "u2", "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4",
              "float": "f4", "float32": "f4", "double": "f8", "float64": "f8"}


def ply_vertex_bounds(path):
    """(min xyz, max xyz) of a PLY mesh's vertices: the part of pyvista.read(...).bounds that
    load_scannet.py:100-104 uses (pyvista is not in this image). Reads binary little/big-endian
    and ASCII PLY; the vertex element must come first (as in ScanNet's *_vh_clean.ply)."""
    with open(path, "rb") as f:
        if f.readline().strip() != b"ply":
            raise ValueError(f"{path}: not a PLY file")
        fmt, n_vert, props, in_vertex = None, 0, [], False
        while True:
            line = f.readline()
            if not line:
                raise ValueError(f"{path}: truncated PLY header")
            tok = line.decode("ascii", "replace").split()
            if not tok:
                continue
            if tok[0] == "format":
                fmt = tok[1]
            elif tok[0] == "element":
                in_vertex = tok[1] == "vertex"
                if in_vertex:
                    n_vert = int(tok[2])
            elif tok[0] == "property" and in_vertex:
                if tok[1] == "list":
                    raise ValueError(f"{path}: list property in the vertex element")
                props.append((tok[2], _PLY_TYPES[tok[1]]))
            elif tok[0] == "end_header":
                break
        if fmt == "ascii":
            rows = np.loadtxt(f, max_rows=n_vert, ndmin=2)
            names = [p[0] for p in props]
            xyz = rows[:, [names.index("x"), names.index("y"), names.index("z")]]
        else:
            end = "<" if fmt == "binary_little_endian" else ">"
            dt = np.dtype([(n, end + t) for n, t in props])
            v = np.frombuffer(f.read(dt.itemsize * n_vert), dtype=dt, count=n_vert)
            xyz = np.stack([v["x"], v["y"], v["z"]], 1).astype(np.float64)
    return xyz.min(0), xyz.max(0)


def load_scannet_data(basedir, sceneID, half_res=False, trainskip=10, testskip=1):
    """load_scannet.py:38-106: a ScanNet scene exported in the nerf_synthetic layout
    (<basedir>/nerfstyle_<sceneID>/transforms_*.json + PNGs) -> imgs [N,H,W,C] fp32, poses [N,4,4]
    (OpenCV -> OpenGL camera axes: y and z columns negated), render_poses [40,4,4], [H, W, focal],
    i_split, bounding_box = the scene mesh's vertex bounds (scans/<sceneID>/<sceneID>_vh_clean.ply)
    padded by 1."""
    scene = os.path.join(basedir, "nerfstyle_" + sceneID)
    metas = {}
    for split in ("train", "val", "test"):
        with open(os.path.join(scene, f"transforms_{split}.json")) as fp:
            metas[split] = json.load(fp)
    img_blocks, pose_blocks, first = [], [], [0]
    for split in ("train", "val", "test"):
        frames = metas[split]["frames"][::trainskip if split == "train" else testskip]
        block = np.array([_imread(os.path.join(scene, fr["file_path"] + ".png")) for fr in frames])
        poses = np.array([fr["transform_matrix"] for fr in frames], np.float64)
        poses[:, :3, 1:3] *= -1        # ScanNet poses use the OpenCV convention
        img_blocks.append((block / 255.).astype(np.float32))
        pose_blocks.append(poses.astype(np.float32))
        first.append(first[-1] + len(frames))
    i_split = [np.arange(first[k], first[k + 1]) for k in range(3)]
    imgs = np.concatenate(img_blocks, 0)
    poses = np.concatenate(pose_blocks, 0)
    H, W = imgs[0].shape[:2]
    focal = .5 * W / np.tan(.5 * float(metas["test"]["camera_angle_x"]))
    render_poses = torch.stack([pose_spherical(a, -30.0, 4.0) for a in np.linspace(-180, 180, 41)[:-1]], 0)
    if half_res:
        H, W, focal = H // 2, W // 2, focal / 2.
        imgs = np.stack([_box_half(im) for im in imgs]).astype(np.float64)
    lo, hi = ply_vertex_bounds(os.path.join(basedir, "scans", sceneID, f"{sceneID}_vh_clean.ply"))
    bounding_box = (torch.tensor(lo) - 1, torch.tensor(hi) + 1)
    return imgs, poses, render_poses, [H, W, focal], i_split, bounding_box
