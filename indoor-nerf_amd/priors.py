"""PocketNeRF structural priors (ScanNet configuration): Manhattan-frame,
planarity and normal-consistency losses on the rendered depth and normal maps of a ray batch.

Same classes, functions, arguments, randomness and return values as
PocketNeRF/structural_priors.py:9-451, so train() (run_nerf.py:1039-1148) calls them unchanged:
ManhattanFrameEstimator, SemanticPlaneDetector, manhattan_sdf_loss, structured_planarity_loss,
spatial_normal_consistency_loss, combine_structural_losses_v2.

The losses are per-ray sized (N_rand rays) and differentiable w.r.t. the depth and normal maps,
through the Manhattan frame too (k-means centres -> torch.svd), exactly as the reference's autograd
graph. They run on the device as torch ops, drawing torch.randn / randperm / randint in the
reference's order (so a shared seed reproduces its samples), with the one O(N x Q) step, the
spatial nearest neighbour of the consistency loss (cdist + argmin over all rays for 200 queries),
in a HIP kernel (csrc/priors.hip), and the 3x3 SVD of the cluster centres in LAPACK on the host.
Reference behaviour kept as is: torch.svd's third output is V, and the frame is U @ V (not
U @ V^T); the data-dependent branches read counts on the host, as the reference's .item()/len()
calls do.
"""
import torch
import torch.nn.functional as F

from . import _lib


class ManhattanFrameEstimator:
    """structural_priors.py:9-77."""

    def __init__(self, confidence_threshold: float = 0.5):
        self.confidence_threshold = confidence_threshold
        self.manhattan_frame = None
        self.frame_confidence = 0.0

    def estimate_frame(self, normals, confidences=None):
        dev = normals.device
        normals = F.normalize(normals, dim=-1)
        if confidences is not None:
            keep = confidences > self.confidence_threshold
            if int(keep.sum()) < 20:
                return torch.eye(3, device=dev)
            normals = normals[keep]
        if normals.shape[0] < 30:
            return torch.eye(3, device=dev)
        centres = self._cluster_normals(normals)
        if centres is None:
            return torch.eye(3, device=dev)
        try:
            # The 3x3 SVD runs in LAPACK on the host: torch.svd's singular-vector signs are
            # backend-defined, and the reference's frame U @ V (its third output is V, not V^T)
            # depends on them; LAPACK's convention is the reference's CPU run (golden F18).
            U, _, V = torch.svd(centres.T.cpu())
            frame = U @ V
            if torch.det(frame) < 0:
                frame[:, -1] *= -1
            frame = frame.to(dev)
            self.manhattan_frame = frame
            return frame
        except Exception:   # the reference's bare except (:42-43)
            return torch.eye(3, device=dev)

    def _cluster_normals(self, normals, n_clusters: int = 3):
        """10 rounds of spherical k-means from torch.randn centres (:48-77)."""
        if normals.shape[0] < n_clusters:
            return None
        centres = F.normalize(torch.randn(n_clusters, 3, device=normals.device), dim=-1)
        for _ in range(10):
            assign = torch.argmax(normals @ centres.T, dim=-1)
            counts = torch.bincount(assign, minlength=n_clusters).tolist()
            rows = []
            for k in range(n_clusters):
                if counts[k] > 0:
                    rows.append(F.normalize(torch.mean(normals[assign == k], dim=0), dim=-1))
                else:
                    rows.append(centres[k])
            centres = torch.stack(rows)
        return centres


class SemanticPlaneDetector:
    """structural_priors.py:80-190: floor (|n_z| > t) and wall (|n_z| < 1 - t) rays among the rays
    whose normal has norm > 0.1."""

    def __init__(self, depth_threshold: float = 0.1, normal_threshold: float = 0.6):
        self.depth_threshold = depth_threshold
        self.normal_threshold = normal_threshold

    def detect_planes(self, depth_map, normals, image_coords=None):
        dev = depth_map.device
        n_rays = depth_map.shape[0]
        nz = F.normalize(normals, dim=-1)
        stable = torch.norm(normals, dim=-1) > 0.1
        empty = torch.zeros(n_rays, dtype=torch.bool, device=dev)
        if int(stable.sum()) < 10:
            return {"floor_mask": empty, "wall_mask": empty.clone(), "wall_clusters": {}, "n_floor": 0, "n_wall": 0}
        # |n . (0,0,1)| and |n_z| are the same number: the floor test and the wall test read n_z
        az = nz[:, 2].abs()
        floor_mask = stable & (az > self.normal_threshold)
        wall_mask = stable & (az < (1 - self.normal_threshold))
        n_wall = int(wall_mask.sum())
        wall_clusters = self._cluster_wall_normals(nz[wall_mask]) if n_wall > 20 else {}
        return {"floor_mask": floor_mask, "wall_mask": wall_mask, "wall_clusters": wall_clusters,
                "n_floor": int(floor_mask.sum()), "n_wall": n_wall}

    def _cluster_wall_normals(self, wall_normals):
        """Two dominant horizontal directions (:157-190; logging only)."""
        w2 = F.normalize(wall_normals[:, :2], dim=-1)
        if w2.shape[0] < 5:
            return {}
        sim = w2 @ w2.T
        k = int(torch.argmin(sim))
        c1, c2 = w2[k // sim.shape[1]], w2[k % sim.shape[1]]
        first = torch.sum(w2 * c1, dim=-1) > torch.sum(w2 * c2, dim=-1)
        out = {}
        if int(first.sum()) > 0:
            out["wall_1"] = torch.mean(w2[first], dim=0)
        if int((~first).sum()) > 0:
            out["wall_2"] = torch.mean(w2[~first], dim=0)
        return out


def manhattan_sdf_loss(normals, depth_map, manhattan_frame, semantic_info, weight=1.0):
    """structural_priors.py:194-256: floor normals along the frame's z (x0.5), wall normals along
    its x or y (x0.3), confident normals along any axis (x0.02); total clamped to [0, 0.1]."""
    nn_ = F.normalize(normals, dim=-1)
    parts = {}
    total = torch.tensor(0.0, device=normals.device)
    if semantic_info["n_floor"] > 50:
        a = torch.sum(nn_[semantic_info["floor_mask"]] * manhattan_frame[:, 2], dim=-1)
        parts["floor"] = torch.mean(torch.clamp(1.0 - torch.abs(a), 0.0, 1.0))
        total = total + parts["floor"] * 0.5
    if semantic_info["n_wall"] > 30:
        w = nn_[semantic_info["wall_mask"]]
        best = torch.maximum(torch.abs(torch.sum(w * manhattan_frame[:, 0], dim=-1)),
                             torch.abs(torch.sum(w * manhattan_frame[:, 1], dim=-1)))
        parts["wall"] = torch.mean(torch.clamp(1.0 - best, 0.0, 1.0))
        total = total + parts["wall"] * 0.3
    best = torch.max(torch.abs(nn_ @ manhattan_frame), dim=-1)[0]
    sure = best > 0.5
    if int(sure.sum()) > 20:
        parts["general"] = torch.mean(torch.clamp(1.0 - best[sure], 0.0, 1.0))
        total = total + parts["general"] * 0.02
    return weight * torch.clamp(total, 0.0, 0.1), parts


def _pair_gap(depth_map, mask, cap):
    """Mean |depth difference| over up to `cap` random disjoint pairs of rays inside `mask`
    (a torch.randperm over the mask's rays, as :273-284), or None."""
    idx = torch.where(mask)[0]
    if len(idx) <= 1:
        return None
    n_pairs = min(cap, len(idx) // 2)
    if n_pairs <= 0:
        return None
    perm = torch.randperm(len(idx))[:n_pairs * 2]
    a, b = idx[perm[:n_pairs]], idx[perm[n_pairs:2 * n_pairs]]
    return torch.mean(torch.abs(depth_map[a] - depth_map[b]))


def structured_planarity_loss(depth_map, normals, rays_d, semantic_info, weight=1.0, smoothness_scale=0.05):
    """structural_priors.py:259-318: depth smoothness between random ray pairs on the floor (x2.0),
    on walls (x1.5) and elsewhere (x0.1)."""
    total = torch.tensor(0.0, device=depth_map.device)
    if depth_map.shape[0] < 10:
        return total
    floor, wall = semantic_info["floor_mask"], semantic_info["wall_mask"]
    for mask, count, cap, scale in ((floor, semantic_info["n_floor"], 100, 2.0),
                                    (wall, semantic_info["n_wall"], 100, 1.5)):
        if count > 5:
            gap = _pair_gap(depth_map, mask, cap)
            if gap is not None:
                total = total + gap * scale
    other = ~(floor | wall)
    if int(other.sum()) > 5:
        gap = _pair_gap(depth_map, other, 50)
        if gap is not None:
            total = total + gap * 0.1
    return weight * total


def nearest_pixel(spatial_coords, idx1):
    """For each query ray idx1[q], the nearest other ray in pixel space and its distance
    (torch.cdist + self-exclusion + argmin of :339-344), csrc/priors.hip."""
    xy = spatial_coords.float().contiguous()
    q = idx1.to(torch.int64).contiguous()
    idx2 = torch.empty_like(q)
    dist = torch.empty(q.shape[0], device=xy.device, dtype=torch.float32)
    _lib.call("nerf_nearest_pixel", _lib.ptr(xy, "spatial_coords"), xy.shape[0], _lib.ptr(q, "idx1", dtype=torch.int64),
              q.shape[0], _lib.ptr(idx2, "idx2", dtype=torch.int64), _lib.ptr(dist, "dist"), _lib.stream())
    return idx2, dist


def spatial_normal_consistency_loss(normals, depth_map, spatial_coords=None, weight=1.0):
    """structural_priors.py:321-371: 1 - cos between a ray's normal and its nearest pixel
    neighbour's (or, without coordinates, the next ray's), weighted by depth similarity (and
    pixel proximity)."""
    n_rays = normals.shape[0]
    dev = normals.device
    if n_rays < 10:
        return torch.tensor(0.0, device=dev)
    nn_ = F.normalize(normals, dim=-1)
    if spatial_coords is not None:
        n_pairs = min(200, n_rays // 2)
        idx1 = torch.randint(0, n_rays, (n_pairs,), device=dev)
        idx2, dist = nearest_pixel(spatial_coords, idx1)
        w = torch.exp(-dist * 0.1) * torch.exp(-torch.abs(depth_map[idx1] - depth_map[idx2]))
        loss = torch.mean(w * (1.0 - torch.sum(nn_[idx1] * nn_[idx2], dim=-1)))
    else:
        n_pairs = min(100, n_rays - 1)
        idx1 = torch.randint(0, n_rays - 1, (n_pairs,), device=dev)
        idx2 = idx1 + 1
        sim = torch.exp(-torch.abs(depth_map[idx1] - depth_map[idx2]))
        loss = torch.mean(sim * (1.0 - torch.sum(nn_[idx1] * nn_[idx2], dim=-1)))
    return weight * loss


def combine_structural_losses_v2(depth_pred, normals, rays_d, spatial_coords=None, weights=None,
                                 manhattan_frame_estimator=None, semantic_detector=None):
    """structural_priors.py:374-451 -> (total_loss, loss_dict)."""
    if weights is None:
        weights = {"manhattan": 1.0, "planarity": 1.0, "normal_consistency": 0.5}
    dev = depth_pred.device
    total = torch.tensor(0.0, device=dev)
    if normals is None:
        print("⚠️  Structural priors: normals is None, skipping normal-based losses")
        return total, {"error": "normals_none"}
    if normals.dim() != 2 or normals.shape[-1] != 3:
        print(f"⚠️  Structural priors: invalid normals shape {normals.shape}, expected [N, 3]")
        return total, {"error": f"invalid_normals_shape_{normals.shape}"}
    if normals.shape[0] == 0:
        print("⚠️  Structural priors: empty normals tensor, skipping")
        return total, {"error": "empty_normals"}
    if depth_pred.shape[0] != normals.shape[0]:
        print(f"⚠️  Structural priors: depth-normal size mismatch {depth_pred.shape[0]} vs {normals.shape[0]}")
        return total, {"error": f"size_mismatch_{depth_pred.shape[0]}_{normals.shape[0]}"}
    if manhattan_frame_estimator is None:
        manhattan_frame_estimator = ManhattanFrameEstimator(confidence_threshold=0.4)
    if semantic_detector is None:
        semantic_detector = SemanticPlaneDetector(normal_threshold=0.5)
    out = {}
    try:
        info = semantic_detector.detect_planes(depth_pred, normals, spatial_coords)
        frame = manhattan_frame_estimator.estimate_frame(normals, torch.norm(normals, dim=-1))
        if "manhattan" in weights:
            m_loss, m_parts = manhattan_sdf_loss(normals, depth_pred, frame, info, weights["manhattan"])
            out.update({f"manhattan_{k}": v for k, v in m_parts.items()})
            total = total + m_loss
        if "planarity" in weights:
            out["planarity"] = structured_planarity_loss(depth_pred, normals, rays_d, info, weights["planarity"])
            total = total + out["planarity"]
        if "normal_consistency" in weights:
            out["normal_consistency"] = spatial_normal_consistency_loss(normals, depth_pred, spatial_coords,
                                                                        weights["normal_consistency"])
            total = total + out["normal_consistency"]
        out["semantic_floor_count"] = info["n_floor"]
        out["semantic_wall_count"] = info["n_wall"]
    except Exception as e:   # the reference swallows failures (:447-449)
        print(f"⚠️  Structural priors computation failed: {e}")
        return torch.tensor(0.0, device=dev), {"error": str(e)}
    return total, out


# ---- device path: the whole combine_structural_losses_v2 in three launches (csrc/priors_fused.hip) ----
_CAPS = (100, 100, 50)


def _fused_workspace(n, device):
    """A workspace of its own for every forward: it carries the forward's state (masks, pairs, the
    frame) to that node's backward, so a second forward before the first backward (e.g. a logging
    call with grad enabled) cannot overwrite it. Under a HIP-graph capture it comes from the graph's
    private pool like every other allocation of the captured step."""
    return torch.empty(int(_lib.load().nerf_priors_workspace_bytes(n)), dtype=torch.uint8, device=device)


class _FusedPriorsFn(torch.autograd.Function):
    """(depth [N], normals [N,3]) -> total structural loss (0-dim), d depth / d normals in backward.
    With addend (a 0-dim loss), returns addend + total from the same launch (its gradient passes through)."""

    @staticmethod
    def forward(ctx, depth, normals, coords, addend, spec):
        dev = depth.device
        N = depth.shape[0]
        d = depth.detach().float().contiguous()
        n = normals.detach().float().contiguous()
        xy = coords.detach().float().contiguous() if coords is not None else None
        ws = spec["workspace"] if spec.get("workspace") is not None else _fused_workspace(N, dev)
        if ws.dtype != torch.uint8 or ws.numel() < int(_lib.load().nerf_priors_workspace_bytes(N)):
            raise ValueError("fused_structural_losses: workspace must be uint8 with nerf_priors_workspace_bytes(N) bytes")
        cfg = _lib.PriorsConfig()
        w = spec["weights"]
        cfg.use_manhattan, cfg.use_planarity, cfg.use_consistency = (int(k in w) for k in
                                                                     ("manhattan", "planarity", "normal_consistency"))
        cfg.w_manhattan = float(w.get("manhattan", 0.0))
        cfg.w_planarity = float(w.get("planarity", 0.0))
        cfg.w_consistency = float(w.get("normal_consistency", 0.0))
        scale = spec.get("scale")
        cfg.d_scale = _lib.ptr(scale, "scale", allow_none=True)
        cfg.confidence_threshold, cfg.normal_threshold = spec["confidence"], spec["normal_threshold"]
        # everything cfg points at stays referenced by ctx until the backward has read it (the ramp
        # `scale` is often a temporary of the caller)
        keep_alive = [] if scale is None else [scale]
        args = (_lib.ptr(d, "depth"), _lib.ptr(n, "normals"), _lib.ptr(xy, "coords", allow_none=True), N)
        wsp = (_lib.ptr(ws, "workspace", dtype=torch.uint8), ws.numel())
        if spec["replay"]:
            _replay_draws(cfg, n, xy, N, spec, keep_alive)
            centres = torch.empty(9, device=dev)
            usv = torch.zeros(21, device=dev)
            keep_alive += [centres, usv]
            cfg.usv = _lib.ptr(usv, "usv")
            _lib.call("nerf_priors_prep", *args, ctypes_ref(cfg), *wsp, _lib.ptr(centres, "centres"), _lib.stream())
            if spec["kmeans"]:   # the frame's SVD on the host (LAPACK: the reference's sign convention, F18)
                U, S, V = torch.svd(centres.reshape(3, 3).T.cpu())
                usv.copy_(torch.cat([U.reshape(-1), S, V.reshape(-1)]))
        else:
            from .render import _rng
            cfg.seed, cfg.offset, rng = _rng()
            cfg.d_rng = rng
            _lib.call("nerf_priors_prep", *args, ctypes_ref(cfg), *wsp, None, _lib.stream())
        loss = torch.empty(1, device=dev)
        parts = torch.empty(7, device=dev)
        if addend is not None:
            addend = addend.detach().float().reshape(1).contiguous()
            keep_alive.append(addend)
        _lib.call("nerf_priors_loss_add", *args, ctypes_ref(cfg), *wsp, _lib.ptr(addend, "addend", allow_none=True),
                  _lib.ptr(loss, "loss"), _lib.ptr(parts, "parts"), _lib.stream())
        ctx.save_for_backward(d, n, xy if xy is not None else torch.empty(0, device=dev))
        ctx.cfg, ctx.ws, ctx.keep, ctx.has_xy, ctx.parts = cfg, ws, keep_alive, xy is not None, parts
        spec["parts"] = parts
        return loss.reshape(())

    @staticmethod
    def backward(ctx, g):
        d, n, xy = ctx.saved_tensors
        N = d.shape[0]
        gd, gn = torch.empty_like(d), torch.empty_like(n)
        g1 = g.detach().float().reshape(1).contiguous()
        _lib.call("nerf_priors_bwd", _lib.ptr(d, "depth"), _lib.ptr(n, "normals"),
                  _lib.ptr(xy, "coords") if ctx.has_xy else None, N, ctypes_ref(ctx.cfg),
                  _lib.ptr(ctx.ws, "workspace", dtype=torch.uint8), ctx.ws.numel(), _lib.ptr(g1, "grad_loss"),
                  _lib.ptr(gd, "grad_depth"), _lib.ptr(gn, "grad_normals"), _lib.stream())
        return gd, gn, None, (g if ctx.needs_input_grad[3] else None), None


def ctypes_ref(cfg):
    import ctypes
    return ctypes.byref(cfg)


def _replay_draws(cfg, n, xy, N, spec, keep_alive):
    """The reference's draws in its order (torch.randn for the k-means init, torch.randperm per
    planarity class, torch.randint for the consistency queries), decided with host counts exactly
    where the reference's branches read them (this mode synchronises; it pins the device path to
    the reference's randomness, golden F18)."""
    dev = n.device
    nrm = torch.norm(n, dim=-1)
    nz = F.normalize(n, dim=-1)
    stable = nrm > 0.1
    t = spec["normal_threshold"]
    if int(stable.sum()) < 10:
        floor = wall = torch.zeros(N, dtype=torch.bool, device=dev)
    else:
        az = nz[:, 2].abs()
        floor, wall = stable & (az > t), stable & (az < 1 - t)
    n_keep = int((nrm > spec["confidence"]).sum())
    spec["kmeans"] = n_keep >= 30
    if spec["kmeans"]:
        c0 = torch.randn(3, 3, device=dev).float().contiguous()
        keep_alive.append(c0)
        cfg.centres0 = _lib.ptr(c0, "centres0")
    perm = torch.zeros(3, 2 * max(_CAPS), dtype=torch.int32, device=dev)
    if N >= 10:
        other = ~(floor | wall)
        counts = (int(floor.sum()), int(wall.sum()), int(other.sum()))
        for k, (cnt, cap) in enumerate(zip(counts, _CAPS)):
            if cnt > 5:
                n_pairs = min(cap, cnt // 2)
                p = torch.randperm(cnt)[:2 * n_pairs]
                perm.view(-1)[2 * sum(_CAPS[:k]):2 * sum(_CAPS[:k]) + p.numel()] = p.to(dev, torch.int32)
    keep_alive.append(perm)
    cfg.perm = _lib.ptr(perm, "perm", dtype=torch.int32)
    if N >= 10:
        if xy is not None:
            idx1 = torch.randint(0, N, (min(200, N // 2),), device=dev)
        else:
            idx1 = torch.randint(0, N - 1, (min(100, N - 1),), device=dev)
        idx1 = idx1.to(torch.int32).contiguous()
        keep_alive.append(idx1)
        cfg.idx1 = _lib.ptr(idx1, "idx1", dtype=torch.int32)


def fused_structural_losses(depth_pred, normals, spatial_coords=None, weights=None, confidence_threshold=0.4,
                            normal_threshold=0.5, scale=None, replay=False, workspace=None, addend=None):
    """combine_structural_losses_v2 on the device (csrc/priors_fused.hip): same losses, branches and
    autograd graph, no host synchronisation (capturable in a HIP graph). scale: optional device [1]
    multiplier of the weights (the train() ramp, a per-step graph slot). replay=True draws the
    reference's torch.randn/randperm/randint in its order and takes the frame's SVD from LAPACK
    (host syncs; the golden F18 parity mode). workspace: optional uint8 device tensor of at least
    nerf_priors_workspace_bytes(N) for this call's state (default: a fresh one per call; pass one to
    inspect the PriorsState afterwards). addend: optional 0-dim loss; then the first result is
    addend + total, formed in the loss launch (nerf_priors_loss_add: the training step's
    `loss + structural_loss` without an add of its own). Returns (total, parts) with parts a device
    [7] tensor (floor, wall, general, manhattan, planarity, consistency, total)."""
    if weights is None:
        weights = {"manhattan": 1.0, "planarity": 1.0, "normal_consistency": 0.5}
    N = depth_pred.shape[0]
    if not (1 <= N <= _lib.PRIORS_MAX_RAYS) or normals is None or normals.shape != (N, 3):
        raise ValueError(f"fused_structural_losses: need depth [N] and normals [N,3], 1 <= N <= {_lib.PRIORS_MAX_RAYS}")
    spec = dict(weights=weights, confidence=float(confidence_threshold), normal_threshold=float(normal_threshold),
                scale=scale, replay=bool(replay), workspace=workspace)
    if addend is not None and addend.numel() != 1:
        raise ValueError("fused_structural_losses: addend must hold one value")
    total = _FusedPriorsFn.apply(depth_pred, normals, spatial_coords, addend, spec)
    if addend is not None:
        total = total.reshape(addend.shape)
    return total, spec["parts"]
