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
