#!/usr/bin/env python3
"""Timing of the binned hash backward on the lego step's point sets: the fine (4096 x 192) and coarse
(4096 x 64) sets binned side by side ("bin": both bin launches), then the owner launch alone
("owner"), HIP-event medians. JSON out. A/B of library builds: run once per build with
NERF_HIP_LIB=<path> (e.g. chunk sizes: tools/build_variant.py); NERF_DET=1 times the
deterministic mode; NERF_FINE_S=128 sizes the fine set to the importance samples alone (DESIGN §8.5:
what the backward and the fine gather ("fwd") would cost without the coarse points' re-encoding)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import indoor_nerf_amd as nerf  # noqa: E402
from indoor_nerf_amd import _lib  # noqa: E402
from indoor_nerf_amd.synthetic import blender_bbox, blender_rays  # noqa: E402


def ray_points(R, S, dev, seed=0):
    """R synthetic Blender rays, S sorted depths in [2, 6) each: [R S, 3] sample points."""
    ro, rd = (torch.from_numpy(v).to(dev) for v in blender_rays(R, seed=seed))
    g = torch.Generator(device=dev).manual_seed(seed)
    z = torch.sort(2 + 4 * torch.rand(R, S, device=dev, generator=g), -1)[0]
    return (ro[:, None] + rd[:, None] * z[..., None]).reshape(-1, 3).contiguous(), rd


def main():
    dev = torch.device("cuda:0")
    lo, hi = blender_bbox()
    emb = nerf.HashEmbedder((torch.from_numpy(lo), torch.from_numpy(hi)), finest_resolution=1024).to(dev)
    meta = emb._meta
    s_fine = int(os.environ.get("NERF_FINE_S", "192"))
    sets = [ray_points(4096, s_fine, dev, seed=1)[0], ray_points(4096, 64, dev, seed=2)[0]]
    tabs = _lib.ptr_array([e.weight.detach() for e in emb.embeddings])
    feat = torch.empty(16, sets[0].shape[0], 2, device=dev)
    keep = torch.empty(sets[0].shape[0], dtype=torch.uint8, device=dev)

    def fwd():
        _lib.call("nerf_hash_encode_fwd", _lib.ptr(sets[0]), sets[0].shape[0], meta["bmin"], meta["bmax"], meta["res"],
                  16, 19, tabs, _lib.ptr(feat), 2, 2 * sets[0].shape[0], _lib.ptr(keep, dtype=torch.uint8),
                  _lib.stream())
    lib = _lib.load()
    C = int(lib.nerf_hash_bwd_chunk_points())
    chunks = [(p.shape[0] + C - 1) // C for p in sets]
    cap = sum(chunks)
    det = int(os.environ.get("NERF_DET", "0"))   # 1: time the deterministic owner pass
    nbytes = int(lib.nerf_hash_encode_bwd_workspace_bytes(16, 19, C * cap, det))
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    grads = [torch.zeros(1 << 19, 2, device=dev) for _ in range(16)]
    gp = _lib.ptr_array(grads)
    ds = [torch.randn(16, p.shape[0], 2, device=dev) for p in sets]

    def bins():
        # the bucket counters start at zero (the owner pass resets them; a bins-only loop does not)
        if hasattr(lib, "nerf_hash_bwd_workspace_init"):   # absent from libraries before the bucket layout
            _lib.call("nerf_hash_bwd_workspace_init", _lib.ptr(ws, dtype=torch.uint8), nbytes, _lib.stream())
        base = 0
        for p, n, d in zip(sets, chunks, ds):
            _lib.call("nerf_hash_encode_bwd_bin", _lib.ptr(p), p.shape[0], meta["bmin"], meta["bmax"], meta["res"], 16, 19,
                      _lib.ptr(d), 2, 2 * p.shape[0], base, cap, det, _lib.ptr(ws, dtype=torch.uint8), nbytes,
                      _lib.stream())
            base += n

    def owner():
        _lib.call("nerf_hash_encode_bwd_owner", 16, 19, cap, cap, gp, det, _lib.ptr(ws, dtype=torch.uint8), nbytes,
                  _lib.stream())

    res = {}
    for rnd in range(5):
        for v in ("bin", "owner", "fwd"):
            ts = []
            for k in range(12):
                bins()   # every owner pass consumes the entries binned before it
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                {"bin": bins, "owner": owner, "fwd": fwd}[v]()
                e1.record()
                if v == "bin":
                    owner()
                torch.cuda.synchronize()
                if k >= 2:
                    ts.append(e0.elapsed_time(e1))
            res.setdefault(v, []).append(float(np.median(ts)))
    print(json.dumps({k: round(float(np.median(v)) * 1e3, 1) for k, v in res.items()} | {"unit": "us", "chunks": cap, "chunk_points": C, "det": det,
                      "fine_samples": s_fine}))


if __name__ == "__main__":
    main()
