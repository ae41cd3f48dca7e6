#!/usr/bin/env python3
"""Per-block timeline of the owner pass (diagnostic build: tools/build_variant.py owner_prof
-DNERF_OWNER_PROF; run with NERF_HIP_LIB=build/variants/owner_prof/libnerfhip.so) on the lego
step's fine + coarse point sets (tools/owner_ab.py's setup): per level the mean block time split into
setup (LDS clear + segment-word scan), entries (the LDS sums) and flush (table rows out), and the
launch's makespan against the sum of block times / 256 CUs (dispatch imbalance). JSON out."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import indoor_nerf_amd as nerf  # noqa: E402
from indoor_nerf_amd import _lib  # noqa: E402
from owner_ab import ray_points  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    from indoor_nerf_amd.synthetic import blender_bbox
    lo, hi = blender_bbox()
    emb = nerf.HashEmbedder((torch.from_numpy(lo), torch.from_numpy(hi)), finest_resolution=1024).to(dev)
    meta = emb._meta
    sets = [ray_points(4096, 192, dev, seed=1)[0], ray_points(4096, 64, dev, seed=2)[0]]
    lib = _lib.load()
    C = int(lib.nerf_hash_bwd_chunk_points())
    chunks = [(p.shape[0] + C - 1) // C for p in sets]
    cap = sum(chunks)
    det = int(os.environ.get("NERF_DET", "0"))
    nbytes = int(lib.nerf_hash_encode_bwd_workspace_bytes(16, 19, C * cap, det))
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    grads = [torch.zeros(1 << 19, 2, device=dev) for _ in range(16)]
    gp = _lib.ptr_array(grads)
    ds = [torch.randn(16, p.shape[0], 2, device=dev) for p in sets]
    base = 0
    for p, n, d in zip(sets, chunks, ds):
        _lib.call("nerf_hash_encode_bwd_bin", _lib.ptr(p), p.shape[0], meta["bmin"], meta["bmax"], meta["res"], 16, 19,
                  _lib.ptr(d), 2, 2 * p.shape[0], base, cap, det, _lib.ptr(ws, dtype=torch.uint8), nbytes, _lib.stream())
        base += n
    n_own = 64
    out = {}
    for rep in range(3):
        _lib.call("nerf_hash_encode_bwd_owner", 16, 19, cap, cap, gp, det | (2 if rep == 2 else 0),
                  _lib.ptr(ws, dtype=torch.uint8), nbytes, _lib.stream())
        torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (16 * 128 * 4))()
    lib.nerf_owner_prof_read.restype = ctypes.c_int
    rc = lib.nerf_owner_prof_read(buf, 16 * 128 * 4)
    assert rc == 0, rc
    t = np.frombuffer(buf, dtype=np.uint64)[:16 * n_own * 4].reshape(16, n_own, 4).astype(np.int64)
    t0 = t[..., 0].min()
    us = (t - t0) / 100.0          # 100 MHz -> us
    dur = us[..., 3] - us[..., 0]
    for l in range(16):
        out[f"level{l}"] = {"block_us": round(float(dur[l].mean()), 2), "max_block_us": round(float(dur[l].max()), 2),
                            "setup_us": round(float((us[l, :, 1] - us[l, :, 0]).mean()), 2),
                            "entries_us": round(float((us[l, :, 2] - us[l, :, 1]).mean()), 2),
                            "flush_us": round(float((us[l, :, 3] - us[l, :, 2]).mean()), 2),
                            "start_us": round(float(us[l, :, 0].mean()), 2), "end_us": round(float(us[l, :, 3].max()), 2)}
    span = float(us[..., 3].max())
    out["makespan_us"] = round(span, 1)
    out["sum_block_us_over_256"] = round(float(dur.sum()) / 256, 1)
    out["mode"] = "overwrite (deferred zero)"
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
