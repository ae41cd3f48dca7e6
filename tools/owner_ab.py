#!/usr/bin/env python3
"""A/B of the hash backward's owner pass (NERF_OWNER_EXP variants) on the lego step's bins: the fine
(4096 x 192) and coarse (4096 x 64) point sets binned side by side, then the owner launch alone,
interleaved rounds, HIP-event medians. JSON out."""
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
from indoor_nerf_amd.synthetic import blender_bbox  # noqa: E402
from kbench import ray_points  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    lo, hi = blender_bbox()
    emb = nerf.HashEmbedder((torch.from_numpy(lo), torch.from_numpy(hi)), finest_resolution=1024).to(dev)
    meta = emb._meta
    sets = [ray_points(4096, 192, dev, seed=1)[0], ray_points(4096, 64, dev, seed=2)[0]]
    chunks = [(p.shape[0] + 255) // 256 for p in sets]
    cap = sum(chunks)
    lib = _lib.load()
    det = int(os.environ.get("NERF_DET", "0"))   # 1: time the deterministic owner pass
    nbytes = int(lib.nerf_hash_encode_bwd_workspace_bytes(16, 19, 256 * cap, det))
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    grads = [torch.zeros(1 << 19, 2, device=dev) for _ in range(16)]
    gp = _lib.ptr_array(grads)
    ds = [torch.randn(16, p.shape[0], 2, device=dev) for p in sets]

    def bins():
        base = 0
        for p, n, d in zip(sets, chunks, ds):
            _lib.call("nerf_hash_encode_bwd_bin", _lib.ptr(p), p.shape[0], meta["bmin"], meta["bmax"], meta["res"], 16, 19,
                      _lib.ptr(d), 2, 2 * p.shape[0], base, cap, det, _lib.ptr(ws, dtype=torch.uint8), nbytes,
                      _lib.stream())
            base += n

    bins()

    def owner():
        _lib.call("nerf_hash_encode_bwd_owner", 16, 19, cap, cap, gp, det, _lib.ptr(ws, dtype=torch.uint8), nbytes,
                  _lib.stream())

    vers = sys.argv[1].split(",") if len(sys.argv) > 1 else ["owner", "bin0", "bin1", "bin2", "bin3"]
    res = {}
    for rnd in range(5):
        for v in vers:
            if v.startswith("bin"):
                os.environ["NERF_BIN_EXP"] = v[3:]
                fn = bins
            else:
                            bins()
                fn = owner
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(10):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            res.setdefault(v, []).append(float(np.median(ts)))
    print(json.dumps({k: round(float(np.median(v)) * 1e3, 1) for k, v in res.items()} | {"unit": "us", "chunks": cap}))


if __name__ == "__main__":
    main()
