#!/usr/bin/env python3
"""Per-block timeline of the hash forward (diagnostic build: tools/build_variant.py fwd_prof
-DNERF_FWD_PROF; run with NERF_HIP_LIB=build/variants/fwd_prof/libnerfhip.so) for the lego step's two
launches: 262,144 coarse points (4096 rays x 64) and 524,288 importance points (4096 x 128). Per launch:
the makespan, per grid row (row 0 = the grouped coarse levels, row r = one level) its first start,
last end and mean block time, the number of blocks in flight over time, and the blocks per XCC. It
answers where a launch's ~46 us of point-count-independent time goes (DESIGN §4 hash_encode_fwd).
JSON out: argv[1]."""
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

N_REC = 65536


def one_launch(lib, emb, pts, reps=5):
    meta = emb._meta
    P = pts.shape[0]
    feat = torch.empty(16, P, 2, device=pts.device)
    keep = torch.empty(P, dtype=torch.uint8, device=pts.device)
    tabs = _lib.ptr_array([e.weight.detach() for e in emb.embeddings])
    args = (_lib.ptr(pts), P, meta["bmin"], meta["bmax"], meta["res"], 16, 19, tabs, None, _lib.ptr(feat), 2, 2 * P,
            _lib.ptr(keep, dtype=torch.uint8), _lib.stream())
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    times = []
    for _ in range(reps):
        ev[0].record()
        _lib.call("nerf_hash_encode_fwd_q", *args)
        ev[1].record()
        torch.cuda.synchronize()
        times.append(ev[0].elapsed_time(ev[1]) * 1e3)
    buf = (ctypes.c_ulonglong * (N_REC * 3))()
    lib.nerf_fwd_prof_read.restype = ctypes.c_int
    assert lib.nerf_fwd_prof_read(buf, N_REC * 3) == 0
    rec = np.frombuffer(buf, dtype=np.uint64).reshape(N_REC, 3)
    ppt = int(os.environ.get("NERF_FWD_ROW_PTS", "2"))
    gx0, gx1 = (2 * P + 255) // 256, (2 * P + 256 * ppt - 1) // (256 * ppt)
    rows = 11   # lego: 6 grouped coarse levels + 10 single-level rows
    n = gx0 + 10 * gx1
    bounds = [0, gx0] + [gx0 + k * gx1 for k in range(1, 11)]
    r = rec[:n].astype(np.int64)
    t0 = r[:, 0].min()
    start, end = (r[:, 0] - t0) / 100.0, (r[:, 1] - t0) / 100.0   # 100 MHz -> us
    xcc = (r[:, 2] >> 32) & 0xF
    out = {"points": P, "row_points_per_thread": ppt, "blocks": [gx0, gx1, n], "event_us": [round(t, 1) for t in times],
           "makespan_us": round(float(end.max()), 1)}
    per_row = []
    for k in range(rows):
        s, e = start[bounds[k]:bounds[k + 1]], end[bounds[k]:bounds[k + 1]]
        d = e - s
        per_row.append({"row": k, "first_start": round(float(s.min()), 1), "last_start": round(float(s.max()), 1),
                        "first_end": round(float(e.min()), 1), "last_end": round(float(e.max()), 1),
                        "block_us_mean": round(float(d.mean()), 2), "block_us_p95": round(float(np.percentile(d, 95)), 2)})
    out["rows"] = per_row
    grid = np.arange(0.0, float(end.max()) + 0.5, 0.5)
    inflight = [int(((start <= t) & (end > t)).sum()) for t in grid]
    out["inflight_every_2us"] = inflight[::4]
    out["mean_inflight"] = round(float(np.mean(inflight)), 1)
    out["blocks_per_xcc"] = np.bincount(xcc, minlength=8).tolist()
    # the first blocks' XCC by blockIdx (dispatch order check): blocks 0..15 of row 0
    out["xcc_of_first_16_blocks"] = xcc[:16].tolist()
    out["block_us_sum_per_cu"] = round(float((end - start).sum() / 256), 1)
    return out


def main():
    dev = torch.device("cuda:0")
    from indoor_nerf_amd.synthetic import blender_bbox
    lo, hi = blender_bbox()
    emb = nerf.HashEmbedder((torch.from_numpy(lo), torch.from_numpy(hi)), finest_resolution=1024).to(dev)
    with torch.no_grad():
        for e in emb.embeddings:
            e.weight.uniform_(-1e-4, 1e-4)
    lib = _lib.load()
    res = {}
    for name, S in (("coarse_64", 64), ("importance_128", 128)):
        res[name] = one_launch(lib, emb, ray_points(4096, S, dev, seed=S)[0])
    with open(sys.argv[1], "w") as f:
        json.dump(res, f, indent=1)
    for k, v in res.items():
        print(k, {kk: vv for kk, vv in v.items() if kk not in ("rows", "inflight_every_2us")})
        for row in v["rows"]:
            print("   ", row)


if __name__ == "__main__":
    main()
