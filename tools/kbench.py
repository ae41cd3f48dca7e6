#!/usr/bin/env python3
"""Kernel micro-benchmark: A/B variants of the hot kernels in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24), on the metric configuration's point sets (4096 lego rays,
64 coarse / 192 fine sorted samples per ray). Prints a JSON summary."""
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
    ro, rd = (torch.from_numpy(v).to(dev) for v in blender_rays(R, seed=seed))
    g = torch.Generator(device=dev).manual_seed(seed)
    z = torch.sort(2 + 4 * torch.rand(R, S, device=dev, generator=g), -1)[0]
    return (ro[:, None] + rd[:, None] * z[..., None]).reshape(-1, 3).contiguous(), rd


def timeit(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts)), float(np.min(ts))


def main():
    dev = torch.device("cuda:0")
    lo, hi = blender_bbox()
    emb = nerf.HashEmbedder((torch.from_numpy(lo), torch.from_numpy(hi)), finest_resolution=1024).to(dev)
    with torch.no_grad():
        for e in emb.embeddings:
            e.weight.uniform_(-0.05, 0.05)
    out = {}
    for name, S in (("coarse", 64), ("fine", 192)):
        pts, rd = ray_points(4096, S, dev)
        P = pts.shape[0]
        meta = emb._meta
        feat = torch.empty(16, P, 2, device=dev)
        keep = torch.empty(P, device=dev, dtype=torch.bool)
        dfeat = torch.randn(16, P, 2, device=dev)
        grads = [torch.zeros_like(e.weight) for e in emb.embeddings]

        def fwd():
            _lib.call("nerf_hash_encode_fwd", _lib.ptr(pts), P, meta["bmin"], meta["bmax"], meta["res"], 16, 19,
                      _lib.ptr_array(emb.tables()), _lib.ptr(feat), 2, 2 * P, _lib.ptr(keep, dtype=torch.bool),
                      _lib.stream())

        def bwd():
            _lib.call("nerf_hash_encode_bwd", _lib.ptr(pts), P, meta["bmin"], meta["bmax"], meta["res"], 16, 19,
                      _lib.ptr(dfeat), 2, 2 * P, _lib.ptr_array(grads), _lib.stream())

        def bwd_ws():
            nerf.hashgrid.hash_encode_bwd(pts, meta, dfeat, 2, 2 * P, grads)

        res = {"points": P, "fwd_ms": timeit(fwd)}
        for g in grads:
            g.zero_()
        bwd()
        ref = torch.stack(grads).clone()
        for g in grads:
            g.zero_()
        bwd_ws()
        cur = torch.stack(grads)
        res["ws_vs_direct_maxrel_diff"] = ((cur - ref).abs().max() / ref.abs().max()).item()
        t_direct, t_ws = [], []
        for _ in range(5):
            t_direct.append(timeit(bwd, reps=5, warm=1)[0])
            t_ws.append(timeit(bwd_ws, reps=5, warm=1)[0])
        res["bwd_direct_ms"], res["bwd_ws_ms"] = float(np.median(t_direct)), float(np.median(t_ws))
        # correctness of the variants against each other
        ref = None
        for v in ("0", "1"):
            os.environ["NERF_HASH_BWD"] = v
            for g in grads:
                g.zero_()
            bwd()
            cur = torch.stack(grads).clone()
            if ref is None:
                ref = cur
            else:
                err = ((cur - ref).abs().max() / ref.abs().max()).item()
                res["bwd_variant_maxrel_diff"] = err
        rounds = {"0": [], "1": []}
        for _ in range(5):
            for v in ("0", "1"):
                os.environ["NERF_HASH_BWD"] = v
                rounds[v].append(timeit(bwd, reps=5, warm=1)[0])
        res["bwd_ms_per_variant"] = {("atomic_per_lane" if v == "0" else "coalesced"): float(np.median(t))
                                     for v, t in rounds.items()}
        out[name] = res
    os.environ["NERF_HASH_BWD"] = "1"
    print(json.dumps(out, indent=1))




def mlp_bench():
    """MLP fwd/bwd kernels on the coarse (262,144) and fine (786,432) point counts."""
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    net = nerf.NeRFSmall(2, 64, 15, 3, 64, 32, 16).to(dev)
    out = {}
    for P in (262144, 786432):
        feat = torch.randn(16, P, 2, device=dev) * 0.3
        vd = torch.nn.functional.normalize(torch.randn(P // 64, 3, device=dev), dim=-1)
        keep = torch.ones(P, device=dev, dtype=torch.bool)
        raw = torch.empty(P, 4, device=dev)
        graw = torch.randn(P, 4, device=dev)
        dfeat = torch.empty_like(feat)
        from indoor_nerf_amd.field import _grads_struct, _weights_struct
        W = net.mlp_weights()

        def fwd():
            _lib.call("nerf_mlp_fwd", _lib.ptr(feat), 2, 2 * P, None, 0, _lib.ptr(vd), 64,
                      _lib.ptr(keep, dtype=torch.bool), P, _weights_struct(W), _lib.ptr(raw), None, _lib.stream())

        def bwd():
            _lib.call("nerf_mlp_bwd", _lib.ptr(feat), 2, 2 * P, None, 0, _lib.ptr(vd), 64,
                      _lib.ptr(keep, dtype=torch.bool), P, _weights_struct(W), _lib.ptr(graw), _grads_struct(W),
                      _lib.ptr(dfeat), None, None, _lib.stream())

        res = {}
        # correctness of the MLP variants against each other (raw and weight grads)
        outs = {}
        for v in ("1", "2"):
            os.environ["NERF_MLP"] = v
            fwd()
            for w in W:
                w.grad = None
            bwd()
            outs[v] = (raw.clone(), [w.grad.clone() for w in W], dfeat.clone())
        res["raw_maxabs_diff"] = (outs["1"][0] - outs["2"][0]).abs().max().item()
        res["dW_maxrel_diff"] = max(((a - b).abs().max() / b.abs().max()).item() for a, b in zip(outs["1"][1], outs["2"][1]))
        res["dfeat_maxabs_diff"] = (outs["1"][2] - outs["2"][2]).abs().max().item()
        res["dfeat_absmax"] = outs["2"][2].abs().max().item()
        # run-to-run determinism of each variant (dfeat has no atomics: must be bit-identical)
        for v in ("1", "2"):
            os.environ["NERF_MLP"] = v
            fwd()
            bwd()
            res[f"v{v}_dfeat_rerun_diff"] = (dfeat - outs[v][2]).abs().max().item()
        for w in W:
            w.grad = None
        _grads_struct(W)
        rounds = {"1": {"fwd": [], "bwd": []}, "2": {"fwd": [], "bwd": []}}
        for _ in range(5):
            for v in ("1", "2"):
                os.environ["NERF_MLP"] = v
                rounds[v]["fwd"].append(timeit(fwd, reps=5, warm=1)[0])
                rounds[v]["bwd"].append(timeit(bwd, reps=5, warm=1)[0])
        for v, d in rounds.items():
            res[f"v{v}"] = {k: float(np.median(t)) for k, t in d.items()}
        out[P] = res
    os.environ["NERF_MLP"] = "2"
    print(json.dumps(out, indent=1))


def levels_bench():
    """Hash fwd/bwd cost per level (one level per launch) on the fine point set: where the backward's
    atomics go (coarse levels: contention on few rows; fine levels: one request per corner pair)."""
    dev = torch.device("cuda:0")
    lo, hi = blender_bbox()
    emb = nerf.HashEmbedder((torch.from_numpy(lo), torch.from_numpy(hi)), finest_resolution=1024).to(dev)
    with torch.no_grad():
        for e in emb.embeddings:
            e.weight.uniform_(-0.05, 0.05)
    meta = emb._meta
    res_all = list(meta["res"])
    out = {}
    lo_t, hi_t = torch.tensor(lo, device=dev), torch.tensor(hi, device=dev)

    def morton_order(pts, bits):
        q = ((pts - lo_t) / (hi_t - lo_t) * (1 << bits)).long().clamp(0, (1 << bits) - 1)
        key = torch.zeros(pts.shape[0], dtype=torch.long, device=dev)
        for b in range(bits):
            for a in range(3):
                key |= ((q[:, a] >> b) & 1) << (3 * b + a)
        return torch.sort(key, stable=True)[1]

    cases = [("coarse", 64, 0), ("fine", 192, 0)]
    for name, S, bits in cases:
        pts, _ = ray_points(4096, S, dev)
        P = pts.shape[0]
        feat = torch.empty(16, P, 2, device=dev)
        keep = torch.empty(P, device=dev, dtype=torch.bool)
        dfeat = torch.randn(16, P, 2, device=dev)
        if bits:
            perm = morton_order(pts, bits)
            pts = pts[perm].contiguous()
            dfeat = dfeat[:, perm].contiguous()
        grads = [torch.zeros_like(e.weight) for e in emb.embeddings]
        tabs = emb.tables()
        rows = []
        for lvl in range(16):
            r = _lib.host_f32([res_all[lvl]])

            def fwd():
                _lib.call("nerf_hash_encode_fwd", _lib.ptr(pts), P, meta["bmin"], meta["bmax"], r, 1, 19,
                          _lib.ptr_array([tabs[lvl]]), _lib.ptr(feat[lvl]), 2, 2 * P, _lib.ptr(keep, dtype=torch.bool),
                          _lib.stream())

            def bwd():
                _lib.call("nerf_hash_encode_bwd", _lib.ptr(pts), P, meta["bmin"], meta["bmax"], r, 1, 19,
                          _lib.ptr(dfeat[lvl]), 2, 2 * P, _lib.ptr_array([grads[lvl]]), _lib.stream())
            row = {"level": lvl, "res": res_all[lvl], "fwd_us": 1e3 * timeit(fwd, reps=10)[0]}
            for v in ("1", "2"):
                os.environ["NERF_HASH_BWD"] = v
                row["bwd_us" if v == "1" else "bwd_noatomic_us"] = 1e3 * timeit(bwd, reps=10)[0]
            os.environ["NERF_HASH_BWD"] = "3"
            for R in (4, 16, 64):
                os.environ["NERF_HASH_REPL"] = str(R)
                row[f"bwd_repl{R}_us"] = 1e3 * timeit(bwd, reps=10)[0]
            os.environ["NERF_HASH_BWD"] = "1"
            rows.append(row)
        out[name] = {"points": P, "levels": rows,
                     "sum_bwd_us": sum(r["bwd_us"] for r in rows), "sum_fwd_us": sum(r["fwd_us"] for r in rows)}
    print(json.dumps(out, indent=1))


def bwd_only(S=192, reps=10):
    """Only the workspace (binned) hash backward on one point set, for rocprofv3 kernel traces."""
    dev = torch.device("cuda:0")
    lo, hi = blender_bbox()
    emb = nerf.HashEmbedder((torch.from_numpy(lo), torch.from_numpy(hi)), finest_resolution=1024).to(dev)
    pts, _ = ray_points(4096, S, dev)
    P = pts.shape[0]
    dfeat = torch.randn(16, P, 2, device=dev)
    grads = [torch.zeros_like(e.weight) for e in emb.embeddings]
    for _ in range(reps):
        nerf.hashgrid.hash_encode_bwd(pts, emb._meta, dfeat, 2, 2 * P, grads)
    torch.cuda.synchronize()
    print(json.dumps({"points": P, "reps": reps}))


def mlp_only(P=786432, reps=10):
    """Only the default MLP fwd + bwd kernels at one point count, for rocprofv3 PMC passes."""
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    net = nerf.NeRFSmall(2, 64, 15, 3, 64, 32, 16).to(dev)
    from indoor_nerf_amd.field import _grads_struct, _weights_struct
    feat = torch.randn(16, P, 2, device=dev) * 0.3
    vd = torch.nn.functional.normalize(torch.randn(P // 64, 3, device=dev), dim=-1)
    keep = torch.ones(P, device=dev, dtype=torch.bool)
    raw = torch.empty(P, 4, device=dev)
    graw = torch.randn(P, 4, device=dev)
    dfeat = torch.empty_like(feat)
    W = net.mlp_weights()
    for _ in range(reps):
        _lib.call("nerf_mlp_fwd", _lib.ptr(feat), 2, 2 * P, None, 0, _lib.ptr(vd), 64,
                  _lib.ptr(keep, dtype=torch.bool), P, _weights_struct(W), _lib.ptr(raw), None, _lib.stream())
        _lib.call("nerf_mlp_bwd", _lib.ptr(feat), 2, 2 * P, None, 0, _lib.ptr(vd), 64,
                  _lib.ptr(keep, dtype=torch.bool), P, _weights_struct(W), _lib.ptr(graw), _grads_struct(W),
                  _lib.ptr(dfeat), None, None, _lib.stream())
    torch.cuda.synchronize()
    print(json.dumps({"points": P, "reps": reps}))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "mlponly":
        mlp_only()
    elif len(sys.argv) > 1 and sys.argv[1] == "bwdws":
        bwd_only(int(sys.argv[2]) if len(sys.argv) > 2 else 192)
    elif len(sys.argv) > 1 and sys.argv[1] == "mlp":
        mlp_bench()
    elif len(sys.argv) > 1 and sys.argv[1] == "levels":
        levels_bench()
    else:
        main()
