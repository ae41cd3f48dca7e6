#!/usr/bin/env python3
"""Timing of the batched MLP backward (nerf_mlp_bwd_batch) on the lego step's two nets: the fine
(4096 x 192 points) and the coarse (4096 x 64) net in one launch, HIP-event median per launch, plus a
checksum of every output (dfeat of both nets, the ten weight gradients) so that builds can be told to
compute the same thing. A/B of library builds: run once per build with NERF_HIP_LIB=<path>
(tools/build_variant.py). JSON out."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import indoor_nerf_amd as nerf  # noqa: E402
from indoor_nerf_amd import _lib  # noqa: E402


def make_job(P, spr, seed, dev):
    g = torch.Generator(device=dev).manual_seed(seed)
    net = nerf.NeRFSmall(2, 64, 15, 3, 64, 32, 16).to(dev)
    feat = (torch.randn(16, P, 2, device=dev, generator=g) * 0.3).contiguous()
    vd = torch.nn.functional.normalize(torch.randn(P // spr, 3, device=dev, generator=g), dim=-1).contiguous()
    keep = (torch.rand(P, device=dev, generator=g) > 0.05).contiguous()
    graw = torch.randn(P, 4, device=dev, generator=g).contiguous()
    dfeat = torch.empty_like(feat)
    ws = [p.detach() for p in net.mlp_weights()]
    grads = [torch.zeros_like(w) for w in ws]
    j = _lib.MlpBwdJob()
    j.feat, j.feat_stride_point, j.feat_stride_level = _lib.ptr(feat), 2, 2 * P
    j.viewdirs, j.samples_per_ray = _lib.ptr(vd), spr
    j.keep = _lib.ptr(keep, dtype=torch.bool)
    j.n_points = P
    w = _lib.MlpWeights()
    gs = _lib.MlpGrads()
    for name, t, gt in zip(("w0", "w1", "c0", "c1", "c2"), ws, grads):
        setattr(w, name, _lib.ptr(t).value)
        setattr(gs, name, _lib.ptr(gt).value)
    j.weights, j.grads = w, gs
    j.graw, j.dfeat = _lib.ptr(graw), _lib.ptr(dfeat)
    return j, dict(feat=feat, vd=vd, keep=keep, graw=graw, dfeat=dfeat, ws=ws, grads=grads)


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    jf, kf = make_job(4096 * 192, 192, 1, dev)
    jc, kc = make_job(4096 * 64, 64, 2, dev)
    arr = (_lib.MlpBwdJob * 2)(jf, jc)
    det = int(os.environ.get("NERF_DET", "0"))
    ws = torch.empty(int(_lib.load().nerf_mlp_bwd_det_workspace_bytes()) // 4, device=dev) if det else None

    def run():
        _lib.call("nerf_mlp_bwd_batch", arr, 2, _lib.ptr(ws, allow_none=True), 0 if ws is None else ws.numel() * 4,
                  _lib.stream())

    for k in (kf, kc):
        for t in k["grads"]:
            t.zero_()
    run()
    torch.cuda.synchronize()
    check = {"dfeat_f": float(kf["dfeat"].double().abs().sum()), "dfeat_c": float(kc["dfeat"].double().abs().sum()),
             "grads": [float(t.double().sum()) for k in (kf, kc) for t in k["grads"]]}
    def timed(fn):
        ts = []
        for rnd in range(5):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            for _ in range(20):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
        return ts

    # forward of the fine net (the lego step's larger MLP forward launch)
    raw = torch.empty(kf["feat"].shape[1], 4, device=dev)
    w = jf.weights

    def fwd():
        _lib.call("nerf_mlp_fwd", _lib.ptr(kf["feat"]), 2, 2 * raw.shape[0], None, 0, _lib.ptr(kf["vd"]), 192,
                  _lib.ptr(kf["keep"], dtype=torch.bool), raw.shape[0], ctypes.byref(w), _lib.ptr(raw), None,
                  _lib.stream())

    fwd()
    torch.cuda.synchronize()
    check["raw"] = float(raw.double().abs().sum())
    ts = timed(run)
    tf = timed(fwd)
    print(json.dumps({"lib": os.environ.get("NERF_HIP_LIB", "default"), "us_median": round(float(np.median(ts)) * 1e3, 1),
                      "us_min": round(float(np.min(ts)) * 1e3, 1), "fwd_us_median": round(float(np.median(tf)) * 1e3, 1),
                      "fwd_us_min": round(float(np.min(tf)) * 1e3, 1), "det": det, "check": check}))

if __name__ == "__main__":
    main()
