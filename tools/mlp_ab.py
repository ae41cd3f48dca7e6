#!/usr/bin/env python3
"""A/B timing of the MLP kernel generations (NERF_MLP=2: f32 MFMA, default: bf16x6) on the lego
fine pass (786,432 points): interleaved rounds in one process, HIP-event medians. JSON out."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import indoor_nerf_amd as nerf  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    net = nerf.NeRFSmall(2, 64, 15, 3, 64, 32, 16).to(dev)
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 786432
    x = torch.randn(P, 48, device=dev) * 0.3
    g = torch.randn(P, 4, device=dev)
    res = {}

    def fwd():
        with torch.no_grad():
            net(x)

    xx = x.clone().requires_grad_(True)

    def fwdbwd():
        raw = net(xx)
        raw.backward(g)

    vers = sys.argv[2].split(",") if len(sys.argv) > 2 else ["2", "3"]
    grads = {}
    for ver in vers:    # same inputs through each generation: max relative gradient difference
        os.environ["NERF_MLP"] = ver
        net.zero_grad()
        xx.grad = None
        fwdbwd()
        grads[ver] = [q.grad.detach().clone() for q in net.parameters()] + [xx.grad.detach().clone()]
    for ver in vers[1:]:
        res[f"maxrel v{ver} vs v{vers[0]}"] = [max(float((a - b).abs().max() / b.abs().max().clamp_min(1e-30)) for a, b in zip(grads[ver], grads[vers[0]]))]
    for rnd in range(5):
        for ver in vers:
            os.environ["NERF_MLP"] = ver
            for name, fn in (("fwd", fwd), ("fwd+bwd", fwdbwd)):
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
                res.setdefault(f"v{ver} {name}", []).append(float(np.median(ts)))
    print(json.dumps({k: float("%.4g" % float(np.median(v))) for k, v in res.items()}))


if __name__ == "__main__":
    main()
