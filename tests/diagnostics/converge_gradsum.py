"""Diagnostic (CPU, this container): the table gradient of ONE training batch summed two ways at the
same state of an F19 training run: in float32 in the reference's order (embedding_dense_backward) and
in float64 rounded once (the HIP owner pass's accumulation). Counts, per level, the rows whose fp32
sum is exactly zero while the fp64 sum is not (and the reverse), sign disagreements, and the RAdam
update either gradient would give a row touched for the first time (eps 1e-15: any nonzero gradient
is a full-size step, an exact zero none).

usage: python tests/diagnostics/converge_gradsum.py --iters 40 --threads 8 [--out stats.json]
"""
import argparse
import ast
import json
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from oracle import nerf_oracle as orc  # noqa: E402
from tables import blender_bbox, closed_form_table, convergence_rays  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    g = np.load(os.path.join(ROOT, "tests", "golden", "f19_converge.npz"))
    c = ast.literal_eval(str(g["config"]))
    lo, hi = (torch.from_numpy(v) for v in blender_bbox())
    res = orc.level_resolutions(16, 1024)
    table = closed_form_table(scale=c["table_scale"], salt=c["table_salt"])
    tabs = [torch.from_numpy(table[i]).clone().requires_grad_(True) for i in range(16)]
    cw = {k: torch.from_numpy(g["coarse0_" + k.replace(".", "_")]).clone().requires_grad_(True) for k in orc.MLP_KEYS}
    fw = {k: torch.from_numpy(g["fine0_" + k.replace(".", "_")]).clone().requires_grad_(True) for k in orc.MLP_KEYS}
    opt = orc.RAdamOracle([
        dict(params=list(cw.values()) + list(fw.values()), lr=c["lrate"], betas=(0.9, 0.99), eps=1e-8,
             weight_decay=1e-6),
        dict(params=tabs, lr=c["lrate"], betas=(0.9, 0.99), eps=1e-15, weight_decay=0.0)])
    (ro, rd, rgb), _, _ = (tuple(torch.from_numpy(x) for x in t) for t in convergence_rays())
    batches = torch.from_numpy(g["batches"].astype(np.int64))

    def grads(it, sum64):
        idx = batches[it - 1]
        o, d, t = ro[idx], rd[idx], rgb[idx]
        for p in tabs + list(cw.values()) + list(fw.values()):
            p.grad = None
        if sum64:
            import converge_oracle as co
            saved = orc.F
            co.apply_variants(["gsum64"])
        out = orc.render_rays(o, d, orc.viewdirs_of(d), 2.0, 6.0, cw, fw, tabs, lo, hi, res)
        loss = ((out["rgb_map"] - t) ** 2).mean() + ((out["rgb0"] - t) ** 2).mean()
        loss = loss + c["sparsity"] * (out["sparsity_loss"].sum() + out["sparsity_loss0"].sum())
        loss.backward()
        if sum64:
            orc.F = saved
        return [p.grad.clone() for p in tabs]

    report = {}
    for it in range(1, a.iters + 1):
        if it == a.iters:
            g32, g64 = grads(it, False), grads(it, True)
            for lvl in range(16):
                a32, a64 = g32[lvl], g64[lvl]
                z32, z64 = a32 == 0, a64 == 0
                both = ~z32 & ~z64
                rel = ((a32 - a64).abs() / a64.abs().clamp_min(1e-38))[both]
                report[f"level{lvl}"] = {
                    "nonzero_fp64": int((~z64).sum()),
                    "zero32_nonzero64": int((z32 & ~z64).sum()),
                    "nonzero32_zero64": int((~z32 & z64).sum()),
                    "sign_differs": int(((a32 * a64) < 0).sum()),
                    "rel_diff_gt_1e-3": int((rel > 1e-3).sum()),
                    "rel_diff_gt_0.5": int((rel > 0.5).sum()),
                }
            break
        for p in tabs + list(cw.values()) + list(fw.values()):
            p.grad = None
        idx = batches[it - 1]
        o, d, t = ro[idx], rd[idx], rgb[idx]
        out = orc.render_rays(o, d, orc.viewdirs_of(d), 2.0, 6.0, cw, fw, tabs, lo, hi, res)
        loss = ((out["rgb_map"] - t) ** 2).mean() + ((out["rgb0"] - t) ** 2).mean()
        loss = loss + c["sparsity"] * (out["sparsity_loss"].sum() + out["sparsity_loss0"].sum())
        loss.backward()
        opt.step()
        lr = c["lrate"] * (0.1 ** (it / (c["lrate_decay"] * 1000)))
        for grp in opt.groups:
            grp["lr"] = lr
    report["iteration"] = a.iters
    print(json.dumps(report, indent=1))
    if a.out:
        json.dump(report, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
