"""Diagnostic (GPU box): the table gradients of ONE training step of F19 (the initial state, batch 1),
HIP path vs the oracle: per level the rows with a nonzero gradient on one side only (and how large
those gradients are), sign disagreements and relative differences where both are nonzero. With
RAdam's eps 1e-15 every row with any nonzero gradient takes a full-size step, so the SET of rows is
what the first update depends on, not only the values.

The first-update tool's docstring follows.
The first RAdam update of F19's training, HIP path vs the oracle (the
reference's algorithm, pinned to the reference's own runs: tests/diagnostics/converge_oracle.py reproduces F19 to
1e-6 dB at a matching thread count), from the same initial state on the same batches. RAdam
(radam.py:58-92, betas (0.9, 0.99)) makes no update while N_sma < 5, i.e. for steps 1-5; step 6 is the
first update, and every HIP run agrees with every other one there while the first PSNR after it
(iteration 7) differs from the reference by ~0.08 dB. Per table level after step 6: the rows whose
update differs by more than half a full step (|dp| ~ lr: with eps 1e-15 any row with a nonzero
gradient history moves by ~lr), split by cause: exp_avg_sq zero on one side only (squares of tiny
gradients underflowing), exp_avg sign disagreement, or neither.

usage (GPU box): python tests/diagnostics/converge_first_update.py --steps 6 > out.json
"""
import argparse
import ast
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import indoor_nerf_amd as nerf  # noqa: E402
from oracle import nerf_oracle as orc  # noqa: E402
from tables import blender_bbox, closed_form_table, convergence_rays  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--it", type=int, default=1)
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    gpu = torch.device("cuda:0")
    g = np.load(os.path.join(ROOT, "tests", "golden", "f19_converge.npz"))
    c = ast.literal_eval(str(g["config"]))
    lo, hi = blender_bbox()
    table = closed_form_table(scale=c["table_scale"], salt=c["table_salt"])
    (ro, rd, rgb), _, _ = convergence_rays()
    idx = g["batches"].astype(np.int64)[a.it - 1]

    emb = nerf.HashEmbedder((torch.from_numpy(lo), torch.from_numpy(hi)), finest_resolution=1024).to(gpu)
    with torch.no_grad():
        for i, e in enumerate(emb.embeddings):
            e.weight.copy_(torch.from_numpy(table[i]))

    def net(prefix):
        n = nerf.NeRFSmall(num_layers=2, hidden_dim=64, geo_feat_dim=15, num_layers_color=3, hidden_dim_color=64,
                           input_ch=32, input_ch_views=16).to(gpu)
        with torch.no_grad():
            for k, p in n.named_parameters():
                p.copy_(torch.from_numpy(g[prefix + k.replace(".", "_")]))
        return n

    coarse, fine = net("coarse0_"), net("fine0_")
    sh = nerf.SHEncoder()
    nqf = lambda inputs, viewdirs, fn: nerf.run_network(inputs, viewdirs, fn, emb, sh)  # noqa: E731
    kw = dict(network_query_fn=nqf, perturb=1.0, N_importance=128, network_fine=fine, N_samples=64,
              network_fn=coarse, embed_fn=emb, use_viewdirs=True, white_bkgd=True, raw_noise_std=0.0,
              predict_normals=False, ndc=False, lindisp=False, near=2.0, far=6.0, pytest=True)
    args = nerf.make_args(lrate=c["lrate"], lrate_decay=c["lrate_decay"], sparse_loss_weight=c["sparsity"],
                          tv_loss_weight=0.0, N_samples=64, N_importance=128, white_bkgd=True)
    opt = nerf.RAdam([{"params": list(coarse.parameters()) + list(fine.parameters()), "weight_decay": 1e-6},
                      {"params": list(emb.parameters()), "eps": 1e-15}], lr=c["lrate"], betas=(0.9, 0.99))
    rog, rdg, rgbg = (torch.from_numpy(x).to(gpu) for x in (ro, rd, rgb))
    it_t = torch.from_numpy(idx).to(gpu)
    nerf.train_step((rog[it_t], rdg[it_t]), rgbg[it_t], kw, opt, args, 1)   # step 1: no update (N_sma < 5)
    torch.cuda.synchronize()
    hg = [e.weight.grad.detach().cpu() for e in emb.embeddings]
    hmlp = {k: p.grad.detach().cpu() for k, p in fine.named_parameters()}

    lo_t, hi_t = torch.from_numpy(lo), torch.from_numpy(hi)
    res = orc.level_resolutions(16, 1024)
    tabs = [torch.from_numpy(table[i]).clone().requires_grad_(True) for i in range(16)]
    cw = {k: torch.from_numpy(g["coarse0_" + k.replace(".", "_")]).clone().requires_grad_(True) for k in orc.MLP_KEYS}
    fw = {k: torch.from_numpy(g["fine0_" + k.replace(".", "_")]).clone().requires_grad_(True) for k in orc.MLP_KEYS}
    ro_t, rd_t, rgb_t = (torch.from_numpy(x) for x in (ro, rd, rgb))
    ii = torch.from_numpy(idx)
    o, d, t = ro_t[ii], rd_t[ii], rgb_t[ii]
    out = orc.render_rays(o, d, orc.viewdirs_of(d), 2.0, 6.0, cw, fw, tabs, lo_t, hi_t, res)
    loss = ((out["rgb_map"] - t) ** 2).mean() + ((out["rgb0"] - t) ** 2).mean()
    loss = loss + c["sparsity"] * (out["sparsity_loss"].sum() + out["sparsity_loss0"].sum())
    loss.backward()

    rep = {"it": a.it}
    for lvl in range(16):
        h, r = hg[lvl].reshape(-1), tabs[lvl].grad.reshape(-1)
        nh, nr = h != 0, r != 0
        both = nh & nr
        rel = ((h - r).abs() / r.abs())[both]
        rep[f"level{lvl}"] = dict(
            nonzero_hip=int(nh.sum()), nonzero_ref=int(nr.sum()), hip_only=int((nh & ~nr).sum()),
            ref_only=int((nr & ~nh).sum()),
            max_abs_hip_only=float(h[nh & ~nr].abs().max()) if bool((nh & ~nr).any()) else 0.0,
            max_abs_ref_only=float(r[nr & ~nh].abs().max()) if bool((nr & ~nh).any()) else 0.0,
            sign_differs=int(((h * r) < 0).sum()),
            rel_diff_q50=float(rel.quantile(0.5)) if rel.numel() else 0.0,
            rel_diff_q99=float(rel.quantile(0.99)) if rel.numel() else 0.0,
            rel_diff_gt_1em2=int((rel > 1e-2).sum()),
            max_abs_ref=float(r.abs().max()), min_abs_nonzero_ref=float(r[nr].abs().min()) if bool(nr.any()) else 0.0)
    rep["fine_mlp_rel_diff"] = {k: float((hmlp[k] - fw[k].grad).norm() / fw[k].grad.norm().clamp_min(1e-30))
                                for k in orc.MLP_KEYS}
    print(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
