"""Diagnostic (GPU box): the first RAdam update of F19's training, HIP path vs the oracle (the
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
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    gpu = torch.device("cuda:0")
    g = np.load(os.path.join(ROOT, "tests", "golden", "f19_converge.npz"))
    c = ast.literal_eval(str(g["config"]))
    lo, hi = blender_bbox()
    table = closed_form_table(scale=c["table_scale"], salt=c["table_salt"])
    (ro, rd, rgb), _, _ = convergence_rays()
    batches = g["batches"].astype(np.int64)

    # ---- HIP path (as tests/test_gpu_converge.py)
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
    for it in range(1, a.steps + 1):
        idx = torch.from_numpy(batches[it - 1]).to(gpu)
        nerf.train_step((rog[idx], rdg[idx]), rgbg[idx], kw, opt, args, it)
    torch.cuda.synchronize()
    hip_p = [e.weight.detach().cpu() for e in emb.embeddings]
    hip_m = [opt.state[e.weight]["exp_avg"].cpu() for e in emb.embeddings]
    hip_v = [opt.state[e.weight]["exp_avg_sq"].cpu() for e in emb.embeddings]

    # ---- oracle (reference algorithm, float32 CPU)
    lo_t, hi_t = torch.from_numpy(lo), torch.from_numpy(hi)
    res = orc.level_resolutions(16, 1024)
    tabs = [torch.from_numpy(table[i]).clone().requires_grad_(True) for i in range(16)]
    cw = {k: torch.from_numpy(g["coarse0_" + k.replace(".", "_")]).clone().requires_grad_(True) for k in orc.MLP_KEYS}
    fw = {k: torch.from_numpy(g["fine0_" + k.replace(".", "_")]).clone().requires_grad_(True) for k in orc.MLP_KEYS}
    oopt = orc.RAdamOracle([
        dict(params=list(cw.values()) + list(fw.values()), lr=c["lrate"], betas=(0.9, 0.99), eps=1e-8,
             weight_decay=1e-6),
        dict(params=tabs, lr=c["lrate"], betas=(0.9, 0.99), eps=1e-15, weight_decay=0.0)])
    ro_t, rd_t, rgb_t = (torch.from_numpy(x) for x in (ro, rd, rgb))
    for it in range(1, a.steps + 1):
        idx = torch.from_numpy(batches[it - 1])
        o, d, t = ro_t[idx], rd_t[idx], rgb_t[idx]
        for p in tabs + list(cw.values()) + list(fw.values()):
            p.grad = None
        out = orc.render_rays(o, d, orc.viewdirs_of(d), 2.0, 6.0, cw, fw, tabs, lo_t, hi_t, res)
        loss = ((out["rgb_map"] - t) ** 2).mean() + ((out["rgb0"] - t) ** 2).mean()
        loss = loss + c["sparsity"] * (out["sparsity_loss"].sum() + out["sparsity_loss0"].sum())
        loss.backward()
        oopt.step()
        lr = c["lrate"] * (0.1 ** (it / (c["lrate_decay"] * 1000)))
        for grp in oopt.groups:
            grp["lr"] = lr

    rep = {"steps": a.steps, "lr": c["lrate"]}
    tot = dict(rows_step_differs=0, v_zero_hip_only=0, v_zero_ref_only=0, m_sign_differs=0)
    for lvl in range(16):
        p0 = torch.from_numpy(table[lvl])
        dh, dr = hip_p[lvl] - p0, tabs[lvl].detach() - p0
        st = oopt.state[id(tabs[lvl])]
        mr, vr = st["m"], st["v"]
        big = (dh - dr).abs() > 0.5 * c["lrate"]
        vz_h, vz_r = hip_v[lvl] == 0, vr == 0
        ms = (hip_m[lvl] * mr) < 0
        e = dict(rows_step_differs=int(big.sum()), v_zero_hip_only=int((vz_h & ~vz_r).sum()),
                 v_zero_ref_only=int((vz_r & ~vz_h).sum()), m_sign_differs=int(ms.sum()),
                 step_differs_with_v_zero_one_side=int((big & (vz_h ^ vz_r)).sum()),
                 step_differs_with_m_sign=int((big & ms).sum()),
                 moved_hip=int((dh.abs() > 0.5 * c["lrate"]).sum()), moved_ref=int((dr.abs() > 0.5 * c["lrate"]).sum()),
                 min_nonzero_v_ref=float(vr[vr > 0].min()) if bool((vr > 0).any()) else 0.0,
                 min_nonzero_v_hip=float(hip_v[lvl][hip_v[lvl] > 0].min()) if bool((hip_v[lvl] > 0).any()) else 0.0)
        rep[f"level{lvl}"] = e
        for k in tot:
            tot[k] += e[k]
    rep["total"] = tot
    print(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
