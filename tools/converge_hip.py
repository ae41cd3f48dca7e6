"""Diagnostic (GPU box): the HIP path trained on F19's scene, initial state and batches, as
tests/test_gpu_converge.py trains it; writes every run's per-iteration training PSNR, the
checkpoint PSNRs and per-iteration table statistics (rows with a nonzero / exactly-zero gradient
per level, mean / max |dp| of the update per level) to an .npz for tests/diagnostics/converge_oracle.py's
counterpart on CPU.

usage: python tools/converge_hip.py --runs 6 --iters 120 --out gpurun_out/conv/hip.npz [--deterministic]
"""
import argparse
import ast
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import indoor_nerf_amd as nerf  # noqa: E402
from tables import blender_bbox, closed_form_table, convergence_rays  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=6)
    ap.add_argument("--iters", type=int, default=120)
    ap.add_argument("--out", default="gpurun_out/conv/hip.npz")
    ap.add_argument("--deterministic", action="store_true")
    ap.add_argument("--stats", action="store_true")
    ap.add_argument("--batch-seeds", default="", help="comma list: replay F19c's runs (ray batches drawn with "
                    "numpy RandomState(seed).choice, tests/golden/make_golden.py gen_converge_seeds); --runs per seed")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    gpu = torch.device("cuda:0")
    if a.deterministic:
        nerf.set_deterministic(True)
    g = np.load(os.path.join(ROOT, "tests", "golden", "f19_converge.npz"))
    c = ast.literal_eval(str(g["config"]))
    lo, hi = blender_bbox()
    emb = nerf.HashEmbedder((torch.from_numpy(lo), torch.from_numpy(hi)), finest_resolution=1024).to(gpu)
    table = closed_form_table(scale=c["table_scale"], salt=c["table_salt"])

    def net():
        return nerf.NeRFSmall(num_layers=2, hidden_dim=64, geo_feat_dim=15, num_layers_color=3, hidden_dim_color=64,
                           input_ch=32, input_ch_views=16).to(gpu)

    coarse, fine = net(), net()
    sh = nerf.SHEncoder()
    nqf = lambda inputs, viewdirs, fn: nerf.run_network(inputs, viewdirs, fn, emb, sh)  # noqa: E731
    kw = dict(network_query_fn=nqf, perturb=1.0, N_importance=128, network_fine=fine, N_samples=64,
              network_fn=coarse, embed_fn=emb, use_viewdirs=True, white_bkgd=True, raw_noise_std=0.0,
              predict_normals=False, ndc=False, lindisp=False, near=2.0, far=6.0, pytest=True)
    kw_test = dict(kw, perturb=0.0, raw_noise_std=0.0, pytest=False)
    args = nerf.make_args(lrate=c["lrate"], lrate_decay=c["lrate_decay"], sparse_loss_weight=c["sparsity"],
                          tv_loss_weight=0.0, N_samples=64, N_importance=128, white_bkgd=True)
    (ro, rd, rgb), (eo, ed, ergb), (no, nd, nrgb) = (tuple(torch.from_numpy(x).to(gpu) for x in t)
                                                     for t in convergence_rays())
    batches = torch.from_numpy(g["batches"].astype(np.int64)).to(gpu)

    def psnr_of(o, d, target):
        with torch.no_grad():
            out, _, _, _ = nerf.render(800, 800, None, rays=(o, d), **kw_test)
            return (-10.0 * torch.log10(((out - target) ** 2).mean())).item()

    seeds = [int(v) for v in a.batch_seeds.split(",") if v] or [None]
    plan = [(s_, k) for s_ in seeds for k in range(a.runs)]
    res = {}
    for r, (seed, _) in enumerate(plan):
        if seed is not None:
            rng = np.random.RandomState(seed)
            bt = np.stack([rng.choice(ro.shape[0], c["R"], replace=False) for _ in range(c["iters"])])
            batches = torch.from_numpy(bt.astype(np.int64)).to(gpu)
            res[f"seed_{r}"] = np.array(seed)
            res[f"batch_sum_{r}"] = np.array(int(bt.astype(np.int64).sum()))
        with torch.no_grad():
            for i, e in enumerate(emb.embeddings):
                e.weight.copy_(torch.from_numpy(table[i]))
            for n, prefix in ((coarse, "coarse0_"), (fine, "fine0_")):
                for k, p in n.named_parameters():
                    p.copy_(torch.from_numpy(g[prefix + k.replace(".", "_")]))
        opt = nerf.RAdam([{"params": list(coarse.parameters()) + list(fine.parameters()), "weight_decay": 1e-6},
                          {"params": list(emb.parameters()), "eps": 1e-15}], lr=c["lrate"], betas=(0.9, 0.99))
        ev, nv, tr = [psnr_of(eo, ed, ergb)], [psnr_of(no, nd, nrgb)], []
        st = {k: [] for k in ("nonzero", "exact_zero", "dp_mean", "dp_max", "g_min_nonzero")}
        for it in range(1, a.iters + 1):
            idx = batches[it - 1]
            before = [e.weight.detach().clone() for e in emb.embeddings] if a.stats else None
            _, psnr = nerf.train_step((ro[idx], rd[idx]), rgb[idx], kw, opt, args, it)
            tr.append(psnr)
            if a.stats:
                nz, ez, dm, dx, gm = [], [], [], [], []
                for e, b in zip(emb.embeddings, before):
                    gr = e.weight.grad.abs().sum(-1)
                    nz.append(int((gr > 0).sum()))
                    ez.append(int((gr == 0).sum()))
                    dp = (e.weight.detach() - b).abs()
                    dm.append(float(dp.mean()))
                    dx.append(float(dp.max()))
                    gm.append(float(gr[gr > 0].min()) if bool((gr > 0).any()) else 0.0)
                for k, v in zip(st, (nz, ez, dm, dx, gm)):
                    st[k].append(v)
            if it % c["every"] == 0:
                ev.append(psnr_of(eo, ed, ergb))
                nv.append(psnr_of(no, nd, nrgb))
                print(f"run {r} it {it}: held-out {ev[-1]:.3f} novel {nv[-1]:.3f}", flush=True)
        res[f"eval_psnr_{r}"] = np.array(ev)
        res[f"novel_psnr_{r}"] = np.array(nv)
        res[f"train_psnr_{r}"] = torch.stack(tr).float().cpu().numpy().reshape(-1)
        for k, v in st.items():
            res[f"{k}_{r}"] = np.array(v)
    np.savez(a.out, **res)
    print("wrote", a.out)


if __name__ == "__main__":
    main()
