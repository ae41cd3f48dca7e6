#!/usr/bin/env python3
"""Run the F19 convergence training (tests/test_gpu_converge.py) K times on the HIP path and print
each run's late-phase (iterations 200-300) mean PSNR next to the reference runs' (diagnostic)."""
import ast
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import indoor_nerf_amd as nerf  # noqa: E402
from tables import blender_bbox, closed_form_table, convergence_rays  # noqa: E402


def main(K=6, det=False):
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "f19_converge.npz")))
    c = ast.literal_eval(str(g["config"]))
    gpu = torch.device("cuda:0")
    lo, hi = blender_bbox()
    emb = nerf.HashEmbedder((torch.from_numpy(lo), torch.from_numpy(hi)), finest_resolution=1024).to(gpu)
    table = closed_form_table(scale=c["table_scale"], salt=c["table_salt"])
    nets = [nerf.NeRFSmall(2, 64, 15, 3, 64, 32, 16).to(gpu) for _ in range(2)]
    sh = nerf.SHEncoder()
    nqf = lambda inputs, viewdirs, fn: nerf.run_network(inputs, viewdirs, fn, emb, sh)  # noqa: E731
    kw = dict(network_query_fn=nqf, perturb=1.0, N_importance=128, network_fine=nets[1], N_samples=64,
              network_fn=nets[0], embed_fn=emb, use_viewdirs=True, white_bkgd=True, raw_noise_std=0.0,
              predict_normals=False, ndc=False, lindisp=False, near=2.0, far=6.0, pytest=True)
    kw_test = dict(kw, perturb=0.0, pytest=False)
    args = nerf.make_args(lrate=c["lrate"], lrate_decay=c["lrate_decay"], sparse_loss_weight=c["sparsity"],
                          tv_loss_weight=0.0, N_samples=64, N_importance=128, white_bkgd=True)
    (ro, rd, rgb), (eo, ed, ergb), (no, nd, nrgb) = [tuple(torch.from_numpy(a).to(gpu) for a in s)
                                                     for s in convergence_rays()]
    batches = torch.from_numpy(g["batches"].astype(np.int64)).to(gpu)
    nerf.set_deterministic(det)

    def psnr_of(o, d, t):
        with torch.no_grad():
            out, _, _, _ = nerf.render(800, 800, None, rays=(o, d), **kw_test)
            return (-10.0 * torch.log10(((out - t) ** 2).mean())).item()

    late = g["eval_iters"] >= 200
    res = []
    for k in range(K):
        with torch.no_grad():
            for i, e in enumerate(emb.embeddings):
                e.weight.copy_(torch.from_numpy(table[i]))
            for net, prefix in zip(nets, ("coarse0_", "fine0_")):
                for name, p in net.named_parameters():
                    p.copy_(torch.from_numpy(g[prefix + name.replace(".", "_")]))
        opt = nerf.RAdam([{"params": [p for n in nets for p in n.parameters()], "weight_decay": 1e-6},
                          {"params": list(emb.parameters()), "eps": 1e-15}], lr=c["lrate"], betas=(0.9, 0.99))
        ev, nv, tr = [psnr_of(eo, ed, ergb)], [psnr_of(no, nd, nrgb)], []
        for it in range(1, c["iters"] + 1):
            _, p = nerf.train_step((ro[batches[it - 1]], rd[batches[it - 1]]), rgb[batches[it - 1]], kw, opt, args, it)
            tr.append(p)
            if it % c["every"] == 0:
                ev.append(psnr_of(eo, ed, ergb))
                nv.append(psnr_of(no, nd, nrgb))
        tr = torch.stack(tr).float().cpu().numpy().reshape(-1)
        res.append(dict(eval=float(np.mean(np.array(ev)[late])), novel=float(np.mean(np.array(nv)[late])),
                        train=float(tr[199:].mean()), eval_curve=[round(x, 3) for x in ev]))
        print(json.dumps(res[-1]), flush=True)
    refs = {name: [float(g[name + s][late].mean()) for s in ("", "_b", "_c", "_d", "_e", "_f") if name + s in g]
            for name in ("eval_psnr", "novel_psnr")}
    refs["train_psnr"] = [float(g["train_psnr" + s][199:].mean()) for s in ("", "_b", "_c", "_d", "_e", "_f") if "train_psnr" + s in g]
    print(json.dumps({"hip_mean": {k: float(np.mean([r[k] for r in res])) for k in ("eval", "novel", "train")},
                      "hip_std": {k: float(np.std([r[k] for r in res], ddof=1)) for k in ("eval", "novel", "train")},
                      "ref": refs, "det": det}))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 6, len(sys.argv) > 2 and sys.argv[2] == "det")
