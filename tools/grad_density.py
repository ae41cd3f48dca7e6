#!/usr/bin/env python3
"""How much work the hash-grid backward does in the bench workload: fraction of table rows with a
non-zero gradient per level after one lego training step, for the reference init U(-1e-4, 1e-4)
(bench.py) and a trained-like N(0, 0.05^2) table; plus the step time of each (graph mode)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import indoor_nerf_amd as nerf  # noqa: E402
from indoor_nerf_amd.graphs import GraphedTrainStep  # noqa: E402
from indoor_nerf_amd.synthetic import blender_bbox, blender_rays  # noqa: E402


def run(init):
    dev = torch.device("cuda:0")
    lo, hi = blender_bbox()
    args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), finest_res=1024, N_samples=64,
                          N_importance=128, white_bkgd=True, perturb=1.0, lrate_decay=500, tv_loss_weight=1e-6)
    torch.manual_seed(0)
    kw, _, _, grad_vars, opt = nerf.create_nerf(args, device=dev)
    kw.update(near=2.0, far=6.0)
    emb = kw["embed_fn"]
    if init == "trained":
        with torch.no_grad():
            g = torch.Generator(device=dev).manual_seed(1)
            for e in emb.embeddings:
                e.weight.normal_(0.0, 0.05, generator=g)
    params = grad_vars + list(emb.parameters())
    arena = nerf.GradArena(params)
    ro, rd = blender_rays(4096, seed=100)
    rays = (torch.from_numpy(ro).to(dev), torch.from_numpy(rd).to(dev))
    target = torch.rand(4096, 3, device=dev)
    st = GraphedTrainStep(rays, target, kw, opt, args, zero_grad=arena.zero_)
    for i in range(1, 9):
        st(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(9, 29):
        st(i)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 20 * 1e3
    st.eager_step(29)
    torch.cuda.synchronize()
    dens = [round(float((e.weight.grad.abs().sum(-1) > 0).float().mean()), 4) for e in emb.embeddings]
    return {"ms_per_step": round(ms, 3), "rays_per_s": round(4096 / ms * 1e3), "nonzero_row_fraction": dens}


print(json.dumps({k: run(k) for k in ("reference", "trained")}))
