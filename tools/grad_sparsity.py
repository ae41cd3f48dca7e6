#!/usr/bin/env python3
"""Diagnostic (GPU box): how many samples of a training iteration receive an exactly-zero upstream
gradient from raw2outputs (composite backward). A sample with relu(sigma + noise) = 0 has alpha = 0,
weight 0 and a zero sigma gradient (run_nerf.py:364-386 autograd), so its whole raw-gradient row is 0
and the MLP backward and hash backward of that point contribute nothing. Prints, per iteration of the
bench's lego workload, the fraction of all-zero rows of the coarse and the fine pass.

usage: python tools/grad_sparsity.py [--steps 30] [--workload lego]
"""
import argparse
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--workload", default="lego")
    a = ap.parse_args()
    import bench
    import indoor_nerf_amd as nerf
    from indoor_nerf_amd.synthetic import blender_bbox, blender_rays
    rmod = importlib.import_module("indoor_nerf_amd.render")
    wl = bench.WORKLOADS[a.workload]
    dev = torch.device("cuda:0")
    lo, hi = blender_bbox()
    ro, rd = blender_rays(4096, seed=100)
    args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), **wl["args"])
    torch.manual_seed(0)
    nerf.manual_seed(1234)
    kw, _, _, grad_vars, opt = nerf.create_nerf(args, device=dev)
    kw.update(near=wl["near"], far=wl["far"])
    params = grad_vars + list(kw["embed_fn"].parameters())
    arena = nerf.GradArena(params, defer_tables=True)
    rays = (torch.from_numpy(ro).to(dev), torch.from_numpy(rd).to(dev))
    target = torch.rand(4096, 3, device=dev, generator=torch.Generator(device=dev).manual_seed(0))
    rec = []
    orig = rmod.CompositeFn.backward

    def spy(ctx, *grads):
        out = orig(ctx, *grads)
        g = out[0]
        rec.append(((g == 0).all(-1).float().mean().item(), g.shape[1]))
        return out
    rmod.CompositeFn.backward = staticmethod(spy)
    gen = torch.Generator().manual_seed(7)
    for it in range(1, a.steps + 1):
        rec.clear()
        nerf.train_step(rays, target, kw, opt, args, it, tv_generator=gen, zero_grad=arena.zero_)
        torch.cuda.synchronize()
        print(f"iteration {it}: zero-gradient sample fraction " +
              ", ".join(f"{S} samples/ray: {f:.3f}" for f, S in rec), flush=True)


if __name__ == "__main__":
    main()
