#!/usr/bin/env python3
"""F19d (test infrastructure): reference-algorithm training runs of F19c's kind — F19's initial state
and hyper-parameters, each run's ray batches drawn with its own seed — computed by the ORACLE
(oracle/nerf_oracle.py, the float32 PyTorch-CPU restatement of the reference) instead of the reference
itself, so that they can run where /root/reference is absent (the GPU box's CPU cores).

Why the oracle stands in for the reference here: at a matching thread count it reproduces the
reference's own training runs through the chaotic regime — F19's 2-thread run to 1.6e-6 dB over 100
iterations, and F19c's seed runs (make_golden.py gen_converge_seeds, 2 threads) as
tests/test_oracle_golden.py::test_oracle_reproduces_reference_seed_run checks on a saved prefix. A
different CPU (its BLAS kernels) or thread count is another rounding of the same algorithm, i.e.
another sample of the reference's run-to-run distribution, like F19's thread-count runs.

usage: make_oracle_converge.py OUT_DIR SEED0 N_SEEDS [PROCS] [THREADS]
   writes OUT_DIR/f19d_seed{S}.npz per finished run (eval/novel/train PSNR, batch checksum); then
   make_oracle_converge.py merge OUT_DIR  ->  tests/golden/f19d_converge.npz
"""
import ast
import math
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)


def oracle_run(seed, threads, iters=None, log=None):
    """One oracle training run of F19 with batches from RandomState(seed) (as gen_converge_seeds)."""
    import torch
    from oracle import nerf_oracle as orc
    from tables import blender_bbox, closed_form_table, convergence_rays
    torch.set_num_threads(threads)
    g = np.load(os.path.join(HERE, "f19_converge.npz"))
    c = ast.literal_eval(str(g["config"]))
    iters = iters or c["iters"]
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
    (ro, rd, rgb), (eo, ed, ergb), (no, nd, nrgb) = (tuple(torch.from_numpy(x) for x in t) for t in convergence_rays())
    rng = np.random.RandomState(seed)
    batches = np.stack([rng.choice(ro.shape[0], c["R"], replace=False) for _ in range(c["iters"])])

    def psnr_of(o, d, target):
        with torch.no_grad():
            out = orc.render_rays(o, d, orc.viewdirs_of(d), 2.0, 6.0, cw, fw, tabs, lo, hi, res, perturb=0.0)
            return float(-10.0 * torch.log10(((out["rgb_map"] - target) ** 2).mean()))

    ev, nv, tr = [psnr_of(eo, ed, ergb)], [psnr_of(no, nd, nrgb)], []
    for it in range(1, iters + 1):
        idx = torch.from_numpy(batches[it - 1].astype(np.int64))
        o, d, t = ro[idx], rd[idx], rgb[idx]
        for p in tabs + list(cw.values()) + list(fw.values()):
            p.grad = None
        out = orc.render_rays(o, d, orc.viewdirs_of(d), 2.0, 6.0, cw, fw, tabs, lo, hi, res)
        img = ((out["rgb_map"] - t) ** 2).mean()
        loss = img + ((out["rgb0"] - t) ** 2).mean()
        loss = loss + c["sparsity"] * (out["sparsity_loss"].sum() + out["sparsity_loss0"].sum())
        loss.backward()
        opt.step()
        lr = c["lrate"] * (0.1 ** (it / (c["lrate_decay"] * 1000)))
        for grp in opt.groups:
            grp["lr"] = lr
        tr.append(float(-10.0 * math.log10(float(img))))
        if it % c["every"] == 0:
            ev.append(psnr_of(eo, ed, ergb))
            nv.append(psnr_of(no, nd, nrgb))
            if log:
                print(f"seed {seed} it {it}: train {tr[-1]:.3f} held-out {ev[-1]:.3f} novel {nv[-1]:.3f}", file=log,
                      flush=True)
    return dict(eval_psnr=np.array(ev), novel_psnr=np.array(nv), train_psnr=np.array(tr),
                batch_sum=np.array(int(batches.astype(np.int64).sum())))


def _worker(job):
    out_dir, seed, threads = job
    t0 = time.time()
    r = oracle_run(seed, threads, log=sys.stdout)
    np.savez(os.path.join(out_dir, f"f19d_seed{seed}.npz"), seed=np.array(seed), threads=np.array(threads),
             seconds=np.array(time.time() - t0), **r)
    return seed


def merge(out_dir):
    files = sorted(f for f in os.listdir(out_dir) if f.startswith("f19d_seed") and f.endswith(".npz"))
    d, seeds = {}, []
    for f in files:
        z = np.load(os.path.join(out_dir, f))
        s = int(z["seed"])
        seeds.append(s)
        for k in ("eval_psnr", "novel_psnr", "train_psnr", "batch_sum"):
            d[f"{k}_s{s}"] = z[k]
    old = os.path.join(HERE, "f19d_converge.npz")
    if os.path.exists(old):   # runs of earlier calls stay
        z = np.load(old)
        for s in z["seeds"]:
            if int(s) not in seeds:
                seeds.append(int(s))
                for k in ("eval_psnr", "novel_psnr", "train_psnr", "batch_sum"):
                    d[f"{k}_s{int(s)}"] = z[f"{k}_s{int(s)}"]
    np.savez_compressed(old, seeds=np.array(sorted(seeds)), **d)
    print("f19d:", len(seeds), "runs")


def main():
    if sys.argv[1] == "merge":
        merge(sys.argv[2])
        return
    out_dir, seed0, n = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    procs = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    threads = int(sys.argv[5]) if len(sys.argv) > 5 else 2
    os.makedirs(out_dir, exist_ok=True)
    from concurrent.futures import ProcessPoolExecutor
    jobs = [(out_dir, s, threads) for s in range(seed0, seed0 + n)]
    with ProcessPoolExecutor(max_workers=procs) as ex:
        for s in ex.map(_worker, jobs):
            print("done seed", s, flush=True)


if __name__ == "__main__":
    main()
