#!/usr/bin/env python3
"""Ensemble comparison for the convergence diagnostics: reference runs (F19's six thread-count runs,
plus F19b's rounding-perturbed runs with --ref f19,f19b) against a set of runs (tests/diagnostics/converge_oracle.py
or tools/converge_hip.py outputs, or another reference set with --vs), per checkpoint: mean difference
and its standard error; per 10-iteration window of training PSNR; and the late-phase (iterations
200-300) means per metric.

usage: converge_compare.py [--ref f19,f19b] [--vs f19b] run1.npz run2.npz ...
       (converge_hip.py files hold several runs: *_0, *_1, ...)
"""
import argparse
import glob
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
NAMES = ("eval_psnr", "novel_psnr", "train_psnr")


def runs_of(path):
    d = np.load(path)
    if "eval_psnr" in d:
        return [{k: d[k] for k in NAMES}]
    out, r = [], 0
    while f"eval_psnr_{r}" in d:
        out.append({k: d[f"{k}_{r}"] for k in NAMES})
        r += 1
    return out


def reference_runs(which):
    """F19's six runs and/or F19b's perturbed runs (the merged file or its parts)."""
    out = []
    if "f19" in which:
        g = np.load(os.path.join(GOLD, "f19_converge.npz"))
        out += [{k: g[k + t] for k in NAMES} for t in ("", "_b", "_c", "_d", "_e", "_f")]
    if "f19b" in which:
        files = [os.path.join(GOLD, "f19b_converge.npz")]
        if not os.path.exists(files[0]):
            files = sorted(glob.glob(os.path.join(GOLD, "f19b_converge_part*.npz")))
        for f in files:
            z = np.load(f)
            for s in z["seeds"]:
                out.append({k: z[f"{k}_n{int(s)}"] for k in NAMES})
    return out


def compare(ref, runs, label):
    n_ev = min(len(r["eval_psnr"]) for r in runs + ref)
    n_tr = min(len(r["train_psnr"]) for r in runs + ref)
    print(f"{label}: {len(runs)} runs vs {len(ref)} reference runs, {n_tr} iterations")
    for name in ("eval_psnr", "novel_psnr"):
        R = np.stack([r[name][:n_ev] for r in ref])
        H = np.stack([r[name][:n_ev] for r in runs])
        d = H.mean(0) - R.mean(0)
        se = np.sqrt(R.var(0, ddof=1) / len(R) + H.var(0, ddof=1) / len(H))
        print(name, " ".join(f"{it * 20}:{x:+.3f}({s:.3f})" for it, (x, s) in enumerate(zip(d, se))))
    w = 10
    R = np.stack([r["train_psnr"][:n_tr] for r in ref]).reshape(len(ref), -1, w).mean(2)
    H = np.stack([r["train_psnr"][:n_tr] for r in runs]).reshape(len(runs), -1, w).mean(2)
    d = H.mean(0) - R.mean(0)
    se = np.sqrt(R.var(0, ddof=1) / len(R) + H.var(0, ddof=1) / len(H))
    print("train (10-it windows)", " ".join(f"{(i + 1) * w}:{x:+.3f}({s:.3f})" for i, (x, s) in enumerate(zip(d, se))))
    if n_tr >= 300:
        for name in NAMES:
            if name == "train_psnr":
                lr_ = np.array([r[name][200:300].mean() for r in ref])
                lh = np.array([r[name][200:300].mean() for r in runs])
            else:
                lr_ = np.array([r[name][10:16].mean() for r in ref])
                lh = np.array([r[name][10:16].mean() for r in runs])
            se = np.sqrt(lr_.var(ddof=1) / len(lr_) + lh.var(ddof=1) / len(lh))
            print(f"late {name}: ref {lr_.mean():.3f} (sd {lr_.std(ddof=1):.3f}) runs {lh.mean():.3f} "
                  f"(sd {lh.std(ddof=1):.3f}) d {lh.mean() - lr_.mean():+.3f} se {se:.3f}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="f19")
    ap.add_argument("--vs", default="")
    ap.add_argument("runs", nargs="*")
    a = ap.parse_args()
    ref = reference_runs(a.ref.split(","))
    runs = [r for p in a.runs for r in runs_of(p)] + (reference_runs(a.vs.split(",")) if a.vs else [])
    compare(ref, runs, f"{','.join(a.runs) or a.vs} vs {a.ref}")


if __name__ == "__main__":
    main()
