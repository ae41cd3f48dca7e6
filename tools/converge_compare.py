#!/usr/bin/env python3
"""Ensemble comparison for the convergence diagnostics: F19's six reference runs against a set of
runs (tools/converge_oracle.py or tools/converge_hip.py outputs), per checkpoint: mean difference,
its standard error, and per 10-iteration window of training PSNR.

usage: converge_compare.py run1.npz run2.npz ...   (converge_hip.py files hold several runs: *_0.._5)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def runs_of(path):
    d = np.load(path)
    if "eval_psnr" in d:
        return [{k: d[k] for k in ("eval_psnr", "novel_psnr", "train_psnr")}]
    out, r = [], 0
    while f"eval_psnr_{r}" in d:
        out.append({k: d[f"{k}_{r}"] for k in ("eval_psnr", "novel_psnr", "train_psnr")})
        r += 1
    return out


def main():
    g = np.load(os.path.join(ROOT, "tests", "golden", "f19_converge.npz"))
    tags = ("", "_b", "_c", "_d", "_e", "_f")
    runs = [r for p in sys.argv[1:] for r in runs_of(p)]
    n_ev = min(len(r["eval_psnr"]) for r in runs)
    n_tr = min(len(r["train_psnr"]) for r in runs)
    print(f"{len(runs)} runs vs 6 reference runs, {n_tr} iterations")
    for name in ("eval_psnr", "novel_psnr"):
        ref = np.stack([g[name + t][:n_ev] for t in tags])
        hip = np.stack([r[name][:n_ev] for r in runs])
        d = hip.mean(0) - ref.mean(0)
        se = np.sqrt(ref.var(0, ddof=1) / len(ref) + hip.var(0, ddof=1) / max(1, len(hip)))
        print(name, " ".join(f"{it * 20}:{x:+.3f}({s:.3f})" for it, (x, s) in enumerate(zip(d, se))))
    w = 10
    ref = np.stack([g["train_psnr" + t][:n_tr] for t in tags]).reshape(6, -1, w).mean(2)
    hip = np.stack([r["train_psnr"][:n_tr] for r in runs]).reshape(len(runs), -1, w).mean(2)
    d = hip.mean(0) - ref.mean(0)
    se = np.sqrt(ref.var(0, ddof=1) / 6 + hip.var(0, ddof=1) / max(1, len(hip)))
    print("train (10-it windows)", " ".join(f"{(i + 1) * w}:{x:+.3f}({s:.3f})" for i, (x, s) in enumerate(zip(d, se))))
    first = [int(np.argmax(np.abs(r["train_psnr"][:n_tr] - g["train_psnr"][:n_tr]) > 1e-4)) + 1 for r in runs]
    print("first iteration differing from reference run 0 by > 1e-4 dB:", first)


if __name__ == "__main__":
    main()
