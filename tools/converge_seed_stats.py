#!/usr/bin/env python3
"""Paired comparison over batch seeds (F19c): per seed the reference run (tests/golden/f19c_converge.npz
or its parts) against the mean of the HIP runs that replay the same batches (tools/converge_hip.py
--batch-seeds ...). Prints per metric the late-phase (iterations 100-300) difference per seed, their
mean D, its standard error over seeds, and per checkpoint the paired mean difference with its t value.
With --json, writes the summary tests/test_gpu_converge.py commits as profiles/r03_psnr_vs_reference.json.

usage: converge_seed_stats.py gpurun_out/conv/hip_seeds.npz [--json out.json --commit SHA]
"""
import argparse
import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
NAMES = ("eval_psnr", "novel_psnr", "train_psnr")


def reference_seed_runs():
    """F19c (the reference) and F19d (the oracle) runs keyed by batch seed; run["source"] says which."""
    files = [os.path.join(GOLD, "f19c_converge.npz")]
    if not os.path.exists(files[0]):
        files = []
    files += sorted(glob.glob(os.path.join(GOLD, "f19c_converge_part*.npz")))
    if os.path.exists(os.path.join(GOLD, "f19d_converge.npz")):
        files.append(os.path.join(GOLD, "f19d_converge.npz"))
    out = {}
    for f in files:
        z = np.load(f)
        for s in z["seeds"]:
            s = int(s)
            out[s] = {k: z[f"{k}_s{s}"] for k in NAMES}
            out[s]["batch_sum"] = int(z[f"batch_sum_s{s}"])
            out[s]["source"] = "oracle" if "f19d" in os.path.basename(f) else "reference"
    return out


LATE = 100   # tests/test_gpu_converge.py LATE


def late(name, x):
    """Late-phase mean: checkpoints at iterations LATE..300, or training batches LATE+1..300."""
    return x[..., LATE:].mean(-1) if name == "train_psnr" else x[..., LATE // 20:].mean(-1)


def paired(ref, hip):
    """ref: {seed: run}, hip: {seed: [runs]} -> per metric dict of late-phase statistics."""
    seeds = sorted(s for s in ref if s in hip)
    res = {"seeds": seeds}
    for name in NAMES:
        d = np.array([late(name, np.stack([r[name] for r in hip[s]])).mean() - late(name, ref[s][name]) for s in seeds])
        res[name] = dict(per_seed=d, D=float(d.mean()), se=float(d.std(ddof=1) / np.sqrt(len(d))),
                         reference_db=float(np.mean([late(name, ref[s][name]) for s in seeds])),
                         hip_db=float(np.mean([late(name, np.stack([r[name] for r in hip[s]])).mean() for s in seeds])))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("hip")
    ap.add_argument("--json", default="")
    ap.add_argument("--commit", default="")
    a = ap.parse_args()
    ref = reference_seed_runs()
    h = np.load(a.hip)
    hip, r = {}, 0
    while f"seed_{r}" in h:
        s = int(h[f"seed_{r}"])
        hip.setdefault(s, []).append({k: h[f"{k}_{r}"] for k in NAMES})
        if s in ref:
            assert int(h[f"batch_sum_{r}"]) == ref[s]["batch_sum"], f"seed {s}: different batches"
        r += 1
    res = paired(ref, hip)
    print(f"{len(res['seeds'])} seeds, {len(next(iter(hip.values())))} HIP runs per seed")
    for name in NAMES:
        v = res[name]
        print(f"{name}: late-phase reference {v['reference_db']:.3f} HIP {v['hip_db']:.3f} D {v['D']:+.3f} "
              f"se {v['se']:.3f} per seed {np.round(v['per_seed'], 3).tolist()}")
    seeds = res["seeds"]
    for name in ("eval_psnr", "novel_psnr"):
        dk = np.stack([np.stack([r[name] for r in hip[s]]).mean(0) - ref[s][name] for s in seeds])
        t = dk.mean(0) / np.maximum(dk.std(0, ddof=1) / np.sqrt(len(seeds)), 1e-12)
        print(name, "per checkpoint D(t):", " ".join(f"{20 * i}:{m:+.3f}({x:+.1f})" for i, (m, x) in enumerate(zip(dk.mean(0), t))))
    if a.json:
        # top level: the reference's own runs (F19c) only; all_seeds adds the oracle's F19d runs
        rref = paired({s: v for s, v in ref.items() if v["source"] == "reference"}, hip)
        summ = lambda r: {name: {"d_db": round(r[name]["D"], 4), "se_db": round(r[name]["se"], 4),  # noqa: E731
                                 "reference_db": round(r[name]["reference_db"], 3), "hip_db": round(r[name]["hip_db"], 3)}
                          for name in NAMES}
        out = summ(rref)
        out["all_seeds"] = summ(res)
        out["all_seeds"]["note"] = (f"{len(seeds)} seeds: {len(rref['seeds'])} reference runs (F19c) + "
                                    f"{len(seeds) - len(rref['seeds'])} ORACLE runs (F19d, oracle/nerf_oracle.py on the "
                                    "GPU box's CPU cores, pinned to the reference by tests/test_oracle_golden.py)")
        out["design"] = (f"F19c: {len(rref['seeds'])} runs of the REFERENCE with their own ray batches (seeds "
                         f"{rref['seeds']}) vs {len(next(iter(hip.values())))} HIP runs replaying each; late-phase "
                         f"(iterations {LATE}-300) mean PSNR difference averaged over seeds")
        if a.commit:
            out["commit"] = a.commit
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from bench import product_tree_sha
        out["tree_sha"] = product_tree_sha()    # bench.py marks the result stale once the tree moves on
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
