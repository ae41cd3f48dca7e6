#!/usr/bin/env python3
"""What tests/test_gpu_dist.py::test_dp_shards_match_one_batch measures, printed per tensor, so its
bars can be set from measurements: the one-process 4,096-ray side against the two-rank 2 x 2,048 side
(each rank on its own half of the CUs), default and deterministic mode; the deterministic two-rank
side run twice (bitwise reproducibility). JSON: argv[1]."""
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

import test_gpu_dist as t  # noqa: E402


def _run(world, overlap, det):
    d = tempfile.mkdtemp()
    mp.start_processes(t._dp_worker, args=(world, t._free_port(), d, 4096, overlap, det), nprocs=world, join=True,
                       start_method="spawn")
    tag = f"dp{world}{'o' if overlap else ''}{'d' if det else ''}"
    return [torch.load(os.path.join(d, f"{tag}_{r}.pt"), weights_only=True) for r in range(world)]


def _grad_stats(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    err = (a - b).abs()
    m = float(a.abs().max())
    out = {"max_err_over_max": float(err.max()) / m if m else 0.0,
           "n": a.numel()}
    for rel, absf in ((1e-6, 1e-6), (1e-5, 1e-6), (1e-5, 1e-5), (1e-4, 1e-5)):
        out[f"off_{rel:g}_{absf:g}"] = int((err > rel * a.abs() + absf * m).sum())
    return out


def _param_stats(a, b, p0):
    err = (b - a).abs()
    bad = err > 2e-5 * a.abs() + 1e-7
    step = float((a - p0).abs().max())
    return {"bad": int(bad.sum()), "n": a.numel(), "max_err_over_step": float(err.max()) / step if step else 0.0}


def main():
    res = {}
    for det in (False, True):
        one = _run(1, False, det)[0]
        runs = [_run(2, True, det) for _ in range(2 if det else 1)]
        r0 = runs[0][0]
        mode = "deterministic" if det else "default"
        res[mode] = {
            "grads": [_grad_stats(a, b) for a, b in zip(one["grads"], r0["grads"])],
            "params": [_param_stats(a, b, p0) for a, b, p0 in zip(one["params"], r0["params"], one["params0"])],
            "ranks_equal": all(torch.equal(x, y) for x, y in zip(runs[0][0]["params"], runs[0][1]["params"])),
        }
        if det:
            res[mode]["two_runs_bitwise"] = {
                "grads": all(torch.equal(x, y) for x, y in zip(runs[0][0]["grads"], runs[1][0]["grads"])),
                "params": all(torch.equal(x, y) for x, y in zip(runs[0][0]["params"], runs[1][0]["params"])),
                "losses": runs[0][0]["losses"] == runs[1][0]["losses"]}
        print(mode, "params bad:", [p["bad"] for p in res[mode]["params"]], flush=True)
        print(mode, "table grads off (1e-5 rel + 1e-6 of max):", [g["off_1e-05_1e-06"] for g in res[mode]["grads"][10:]],
              "(1e-6 rel + 1e-6 of max):", [g["off_1e-06_1e-06"] for g in res[mode]["grads"][10:]], flush=True)
        print(mode, "max err / max |g| per table:", [f"{g['max_err_over_max']:.1e}" for g in res[mode]["grads"][10:]],
              flush=True)
        if det:
            print(mode, "two two-rank runs bitwise:", res[mode]["two_runs_bitwise"], flush=True)
    json.dump(res, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
