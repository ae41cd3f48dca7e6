#!/usr/bin/env python3
"""Run-to-run reproducibility of the deterministic DP rehearsal (tests/test_gpu_dist.py's _dp_worker:
2 gloo ranks on one GPU, ZeRO-1 with overlap, deterministic mode, 7 iterations) and of the
one-process deterministic reference side: two runs of each, compared bit for bit. JSON out: argv[1]."""
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


def dp2_runs(dst, K):
    """--runs K: K runs of the deterministic two-rank rehearsal (_dp_worker, ZeRO-1 with overlap and the
    gated all-gather), each compared bit for bit with the first: one-iteration all-reduced gradients,
    parameters after 7 steps, losses."""
    res, first = [], None
    for k in range(K):
        d = tempfile.mkdtemp()
        mp.start_processes(t._dp_worker, args=(2, t._free_port(), d, 4096, True, True), nprocs=2, join=True,
                           start_method="spawn")
        cur = [torch.load(os.path.join(d, f"dp2od_{r}.pt"), weights_only=True) for r in range(2)]
        if first is None:
            first = cur
            continue
        row = {f"rank{r}_{w}": [int((x != y).sum()) for x, y in zip(first[r][w], cur[r][w])]
               for r in range(2) for w in ("grads", "params")}
        row["losses_equal"] = all(first[r]["losses"] == cur[r]["losses"] for r in range(2))
        res.append(row)
        print(f"run {k}:", json.dumps({k_: v for k_, v in row.items() if not isinstance(v, list) or any(v)}),
              flush=True)
    json.dump({"runs": K, "vs_run0": res}, open(dst, "w"), indent=1)


def main():
    if "--runs" in sys.argv:
        return dp2_runs(sys.argv[1], int(sys.argv[sys.argv.index("--runs") + 1]))
    out = {}
    runs = {}
    for tag, world, overlap in (("one", 1, False), ("dp2", 2, True)):
        for k in range(2):
            d = tempfile.mkdtemp()
            mp.start_processes(t._dp_worker, args=(world, t._free_port(), d, 4096, overlap, True), nprocs=world,
                               join=True, start_method="spawn")
            name = ("dp2od" if world == 2 else "dp1d") + "_0.pt"
            runs[(tag, k)] = torch.load(os.path.join(d, name), weights_only=True)
    for tag in ("one", "dp2"):
        a, b = runs[(tag, 0)], runs[(tag, 1)]
        out[tag] = {
            "grads_identical": [bool(torch.equal(x, y)) for x, y in zip(a["grads"], b["grads"])],
            "params_identical": [bool(torch.equal(x, y)) for x, y in zip(a["params"], b["params"])],
            "params_differing_elements": [int((x != y).sum()) for x, y in zip(a["params"], b["params"])],
            "losses": [a["losses"], b["losses"]]}
    json.dump(out, open(sys.argv[1], "w"), indent=1)
    print(json.dumps({k: {"grads": all(v["grads_identical"]), "params": all(v["params_identical"])} for k, v in out.items()}))


if __name__ == "__main__":
    main()
