#!/usr/bin/env python3
"""Where the deterministic two-rank rehearsal stops being reproducible (tools/det_repro.py found its
one-iteration all-reduced table gradients differ run to run): part (a) of tests/test_gpu_dist.py's
_dp_worker only, deterministic mode, each rank's gradients saved BEFORE and AFTER the gloo all-reduce;
two runs with both ranks computing at once on the one GPU and two with the ranks taking turns
(barrier-separated), and twice two runs exactly as _dp_worker's part (a) ("nosync": no device sync or
barrier between the backward and the all-reduce; "pre" = stream-ordered device copies). --garbage: two
synchronised runs whose caching allocators start filled with different seeded random values. Per rank and parameter: elements that differ between the two runs. JSON: argv[1]."""
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


def _worker(rank, world, port, out, R, serial, garbage=None):
    t._init(rank, world, port)
    if serial == "nosync_garbage":
        serial = "nosync"
    if garbage is not None:   # leave seeded random bytes in the caching allocator's blocks: a read of
        g = torch.Generator(device="cuda:0").manual_seed(abs(garbage))   # memory no kernel wrote shows up
        x = torch.empty(1 << 31, device="cuda:0")                   # as a run-to-run difference
        x.uniform_(-1e3, 1e3, generator=g)
        del x
        if garbage < 0:   # the small pool too (requests <= 1 MiB come from 2 MiB segments of their own)
            xs = [torch.empty(n, device="cuda:0").uniform_(-1e3, 1e3, generator=g)
                  for n in [64, 1000, 4096, 16384, 65536, 262144] * 300]
            del xs
    import importlib
    import indoor_nerf_amd as nerf
    nerf.set_deterministic(True)
    from indoor_nerf_amd.model import forward_backward
    rmod = importlib.import_module("indoor_nerf_amd.render")
    from tables import synthetic_rays
    dev = torch.device("cuda:0")
    rmod.pytest_shard(rank, world)
    ro, rd = synthetic_rays(R, seed=21)
    target = torch.rand(R, 3, generator=torch.Generator().manual_seed(5))
    n = R // world
    rays = (torch.from_numpy(ro[rank * n:(rank + 1) * n]).to(dev), torch.from_numpy(rd[rank * n:(rank + 1) * n]).to(dev))
    tgt = target[rank * n:(rank + 1) * n].to(dev)
    args, kw, opt, params = t._f10_model(nerf, dev, world)
    arena = nerf.GradArena(params, defer_tables=True)

    def fb():
        forward_backward(rays, tgt, kw, opt, args, 1, loss_scale_sparsity=float(world),
                         tv_generator=torch.Generator().manual_seed(7), zero_grad=arena.zero_)
        torch.cuda.synchronize()

    if serial == "nosync":   # exactly as _dp_worker: no device sync or barrier between the backward and the
        forward_backward(rays, tgt, kw, opt, args, 1, loss_scale_sparsity=float(world),   # all-reduce
                         tv_generator=torch.Generator().manual_seed(7), zero_grad=arena.zero_)
        pre = [p.grad.detach().clone() for p in params]   # stream-ordered device copies
        arena.allreduce_mean()
        torch.cuda.synchronize()
        torch.save({"pre": [x.cpu() for x in pre], "post": [p.grad.detach().cpu().clone() for p in params]},
                   os.path.join(out, f"a_{rank}.pt"))
        torch.distributed.destroy_process_group()
        return
    torch.distributed.barrier()
    for r in range(world):
        if r == rank or not serial:
            if r == rank:
                fb()
        if serial:
            torch.distributed.barrier()
    if not serial:
        torch.distributed.barrier()
    pre = [p.grad.detach().cpu().clone() for p in params]
    arena.allreduce_mean()
    torch.cuda.synchronize()
    post = [p.grad.detach().cpu().clone() for p in params]
    torch.save({"pre": pre, "post": post}, os.path.join(out, f"a_{rank}.pt"))
    torch.distributed.destroy_process_group()


def nosync_runs(dst, K):
    """--nosync-runs K: K fresh two-rank process pairs run exactly as _dp_worker's part (a); every run's
    pre / post all-reduce gradients compared with the first run's."""
    res, first = [], None
    for k in range(K):
        d = tempfile.mkdtemp()
        mp.start_processes(_worker, args=(2, t._free_port(), d, 4096, "nosync", None), nprocs=2, join=True,
                           start_method="spawn")
        cur = [torch.load(os.path.join(d, f"a_{r}.pt"), weights_only=True) for r in range(2)]
        if first is None:
            first = cur
            continue
        row = {f"rank{r}_{w}": [int((x != y).sum()) for x, y in zip(first[r][w], cur[r][w])]
               for r in range(2) for w in ("pre", "post")}
        res.append(row)
        print(f"run {k}:", json.dumps({k_: v for k_, v in row.items() if any(v)}), flush=True)
    json.dump({"runs": K, "vs_run0": res}, open(dst, "w"), indent=1)


def garbage_runs(dst, K):
    """--garbage-runs K: K two-rank pairs run as _dp_worker's part (a) (nosync), each with the large
    AND the small pool of the caching allocator filled with another seed's random values first;
    pre / post all-reduce gradients compared with the first run's."""
    res, first = [], None
    for k in range(K):
        d = tempfile.mkdtemp()
        mp.start_processes(_worker, args=(2, t._free_port(), d, 4096, "nosync_garbage", -(101 + k)), nprocs=2,
                           join=True, start_method="spawn")
        cur = [torch.load(os.path.join(d, f"a_{r}.pt"), weights_only=True) for r in range(2)]
        if first is None:
            first = cur
            continue
        row = {f"rank{r}_{w}": [int((x != y).sum()) for x, y in zip(first[r][w], cur[r][w])]
               for r in range(2) for w in ("pre", "post")}
        res.append(row)
        print(f"garbage run {k}:", json.dumps({k_: v for k_, v in row.items() if any(v)}), flush=True)
    json.dump({"runs": K, "vs_run0": res}, open(dst, "w"), indent=1)


def main():
    if "--garbage-runs" in sys.argv:
        return garbage_runs(sys.argv[1], int(sys.argv[sys.argv.index("--garbage-runs") + 1]))
    if "--nosync-runs" in sys.argv:
        return nosync_runs(sys.argv[1], int(sys.argv[sys.argv.index("--nosync-runs") + 1]))
    res = {}
    modes = ("garbage",) if "--garbage" in sys.argv else ("nosync", False, "nosync", True)
    for serial in modes:
        runs = []
        for k in range(2):
            d = tempfile.mkdtemp()
            gb = (11 + k) if serial == "garbage" else None
            mp.start_processes(_worker, args=(2, t._free_port(), d, 4096, False if gb else serial, gb), nprocs=2,
                               join=True, start_method="spawn")
            runs.append([torch.load(os.path.join(d, f"a_{r}.pt"), weights_only=True) for r in range(2)])
        tag = {"nosync": "nosync", False: "concurrent", True: "serial", "garbage": "garbage_synced"}[serial]
        tag = tag + ("_b" if tag in res else "")
        res[tag] = {f"rank{r}_{w}": [int((x != y).sum()) for x, y in zip(runs[0][r][w], runs[1][r][w])]
                    for r in range(2) for w in ("pre", "post")}
        print(tag, json.dumps(res[tag]), flush=True)
    json.dump(res, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
