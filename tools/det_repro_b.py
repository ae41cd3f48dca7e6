#!/usr/bin/env python3
"""Which buffer of the deterministic backward first varies from run to run (round-5 open issue,
DESIGN §8: the two-rank rehearsal's table gradients of levels 7-15 differ between runs).

Each rank (deterministic mode, tests/test_gpu_dist.py's F10 model, its half of the 4,096-ray batch,
pytest draws) runs `reps` identical forward_backward calls back to back — no optimizer step, the
same draws and TV corners every time — so every buffer of every rep should equal rep 0's bit for
bit. Both ranks run at once on the one GPU (world 2), or one process alone (world 1, the control).
Per rep and per captured buffer the number of elements that differ from rep 0 (per level where the
buffer is level-major):
  graw_<job>     the MLP backward's upstream gradient (composite backward output)
  dfeat<i>       / dfeat2_<i>: the d feat a bin launch reads (MLP backward output)
  xyz<i>         the points a bin launch reads
  tv_verts / tv_g  the TV bin's inputs
  seg / cmax     the bin launches' segment words / per-chunk maxima (order-free: counts, offsets, max)
  grad<k>        the parameters' gradients after the owner pass
JSON: argv[1] (+ --reps N, --world W, --sync: device synchronize after every rep)."""
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


def _diff(a, b, levels=None):
    if a.shape != b.shape:
        return "shape"
    ne = a.view(torch.int32) != b.view(torch.int32) if a.dtype == torch.float32 else a != b
    if levels:
        return [int(x) for x in ne.reshape(levels, -1).sum(1).tolist()]
    return int(ne.sum())


def _detail(a, b):
    """Where a float32 buffer's elements differ: count, rows (first 12), 2^12-row owner slices hit,
    largest |a - b| relative to max |a| and to |a| at that element."""
    ne = (a.view(torch.int32) != b.view(torch.int32)).reshape(a.shape[0], -1).any(1)
    rows = ne.nonzero().flatten()
    if rows.numel() == 0:
        return None
    d = (a.double() - b.double()).abs().reshape(a.shape[0], -1)[rows].max(1).values
    ref = a.double().abs().reshape(a.shape[0], -1)[rows].max(1).values
    k = int(d.argmax())
    return {"rows": int(rows.numel()), "first": rows[:12].tolist(),
            "slices": sorted(set((rows >> 12).tolist()))[:32],
            "max_rel_to_tensor": float(d.max() / a.double().abs().max().clamp_min(1e-300)),
            "at_max": [float(d[k]), float(ref[k])]}


def _worker(rank, world, port, out, R, reps, sync, save=False):
    if world > 1:
        t._init(rank, world, port)
    else:
        import sys as _s
        for p in (ROOT, os.path.join(ROOT, "tests", "golden")):
            if p not in _s.path:
                _s.path.insert(0, p)
        torch.cuda.set_device(0)
    import importlib
    import indoor_nerf_amd as nerf
    from indoor_nerf_amd import field, hashgrid
    nerf.set_deterministic(True)
    from indoor_nerf_amd.model import forward_backward
    rmod = importlib.import_module("indoor_nerf_amd.render")
    from tables import synthetic_rays
    dev = torch.device("cuda:0")
    rmod.pytest_shard(rank, max(world, 2))     # world 1 = rank 0's half alone (the same work per process)
    ro, rd = synthetic_rays(R, seed=21)
    target = torch.rand(R, 3, generator=torch.Generator().manual_seed(5))
    n = R // max(world, 2)
    rays = (torch.from_numpy(ro[rank * n:(rank + 1) * n]).to(dev), torch.from_numpy(rd[rank * n:(rank + 1) * n]).to(dev))
    tgt = target[rank * n:(rank + 1) * n].to(dev)
    args, kw, opt, params = t._f10_model(nerf, dev, max(world, 2))
    arena = nerf.GradArena(params, defer_tables=True)

    cap = {}     # name -> (tensor clone, levels)
    ptrs = {}    # buffer addresses of this process (does a result follow them?)

    def keep(name, x, levels=None):
        if x is not None:
            k, i = name, 0
            while k in cap:
                i += 1
                k = f"{name}.{i}"
            cap[k] = (x.detach().clone(), levels)

    orig_bwd = hashgrid.hash_encode_bwd

    def hash_encode_bwd(xyz, meta, dfeat, sp, sl, grad_tables, defer=None, queue=True, **rows):
        L = len(grad_tables)
        keep("xyz", xyz)
        keep("dfeat", dfeat, L)
        keep("dfeat2", rows.get("dfeat2"), L)
        return orig_bwd(xyz, meta, dfeat, sp, sl, grad_tables, defer=defer, queue=queue, **rows)
    field.hash_encode_bwd = hash_encode_bwd
    hashgrid.hash_encode_bwd = hash_encode_bwd

    orig_jobs = field._run_field_jobs

    def run_field_jobs(jobs):
        out = orig_jobs(jobs)
        for j in jobs:      # after the launches: graw is written by the deferred compositing backward
            if isinstance(j, field._FieldJob):
                keep("graw", j.g)
                keep("feat", j.feat, j.feat.shape[0])
                ptrs[f"job{len(ptrs)}"] = [j.g.data_ptr(), j.feat.data_ptr(), j.pts.data_ptr()]
        return out
    field._run_field_jobs = run_field_jobs

    orig_tv = hashgrid._PendingBins.add_tv

    def add_tv(self, job, queue=True):
        keep("tv_verts", job.verts)
        keep("tv_g", job.g)
        return orig_tv(self, job, queue)
    hashgrid._PendingBins.add_tv = add_tv

    orig_run = hashgrid.HeldOwner.run

    def run(self, lb, le):
        L, cap_ = self.L, self.cap
        entries = L * cap_ * 8 * int(nerf._lib.load().nerf_hash_bwd_chunk_points())   # kChunkCap per chunk
        up = lambda v: (v + 255) & ~255  # noqa: E731
        off_h = up(entries * 8)
        off_off = off_h + up(entries * 2)
        n_own = 1 << (self.log2_T - 12)     # deterministic slices: 2^12 rows
        off_max = off_off + up(L * cap_ * n_own * 4)
        ws = self.ws
        seg = ws[off_off:off_off + L * cap_ * n_own * 4].view(torch.int32).view(L, n_own, cap_)[:, :, :self.used]
        cmax = ws[off_max:off_max + L * cap_ * 4].view(torch.float32).view(L, cap_)[:, :self.used]
        keep("seg", seg.contiguous(), L)
        keep("cmax", cmax.contiguous(), L)
        return orig_run(self, lb, le)
    hashgrid.HeldOwner.run = run

    ref, res = None, []
    for k in range(reps):
        cap.clear()
        forward_backward(rays, tgt, kw, opt, args, 1, loss_scale_sparsity=float(max(world, 2)),
                         tv_generator=torch.Generator().manual_seed(7), zero_grad=arena.zero_)
        for i, p in enumerate(params):
            keep(f"grad{i}", p.grad, 16 if i >= 10 else None)
        if sync:
            torch.cuda.synchronize()
        if save and ref is None:    # --runs: rep 0's buffers to disk, compared across processes by main()
            pb = hashgrid.pending_bins(dev)
            ptrs["ws"] = pb.ws.data_ptr()
            ptrs["grads"] = [p.grad.data_ptr() for p in params]
            torch.save({"cap": {k: x.cpu() for k, (x, _) in cap.items()}, "levels": {k: lv for k, (_, lv) in cap.items()},
                        "ptrs": ptrs}, os.path.join(out, f"run_{rank}.pt"))
        if ref is None:
            ref = dict(cap)
            continue
        row = {}
        for name, (x, levels) in cap.items():
            if name not in ref:
                row[name] = "missing in rep 0"
                continue
            d = _diff(ref[name][0], x, levels)
            if d != 0 and d != [0] * (levels or 0):
                row[name] = d
                if name.startswith("grad") and x.dtype == torch.float32:
                    row[name + "_detail"] = _detail(ref[name][0].cpu(), x.cpu())
        res.append(row)
    torch.cuda.synchronize()
    names = {n: list(x.shape) for n, (x, _) in ref.items()}
    json.dump({"rank": rank, "world": world, "reps": reps, "sync": sync, "buffers": names, "diffs": res},
              open(os.path.join(out, f"b_{rank}.json"), "w"), indent=None)
    if world > 1:
        torch.distributed.destroy_process_group()


def cross_runs(dst, runs, world, sync):
    """--runs K: K fresh process sets (world ranks each, one forward_backward), every captured buffer
    of each run compared with run 0's (per rank)."""
    import shutil
    base = tempfile.mkdtemp()
    res = []
    ref = None
    for k in range(runs):
        d = os.path.join(base, str(k))
        os.makedirs(d)
        mp.start_processes(_worker, args=(world, t._free_port(), d, 4096, 1, sync, True), nprocs=world, join=True,
                           start_method="spawn")
        cur = [torch.load(os.path.join(d, f"run_{r}.pt"), weights_only=True) for r in range(world)]
        if ref is None:
            ref = cur
            shutil.rmtree(d)
            continue
        row = {}
        for r in range(world):
            a, b = ref[r], cur[r]
            for name, x in b["cap"].items():
                y = a["cap"].get(name)
                if y is None:
                    row[f"r{r}.{name}"] = "missing in run 0"
                    continue
                lv = b["levels"][name]
                dd = _diff(y, x, lv)
                if dd != 0 and dd != [0] * (lv or 0):
                    row[f"r{r}.{name}"] = dd
                    if x.dtype == torch.float32 and x.dim() >= 2:
                        row[f"r{r}.{name}_detail"] = _detail(y.reshape(y.shape[0], -1), x.reshape(x.shape[0], -1))
            row[f"r{r}.ptrs_same"] = a["ptrs"] == b["ptrs"]
        res.append(row)
        print(f"run {k}: {len([v for v in row if not v.endswith('ptrs_same')])} buffers differ from run 0;",
              json.dumps(row)[:3000], flush=True)
        shutil.rmtree(d)
    json.dump({"runs": runs, "world": world, "sync": sync, "ptrs_run0": [x["ptrs"] for x in ref], "diffs": res},
              open(dst, "w"), indent=1)
    shutil.rmtree(base)


def main():
    argv = sys.argv[1:]
    dst = argv[0]
    reps = int(argv[argv.index("--reps") + 1]) if "--reps" in argv else 10
    world = int(argv[argv.index("--world") + 1]) if "--world" in argv else 2
    sync = "--sync" in argv
    if "--runs" in argv:
        return cross_runs(dst, int(argv[argv.index("--runs") + 1]), world, sync)
    d = tempfile.mkdtemp()
    mp.start_processes(_worker, args=(world, t._free_port(), d, 4096, reps, sync), nprocs=world, join=True,
                       start_method="spawn")
    out = [json.load(open(os.path.join(d, f"b_{r}.json"))) for r in range(world)]
    for o in out:
        bad = [(k + 1, row) for k, row in enumerate(o["diffs"]) if row]
        print(f"rank {o['rank']}: {len(bad)} of {len(o['diffs'])} reps differ from rep 0", flush=True)
        for k, row in bad[:4]:
            print("  rep", k, json.dumps(row)[:2000], flush=True)
    json.dump(out, open(dst, "w"), indent=1)


if __name__ == "__main__":
    main()
