#!/usr/bin/env python3
"""Which buffer of the deterministic two-rank rehearsal first differs between runs (DESIGN §8 open
issue; tools/det_repro.py --runs reproduces it: some runs' gradients / parameters differ).

Each run is tests/test_gpu_dist.py's _dp_worker exactly (2 gloo ranks on one GPU, deterministic mode,
part (a) one iteration + all-reduce, part (b) 7 ZeRO-1 steps with overlap and the gated all-gather),
with hooks that record stream-ordered int64 checksums (sum of the int32 bit patterns, per level where
the buffer is level-major) of every buffer the hash backward reads or writes, in launch order:
  graw / feat     the MLP backward's upstream gradient and features (after the MLP launch)
  dfeat / dfeat2  the d feat a bin launch reads (MLP backward output)
  xyz             the points a bin launch reads
  tv_verts / tv_g the TV bin's inputs
  seg / cmax      the bin launches' segment words / per-chunk maxima, before the owner launch
  owner_out       the table gradients of the owner launch's levels, after it
  mlp_grad        the MLP weight gradients after the field backward
  det_ws          the deterministic MLP backward's per-block weight-gradient images
Runs are compared with the first: per rank, the first events whose checksums differ. JSON: argv[1]
(--runs K)."""
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

RERUN = int(os.environ.get("DET_RERUN", "0"))


def _cs(x, levels=None):
    v = x.detach().contiguous().view(-1)
    if v.dtype in (torch.float32, torch.int32):
        v = v.view(torch.int32)
    elif v.dtype == torch.uint8:
        v = v[:v.numel() // 4 * 4].view(torch.int32)
    v = v.to(torch.int64)
    if levels:
        return v.reshape(levels, -1).sum(1)
    return v.sum().reshape(1)


def _worker(rank, world, port, out, R):
    for p in (ROOT, os.path.join(ROOT, "tests", "golden")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import indoor_nerf_amd as nerf
    from indoor_nerf_amd import field, hashgrid
    log = []   # (name, device checksum tensor)

    def rec(name, x, levels=None):
        if x is not None:
            log.append((name, _cs(x, levels)))

    orig_bwd = hashgrid.hash_encode_bwd

    def hash_encode_bwd(xyz, meta, dfeat, sp, sl, grad_tables, defer=None, queue=True, **rows):
        L = len(grad_tables)
        rec("xyz", xyz)
        rec("dfeat", dfeat, L)
        rec("dfeat2", rows.get("dfeat2"), L)
        return orig_bwd(xyz, meta, dfeat, sp, sl, grad_tables, defer=defer, queue=queue, **rows)
    field.hash_encode_bwd = hash_encode_bwd
    hashgrid.hash_encode_bwd = hash_encode_bwd

    orig_jobs = field._run_field_jobs

    def run_field_jobs(jobs):
        fj = [j for j in jobs if isinstance(j, field._FieldJob)]
        res = orig_jobs(jobs)
        for j in fj:
            rec("graw", j.g)
            rec("feat", j.feat, j.feat.shape[0])
            for k, w in enumerate(j.weights):
                rec(f"mlp_grad{k}", w.grad)
        ws = field._DETERMINISTIC["ws"].get("cuda:0")
        rec("det_ws", ws, 16 if ws is not None and ws.numel() % 16 == 0 else None)
        return res
    field._run_field_jobs = run_field_jobs

    orig_tv = hashgrid._PendingBins.add_tv

    def add_tv(self, job, queue=True):
        rec("tv_verts", job.verts)
        rec("tv_g", job.g)
        return orig_tv(self, job, queue)
    hashgrid._PendingBins.add_tv = add_tv

    orig_run = hashgrid.HeldOwner.run

    def run(self, lb, le):
        L, cap_ = self.L, self.cap
        C = int(nerf._lib.load().nerf_hash_bwd_chunk_points())
        entries = L * cap_ * C * 8   # kChunkCap = 8 entries per point of a chunk
        up = lambda v: (v + 255) & ~255  # noqa: E731
        off_off = up(entries * 8) + up(entries * 2)
        n_own = 1 << (self.log2_T - 12)     # deterministic slices: 2^12 rows
        off_max = off_off + up(L * cap_ * n_own * 4)
        ws = self.ws
        seg = ws[off_off:off_off + L * cap_ * n_own * 4].view(torch.int32).view(L, n_own, cap_)[lb:le, :, :self.used]
        cmax = ws[off_max:off_max + L * cap_ * 4].view(torch.float32).view(L, cap_)[lb:le, :self.used]
        rec(f"seg[{lb}:{le}]", seg, le - lb)
        rec(f"cmax[{lb}:{le}]", cmax, le - lb)
        # the valid entries of the range (slots [0, total) of each chunk region; the rest are stale)
        K = 8 * C
        tot = ((seg >> 16) & 0xFFFF).sum(1)                                   # [levels, used]
        mask = torch.arange(K, device=ws.device)[None, None, :] < tot[:, :, None]
        g = ws[:entries * 8].view(torch.int32).view(L, cap_, K, 2)[lb:le, :self.used]
        hh = ws[up(entries * 8):up(entries * 8) + entries * 2].view(torch.int16).view(L, cap_, K)[lb:le, :self.used]
        rec(f"entries_g[{lb}:{le}]", torch.where(mask[..., None], g, 0), le - lb)
        rec(f"entries_h[{lb}:{le}]", torch.where(mask, hh.to(torch.int32), 0), le - lb)
        r = orig_run(self, lb, le)
        outs = [_cs(self.grads[lv]) for lv in range(lb, le)]
        for lv in range(lb, le):
            rec(f"owner_out{lv}", self.grads[lv])
        if RERUN:   # the same launch again (overwrite mode: idempotent for the same inputs)
            for k in range(RERUN):
                orig_run(self, lb, le)
                again = [_cs(self.grads[lv]) for lv in range(lb, le)]
                log.append((f"rerun{k}_same[{lb}:{le}]", torch.stack([(a == b).all() for a, b in zip(outs, again)]).to(torch.int64)))
        return r
    hashgrid.HeldOwner.run = run

    try:
        t._dp_worker(rank, world, port, out, R, True, True)
    finally:
        torch.cuda.synchronize()
        torch.save({"names": [n for n, _ in log], "cs": [c.cpu() for _, c in log]},
                   os.path.join(out, f"cs_{rank}.pt"))


def main():
    argv = sys.argv[1:]
    dst = argv[0]
    K = int(argv[argv.index("--runs") + 1]) if "--runs" in argv else 8
    first, res, outcomes = None, [], []
    for k in range(K):
        d = tempfile.mkdtemp()
        mp.start_processes(_worker, args=(2, t._free_port(), d, 4096), nprocs=2, join=True, start_method="spawn")
        cur = [torch.load(os.path.join(d, f"cs_{r}.pt"), weights_only=True) for r in range(2)]
        fin = [torch.load(os.path.join(d, f"dp2od_{r}.pt"), weights_only=True) for r in range(2)]
        import hashlib
        hsh = hashlib.sha256(b"".join(x.numpy().tobytes() for x in fin[0]["grads"] + fin[0]["params"])).hexdigest()[:12]
        outcomes.append(hsh)
        for r in range(2):   # within-run reruns of the owner launch that did not reproduce its output
            rr = [(i, n, c.tolist()) for i, (n, c) in enumerate(zip(cur[r]["names"], cur[r]["cs"]))
                  if n.startswith("rerun") and not bool(c.all())]
            if rr:
                print(f"run {k} rank {r}: {len(rr)} owner reruns differ from the first launch:", rr[:8], flush=True)
        if first is None:
            first = (cur, fin)
            print(f"run 0: {len(cur[0]['names'])} / {len(cur[1]['names'])} events:", " ".join(f"{i}:{n}" for i, n in enumerate(cur[0]["names"][:80])), flush=True)
            continue
        row = {"params_differ": [int(sum(int((x != y).sum()) for x, y in zip(first[1][r]["params"], fin[r]["params"])))
                                 for r in range(2)],
               "grads_differ": [int(sum(int((x != y).sum()) for x, y in zip(first[1][r]["grads"], fin[r]["grads"])))
                                for r in range(2)]}
        for r in range(2):
            a, b = first[0][r], cur[r]
            if a["names"] != b["names"]:
                row[f"rank{r}"] = "event lists differ"
                continue
            bad = []
            for i, (n, x, y) in enumerate(zip(a["names"], a["cs"], b["cs"])):
                if not torch.equal(x, y):
                    bad.append({"event": i, "name": n,
                                "levels": (x != y).nonzero().flatten().tolist() if x.numel() > 1 else None})
            row[f"rank{r}"] = {"n_bad": len(bad), "first": bad[:12]}
        res.append(row)
        print(f"run {k}:", json.dumps(row)[:2500], flush=True)
    print(f"distinct outcomes (one-iteration gradients + final parameters): {len(set(outcomes))} of {K} runs:",
          outcomes, flush=True)
    json.dump({"runs": K, "outcomes": outcomes, "events": first[0][0]["names"], "vs_run0": res}, open(dst, "w"), indent=None)


if __name__ == "__main__":
    main()
