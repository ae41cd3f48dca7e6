#!/usr/bin/env python3
"""Is the hash bin launch itself reproducible? (DESIGN §8 open issue; tools/det_repro_c.py found the
deterministic two-rank rehearsal's bin ENTRY VALUES differing between runs while every input it reads
— xyz, d feat, the TV rows — and the segment words were identical.)

tests/test_gpu_dist.py's _dp_worker (2 gloo ranks on one GPU, deterministic mode, ZeRO-1 + overlap),
with every nerf_hash_encode_bwd_bin_batch launch repeated REPS times on the same inputs (the launch is
idempotent: each block writes its own chunk region). After each repeat the valid entries of every
(level, chunk) are compared with the first launch's as multisets (sorted (row, value bits) records;
the order inside a segment follows LDS atomics). A mismatch is dumped: level, chunk, job (TV / fine /
coarse from the chunk base), the differing records of both launches. JSON: argv[1] (--runs K, --reps R)."""
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

SYNC_MLP = os.environ.get("DET_SYNC_MLP", "0") == "1"
SHIFT = int(os.environ.get("DET_SHIFT_GIB", "0"))
CU_SPLIT = os.environ.get("DET_CU_SPLIT", "0") == "1"
_KEEP = []


def _entries(pb, C):
    """(g [L, cap, K, 2] int32 view, h [L, cap, K] int16 view, counts [L, cap]) of the open workspace."""
    L, log2_T, _, det = pb.tag
    cap, K = pb.cap, 8 * C
    entries = L * cap * K
    up = lambda v: (v + 255) & ~255  # noqa: E731
    ws = pb.ws
    off_h = up(entries * 8)
    off_off = off_h + up(entries * 2)
    n_own = 1 << (log2_T - (12 if det else 13))
    g = ws[:entries * 8].view(torch.int32).view(L, cap, K, 2)
    h = ws[off_h:off_h + entries * 2].view(torch.int16).view(L, cap, K)
    seg = ws[off_off:off_off + L * cap * n_own * 4].view(torch.int32).view(L, n_own, cap)
    cnt = ((seg >> 16) & 0xFFFF).sum(1)
    return g, h, cnt


def _records(g, h, cnt, l, c):
    n = int(cnt[l, c])
    rec = torch.stack([h[l, c, :n].to(torch.int64) & 0xFFFF, g[l, c, :n, 0].to(torch.int64),
                       g[l, c, :n, 1].to(torch.int64)], 1)
    key = (rec[:, 0] << 40) ^ ((rec[:, 1] & 0xFFFFF) << 20) ^ (rec[:, 2] & 0xFFFFF)
    return rec[torch.argsort(key * 3 + rec[:, 1] % 3)]   # any total order of the multiset


def _worker(rank, world, port, out, R, reps):
    if world > 1:   # DET_CU_SPLIT=1: disjoint CU sets per rank (tests/test_gpu_dist.py _init's default);
        if CU_SPLIT:  # 0: both ranks on every CU (an explicit full mask keeps _init from splitting)
            t._cu_mask(rank, world)
        else:
            os.environ["HSA_CU_MASK"] = f"0:0-{t.MI355X_CUS - 1}"
    for p in (ROOT, os.path.join(ROOT, "tests", "golden")):
        if p not in sys.path:
            sys.path.insert(0, p)
    if SHIFT:   # move every later device allocation of rank r by r x SHIFT GiB of virtual address space
        torch.cuda.set_device(0)
        keep = torch.empty((rank * SHIFT) << 28, device="cuda:0") if rank else None   # noqa: F841
        _KEEP.append(keep)
    import indoor_nerf_amd as nerf
    from indoor_nerf_amd import hashgrid
    C = int(nerf._lib.load().nerf_hash_bwd_chunk_points())
    found, launches = [], [0]
    orig = hashgrid._PendingBins._launch_bins

    def launch_bins(self, jobs, common, det):
        orig(self, jobs, common, det)
        launches[0] += 1
        g0, h0, c0 = (x.clone() for x in _entries(self, C))
        bases = [int(j.chunk_base) for j in jobs]
        for k in range(reps):
            orig(self, jobs, common, det)
            g1, h1, c1 = _entries(self, C)
            K = g1.shape[2]
            valid = torch.arange(K, device=g1.device)[None, None, :] < c1[:, :, None]
            # per (level, chunk): sums of the valid records' words (order-free), compared exactly
            s0 = [torch.where(valid, x, 0).to(torch.int64).sum(2) for x in (g0[..., 0], g0[..., 1], h0.to(torch.int32))]
            s1 = [torch.where(valid, x, 0).to(torch.int64).sum(2) for x in (g1[..., 0], g1[..., 1], h1.to(torch.int32))]
            bad = ((s0[0] != s1[0]) | (s0[1] != s1[1]) | (s0[2] != s1[2]) | (c0 != c1)).nonzero().tolist()
            if bad:
                for l, c in bad[:6]:
                    a, b = _records(g0, h0, c0, l, c), _records(g1, h1, c1, l, c)
                    n = min(a.shape[0], b.shape[0])
                    diff = (a[:n] != b[:n]).any(1).nonzero().flatten()[:8].tolist()
                    found.append({"launch": launches[0], "rerun": k, "level": l, "chunk": c, "bases": bases,
                                  "n": [int(c0[l, c]), int(c1[l, c])],
                                  "first": [a[i].tolist() for i in diff], "rerun_rec": [b[i].tolist() for i in diff]})
                found.append({"launch": launches[0], "rerun": k, "n_bad_chunks": len(bad)})
                g0, h0, c0 = (x.clone() for x in (g1, h1, c1))
    hashgrid._PendingBins._launch_bins = launch_bins
    import threading
    streams = []
    orig_call = nerf._lib.call

    def call(name, *args):    # which stream / thread each launch of the backward goes to
        if name in ("nerf_mlp_bwd_batch", "nerf_hash_encode_bwd_bin_batch", "nerf_tv_bwd_bin",
                    "nerf_hash_encode_bwd_owner_step") and len(streams) < 64:
            streams.append((name, int(torch.cuda.current_stream().cuda_stream), threading.current_thread().name))
        r = orig_call(name, *args)
        if SYNC_MLP and name == "nerf_mlp_bwd_batch":
            torch.cuda.synchronize()
        return r
    nerf._lib.call = call
    try:
        t._dp_worker(rank, world, port, out, R, True, True)
    finally:
        torch.cuda.synchronize()
        json.dump({"rank": rank, "launches": launches[0], "found": found, "streams": streams,
                   "ws_ptr": int(hashgrid.pending_bins(torch.device("cuda:0")).ws.data_ptr())}, open(os.path.join(out, f"d_{rank}.json"), "w"))


def main():
    argv = sys.argv[1:]
    dst = argv[0]
    K = int(argv[argv.index("--runs") + 1]) if "--runs" in argv else 4
    reps = int(argv[argv.index("--reps") + 1]) if "--reps" in argv else 3
    world = int(argv[argv.index("--world") + 1]) if "--world" in argv else 2
    stress = None
    if "--stress" in argv:   # an unrelated GPU process (fp32 matmuls) running beside the runs
        import subprocess
        code = ("import torch,time\nx=torch.randn(4096,4096,device='cuda')\nt0=time.time()\n"
                "while time.time()-t0<%d:\n    y=x@x\n    torch.cuda.synchronize()\n" % int(argv[argv.index("--stress") + 1]))
        stress = subprocess.Popen([sys.executable, "-c", code])
    res = []
    for k in range(K):
        d = tempfile.mkdtemp()
        mp.start_processes(_worker, args=(world, t._free_port(), d, 4096, reps), nprocs=world, join=True,
                           start_method="spawn")
        cur = [json.load(open(os.path.join(d, f"d_{r}.json"))) for r in range(world)]
        res.append(cur)
        for c in cur:
            if k == 0:
                print("streams:", sorted(set(map(tuple, c["streams"]))), "workspace at", hex(c["ws_ptr"]), flush=True)
            print(f"run {k} rank {c['rank']}: {c['launches']} bin launches x {reps} reruns, "
                  f"{sum(1 for f in c['found'] if 'n_bad_chunks' in f)} reruns differ", json.dumps(c["found"][:3])[:1500],
                  flush=True)
    json.dump(res, open(dst, "w"))
    if stress is not None:
        stress.kill()
        stress.wait()


if __name__ == "__main__":
    main()
