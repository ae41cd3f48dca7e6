#!/usr/bin/env python3
"""Timeline of the ZeRO-1 owner-pass / reduce-scatter overlap (dist.ShardedOptimizer(overlap=True),
DESIGN.md §6) on ONE GPU: run under torchrun with 2 ranks and NERF_DIST_BACKEND=gloo, with bench.py's
arguments, eager steps (--graph 0: torch on ROCm refuses timing events inside a capture), e.g.

  NERF_DIST_BACKEND=gloo python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
      tools/dist_overlap_trace.py OUT.json --gpus 2 --steps 6 --warmup 3 --graph 0 --zero 1 --overlap 1 \\
      --no-cpu-baseline --profile-kernels 0

HIP events are recorded around every owner level-range launch (main stream) and every bucket's
reduce-scatter (the side stream it is issued on), plus host times; per rank, the last step's spans
(us from the step's first stamp) go to OUT.json (rank r writes OUT.json.r<r>). With gloo the
collective itself runs on the host between a device->host and a host->device copy on the side stream,
so what the trace shows is the side stream's bucket-0 span running while the main stream still
executes the owner blocks of bucket 1's levels — the RCCL collective would sit in the same place.
The gated parameter all-gather (ShardedOptimizer.gather_params with overlap): the bucket of levels
8-15 starts on the side stream at the end of step i (gloo: asynchronously in gloo's thread), and step
i + 1's hash forward launches levels 0-7, joins the gate (host wait for gloo + the copy back on the side
stream + the main stream's event wait), then launches levels 8-15; the last two steps are written."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import indoor_nerf_amd as nerf  # noqa: E402
from indoor_nerf_amd import dist as ndist, hashgrid  # noqa: E402

STEPS = []   # per train step: list of (name, cuda event, host time)


def stamp(name, stream=None):
    ev = torch.cuda.Event(enable_timing=True)
    ev.record(stream)
    STEPS[-1].append((name, ev, time.perf_counter()))


def main():
    out = sys.argv.pop(1)
    orig_step, orig_run, orig_rs = nerf.train_step, hashgrid.HeldOwner.run, ndist._reduce_scatter

    def train_step(*a, **k):
        STEPS.append([])
        stamp("step")
        r = orig_step(*a, **k)
        stamp("step end")
        return r

    def run(self, lb, le):
        stamp(f"owner levels [{lb},{le}) start")
        r = orig_run(self, lb, le)
        stamp(f"owner levels [{lb},{le}) end")
        return r

    def rs(o, i, group=None):
        s = torch.cuda.current_stream()
        n = sum(1 for x in STEPS[-1] if x[0].startswith("reduce-scatter") and " start" in x[0])
        stamp(f"reduce-scatter bucket {n} start ({'side' if s != torch.cuda.default_stream() else 'main'} stream)", s)
        r = orig_rs(o, i, group)
        stamp(f"reduce-scatter bucket {n} end", s)
        return r

    orig_ag, orig_join, orig_slice = ndist._all_gather_begin, hashgrid.TableGate.join, hashgrid.HashEmbedder._level_slice

    def ag(o, i, group, stream):
        stamp("all-gather gated bucket start (side stream)", stream)
        ev, finish = orig_ag(o, i, group, stream)

        def fin():
            if finish is not None:
                finish()
            stamp("all-gather gated bucket end (side stream)", stream)
        return ev, fin

    def join(self, stream):
        stamp(f"gate level {self.level}: join (host) ", stream)
        orig_join(self, stream)
        stamp(f"gate level {self.level}: main stream past the wait", stream)

    def level_slice(self, lb, le):
        stamp(f"hash forward levels [{lb},{le}) launch")
        return orig_slice(self, lb, le)

    ndist._all_gather_begin, hashgrid.TableGate.join, hashgrid.HashEmbedder._level_slice = ag, join, level_slice
    nerf.train_step, hashgrid.HeldOwner.run, ndist._reduce_scatter = train_step, run, rs
    import bench
    bench.main()
    torch.cuda.synchronize()
    rank = int(os.environ.get("RANK", "0"))
    last = STEPS[-1]
    ref, h0 = last[0][1], last[0][2]
    spans = [{"event": n, "gpu_us": round(1e3 * ref.elapsed_time(ev), 1), "host_us": round(1e6 * (h - h0), 1)}
             for n, ev, h in last]
    two = STEPS[-2] + STEPS[-1]
    ref2, h2 = two[0][1], two[0][2]
    spans2 = [{"event": n, "gpu_us": round(1e3 * ref2.elapsed_time(ev), 1), "host_us": round(1e6 * (h - h2), 1)}
              for n, ev, h in two]
    with open(f"{out}.r{rank}", "w") as f:
        json.dump({"rank": rank, "steps_recorded": len(STEPS), "last_step": spans, "last_two_steps": spans2},
                  f, indent=1)


if __name__ == "__main__":
    main()
