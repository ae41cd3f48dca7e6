#!/usr/bin/env python3
"""Summary of an alternating A/B (tools/gpu_ab_bench.sh results.jsonl): per variant the mean step time
and the mean event-timed ms per step of each op in the line's `ops` (argv[1]: the jsonl)."""
import json
import sys
from collections import defaultdict

rows = [json.loads(line) for line in open(sys.argv[1])]
by = defaultdict(list)
for r in rows:
    by[r["variant"]].append(r["result"])
for v, rs in by.items():
    ops = defaultdict(list)
    for res in rs:
        for o in res.get("ops", []):
            ops[o["op"]].append(o["ms_per_step"] * 1000)
    step = sum(r["ms_per_step"] for r in rs) / len(rs)
    fresh = [r.get("fresh_rays_ms_per_step") for r in rs if r.get("fresh_rays_ms_per_step")]
    steps = ", ".join("%.3f" % r["ms_per_step"] for r in rs)
    print(f"{v:12s} step {step:.4f} ms ({steps})"
          + (f" fresh {sum(fresh) / len(fresh):.4f}" if fresh else "") + " | "
          + " ".join(f"{k} {sum(x) / len(x):.1f}" for k, x in ops.items()))
