"""Python call sites of torch fills inside a bench step (a diagnostic): wraps Tensor.zero_ / fill_,
torch.zeros / zeros_like / full / ones_like and prints each distinct call site with a count, over
a few eager steps of `bench.py --graph 0`. usage: python tools/fill_sources.py --workload scannet"""
import collections
import os
import sys
import traceback

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

SITES = collections.Counter()


def wrap(owner, name):
    fn = getattr(owner, name)

    def w(*a, **k):
        out = fn(*a, **k)
        t = out if isinstance(out, torch.Tensor) else (a[0] if a and isinstance(a[0], torch.Tensor) else None)
        if t is not None and t.is_cuda and t.numel() > 0:
            fr = [f for f in traceback.extract_stack()[:-1] if "indoor-nerf_amd" in f.filename or "bench.py" in f.filename]
            if fr:
                SITES[(name, f"{os.path.basename(fr[-1].filename)}:{fr[-1].lineno}")] += 1
        return out
    setattr(owner, name, w)


for n in ("zero_", "fill_"):
    wrap(torch.Tensor, n)
for n in ("zeros", "zeros_like", "full", "ones_like", "ones"):
    wrap(torch, n)
wl = sys.argv[sys.argv.index("--workload") + 1] if "--workload" in sys.argv else "lego"
sys.argv = ["bench.py", "--workload", wl, "--graph", "0", "--steps", "3", "--warmup", "4", "--profile-kernels", "0",
            "--no-cpu-baseline"]
bench.main()
for (name, site), c in SITES.most_common():
    print(f"{c:5d} {name:12s} {site}")
