"""Which torch ops launch device work inside a bench step (eager, --graph 0): runs bench.main() under
torch.profiler with Python stacks and prints every aten op that launched a kernel or memcpy, with
the innermost repo frame. usage: python tools/torch_ops_trace.py --workload scannet"""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

wl = sys.argv[sys.argv.index("--workload") + 1] if "--workload" in sys.argv else "lego"
sys.argv = ["bench.py", "--workload", wl, "--graph", "0", "--steps", "2", "--warmup", "3", "--profile-kernels", "0",
            "--no-cpu-baseline"]
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    bench.main()
seen = {}
for e in prof.events():
    if not e.name.startswith("aten::") or e.device_type != torch.autograd.DeviceType.CPU:
        continue
    if not e.kernels:
        continue
    chain, x, frames = [e.name], e, []
    while x is not None and not frames:   # an op nested in another (copy_ in contiguous) has no stack of its own
        frames = [f for f in (x.stack or []) if "indoor-nerf_amd" in f or "bench.py" in f]
        x = x.cpu_parent
        if x is not None and not frames:
            chain.append(x.name)
    key = ("<".join(chain[:4]) + " [" + e.kernels[0].name[:40] + "]", frames[0] if frames else "?")
    seen[key] = seen.get(key, 0) + 1
for (name, fr), n in sorted(seen.items(), key=lambda kv: -kv[1]):
    print(f"{n:5d}  {name:28s} {fr}")
