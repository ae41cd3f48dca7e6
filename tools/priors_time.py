"""Device priors forward + backward time (HIP events, 50 reps) on a ScanNet-sized batch with and
without pixel coordinates (the no_batching path passes select_coords, run_nerf.py:1113-1117)."""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from indoor_nerf_amd import priors  # noqa: E402

dev = torch.device("cuda", 0)
N = 4096
g = torch.Generator().manual_seed(0)
n = torch.randn(N, 3, generator=g)
n[: N // 3] = torch.tensor([0.05, 0.02, 1.0]) + 0.1 * torch.randn(N // 3, 3, generator=g)
d = torch.rand(N, generator=g) * 3 + 0.5
xy = torch.stack([torch.randint(0, 640, (N,), generator=g), torch.randint(0, 480, (N,), generator=g)], -1).float()
d, n, xy = d.to(dev).requires_grad_(True), n.to(dev).requires_grad_(True), xy.to(dev)
for coords in (None, xy):
    ts = []
    for r in range(60):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        t, _ = priors.fused_structural_losses(d, n, coords)
        t.backward()
        b.record()
        torch.cuda.synchronize()
        if r >= 10:
            ts.append(a.elapsed_time(b) * 1000)
    ts.sort()
    print(f"coords={'yes' if coords is not None else 'no '}  fwd+bwd median {ts[len(ts) // 2]:.1f} us  loss {float(t):.6f}")
