#!/usr/bin/env python3
"""The default MLP kernels, fwd+bwd on the lego fine pass, a few reps: a short target for
rocprofv3 PMC passes (tools/pmc_mlp.sh)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import indoor_nerf_amd as nerf  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
net = nerf.NeRFSmall(2, 64, 15, 3, 64, 32, 16).to(dev)
x = (torch.randn(786432, 48, device=dev) * 0.3).requires_grad_(True)
g = torch.randn(786432, 4, device=dev)
for _ in range(4):
    net(x).backward(g)
torch.cuda.synchronize()
