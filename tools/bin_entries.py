#!/usr/bin/env python3
"""Entries the binned hash backward writes per (level) in one lego training step's last (coarse)
hash backward: sum of the per-(level, owner, chunk) segment counts in the workspace."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import indoor_nerf_amd as nerf  # noqa: E402
from indoor_nerf_amd import hashgrid  # noqa: E402
from indoor_nerf_amd.synthetic import blender_bbox, blender_rays  # noqa: E402

dev = torch.device("cuda:0")
lo, hi = blender_bbox()
args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), finest_res=1024, N_samples=64,
                      N_importance=128, white_bkgd=True, perturb=1.0, lrate_decay=500, tv_loss_weight=1e-6)
torch.manual_seed(0)
kw, _, _, grad_vars, opt = nerf.create_nerf(args, device=dev)
kw.update(near=2.0, far=6.0)
ro, rd = blender_rays(4096, seed=100)
rays = (torch.from_numpy(ro).to(dev), torch.from_numpy(rd).to(dev))
target = torch.rand(4096, 3, device=dev)
for i in range(1, 4):
    nerf.train_step(rays, target, kw, opt, args, i)
torch.cuda.synchronize()
P, L = 4096 * 64, 16
nchunks = (P + 255) // 256
n_own = 64
up = lambda v: (v + 255) & ~255  # noqa: E731
entries_cap = L * nchunks * 2048
off_h = up(entries_cap * 8)
off_off = off_h + up(entries_cap * 2)
ws = next(iter(hashgrid._BWD_WORKSPACE.values()))[0] if hashgrid._BWD_WORKSPACE else None
names = [n for n in dir(hashgrid) if n.startswith("_")]
if ws is None:
    print(json.dumps({"error": "workspace cache not found", "names": names}))
    sys.exit(0)
seg = ws[off_off:off_off + 4 * L * n_own * nchunks].view(torch.int32).cpu().numpy().view("uint32")
cnt = (seg >> 16).reshape(L, n_own, nchunks).sum(axis=(1, 2))
print(json.dumps({"points": P, "entries_per_level": [int(c) for c in cnt], "total": int(cnt.sum()),
                  "max_possible": P * 8 * L}))
