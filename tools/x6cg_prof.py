#!/usr/bin/env python3
"""Chain / weight-gradient wave balance of the MLP backward (diagnostic library built with
-DNERF_X6CG_PROF: tools/build_variant.py x6prof -DNERF_X6CG_PROF). Runs the lego step's batched
backward (fine 786,432 + coarse 262,144 points) and prints each role's waiting share."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import indoor_nerf_amd as nerf  # noqa: E402
from indoor_nerf_amd import _lib  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    nets = [nerf.NeRFSmall(2, 64, 15, 3, 64, 32, 16).to(dev) for _ in range(2)] if "--train" not in sys.argv else []
    xs = [(torch.randn(n, 48, device=dev) * 0.3).requires_grad_(True) for n in (786432, 262144)]
    gs = [torch.randn(x.shape[0], 4, device=dev) for x in xs]
    lib = _lib.load()
    fn = lib.nerf_x6cg_prof
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    out = (ctypes.c_ulonglong * 12)()
    if "--train" in sys.argv:   # the lego training step's own backward (saved h3, both nets in one launch)
        sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
        from tables import blender_bbox, synthetic_rays
        from indoor_nerf_amd import model
        lo, hi = blender_bbox()
        args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), finest_res=1024,
                              N_samples=64, N_importance=128, white_bkgd=True, tv_loss_weight=1e-6)
        kw, _, _, _, opt = nerf.create_nerf(args, device=dev)
        kw.update(near=2.0, far=6.0)
        ro, rd = synthetic_rays(4096, seed=13)
        rays = (torch.from_numpy(ro).to(dev), torch.from_numpy(rd).to(dev))
        target = torch.rand(4096, 3, device=dev)
        for it in range(4):
            model.forward_backward(rays, target, kw, opt, args, it + 1)
            torch.cuda.synchronize()
            assert fn(out) == 0
        nets = xs = gs = []
    for it in range(0 if "--train" in sys.argv else 4):
        loss = sum((net(x) * g).sum() for net, x, g in zip(nets, xs, gs))
        loss.backward()
        torch.cuda.synchronize()
        assert fn(out) == 0
    chain_wait, chain_total, wg_wait, wg_total = (int(v) for v in out[:4])
    stage = [int(v) for v in out[4:11]]
    print(json.dumps({"chain_wait_frac": round(chain_wait / max(chain_total, 1), 3),
                      "wgrad_wait_frac": round(wg_wait / max(wg_total, 1), 3),
                      "chain_total": chain_total, "wgrad_total": wg_total,
                      # chain wave's wait before stage k (1..7) of a tile, as a share of its total time
                      "chain_wait_by_stage": [round(w / max(chain_total, 1), 3) for w in stage]}))


if __name__ == "__main__":
    main()
