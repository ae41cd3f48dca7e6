"""Diagnostic (CPU, this container): train the ORACLE on F19's scene, initial state and batches and
compare its PSNR curve with the reference runs F19 holds.

If the oracle shows the same iteration 40-80 lag as the HIP ensemble, the cause is an algorithmic
choice shared by the oracle and the HIP path (both restate the reference); if it does not, the cause
is HIP-side numerics. Optional per-iteration diagnostics (--stats) record, per table level, the rows
with a nonzero / exactly-zero gradient and |dp| statistics of the update.

usage: python tests/diagnostics/converge_oracle.py --iters 120 --threads 8 [--stats out.npz]
"""
import argparse
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
from oracle import nerf_oracle as orc  # noqa: E402
from tables import blender_bbox, closed_form_table, convergence_rays  # noqa: E402


class _Embed64(torch.autograd.Function):
    """F.embedding whose table gradient is summed in fp64 and rounded to fp32 once (the HIP owner
    pass's accumulation) instead of embedding_dense_backward's fp32 sums."""

    @staticmethod
    def forward(ctx, idx, table):
        ctx.save_for_backward(idx)
        ctx.shape = table.shape
        return table[idx]

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        acc = torch.zeros(ctx.shape, dtype=torch.float64)
        acc.index_add_(0, idx.reshape(-1), g.reshape(-1, ctx.shape[1]).double())
        return None, acc.float()


class _Embed32Shuffled(torch.autograd.Function):
    """F.embedding whose table gradient is summed in fp32 in a seeded random order of the (point,
    corner) contributions instead of embedding_dense_backward's fixed order (the reference runs all
    share that order whatever their thread count)."""
    gen = torch.Generator().manual_seed(0)

    @staticmethod
    def forward(ctx, idx, table):
        ctx.save_for_backward(idx)
        ctx.shape = table.shape
        return table[idx]

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        i = idx.reshape(-1)
        perm = torch.randperm(i.numel(), generator=_Embed32Shuffled.gen)
        acc = torch.zeros(ctx.shape, dtype=torch.float32)
        acc.index_add_(0, i[perm], g.reshape(-1, ctx.shape[1])[perm])
        return None, acc


def _split3(v):
    """v = v0 + v1 + v2, three round-to-nearest bf16 pieces (as fp32 tensors), as csrc/field_x6.hip."""
    v0 = v.to(torch.bfloat16).float()
    r = v - v0
    v1 = r.to(torch.bfloat16).float()
    v2 = (r - v1).to(torch.bfloat16).float()
    return v0, v1, v2


def _mm6(a, b):
    """a @ b as the bf16x6 MFMA products (a0b2 + a2b0 + a1b1 + a0b1 + a1b0 + a0b0, small terms first;
    each bf16 x bf16 product is exact in fp32), fp32 accumulation."""
    a0, a1, a2 = _split3(a)
    b0, b1, b2 = _split3(b)
    out = a0 @ b2
    for x, y in ((a2, b0), (a1, b1), (a0, b1), (a1, b0), (a0, b0)):
        out = out + x @ y
    return out


class _Linear6(torch.autograd.Function):
    """x @ w.t() with the forward and both backward products in bf16x6 (the HIP MLP kernels)."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return _mm6(x, w.t())

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        return _mm6(g, w), _mm6(g.t(), x)


def apply_variants(variants, seed=0):
    if "gsum64" in variants:
        orc.F = type("F", (), {k: getattr(torch.nn.functional, k) for k in dir(torch.nn.functional)
                               if not k.startswith("_")})
        orc.F.embedding = staticmethod(lambda idx, table: _Embed64.apply(idx, table))
    if "gsum32shuf" in variants:
        _Embed32Shuffled.gen.manual_seed(seed)
        orc.F = type("F", (), {k: getattr(torch.nn.functional, k) for k in dir(torch.nn.functional)
                               if not k.startswith("_")})
        orc.F.embedding = staticmethod(lambda idx, table: _Embed32Shuffled.apply(idx, table))
    if "mlpx6" in variants:
        import torch.nn.functional as tf

        def mlp_forward6(x, w, n_feat=32, quant=None):
            pts, views = x[:, :n_feat], x[:, n_feat:]
            lin = lambda a, k: _Linear6.apply(a, w[k])  # noqa: E731
            h = tf.relu(lin(pts, "sigma_net.0.weight"))
            o = lin(h, "sigma_net.1.weight")
            sigma, geo = o[:, 0], o[:, 1:]
            c = torch.cat([views, geo], -1)
            c = tf.relu(lin(c, "color_net.0.weight"))
            c = tf.relu(lin(c, "color_net.1.weight"))
            rgb = lin(c, "color_net.2.weight")
            return torch.cat([rgb, sigma[:, None]], -1)
        orc.mlp_forward = mlp_forward6
    if "comp64" in variants:
        base = orc.composite

        def composite64(raw, z, rays_d, noise=None, white_bkgd=False):
            out = base(raw.double(), z.double(), rays_d.double(), None if noise is None else noise.double(), white_bkgd)
            return tuple(o.float() for o in out)
        orc.composite = composite64


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=120)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--stats", default="")
    ap.add_argument("--out", default="")
    ap.add_argument("--variant", default="", help="comma list: gsum64 (table gradients summed in fp64, as the "
                    "HIP owner pass), gsum32shuf (fp32 sums in a seeded random order), comp64 (compositing in fp64), mlpx6 (MLP products as the "
                    "bf16x6 MFMA kernels)")
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    apply_variants([v for v in a.variant.split(",") if v], seed=a.threads)
    g = np.load(os.path.join(ROOT, "tests", "golden", "f19_converge.npz"))
    import ast
    c = ast.literal_eval(str(g["config"]))
    lo, hi = (torch.from_numpy(v) for v in blender_bbox())
    res = orc.level_resolutions(16, 1024)
    table = closed_form_table(scale=c["table_scale"], salt=c["table_salt"])
    tabs = [torch.from_numpy(table[i]).clone().requires_grad_(True) for i in range(16)]
    cw = {k: torch.from_numpy(g["coarse0_" + k.replace(".", "_")]).clone().requires_grad_(True) for k in orc.MLP_KEYS}
    fw = {k: torch.from_numpy(g["fine0_" + k.replace(".", "_")]).clone().requires_grad_(True) for k in orc.MLP_KEYS}
    opt = orc.RAdamOracle([
        dict(params=list(cw.values()) + list(fw.values()), lr=c["lrate"], betas=(0.9, 0.99), eps=1e-8,
             weight_decay=1e-6),
        dict(params=tabs, lr=c["lrate"], betas=(0.9, 0.99), eps=1e-15, weight_decay=0.0)])
    (ro, rd, rgb), (eo, ed, ergb), (no, nd, nrgb) = (tuple(torch.from_numpy(x) for x in t) for t in convergence_rays())
    batches = torch.from_numpy(g["batches"].astype(np.int64))

    def psnr_of(o, d, target):
        with torch.no_grad():
            out = orc.render_rays(o, d, orc.viewdirs_of(d), 2.0, 6.0, cw, fw, tabs, lo, hi, res, perturb=0.0)
            return float(-10.0 * torch.log10(((out["rgb_map"] - target) ** 2).mean()))

    ev, nv, tr = [psnr_of(eo, ed, ergb)], [psnr_of(no, nd, nrgb)], []
    stats = {k: [] for k in ("nonzero", "exact_zero", "dp_mean", "dp_max", "g_min_nonzero")}
    for it in range(1, a.iters + 1):
        idx = batches[it - 1]
        o, d, t = ro[idx], rd[idx], rgb[idx]
        for p in tabs + list(cw.values()) + list(fw.values()):
            p.grad = None
        out = orc.render_rays(o, d, orc.viewdirs_of(d), 2.0, 6.0, cw, fw, tabs, lo, hi, res)
        img = ((out["rgb_map"] - t) ** 2).mean()
        loss = img + ((out["rgb0"] - t) ** 2).mean()
        loss = loss + c["sparsity"] * (out["sparsity_loss"].sum() + out["sparsity_loss0"].sum())
        loss.backward()
        before = [p.detach().clone() for p in tabs] if a.stats else None
        opt.step()
        lr = c["lrate"] * (0.1 ** (it / (c["lrate_decay"] * 1000)))
        for grp in opt.groups:
            grp["lr"] = lr
        tr.append(float(-10.0 * math.log10(float(img))))
        if a.stats:
            nz, ez, dm, dx, gm = [], [], [], [], []
            for p, b in zip(tabs, before):
                gr = p.grad.abs().sum(-1)
                nz.append(int((gr > 0).sum()))
                ez.append(int((gr == 0).sum()))
                dp = (p.detach() - b).abs()
                dm.append(float(dp.mean()))
                dx.append(float(dp.max()))
                gm.append(float(gr[gr > 0].min()) if (gr > 0).any() else 0.0)
            for k, v in zip(stats, (nz, ez, dm, dx, gm)):
                stats[k].append(v)
        if it % c["every"] == 0:
            ev.append(psnr_of(eo, ed, ergb))
            nv.append(psnr_of(no, nd, nrgb))
            print(f"it {it}: train {tr[-1]:.3f} held-out {ev[-1]:.3f} novel {nv[-1]:.3f}", flush=True)
    if a.out:
        np.savez(a.out, eval_psnr=np.array(ev), novel_psnr=np.array(nv), train_psnr=np.array(tr))
    if a.stats:
        np.savez(a.stats, **{k: np.array(v) for k, v in stats.items()})


if __name__ == "__main__":
    main()
