#!/usr/bin/env python3
"""Headline benchmark: train rays/sec of the render_rays hot path (BASELINE.json `metric`).

A step = one full training iteration of PocketNeRF's train() on the lego configuration
(configs/lego.txt + finest_res 1024): 4096 rays (BASELINE's batch), 64 stratified coarse samples,
128 importance samples (192 fine), L=16 levels, T=2^19, white background, perturb=1, TV loss
(weight 1e-6, the first 1000 iterations), sparsity loss, backward, RAdam, lr decay. Rays are
synthetic (the lego rig's spiral poses; no dataset on the box) and resident in HBM before timing.

Multi-GPU (torchrun, one process per GPU): each rank trains its own 4096-ray shard (weak
scaling); gradients are all-reduced once per step over RCCL (one 67 MB bucket).

Prints ONE JSON line (rank 0) with `roofline` for the dominant kernel (HIP-event timed inside the
timed region) and `cpu_baseline` (the oracle's CPU training step on a bounded sample, N=1 only).
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: f32 matrix (v_mfma_f32_32x32x2_f32) dense peak
# The default MLP kernels (csrc/field_x6.hip) form each fp32-accurate product from six bf16 MFMA
# products, so their arithmetic peak is the dense bf16 rate (~2.5 PFLOP/s) / 6.
X6_PEAK_TFLOPS = 2500.0 / 6

# Algorithmic cost per unit of each OP: bytes (HBM-bound) or FLOPs (MFMA). An op is
# one or more ABI calls priced together: the hash backward is the bin pass (once per render pass)
# plus the owner pass (once per iteration), and only their sum is a complete scatter-add.
# Hash ops are priced per DISTINCT point encoded ("hash_point"): with the coarse-feature reuse (DESIGN
# §8.5) the fine pass encodes only its importance samples, so an iteration encodes R x (64 + 128) points
# (R x (64 + 192) without it); the MLP forward and compositing ops run on every point / sample of both
# passes. The backward ops are priced by the points they walk ("bwd_point", "bwd_hash_point"): with
# the active-point backward (field.set_active_points) only the samples with a nonzero raw gradient.
#   hash fwd : per point  16 levels x 8 corners x 8 B gathered + 12 B xyz + 128 B features + 1 B keep
#   hash fwd packed (A-CAQ eval): as hash fwd with 2-B entries (two 8-bit codes)
#   hash bwd : per point  16 x 8 x 8 B read+write of the added rows (2 x 1024) + 12 B xyz + 128 B d feat
#   mlp fwd  : per point  9,344 MACs = 18,688 FLOP
#   mlp bwd  : per point  2 x 18,688 FLOP (input + weight grads; the recomputed forward is not counted)
#   composite: per sample 16 B raw + 4 B z + 4 B weights (fwd) / + 16 B grad (bwd)
#   radam    : per table/MLP element 28 B (read p, g, m, v; write p, m, v)
OPS = {
    # (with the TV bins in the hash bin launch, nerf_hash_encode_bwd_bin_batch_tv, their time is the op's)
    "hash_bwd": dict(calls=("nerf_hash_encode_bwd_bin", "nerf_hash_encode_bwd_bin_rows", "nerf_hash_encode_bwd_bin_batch",
                            "nerf_hash_encode_bwd_bin_batch_tv",
                            "nerf_hash_encode_bwd_owner",
                            "nerf_hash_encode_bwd_owner_range", "nerf_hash_encode_bwd_owner_step",
                            "nerf_hash_encode_bwd_ws", "nerf_hash_encode_bwd"),
                     bound="hbm",
                     per_unit=2 * 16 * 8 * 8 + 12 + 128, unit="bwd_hash_point"),
    "hash_fwd": dict(calls=("nerf_hash_encode_fwd",), bound="hbm",
                     per_unit=16 * 8 * 8 + 12 + 128 + 1, unit="hash_point"),
    # A-CAQ eval (int-packed tables, configs[4]): 8-bit codes = 2 B per corner entry (two features)
    "hash_fwd_packed": dict(calls=("nerf_hash_encode_fwd_packed",), bound="hbm", per_unit=16 * 8 * 2 + 12 + 128 + 1,
                            unit="hash_point"),
    "mlp_bwd": dict(calls=("nerf_mlp_bwd", "nerf_mlp_bwd_batch"), bound="mfma", per_unit=2 * 18688, unit="bwd_point"),
    "mlp_fwd": dict(calls=("nerf_mlp_fwd",), bound="mfma", per_unit=18688, unit="point"),
    # the coarse pass's compositing runs in the sampler's launch (nerf_composite_sample_fine): its time
    # is the op's, the sampler's bytes are not priced (a lower bound on the op's fraction)
    "composite_fwd": dict(calls=("nerf_composite_fwd", "nerf_composite_sample_fine", "nerf_composite_fwd_tv"),
                          bound="hbm", per_unit=24,
                          unit="sample"),
    "composite_bwd": dict(calls=("nerf_composite_bwd", "nerf_composite_bwd_batch"), bound="hbm", per_unit=40,
                          unit="sample"),
    "radam": dict(calls=("nerf_radam_step",), bound="hbm", per_unit=28, unit="element"),
}
# algorithmic HBM bytes of one whole iteration per ray at 64 + 128 samples
# (256 points x 3,072 B + 8 x 64 MiB dense table traffic / 4096 + 64 B ray I/O): 3,758,358,528 B
# per 4096-ray step
STEP_BYTES_PER_POINT = 3 * 1024
STEP_DENSE_BYTES = 8 * 16 * (1 << 19) * 2 * 4
STEP_RAY_BYTES = 64


# ABI call -> the kernel symbols it launches (rocprofv3 names), to attach PMC traffic per call
KERNEL_SYMBOLS = {
    "nerf_hash_encode_fwd": ["nerf::hash_encode_fwd_pair_kernel<false>"],
    "nerf_hash_encode_fwd_packed": ["nerf::hash_encode_fwd_packed_pair_kernel"],
    "nerf_hash_encode_bwd_bin": ["nerf::hash_encode_bwd_kernel<3, 512>"],
    "nerf_hash_encode_bwd_bin_rows": ["nerf::hash_encode_bwd_kernel<3, 512>"],
    "nerf_hash_encode_bwd_bin_batch": ["nerf::hash_encode_bwd_pair_kernel<512>"],
    "nerf_hash_encode_bwd_bin_batch_tv": ["nerf::hash_encode_bwd_tv_pair_kernel<512>"],
    "nerf_tv_bwd_bin": ["nerf::tv_bwd_bin_kernel<512>"],
    "nerf_hash_encode_bwd_owner": ["nerf::hash_bwd_owner_kernel<13, 1024, false>"],
    "nerf_hash_encode_bwd_owner_range": ["nerf::hash_bwd_owner_kernel<13, 1024, false>"],
    "nerf_hash_encode_bwd_owner_step": ["nerf::hash_bwd_owner_kernel<13, 1024, false>"],
    "nerf_mlp_fwd": ["nerf::mlp_fwd_x6_kernel<false>"],
    "nerf_mlp_bwd": ["nerf::mlp_bwd_x6cg_kernel<false>"],
    "nerf_mlp_bwd_batch": ["nerf::mlp_bwd_x6cg_kernel<false>"],
    "nerf_radam_step": ["nerf::radam_kernel"],
    "nerf_composite_sample_fine": ["nerf::composite_sample_fine_kernel<1>"],
    "nerf_composite_bwd_batch": ["nerf::composite_bwd_pair_kernel<3, 1>"],
}
# calls whose every launch runs ONE of the listed kernels (the coarse pass's K = 1 and the fine pass's
# K = 3 compositing, one launch each per iteration, with the fused sampler and the batched backward
# off): per-call traffic = the mean over the kernels
KERNEL_VARIANTS = {
    "nerf_composite_fwd": ["nerf::composite_fwd_kernel<1>", "nerf::composite_fwd_kernel<3>"],
    "nerf_composite_bwd": ["nerf::composite_bwd_kernel<1>", "nerf::composite_bwd_kernel<3>"],
}


def base_name(abi_name):
    """nerf_mlp_fwd_q / _ord / _h3 -> nerf_mlp_fwd: the _q entry points are the same kernels with
    optional A-CAQ records (NULL on the unquantized path), _ord with an optional point order, _h3 also
    storing layer C1's outputs for the backward."""
    for suffix in ("_q", "_ord", "_h3"):
        if abi_name.endswith(suffix):
            return abi_name[:-len(suffix)]
    return abi_name


def traffic_file():
    """The newest committed PMC traffic summary (tools/profile_bench.sh), or None."""
    for name in ("r06_traffic.json", "r05_traffic.json", "r04_traffic.json", "r03_traffic.json", "r02_traffic.json", "r01j_traffic.json"):
        path = os.path.join(ROOT, "profiles", name)
        if os.path.exists(path):
            return path
    return None


def pmc_traffic(abi_name):
    """HBM-side bytes per call of `abi_name` from the committed PMC passes (tools/profile_bench.sh:
    FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes of this bench), or None."""
    abi_name = base_name(abi_name)
    path = traffic_file()
    if path is None or (abi_name not in KERNEL_SYMBOLS and abi_name not in KERNEL_VARIANTS):
        return None
    t = json.load(open(path))
    syms = KERNEL_SYMBOLS.get(abi_name) or KERNEL_VARIANTS[abi_name]
    parts = [t.get(k, {}).get("traffic_bytes") for k in syms]
    if any(p is None for p in parts):
        return None
    return float(sum(parts)) / (len(parts) if abi_name in KERNEL_VARIANTS else 1)


def gpu_clocks():
    """Current shader / memory clocks of the visible GPUs (rocm-smi, a child process), so that a
    box-to-box spread in the bench line can be told apart from a code regression. Skipped under
    rocprofv3: its preloaded library would start in the child too (rocm-smi is a script that execs
    its interpreter after that library has initialised the GPU)."""
    import subprocess
    if any(k.startswith("ROCPROF") for k in os.environ):
        return None
    try:
        r = subprocess.run(["rocm-smi", "--showclocks", "--json"], capture_output=True, text=True, timeout=20)
        d = json.loads(r.stdout)
    except Exception:
        return None
    out = {}
    for card, v in d.items():
        if isinstance(v, dict):
            out[card] = {k.split("(")[1].rstrip(")") if "(" in k else k: val for k, val in v.items()
                         if "sclk" in k or "mclk" in k or "fclk" in k}
    return out or None


def op_rooflines(kernels, steps, units, dense_elems, hash_entries=None, fused_elems=0):
    """Per OP (OPS) per iteration: achieved = algorithmic bytes (FLOPs) of the op's units in one
    iteration / the op's summed kernel time in one iteration (HIP events), against the MI355X peak;
    traffic = the committed PMC bytes of the op's kernels per iteration. units: {"point", "sample",
    "hash_point"} counts per iteration. hash_entries: entries the hash backward's bins emitted in one
    iteration (nerf_hash_bwd_entry_count): when they are fewer than 0.1 per point-level the backward
    did not do the priced work (the A-CAQ configuration's zero feature gradients), and the
    op is reported without a roofline fraction. fused_elems: table elements whose RAdam step ran inside
    the owner pass (hashgrid.fused_table_step): priced in hash_bwd at 24 B each (parameter and both
    moments read and written; the gradient is stored once either way and not read back), and out of
    radam's elements."""
    out = []
    for op, d in OPS.items():
        calls = [c for c in kernels if base_name(c) in d["calls"]]
        if not calls:
            continue
        t_step = sum(kernels[c]["total_ms"] for c in calls) * 1e-3 / steps
        n = dense_elems - fused_elems if d["unit"] == "element" else units[d["unit"]]
        work = d["per_unit"] * n + (24 * fused_elems if op == "hash_bwd" else 0)
        traffic = 0.0
        for c in calls:
            tc = pmc_traffic(c)
            if tc is None:
                traffic = None
                break
            traffic += tc * kernels[c]["launches"] / steps
        if d["bound"] == "hbm":
            ach = work / t_step / 1e9
            r = {"op": op, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None if traffic is None else round(traffic),
                 "algorithmic_bytes": work}
        else:
            ach = work / t_step / 1e12
            r = {"op": op, "bound": "mfma", "achieved": round(ach, 2), "peak": round(X6_PEAK_TFLOPS, 1),
                 "unit": "TFLOP/s", "frac": round(ach / X6_PEAK_TFLOPS, 4),
                 "traffic": None if traffic is None else round(traffic), "algorithmic_flops": work,
                 "peak_note": "bf16 dense MFMA peak / 6: each fp32-accurate product is six bf16 products "
                              "(csrc/field_x6.hip)"}
        r.update(ms_per_step=round(1e3 * t_step, 4), calls={c: kernels[c]["launches"] // max(1, steps) for c in calls},
                 units_per_step=n, per_unit=d["per_unit"], unit_name=d["unit"])
        if op == "hash_bwd" and fused_elems:
            r["fused_table_step_bytes"] = 24 * fused_elems
        if op == "hash_bwd" and hash_entries is not None:
            per_pl = hash_entries / max(1, n * 16)
            r.update(entries_per_step=hash_entries, entries_per_point_level=round(per_pl, 3))
            if per_pl < 0.1:
                r.update(degenerate=True, achieved=None, frac=None,
                         note="the bins emitted < 0.1 entries per point-level (zero feature gradients): the kernels "
                              "did not do the priced work, so no roofline fraction is claimed")
        out.append(r)
    out.sort(key=lambda r: -r["ms_per_step"])
    return out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # steady state: after the warm-up's capture and the barrier, the replayed step settles over ~20
    # iterations (1.217 / 1.214 ms averaged over 20 timed steps after 8 warm-ups vs 1.192 / 1.195 ms
    # over 60 after 40 and 1.191 / 1.195 ms over 100 after 8, same box, profiles/r05ap_bench_warmup_length.jsonl)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--rays", type=int, default=4096)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-rays", type=int, default=4096, help="rays of the CPU leg's timed iterations (the bench batch)")
    ap.add_argument("--cpu-warmup", type=int, default=6)
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--profile-kernels", type=int, default=1, help="record HIP events per kernel in the timed region")
    ap.add_argument("--workload", default="lego", choices=sorted(WORKLOADS),
                    help="BASELINE config: lego (configs[1], the headline), fern (configs[2], LLFF NDC), "
                         "scannet (configs[3], normals + structural priors, meant for --gpus 8), "
                         "acaq (configs[4], A-CAQ quantized tables)")
    ap.add_argument("--graph", type=int, default=1,
                    help="train mode: replay the iteration from HIP graphs (graphs.GraphedTrainStep); 0 = eager")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: every rank trains --rays rays (the driver's default); strong: one global batch of "
                         "--rays rays split evenly over the ranks (dist.shard)")
    ap.add_argument("--zero", type=int, default=1,
                    help="N>1: shard the optimizer (reduce-scatter -> RAdam on 1/N -> all-gather, dist.ShardedOptimizer); "
                         "0 = all-reduce + replicated RAdam")
    ap.add_argument("--fused-table-step", type=int, default=1,
                    help="1: the tables' RAdam step runs inside the owner pass (one process; hashgrid.fused_table_step)")
    ap.add_argument("--fused-sampler", type=int, default=1,
                    help="1: the coarse compositing and the hierarchical sampler in one launch "
                         "(render.set_fused_coarse_sampler)")
    ap.add_argument("--batched-composite", type=int, default=1,
                    help="1: the fine and coarse compositing backwards in one launch (render.set_batched_composite_bwd)")
    ap.add_argument("--bin-batch", type=int, default=1,
                    help="1: the pass's hash bins as one launch (field.set_bin_batch)")
    ap.add_argument("--sh-rows", type=int, default=1,
                    help="1: per-ray SH4 rows written by the stratified sampler, loaded by the MLP kernels "
                         "(render.set_sh_rows)")
    ap.add_argument("--fold-fills", type=int, default=1,
                    help="1: the step's gradient and TV-accumulator zero fills run inside render()'s first launch "
                         "(_lib.set_fold_fills)")
    ap.add_argument("--overlap", type=int, default=1,
                    help="N>1 with --zero 1: reduce-scatter the first gradient bucket while the owner pass sums the "
                         "second (dist.ShardedOptimizer(overlap=True)); 0 = one reduce-scatter after the backward")
    ap.add_argument("--deterministic", type=int, default=0,
                    help="1: bitwise-reproducible backward (nerf.set_deterministic: fixed-point hash owner pass, "
                         "ordered MLP weight-gradient reduction)")
    ap.add_argument("--active-points", type=int, default=0,
                    help="1: the field backward walks only the samples with a nonzero raw gradient "
                         "(field.set_active_points; pays on sparse scenes, not on this synthetic workload); "
                         "0: every sample")
    ap.add_argument("--coarse-reuse", type=int, default=1,
                    help="1: the fine pass reuses the coarse pass's hash encoding (DESIGN §8.5); 0: re-encode (A/B)")
    ap.add_argument("--fresh-rays", type=int, default=1,
                    help="also time the step with a new ray batch every iteration (train()'s no_batching draw: "
                         "one random view, N_rand random pixels; blender-rig workloads, graph mode): "
                         "fresh_rays_ms_per_step in the line")
    ap.add_argument("--mode", default="train", choices=["train", "render"],
                    help="train: full training iteration (the metric); render: render-only (eval modules, no grad)")
    return ap.parse_args()


# BASELINE.json configs measured by this bench (the default line is configs[1], lego)
WORKLOADS = {
    "lego": dict(args=dict(finest_res=1024, N_samples=64, N_importance=128, white_bkgd=True, perturb=1.0,
                           lrate_decay=500, tv_loss_weight=1e-6),
                 near=2.0, far=6.0, rays="blender",
                 desc="lego train step: {R} rays/GPU x (64 coarse + 128 fine) samples, finest_res 1024, L=16, F=2, "
                      "T=2^19, RAdam, TV+sparsity losses"),
    "fern": dict(args=dict(finest_res=512, N_samples=64, N_importance=64, white_bkgd=False, perturb=1.0,
                           raw_noise_std=1.0, dataset_type="llff", tv_loss_weight=1e-6),
                 near=0.0, far=1.0, rays="llff", ndc=True,
                 desc="fern (LLFF) train step: {R} rays/GPU x (64 coarse + 64 fine) samples, NDC, raw noise 1, "
                      "finest_res 512, RAdam, TV+sparsity losses"),
    "scannet": dict(args=dict(finest_res=512, N_samples=64, N_importance=128, white_bkgd=False, perturb=1.0,
                              lrate_decay=500, tv_loss_weight=1e-6, use_structural_priors=True,
                              structural_loss_start_iter=0, structural_loss_ramp_iters=1),
                    near=0.1, far=10.0, rays="scannet",
                    desc="ScanNet-like indoor train step: {R} rays/GPU x (64 + 128) samples, near 0.1 far 10, normals "
                         "head (7-channel compositing), structural priors (Manhattan + planarity + normal "
                         "consistency, full ramp), RAdam, TV+sparsity losses"),
    "acaq": dict(args=dict(finest_res=1024, N_samples=64, N_importance=128, white_bkgd=True, perturb=1.0,
                           lrate_decay=500, tv_loss_weight=1e-6, use_quantization=True, quantization_bits=8),
                 near=2.0, far=6.0, rays="blender", quantized=True,
                 desc="lego + A-CAQ train step: {R} rays/GPU x (64 + 128) samples, 8-bit learned-bitwidth quantizers "
                      "on the 16 levels, W0 and the hidden activation (past warm-up, calibrated)"),
}


PRODUCT_TREE = ("indoor-nerf_amd", "include")


def product_tree_sha():
    """sha256 over the product's sources (indoor-nerf_amd/*.py, csrc/*, include/*.h), path-sorted:
    identifies the tree a committed result (profiles/*_psnr_vs_reference.json) was produced by. Works
    without git (the GPU box receives the tree without .git)."""
    import hashlib
    h = hashlib.sha256()
    files = []
    for top in PRODUCT_TREE:
        for dp, dns, fns in os.walk(os.path.join(ROOT, top)):
            dns[:] = sorted(d for d in dns if d != "__pycache__")
            files += [os.path.join(dp, f) for f in fns if f.endswith((".py", ".hip", ".h", ".cpp"))]
    for f in sorted(files):
        h.update(os.path.relpath(f, ROOT).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def cpu_threads():
    """Threads for the CPU legs: (logical CPUs of this process's affinity mask, the job's CPU share
    (OMP_NUM_THREADS: 16 per GPU on the pool's boxes, whose affinity mask shows the whole machine;
    unset here: the mask alone), physical cores of the mask (all physical cores))."""
    cpus = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count()))
    share = os.environ.get("OMP_NUM_THREADS")
    physical = set()
    for c in cpus:
        base = f"/sys/devices/system/cpu/cpu{c}/topology/"
        try:
            physical.add((open(base + "physical_package_id").read().strip(), open(base + "core_id").read().strip()))
        except OSError:
            physical.add(("cpu", str(c)))
    return len(cpus), max(1, min(len(cpus), int(share))) if share else len(cpus), max(1, len(physical))


def cpu_leg(n_rays, finest, H, warmup, timed):
    """The oracle (CPU PyTorch restatement of the reference, oracle/nerf_oracle.py) on one bounded
    sample: a full training iteration (coarse 64 + fine 128 render, MSE x2 + sparsity + TV, backward,
    RAdam) on n_rays rays of the synthetic Blender rig at H x H, `warmup` iterations first (RAdam's
    update is a no-op until N_sma >= 5 at step 6, radam.py:63-92) and the median of `timed`; then the
    median of `timed` render-only passes (no grad) of the same rays."""
    from oracle import nerf_oracle as orc
    from indoor_nerf_amd.synthetic import blender_bbox, blender_rays
    lo, hi = (torch.from_numpy(v) for v in blender_bbox())
    res = orc.level_resolutions(16, finest)
    g = torch.Generator().manual_seed(0)
    tabs = [((torch.rand(1 << 19, 2, generator=g) * 2 - 1) * 1e-4).requires_grad_(True) for _ in range(16)]
    cw = {k: v.requires_grad_(True) for k, v in orc.mlp_init(1).items()}
    fw = {k: v.requires_grad_(True) for k, v in orc.mlp_init(2).items()}
    opt = orc.RAdamOracle([dict(params=list(cw.values()) + list(fw.values()), lr=5e-4, betas=(0.9, 0.99), eps=1e-8,
                                weight_decay=1e-6), dict(params=tabs, lr=5e-4, betas=(0.9, 0.99), eps=1e-15,
                                                         weight_decay=0)])
    ro, rd = (torch.from_numpy(v) for v in blender_rays(n_rays, H=H, W=H, seed=11))
    vd = orc.viewdirs_of(rd)
    target = torch.rand(n_rays, 3, generator=g)

    def step():
        out = orc.render_rays(ro, rd, vd, 2.0, 6.0, cw, fw, tabs, lo, hi, res)
        for p in list(cw.values()) + list(fw.values()) + tabs:
            p.grad = None
        loss = torch.mean((out["rgb_map"] - target) ** 2) + torch.mean((out["rgb0"] - target) ** 2)
        loss = loss + 1e-10 * (out["sparsity_loss"].sum() + out["sparsity_loss0"].sum())
        tv = 0
        for lvl in range(16):
            r, cube = orc.tv_cube(lvl, 16, finest)
            mv = torch.randint(0, r - cube, (3,), generator=g)
            tv = tv + orc.tv_loss(tabs[lvl], lvl, mv, 16, finest)
        loss = loss + 1e-6 * tv
        loss.backward()
        opt.step()

    for k in range(warmup):
        t0 = time.perf_counter()
        step()
        print(f"cpu leg {n_rays} rays finest {finest}: warm-up {k} {time.perf_counter() - t0:.2f} s", file=sys.stderr,
              flush=True)
    times = []
    for _ in range(timed):
        t0 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t0)
        print(f"cpu leg {n_rays} rays finest {finest}: timed {times[-1]:.2f} s", file=sys.stderr, flush=True)
    t = float(np.median(times))
    rt = []
    with torch.no_grad():
        for _ in range(timed):
            t0 = time.perf_counter()
            orc.render_rays(ro, rd, vd, 2.0, 6.0, cw, fw, tabs, lo, hi, res)
            rt.append(time.perf_counter() - t0)
    return {"value": round(n_rays / t, 2), "unit": "rays/s", "step_s": round(t, 3),
            "render_only": {"value": round(n_rays / float(np.median(rt)), 2), "unit": "rays/s"},
            "sample": f"{n_rays} rays of a {H}x{H} Blender rig x (64 coarse + 128 fine) samples, finest_res {finest}, "
                      f"full train iteration incl. TV + RAdam; median of {timed} iterations after {warmup} warm-up "
                      f"iterations (RAdam active); render-only = median of {timed} no-grad passes"}


def cpu_baseline(n_rays, warmup, timed):
    """SURVEY.md §8(d)'s CPU baseline on the GPU box's host cores, rank 0 at N=1 only. `value` is the
    lego leg (configs[1]: finest 1024, 800x800) at the bench's own batch (n_rays = 4096), `warmup`
    (6) warm-up iterations, so RAdam's update is active (radam.py:63-92: N_sma >= 5 from step 6), and
    the median of `timed` (3). The chair leg is BASELINE configs[0] (chair 400x400, finest_res 512, the
    reference's CPU path: configs/chair.txt) at its own N_rand of 1024.

    Threads: the fastest count measured on the pool's boxes. Their affinity mask shows the whole
    machine (256 logical / 128 physical cores) but the job runs in a CPU share of 16
    (OMP_NUM_THREADS); the same iteration at 16 / 32 / 64 / 128 threads took 13.3 / 16.5 / 22.6 /
    39.4 s (profiles/r06w_cpu_threads.json, tools/cpu_threads_probe.py): every physical core of the
    mask is 3x SLOWER than the share, and at 128 threads this leg alone ran past the box's silence
    limit. So the leg runs at min(physical cores, share) threads, and the line carries the
    full-mask probe beside it."""
    logical, share, physical = cpu_threads()
    threads = min(physical, share)
    torch.set_num_threads(threads)
    lego = cpu_leg(n_rays, 1024, 800, warmup, timed)
    chair = cpu_leg(1024, 512, 400, warmup, timed)
    chair["threads"] = threads
    probe = None
    pf = os.path.join(ROOT, "profiles", "r06w_cpu_threads.json")
    if os.path.exists(pf):
        probe = {"source": "profiles/r06w_cpu_threads.json",
                 "rays_per_s_by_threads": {str(r["threads"]): r["rays_per_s"] for r in json.load(open(pf))["rows"]}}
    return {"value": lego["value"], "unit": "rays/s", "cores": threads, "kind": "port",
            "render_only": lego["render_only"], "step_s": lego["step_s"],
            "sample": "lego leg: " + lego["sample"],
            "cpu": cpu_model(), "affinity_cpus": logical, "physical_cores": physical, "job_share_threads": share,
            "threads_note": "torch.set_num_threads = min(physical cores of the affinity mask, the job's CPU share "
                            "OMP_NUM_THREADS): the fastest count measured on these boxes (more threads than the share "
                            "run slower: full_mask_probe)",
            "full_mask_probe": probe,
            "chair": {**chair, "config": "BASELINE configs[0]: chair 400x400, finest_res 512 (configs/chair.txt)"}}


def fresh_rays_leg(a, kw, opt, args, arena, hook, post, world, dev, it, rank):
    """The same training step with a NEW ray batch every iteration, as train() draws it for the lego
    config (configs/lego.txt: no_batching = True; run_nerf.py:975-1004): one of the rig's 100 training
    views (np.random.choice) and N_rand = R distinct pixels of it (rays.RaySampler: the image set and
    the cameras resident in HBM, one nerf_sample_rays_sel launch inside the captured step reading the
    replay's (image, seed, offset) slot). Past the precrop phase (precrop_iters = 500 of 8,001
    iterations): the whole 800 x 800 image. Synthetic images (no dataset on the box): U[0,1) colours.
    Returns (ms per step over a.steps timed steps after a.warmup, the next iteration index)."""
    from indoor_nerf_amd import RaySampler
    from indoor_nerf_amd.graphs import GraphedTrainStep
    from indoor_nerf_amd.synthetic import CAMERA_ANGLE_X, pose_spherical
    H = W = 800
    n_img = 100
    focal = 0.5 * W / np.tan(0.5 * CAMERA_ANGLE_X)
    K = np.array([[focal, 0, 0.5 * W], [0, focal, 0.5 * H], [0, 0, 1]])
    poses = np.stack([pose_spherical(t, -30.0, 4.0311) for t in np.linspace(-180, 180, n_img + 1)[:-1]])
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    images = torch.rand(n_img, H, W, 3, device=dev, generator=g)
    R = a.rays if a.scaling == "weak" else a.rays // world
    np.random.seed(2000 + rank)            # the image draw (np.random.choice, as train())
    sampler = RaySampler(images, poses, H, W, K, np.arange(n_img), R, precrop_iters=0, device=dev)
    del images
    rays = (torch.empty(R, 3, device=dev), torch.empty(R, 3, device=dev))
    target = torch.empty(R, 3, device=dev)
    tv_gen = torch.Generator().manual_seed(8)
    st = GraphedTrainStep(rays, target, kw, opt, args, H=H, W=W, grad_hook=hook, loss_scale_sparsity=float(world),
                          tv_generator=tv_gen, zero_grad=arena.zero_, post_hook=post, sampler=sampler)
    for _ in range(a.warmup):
        st(it)
        it += 1
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        st(it)
        it += 1
    wait = getattr(getattr(post, "__self__", None), "wait_params", None)
    if wait is not None:
        wait()                             # the last step's gated all-gather (ZeRO-1 with overlap)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    return 1e3 * elapsed / a.steps, it, bool(st.captures > 0)


def launch_ranks(a):
    """`--gpus N` (N > 1) without torchrun's environment: start the N rank processes here (torch's
    elastic launcher as a CHILD process, one rank per GPU, rendezvous on 127.0.0.1) and return its
    exit status. Nothing in this process has touched the GPU (torch.cuda.device_count() does not
    initialise it on this image). Refuses when fewer than N GPUs are visible: RCCL rejects two ranks
    on one GPU ("Duplicate GPU detected"), and a line with fewer ranks would misreport n_gpus.
    NERF_DIST_BACKEND=gloo rehearses N ranks on fewer GPUs (host-staged collectives)."""
    import socket
    import subprocess
    visible = torch.cuda.device_count()
    if visible < a.gpus and os.environ.get("NERF_DIST_BACKEND") != "gloo":
        print(f"bench.py: --gpus {a.gpus} needs {a.gpus} GPUs, {visible} visible; refusing (RCCL rejects two ranks "
              f"on one GPU: 'Duplicate GPU detected'; NERF_DIST_BACKEND=gloo rehearses the ranks on fewer GPUs)",
              file=sys.stderr, flush=True)
        return 3
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def main():
    a = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and a.gpus > 1:
        sys.exit(launch_ranks(a))
    if world_env is not None and int(world_env) != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world_env} (torchrun --nproc-per-node must equal --gpus)",
              file=sys.stderr, flush=True)
        sys.exit(2)
    if a.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if a.gpus > 1 and torch.cuda.device_count() < a.gpus and os.environ.get("NERF_DIST_BACKEND") != "gloo":
        print(f"bench.py: rank of a {a.gpus}-GPU run with {torch.cuda.device_count()} GPUs visible; refusing (RCCL "
              f"rejects two ranks on one GPU: 'Duplicate GPU detected')", file=sys.stderr, flush=True)
        sys.exit(3)
    import indoor_nerf_amd as nerf
    from indoor_nerf_amd import _lib
    from indoor_nerf_amd.synthetic import blender_bbox, blender_rays, llff_bbox, llff_rays

    wl = WORKLOADS[a.workload]
    # NERF_DIST_FORCE=1: a one-rank process group (RCCL on one GPU) running the N > 1 code path — ZeRO-1
    # reduce-scatter / RAdam on the shard / gated all-gather — as a hardware rehearsal of it
    force_dist = os.environ.get("NERF_DIST_FORCE") == "1"
    rank, world, local = nerf.init_process_group(force=force_dist)
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))   # ranks > GPUs only in rehearsals
    torch.cuda.set_device(dev)
    strong = a.scaling == "strong"
    if strong and a.rays % world:
        raise SystemExit(f"--scaling strong: --rays {a.rays} is not divisible by {world} ranks")
    # weak: each rank its own batch; strong: the same global batch on every rank, then its shard
    seed = 100 if strong else 100 + rank
    if wl["rays"] == "blender":
        lo, hi = blender_bbox()
        ro, rd = blender_rays(a.rays, seed=seed)
        H = W = 800
        K = None
    elif wl["rays"] == "scannet":
        from indoor_nerf_amd.synthetic import scannet_bbox, scannet_rays
        lo, hi = scannet_bbox()
        ro, rd, _coords = scannet_rays(a.rays, seed=seed)
        H, W, K = 480, 640, None
    else:
        lo, hi = llff_bbox()
        ro, rd, (H, W, K) = llff_rays(a.rays, seed=seed)
    if strong:
        ro = nerf.shard(torch.from_numpy(ro), rank, world).numpy()
        rd = nerf.shard(torch.from_numpy(rd), rank, world).numpy()
    R = ro.shape[0]              # this rank's rays per step
    args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), **wl["args"])
    torch.manual_seed(0)
    nerf.manual_seed(1234 + rank)
    if a.deterministic:
        nerf.set_deterministic(True)
    nerf.set_coarse_reuse(bool(a.coarse_reuse))
    nerf.set_fused_table_step(bool(a.fused_table_step))
    nerf.set_fused_coarse_sampler(bool(a.fused_sampler))
    nerf.set_batched_composite_bwd(bool(a.batched_composite))
    nerf.set_active_points(bool(a.active_points))
    _lib.set_fold_fills(bool(a.fold_fills))
    nerf.set_sh_rows(bool(a.sh_rows))
    from indoor_nerf_amd import field as _field
    _field.set_bin_batch(bool(a.bin_batch))
    kw, kw_test, _, grad_vars, opt = nerf.create_nerf(args, device=dev)
    for d in (kw, kw_test):
        d.update(near=wl["near"], far=wl["far"])     # train() adds the scene bounds (run_nerf.py:768-770,865-869)
    if wl.get("ndc"):
        for d in (kw, kw_test):
            d.update(ndc=True, lindisp=False)
    if wl.get("quantized"):
        kw["embed_fn"].current_step = kw["embed_fn"].warmup_steps   # past the 500-call warm-up (hash_encoding.py:97)
    params = grad_vars + list(kw["embed_fn"].parameters())
    nerf.broadcast_params(params)
    zero = (world > 1 or force_dist) and a.zero and a.mode == "train"
    # defer_tables: no memset of the 64 MiB of table gradients; the owner pass overwrites them.
    # ZeRO-1 with --overlap: two gradient buckets (MLP + table levels 0..7 | levels 8..15), the first
    # reduce-scattered while the owner pass sums the second (dist.ShardedOptimizer)
    tabs = kw["embed_fn"].tables()
    split = [tabs[len(tabs) // 2]] if (zero and a.overlap) else []
    arena = nerf.GradArena(params, pad_to=world * 64 if zero else 1, defer_tables=True, bucket_starts=split)
    rays = (torch.from_numpy(ro).to(dev), torch.from_numpy(rd).to(dev))
    if strong:
        target = nerf.shard(torch.rand(a.rays, 3, device=dev, generator=torch.Generator(device=dev).manual_seed(0)),
                            rank, world).contiguous()
    else:
        target = torch.rand(R, 3, device=dev, generator=torch.Generator(device=dev).manual_seed(rank))
    tv_gen = torch.Generator().manual_seed(7)       # same TV cuboids on every rank
    post = None
    if zero:
        sharded = nerf.ShardedOptimizer(opt, arena, overlap=bool(a.overlap))
        hook, post = sharded.reduce_grads, sharded.gather_params
    else:
        hook = (lambda: arena.allreduce_mean()) if (world > 1 or force_dist) else None

    gstep = None
    if a.mode == "train" and a.graph:
        from indoor_nerf_amd.graphs import GraphedTrainStep
        gstep = GraphedTrainStep(rays, target, kw, opt, args, H=H, W=W, K=K, grad_hook=hook,
                                 loss_scale_sparsity=float(world), tv_generator=tv_gen, zero_grad=arena.zero_,
                                 post_hook=post)
        step = gstep
    elif a.mode == "train":
        def step(i):
            return nerf.train_step(rays, target, kw, opt, args, i, H=H, W=W, K=K, grad_hook=hook,
                                   loss_scale_sparsity=float(world), tv_generator=tv_gen, zero_grad=arena.zero_,
                                   post_hook=post)
    else:
        for m in (kw["network_fn"], kw["network_fine"], kw["embed_fn"]):
            m.eval()

        def step(i):
            with torch.no_grad():
                rgb, _, _, _ = nerf.render(H, W, K, chunk=args.chunk, rays=rays, **kw_test)
            return rgb.mean(), rgb.mean()

    it = 1
    if wl.get("quantized") and a.mode == "render":
        # calibrate the quantizers with one training iteration first (they calibrate on their
        # first training call), then switch to eval (int-packed tables)
        for m in (kw["network_fn"], kw["network_fine"], kw["embed_fn"]):
            m.train()
        nerf.train_step(rays, target, kw, opt, args, 1, H=H, W=W, K=K, tv_generator=tv_gen, zero_grad=arena.zero_)
        for m in (kw["network_fn"], kw["network_fine"], kw["embed_fn"]):
            m.eval()
    for _ in range(a.warmup):
        step(it)
        it += 1
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    if a.profile_kernels and gstep is None:
        _lib.set_timing(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss, psnr = step(it)
        it += 1
    if zero:
        sharded.wait_params()      # the last step's gated all-gather is part of the timed work
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if gstep is not None:
        gstep.check()              # every replay fetched its own scalar slot (outside the timed region)
    clocks = gpu_clocks() if rank == 0 else None
    recs = _lib.timing_records()
    _lib.set_timing(False)
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())

    # per-kernel timing: eager -> HIP-event pairs around every launch of the timed region. graph ->
    # torch on ROCm cannot capture timing events, so K further iterations of the same launches run
    # eagerly right after the timed region with the event pairs (same kernels, inputs and state)
    per = {}
    if gstep is not None and a.profile_kernels:
        _lib.set_timing(True)
        for _ in range(a.steps):
            gstep.eager_step(it)
            it += 1
        torch.cuda.synchronize()
        recs = _lib.timing_records()
        _lib.set_timing(False)
    for name, e0, e1 in recs:
        per.setdefault(name, []).append(e0.elapsed_time(e1) * 1e-3)
    kernels = {}
    for name, ts in per.items():
        kernels[name] = {"launches": len(ts), "avg_ms": 1e3 * float(np.mean(ts)), "total_ms": 1e3 * float(np.sum(ts))}
    roofline, ops = None, []
    ns, ni = wl["args"]["N_samples"], wl["args"]["N_importance"]
    points_per_step = R * (ns + (ns + ni if ni else 0))
    # distinct points the hash encoding handles: fewer when the fine pass reused the coarse features
    from indoor_nerf_amd.render import last_reuse_used
    from indoor_nerf_amd.hashgrid import last_fused_table_step
    fused_step = last_fused_table_step()
    reused = last_reuse_used()
    units = {"point": points_per_step, "sample": points_per_step,
             "hash_point": R * (ns + ni) if (reused and ni) else points_per_step}
    units["bwd_point"], units["bwd_hash_point"] = units["point"], units["hash_point"]
    hash_entries = active = None
    if kernels and a.mode == "train":
        from indoor_nerf_amd.field import last_active_units
        from indoor_nerf_amd.hashgrid import pending_bins
        hash_entries = pending_bins(dev).last_entry_count()
        active = last_active_units()
        if active is not None:
            # the backward walks the active points only (field.set_active_points): price the work it did
            units["bwd_point"] = active["mlp_points"]
            units["bwd_hash_point"] = active["hash_points"]
    if kernels:
        # with the fused sampler only the fine pass calls nerf_composite_fwd: its own K kernel
        if a.fused_sampler and ni:
            KERNEL_VARIANTS["nerf_composite_fwd"] = [f"nerf::composite_fwd_kernel<{(ns + ni + 63) // 64}>"]
        if a.batched_composite and ni:
            KERNEL_SYMBOLS["nerf_composite_bwd_batch"] = [
                f"nerf::composite_bwd_pair_kernel<{(ns + ni + 63) // 64}, {(ns + 63) // 64}>"]
        from indoor_nerf_amd.hashgrid import last_fused_table_step
        fused_elems = sum(t.numel() for t in kw["embed_fn"].tables()) if last_fused_table_step() else 0
        ops = op_rooflines(kernels, a.steps, units, sum(p.numel() for p in params), hash_entries, fused_elems)
        ranked = [o for o in ops if not o.get("degenerate")]
        if ranked:
            # the dominant op: largest kernel time per iteration after grouping (hash bwd = bin + owner)
            d = ranked[0]
            roofline = {k: d[k] for k in ("bound", "achieved", "peak", "unit", "frac", "traffic")}
            roofline.update(op=d["op"], ms_per_step=d["ms_per_step"], calls_per_step=d["calls"],
                            units_per_step=d["units_per_step"], per_unit=d["per_unit"], unit_name=d["unit_name"],
                            top3=[{k: o[k] for k in ("op", "bound", "ms_per_step", "achieved", "unit", "frac")}
                                  for o in ranked[:3]])
            if d["traffic"] is not None:
                roofline["traffic_source"] = (os.path.relpath(traffic_file(), ROOT) + ": rocprofv3 FETCH_SIZE x the "
                                              "calibrated factor per access pattern (x2 for 4/8/16-B per-lane reads; "
                                              "x1.56 for the owner pass's 8-B + 2-B entries: "
                                              "profiles/r03a_pmc_calibration.json) + WRITE_SIZE per call, separate "
                                              "PMC passes of this bench, x calls per iteration")
    fresh = None
    if a.fresh_rays and gstep is not None and wl["rays"] == "blender":
        fresh_ms, it, fresh_graphed = fresh_rays_leg(a, kw, opt, args, arena, hook, post, world, dev, it, rank)
        fresh = {"ms_per_step": round(fresh_ms, 3),
                 "value": round((a.rays if strong else world * a.rays) / (fresh_ms * 1e-3), 1), "unit": "rays/s",
                 "hip_graph": fresh_graphed,
                 "batch": "a new batch every iteration as train() draws it for configs/lego.txt (no_batching): one "
                          "of 100 lego-rig views at random, R distinct random pixels of the whole 800x800 image "
                          "(past precrop), drawn on the device inside the captured step (nerf_sample_rays_sel); "
                          "synthetic U[0,1) images",
                 "vs_fixed_batch_ms": round(fresh_ms - 1e3 * elapsed / a.steps, 3)}
    step_s = elapsed / a.steps
    step_bytes = points_per_step * STEP_BYTES_PER_POINT + STEP_DENSE_BYTES + R * STEP_RAY_BYTES
    step_roofline = None
    if a.mode == "train":
        # the whole iteration's algorithmic HBM bytes over its wall time
        step_roofline = {"bytes_per_step": step_bytes, "achieved": round(step_bytes / step_s / 1e9, 1),
                         "unit": "GB/s", "peak": HBM_PEAK_GBS,
                         "frac": round(step_bytes / step_s / 1e9 / HBM_PEAK_GBS, 4),
                         "bound_ms": round(1e3 * step_bytes / (HBM_PEAK_GBS * 1e9), 4)}

    value = (a.rays if strong else world * a.rays) * a.steps / elapsed
    out = {
        "metric": (f"train rays/sec ({R} rays x {(ns + ni) if ni else ns} samples)" if a.mode == "train"
                   else "render rays/sec (eval)"),
        "value": round(value, 1),
        "unit": "rays/s",
        "n_gpus": a.gpus,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(1e3 * elapsed / a.steps, 3),
        "higher_is_better": True,
        "scaling": a.scaling,
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic ({} rays, random-init hash tables and MLPs)".format(
            {"blender": "lego spiral-pose", "llff": "forward-facing LLFF rig", "scannet": "indoor room"}[wl["rays"]]),
        "config": {"workload": wl["desc"].format(R=R) + ("" if a.mode == "train" else " [render only]"),
                   "name": a.workload, "rays_per_gpu": R, "global_batch": R * world,
                   "samples": f"{wl['args']['N_samples']}+{wl['args']['N_importance']}",
                   "parallelism": f"dp{world}" + ("-zero1" if zero else "") + ("-overlap" if zero and a.overlap else "")},
        "hip_graph": bool(gstep is not None and gstep.captures > 0),
        "coarse_reuse": reused,
        "fused_table_step": fused_step,
        "fused_coarse_sampler": bool(a.fused_sampler and ni),
        "batched_composite_bwd": bool(a.batched_composite and ni),
        "active_points": None if active is None else {"fraction": round(active["fraction"], 4),
                                                      "mlp_bwd_points": active["mlp_points"],
                                                      "hash_bwd_points": active["hash_points"]},
        "loss": round(float(loss), 6),
        "fresh_rays_ms_per_step": None if fresh is None else fresh["ms_per_step"],
        "fresh_rays": fresh,
        "roofline": roofline,
        "step_roofline": step_roofline,
        "ops": ops,
        "gpu_clocks": clocks,
        "kernels": {k: {kk: round(vv, 4) if isinstance(vv, float) else vv for kk, vv in v.items()}
                    for k, v in sorted(kernels.items(), key=lambda kv: -kv[1]["total_ms"])},
    }
    if a.deterministic:
        out["deterministic"] = True
    if force_dist:
        out["dist_rehearsal"] = (f"one-rank {torch.distributed.get_backend()} process group: the N > 1 code path "
                                 f"({'ZeRO-1' if zero else 'all-reduce'}), collectives of one rank")
    # north star "PSNR within 0.1 dB of reference": the committed result of tests/test_gpu_converge.py
    # (the reference trained on F19 six times vs six HIP runs; late-phase mean PSNR difference per metric)
    for name in [f"r0{k}_psnr_vs_reference.json" for k in range(6, 1, -1)]:
        pv = os.path.join(ROOT, "profiles", name)
        if os.path.exists(pv):
            pj = json.load(open(pv))
            out["psnr_vs_reference"] = {k: {"d_db": v["d_db"], "reference_db": v["reference_db"], "hip_db": v["hip_db"]}
                                        for k, v in pj.items() if isinstance(v, dict) and "d_db" in v}
            if isinstance(pj.get("design"), str):
                out["psnr_vs_reference"]["runs"] = pj["design"]
            if isinstance(pj.get("all_seeds"), dict):
                out["psnr_vs_reference"]["with_oracle_runs"] = {
                    k: v["d_db"] for k, v in pj["all_seeds"].items() if isinstance(v, dict)}
            out["psnr_vs_reference"]["source"] = "profiles/" + name + (
                " (commit " + pj["commit"] + ")" if isinstance(pj.get("commit"), str) else "")
            # stale: the file was produced by another product tree than the one benched here (or does not
            # say which); tests/test_gpu_converge.py re-checks the bar at every GPU test run
            out["psnr_vs_reference"]["tree_sha"] = pj.get("tree_sha")
            out["psnr_vs_reference"]["stale"] = pj.get("tree_sha") != product_tree_sha()
            break
    if rank == 0 and world == 1 and not a.no_cpu_baseline and a.workload == "lego" and a.mode == "train":
        out["cpu_baseline"] = cpu_baseline(a.cpu_rays, a.cpu_warmup, a.cpu_steps)
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
