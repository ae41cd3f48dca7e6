"""Convergence parity (north star: "PSNR within 0.1 dB of reference"), needs an MI355X.

Reference fixtures (tests/golden/make_golden.py, the reference's own code trained on the CPU):
  F19  the reference trained 300 iterations on a procedural two-sphere scene (tables.convergence_rays):
       256 rays per iteration drawn with a seeded RandomState, coarse 64 + fine 128 samples with the
       pytest=True draws, img + img0 MSE + sparsity, RAdam with create_nerf's param groups, lr decay;
       every 20 iterations the PSNR of held-out pixels of the training views and of a novel view, and
       the PSNR of every training batch. Six runs (8, 4, 6, 2, 3, 5 CPU threads).
  F19b F19 again from twelve one-ulp perturbations of 1 % of the initial table entries.
  F19c the same training with each run's ray batches drawn from its own seed (100, 101, ...).
  F19d more runs of F19c's kind (seeds 200, 201, ...) computed by the oracle on the GPU box's CPU cores
       (tests/golden/make_oracle_converge.py): at a matching thread count the oracle reproduces the
       reference's runs through the chaotic regime (F19's 2-thread run to 1.6e-6 dB over 100
       iterations; tests/test_oracle_golden.py::test_oracle_reproduces_reference_seed_run), so another
       CPU is another rounding of the same algorithm — another sample of the reference's runs.

Why F19c decides. RAdam (radam.py:58-92, betas (0.9, 0.99)) makes no update while N_sma < 5: the first
update is step 6. Before it, the HIP path reproduces the reference's training PSNR to 1e-6 dB. At it,
the two part DETERMINISTICALLY: every one of 24 HIP runs on F19's batches gives the same PSNR at
iteration 7, and so does every reference run (six thread counts, twelve perturbed starts), 0.08 dB
apart (profiles/r03j_converge_first_iterations.txt). The per-element table gradients of this initial
state are ill-conditioned — HIP vs the oracle differ by a median 0.2-3 % per element, and so does the
oracle vs itself with only its compositing moved to fp64 (profiles/r03j_converge_grad_diff_step1.json)
— and RAdam's eps 1e-15 normalises every element's step, so the first update depends on rounding
details that no reference run varies. All F19/F19b runs therefore share one early trajectory and all
HIP runs another; comparing those two conditional ensembles measured the luck of two early
trajectories (the "lag at iterations 40-80" of rounds 1-2). With their own batches (F19c) the sign of
the iteration-7 difference changes from seed to seed (HIP higher, lower, or identical), and the
comparison is over the training's randomness itself.

The test: for every F19c / F19d seed, K HIP runs replay that seed's batches (same initial state); per seed
d = mean(HIP) - run for the late-phase (iterations 100-300) mean of each metric — held-out pixels,
the novel view, the training batches — and D = the mean of d over seeds. Bars:
  * |D| <= 0.1 dB for every metric over the F19c seeds alone — runs of the reference itself (the
    north star, fixed) — and over all seeds (F19c + the oracle's F19d runs, which only add samples);
  * per checkpoint (every 20 iterations, and 20-iteration windows of training PSNR): a paired t-test
    over seeds, Bonferroni over all checkpoints at a family-wise 1 % (+0.02 dB for the iterations
    before the first update, where both sides agree to 1e-6 dB).
F19's batches are trained too (HIP six runs vs F19 + F19b) and reported, not asserted.
"""
import ast

import numpy as np
import pytest
import torch

from tables import blender_bbox, closed_form_table, convergence_rays

pytestmark = pytest.mark.gpu

K = 1               # HIP runs per batch seed: the single reference run per seed dominates the variance, and
                    # the suite must not fall silent for minutes (~0.4 s per HIP run)
LATE = 100          # late phase: iterations LATE..300


def _net(nerf, gpu, d, prefix):
    net = nerf.NeRFSmall(num_layers=2, hidden_dim=64, geo_feat_dim=15, num_layers_color=3, hidden_dim_color=64,
                         input_ch=32, input_ch_views=16).to(gpu)
    with torch.no_grad():
        for k, p in net.named_parameters():
            p.copy_(torch.from_numpy(d[prefix + k.replace(".", "_")]))
    return net


def _late(name, x, every):
    """Late-phase mean: checkpoints at iterations LATE..300, or training batches LATE+1..300."""
    if name == "train_psnr":
        return x[..., LATE:].mean(-1)
    return x[..., LATE // every:].mean(-1)


@pytest.mark.timeout(900)   # ~0.4 s per HIP run: K runs x ~150 seeds, plus F19's six
def test_convergence_psnr_within_0p1_db(nerf, gpu, golden):
    g = golden("f19_converge")
    cs = golden("f19c_converge")
    c = ast.literal_eval(str(g["config"]))
    every = c["every"]
    lo, hi = blender_bbox()
    emb = nerf.HashEmbedder((torch.from_numpy(lo), torch.from_numpy(hi)), finest_resolution=1024).to(gpu)
    table = closed_form_table(scale=c["table_scale"], salt=c["table_salt"])
    coarse, fine = _net(nerf, gpu, g, "coarse0_"), _net(nerf, gpu, g, "fine0_")
    sh = nerf.SHEncoder()
    nqf = lambda inputs, viewdirs, fn: nerf.run_network(inputs, viewdirs, fn, emb, sh)  # noqa: E731
    kw = dict(network_query_fn=nqf, perturb=1.0, N_importance=128, network_fine=fine, N_samples=64,
              network_fn=coarse, embed_fn=emb, use_viewdirs=True, white_bkgd=True, raw_noise_std=0.0,
              predict_normals=False, ndc=False, lindisp=False, near=2.0, far=6.0, pytest=True)
    kw_test = dict(kw, perturb=0.0, raw_noise_std=0.0, pytest=False)
    args = nerf.make_args(lrate=c["lrate"], lrate_decay=c["lrate_decay"], sparse_loss_weight=c["sparsity"],
                          tv_loss_weight=0.0, N_samples=64, N_importance=128, white_bkgd=True)
    (ro, rd, rgb), (eo, ed, ergb), (no, nd, nrgb) = convergence_rays()
    n_pool = ro.shape[0]
    ro, rd, rgb = (torch.from_numpy(a).to(gpu) for a in (ro, rd, rgb))
    eo, ed, ergb = (torch.from_numpy(a).to(gpu) for a in (eo, ed, ergb))
    no, nd, nrgb = (torch.from_numpy(a).to(gpu) for a in (no, nd, nrgb))

    def psnr_of(o, d, target):
        with torch.no_grad():
            out, _, _, _ = nerf.render(800, 800, None, rays=(o, d), **kw_test)
            return (-10.0 * torch.log10(((out - target) ** 2).mean())).item()

    def train_run(batches):
        with torch.no_grad():
            for i, e in enumerate(emb.embeddings):
                e.weight.copy_(torch.from_numpy(table[i]))
            for net, prefix in ((coarse, "coarse0_"), (fine, "fine0_")):
                for k, p in net.named_parameters():
                    p.copy_(torch.from_numpy(g[prefix + k.replace(".", "_")]))
        opt = nerf.RAdam([{"params": list(coarse.parameters()) + list(fine.parameters()), "weight_decay": 1e-6},
                          {"params": list(emb.parameters()), "eps": 1e-15}], lr=c["lrate"], betas=(0.9, 0.99))
        ev, nv, tr = [psnr_of(eo, ed, ergb)], [psnr_of(no, nd, nrgb)], []
        for it in range(1, c["iters"] + 1):
            idx = batches[it - 1]
            _, psnr = nerf.train_step((ro[idx], rd[idx]), rgb[idx], kw, opt, args, it)
            tr.append(psnr)
            if it % every == 0:
                ev.append(psnr_of(eo, ed, ergb))
                nv.append(psnr_of(no, nd, nrgb))
        return {"eval_psnr": np.array(ev), "novel_psnr": np.array(nv),
                "train_psnr": torch.stack(tr).float().cpu().numpy().reshape(-1)}

    names = ("eval_psnr", "novel_psnr", "train_psnr")
    runs = {int(s): {k: cs[f"{k}_s{int(s)}"] for k in names + ("batch_sum",)} for s in cs["seeds"]}
    ref_seeds = sorted(runs)      # F19c: the reference's own runs
    try:
        cd = golden("f19d_converge")
        runs.update({int(s): {k: cd[f"{k}_s{int(s)}"] for k in names + ("batch_sum",)} for s in cd["seeds"]})
    except FileNotFoundError:
        pass
    seeds = sorted(runs)
    hip = {}
    for s in seeds:   # each run's batches (make_golden.gen_converge_seeds / make_oracle_converge.oracle_run)
        rng = np.random.RandomState(s)
        bt = np.stack([rng.choice(n_pool, c["R"], replace=False) for _ in range(c["iters"])])
        assert int(bt.astype(np.int64).sum()) == int(runs[s]["batch_sum"]), f"seed {s}: batches differ"
        bt = torch.from_numpy(bt.astype(np.int64)).to(gpu)
        hip[s] = [train_run(bt) for _ in range(K)]
        if len(hip) % 16 == 0:
            print(f"  {len(hip)}/{len(seeds)} seeds trained", flush=True)

    from scipy import stats
    lines, fails = [], []
    win = lambda x: x.reshape(*x.shape[:-1], -1, every).mean(-1)  # noqa: E731
    n_checks = 2 * len(g["eval_iters"]) + c["iters"] // every
    for name in names:
        ref = np.stack([runs[s][name] for s in seeds])                            # [S, T]
        hmean = np.stack([np.stack([r[name] for r in hip[s]]).mean(0) for s in seeds])
        d = _late(name, hmean, every) - _late(name, ref, every)
        D, se = float(d.mean()), float(d.std(ddof=1) / np.sqrt(len(d)))
        is_ref = np.array([s in ref_seeds for s in seeds])
        Dr, ser = float(d[is_ref].mean()), float(d[is_ref].std(ddof=1) / np.sqrt(int(is_ref.sum())))
        lines.append(f"{name}: late-phase (iterations {LATE}-300) F19c (the reference, {int(is_ref.sum())} seeds): "
                     f"D {Dr:+.3f} dB (se {ser:.3f}); all {len(seeds)} seeds (F19c + the oracle's F19d) reference "
                     f"{_late(name, ref, every).mean():.3f} dB, HIP {_late(name, hmean, every).mean():.3f} dB: D {D:+.3f} "
                     f"dB (se {se:.3f}, {K} HIP runs per seed; per seed {np.round(d, 3).tolist()})")
        if abs(Dr) > 0.1:
            fails.append(f"{name}: |D| over the reference's own seeds = {abs(Dr):.3f} dB > 0.1 dB")
        if abs(D) > 0.1:
            fails.append(f"{name}: |D| over all seeds = {abs(D):.3f} dB > 0.1 dB")
        # per checkpoint: paired t over seeds, Bonferroni (family-wise 1 %)
        dk = hmean - ref
        if name == "train_psnr":
            dk = win(dk)
        m, sk = dk.mean(0), dk.std(0, ddof=1) / np.sqrt(len(seeds))
        crit = stats.t.ppf(1.0 - 0.01 / (2 * n_checks), len(seeds) - 1)
        out = np.abs(m) > crit * sk + 0.02
        if out.any():
            fails.append(f"{name}: {int(out.sum())} checkpoints where HIP and the reference differ "
                         f"(first at index {int(np.argmax(out))})")
    # F19's batches (reported): six HIP runs vs F19 (6) + F19b (12)
    b = golden("f19b_converge")
    f19 = [run for run in (train_run(torch.from_numpy(g["batches"].astype(np.int64)).to(gpu)) for _ in range(6))]
    for name in names:
        refs = [g[name + t] for t in ("", "_b", "_c", "_d", "_e", "_f")] + [b[f"{name}_n{int(k)}"] for k in b["seeds"]]
        lr_ = np.array([_late(name, r, every) for r in refs])
        lh = np.array([_late(name, r[name], every) for r in f19])
        lines.append(f"  F19 batches (reported): {name} reference {lr_.mean():.3f} (sd {lr_.std(ddof=1):.3f}, "
                     f"{len(lr_)} runs), HIP {lh.mean():.3f} (sd {lh.std(ddof=1):.3f}, {len(lh)} runs)")
    report = "\n".join(lines)
    print("\nPSNR (dB), reference vs HIP:\n" + report)
    assert np.mean([runs[s]["eval_psnr"][-1] - runs[s]["eval_psnr"][0] for s in seeds]) > 3.0, \
        "fixture: the reference runs should learn the scene"
    assert not fails, f"{fails}\n{report}"
