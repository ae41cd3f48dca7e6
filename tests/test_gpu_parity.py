"""HIP kernels vs the reference's golden vectors and the CPU oracle (needs an MI355X).

Tolerances: indices, keep masks, hash-grid features and SH are bit-exact (same fp32 op order, no
contraction); MLP outputs use fp32 MFMA (k-ordered fma chain vs the CPU's blocked GEMM) and
compositing/sampling sums run in a different order, so they are compared at fp32 rounding level
(rtol 1e-4..1e-5); gradients accumulated with fp32 atomics at rtol 1e-4.
"""
import numpy as np
import pytest
import torch

from tables import blender_bbox, closed_form_table, synthetic_rays

pytestmark = pytest.mark.gpu

MLP_KEYS = ("sigma_net.0.weight", "sigma_net.1.weight", "color_net.0.weight", "color_net.1.weight",
            "color_net.2.weight")


def _bbox_t():
    lo, hi = blender_bbox()
    return torch.from_numpy(lo), torch.from_numpy(hi)


def _embedder(nerf, gpu, finest, table):
    emb = nerf.HashEmbedder(_bbox_t(), finest_resolution=finest).to(gpu)
    with torch.no_grad():
        for i, e in enumerate(emb.embeddings):
            e.weight.copy_(torch.from_numpy(table[i]))
    return emb


def _mlp(nerf, gpu, d, prefix):
    net = nerf.NeRFSmall(num_layers=2, hidden_dim=64, geo_feat_dim=15, num_layers_color=3, hidden_dim_color=64,
                         input_ch=32, input_ch_views=16).to(gpu)
    with torch.no_grad():
        for k, p in net.named_parameters():
            p.copy_(torch.from_numpy(d[prefix + k.replace(".", "_")]))
    return net


def test_hash_encode_fwd_bit_exact(nerf, gpu, golden):
    g = golden("f3_hash_fwd")
    table = closed_form_table()
    for finest in (512, 1024):
        emb = _embedder(nerf, gpu, finest, table)
        x = torch.from_numpy(g[f"xyz_{finest}"]).to(gpu)
        with torch.no_grad():
            feat, keep = emb(x)
            feat_l, keep_l = emb.encode(x, "level")
        np.testing.assert_array_equal(feat.cpu().numpy(), g[f"feat_{finest}"])
        np.testing.assert_array_equal(keep.cpu().numpy(), g[f"keep_{finest}"])
        np.testing.assert_array_equal(feat_l.permute(1, 0, 2).reshape(x.shape[0], 32).cpu().numpy(),
                                      g[f"feat_{finest}"])


def test_hash_encode_bwd(nerf, gpu, golden):
    g = golden("f4_hash_bwd")
    emb = _embedder(nerf, gpu, 1024, closed_form_table())
    feat, _ = emb(torch.from_numpy(g["xyz"]).to(gpu))
    (feat * torch.from_numpy(g["dfeat"]).to(gpu)).sum().backward()
    dense = np.zeros((16, 1 << 19, 2), np.float32)
    dense[g["level"], g["row"]] = g["grad"]
    got = np.stack([e.weight.grad.cpu().numpy() for e in emb.embeddings])
    np.testing.assert_allclose(got, dense, rtol=1e-5, atol=1e-7)


def test_hash_encode_large_vs_c_oracle(nerf, gpu):
    """786,432 points (the fine pass at the metric config): bit-exact against the C oracle on a
    strided subset, and keep-mask exact everywhere."""
    from test_abi import _c_hash
    table = closed_form_table()
    emb = _embedder(nerf, gpu, 1024, table)
    lo, hi = blender_bbox()
    rng = np.random.RandomState(5)
    x = (lo - 0.2 + (hi - lo + 0.4) * rng.rand(786432, 3)).astype(np.float32)
    with torch.no_grad():
        feat, keep = emb(torch.from_numpy(x).to(gpu))
    sub = slice(0, None, 97)
    ref, ref_keep, *_ = _c_hash(x[sub], emb.level_res, table)
    np.testing.assert_array_equal(feat.cpu().numpy()[sub], ref)
    np.testing.assert_array_equal(keep.cpu().numpy()[sub], ref_keep)
    inside = np.all((x >= lo) & (x <= hi), axis=1)
    np.testing.assert_array_equal(keep.cpu().numpy(), inside)


def test_hash_encode_edge_points_vs_c_oracle(nerf, gpu):
    """Every point bit-exact against the C oracle (IEEE division) where the voxel math is most
    fragile: points exactly on grid vertices of every level, on and outside the box bounds, zero,
    subnormal, tiny and huge coordinates, spread over waves and in runs. The kernels' fast division
    (div_rn<true>, csrc/hash_common.h) serves the waves whose coordinates pass fastdiv_point_ok and
    the IEEE division the others; both must reproduce utils.py:103-112 bit for bit."""
    from test_abi import _c_hash
    table = closed_form_table()
    emb = _embedder(nerf, gpu, 1024, table)
    lo, hi = blender_bbox()
    rng = np.random.RandomState(11)
    n = 1 << 20
    x = (lo - 0.3 + (hi - lo + 0.6) * rng.rand(n, 3)).astype(np.float32)
    res = np.asarray(emb.level_res, np.float32)
    cell = ((hi.astype(np.float32) - lo.astype(np.float32))[None, :] / res[:, None]).astype(np.float32)   # [L, 3]
    # grid vertices: base * cell + lo in fp32 (the kernels' vmin), every level, random axes
    m = n // 4
    lv = rng.randint(0, len(res), m)
    k = np.floor(rng.rand(m, 3) * res[lv][:, None]).astype(np.float32)
    verts = (k * cell[lv] + lo.astype(np.float32)).astype(np.float32)
    axes = rng.rand(m, 3) < 0.6
    x[:m][axes] = verts[axes]
    specials = np.array([0.0, -0.0, 1e-30, -1e-30, 1e-40, 1e-45, 3e-22, 1e30, -1e30, 1e-6, -1e-6],
                        np.float32)
    sel = rng.rand(n, 3) < 0.002                                   # scattered: one wave in ~10
    x[sel] = rng.choice(specials, int(sel.sum()))
    for a in range(3):                                             # exact box bounds
        b = rng.rand(n) < 0.01
        x[b, a] = np.where(rng.rand(int(b.sum())) < 0.5, lo[a], hi[a]).astype(np.float32)
    x[n - 4096:n - 2048, 1] = 0.0                                   # a run of zero coordinates
    x[n - 2048:, 2] = 1e-38
    perm = rng.permutation(n - 4096)
    x[:n - 4096] = x[perm]
    with torch.no_grad():
        feat, keep = emb(torch.from_numpy(x).to(gpu))
    ref, ref_keep, *_ = _c_hash(x, emb.level_res, table)
    np.testing.assert_array_equal(feat.cpu().numpy(), ref)
    np.testing.assert_array_equal(keep.cpu().numpy(), ref_keep)


@pytest.mark.parametrize("log2_T", [12, 15])
def test_hash_encode_small_tables_vs_oracle(nerf, gpu, oracle, log2_T):
    """Tables smaller than the default 2^19: the forward groups the coarse levels whose (res+1)^3
    vertices fit the table (2^15: three levels, an odd count for the two-level rounds; 2^12: none, every
    level in its own grid row) and the binned backward runs one partial owner slice per level.
    Features bit-exact and gradients at fp64-scatter accuracy vs the oracle (utils.py:95-117,
    hash_encoding.py:56-107)."""
    lo, hi = blender_bbox()
    emb = nerf.HashEmbedder(_bbox_t(), finest_resolution=1024, log2_hashmap_size=log2_T).to(gpu)
    g = torch.Generator().manual_seed(log2_T)
    tabs = [torch.randn(1 << log2_T, 2, generator=g) * 0.1 for _ in range(16)]
    with torch.no_grad():
        for e, t in zip(emb.embeddings, tabs):
            e.weight.copy_(t)
    rng = np.random.RandomState(log2_T)
    x = (lo - 0.1 + (hi - lo + 0.2) * rng.rand(65536, 3)).astype(np.float32)
    xt = torch.from_numpy(x)
    res = [torch.tensor(r, dtype=torch.float32) for r in emb.level_res]
    bmin, bmax = (torch.from_numpy(v) for v in (lo, hi))
    ref, ref_keep = oracle.hash_encode(xt, tabs, bmin, bmax, res, log2_T=log2_T)
    feat, keep = emb(xt.to(gpu))
    np.testing.assert_array_equal(feat.detach().cpu().numpy(), ref.numpy())
    np.testing.assert_array_equal(keep.cpu().numpy(), ref_keep.numpy())
    dfeat = torch.from_numpy(rng.randn(65536, 32).astype(np.float32))
    (feat * dfeat.to(gpu)).sum().backward()
    for lvl in (0, 3, 9, 15):
        vmin, vmax, idx, _ = oracle.voxel_corners(xt, bmin, bmax, res[lvl], log2_T)
        w = ((xt - vmin) / (vmax - vmin)).double()
        wx, wy, wz = w[:, 0:1], w[:, 1:2], w[:, 2:3]
        gl = dfeat[:, 2 * lvl:2 * lvl + 2].double()
        contrib = []
        for c in range(8):
            i, j, k = (c >> 2) & 1, (c >> 1) & 1, c & 1
            contrib.append(gl * ((wz if k else 1 - wz) * (wy if j else 1 - wy) * (wx if i else 1 - wx)))
        contrib = torch.stack(contrib, 1).reshape(-1, 2)
        want = torch.zeros(1 << log2_T, 2, dtype=torch.float64).index_add_(0, idx.reshape(-1), contrib)
        scale = torch.zeros(1 << log2_T, 2, dtype=torch.float64).index_add_(0, idx.reshape(-1), contrib.abs())
        got = emb.embeddings[lvl].weight.grad.cpu().double()
        bad = (got - want).abs() > 2e-6 * scale + 1e-30
        assert not bool(bad.any()), f"level {lvl}: {int(bad.sum())} rows off"


def test_sh4_bit_exact(nerf, gpu, golden):
    g = golden("f5_sh")
    with torch.no_grad():
        sh = nerf.SHEncoder()(torch.from_numpy(g["dirs"]).to(gpu))
    np.testing.assert_array_equal(sh.cpu().numpy(), g["sh"])


def test_mlp_fwd_bwd(nerf, gpu, golden):
    g = golden("f6_mlp")
    net = _mlp(nerf, gpu, g, "w_")
    x = torch.from_numpy(g["x"]).to(gpu).requires_grad_(True)
    raw = net(x)
    np.testing.assert_allclose(raw.detach().cpu().numpy(), g["raw"], rtol=1e-4, atol=2e-6)
    (raw * torch.from_numpy(g["g_raw"]).to(gpu)).sum().backward()
    np.testing.assert_allclose(x.grad.cpu().numpy(), g["dx"], rtol=1e-4, atol=2e-6)
    for k, p in net.named_parameters():
        np.testing.assert_allclose(p.grad.cpu().numpy(), g["dw_" + k.replace(".", "_")], rtol=1e-4, atol=1e-4)


def test_mlp_large_vs_torch_fp32(nerf, gpu):
    """262,144 points (the coarse pass): forward against a plain PyTorch fp32 MLP; weight grads (sums
    over 262,144 points) against an fp64 reference, bounded by fp32 summation error relative to the
    sum of |terms| (the plain fp32 torch GEMM is held to the same bound)."""
    torch.manual_seed(0)
    net = nerf.NeRFSmall(2, 64, 15, 3, 64, 32, 16).to(gpu)
    x = (torch.randn(262144, 48, device=gpu) * 0.5)
    graw = torch.randn(262144, 4, device=gpu)
    raw = net(x)
    torch.backends.cuda.matmul.allow_tf32 = False

    def ref_mlp(W, xx):
        h = torch.relu(xx[:, :32] @ W["sigma_net.0.weight"].t())
        o = h @ W["sigma_net.1.weight"].t()
        c = torch.relu(torch.cat([xx[:, 32:], o[:, 1:]], -1) @ W["color_net.0.weight"].t())
        c = torch.relu(c @ W["color_net.1.weight"].t())
        return torch.cat([c @ W["color_net.2.weight"].t(), o[:, :1]], -1), (h, o, c)

    W32 = {k: p.detach().clone().requires_grad_(True) for k, p in net.named_parameters()}
    W64 = {k: p.detach().double().clone().requires_grad_(True) for k, p in net.named_parameters()}
    ref32, _ = ref_mlp(W32, x)
    ref64, _ = ref_mlp(W64, x.double())
    torch.testing.assert_close(raw.detach(), ref32.detach(), rtol=1e-4, atol=1e-5)
    (raw * graw).sum().backward()
    (ref32 * graw).sum().backward()
    (ref64 * graw.double()).sum().backward()
    # |terms| bound: the same backward on |W|, |x|, |graw| (an upper bound of sum |g_i x_j| per entry)
    Wabs = {k: p.detach().double().abs().requires_grad_(True) for k, p in net.named_parameters()}
    refabs, _ = ref_mlp(Wabs, x.double().abs())
    (refabs * graw.double().abs()).sum().backward()
    for k, p in net.named_parameters():
        bound = 2e-5 * Wabs[k].grad + 1e-6
        err = (p.grad.double() - W64[k].grad).abs()
        err_torch = (W32[k].grad.double() - W64[k].grad).abs()
        assert (err <= bound).all(), f"{k}: max err/bound {(err / bound).max().item():.3f}"
        assert (err_torch <= bound).all(), f"{k}: the fp32 torch reference exceeds the bound"


def test_composite_fwd_bwd(nerf, gpu, golden):
    g = golden("f7_composite")
    names = ["rgb", "disp", "acc", "weights", "depth", "entropy"]
    for S in (64, 192):
        for white in (0, 1):
            tag = f"S{S}_w{white}"
            T = lambda k: torch.from_numpy(g[f"{k}_{tag}"]).to(gpu)  # noqa: E731
            with torch.no_grad():
                out = nerf.raw2outputs(T("raw"), T("z"), T("d"), 0, bool(white))
            for n, v in zip(names, out):
                np.testing.assert_allclose(v.cpu().numpy(), g[f"{n}_{tag}"], rtol=1e-5, atol=2e-6, equal_nan=True,
                                           err_msg=f"{n} {tag}")
            raw = T("braw").requires_grad_(True)
            out = nerf.raw2outputs(raw, T("bz"), T("bd"), 0, bool(white))
            loss = sum((o * T(f"g_{n}")).sum() for o, n in zip(out, ["rgb", "disp", "acc", "w", "depth", "ent"]))
            loss.backward()
            np.testing.assert_allclose(raw.grad.cpu().numpy(), g[f"draw_{tag}"], rtol=1e-4, atol=1e-5,
                                       err_msg=f"grad {tag}")
    with torch.no_grad():
        out = nerf.raw2outputs(torch.from_numpy(g["raw_noise"]).to(gpu), torch.from_numpy(g["z_noise"]).to(gpu),
                               torch.from_numpy(g["d_noise"]).to(gpu), 1.0, False, pytest=True)
    for n, v in zip(names, out):
        np.testing.assert_allclose(v.cpu().numpy(), g[f"{n}_noise"], rtol=1e-5, atol=2e-6)


def test_composite_large_vs_oracle(nerf, gpu, oracle):
    """4096 rays x 192 samples (metric config): forward and raw-gradient against the CPU oracle."""
    rng = np.random.RandomState(9)
    R, S = 4096, 192
    raw = (rng.randn(R, S, 4) * 2).astype(np.float32)
    z = np.sort(2 + 4 * rng.rand(R, S), -1).astype(np.float32)
    d = rng.randn(R, 3).astype(np.float32)
    gr = rng.randn(R, 3).astype(np.float32)
    rt = torch.from_numpy(raw).to(gpu).requires_grad_(True)
    out = nerf.raw2outputs(rt, torch.from_numpy(z).to(gpu), torch.from_numpy(d).to(gpu), 0, True)
    (out[0] * torch.from_numpy(gr).to(gpu)).sum().backward()
    rc = torch.from_numpy(raw).requires_grad_(True)
    ref = oracle.composite(rc, torch.from_numpy(z), torch.from_numpy(d), None, True)
    (ref[0] * torch.from_numpy(gr)).sum().backward()
    for a, b in zip(out, ref):
        np.testing.assert_allclose(a.detach().cpu().numpy(), b.detach().numpy(), rtol=1e-4, atol=1e-5, equal_nan=True)
    np.testing.assert_allclose(rt.grad.cpu().numpy(), rc.grad.numpy(), rtol=1e-3, atol=1e-5)


def _check_pdf_samples(got, want, weights, tol=1e-5):
    """sample_pdf is continuous in the CDF except through the reference's own `denom < 1e-5 -> 1`
    rule (run_nerf_helpers.py:393): inside a bin whose probability mass is < 1e-5 the sample jumps
    with a 1-ulp change of the float32 CDF (the CPU reference sums with AVX lanes, the GPU with a
    wave tree, and torch-CUDA differently again). Outside those bins the samples must agree to
    `tol`; mismatches are allowed only in rows that have such bins, and must stay rare."""
    bad = ~np.isclose(got, want, rtol=tol, atol=tol)
    pdf = (weights + 1e-5) / (weights + 1e-5).sum(-1, keepdims=True)
    has_thin = (pdf < 1e-5).any(-1)
    assert not (bad.any(-1) & ~has_thin).any(), "sample mismatch in a row without thin bins"
    assert bad.mean() <= 2e-3, f"{bad.sum()} mismatching samples"


def test_sample_pdf(nerf, gpu, golden):
    g = golden("f8_pdf")
    bins, w = torch.from_numpy(g["bins"]).to(gpu), torch.from_numpy(g["weights"]).to(gpu)
    _check_pdf_samples(nerf.sample_pdf(bins, w, 128, det=True).cpu().numpy(), g["det"], g["weights"])
    _check_pdf_samples(nerf.sample_pdf(bins, w, 128, det=False, pytest=True).cpu().numpy(), g["rand_pytest"],
                       g["weights"])


def _render_kwargs(nerf, gpu, g, tag, emb, n_samples, n_importance, perturb, noise, lindisp):
    coarse, fine = _mlp(nerf, gpu, g, f"coarse_{tag}_"), _mlp(nerf, gpu, g, f"fine_{tag}_")
    sh = nerf.SHEncoder()
    nqf = lambda inputs, viewdirs, fn: nerf.run_network(inputs, viewdirs, fn, emb, sh)  # noqa: E731
    return dict(network_query_fn=nqf, perturb=perturb, N_importance=n_importance, network_fine=fine,
                N_samples=n_samples, network_fn=coarse, embed_fn=emb, use_viewdirs=True, white_bkgd=True,
                raw_noise_std=noise, predict_normals=False, ndc=False, lindisp=lindisp, near=2.0, far=6.0)


def test_render_end_to_end(nerf, gpu, golden):
    g = golden("f9_render")
    table = closed_form_table()
    variants = {"A": (64, 128, 1.0, 0.0, False), "B": (64, 64, 0.0, 1.0, True)}
    for tag, v in variants.items():
        emb = _embedder(nerf, gpu, 1024, table)
        kw = _render_kwargs(nerf, gpu, g, tag, emb, *v)
        ro, rd = (torch.from_numpy(g[f"rays_{k}_{tag}"]).to(gpu) for k in ("o", "d"))
        with torch.no_grad():
            rgb, depth, acc, ex = nerf.render(800, 800, None, rays=(ro, rd), retraw=True, pytest=True, **kw)
        # coarse pass: same samples as the reference -> fp32 rounding level
        for k in ["rgb0", "depth0", "acc0", "sparsity_loss0"]:
            np.testing.assert_allclose(ex[k].cpu().numpy(), g[f"{k}_{tag}"], rtol=1e-4, atol=1e-4, err_msg=k + tag)
        # fine pass: importance samples inherit sample_pdf's thin-bin discontinuity (see
        # _check_pdf_samples), which moves samples only in near-empty space. PSNR-equivalent bound:
        # |d rgb| <= 1e-3 (a 30 dB image has RMS error 3e-2), depth/z_std to 0.1 %.
        np.testing.assert_allclose(rgb.cpu().numpy(), g[f"rgb_{tag}"], rtol=0, atol=1e-3, err_msg="rgb" + tag)
        np.testing.assert_allclose(acc.cpu().numpy(), g[f"acc_{tag}"], rtol=0, atol=1e-3, err_msg="acc" + tag)
        np.testing.assert_allclose(depth.cpu().numpy(), g[f"depth_{tag}"], rtol=1e-3, atol=1e-3, err_msg="depth" + tag)
        np.testing.assert_allclose(ex["z_std"].cpu().numpy(), g[f"z_std_{tag}"], rtol=1e-3, atol=1e-3)
        mse = float(((rgb.cpu().numpy() - g[f"rgb_{tag}"]) ** 2).mean())
        assert mse < 1e-7, f"rgb MSE vs reference {mse}"


def test_train_step_and_radam(nerf, gpu, golden):
    """Seven reference training iterations (render + losses + backward + RAdam + lr decay).

    F10 is a well-conditioned, trained-like state (tests/golden/make_golden.py: tables U(-0.3, 0.3),
    the sigma output rows scaled by 60, so sigma ~ O(1-10) and alpha = 1 - exp(-sigma delta) is not
    cancellation-dominated). Measured on the MI355X (r02an): losses equal to the printed precision,
    MLP gradients within 2e-5 (fine net) / 9e-7 (coarse) relative in norm, table-gradient checksums
    within 1e-6, parameters after the 7 steps (2 RAdam updates) within 4e-8 absolute. The bars are
    ~10x those: losses 1e-5, MLP grads 2e-4, checksums 1e-5, parameters 2e-5 rel + 1e-7 abs."""
    g = golden("f10_train")
    emb = _embedder(nerf, gpu, 1024, closed_form_table(scale=float(g["table_scale"]), salt=3))
    kw = _render_kwargs(nerf, gpu, {**{k.replace("coarse0_", "coarse_T_"): v for k, v in g.items()},
                                    **{k.replace("fine0_", "fine_T_"): v for k, v in g.items()}},
                        "T", emb, 64, 128, 1.0, 0.0, False)
    coarse, fine = kw["network_fn"], kw["network_fine"]
    opt = nerf.RAdam([{"params": list(coarse.parameters()) + list(fine.parameters()), "weight_decay": 1e-6},
                      {"params": list(emb.parameters()), "eps": 1e-15}], lr=5e-4, betas=(0.9, 0.99))
    ro, rd, target = (torch.from_numpy(g[k]).to(gpu) for k in ("rays_o", "rays_d", "target"))
    losses = []
    for step in range(7):
        rgb, _, _, ex = nerf.render(800, 800, None, rays=(ro, rd), retraw=True, pytest=True, **kw)
        opt.zero_grad()
        l_img = nerf.img2mse(rgb, target)
        l_img0 = nerf.img2mse(ex["rgb0"], target)
        l_sp = 1e-10 * (ex["sparsity_loss"].sum() + ex["sparsity_loss0"].sum())
        loss = l_img + l_img0 + l_sp
        loss.backward()
        if step == 0:
            np.testing.assert_allclose([l_img.item(), l_img0.item(), loss.item()], g["loss0"][[0, 1, 3]], rtol=1e-5)
            np.testing.assert_allclose(l_sp.item(), g["loss0"][2], rtol=1e-4)
            for prefix, net in (("gcoarse_", coarse), ("gfine_", fine)):
                for k, p in net.named_parameters():
                    want = g[prefix + k.replace(".", "_")]
                    rel = np.linalg.norm(p.grad.cpu().numpy() - want) / np.linalg.norm(want)
                    assert rel < 2e-4, f"{prefix}{k}: relative grad error {rel:.2e}"
            for i, e in enumerate(emb.embeddings):
                gd = e.weight.grad.double()
                cs = g["gtable_checksum"][i]
                np.testing.assert_allclose([(gd * gd).sum().item(), gd.abs().sum().item()], cs[1:], rtol=1e-5,
                                           err_msg=f"level {i}")
                assert abs(gd.sum().item() - cs[0]) <= 1e-5 * cs[2], f"level {i} gradient sum"
        opt.step()
        for grp in opt.param_groups:
            grp["lr"] = 5e-4 * (0.1 ** (step / (500 * 1000)))
        losses.append(loss.item())
    np.testing.assert_allclose(losses, g["losses"], rtol=1e-5)
    for k, p in coarse.named_parameters():
        np.testing.assert_allclose(p.detach().cpu().numpy(), g["coarse7_" + k.replace(".", "_")], rtol=2e-5, atol=1e-7)
    for i, e in enumerate(emb.embeddings):
        np.testing.assert_allclose(e.weight.detach().cpu().numpy()[g["table_rows"]], g["table_samples"][i],
                                   rtol=2e-5, atol=1e-7)


def test_radam_vs_oracle(nerf, gpu, oracle):
    torch.manual_seed(3)
    ps = [torch.randn(1000, device=gpu), torch.randn(33, 7, device=gpu)]
    cps = [p.detach().cpu().clone() for p in ps]
    ps = [torch.nn.Parameter(p) for p in ps]
    cps = [torch.nn.Parameter(p) for p in cps]
    opt = nerf.RAdam([{"params": ps[:1], "weight_decay": 1e-6}, {"params": ps[1:], "eps": 1e-15}], lr=5e-4,
                     betas=(0.9, 0.99))
    ref = oracle.RAdamOracle([dict(params=cps[:1], lr=5e-4, betas=(0.9, 0.99), eps=1e-8, weight_decay=1e-6),
                              dict(params=cps[1:], lr=5e-4, betas=(0.9, 0.99), eps=1e-15, weight_decay=0)])
    for it in range(9):
        grads = [torch.randn_like(c) for c in cps]
        for p, c, gr in zip(ps, cps, grads):
            p.grad = gr.to(gpu)
            c.grad = gr.clone()
        opt.step()
        ref.step()
        for p, c in zip(ps, cps):
            np.testing.assert_allclose(p.detach().cpu().numpy(), c.detach().numpy(), rtol=1e-6, atol=1e-7)


def test_tv_loss(nerf, gpu, golden):
    g = golden("f12_tv")
    emb = _embedder(nerf, gpu, 1024, closed_form_table(scale=0.05, salt=5))
    losses = nerf.total_variation_all(emb, min_vertex=torch.from_numpy(g["min_vertex"]))
    np.testing.assert_allclose(losses.detach().cpu().numpy(), g["level_loss"], rtol=1e-5)
    losses.sum().backward()
    for i, e in enumerate(emb.embeddings):
        gd = e.weight.grad.double().cpu().numpy()
        # the plain sum of a TV gradient is 0 up to cancellation: compare it against the abs-sum scale
        cs = g["grad_checksum"][i]
        np.testing.assert_allclose([(gd * gd).sum(), np.abs(gd).sum()], cs[1:], rtol=1e-4)
        assert abs(gd.sum() - cs[0]) <= 1e-6 * cs[2]
    for i in range(3):
        sel = g["level"] == i
        np.testing.assert_allclose(emb.embeddings[i].weight.grad.cpu().numpy()[g["row"][sel]], g["grad"][sel],
                                   rtol=1e-5, atol=1e-9)


def test_tv_binned_matches_atomic(nerf, gpu, golden):
    """The TV backward binned into the hash workspace and summed by the owner pass (nerf_tv_bwd_bin,
    the autograd path) against the float-atomic kernel (nerf_tv_bwd) on the F12 cuboids of all 16
    levels; the deterministic mode gives bitwise-identical gradients on a repeat."""
    from indoor_nerf_amd import _lib
    g = golden("f12_tv")
    emb = _embedder(nerf, gpu, 1024, closed_form_table(scale=0.05, salt=5))
    mv = torch.from_numpy(g["min_vertex"])

    def binned(det):
        for e in emb.embeddings:
            e.weight.grad = None
        nerf.set_deterministic(det)
        try:
            nerf.total_variation_all(emb, min_vertex=mv).sum().backward()
        finally:
            nerf.set_deterministic(False)
        return [e.weight.grad.clone() for e in emb.embeddings]

    got = binned(False)
    tables = [e.weight for e in emb.embeddings]
    L = len(tables)
    from indoor_nerf_amd.losses import tv_cube
    cubes = [tv_cube(l, emb.base_resolution, emb.finest_resolution, L)[1] for l in range(L)]
    ref = [torch.zeros_like(t) for t in tables]
    scale = torch.ones(L, device=gpu)
    _lib.call("nerf_tv_bwd", _lib.ptr_array(tables), L, emb.log2_hashmap_size,
              (_lib.c_i64 * (3 * L))(*[int(v) for v in mv.reshape(-1).tolist()]), None, (_lib.c_int * L)(*cubes),
              _lib.ptr(scale), _lib.ptr_array(ref), _lib.stream())
    torch.cuda.synchronize()
    for a, b in zip(got, ref):
        assert a.abs().sum().item() > 0
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-9)
    d1, d2 = binned(True), binned(True)
    for a, b, r in zip(d1, d2, ref):
        assert torch.equal(a, b)
        torch.testing.assert_close(a, r, rtol=1e-5, atol=1e-9)
    # without the forward's vertex rows (d_verts NULL): the kernel gathers the hashed rows itself
    from indoor_nerf_amd import hashgrid
    from indoor_nerf_amd.losses import TVBinJob
    grads = [torch.zeros_like(t) for t in tables]
    cb = (_lib.c_int * L)(*cubes)
    mvh = (_lib.c_i64 * (3 * L))(*[int(v) for v in mv.reshape(-1).tolist()])
    n_ch = int(_lib.load().nerf_tv_bwd_bin_chunks(L, cb))
    pb = hashgrid.pending_bins(gpu)
    pb.reserve(n_ch)
    pb.add_tv(TVBinJob(tables, grads, scale, mvh, None, cb, emb.log2_hashmap_size, n_ch), queue=False)
    pb.flush()
    torch.cuda.synchronize()
    for a, r in zip(grads, got):
        torch.testing.assert_close(a, r, rtol=1e-6, atol=1e-12)


def test_train_step_full_size_finite(nerf, gpu):
    """The metric configuration: 4096 rays x (64 + 128) samples, finest 1024, one full iteration."""
    lo, hi = blender_bbox()
    args = nerf.make_args(bounding_box=(torch.from_numpy(lo), torch.from_numpy(hi)), finest_res=1024, N_samples=64,
                          N_importance=128, white_bkgd=True)
    kw, _, _, grad_vars, opt = nerf.create_nerf(args, device=gpu)
    kw.update(near=2.0, far=6.0)
    ro, rd = synthetic_rays(4096, seed=4)
    rays = (torch.from_numpy(ro).to(gpu), torch.from_numpy(rd).to(gpu))
    target = torch.rand(4096, 3, device=gpu)
    for it in range(1, 8):
        loss, psnr = nerf.train_step(rays, target, kw, opt, args, it)
    assert torch.isfinite(loss).item()
    for p in grad_vars:
        assert torch.isfinite(p).all().item()


@pytest.mark.gpu
def test_train_loss_head_vs_torch_fp32(nerf, gpu):
    """Fused loss head (csrc/loss.hip) against the reference's own torch expressions
    (run_nerf.py:1011-1037) in fp32; gradients bit-exact (same op order as autograd)."""
    g = torch.Generator().manual_seed(3)
    R = 4096
    rgb, rgb0, t = (torch.rand(R, 3, generator=g) for _ in range(3))
    sp, sp0 = torch.rand(R, generator=g) * 5, torch.rand(R, generator=g) * 5
    tv = torch.rand(16, generator=g)
    sw, tw = 1e-4, 1e-3
    leaves = [x.clone().to(gpu).requires_grad_(True) for x in (rgb, rgb0, sp, sp0, tv)]
    loss, img, psnr = nerf.train_loss(leaves[0], leaves[1], t.to(gpu), leaves[2], leaves[3], leaves[4], sw, tw)
    loss.backward()
    ref_leaves = [x.clone().double().requires_grad_(True) for x in (rgb, rgb0, sp, sp0, tv)]
    r_rgb, r_rgb0, r_sp, r_sp0, r_tv = ref_leaves
    td = t.double()
    r_img = torch.mean((r_rgb - td) ** 2)
    r_loss = r_img + torch.mean((r_rgb0 - td) ** 2) + sw * (r_sp.sum() + r_sp0.sum()) + tw * sum(r_tv[i] for i in range(16))
    r_loss.backward()
    assert abs(float(loss) - float(r_loss)) <= 2e-6 * abs(float(r_loss))
    assert abs(float(img) - float(r_img)) <= 2e-6 * float(r_img)
    assert abs(float(psnr) - float(-10 * torch.log10(r_img))) <= 1e-4
    # fp32 autograd of the same expressions: bit-exact gradients
    f_leaves = [x.clone().requires_grad_(True) for x in (rgb, rgb0, sp, sp0, tv)]
    f_rgb, f_rgb0, f_sp, f_sp0, f_tv = f_leaves
    f_loss = torch.mean((f_rgb - t) ** 2) + torch.mean((f_rgb0 - t) ** 2) + sw * (f_sp.sum() + f_sp0.sum()) \
        + tw * sum(f_tv[i] for i in range(16))
    f_loss.backward()
    for mine, ref in zip(leaves, f_leaves):
        assert torch.equal(mine.grad.cpu(), ref.grad), float((mine.grad.cpu() - ref.grad).abs().max())


@pytest.mark.gpu
def test_hash_encode_bwd_deferred_two_passes(nerf, gpu):
    """Two HashEmbedder forwards in one autograd pass (the coarse and the fine pass of a step) bin
    into one workspace and share ONE owner launch at the end of the pass (hashgrid._PendingBins):
    the gradient equals two direct binned backwards (same entries, one fp32 rounding fewer), also
    when a later, larger pass outgrows the workspace (early flush, then a regrown capacity)."""
    emb = _embedder(nerf, gpu, 1024, closed_form_table())
    lo, hi = blender_bbox()
    rng = np.random.RandomState(7)
    for sizes in ((70_001, 20_000), (200_000, 70_001, 513), (200_000, 70_001, 513)):
        xs = [torch.from_numpy((lo + (hi - lo) * rng.rand(n, 3)).astype(np.float32)).to(gpu) for n in sizes]
        ds = [torch.from_numpy(rng.randn(n, 32).astype(np.float32)).to(gpu) for n in sizes]
        for e in emb.embeddings:
            e.weight.grad = None
        sum((emb(x)[0] * d).sum() for x, d in zip(xs, ds)).backward()
        got = torch.stack([e.weight.grad for e in emb.embeddings])
        ref = [torch.zeros(1 << 19, 2, device=gpu) for _ in range(16)]
        for x, d in zip(xs, ds):
            nerf.hashgrid.hash_encode_bwd(x, emb._meta, d, 32, 2, ref, defer=False)
        ref = torch.stack(ref)
        # the reference rounds each pass's slice sum to fp32 before adding: cancelling rows differ
        # by a few ulp of the level's largest gradient
        torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6 * float(ref.abs().max()))


@pytest.mark.gpu
def test_hash_encode_bwd_large_ray_ordered(nerf, gpu, oracle):
    """The coarse pass at the metric config (4096 lego rays x 64 sorted samples, finest 1024):
    gradient tables of the binned path (workspace; LDS owner sums) and of the direct atomic path
    against an fp64 scatter of the oracle's corner indices and weights. Bound per row:
    |got - ref| <= 2e-6 * sum |contributions| (fp32 products, fp32 atomic sums in any order)."""
    from indoor_nerf_amd import _lib
    lo, hi = blender_bbox()
    ro, rd = synthetic_rays(4096, seed=21)
    rng = np.random.RandomState(21)
    z = np.sort(2.0 + 4.0 * rng.rand(4096, 64), axis=1).astype(np.float32)
    x = (ro[:, None, :] + rd[:, None, :] * z[..., None]).reshape(-1, 3).astype(np.float32)
    P = x.shape[0]
    dfeat = rng.randn(16, P, 2).astype(np.float32)
    emb = _embedder(nerf, gpu, 1024, closed_form_table())
    xt, dt = torch.from_numpy(x).to(gpu), torch.from_numpy(dfeat).to(gpu)
    meta = emb._meta
    got_ws = [torch.zeros(1 << 19, 2, device=gpu) for _ in range(16)]
    nerf.hashgrid.hash_encode_bwd(xt, meta, dt, 2, 2 * P, got_ws)
    got_direct = [torch.zeros(1 << 19, 2, device=gpu) for _ in range(16)]
    _lib.call("nerf_hash_encode_bwd", _lib.ptr(xt), P, meta["bmin"], meta["bmax"], meta["res"], 16, 19,
              _lib.ptr(dt), 2, 2 * P, _lib.ptr_array(got_direct), _lib.stream())
    xc = torch.from_numpy(x)
    bmin, bmax = torch.from_numpy(lo), torch.from_numpy(hi)
    for lvl in range(16):
        vmin, vmax, idx, _ = oracle.voxel_corners(xc, bmin, bmax, torch.tensor(emb.level_res[lvl]), 19)
        w = ((xc - vmin) / (vmax - vmin)).double()
        wx, wy, wz = w[:, 0:1], w[:, 1:2], w[:, 2:3]
        g = torch.from_numpy(dfeat[lvl]).double()
        cw = []
        for c in range(8):
            i, j, k = (c >> 2) & 1, (c >> 1) & 1, c & 1
            cw.append((wz if k else 1 - wz) * (wy if j else 1 - wy) * (wx if i else 1 - wx))
        contrib = torch.stack([g * cwc for cwc in cw], 1)          # [P, 8, 2]
        ref = torch.zeros(1 << 19, 2, dtype=torch.float64).index_add_(0, idx.reshape(-1), contrib.reshape(-1, 2))
        scale = torch.zeros(1 << 19, 2, dtype=torch.float64).index_add_(0, idx.reshape(-1),
                                                                          contrib.abs().reshape(-1, 2))
        for name, got in (("workspace", got_ws), ("direct", got_direct)):
            err = (got[lvl].cpu().double() - ref).abs()
            bad = err > 2e-6 * scale + 1e-30
            assert not bool(bad.any()), f"{name} level {lvl}: {int(bad.sum())} rows off, max err {float(err.max()):.3e}"


def _mlp_n(nerf, gpu, d, prefix, normals):
    net = nerf.NeRFSmall(num_layers=2, hidden_dim=64, geo_feat_dim=15, num_layers_color=3, hidden_dim_color=64,
                         input_ch=32, input_ch_views=16, predict_normals=normals).to(gpu)
    with torch.no_grad():
        for k, p in net.named_parameters():
            p.copy_(torch.from_numpy(d[prefix + k.replace(".", "_")]))
    return net


def test_normals_head_fwd_bwd(nerf, gpu, golden):
    """NeRFSmall(predict_normals=True) (run_nerf_helpers.py:259-263, :298-302): raw [P,7] and every
    gradient (MLP weights, normals head weights and biases, inputs) against the reference (F13)."""
    g = golden("f13_normals")
    net = _mlp_n(nerf, gpu, g, "w_", True)
    x = torch.from_numpy(g["x"]).to(gpu).requires_grad_(True)
    raw = net(x)
    assert raw.shape == (1024, 7)
    np.testing.assert_allclose(raw.detach().cpu().numpy(), g["raw"], rtol=1e-4, atol=2e-6)
    (raw * torch.from_numpy(g["g_raw"]).to(gpu)).sum().backward()
    np.testing.assert_allclose(x.grad.cpu().numpy(), g["dx"], rtol=1e-4, atol=2e-6)
    for k, p in net.named_parameters():
        np.testing.assert_allclose(p.grad.cpu().numpy(), g["dw_" + k.replace(".", "_")], rtol=1e-4, atol=1e-4,
                                   err_msg=k)


def test_composite_normals(nerf, gpu, golden):
    """raw2outputs(predict_normals=True) on a 7-channel raw: normal map and d raw (F13)."""
    g = golden("f13_normals")
    raw = torch.from_numpy(g["c_raw"]).to(gpu).requires_grad_(True)
    out = nerf.raw2outputs(raw, torch.from_numpy(g["c_z"]).to(gpu), torch.from_numpy(g["c_d"]).to(gpu), 0, True,
                           predict_normals=True)
    assert len(out) == 7
    np.testing.assert_allclose(out[0].detach().cpu().numpy(), g["c_rgb"], rtol=1e-5, atol=2e-6)
    np.testing.assert_allclose(out[6].detach().cpu().numpy(), g["c_normal"], rtol=1e-4, atol=2e-6)
    ((out[6] * torch.from_numpy(g["c_gn"]).to(gpu)).sum() + (out[0] * torch.from_numpy(g["c_gr"]).to(gpu)).sum()
     ).backward()
    np.testing.assert_allclose(raw.grad.cpu().numpy(), g["c_draw"], rtol=1e-4, atol=1e-5)


def test_render_with_normals(nerf, gpu, golden):
    """Full render with predict_normals=True (coarse net without the head, fine net with it, as
    create_nerf builds them): normal_map, the empty [R, 0] normal0 of the 4-channel coarse pass, and
    run_network's mask on the LAST channel (n_z, not sigma) for samples outside the bbox (F13)."""
    g = golden("f13_normals")
    emb = _embedder(nerf, gpu, 1024, closed_form_table())
    coarse, fine = _mlp_n(nerf, gpu, g, "r_coarse_", False), _mlp_n(nerf, gpu, g, "r_fine_", True)
    sh = nerf.SHEncoder()
    nqf = lambda inputs, viewdirs, fn: nerf.run_network(inputs, viewdirs, fn, emb, sh)  # noqa: E731
    kw = dict(network_query_fn=nqf, perturb=1.0, N_importance=64, network_fine=fine, N_samples=64, network_fn=coarse,
              embed_fn=emb, use_viewdirs=True, white_bkgd=True, raw_noise_std=0.0, predict_normals=True, ndc=False,
              lindisp=False, near=2.0, far=6.0)
    ro, rd = (torch.from_numpy(g[f"r_rays_{k}"]).to(gpu) for k in ("o", "d"))
    with torch.no_grad():
        rgb, depth, acc, ex = nerf.render(800, 800, None, rays=(ro, rd), retraw=True, pytest=True, **kw)
    assert tuple(ex["normal0"].shape) == tuple(g["r_normal0_shape"])
    np.testing.assert_allclose(ex["rgb0"].cpu().numpy(), g["r_rgb0"], rtol=1e-4, atol=1e-4)
    raw = ex["raw"].cpu().numpy()
    ref_raw = g["r_raw"]
    assert raw.shape == ref_raw.shape
    # fine samples follow sample_pdf (PSNR-equivalent bounds, as test_render_end_to_end)
    np.testing.assert_allclose(rgb.cpu().numpy(), g["r_rgb"], rtol=0, atol=1e-3)
    np.testing.assert_allclose(ex["normal_map"].cpu().numpy(), g["r_normal"], rtol=0, atol=2e-3)
    # the mask: n_z == 0 exactly where the reference has it (out-of-bbox samples), sigma never masked
    masked = ref_raw[..., 6] == 0
    assert masked.sum() > 0
    np.testing.assert_array_equal(raw[..., 6] == 0, masked)
    assert not np.any((raw[..., 3] == 0) & masked)


def test_mlp_bwd_geo_gradient_superposition(nerf, gpu):
    """The MLP backward's extra d geo input (from the normals head) against torch fp32 autograd of the
    same MLP with an extra (o * d_geo) term, alone and together with d raw (a VALU patch of the
    MFMA accumulator once broke only the combined case)."""
    from indoor_nerf_amd import _lib, field
    torch.manual_seed(0)
    net = nerf.NeRFSmall(2, 64, 15, 3, 64, 32, 16).to(gpu)
    P = 1024
    x = torch.randn(P, 48, device=gpu) * 0.5
    W = [w.detach() for w in net.mlp_weights()]

    def ours(gr4, dgeo):
        dfeat = torch.zeros(P, 48, device=gpu)
        for w in net.mlp_weights():
            w.grad = None
        grads = field._grads_struct(net.mlp_weights())
        _lib.call("nerf_mlp_bwd", _lib.ptr(x), 48, 2, _lib.c_vp(x.data_ptr() + 128), 48, None, 1, None, P,
                  field._weights_struct(net.mlp_weights()), _lib.ptr(gr4), grads, _lib.ptr(dfeat), None,
                  _lib.ptr(dgeo, allow_none=True), _lib.stream())
        return dfeat[:, :32].clone(), [w.grad.clone() for w in net.mlp_weights()]

    def ref(gr4, dgeo):
        xr = x.clone().requires_grad_(True)
        Wr = [w.clone().requires_grad_(True) for w in W]
        h = torch.relu(xr[:, :32] @ Wr[0].t())
        o = h @ Wr[1].t()
        c = torch.relu(torch.cat([xr[:, 32:], o[:, 1:]], -1) @ Wr[2].t())
        c = torch.relu(c @ Wr[3].t())
        out = torch.cat([c @ Wr[4].t(), o[:, :1]], -1)
        ((out * gr4).sum() + (o * dgeo).sum()).backward()
        return xr.grad[:, :32], [w.grad for w in Wr]

    torch.backends.cuda.matmul.allow_tf32 = False
    gr4 = torch.randn(P, 4, device=gpu)
    dgeo = torch.randn(P, 16, device=gpu)
    dgeo[:, 0] = 0
    for a, b in ((torch.zeros_like(gr4), dgeo), (gr4, dgeo)):
        f1, w1 = ours(a, b)
        f2, w2 = ref(a, b)
        torch.testing.assert_close(f1, f2, rtol=1e-4, atol=1e-5)
        for p, q in zip(w1, w2):
            torch.testing.assert_close(p, q, rtol=1e-4, atol=1e-4)


def test_llff_ndc_render_and_grads(nerf, gpu, golden):
    """Config 3 (LLFF fern): render(ndc=True) with the NDC bbox, near 0 / far 1, 64 + 64 samples,
    raw_noise_std 1 (pytest draws), no white background, + one backward (F15). Coarse pass at fp32
    rounding; fine pass PSNR-equivalent (sample_pdf, as test_render_end_to_end)."""
    g = golden("f15_llff")
    H, W, focal = int(g["hwf"][0]), int(g["hwf"][1]), float(g["hwf"][2])
    bbox = (torch.from_numpy(g["bbox_min"]), torch.from_numpy(g["bbox_max"]))
    emb = nerf.HashEmbedder(bbox, finest_resolution=512).to(gpu)
    table = closed_form_table(scale=0.3, salt=9)
    with torch.no_grad():
        for i, e in enumerate(emb.embeddings):
            e.weight.copy_(torch.from_numpy(table[i]))
    coarse, fine = _mlp(nerf, gpu, g, "coarse_"), _mlp(nerf, gpu, g, "fine_")
    sh = nerf.SHEncoder()
    nqf = lambda inputs, viewdirs, fn: nerf.run_network(inputs, viewdirs, fn, emb, sh)  # noqa: E731
    kw = dict(network_query_fn=nqf, perturb=1.0, N_importance=64, network_fine=fine, N_samples=64, network_fn=coarse,
              embed_fn=emb, use_viewdirs=True, white_bkgd=False, raw_noise_std=1.0, predict_normals=False, ndc=True,
              lindisp=False, near=0.0, far=1.0)
    ro, rd = (torch.from_numpy(g[k]).to(gpu) for k in ("rays_o", "rays_d"))
    rgb, depth, acc, ex = nerf.render(H, W, g["K"], rays=(ro, rd), retraw=True, pytest=True, **kw)
    for k in ("rgb0", "depth0", "acc0", "sparsity_loss0"):
        np.testing.assert_allclose(ex[k].detach().cpu().numpy(), g[k], rtol=1e-4, atol=1e-4, err_msg=k)
    np.testing.assert_allclose(rgb.detach().cpu().numpy(), g["rgb"], rtol=0, atol=1e-3)
    np.testing.assert_allclose(acc.detach().cpu().numpy(), g["acc"], rtol=0, atol=1e-3)
    np.testing.assert_allclose(depth.detach().cpu().numpy(), g["depth"], rtol=1e-3, atol=1e-3)
    np.testing.assert_allclose(ex["z_std"].detach().cpu().numpy(), g["z_std"], rtol=1e-3, atol=1e-3)
    target = torch.from_numpy(g["target"]).to(gpu)
    loss = nerf.img2mse(rgb, target) + nerf.img2mse(ex["rgb0"], target)
    loss.backward()
    np.testing.assert_allclose(loss.item(), float(g["loss"]), rtol=1e-3)
    for prefix, net in (("gcoarse_", coarse), ("gfine_", fine)):
        for k, p in net.named_parameters():
            want = g[prefix + k.replace(".", "_")]
            rel = np.linalg.norm(p.grad.cpu().numpy() - want) / np.linalg.norm(want)
            assert rel < 2e-2, f"{prefix}{k}: relative grad error {rel:.2e}"
    for i, e in enumerate(emb.embeddings):
        gd = e.weight.grad.double()
        np.testing.assert_allclose([(gd * gd).sum().item(), gd.abs().sum().item()], g["gtable_checksum"][i][1:],
                                   rtol=2e-2, err_msg=f"level {i}")


def test_get_rays_vs_reference(nerf, gpu, golden):
    """Device get_rays (csrc/rays.hip) vs run_nerf_helpers.get_rays (F16) with train()'s float64 K:
    a centred and an off-centre anisotropic camera, every pixel of a 60 x 80 image; bit-exact."""
    g = golden("f16_rays")
    H, W = int(g["H"]), int(g["W"])
    for tag in ("a", "b"):
        ro, rd = nerf.get_rays(H, W, g[f"K_{tag}"], torch.from_numpy(g[f"c2w_{tag}"]).to(gpu))
        np.testing.assert_array_equal(ro.cpu().numpy(), g[f"rays_o_{tag}"])
        np.testing.assert_array_equal(rd.cpu().numpy(), g[f"rays_d_{tag}"])


def test_ray_sampler_batches(nerf, gpu, golden):
    """RaySampler (train()'s no_batching batch, run_nerf.py:973-1004): N_rand distinct pixels,
    inside the precrop window before precrop_iters, rays equal to get_rays at those pixels and
    targets equal to the image there; over many draws every pixel is drawn about equally often."""
    g = golden("f16_rays")
    H, W = int(g["H"]), int(g["W"])
    rng = np.random.RandomState(0)
    images = rng.rand(2, H, W, 4).astype(np.float32)
    poses = np.stack([g["c2w_a"], g["c2w_b"]])
    K = g["K_a"]
    sampler = nerf.RaySampler(images, poses, H, W, K, i_train=[0, 1], N_rand=1024, precrop_iters=10,
                              precrop_frac=0.5, device=gpu)
    for it, img_i in ((3, 0), (20, 1)):
        rays, target, coords = sampler.sample(it, img_i=img_i, return_coords=True)
        c = coords.cpu().numpy()
        flat = c[:, 0] * W + c[:, 1]
        assert len(np.unique(flat)) == 1024, "pixels must be drawn without replacement"
        r0, c0, h, w = nerf.crop_window(H, W, it, 10, 0.5)
        assert c[:, 0].min() >= r0 and c[:, 0].max() < r0 + h and c[:, 1].min() >= c0 and c[:, 1].max() < c0 + w
        tag = "a" if img_i == 0 else "b"
        Kt = g[f"K_{tag}"] if img_i == 1 else K
        if img_i == 1:
            sampler.K = Kt
            sampler._cams.clear()
            rays, target, coords = sampler.sample(it, img_i=img_i, return_coords=True, seed=5)
            c = coords.cpu().numpy()
        np.testing.assert_array_equal(rays[0].cpu().numpy(), g[f"rays_o_{tag}"][c[:, 0], c[:, 1]])
        np.testing.assert_array_equal(rays[1].cpu().numpy(), g[f"rays_d_{tag}"][c[:, 0], c[:, 1]])
        np.testing.assert_array_equal(target.cpu().numpy(), images[img_i][c[:, 0], c[:, 1], :3])
    # uniformity: 300 draws of 1024 of the 4800 pixels -> 64 expected hits per pixel
    counts = np.zeros(H * W)
    for s in range(300):
        _, _, coords = sampler.sample(100 + s, img_i=0, seed=1000 + s, return_coords=True)
        c = coords.cpu().numpy()
        counts += np.bincount(c[:, 0] * W + c[:, 1], minlength=H * W)
    expect = 300 * 1024 / (H * W)
    z = (counts - expect) / np.sqrt(expect)
    assert abs(counts.sum() - 300 * 1024) < 1e-6
    assert np.abs(z).max() < 6.0 and abs(z.mean()) < 0.1 and 0.7 < z.std() < 1.3, (z.min(), z.max(), z.std())


@pytest.mark.parametrize("S,N,det,shuffle", [(64, 128, 1, False), (37, 30, 1, False), (16, 9, 1, False),
                                              (64, 256, 1, False), (64, 128, 0, False), (37, 30, 0, False),
                                              (64, 128, 0, True)])
def test_sample_fine_merge_vs_torch_sort(nerf, gpu, S, N, det, shuffle):
    """nerf_sample_fine's merged z / points vs torch.sort(cat(z, samples)) (run_nerf.py:486-490).

    Ragged sizes (M = S + N from 25 to 320, M % 4 != 0) with tied z values (coarse z quantised to
    1/8, det samples at bin edges): ties are broken by position, as a stable sort would. det=0 draws
    unsorted importance samples (Philox), which the kernel sorts (bitonic) before the merge; shuffle
    passes unsorted coarse z, which takes the kernel's rank-sort path.
    Sorting is exact: z_fine must equal the sorted values bit for bit; the points are o + d * z in
    fp32 (one rounding each, no contraction) and are compared at 1 ulp-level tolerance."""
    from indoor_nerf_amd import _lib
    R, C = 67, 11
    g = torch.Generator().manual_seed(S * 1000 + N)
    rays = torch.rand(R, C, generator=g).to(gpu)
    z = torch.sort(torch.round(torch.rand(R, S, generator=g) * 8 * 6) / 8 + 0.5, dim=1).values.to(gpu)
    if shuffle:
        z = z[:, torch.randperm(S, generator=g).to(gpu)].contiguous()
    w = torch.rand(R, S, generator=g).to(gpu)
    t_imp = torch.linspace(0.0, 1.0, N).to(gpu)
    z_fine = torch.empty(R, S + N, device=gpu)
    pts = torch.empty(R, S + N, 3, device=gpu)
    z_std = torch.empty(R, device=gpu)
    samples = torch.empty(R, N, device=gpu)
    _lib.call("nerf_sample_fine", _lib.ptr(rays), C, _lib.ptr(z), _lib.ptr(w), R, S, N, det, _lib.ptr(t_imp), None,
              7, 3, None, _lib.ptr(z_fine), _lib.ptr(pts), _lib.ptr(z_std), _lib.ptr(samples), _lib.stream())
    torch.cuda.synchronize()
    want = torch.sort(torch.cat([z, samples], -1), -1).values
    assert torch.equal(z_fine, want)
    want_pts = rays[:, None, 0:3] + rays[:, None, 3:6] * want[..., None]
    torch.testing.assert_close(pts, want_pts, rtol=1e-6, atol=1e-6)
    if det:
        assert (want[:, 1:] == want[:, :-1]).any(), "the case must contain ties"
    else:
        assert not bool((samples[:, 1:] >= samples[:, :-1]).all()), "importance samples must arrive unsorted"


@pytest.mark.gpu
@pytest.mark.parametrize("P", [1, 127, 100_003, 786_432])
def test_normal_head_bwd_vs_torch_fp64(nerf, gpu, P):
    """The normals head's backward kernel (csrc/normals.hip: per-point part, register-blocked weight
    gradients over 128-point tiles, per-block partials summed in order) against torch fp64 autograd of
    n = normalize(N1 relu(N0 geo + b0) + b1) with run_network's n_z mask, at ragged sizes up to the
    ScanNet step's 786,432 points: d raw4, d geo and the four weight gradients."""
    from indoor_nerf_amd import field
    g = torch.Generator().manual_seed(P)
    o16 = torch.randn(P, 16, generator=g) * 0.5
    keep = torch.rand(P, generator=g) > 0.1
    head = [torch.randn(32, 15, generator=g) * 0.3, torch.randn(32, generator=g) * 0.1,
            torch.randn(3, 32, generator=g) * 0.3, torch.randn(3, generator=g) * 0.1]
    g7 = torch.randn(P, 7, generator=g)
    dev = [t.to(gpu).requires_grad_(True) for t in head]
    for t in dev:
        t.grad = None
    graw4, dgeo = field._head_backward(o16.to(gpu), keep.to(gpu), dev, g7.to(gpu), [True] * 4)
    torch.cuda.synchronize()
    # fp64 reference
    ref = [t.double().requires_grad_(True) for t in head]
    geo = o16[:, 1:].double().requires_grad_(True)
    hdn = geo @ ref[0].T + ref[1]
    nn_ = torch.relu(hdn) @ ref[2].T + ref[3]
    nrm = torch.nn.functional.normalize(nn_, dim=-1)
    mask = torch.ones(P, 3, dtype=torch.float64)
    mask[:, 2] = keep.double()
    (nrm * mask * g7[:, 4:].double()).sum().backward()
    np.testing.assert_array_equal(graw4.cpu().numpy(), g7[:, :4].numpy())
    d = dgeo.cpu().double()
    assert torch.all(d[:, 0] == 0)
    # fp32 per-point arithmetic (the op order of the head's forward / normalize backward): 1e-4 absolute
    # covers the few points whose ||n|| is small enough to amplify one rounding (1 in 1.5 M at 1e-5)
    np.testing.assert_allclose(d[:, 1:].numpy(), geo.grad.numpy(), rtol=1e-4, atol=1e-4)
    for i, (mine, r) in enumerate(zip(dev, ref)):
        m = float(r.grad.abs().max())
        err = float((mine.grad.cpu().double() - r.grad).abs().max())
        assert err <= 1e-5 * m + 1e-6 * (P ** 0.5), (i, err, m)


@pytest.mark.gpu
@pytest.mark.parametrize("P", [1, 255, 786_432])
def test_normal_head_fwd_rows_matches_scatter(nerf, gpu, P):
    """nerf_normal_head_fwd_rows (the fine pass with coarse-feature reuse: keep flags in the MLP's
    importance-first order, rows = the merged row of each) against the plain forward after the
    scatter it replaces (keep_m[rows] = keep): raw7 and the merged keep flags bit for bit."""
    from indoor_nerf_amd import field
    g = torch.Generator().manual_seed(P + 7)
    o16 = (torch.randn(P, 16, generator=g) * 0.5).to(gpu)
    raw4 = torch.randn(P, 4, generator=g).to(gpu)
    keep = (torch.rand(P, generator=g) > 0.2).to(gpu)
    rows = torch.randperm(P, generator=g).to(torch.int32).to(gpu)
    head = [(torch.randn(32, 15, generator=g) * 0.3).to(gpu), (torch.randn(32, generator=g) * 0.1).to(gpu),
            (torch.randn(3, 32, generator=g) * 0.3).to(gpu), (torch.randn(3, generator=g) * 0.1).to(gpu)]
    raw7, keep_m = field._head_forward(o16, raw4, keep, head, rows=rows)
    want_keep = torch.empty_like(keep).index_put_((rows.long(),), keep)
    want = field._head_forward(o16, raw4, want_keep, head)
    torch.cuda.synchronize()
    assert torch.equal(keep_m, want_keep)
    assert torch.equal(raw7, want)


@pytest.mark.gpu
@pytest.mark.parametrize("std", [1.0, 0.37, 1e-3])
def test_raw_noise_one_launch_matches_randn_times_std(gpu, std):
    """raw2outputs' noise as normal_(0, std) in one launch: bit-identical to the reference's
    torch.randn(shape) * raw_noise_std from the same generator state (odd sizes included)."""
    for shape in ((4096, 64), (37, 13)):
        torch.manual_seed(123)
        want = torch.randn(*shape, device=gpu) * std
        torch.manual_seed(123)
        got = torch.empty(*shape, device=gpu).normal_(0.0, std)
        assert torch.equal(got, want), (shape, std)
