"""A-CAQ (BASELINE config 5) on the HIP path vs the reference (F14) and the oracle.

Tolerances:
  * hash features through the quantized gather (training/STE records and the eval-mode int-packed
    tables): BIT-EXACT vs the oracle — the quantizer is elementwise fp32 with the reference's op
    order, and the packed codes reproduce (q - zp) * scale exactly;
  * calibration: hash levels and W0 bit-exact (min/max of identical values); the activation
    quantizer's range is a max of MFMA outputs: rtol 1e-5;
  * render / grads: the activation quantizer rounds relu(x W0q^T) to 2^B codes, and MFMA vs CPU
    GEMM rounding can move a pre-activation across a code boundary (one code = range / (2^B - 1)).
    raw: >= 99.9 % of values within 1e-4 (a coarse-pass flip also moves the ray's fine samples);
    rgb within 2e-3 (PSNR-equivalent);
    grads in norm 2e-2.
"""
import numpy as np
import pytest
import torch

from tables import blender_bbox, closed_form_table

pytestmark = pytest.mark.gpu


def _bbox_t():
    lo, hi = blender_bbox()
    return torch.from_numpy(lo), torch.from_numpy(hi)


def _qmodules(nerf, gpu, g):
    table = closed_form_table(scale=0.3, salt=3)
    emb = nerf.HashEmbedder(_bbox_t(), finest_resolution=1024, use_quantization=True, quantization_bits=8).to(gpu)
    with torch.no_grad():
        for i, e in enumerate(emb.embeddings):
            e.weight.copy_(torch.from_numpy(table[i]))
    nets = []
    for prefix in ("coarse0_", "fine0_"):
        net = nerf.NeRFSmall(num_layers=2, hidden_dim=64, geo_feat_dim=15, num_layers_color=3, hidden_dim_color=64,
                             input_ch=32, input_ch_views=16, use_quantization=True, quantization_bits=8).to(gpu)
        sd = {k: torch.from_numpy(np.asarray(g[prefix + k.replace(".", "_")])) for k in net.state_dict()}
        net.load_state_dict(sd)
        nets.append(net)
    sh = nerf.SHEncoder()
    nqf = lambda inputs, viewdirs, fn: nerf.run_network(inputs, viewdirs, fn, emb, sh, netchunk=65536)  # noqa: E731
    kw = dict(network_query_fn=nqf, perturb=1.0, N_importance=128, network_fine=nets[1], N_samples=64,
              network_fn=nets[0], embed_fn=emb, use_viewdirs=True, white_bkgd=True, raw_noise_std=0.0,
              predict_normals=False, ndc=False, lindisp=False, near=2.0, far=6.0)
    return emb, nets, kw


def _set_state(emb, nets, g, p):
    with torch.no_grad():
        for i, q in enumerate(emb.quantizers):
            for k in ("soft_bits", "range_scale", "v_max", "running_min", "running_max"):
                getattr(q, k).fill_(float(g[p + "emb_" + k][i]))
        for tag, net in zip(("coarse", "fine"), nets):
            a, w = net.sigma_act_quantizers[0], net.sigma_weight_quantizer
            for k in ("soft_bits", "range_scale", "v_max", "running_min", "running_max"):
                getattr(a, k).fill_(float(g[f"{p}{tag}_act_{k}"]))
            for k in ("soft_bits", "range_scale", "running_min", "running_max"):
                getattr(w, k).fill_(float(g[f"{p}{tag}_w_{k}"]))


def _check_raw(raw, want, tag):
    """Fine-pass raw: a code flip in the coarse pass also moves that ray's importance samples
    (sample_pdf), so the few differing values are bounded only by raw's own range; the bulk must
    agree to fp32 rounding."""
    d = np.abs(raw - want)
    frac = float((d <= 1e-4 + 1e-4 * np.abs(want)).mean())
    print(f"{tag}: {frac:.5f} of raw within 1e-4, max |d raw| {d.max():.3e}")
    assert frac >= 0.999, f"{tag}: only {frac:.5f} of raw within 1e-4 (max |d| {d.max():.3e})"
    assert np.all(np.isfinite(raw) == np.isfinite(want))


def _render(nerf, kw, g, gpu, grad):
    ro, rd = (torch.from_numpy(g[k]).to(gpu) for k in ("rays_o", "rays_d"))
    with torch.set_grad_enabled(grad):
        return nerf.render(800, 800, None, rays=(ro, rd), retraw=True, pytest=True, **kw)


def _params(emb, nets):
    return list(emb.parameters()) + [p for n in nets for p in n.parameters()]


def test_acaq_calibration_and_collapse(nerf, gpu, golden):
    """a: the first quantized training iteration calibrates every quantizer; with the reference's
    v_max = running max, the activation quantizer's zero point is qmax and every relu output
    quantizes to 0 — sigma = 0, white background, zero gradients (the reference's behaviour)."""
    g = golden("f14_acaq")
    emb, nets, kw = _qmodules(nerf, gpu, g)
    emb.current_step = 499
    rgb, depth, acc, ex = _render(nerf, kw, g, gpu, True)
    assert emb.current_step == int(g["a_current_step"])
    for k in ("running_min", "running_max", "range_scale", "v_max"):
        got = np.array([float(getattr(q, k)) for q in emb.quantizers], np.float32)
        np.testing.assert_array_equal(got, g["a_emb_" + k], err_msg=k)
    for tag, net in zip(("coarse", "fine"), nets):
        w, a = net.sigma_weight_quantizer, net.sigma_act_quantizers[0]
        for k in ("running_min", "running_max", "range_scale"):
            assert float(getattr(w, k)) == float(g[f"a_{tag}_w_{k}"]), (tag, k)
        for k in ("running_min", "running_max", "range_scale", "v_max"):
            np.testing.assert_allclose(float(getattr(a, k)), g[f"a_{tag}_act_{k}"], rtol=1e-5, err_msg=(tag, k))
    np.testing.assert_array_equal(rgb.detach().cpu().numpy(), g["a_rgb"])
    np.testing.assert_array_equal(ex["rgb0"].detach().cpu().numpy(), g["a_rgb0"])
    _check_raw(ex["raw"].detach().cpu().numpy(), g["a_raw"], "a")
    target = torch.from_numpy(g["target"]).to(gpu)
    loss = nerf.img2mse(rgb, target) + nerf.img2mse(ex["rgb0"], target)
    loss.backward()
    assert abs(loss.item() - float(g["a_loss"])) <= 1e-6
    for net in nets:
        for p in net.mlp_weights():
            assert float(p.grad.abs().max()) == 0.0
    # quantizer scalars never receive gradients (their uses are detached)
    for q in list(emb.quantizers) + [nets[0].sigma_act_quantizers[0], nets[0].sigma_weight_quantizer]:
        assert all(p.grad is None for p in q.parameters())


def test_acaq_soft_bits_train_and_eval(nerf, gpu, golden):
    """b: float bit widths in training mode (+ backward through the STE); c: eval mode, where the
    embedder reads int-packed tables (2..32-bit levels: 4/8/16-bit codes and fp32)."""
    g = golden("f14_acaq")
    emb, nets, kw = _qmodules(nerf, gpu, g)
    emb.current_step = 10_000
    for q in list(emb.quantizers) + [m for n in nets for m in (n.sigma_act_quantizers[0], n.sigma_weight_quantizer)]:
        q.calibrated = True
    _set_state(emb, nets, g, "b_")
    rgb, depth, acc, ex = _render(nerf, kw, g, gpu, True)
    _check_raw(ex["raw"].detach().cpu().numpy(), g["b_raw"], "b")
    np.testing.assert_allclose(rgb.detach().cpu().numpy(), g["b_rgb"], rtol=0, atol=2e-3)
    np.testing.assert_allclose(ex["rgb0"].detach().cpu().numpy(), g["b_rgb0"], rtol=0, atol=2e-3)
    target = torch.from_numpy(g["target"]).to(gpu)
    loss = nerf.img2mse(rgb, target) + nerf.img2mse(ex["rgb0"], target)
    loss.backward()
    np.testing.assert_allclose(loss.item(), float(g["b_loss"]), rtol=1e-3)
    for tag, net in zip(("coarse", "fine"), nets):
        for k, p in net.named_parameters():
            key = f"b_g{tag}_" + k.replace(".", "_")
            if key not in g:
                assert p.grad is None, k
                continue
            want = g[key]
            rel = np.linalg.norm(p.grad.cpu().numpy() - want) / max(np.linalg.norm(want), 1e-30)
            assert rel < 2e-2, f"{tag} {k}: relative grad error {rel:.2e}"
    for i, e in enumerate(emb.embeddings):
        gd = e.weight.grad.double()
        np.testing.assert_allclose([(gd * gd).sum().item(), gd.abs().sum().item()], g["b_gtable_checksum"][i][1:],
                                   rtol=2e-2, err_msg=f"level {i}")
    # c: eval mode with integer widths 2..32 (packed gather)
    with torch.no_grad():
        for i, q in enumerate(emb.quantizers):
            q.soft_bits.fill_(float(g["c_emb_soft_bits"][i]))
    emb.eval()
    for n in nets:
        n.eval()
    rgb, depth, acc, ex = _render(nerf, kw, g, gpu, False)
    assert emb._packed is not None, "eval-mode quantized render must use the int-packed tables"
    _check_raw(ex["raw"].cpu().numpy(), g["c_raw"], "c")
    np.testing.assert_allclose(rgb.cpu().numpy(), g["c_rgb"], rtol=0, atol=2e-3)
    np.testing.assert_allclose(ex["rgb0"].cpu().numpy(), g["c_rgb0"], rtol=0, atol=2e-3)


def _points(n, seed):
    rng = np.random.RandomState(seed)
    lo, hi = blender_bbox()
    pts = (lo + (hi - lo) * rng.rand(n, 3)).astype(np.float32)
    pts[:64] = (lo - 0.3 + (hi - lo + 0.6) * rng.rand(64, 3)).astype(np.float32)   # some outside the bbox
    return pts


def _soft_bits(train):
    return [8.0, 7.6, 6.3, 5.5, 9.2, 4.45, 8.0, 6.5, 7.0, 3.7, 10.3, 8.8, 2.4, 12.6, 5.0, 7.5] if train else \
        [2, 3, 4, 5, 6, 7, 8, 9, 10, 12, 14, 16, 17, 20, 24, 32]


@pytest.mark.parametrize("training", [True, False])
def test_quantized_gather_bit_exact_vs_oracle(nerf, gpu, oracle, training):
    """Quantized hash features (training: fused fake-quant gather; eval: int-packed tables) are
    bit-identical to the oracle's hash_encode with the reference quantizers, at 65,536 points."""
    table = closed_form_table(scale=0.3, salt=3)
    emb = nerf.HashEmbedder(_bbox_t(), finest_resolution=1024, use_quantization=True).to(gpu)
    bits = _soft_bits(training)
    with torch.no_grad():
        for i, e in enumerate(emb.embeddings):
            e.weight.copy_(torch.from_numpy(table[i]))
        for i, q in enumerate(emb.quantizers):
            q.soft_bits.fill_(float(bits[i]))
            q.range_scale.fill_(0.59 + 0.001 * i)
            q.v_max.fill_(0.29 - 0.002 * i)
            q.calibrated = True
    emb.current_step = 10_000
    emb.train(training)
    pts = _points(65536, 5)
    with torch.no_grad():
        feat, keep = emb(torch.from_numpy(pts).to(gpu))
    if not training:
        assert emb._packed is not None
    lv = [(float(np.float32(bits[i])), float(np.float32(0.59 + 0.001 * i)), float(np.float32(0.29 - 0.002 * i)))
          for i in range(16)]
    lo, hi = _bbox_t()
    ref, ref_keep = oracle.hash_encode(torch.from_numpy(pts), [torch.from_numpy(t) for t in table], lo, hi,
                                       oracle.level_resolutions(16, 1024), 19, oracle.level_quantizers(lv, training))
    np.testing.assert_array_equal(feat.cpu().numpy(), ref.numpy())
    np.testing.assert_array_equal(keep.cpu().numpy(), ref_keep.numpy())


def test_packed_equals_fake_quant_full_size(nerf, gpu):
    """At the fine pass's size (786,432 points) the eval-mode packed gather equals the fused
    fake-quant gather with eval records, bit for bit (size-independent property)."""
    from indoor_nerf_amd import _lib
    from indoor_nerf_amd.quantization import quant_records
    table = closed_form_table(scale=0.3, salt=7)
    emb = nerf.HashEmbedder(_bbox_t(), finest_resolution=1024, use_quantization=True).to(gpu)
    with torch.no_grad():
        for i, e in enumerate(emb.embeddings):
            e.weight.copy_(torch.from_numpy(table[i]))
        for i, q in enumerate(emb.quantizers):
            q.soft_bits.fill_(float(_soft_bits(False)[i]))
            q.range_scale.fill_(0.6)
            q.v_max.fill_(0.3)
    emb.eval()
    x = torch.from_numpy(_points(786432, 6)).to(gpu)
    with torch.no_grad():
        f_packed, k_packed = emb(x)
    rec = quant_records(list(emb.quantizers), False)
    f_fq = torch.empty_like(f_packed)
    k_fq = torch.empty_like(k_packed)
    m = emb._meta
    _lib.call("nerf_hash_encode_fwd_q", _lib.ptr(x), x.shape[0], m["bmin"], m["bmax"], m["res"], 16, 19,
              _lib.ptr_array(emb.tables()), _lib.ptr(rec), _lib.ptr(f_fq), 32, 2, _lib.ptr(k_fq, dtype=torch.bool),
              _lib.stream())
    assert torch.equal(f_packed, f_fq)
    assert torch.equal(k_packed, k_fq)
    # a second eval forward after changing one level's bit width repacks that level only
    with torch.no_grad():
        emb.quantizers[3].soft_bits.fill_(11.0)
        f2, _ = emb(x)
    dirty = emb._packed["dirty"].cpu().numpy()
    assert dirty.tolist() == [0, 0, 0, 1] + [0] * 12
    rec2 = quant_records(list(emb.quantizers), False)
    _lib.call("nerf_hash_encode_fwd_q", _lib.ptr(x), x.shape[0], m["bmin"], m["bmax"], m["res"], 16, 19,
              _lib.ptr_array(emb.tables()), _lib.ptr(rec2), _lib.ptr(f_fq), 32, 2, _lib.ptr(k_fq, dtype=torch.bool),
              _lib.stream())
    assert torch.equal(f2, f_fq)


def test_quantizer_module_vs_golden(nerf, gpu, golden):
    """LearnedBitwidthQuantizer (standalone module) vs F11: calibration + STE forward, bit-exact."""
    g = golden("f11_quant")
    q = nerf.LearnedBitwidthQuantizer(init_bits=8.0, min_bits=2.0, max_bits=32.0, symmetric=False).to(gpu)
    x = torch.from_numpy(g["asym_x"]).to(gpu).requires_grad_(True)
    y = q(x)
    np.testing.assert_array_equal(y.detach().cpu().numpy(), g["asym_y"])
    np.testing.assert_array_equal(q.range_scale.detach().cpu().numpy(), g["asym_range"])
    np.testing.assert_array_equal(q.v_max.detach().cpu().numpy(), g["asym_vmax"])
    y.sum().backward()
    np.testing.assert_array_equal(x.grad.cpu().numpy(), g["asym_dx"])
    y2 = q(torch.from_numpy(g["asym_x2"]).to(gpu))
    np.testing.assert_array_equal(y2.detach().cpu().numpy(), g["asym_y2"])
    qs = nerf.LearnedBitwidthQuantizer(init_bits=8.0, symmetric=True).to(gpu)
    np.testing.assert_array_equal(qs(torch.from_numpy(g["sym_w"]).to(gpu)).detach().cpu().numpy(), g["sym_y"])
    assert q.integer_bit_width == 8 and q.get_quantization_params() == (0, 255)


def _acaq_reference_step(bits, current_loss, state, target_metric, bit_penalty, min_bits=2.0, max_bits=32.0):
    """run_nerf.py:1209-1250 restated with Python doubles on float32 soft_bits (the test's oracle)."""
    if target_metric is not None:
        target = target_metric
    else:
        state["best"] = current_loss if "best" not in state else min(state["best"], current_loss)
        target = state["best"] * 1.2
    out = []
    n = len(bits)
    for idx, b in enumerate(bits):
        loss_ratio = current_loss / target
        delta = -0.3 if loss_ratio < 0.95 else (-0.1 if loss_ratio < 1.05 else 0.2)
        delta -= bit_penalty * float(b) / 8.0
        delta *= 1.0 + (idx - n / 2) * 0.02
        nb = np.float32(np.float32(b) + np.float32(delta))
        out.append(np.float32(min(max(nb, np.float32(min_bits)), np.float32(max_bits))))
    return out


@pytest.mark.parametrize("target_metric", [None, 0.05])
def test_acaq_controller_vs_reference_loop(nerf, gpu, target_metric):
    """acaq_update (device) vs the reference's bit-width loop restated in Python: 18 quantizers
    (16 levels + the coarse net's two), iterations 1000..1090, a loss sequence that visits all
    three delta branches; soft_bits equal bit for bit, untouched off the 10-iteration grid."""
    from types import SimpleNamespace
    emb = nerf.HashEmbedder(_bbox_t(), use_quantization=True).to(gpu)
    net = nerf.NeRFSmall(2, 64, 15, 3, 64, 32, 16, use_quantization=True).to(gpu)
    kw = dict(embed_fn=emb, network_fn=net)
    qs = nerf.acaq_quantizers(kw)
    assert len(qs) == 18
    rng = np.random.RandomState(3)
    with torch.no_grad():
        for q in qs:
            q.soft_bits.fill_(float(np.float32(rng.uniform(3, 12))))
    args = SimpleNamespace(use_acaq=True, use_quantization=True, acaq_start_iter=1000, target_metric=target_metric,
                           bit_penalty=1e-3)
    bits = [np.float32(float(q.soft_bits)) for q in qs]
    state = {}
    losses = [0.06, 0.05, 0.045, 0.08, 0.03, 0.052, 0.07, 0.02, 0.05, 0.09, 0.051]
    for k, loss in enumerate(losses):
        i = 1000 + 5 * k
        lt = torch.tensor(np.float32(loss), device=gpu)
        nerf.acaq_update(i, lt, kw, args)
        if i % 10 == 0:
            bits = _acaq_reference_step(bits, float(np.float32(loss)), state, target_metric, 1e-3)
        got = [np.float32(float(q.soft_bits)) for q in qs]
        np.testing.assert_array_equal(np.array(got), np.array(bits), err_msg=f"iteration {i}")
    nerf.acaq_update(999, torch.tensor(0.5, device=gpu), kw, args)     # before acaq_start_iter: no-op
    np.testing.assert_array_equal(np.array([np.float32(float(q.soft_bits)) for q in qs]), np.array(bits))
