"""Radiance field: NeRFSmall and run_network on the fused HIP MLP.

API mirror of PocketNeRF/run_nerf_helpers.py:169-306 (NeRFSmall, same constructor arguments, same
parameters `sigma_net.{0,1}.weight`, `color_net.{0,1,2}.weight`) and run_network / batchify
(PocketNeRF/run_nerf.py:43-68). When run_network is handed this package's HashEmbedder, SHEncoder
and NeRFSmall it runs the fused path (FieldFn): hash encoding in a level-major layout, SH of each
ray's view direction computed once per point inside the MLP kernel's prologue, and the
sigma := 0 mask in its epilogue — no [P,48] concat and no per-sample SH tensor.
"""
import torch
import torch.nn as nn

from . import _lib
from .hashgrid import HashEmbedder, HashEncodeFn, SHEncoder, accumulate_grad_buffers, hash_encode_bwd


def _weights_struct(weights):
    w = _lib.MlpWeights()
    for name, t in zip(("w0", "w1", "c0", "c1", "c2"), weights):
        setattr(w, name, _lib.ptr(t.detach(), name).value)
    return w


def _grads_struct(weights):
    g = _lib.MlpGrads()
    for name, t in zip(("w0", "w1", "c0", "c1", "c2"), accumulate_grad_buffers(weights)):
        setattr(g, name, _lib.ptr(t, "grad_" + name).value)
    return g


class MLPFn(torch.autograd.Function):
    """x [P, 48] = [hash feat 32 | SH 16] -> raw [P, 4]. Weight grads accumulate into .grad."""

    @staticmethod
    def forward(ctx, x, net, *weights):
        x = x.contiguous()
        P = x.shape[0]
        raw = torch.empty(P, 4, device=x.device, dtype=torch.float32)
        xp = _lib.ptr(x, "x")
        sh_ptr = _lib.c_vp(x.data_ptr() + 32 * 4) if P > 0 else xp
        _lib.call("nerf_mlp_fwd", xp, 48, 2, sh_ptr, 48, None, 1, None, P, _weights_struct(weights),
                  _lib.ptr(raw, "raw"), _lib.stream())
        ctx.save_for_backward(x, *weights)
        return raw

    @staticmethod
    def backward(ctx, g_raw):
        x, *weights = ctx.saved_tensors
        P = x.shape[0]
        g = g_raw.contiguous()
        need_x = ctx.needs_input_grad[0]
        dx = torch.zeros_like(x) if need_x else None
        if any(w.requires_grad for w in weights) or need_x:
            grads = _grads_struct(weights) if any(w.requires_grad for w in weights) else _scratch_grads(weights)
            xp = _lib.ptr(x, "x")
            sh_ptr = _lib.c_vp(x.data_ptr() + 32 * 4) if P > 0 else xp
            dfeat = _lib.ptr(dx, "dx") if need_x else None
            dsh = None
            if need_x:
                dsh_t = torch.empty(P, 16, device=x.device, dtype=torch.float32)
                dsh = _lib.ptr(dsh_t, "dsh")
            _lib.call("nerf_mlp_bwd", xp, 48, 2, sh_ptr, 48, None, 1, None, P, _weights_struct(weights),
                      _lib.ptr(g, "grad_raw"), grads, dfeat, dsh, _lib.stream())
            if need_x:
                dx[:, 32:] = dsh_t
        return (dx, None) + (None,) * len(weights)


def _scratch_grads(weights):
    g = _lib.MlpGrads()
    for name, t in zip(("w0", "w1", "c0", "c1", "c2"), weights):
        setattr(g, name, _lib.ptr(torch.zeros_like(t), "scratch").value)
    return g


class FieldFn(torch.autograd.Function):
    """Fused run_network: pts [P,3], viewdirs [R,3] (P = R*S) -> raw [P,4]."""

    @staticmethod
    def forward(ctx, pts, viewdirs, samples_per_ray, embedder, net, *params):
        if pts.requires_grad or viewdirs.requires_grad:
            raise NotImplementedError("run_network: gradients w.r.t. positions/directions are not implemented")
        n_tab = embedder.n_levels
        tables, weights = params[:n_tab], params[n_tab:]
        pts = pts.contiguous()
        viewdirs = viewdirs.contiguous()
        P = pts.shape[0]
        feat = torch.empty(n_tab, P, 2, device=pts.device, dtype=torch.float32)
        keep = torch.empty(P, device=pts.device, dtype=torch.bool)
        meta = embedder._meta
        _lib.call("nerf_hash_encode_fwd", _lib.ptr(pts, "pts"), P, meta["bmin"], meta["bmax"], meta["res"], n_tab,
                  meta["log2_T"], _lib.ptr_array(tables), _lib.ptr(feat, "feat"), 2, 2 * P,
                  _lib.ptr(keep, "keep", dtype=torch.bool), _lib.stream())
        raw = torch.empty(P, 4, device=pts.device, dtype=torch.float32)
        _lib.call("nerf_mlp_fwd", _lib.ptr(feat, "feat"), 2, 2 * P, None, 0, _lib.ptr(viewdirs, "viewdirs"),
                  samples_per_ray, _lib.ptr(keep, "keep", dtype=torch.bool), P, _weights_struct(weights),
                  _lib.ptr(raw, "raw"), _lib.stream())
        ctx.save_for_backward(pts, viewdirs, feat, keep, *params)
        ctx.spr, ctx.embedder, ctx.n_tab = samples_per_ray, embedder, n_tab
        return raw

    @staticmethod
    def backward(ctx, g_raw):
        pts, viewdirs, feat, keep, *params = ctx.saved_tensors
        tables, weights = params[:ctx.n_tab], params[ctx.n_tab:]
        P = pts.shape[0]
        g = g_raw.contiguous()
        need_tab = any(t.requires_grad for t in tables)
        dfeat = torch.empty_like(feat) if need_tab else None
        if any(w.requires_grad for w in weights) or need_tab:
            grads = _grads_struct(weights) if any(w.requires_grad for w in weights) else _scratch_grads(weights)
            _lib.call("nerf_mlp_bwd", _lib.ptr(feat, "feat"), 2, 2 * P, None, 0, _lib.ptr(viewdirs, "viewdirs"),
                      ctx.spr, _lib.ptr(keep, "keep", dtype=torch.bool), P, _weights_struct(weights),
                      _lib.ptr(g, "grad_raw"), grads, _lib.ptr(dfeat, "dfeat", allow_none=True), None,
                      _lib.stream())
        if need_tab:
            hash_encode_bwd(pts, ctx.embedder._meta, dfeat, 2, 2 * P, accumulate_grad_buffers(tables))
        return (None,) * (5 + len(params))


class NeRFSmall(nn.Module):
    """run_nerf_helpers.py:169-306 on the fused MFMA MLP. create_nerf builds it with
    num_layers=2, hidden_dim=64, geo_feat_dim=15, num_layers_color=3, hidden_dim_color=64,
    input_ch=32 (hash), input_ch_views=16 (SH) — the only shape the kernel implements."""

    def __init__(self, num_layers=3, hidden_dim=64, geo_feat_dim=15, num_layers_color=4, hidden_dim_color=64,
                 input_ch=3, input_ch_views=3, use_quantization=False, quantization_bits=8, predict_normals=False):
        super().__init__()
        shape = (num_layers, hidden_dim, geo_feat_dim, num_layers_color, hidden_dim_color, input_ch, input_ch_views)
        if shape != (2, 64, 15, 3, 64, 32, 16):
            raise NotImplementedError(f"NeRFSmall{shape}: the HIP MLP implements create_nerf's configuration "
                                      "(2, 64, 15, 3, 64, 32, 16)")
        if use_quantization:
            raise NotImplementedError("NeRFSmall(use_quantization=True): A-CAQ MLP quantizers are not built yet")
        if predict_normals:
            raise NotImplementedError("NeRFSmall(predict_normals=True): the normals head is not built yet")
        self.input_ch = input_ch
        self.input_ch_views = input_ch_views
        self.use_quantization = use_quantization
        self.num_layers = num_layers
        self.geo_feat_dim = geo_feat_dim
        self.num_layers_color = num_layers_color
        self.predict_normals = predict_normals
        self.sigma_act_quantizers = None
        self.sigma_weight_quantizer = None
        self.sigma_net = nn.ModuleList([nn.Linear(input_ch, hidden_dim, bias=False),
                                        nn.Linear(hidden_dim, 1 + geo_feat_dim, bias=False)])
        self.color_net = nn.ModuleList([nn.Linear(input_ch_views + geo_feat_dim, hidden_dim_color, bias=False),
                                        nn.Linear(hidden_dim_color, hidden_dim_color, bias=False),
                                        nn.Linear(hidden_dim_color, 3, bias=False)])

    def mlp_weights(self):
        return [self.sigma_net[0].weight, self.sigma_net[1].weight, self.color_net[0].weight,
                self.color_net[1].weight, self.color_net[2].weight]

    def forward(self, x):
        for w in self.mlp_weights():
            if not w.is_contiguous():
                raise ValueError("NeRFSmall: weights must be contiguous")
        return MLPFn.apply(x.float(), self, *self.mlp_weights())


def batchify(fn, chunk):
    """run_nerf.py:43-50."""
    if chunk is None:
        return fn

    def ret(inputs):
        return torch.cat([fn(inputs[i:i + chunk]) for i in range(0, inputs.shape[0], chunk)], 0)
    return ret


def run_network(inputs, viewdirs, fn, embed_fn, embeddirs_fn, netchunk=1024 * 64):
    """run_nerf.py:53-68. inputs [..., S, 3], viewdirs [R, 3]. Fused when the modules are ours;
    netchunk is then only a memory knob the fused kernels do not need."""
    fused = (isinstance(embed_fn, HashEmbedder) and isinstance(fn, NeRFSmall)
             and isinstance(embeddirs_fn, SHEncoder) and viewdirs is not None and inputs.dim() == 3)
    if fused:
        if embed_fn.training:
            embed_fn.current_step += 1
        R, S = inputs.shape[0], inputs.shape[1]
        raw = FieldFn.apply(inputs.reshape(-1, 3), viewdirs, S, embed_fn, fn,
                            *embed_fn.tables(), *fn.mlp_weights())
        return raw.reshape(R, S, 4)
    inputs_flat = torch.reshape(inputs, [-1, inputs.shape[-1]])
    embedded, keep_mask = embed_fn(inputs_flat)
    if viewdirs is not None:
        input_dirs = viewdirs[:, None].expand(inputs.shape)
        embedded = torch.cat([embedded, embeddirs_fn(torch.reshape(input_dirs, [-1, input_dirs.shape[-1]]))], -1)
    outputs_flat = batchify(fn, netchunk)(embedded)
    outputs_flat = outputs_flat.clone()
    outputs_flat[~keep_mask, -1] = 0
    return torch.reshape(outputs_flat, list(inputs.shape[:-1]) + [outputs_flat.shape[-1]])
