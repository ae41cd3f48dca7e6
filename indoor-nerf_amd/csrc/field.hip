// Radiance field MLP of NeRFSmall (PocketNeRF/run_nerf_helpers.py:169-306, as create_nerf builds
// it, run_nerf.py:240-247): sigma net 32 -> 64 -> 16, colour net [SH16 | geo15] -> 64 -> 64 -> 3,
// no biases, ReLU between layers, no output activation; plus run_network's sigma := 0 outside the
// bbox (run_nerf.py:66) and SHEncoder degree 4 (hash_encoding.py:153-191) in the prologue.
//
// This file holds the SH kernel and the C ABI of the MLP; the kernels are the fp32-accurate
// bf16x6 MFMA kernels of field_x6.hip (forward, activation-quantizer calibration, and the
// chain / weight-gradient wave-pair backward).
#include "field_common.h"

namespace nerf {

__global__ void __launch_bounds__(256) sh4_fwd_kernel(const float* __restrict__ d, int64_t n, float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float o[16];
    sh4_eval(d[3 * i], d[3 * i + 1], d[3 * i + 2], o);
#pragma unroll
    for (int k = 0; k < 16; k += 4)
        *reinterpret_cast<float4*>(out + 16 * i + k) = make_float4(o[k], o[k + 1], o[k + 2], o[k + 3]);
}

int launch_mlp_fwd_x6(const MlpArgs& a, hipStream_t stream);     // field_x6.hip
int launch_mlp_act_minmax_x6(const MlpArgs& a, hipStream_t stream);
int launch_mlp_bwd_x6(const MlpArgs* jobs, int n_jobs, float* det_ws, hipStream_t stream);

static int fill_args(MlpArgs& a, const float* d_feat, int64_t sp, int64_t sl, const float* d_sh, int64_t sh_stride,
                     const float* d_viewdirs, int64_t spr, const uint8_t* d_keep, int64_t n,
                     const nerf_mlp_weights* w) {
    NERF_REQUIRE(n >= 0, "mlp: n_points < 0");
    NERF_REQUIRE((n == 0 || d_feat) && w && w->w0 && w->w1 && w->c0 && w->c1 && w->c2, "mlp: null feature/weight pointer");
    NERF_REQUIRE(n == 0 || d_viewdirs || d_sh, "mlp: need d_sh or d_viewdirs");
    NERF_REQUIRE(!d_viewdirs || spr >= 1, "mlp: samples_per_ray must be >= 1");
    NERF_REQUIRE(d_viewdirs || sh_stride != 0 || spr >= 1, "mlp: per-ray SH rows need samples_per_ray >= 1");
    NERF_REQUIRE(d_viewdirs || sh_stride != 0 || ((uintptr_t)d_sh & 15) == 0, "mlp: per-ray SH rows must be 16-B aligned");
    a.feat = d_feat; a.sp = sp; a.sl = sl; a.sh = d_sh; a.sh_stride = sh_stride;
    a.viewdirs = d_viewdirs; a.spr = spr; a.keep = d_keep; a.P = n; a.W = *w;
    a.dsp = sp; a.dsl = sl;
    a.io_rows = nullptr; a.seg_split = n; a.spr2 = 1;
    ray_div_magic(spr, a.rd_m1, a.rd_s1);
    ray_div_magic(1, a.rd_m2, a.rd_s2);
    return NERF_OK;
}

static int fill_order(MlpArgs& a, const nerf_point_order* o) {
    if (!o) return NERF_OK;
    a.io_rows = o->io_rows;
    if (o->spr2 == 0) return NERF_OK;   // one segment (a zero-filled order)
    NERF_REQUIRE(o->seg_split >= 0 && o->seg_split <= a.P && o->spr2 >= 1,
                 "mlp: point order: seg_split %lld of %lld points, spr2 %lld", (long long)o->seg_split,
                 (long long)a.P, (long long)o->spr2);
    a.seg_split = o->seg_split;
    a.spr2 = o->spr2;
    ray_div_magic(a.spr2, a.rd_m2, a.rd_s2);
    return NERF_OK;
}

}  // namespace nerf

using namespace nerf;

extern "C" int nerf_sh4_fwd(const float* d_dirs, int64_t n, float* d_out, void* stream) {
    NERF_REQUIRE(n >= 0 && (n == 0 || (d_dirs && d_out)), "sh4_fwd: bad args");
    if (n == 0) return NERF_OK;
    hipLaunchKernelGGL(sh4_fwd_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, as_stream(stream), d_dirs, n, d_out);
    NERF_CHECK_LAUNCH("sh4_fwd");
    return NERF_OK;
}

extern "C" size_t nerf_mlp_h3_bytes(int64_t n_points) {
    return n_points > 0 ? (size_t)((n_points + 31) / 32) * 2048 * sizeof(float) : 0;
}

extern "C" int nerf_mlp_fwd_h3(const float* d_feat, int64_t feat_stride_point, int64_t feat_stride_level,
                               const float* d_sh, int64_t sh_stride, const float* d_viewdirs, int64_t samples_per_ray,
                               const uint8_t* d_keep, int64_t n_points, const nerf_mlp_weights* weights, float* d_raw,
                               float* d_geo, const float* d_act_qrec, uint32_t* d_act_minmax,
                               int64_t act_calib_points, const nerf_point_order* order, float* d_h3, void* stream) {
    MlpArgs a{};
    int rc = fill_args(a, d_feat, feat_stride_point, feat_stride_level, d_sh, sh_stride, d_viewdirs, samples_per_ray,
                       d_keep, n_points, weights);
    if (rc) return rc;
    rc = fill_order(a, order);
    if (rc) return rc;
    NERF_REQUIRE(n_points == 0 || d_raw || d_act_minmax, "mlp_fwd: null output");
    NERF_REQUIRE(!d_h3 || (!d_act_qrec && !d_act_minmax), "mlp_fwd: saved h3 with A-CAQ (its backward recomputes)");
    if (n_points == 0) return NERF_OK;
    a.raw = d_raw;
    a.geo_out = d_geo;
    a.aq = reinterpret_cast<const QuantRec*>(d_act_qrec);
    a.act_minmax = d_act_minmax;
    a.calib_points = act_calib_points;
    a.h3 = d_h3;
    // the calibration-only launch (d_act_minmax) computes layer 0 and its statistics, nothing else
    return a.act_minmax ? launch_mlp_act_minmax_x6(a, as_stream(stream)) : launch_mlp_fwd_x6(a, as_stream(stream));
}

extern "C" int nerf_mlp_fwd_ord(const float* d_feat, int64_t feat_stride_point, int64_t feat_stride_level,
                                const float* d_sh, int64_t sh_stride, const float* d_viewdirs, int64_t samples_per_ray,
                                const uint8_t* d_keep, int64_t n_points, const nerf_mlp_weights* weights, float* d_raw,
                                float* d_geo, const float* d_act_qrec, uint32_t* d_act_minmax,
                                int64_t act_calib_points, const nerf_point_order* order, void* stream) {
    return nerf_mlp_fwd_h3(d_feat, feat_stride_point, feat_stride_level, d_sh, sh_stride, d_viewdirs, samples_per_ray,
                           d_keep, n_points, weights, d_raw, d_geo, d_act_qrec, d_act_minmax, act_calib_points, order,
                           nullptr, stream);
}

extern "C" int nerf_mlp_fwd_q(const float* d_feat, int64_t feat_stride_point, int64_t feat_stride_level,
                              const float* d_sh, int64_t sh_stride, const float* d_viewdirs, int64_t samples_per_ray,
                              const uint8_t* d_keep, int64_t n_points, const nerf_mlp_weights* weights, float* d_raw,
                              float* d_geo, const float* d_act_qrec, uint32_t* d_act_minmax, int64_t act_calib_points,
                              void* stream) {
    return nerf_mlp_fwd_ord(d_feat, feat_stride_point, feat_stride_level, d_sh, sh_stride, d_viewdirs, samples_per_ray,
                            d_keep, n_points, weights, d_raw, d_geo, d_act_qrec, d_act_minmax, act_calib_points, nullptr,
                            stream);
}

extern "C" int nerf_mlp_fwd(const float* d_feat, int64_t feat_stride_point, int64_t feat_stride_level,
                            const float* d_sh, int64_t sh_stride, const float* d_viewdirs, int64_t samples_per_ray,
                            const uint8_t* d_keep, int64_t n_points, const nerf_mlp_weights* weights, float* d_raw,
                            float* d_geo, void* stream) {
    return nerf_mlp_fwd_q(d_feat, feat_stride_point, feat_stride_level, d_sh, sh_stride, d_viewdirs, samples_per_ray,
                          d_keep, n_points, weights, d_raw, d_geo, nullptr, nullptr, 0, stream);
}

extern "C" int nerf_mlp_bwd_q(const float* d_feat, int64_t feat_stride_point, int64_t feat_stride_level,
                              const float* d_sh, int64_t sh_stride, const float* d_viewdirs, int64_t samples_per_ray,
                              const uint8_t* d_keep, int64_t n_points, const nerf_mlp_weights* weights,
                              const float* d_graw, const nerf_mlp_grads* grads, float* d_dfeat, float* d_dsh,
                              const float* d_dgeo, const float* d_act_qrec, void* stream) {
    MlpArgs a{};
    int rc = fill_args(a, d_feat, feat_stride_point, feat_stride_level, d_sh, sh_stride, d_viewdirs, samples_per_ray,
                       d_keep, n_points, weights);
    if (rc) return rc;
    NERF_REQUIRE((n_points == 0 || d_graw) && grads && grads->w0 && grads->w1 && grads->c0 && grads->c1 && grads->c2,
                 "mlp_bwd: null gradient pointer");
    if (n_points == 0) return NERF_OK;
    a.graw = d_graw; a.G = *grads; a.dfeat = d_dfeat; a.dsh = d_dsh; a.dgeo = d_dgeo;
    a.aq = reinterpret_cast<const QuantRec*>(d_act_qrec);
    return launch_mlp_bwd_x6(&a, 1, nullptr, as_stream(stream));
}

extern "C" size_t nerf_mlp_bwd_det_workspace_bytes(void) {
    return (size_t)kMlpBwdMaxBlocks * GW_TOTAL * sizeof(float);
}

extern "C" int nerf_mlp_bwd_batch(const nerf_mlp_bwd_job* jobs, int n_jobs, float* d_det_workspace,
                                  size_t det_workspace_bytes, void* stream) {
    NERF_REQUIRE(jobs && n_jobs >= 1 && n_jobs <= NERF_MLP_MAX_JOBS, "mlp_bwd_batch: %d jobs (1..%d)", n_jobs,
                 NERF_MLP_MAX_JOBS);
    NERF_REQUIRE(!d_det_workspace || det_workspace_bytes >= nerf_mlp_bwd_det_workspace_bytes(),
                 "mlp_bwd_batch: deterministic workspace %zu B < %zu B", det_workspace_bytes,
                 nerf_mlp_bwd_det_workspace_bytes());
    MlpArgs a[NERF_MLP_MAX_JOBS]{};
    int n = 0;
    for (int k = 0; k < n_jobs; ++k) {
        const nerf_mlp_bwd_job& j = jobs[k];
        MlpArgs& x = a[n];
        int rc = fill_args(x, j.feat, j.feat_stride_point, j.feat_stride_level, j.sh, j.sh_stride, j.viewdirs,
                           j.samples_per_ray, j.keep, j.n_points, &j.weights);
        if (rc) return rc;
        const nerf_mlp_grads& g = j.grads;
        NERF_REQUIRE((j.n_points == 0 || j.graw) && g.w0 && g.w1 && g.c0 && g.c1 && g.c2, "mlp_bwd_batch: job %d: null gradient pointer", k);
        x.graw = j.graw; x.G = g; x.dfeat = j.dfeat; x.dsh = j.dsh; x.dgeo = j.dgeo;
        x.aq = reinterpret_cast<const QuantRec*>(j.act_qrec);
        rc = fill_order(x, &j.order);
        if (rc) return rc;
        if (j.dfeat_stride_level) {
            x.dsp = j.dfeat_stride_point;
            x.dsl = j.dfeat_stride_level;
        }
        NERF_REQUIRE(!j.rows == !j.d_count, "mlp_bwd_batch: job %d: rows and d_count go together", k);
        x.rows = j.rows;
        x.count = j.d_count;
        NERF_REQUIRE(!j.h3 || (!j.act_qrec && !j.rows), "mlp_bwd_batch: job %d: saved h3 with A-CAQ or active rows", k);
        x.h3 = const_cast<float*>(j.h3);
        if (x.P > 0) ++n;   // empty jobs launch nothing
    }
    if (n == 0) return NERF_OK;
    if (n == 2 && ((a[0].aq != nullptr) != (a[1].aq != nullptr) ||
                   (a[0].h3 != nullptr) != (a[1].h3 != nullptr))) {   // one quantizer / h3 mode per launch
        int rc = launch_mlp_bwd_x6(&a[0], 1, d_det_workspace, as_stream(stream));
        return rc ? rc : launch_mlp_bwd_x6(&a[1], 1, d_det_workspace, as_stream(stream));
    }
    return launch_mlp_bwd_x6(a, n, d_det_workspace, as_stream(stream));
}

extern "C" int nerf_mlp_bwd(const float* d_feat, int64_t feat_stride_point, int64_t feat_stride_level,
                            const float* d_sh, int64_t sh_stride, const float* d_viewdirs, int64_t samples_per_ray,
                            const uint8_t* d_keep, int64_t n_points, const nerf_mlp_weights* weights,
                            const float* d_graw, const nerf_mlp_grads* grads, float* d_dfeat, float* d_dsh,
                            const float* d_dgeo, void* stream) {
    return nerf_mlp_bwd_q(d_feat, feat_stride_point, feat_stride_level, d_sh, sh_stride, d_viewdirs, samples_per_ray,
                          d_keep, n_points, weights, d_graw, grads, d_dfeat, d_dsh, d_dgeo, nullptr, stream);
}
