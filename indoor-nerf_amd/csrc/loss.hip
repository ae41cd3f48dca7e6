// Training-loss head of one iteration (run_nerf.py:1011-1037), fused: photometric MSE of the fine
// and coarse passes, sparsity, TV, and PSNR in ONE single-workgroup launch; its backward in ONE
// elementwise launch. Replaces ~30 tiny torch kernels per step (each ~5 us of GPU time on gfx950).
//
//   img_loss  = mean((rgb - t)^2)                          img2mse, run_nerf_helpers.py:10
//   loss      = img_loss + mean((rgb0 - t)^2)              :1012-1019
//             + sparse_w * (sum(sp) + sum(sp0))            :1022-1023
//             + tv_w * (((0 + tv[0]) + tv[1]) + ...)       :1031-1035 (python sum over levels)
//   psnr      = -10 * log(img_loss) / log(10)              mse2psnr, run_nerf_helpers.py:11
//
// Backward, in autograd's operation order (MeanBackward then PowBackward):
//   d rgb = (g / N) * (2 * (rgb - t)),  d sp = sparse_w * g,  d tv[l] = tv_w * g.
#include "common.h"

namespace nerf {

constexpr int kLossThreads = 1024;

struct LossArgs {
    const float* rgb;
    const float* rgb0;     // may be null (no coarse pass)
    const float* target;
    int64_t n_rgb;         // R * 3
    const float* sp;       // may be null
    const float* sp0;      // may be null
    int64_t n_sp;          // R
    float sparse_w;
    const float* tv;       // may be null
    int n_tv;
    float tv_w;
    float* loss;
    float* img_loss;
    float* psnr;
};

// Sums in fp64 (one workgroup; the inputs are a few thousand values), rounded once to fp32: closer
// to the exact mean than torch's fp32 tree, which is what the parity tolerance is written against.
__global__ void __launch_bounds__(kLossThreads) train_loss_fwd_kernel(LossArgs a) {
    __shared__ double s_red4[4][kLossThreads / 64];
    double se = 0.0, se0 = 0.0, ssp = 0.0, ssp0 = 0.0;
    // every load of a round is issued before the first add (one memory round trip per round: the
    // lego batch, 12,288 colour values + 4,096 sparsity values, is one round); each thread still
    // adds its elements in index order, so the sums are those of the plain strided loops
    constexpr int UR = 16, US = 4;
    for (int64_t i0 = threadIdx.x, j0 = threadIdx.x; i0 < a.n_rgb || j0 < a.n_sp;
         i0 += UR * kLossThreads, j0 += US * kLossThreads) {
        float t[UR], r[UR], r0[UR], s[US], s0[US];
#pragma unroll
        for (int u = 0; u < UR; ++u) {
            const int64_t i = i0 + (int64_t)u * kLossThreads;
            const bool ok = i < a.n_rgb;
            t[u] = ok ? a.target[i] : 0.f;
            r[u] = ok ? a.rgb[i] : 0.f;
            r0[u] = (ok && a.rgb0) ? a.rgb0[i] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < US; ++u) {
            const int64_t j = j0 + (int64_t)u * kLossThreads;
            const bool ok = j < a.n_sp;
            s[u] = (ok && a.sp) ? a.sp[j] : 0.f;
            s0[u] = (ok && a.sp0) ? a.sp0[j] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < UR; ++u) {
            if (i0 + (int64_t)u * kLossThreads < a.n_rgb) {
                const float d = r[u] - t[u];
                se += (double)(d * d);
                if (a.rgb0) {
                    const float d0 = r0[u] - t[u];
                    se0 += (double)(d0 * d0);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < US; ++u) {
            if (j0 + (int64_t)u * kLossThreads < a.n_sp) {
                if (a.sp) ssp += (double)s[u];
                if (a.sp0) ssp0 += (double)s0[u];
            }
        }
    }
    // the four block sums share one barrier: wave sums (DPP lane moves), then thread 0 adds the waves' partials in
    // wave order (one barrier instead of two per sum)
    {
        const double w0 = wave_sum_dpp(se), w1 = wave_sum_dpp(se0), w2 = wave_sum_dpp(ssp), w3 = wave_sum_dpp(ssp0);
        const int w = threadIdx.x >> 6;
        if ((threadIdx.x & 63) == 0) { s_red4[0][w] = w0; s_red4[1][w] = w1; s_red4[2][w] = w2; s_red4[3][w] = w3; }
        __syncthreads();
        se = se0 = ssp = ssp0 = 0.0;
        if (threadIdx.x == 0)
            for (int i = 0; i < kLossThreads / 64; ++i) {
                se += s_red4[0][i];
                se0 += s_red4[1][i];
                ssp += s_red4[2][i];
                ssp0 += s_red4[3][i];
            }
    }
    if (threadIdx.x == 0) {
        const float n = (float)a.n_rgb;
        const float img = (float)se / n;
        float loss = img;
        if (a.rgb0) loss = loss + (float)se0 / n;
        if (a.sp || a.sp0) {
            float s = a.sp ? (float)ssp : 0.f;
            if (a.sp0) s = s + (float)ssp0;
            loss = loss + a.sparse_w * s;
        }
        if (a.tv) {
            float tv = 0.f;
            for (int l = 0; l < a.n_tv; ++l) tv = tv + a.tv[l];
            loss = loss + a.tv_w * tv;
        }
        *a.loss = loss;
        *a.img_loss = img;
        *a.psnr = -10.0f * logf(img) / 2.30258512496948242f;   // float32(log(10)), as torch.log(Tensor([10.]))
    }
}

struct LossGradArgs {
    const float* rgb;
    const float* rgb0;
    const float* target;
    int64_t n_rgb;
    int64_t n_sp;
    float sparse_w;
    int n_tv;
    float tv_w;
    const float* g;        // device scalar: upstream gradient of loss
    float* d_rgb;
    float* d_rgb0;         // null when rgb0 is null
    float* d_sp;           // may be null
    float* d_sp0;          // may be null
    float* d_tv;           // may be null
};

__global__ void __launch_bounds__(256) train_loss_bwd_kernel(LossGradArgs a) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const float g = *a.g;
    const float gm = g / (float)a.n_rgb;
    if (i < a.n_rgb) {
        const float t = a.target[i];
        a.d_rgb[i] = gm * (2.0f * (a.rgb[i] - t));
        if (a.d_rgb0) a.d_rgb0[i] = gm * (2.0f * (a.rgb0[i] - t));
    }
    if (i < a.n_sp) {
        const float gs = a.sparse_w * g;
        if (a.d_sp) a.d_sp[i] = gs;
        if (a.d_sp0) a.d_sp0[i] = gs;
    }
    if (a.d_tv && i < a.n_tv) a.d_tv[i] = a.tv_w * g;
}

}  // namespace nerf

using namespace nerf;

extern "C" int nerf_train_loss_fwd(const float* d_rgb, const float* d_rgb0, const float* d_target, int64_t n_rays,
                                   const float* d_sparsity, const float* d_sparsity0, float sparse_w,
                                   const float* d_tv, int n_tv, float tv_w, float* d_loss, float* d_img_loss,
                                   float* d_psnr, void* stream) {
    NERF_REQUIRE(n_rays > 0, "train_loss_fwd: n_rays %lld", (long long)n_rays);
    NERF_REQUIRE(d_rgb && d_target && d_loss && d_img_loss && d_psnr, "train_loss_fwd: null arg");
    NERF_REQUIRE(n_tv >= 0 && (n_tv == 0 || d_tv), "train_loss_fwd: n_tv %d", n_tv);
    LossArgs a{d_rgb, d_rgb0, d_target, 3 * n_rays, d_sparsity, d_sparsity0, n_rays, sparse_w,
               n_tv ? d_tv : nullptr, n_tv, tv_w, d_loss, d_img_loss, d_psnr};
    hipLaunchKernelGGL(train_loss_fwd_kernel, dim3(1), dim3(kLossThreads), 0, as_stream(stream), a);
    NERF_CHECK_LAUNCH("train_loss_fwd");
    return NERF_OK;
}

extern "C" int nerf_train_loss_bwd(const float* d_rgb, const float* d_rgb0, const float* d_target, int64_t n_rays,
                                   float sparse_w, int n_tv, float tv_w, const float* d_grad_loss, float* d_grad_rgb,
                                   float* d_grad_rgb0, float* d_grad_sparsity, float* d_grad_sparsity0,
                                   float* d_grad_tv, void* stream) {
    NERF_REQUIRE(n_rays > 0, "train_loss_bwd: n_rays %lld", (long long)n_rays);
    NERF_REQUIRE(d_rgb && d_target && d_grad_loss && d_grad_rgb, "train_loss_bwd: null arg");
    NERF_REQUIRE(!d_grad_rgb0 || d_rgb0, "train_loss_bwd: grad_rgb0 without rgb0");
    NERF_REQUIRE(n_tv >= 0, "train_loss_bwd: n_tv %d", n_tv);
    LossGradArgs a{d_rgb, d_rgb0, d_target, 3 * n_rays, n_rays, sparse_w, n_tv, tv_w, d_grad_loss,
                   d_grad_rgb, d_grad_rgb0, d_grad_sparsity, d_grad_sparsity0, n_tv ? d_grad_tv : nullptr};
    const int64_t n = std::max<int64_t>(3 * n_rays, n_tv);
    hipLaunchKernelGGL(train_loss_bwd_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, as_stream(stream), a);
    NERF_CHECK_LAUNCH("train_loss_bwd");
    return NERF_OK;
}
