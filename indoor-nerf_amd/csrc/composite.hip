// Volume compositing: raw2outputs (PocketNeRF/run_nerf.py:347-411) forward and backward.
//
// One wavefront per ray (composite_common.h). The backward's suffix recurrence
//   U_j = sum_{k>j} gw_k alpha_k prod_{j<m<k} t_m,   dL/dalpha_j = T_j (gw_j - U_j)
// is a wave-level suffix scan of affine maps (X, P) -> X + P*U in fp64.
#include "composite_common.h"
#include "hash_common.h"   // TVParams, fill_tv, tv_fwd_block (the TV forward beside the fine compositing)

namespace nerf {

template <int K>
__global__ void __launch_bounds__(256) composite_fwd_kernel(CompositeArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t ray = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (ray >= a.R) return;   // wave-uniform
    composite_fwd_ray<K>(a, ray, lane, nullptr);
}


// The fine pass's compositing with the iteration's TV forward in the same launch
// (nerf_composite_fwd_tv): blocks [0, tv_blocks) are TV blocks (level = x / kTVFusedBlocks, four
// vertices per thread: the composite rays' registers), the rest one ray per wave as
// composite_fwd_kernel. The TV's gathers (17.5 us as a launch of their own, rocprof r06h) run beside
// the 4,096 one-wave rays (10 us).
constexpr int kTVFusedBlocks = 136, kTVFusedUnroll = 4;   // 136 x 256 x 4 >= 51^3: one round per thread
template <int K>
__global__ void __launch_bounds__(256) composite_fwd_tv_kernel(CompositeArgs a, TVParams tv, unsigned tv_blocks) {
    if (blockIdx.x < tv_blocks) {
        tv_fwd_block<kTVFusedUnroll>(tv, (int)(blockIdx.x / kTVFusedBlocks), blockIdx.x % kTVFusedBlocks,
                                     kTVFusedBlocks);
        return;
    }
    const int lane = threadIdx.x & 63;
    const int64_t ray = (int64_t)(blockIdx.x - tv_blocks) * 4 + (threadIdx.x >> 6);
    if (ray >= a.R) return;   // wave-uniform
    composite_fwd_ray<K>(a, ray, lane, nullptr);
}
static_assert(sizeof(CompositeArgs) + sizeof(TVParams) + 16 <= 4096, "composite_fwd_tv_kernel: kernel arguments");

// The backward of one ray (the wave's).
template <int K>
__device__ __forceinline__ void composite_bwd_ray(const CompositeArgs& a, int64_t ray, int lane) {
    RayState<K> st;
    float norm_d;
    ray_forward<K>(a, ray, lane, st, norm_d);
    const bool need_ent = a.g_ent != nullptr && a.g_ent[ray] != 0.f;
    const RaySums s = ray_sums<K>(a, st, false, false, a.g_depth != nullptr || a.g_disp != nullptr);

    // ---- per-ray upstream gradients
    float gr[3] = {0.f, 0.f, 0.f};
    if (a.g_rgb) { gr[0] = a.g_rgb[3 * ray]; gr[1] = a.g_rgb[3 * ray + 1]; gr[2] = a.g_rgb[3 * ray + 2]; }
    float g_acc = a.g_acc ? a.g_acc[ray] : 0.f;
    if (a.white) g_acc = g_acc - ((gr[0] + gr[1]) + gr[2]);     // rgb_map + (1 - acc)
    float g_depth = a.g_depth ? a.g_depth[ray] : 0.f;
    if (a.g_disp) {
        const float gd = a.g_disp[ray];
        if (gd != 0.f) {
            const float m = fmaxf(1e-10f, s.depth);
            const float gm = -gd / (m * m);
            if (s.depth > 1e-10f || s.depth != s.depth) g_depth += gm;
            else if (s.depth == 1e-10f) g_depth += 0.5f * gm;
        }
    }
    float gN = 0.f, gA = 0.f;      // depth = N / A
    const bool use_depth = g_depth != 0.f;
    if (use_depth) {
        gN = g_depth / s.acc;
        gA = -g_depth * s.depth_num / (s.acc * s.acc);
    }
    // normals: n = nraw / max(|nraw|, 1e-12)
    float gnr[3] = {0.f, 0.f, 0.f};
    if (a.C >= 7 && a.g_normal) {
        const float g0 = a.g_normal[3 * ray], g1 = a.g_normal[3 * ray + 1], g2 = a.g_normal[3 * ray + 2];
        const float dot = g0 * s.nraw[0] + g1 * s.nraw[1] + g2 * s.nraw[2];
        const float k = (s.nnorm >= 1e-12f) ? dot / (s.nden * s.nden) / s.nnorm : 0.f;
        gnr[0] = g0 / s.nden - k * s.nraw[0];
        gnr[1] = g1 / s.nden - k * s.nraw[1];
        gnr[2] = g2 / s.nden - k * s.nraw[2];
    }
    // entropy over probs = [w, q], normalised by Z
    const float eps = 1.1920928955078125e-07f;
    float gent_w_common = 0.f;     // added to every w_j: gZ + g_Wsum
    float ge = 0.f;
    float dpk[K];                  // d entropy / d p_j of this lane's samples (used twice)
    if (need_ent) {
        ge = a.g_ent[ray];
        double dot = 0;   // sum_i dp_i * probs_i
#pragma unroll
        for (int q = 0; q < K; ++q) {
            const float p = st.w[q] / s.Z;
            const float cp = fminf(fmaxf(p, eps), 1.0f - eps);
            const float mask = (p >= eps && p <= 1.0f - eps) ? 1.f : 0.f;
            dpk[q] = -ge * (logf(cp) + p * mask / cp);
            dot += (double)(dpk[q] * st.w[q]);
        }
        dot = wave_sum_dpp(dot);
        const float pq = s.q / s.Z;
        const float cpq = fminf(fmaxf(pq, eps), 1.0f - eps);
        const float maskq = (pq >= eps && pq <= 1.0f - eps) ? 1.f : 0.f;
        const float dpq = -ge * (logf(cpq) + pq * maskq / cpq);
        dot += (double)(dpq * s.q);
        const float gZ = (float)(-dot / ((double)s.Z * (double)s.Z));
        const float gq = dpq / s.Z + gZ;
        const float gW = (1.0f - s.wsum >= 1e-6f) ? -gq : 0.f;
        gent_w_common = gZ + gW;
    }

    // ---- per-sample dL/dw
    float gw[K];
#pragma unroll
    for (int q = 0; q < K; ++q) {
        const int j = lane * K + q;
        float g = 0.f;
        if (j < a.S) {
            g = (gr[0] * st.c[q][0] + gr[1] * st.c[q][1]) + gr[2] * st.c[q][2];
            g += g_acc;
            if (a.g_w) g += a.g_w[ray * a.S + j];
            if (use_depth) g += gN * st.z[q] + gA;
            if (need_ent) g += dpk[q] / s.Z + gent_w_common;
            if (a.C >= 7) g += gnr[0] * st.n[q][0] + gnr[1] * st.n[q][1] + gnr[2] * st.n[q][2];
        }
        gw[q] = g;
    }
    // ---- U recurrence: block map over this lane's samples, then suffix scan across lanes
    double X = 0.0, P = 1.0;       // U_{start-1} = X + P * U_{end-1}
#pragma unroll
    for (int q = K - 1; q >= 0; --q) {
        // U_{j-1} = gw_j alpha_j + t_j U_j
        X = (double)gw[q] * (double)st.alpha[q] + (double)st.t[q] * X;
        P = (double)st.t[q] * P;
    }
    double U = wave_excl_suffix_affine_dpp(X, P, lane);   // U at this lane's last sample
    float* out = a.graw;
#pragma unroll
    for (int q = K - 1; q >= 0; --q) {
        const int j = lane * K + q;
        const double galpha = st.T[q] * ((double)gw[q] - U);
        U = (double)gw[q] * (double)st.alpha[q] + (double)st.t[q] * U;
        if (j < a.S) {
            float* g = out + (ray * a.S + j) * a.C;
            const float wj = st.w[q];
            g[0] = (wj * gr[0]) * (st.c[q][0] * (1.0f - st.c[q][0]));
            g[1] = (wj * gr[1]) * (st.c[q][1] * (1.0f - st.c[q][1]));
            g[2] = (wj * gr[2]) * (st.c[q][2] * (1.0f - st.c[q][2]));
            g[3] = st.s[q] > 0.f ? (float)galpha * st.e[q] * st.delta[q] : 0.f;
            if (a.C >= 7) {
                g[4] = wj * gnr[0];
                g[5] = wj * gnr[1];
                g[6] = wj * gnr[2];
            }
        }
    }
}

template <int K>
__global__ void __launch_bounds__(256) composite_bwd_kernel(CompositeArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t ray = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (ray >= a.R) return;   // wave-uniform
    composite_bwd_ray<K>(a, ray, lane);
}

// Two compositing backwards in one launch (the fine and the coarse pass of a training iteration):
// blocks [0, split) take a0's rays, the rest a1's; each wave runs the single-job code above.
template <int K0, int K1>
__global__ void __launch_bounds__(256) composite_bwd_pair_kernel(CompositeArgs a0, CompositeArgs a1, unsigned split) {
    const int lane = threadIdx.x & 63;
    if (blockIdx.x < split) {
        const int64_t ray = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
        if (ray < a0.R) composite_bwd_ray<K0>(a0, ray, lane);
    } else {
        const int64_t ray = (int64_t)(blockIdx.x - split) * 4 + (threadIdx.x >> 6);
        if (ray < a1.R) composite_bwd_ray<K1>(a1, ray, lane);
    }
}

}  // namespace nerf

using namespace nerf;

static int pick_k(int S) { return (S + 63) / 64; }

#define NERF_COMPOSITE_DISPATCH(KERNEL, S, grid, stream, args)                                     \
    switch (pick_k(S)) {                                                                            \
        case 1: hipLaunchKernelGGL(KERNEL<1>, grid, dim3(256), 0, stream, args); break;             \
        case 2: hipLaunchKernelGGL(KERNEL<2>, grid, dim3(256), 0, stream, args); break;             \
        case 3: hipLaunchKernelGGL(KERNEL<3>, grid, dim3(256), 0, stream, args); break;             \
        case 4: hipLaunchKernelGGL(KERNEL<4>, grid, dim3(256), 0, stream, args); break;             \
        case 5: case 6: hipLaunchKernelGGL(KERNEL<6>, grid, dim3(256), 0, stream, args); break;     \
        default: hipLaunchKernelGGL(KERNEL<8>, grid, dim3(256), 0, stream, args); break;            \
    }

extern "C" int nerf_composite_fwd(const float* d_raw, int raw_channels, const float* d_z, const float* d_rays_d,
                                  const float* d_noise, int64_t n_rays, int n_samples, int white_bkgd,
                                  float* d_rgb, float* d_disp, float* d_acc, float* d_weights, float* d_depth,
                                  float* d_entropy, float* d_normal, void* stream) {
    NERF_REQUIRE(n_rays >= 0 && n_samples >= 1 && n_samples <= 512, "composite_fwd: R=%lld S=%d (S must be 1..512)",
                 (long long)n_rays, n_samples);
    NERF_REQUIRE(raw_channels == 4 || raw_channels == 7, "composite_fwd: raw_channels %d", raw_channels);
    NERF_REQUIRE(n_rays == 0 || (d_raw && d_z && d_rays_d && d_weights), "composite_fwd: null arg");
    NERF_REQUIRE(!(d_normal && raw_channels != 7), "composite_fwd: normal output needs 7 raw channels");
    if (n_rays == 0) return NERF_OK;
    CompositeArgs a{};
    a.raw = d_raw; a.C = raw_channels; a.z = d_z; a.rays_d = d_rays_d; a.noise = d_noise;
    a.R = n_rays; a.S = n_samples; a.white = white_bkgd;
    a.rgb = d_rgb; a.disp = d_disp; a.acc = d_acc; a.weights = d_weights; a.depth = d_depth;
    a.entropy = d_entropy; a.normal = d_normal;
    dim3 grid(blocks_for(n_rays, 4));
    NERF_COMPOSITE_DISPATCH(composite_fwd_kernel, n_samples, grid, as_stream(stream), a);
    NERF_CHECK_LAUNCH("composite_fwd");
    return NERF_OK;
}

extern "C" int nerf_composite_fwd_tv(const float* d_raw, int raw_channels, const float* d_z, const float* d_rays_d,
                                     const float* d_noise, int64_t n_rays, int n_samples, int white_bkgd,
                                     float* d_rgb, float* d_disp, float* d_acc, float* d_weights, float* d_depth,
                                     float* d_entropy, float* d_normal, const nerf_tv_fwd_job* tv, int n_levels,
                                     int log2_T, void* stream) {
    if (!tv)
        return nerf_composite_fwd(d_raw, raw_channels, d_z, d_rays_d, d_noise, n_rays, n_samples, white_bkgd, d_rgb,
                                  d_disp, d_acc, d_weights, d_depth, d_entropy, d_normal, stream);
    NERF_REQUIRE(n_rays >= 0 && n_samples >= 1 && n_samples <= 512, "composite_fwd_tv: R=%lld S=%d (S must be 1..512)",
                 (long long)n_rays, n_samples);
    NERF_REQUIRE(raw_channels == 4 || raw_channels == 7, "composite_fwd_tv: raw_channels %d", raw_channels);
    NERF_REQUIRE(n_rays == 0 || (d_raw && d_z && d_rays_d && d_weights), "composite_fwd_tv: null arg");
    NERF_REQUIRE(!(d_normal && raw_channels != 7), "composite_fwd_tv: normal output needs 7 raw channels");
    TVParams P{};
    const int rc = fill_tv(P, n_levels, log2_T, tv->min_vertex, tv->d_min_vertex, tv->cube);
    if (rc) return rc;
    NERF_REQUIRE(tv->d_tables && tv->d_loss, "composite_fwd_tv: null TV arg");
    for (int l = 0; l < n_levels; ++l) {
        NERF_REQUIRE(tv->d_tables[l], "composite_fwd_tv: TV table %d null", l);
        P.tables[l] = tv->d_tables[l];
    }
    P.loss = tv->d_loss;
    P.verts = reinterpret_cast<float2*>(tv->d_verts);
    CompositeArgs a{};
    a.raw = d_raw; a.C = raw_channels; a.z = d_z; a.rays_d = d_rays_d; a.noise = d_noise;
    a.R = n_rays; a.S = n_samples; a.white = white_bkgd;
    a.rgb = d_rgb; a.disp = d_disp; a.acc = d_acc; a.weights = d_weights; a.depth = d_depth;
    a.entropy = d_entropy; a.normal = d_normal;
    const unsigned tvb = (unsigned)(kTVFusedBlocks * n_levels);
    const dim3 grid((unsigned)(tvb + blocks_for(n_rays, 4)));
    hipStream_t st = as_stream(stream);
    switch (pick_k(n_samples)) {
        case 1: hipLaunchKernelGGL(composite_fwd_tv_kernel<1>, grid, dim3(256), 0, st, a, P, tvb); break;
        case 2: hipLaunchKernelGGL(composite_fwd_tv_kernel<2>, grid, dim3(256), 0, st, a, P, tvb); break;
        case 3: hipLaunchKernelGGL(composite_fwd_tv_kernel<3>, grid, dim3(256), 0, st, a, P, tvb); break;
        case 4: hipLaunchKernelGGL(composite_fwd_tv_kernel<4>, grid, dim3(256), 0, st, a, P, tvb); break;
        case 5: case 6: hipLaunchKernelGGL(composite_fwd_tv_kernel<6>, grid, dim3(256), 0, st, a, P, tvb); break;
        default: hipLaunchKernelGGL(composite_fwd_tv_kernel<8>, grid, dim3(256), 0, st, a, P, tvb); break;
    }
    NERF_CHECK_LAUNCH("composite_fwd_tv");
    return NERF_OK;
}

static int composite_bwd_args(const nerf_composite_bwd_job& j, CompositeArgs& a) {
    NERF_REQUIRE(j.n_rays >= 0 && j.n_samples >= 1 && j.n_samples <= 512,
                 "composite_bwd: R=%lld S=%d (S must be 1..512)", (long long)j.n_rays, j.n_samples);
    NERF_REQUIRE(j.raw_channels == 4 || j.raw_channels == 7, "composite_bwd: raw_channels %d", j.raw_channels);
    NERF_REQUIRE(j.n_rays == 0 || (j.raw && j.z && j.rays_d && j.graw), "composite_bwd: null arg");
    a = CompositeArgs{};
    a.raw = j.raw; a.C = j.raw_channels; a.z = j.z; a.rays_d = j.rays_d; a.noise = j.noise;
    a.R = j.n_rays; a.S = j.n_samples; a.white = j.white_bkgd;
    a.g_rgb = j.g_rgb; a.g_disp = j.g_disp; a.g_acc = j.g_acc; a.g_w = j.g_weights; a.g_depth = j.g_depth;
    a.g_ent = j.g_entropy; a.g_normal = j.g_normal; a.graw = j.graw;
    return NERF_OK;
}

static void composite_bwd_launch(const CompositeArgs& a, hipStream_t stream) {
    NERF_COMPOSITE_DISPATCH(composite_bwd_kernel, a.S, dim3(blocks_for(a.R, 4)), stream, a);
}

extern "C" int nerf_composite_bwd(const float* d_raw, int raw_channels, const float* d_z, const float* d_rays_d,
                                  const float* d_noise, int64_t n_rays, int n_samples, int white_bkgd,
                                  const float* d_g_rgb, const float* d_g_disp, const float* d_g_acc,
                                  const float* d_g_weights, const float* d_g_depth, const float* d_g_entropy,
                                  const float* d_g_normal, float* d_graw, void* stream) {
    const nerf_composite_bwd_job j{d_raw, raw_channels, d_z, d_rays_d, d_noise, n_rays, n_samples, white_bkgd,
                                   d_g_rgb, d_g_disp, d_g_acc, d_g_weights, d_g_depth, d_g_entropy, d_g_normal,
                                   d_graw};
    CompositeArgs a;
    const int rc = composite_bwd_args(j, a);
    if (rc != NERF_OK) return rc;
    if (n_rays == 0) return NERF_OK;
    composite_bwd_launch(a, as_stream(stream));
    NERF_CHECK_LAUNCH("composite_bwd");
    return NERF_OK;
}

#define NERF_PAIR(K0, K1) \
    case 10 * K0 + K1: hipLaunchKernelGGL((composite_bwd_pair_kernel<K0, K1>), grid, dim3(256), 0, st, a0, a1, split); break;

extern "C" int nerf_composite_bwd_batch(const nerf_composite_bwd_job* jobs, int n_jobs, void* stream) {
    NERF_REQUIRE(n_jobs >= 0 && (n_jobs == 0 || jobs), "composite_bwd_batch: %d jobs", n_jobs);
    CompositeArgs args[2];
    int live = 0;
    for (int i = 0; i < n_jobs; ++i) {   // every job validated before anything is launched
        CompositeArgs a;
        const int rc = composite_bwd_args(jobs[i], a);
        if (rc != NERF_OK) return rc;
    }
    hipStream_t st = as_stream(stream);
    for (int i = 0; i < n_jobs; ++i) {
        CompositeArgs a;
        composite_bwd_args(jobs[i], a);
        if (a.R == 0) continue;
        if (live == 2) {   // more than two: the rest one launch each
            composite_bwd_launch(a, st);
            continue;
        }
        args[live++] = a;
    }
    if (live == 2) {
        // the heavier job's blocks first (the launch's tail is the lighter job's short waves)
        if (pick_k(args[1].S) > pick_k(args[0].S)) std::swap(args[0], args[1]);
        const CompositeArgs& a0 = args[0];
        const CompositeArgs& a1 = args[1];
        const unsigned split = blocks_for(a0.R, 4);
        const dim3 grid(split + blocks_for(a1.R, 4));
        switch (10 * pick_k(a0.S) + pick_k(a1.S)) {
            NERF_PAIR(1, 1) NERF_PAIR(2, 1) NERF_PAIR(3, 1) NERF_PAIR(4, 1) NERF_PAIR(2, 2) NERF_PAIR(3, 2)
            NERF_PAIR(4, 2) NERF_PAIR(3, 3)
            default:
                composite_bwd_launch(a0, st);
                composite_bwd_launch(a1, st);
        }
    } else if (live == 1) {
        composite_bwd_launch(args[0], st);
    }
    NERF_CHECK_LAUNCH("composite_bwd_batch");
    return NERF_OK;
}
#undef NERF_PAIR
