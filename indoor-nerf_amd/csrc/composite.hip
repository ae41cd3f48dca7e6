// Volume compositing: raw2outputs (PocketNeRF/run_nerf.py:347-411) forward and backward.
//
// One wavefront per ray; lane L owns the K = ceil(S/64) consecutive samples [K*L, K*L+K). The
// transmittance T_j = prod_{k<j}(1 - alpha_k + 1e-10) is a wave-level exclusive product scan over
// the lanes' local products (DPP lane moves: common.h wave_excl_prod_dpp); the backward's suffix
// recurrence
//   U_j = sum_{k>j} gw_k alpha_k prod_{j<m<k} t_m,   dL/dalpha_j = T_j (gw_j - U_j)
// is a wave-level suffix scan of affine maps (X, P) -> X + P*U. Scans and ray sums run in fp64:
// the reference's CPU cumprod/cumsum accumulate in double, and the cost here is negligible.
// Quirks kept: last delta = 1e10, +1e-10 inside the product, NaN depth when sum(w) == 0,
// disp = 1/max(1e-10, depth) (NaN propagates), Categorical entropy over [w, max(1-sum w, 1e-6)].
#include "common.h"

namespace nerf {

struct CompositeArgs {
    const float* raw; int C;
    const float* z;
    const float* rays_d;
    const float* noise;
    int64_t R; int S; int white;
    // forward outputs
    float* rgb; float* disp; float* acc; float* weights; float* depth; float* entropy; float* normal;
    // backward inputs/outputs
    const float* g_rgb; const float* g_disp; const float* g_acc; const float* g_w;
    const float* g_depth; const float* g_ent; const float* g_normal;
    float* graw;
};

__device__ __forceinline__ float sigmoidf(float x) { return 1.0f / (1.0f + expf(-x)); }

// Per-sample forward quantities.
template <int K>
struct RayState {
    float c[K][3];     // sigmoid(rgb_raw)
    float n[K][3];     // normals (C == 7)
    float s[K];        // sigma + noise
    float delta[K];    // dists * |d|
    float e[K];        // exp(-relu(s) * delta)
    float alpha[K];
    float t[K];        // 1 - alpha + 1e-10
    float z[K];
    double T[K];       // transmittance (exclusive product)
    float w[K];        // weights
};


template <int K>
__device__ __forceinline__ void ray_forward(const CompositeArgs& a, int64_t ray, int lane, RayState<K>& st,
                                            float& norm_d) {
    const float dx = a.rays_d[3 * ray + 0], dy = a.rays_d[3 * ray + 1], dz = a.rays_d[3 * ray + 2];
    norm_d = sqrtf(dx * dx + dy * dy + dz * dz);
    const float* zr = a.z + ray * a.S;
    double lprod = 1.0;
    double Tloc[K];
#pragma unroll
    for (int q = 0; q < K; ++q) {
        const int j = lane * K + q;
        Tloc[q] = lprod;
        if (j < a.S) {
            const float* r = a.raw + (ray * a.S + j) * a.C;
            const float zj = zr[j];
            st.z[q] = zj;
            const float dist = (j + 1 < a.S) ? (zr[j + 1] - zj) : 1e10f;
            st.delta[q] = dist * norm_d;
            st.c[q][0] = sigmoidf(r[0]);
            st.c[q][1] = sigmoidf(r[1]);
            st.c[q][2] = sigmoidf(r[2]);
            float sg = r[3];
            if (a.noise) sg = sg + a.noise[ray * a.S + j];
            st.s[q] = sg;
            const float relu_s = sg > 0.f ? sg : 0.f;
            st.e[q] = expf(-relu_s * st.delta[q]);
            st.alpha[q] = 1.0f - st.e[q];
            st.t[q] = (1.0f - st.alpha[q]) + 1e-10f;
            if (a.C >= 7) {
                st.n[q][0] = r[4]; st.n[q][1] = r[5]; st.n[q][2] = r[6];
            } else {
                st.n[q][0] = st.n[q][1] = st.n[q][2] = 0.f;
            }
            lprod *= (double)st.t[q];
        } else {
            st.z[q] = 0.f; st.delta[q] = 0.f; st.s[q] = 0.f; st.e[q] = 1.f; st.alpha[q] = 0.f; st.t[q] = 1.f;
            st.c[q][0] = st.c[q][1] = st.c[q][2] = 0.f;
            st.n[q][0] = st.n[q][1] = st.n[q][2] = 0.f;
        }
    }
    const double pre = wave_excl_prod_dpp(lprod);
#pragma unroll
    for (int q = 0; q < K; ++q) {
        st.T[q] = pre * Tloc[q];
        st.w[q] = st.alpha[q] * (float)st.T[q];
    }
}

struct RaySums {
    float rgb[3], acc, depth_num, depth, disp, wsum, q, Z, ent, nraw[3], nden, nnorm;
};

// need_rgb / need_depth (wave-uniform): the backward needs neither the colour sums nor, without a
// depth or disparity gradient, the depth numerator — each skipped sum is one fp64 wave reduction
template <int K>
__device__ __forceinline__ RaySums ray_sums(const CompositeArgs& a, const RayState<K>& st, bool need_ent,
                                           bool need_rgb = true, bool need_depth = true) {
    double r0 = 0, r1 = 0, r2 = 0, acc = 0, dn = 0, n0 = 0, n1 = 0, n2 = 0;
    const bool normals = a.C >= 7;   // wave-uniform
#pragma unroll
    for (int q = 0; q < K; ++q) {
        const double w = st.w[q];
        r0 += (double)(st.w[q] * st.c[q][0]);
        r1 += (double)(st.w[q] * st.c[q][1]);
        r2 += (double)(st.w[q] * st.c[q][2]);
        acc += w;
        dn += (double)(st.w[q] * st.z[q]);
        n0 += (double)(st.w[q] * st.n[q][0]);
        n1 += (double)(st.w[q] * st.n[q][1]);
        n2 += (double)(st.w[q] * st.n[q][2]);
    }
    RaySums s;
    s.rgb[0] = s.rgb[1] = s.rgb[2] = 0.f;
    if (need_rgb) {
        s.rgb[0] = (float)wave_sum_dpp(r0);
        s.rgb[1] = (float)wave_sum_dpp(r1);
        s.rgb[2] = (float)wave_sum_dpp(r2);
    }
    s.acc = (float)wave_sum_dpp(acc);
    s.depth_num = need_depth ? (float)wave_sum_dpp(dn) : 0.f;
    s.depth = s.depth_num / s.acc;
    {
        const float m = (s.depth != s.depth) ? s.depth : fmaxf(1e-10f, s.depth);   // torch.max keeps NaN
        s.disp = 1.0f / m;
    }
    s.wsum = s.acc;
    s.q = fmaxf(1.0f - s.wsum, 1e-6f);
    if (!(1.0f - s.wsum == 1.0f - s.wsum)) s.q = 1.0f - s.wsum;   // NaN stays NaN under clamp
    s.Z = (float)((double)s.acc + (double)s.q);
    s.ent = 0.f;
    if (need_ent) {
        const float eps = 1.1920928955078125e-07f;
        double h = 0;
#pragma unroll
        for (int q = 0; q < K; ++q) {
            const float p = st.w[q] / s.Z;
            h += (double)(logf(fminf(fmaxf(p, eps), 1.0f - eps)) * p);
        }
        h = wave_sum_dpp(h);
        const float pq = s.q / s.Z;
        h += (double)(logf(fminf(fmaxf(pq, eps), 1.0f - eps)) * pq);
        s.ent = (float)(-h);
    }
    s.nraw[0] = s.nraw[1] = s.nraw[2] = 0.f;
    if (normals) {
        s.nraw[0] = (float)wave_sum_dpp(n0);
        s.nraw[1] = (float)wave_sum_dpp(n1);
        s.nraw[2] = (float)wave_sum_dpp(n2);
    }
    s.nnorm = sqrtf(s.nraw[0] * s.nraw[0] + s.nraw[1] * s.nraw[1] + s.nraw[2] * s.nraw[2]);
    s.nden = fmaxf(s.nnorm, 1e-12f);
    return s;
}

template <int K>
__global__ void __launch_bounds__(256) composite_fwd_kernel(CompositeArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t ray = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (ray >= a.R) return;   // wave-uniform
    RayState<K> st;
    float norm_d;
    ray_forward<K>(a, ray, lane, st, norm_d);
    const RaySums s = ray_sums<K>(a, st, a.entropy != nullptr);
#pragma unroll
    for (int q = 0; q < K; ++q) {
        const int j = lane * K + q;
        if (j < a.S) a.weights[ray * a.S + j] = st.w[q];
    }
    if (lane == 0) {
        float rgb0 = s.rgb[0], rgb1 = s.rgb[1], rgb2 = s.rgb[2];
        if (a.white) {
            const float bg = 1.0f - s.acc;
            rgb0 = rgb0 + bg; rgb1 = rgb1 + bg; rgb2 = rgb2 + bg;
        }
        if (a.rgb) { a.rgb[3 * ray] = rgb0; a.rgb[3 * ray + 1] = rgb1; a.rgb[3 * ray + 2] = rgb2; }
        if (a.acc) a.acc[ray] = s.acc;
        if (a.depth) a.depth[ray] = s.depth;
        if (a.disp) a.disp[ray] = s.disp;
        if (a.entropy) a.entropy[ray] = s.ent;
        if (a.normal) {
            a.normal[3 * ray + 0] = s.nraw[0] / s.nden;
            a.normal[3 * ray + 1] = s.nraw[1] / s.nden;
            a.normal[3 * ray + 2] = s.nraw[2] / s.nden;
        }
    }
}


template <int K>
__global__ void __launch_bounds__(256) composite_bwd_kernel(CompositeArgs a) {
    const int lane = threadIdx.x & 63;
    const int64_t ray = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (ray >= a.R) return;
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

extern "C" int nerf_composite_bwd(const float* d_raw, int raw_channels, const float* d_z, const float* d_rays_d,
                                  const float* d_noise, int64_t n_rays, int n_samples, int white_bkgd,
                                  const float* d_g_rgb, const float* d_g_disp, const float* d_g_acc,
                                  const float* d_g_weights, const float* d_g_depth, const float* d_g_entropy,
                                  const float* d_g_normal, float* d_graw, void* stream) {
    NERF_REQUIRE(n_rays >= 0 && n_samples >= 1 && n_samples <= 512, "composite_bwd: R=%lld S=%d (S must be 1..512)",
                 (long long)n_rays, n_samples);
    NERF_REQUIRE(raw_channels == 4 || raw_channels == 7, "composite_bwd: raw_channels %d", raw_channels);
    NERF_REQUIRE(n_rays == 0 || (d_raw && d_z && d_rays_d && d_graw), "composite_bwd: null arg");
    if (n_rays == 0) return NERF_OK;
    CompositeArgs a{};
    a.raw = d_raw; a.C = raw_channels; a.z = d_z; a.rays_d = d_rays_d; a.noise = d_noise;
    a.R = n_rays; a.S = n_samples; a.white = white_bkgd;
    a.g_rgb = d_g_rgb; a.g_disp = d_g_disp; a.g_acc = d_g_acc; a.g_w = d_g_weights; a.g_depth = d_g_depth;
    a.g_ent = d_g_entropy; a.g_normal = d_g_normal; a.graw = d_graw;
    dim3 grid(blocks_for(n_rays, 4));
    NERF_COMPOSITE_DISPATCH(composite_bwd_kernel, n_samples, grid, as_stream(stream), a);
    NERF_CHECK_LAUNCH("composite_bwd");
    return NERF_OK;
}
