// Volume compositing (raw2outputs, PocketNeRF/run_nerf.py:347-411): the per-ray device code shared by
// the compositing kernels (composite.hip) and the coarse pass's composite + hierarchical-sampling
// launch (sampling.hip composite_sample_fine_kernel).
//
// One wavefront per ray; lane L owns the K = ceil(S/64) consecutive samples [K*L, K*L+K). The
// transmittance T_j = prod_{k<j}(1 - alpha_k + 1e-10) is a wave-level exclusive product scan over
// the lanes' local products (DPP lane moves: common.h wave_excl_prod_dpp). Scans and ray sums run in
// fp64: the reference's CPU cumprod/cumsum accumulate in double.
// Quirks kept: last delta = 1e10, +1e-10 inside the product, NaN depth when sum(w) == 0,
// disp = 1/max(1e-10, depth) (NaN propagates), Categorical entropy over [w, max(1-sum w, 1e-6)].
#pragma once
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

// The forward of one ray (the wave's): per-ray outputs from lane 0, weights [R,S]; w_lds (optional,
// this wave's LDS row of >= 64*K floats) receives the weights too, for a sampler in the same launch.
template <int K>
__device__ __forceinline__ void composite_fwd_ray(const CompositeArgs& a, int64_t ray, int lane, float* w_lds) {
    RayState<K> st;
    float norm_d;
    ray_forward<K>(a, ray, lane, st, norm_d);
    const RaySums s = ray_sums<K>(a, st, a.entropy != nullptr);
#pragma unroll
    for (int q = 0; q < K; ++q) {
        const int j = lane * K + q;
        if (j < a.S) {
            a.weights[ray * a.S + j] = st.w[q];
            if (w_lds) w_lds[j] = st.w[q];
        }
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

}  // namespace nerf
