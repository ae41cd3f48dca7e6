// Ray sampling of render_rays: stratified depths (PocketNeRF/run_nerf.py:466-490) and the
// hierarchical step (run_nerf.py:508-513 + sample_pdf, run_nerf_helpers.py:354-397 + z_std :541).
#include "composite_common.h"
#include "field_common.h"

namespace nerf {

struct StratArgs {
    const float* rays; int64_t stride; int64_t R; int S;
    const float* t; int lindisp; int perturb; const float* u; uint64_t seed, offset;
    const uint64_t* rng;   // optional device (seed, offset): graph replays draw fresh numbers
    float* z; float* pts;
    float* dirs;       // optional [R,3]: the rays' directions (columns 3..5), contiguous
    float* viewdirs;   // optional [R,3]: the rays' view directions (the last three columns)
    float* sh;         // optional [R,16]: SH4 of the view directions (field_common.h sh4_eval)
};

__device__ __forceinline__ float base_depth(float near, float far, float t, int lindisp) {
    if (!lindisp) return near * (1.0f - t) + far * t;
    return 1.0f / ((1.0f / near) * (1.0f - t) + (1.0f / far) * t);
}

__global__ void __launch_bounds__(256) sample_stratified_kernel(StratArgs a) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.R * a.S) return;
    const int64_t r = i / a.S;
    const int j = (int)(i - r * a.S);
    const float* ray = a.rays + r * a.stride;
    const float near = ray[6], far = ray[7];
    float z = base_depth(near, far, a.t[j], a.lindisp);
    if (a.perturb) {
        const float zl = j > 0 ? base_depth(near, far, a.t[j - 1], a.lindisp) : 0.f;
        const float zh = j + 1 < a.S ? base_depth(near, far, a.t[j + 1], a.lindisp) : 0.f;
        const float upper = j + 1 < a.S ? 0.5f * (zh + z) : z;
        const float lower = j > 0 ? 0.5f * (z + zl) : z;
        const float u = a.u ? a.u[i]
                            : (a.rng ? philox_uniform(a.rng[0], a.rng[1], (uint64_t)i)
                                     : philox_uniform(a.seed, a.offset, (uint64_t)i));
        z = lower + (upper - lower) * u;
    }
    a.z[i] = z;
    if (j == 0) {   // the contiguous per-ray copies render_rays hands to the field and compositing
        if (a.dirs) {
            a.dirs[3 * r + 0] = ray[3]; a.dirs[3 * r + 1] = ray[4]; a.dirs[3 * r + 2] = ray[5];
        }
        if (a.viewdirs) {
            const float* v = ray + a.stride - 3;
            a.viewdirs[3 * r + 0] = v[0]; a.viewdirs[3 * r + 1] = v[1]; a.viewdirs[3 * r + 2] = v[2];
        }
        if (a.sh) {
            const float* v = ray + a.stride - 3;
            float o[16];
            sh4_eval(v[0], v[1], v[2], o);
            float4* dst = reinterpret_cast<float4*>(a.sh + kShRecord * r);
            dst[0] = make_float4(o[0], o[1], o[2], o[3]);
            dst[1] = make_float4(o[4], o[5], o[6], o[7]);
            dst[2] = make_float4(o[8], o[9], o[10], o[11]);
            dst[3] = make_float4(o[12], o[13], o[14], o[15]);
            __bf16* pc = reinterpret_cast<__bf16*>(a.sh + kShRecord * r + 16);   // the MLP's pre-split operand
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const __bf16 p0 = (__bf16)o[k];
                const float r1 = o[k] - (float)p0;
                const __bf16 p1 = (__bf16)r1;
                pc[k] = p0;
                pc[16 + k] = p1;
                pc[32 + k] = (__bf16)(r1 - (float)p1);
            }
        }
    }
    if (a.pts) {
        a.pts[3 * i + 0] = ray[0] + ray[3] * z;
        a.pts[3 * i + 1] = ray[1] + ray[4] * z;
        a.pts[3 * i + 2] = ray[2] + ray[5] * z;
    }
}

// ---------------------------------------------------------------- inverse-CDF sampling
constexpr int kMaxBins = 256;        // coarse samples per ray
constexpr int kMaxMerged = 1024;     // coarse + importance samples per ray

struct PdfArgs {
    // source of bins / weights: either explicit arrays (sample_pdf API) or the coarse z/weights
    const float* bins; int64_t bins_stride;
    const float* w; int64_t w_stride;
    int64_t R; int nb;                 // nb = number of bins (cdf entries)
    int N; int det; const float* t_imp; const float* u; uint64_t seed, offset;
    const uint64_t* rng;   // optional device (seed, offset)
    float* samples;
    // fine mode
    const float* rays; int64_t ray_stride; const float* z; int S;
    float* z_fine; float* pts_fine; float* z_std;
    // optional fine-row maps (coarse-feature reuse): absolute row r*M + rank of coarse
    // sample i ([R,S]) and of the k-th importance sample in emission order ([R,N]); the importance
    // samples' points in that order ([R,N,3]); perm [R*M]: fine row -> its position in the
    // importance-first order (importance k of ray r -> r*N + k, coarse i -> R*N + r*S + i)
    int32_t* coarse_rows; int32_t* imp_rows; float* imp_pts; int32_t* perm;
};

// Build the CDF of weights (+1e-5, normalised, cumsum in fp64 as the CPU reference does) in LDS and
// invert it for the wave's ray. bins_l / cdf_l are this wave's LDS slices; w_at(i) gives weight i.
template <typename WAt>
__device__ __forceinline__ void build_cdf(int nb, WAt w_at, float* cdf_l, int lane) {
    const int nw = nb - 1;
    // sum of (w + 1e-5)
    double part = 0.0;
    for (int i = lane; i < nw; i += 64) part += (double)(w_at(i) + 1e-5f);
    const float wsum = (float)wave_sum_dpp(part);
    // contiguous chunk per lane for the prefix sum
    const int per = (nw + 63) / 64;
    const int i0 = lane * per;
    double loc = 0.0;
    for (int k = 0; k < per; ++k) {
        const int i = i0 + k;
        if (i < nw) loc += (double)((w_at(i) + 1e-5f) / wsum);
    }
    const double incl = wave_incl_sum_dpp(loc);
    double run = incl - loc;
    for (int k = 0; k < per; ++k) {
        const int i = i0 + k;
        if (i < nw) {
            run += (double)((w_at(i) + 1e-5f) / wsum);
            cdf_l[i + 1] = (float)run;
        }
    }
    if (lane == 0) cdf_l[0] = 0.0f;
}

__device__ __forceinline__ float invert_cdf(const float* cdf_l, const float* bins_l, int nb, float u) {
    // searchsorted(cdf, u, right=True): first index with cdf > u
    int lo = 0, hi = nb;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cdf_l[mid] <= u) lo = mid + 1; else hi = mid;
    }
    const int below = max(lo - 1, 0);
    const int above = min(lo, nb - 1);
    const float c0 = cdf_l[below], c1 = cdf_l[above];
    const float b0 = bins_l[below], b1 = bins_l[above];
    float denom = c1 - c0;
    if (denom < 1e-5f) denom = 1.0f;
    const float t = (u - c0) / denom;
    return b0 + t * (b1 - b0);
}

__device__ __forceinline__ float draw_u(const PdfArgs& a, int64_t r, int k) {
    if (a.det) return a.t_imp[k];
    const int64_t idx = r * a.N + k;
    if (a.u) return a.u[idx];
    return a.rng ? philox_uniform(a.rng[0], a.rng[1], (uint64_t)idx) : philox_uniform(a.seed, a.offset, (uint64_t)idx);
}

__global__ void __launch_bounds__(256) sample_pdf_kernel(PdfArgs a) {
    __shared__ float s_cdf[4][kMaxBins];
    __shared__ float s_bins[4][kMaxBins];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + wv;
    if (r >= a.R) return;
    float* cdf_l = s_cdf[wv];
    float* bins_l = s_bins[wv];
    const float* br = a.bins + r * a.bins_stride;
    const float* wr = a.w + r * a.w_stride;
    for (int i = lane; i < a.nb; i += 64) bins_l[i] = br[i];
    build_cdf(a.nb, [&](int i) { return wr[i]; }, cdf_l, lane);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    for (int k = lane; k < a.N; k += 64)
        a.samples[r * a.N + k] = invert_cdf(cdf_l, bins_l, a.nb, draw_u(a, r, k));
}

// Fine-pass sampler of ray r (the wave's): z_mid bins, weights[...,1:-1], importance samples,
// rank-sort merge, points. w_at(i) gives coarse weight i; cdf_l / bins_l / all_l are the wave's LDS rows.
template <typename WAt>
__device__ __forceinline__ void sample_fine_ray(const PdfArgs& a, int64_t r, int lane, WAt w_at, float* cdf_l,
                                                float* bins_l, float* all_l) {
    const int S = a.S, N = a.N, M = S + N, nb = S - 1;
    const float* zr = a.z + r * S;
    for (int i = lane; i < S; i += 64) {
        const float zi = zr[i];
        all_l[i] = zi;
        if (i + 1 < S) bins_l[i] = 0.5f * (zr[i + 1] + zi);      // .5 * (z[1:] + z[:-1])
    }
    build_cdf(nb, [&](int i) { return w_at(i + 1); }, cdf_l, lane);   // weights[..., 1:-1]
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    double sum = 0.0;
    for (int k = lane; k < N; k += 64) {
        const float s = invert_cdf(cdf_l, bins_l, nb, draw_u(a, r, k));
        all_l[S + k] = s;
        if (a.samples) a.samples[r * N + k] = s;
        sum += (double)s;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (a.z_std) {
        const double mean = wave_sum_dpp(sum) / (double)N;
        double ss = 0.0;
        for (int k = lane; k < N; k += 64) {
            const double d = (double)all_l[S + k] - mean;
            ss += d * d;
        }
        ss = wave_sum_dpp(ss);
        if (lane == 0) a.z_std[r] = (float)sqrt(ss / (double)N);
    }
    const float* ray = a.rays + r * a.ray_stride;
    const float ox = ray[0], oy = ray[1], oz = ray[2], dx = ray[3], dy = ray[4], dz = ray[5];
    // writes merged position `rank` of the ray, returns its absolute row r*M + rank
    auto put = [&](int rank, float v) {
        const int64_t o = r * M + rank;
        a.z_fine[o] = v;
        if (a.pts_fine) {
            a.pts_fine[3 * o + 0] = ox + dx * v;
            a.pts_fine[3 * o + 1] = oy + dy * v;
            a.pts_fine[3 * o + 2] = oz + dz * v;
        }
        return o;
    };
    // importance sample k of the ray at fine row o: the row maps and its point (same ops as pts_fine)
    auto imp = [&](int k, int64_t o, float v) {
        const int64_t q = r * N + k;
        if (a.imp_rows) a.imp_rows[q] = (int32_t)o;
        if (a.perm) a.perm[o] = (int32_t)q;
        if (a.imp_pts) {
            a.imp_pts[3 * q + 0] = ox + dx * v;
            a.imp_pts[3 * q + 1] = oy + dy * v;
            a.imp_pts[3 * q + 2] = oz + dz * v;
        }
    };
    // torch.sort(cat(z_vals, z_samples)) (run_nerf.py:573). The stratified coarse depths are already
    // ascending; the importance samples are sorted in place (bitonic, padded with +inf to a power of
    // two in the LDS row after them) and the two runs merged by rank: rank = own index + the count of
    // the other run below it (binary search; coarse first on ties). Sorted output values do not depend
    // on how ties are ordered, so this equals the rank sort below, which remains for unsorted coarse
    // depths (callers passing their own z).
    bool coarse_sorted = true;
    for (int i = lane; i + 1 < S; i += 64) coarse_sorted &= !(all_l[i + 1] < all_l[i]);   // the LDS copy: no reload
    int P2 = 1;
    while (P2 < N) P2 <<= 1;
    if (__ballot(!coarse_sorted) == 0ull && S + P2 <= kMaxMerged) {
        float* f = all_l + S;
        if (P2 <= 128) {
            // in registers: element e = lane + 64 h (h < P2 / 64; below 64 elements the lanes past P2 hold
            // +inf); partners across lanes through __shfl_xor, across h in the lane itself. Lower index of
            // a pair keeps the min in an ascending block, the max in a descending one (== the swap below)
            float v[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int e = lane + 64 * h;
                v[h] = e < N ? f[e] : INFINITY;
            }
            const int H = P2 > 64 ? 2 : 1;
            for (int k = 2; k <= P2; k <<= 1) {
                for (int j = k >> 1; j > 0; j >>= 1) {
                    if (j == 64) {   // k == 128: the whole run ascends; lower = h 0
                        const float a = fminf(v[0], v[1]), b = fmaxf(v[0], v[1]);
                        v[0] = a;
                        v[1] = b;
                        continue;
                    }
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        if (h >= H) break;
                        const int e = lane + 64 * h;
                        const float y = __shfl_xor(v[h], j, 64);
                        const bool lower = (lane & j) == 0, up = (e & k) == 0;
                        v[h] = (lower == up) ? fminf(v[h], y) : fmaxf(v[h], y);
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
            for (int h = 0; h < 2; ++h)
                if (h < H && lane + 64 * h < P2) f[lane + 64 * h] = v[h];
        } else {
            for (int i = N + lane; i < P2; i += 64) f[i] = INFINITY;
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            for (int k = 2; k <= P2; k <<= 1) {
                for (int j = k >> 1; j > 0; j >>= 1) {
                    for (int i = lane; i < P2; i += 64) {
                        const int l = i ^ j;
                        if (l > i) {
                            const float x = f[i], y = f[l];
                            const bool up = (i & k) == 0;
                            if (up ? (y < x) : (x < y)) { f[i] = y; f[l] = x; }
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        // coarse i: i + #{fine < v}; fine j: j + #{coarse <= v}
        for (int i = lane; i < S; i += 64) {
            const float v = all_l[i];
            int lo = 0, hi = N;
            while (lo < hi) { const int mid = (lo + hi) >> 1; if (f[mid] < v) lo = mid + 1; else hi = mid; }
            const int64_t o = put(i + lo, v);
            if (a.coarse_rows) a.coarse_rows[r * S + i] = (int32_t)o;
            if (a.perm) a.perm[o] = (int32_t)(a.R * N + r * S + i);
        }
        for (int j = lane; j < N; j += 64) {
            const float v = f[j];
            int lo = 0, hi = S;
            while (lo < hi) { const int mid = (lo + hi) >> 1; if (all_l[mid] <= v) lo = mid + 1; else hi = mid; }
            const int64_t o = put(j + lo, v);
            imp(j, o, v);   // ascending along the ray
        }
        return;
    }
    // rank sort (ties broken by position): out[rank(e)] = v_e
    for (int e = lane; e < M; e += 64) {
        const float v = all_l[e];
        int rank = 0;
        for (int i = 0; i < M; ++i) {
            const float w = all_l[i];
            rank += (w < v) || (w == v && i < e);
        }
        const int64_t o = put(rank, v);
        if (e < S) {
            if (a.coarse_rows) a.coarse_rows[r * S + e] = (int32_t)o;
            if (a.perm) a.perm[o] = (int32_t)(a.R * N + r * S + e);
        } else {
            imp(e - S, o, v);
        }
    }
}

__global__ void __launch_bounds__(256) sample_fine_kernel(PdfArgs a) {
    __shared__ float s_cdf[4][kMaxBins];
    __shared__ float s_bins[4][kMaxBins];
    __shared__ float s_all[4][kMaxMerged];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + wv;
    if (r >= a.R) return;
    const float* wr = a.w + r * a.S;
    sample_fine_ray(a, r, lane, [&](int i) { return wr[i]; }, s_cdf[wv], s_bins[wv], s_all[wv]);
}

// The coarse pass's compositing (composite_common.h) and the hierarchical sampler in one launch: the
// wave composites its ray, keeps the weights in LDS (they also go to c.weights) and samples from
// them — the same values the separate launches pass through HBM, so every output is bit-identical.
template <int K>
__global__ void __launch_bounds__(256) composite_sample_fine_kernel(CompositeArgs c, PdfArgs a) {
    __shared__ float s_cdf[4][kMaxBins];
    __shared__ float s_bins[4][kMaxBins];
    __shared__ float s_all[4][kMaxMerged];
    __shared__ float s_w[4][64 * K];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * 4 + wv;
    if (r >= a.R) return;   // wave-uniform
    float* w_l = s_w[wv];
    composite_fwd_ray<K>(c, r, lane, w_l);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    sample_fine_ray(a, r, lane, [&](int i) { return w_l[i]; }, s_cdf[wv], s_bins[wv], s_all[wv]);
}

}  // namespace nerf

using namespace nerf;

extern "C" int nerf_sample_stratified(const float* d_rays, int64_t ray_stride, int64_t n_rays, int n_samples,
                                      const float* d_t, int lindisp, int perturb, const float* d_u, uint64_t seed,
                                      uint64_t offset, const uint64_t* d_rng, float* d_z, float* d_pts,
                                      float* d_dirs, float* d_viewdirs, void* stream) {
    return nerf_sample_stratified_sh(d_rays, ray_stride, n_rays, n_samples, d_t, lindisp, perturb, d_u, seed, offset,
                                     d_rng, d_z, d_pts, d_dirs, d_viewdirs, nullptr, stream);
}

extern "C" int nerf_sample_stratified_sh(const float* d_rays, int64_t ray_stride, int64_t n_rays, int n_samples,
                                         const float* d_t, int lindisp, int perturb, const float* d_u, uint64_t seed,
                                         uint64_t offset, const uint64_t* d_rng, float* d_z, float* d_pts,
                                         float* d_dirs, float* d_viewdirs, float* d_sh, void* stream) {
    NERF_REQUIRE(n_rays >= 0 && n_samples >= 1, "sample_stratified: R=%lld S=%d", (long long)n_rays, n_samples);
    NERF_REQUIRE(ray_stride >= 8, "sample_stratified: ray_stride %lld < 8", (long long)ray_stride);
    if (n_rays == 0) return NERF_OK;   // empty batches: nothing is read or written (NULL data allowed)
    NERF_REQUIRE(d_rays && d_t && d_z, "sample_stratified: null arg");
    NERF_REQUIRE(!d_viewdirs || ray_stride > 8, "sample_stratified: viewdirs need ray_stride > 8 (got %lld)",
                 (long long)ray_stride);
    NERF_REQUIRE(!d_sh || (ray_stride > 8 && ((uintptr_t)d_sh & 15) == 0),
                 "sample_stratified: SH rows need ray_stride > 8 and 16-B alignment");
    StratArgs a{d_rays, ray_stride, n_rays, n_samples, d_t, lindisp, perturb, d_u, seed, offset, d_rng, d_z, d_pts,
                d_dirs, d_viewdirs, d_sh};
    hipLaunchKernelGGL(sample_stratified_kernel, dim3(blocks_for(n_rays * n_samples, 256)), dim3(256), 0,
                       as_stream(stream), a);
    NERF_CHECK_LAUNCH("sample_stratified");
    return NERF_OK;
}

extern "C" int nerf_sample_pdf(const float* d_bins, int64_t bins_stride, const float* d_weights,
                               int64_t weights_stride, int64_t n_rays, int n_bins, int n_importance, int det,
                               const float* d_t_imp, const float* d_u, uint64_t seed, uint64_t offset,
                               const uint64_t* d_rng, float* d_samples, void* stream) {
    NERF_REQUIRE(n_rays >= 0 && n_bins >= 2 && n_bins <= kMaxBins && n_importance >= 1,
                 "sample_pdf: R=%lld bins=%d N=%d (bins must be 2..%d)", (long long)n_rays, n_bins, n_importance,
                 kMaxBins);
    if (n_rays == 0) return NERF_OK;
    NERF_REQUIRE(d_bins && d_weights && d_samples && (!det || d_t_imp), "sample_pdf: null arg");
    PdfArgs a{};
    a.bins = d_bins; a.bins_stride = bins_stride; a.w = d_weights; a.w_stride = weights_stride;
    a.R = n_rays; a.nb = n_bins; a.N = n_importance; a.det = det; a.t_imp = d_t_imp; a.u = d_u;
    a.seed = seed; a.offset = offset; a.rng = d_rng; a.samples = d_samples;
    hipLaunchKernelGGL(sample_pdf_kernel, dim3(blocks_for(n_rays, 4)), dim3(256), 0, as_stream(stream), a);
    NERF_CHECK_LAUNCH("sample_pdf");
    return NERF_OK;
}

extern "C" int nerf_sample_fine_rows(const float* d_rays, int64_t ray_stride, const float* d_z, const float* d_weights,
                                     int64_t n_rays, int n_samples, int n_importance, int det, const float* d_t_imp,
                                     const float* d_u, uint64_t seed, uint64_t offset, const uint64_t* d_rng,
                                     float* d_z_fine, float* d_pts_fine, float* d_z_std, float* d_samples,
                                     int32_t* d_coarse_rows, int32_t* d_imp_rows, float* d_imp_pts, int32_t* d_perm,
                                     void* stream) {
    NERF_REQUIRE(n_rays >= 0 && n_samples >= 3 && n_samples <= kMaxBins && n_importance >= 1 &&
                     n_samples + n_importance <= kMaxMerged,
                 "sample_fine: R=%lld S=%d N=%d (S in 3..%d, S+N <= %d)", (long long)n_rays, n_samples,
                 n_importance, kMaxBins, kMaxMerged);
    NERF_REQUIRE(ray_stride >= 6, "sample_fine: ray_stride %lld < 6", (long long)ray_stride);
    NERF_REQUIRE((!d_coarse_rows && !d_imp_rows && !d_perm) || n_rays * (int64_t)(n_samples + n_importance) <= INT32_MAX,
                 "sample_fine: %lld fine rows do not fit the int32 row maps",
                 (long long)(n_rays * (int64_t)(n_samples + n_importance)));
    if (n_rays == 0) return NERF_OK;
    NERF_REQUIRE(d_rays && d_z && d_weights && d_z_fine && (!det || d_t_imp), "sample_fine: null arg");
    PdfArgs a{};
    a.R = n_rays; a.N = n_importance; a.det = det; a.t_imp = d_t_imp; a.u = d_u; a.seed = seed; a.offset = offset;
    a.rng = d_rng;
    a.samples = d_samples; a.rays = d_rays; a.ray_stride = ray_stride; a.z = d_z; a.w = d_weights; a.S = n_samples;
    a.z_fine = d_z_fine; a.pts_fine = d_pts_fine; a.z_std = d_z_std;
    a.coarse_rows = d_coarse_rows; a.imp_rows = d_imp_rows; a.imp_pts = d_imp_pts; a.perm = d_perm;
    hipLaunchKernelGGL(sample_fine_kernel, dim3(blocks_for(n_rays, 4)), dim3(256), 0, as_stream(stream), a);
    NERF_CHECK_LAUNCH("sample_fine");
    return NERF_OK;
}

extern "C" int nerf_composite_sample_fine(
    const float* d_raw, int raw_channels, const float* d_z, const float* d_rays_d, const float* d_noise, int64_t n_rays,
    int n_samples, int white_bkgd, float* d_rgb, float* d_disp, float* d_acc, float* d_weights, float* d_depth,
    float* d_entropy, float* d_normal, const float* d_rays, int64_t ray_stride, int n_importance, int det,
    const float* d_t_imp, const float* d_u, uint64_t seed, uint64_t offset, const uint64_t* d_rng, float* d_z_fine,
    float* d_pts_fine, float* d_z_std, float* d_samples, int32_t* d_coarse_rows, int32_t* d_imp_rows,
    float* d_imp_pts, int32_t* d_perm, void* stream) {
    const int K = (n_samples + 63) / 64;
    if (n_rays == 0 || K > 2 || n_samples < 3 || n_samples > kMaxBins) {
        // the two launches (their own checks and messages); one launch covers K = 1, 2
        int rc = nerf_composite_fwd(d_raw, raw_channels, d_z, d_rays_d, d_noise, n_rays, n_samples, white_bkgd, d_rgb,
                                    d_disp, d_acc, d_weights, d_depth, d_entropy, d_normal, stream);
        if (rc != NERF_OK) return rc;
        return nerf_sample_fine_rows(d_rays, ray_stride, d_z, d_weights, n_rays, n_samples, n_importance, det, d_t_imp,
                                     d_u, seed, offset, d_rng, d_z_fine, d_pts_fine, d_z_std, d_samples, d_coarse_rows,
                                     d_imp_rows, d_imp_pts, d_perm, stream);
    }
    NERF_REQUIRE(raw_channels == 4 || raw_channels == 7, "composite_sample_fine: raw_channels %d", raw_channels);
    NERF_REQUIRE(d_raw && d_z && d_rays_d && d_weights, "composite_sample_fine: null compositing arg");
    NERF_REQUIRE(!(d_normal && raw_channels != 7), "composite_sample_fine: normal output needs 7 raw channels");
    NERF_REQUIRE(n_importance >= 1 && n_samples + n_importance <= kMaxMerged,
                 "composite_sample_fine: S=%d N=%d (S+N <= %d)", n_samples, n_importance, kMaxMerged);
    NERF_REQUIRE(ray_stride >= 6, "composite_sample_fine: ray_stride %lld < 6", (long long)ray_stride);
    NERF_REQUIRE((!d_coarse_rows && !d_imp_rows && !d_perm) || n_rays * (int64_t)(n_samples + n_importance) <= INT32_MAX,
                 "composite_sample_fine: %lld fine rows do not fit the int32 row maps",
                 (long long)(n_rays * (int64_t)(n_samples + n_importance)));
    NERF_REQUIRE(d_rays && d_z_fine && (!det || d_t_imp), "composite_sample_fine: null sampling arg");
    CompositeArgs c{};
    c.raw = d_raw; c.C = raw_channels; c.z = d_z; c.rays_d = d_rays_d; c.noise = d_noise;
    c.R = n_rays; c.S = n_samples; c.white = white_bkgd;
    c.rgb = d_rgb; c.disp = d_disp; c.acc = d_acc; c.weights = d_weights; c.depth = d_depth;
    c.entropy = d_entropy; c.normal = d_normal;
    PdfArgs a{};
    a.R = n_rays; a.N = n_importance; a.det = det; a.t_imp = d_t_imp; a.u = d_u; a.seed = seed; a.offset = offset;
    a.rng = d_rng;
    a.samples = d_samples; a.rays = d_rays; a.ray_stride = ray_stride; a.z = d_z; a.w = d_weights; a.S = n_samples;
    a.z_fine = d_z_fine; a.pts_fine = d_pts_fine; a.z_std = d_z_std;
    a.coarse_rows = d_coarse_rows; a.imp_rows = d_imp_rows; a.imp_pts = d_imp_pts; a.perm = d_perm;
    const dim3 grid(blocks_for(n_rays, 4));
    if (K == 1)
        hipLaunchKernelGGL(composite_sample_fine_kernel<1>, grid, dim3(256), 0, as_stream(stream), c, a);
    else
        hipLaunchKernelGGL(composite_sample_fine_kernel<2>, grid, dim3(256), 0, as_stream(stream), c, a);
    NERF_CHECK_LAUNCH("composite_sample_fine");
    return NERF_OK;
}

extern "C" int nerf_sample_fine(const float* d_rays, int64_t ray_stride, const float* d_z, const float* d_weights,
                                int64_t n_rays, int n_samples, int n_importance, int det, const float* d_t_imp,
                                const float* d_u, uint64_t seed, uint64_t offset, const uint64_t* d_rng,
                                float* d_z_fine, float* d_pts_fine, float* d_z_std, float* d_samples, void* stream) {
    return nerf_sample_fine_rows(d_rays, ray_stride, d_z, d_weights, n_rays, n_samples, n_importance, det, d_t_imp,
                                 d_u, seed, offset, d_rng, d_z_fine, d_pts_fine, d_z_std, d_samples, nullptr, nullptr,
                                 nullptr, nullptr, stream);
}
