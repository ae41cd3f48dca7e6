// Fused RAdam step (PocketNeRF/radam.py:28-94) over a list of tensor segments in ONE launch, and
// the total-variation loss on one hashed cuboid per level (PocketNeRF/loss.py:11-43).
#include "hash_common.h"

namespace nerf {

constexpr int kMaxSegs = 32;
constexpr int kRAdamVec = 4;
constexpr int kRAdamThreads = 256;

struct RAdamSegs {
    nerf_radam_segment seg[kMaxSegs];
    const float* coef;   // optional device [n][4] = (decay_coef, step_coef, mode, 0) of this step
    int64_t block_start[kMaxSegs + 1];   // first block of each segment
    int n;
};

// radam_elem (the elementwise update, in the reference's op order): hash_common.h

__global__ void __launch_bounds__(kRAdamThreads) radam_kernel(RAdamSegs S) {
    const int64_t b = blockIdx.x;
    int si = 0;
    while (si + 1 < S.n && b >= S.block_start[si + 1]) ++si;
    nerf_radam_segment s = S.seg[si];
    if (S.coef) {   // per-step scalars from device memory (graph replays)
        s.decay_coef = S.coef[4 * si];
        s.step_coef = S.coef[4 * si + 1];
        s.mode = (int)S.coef[4 * si + 2];
    }
    const int64_t i0 = ((b - S.block_start[si]) * kRAdamThreads + threadIdx.x) * kRAdamVec;
    if (i0 >= s.n) return;
    const float gs = s.grad_scale != 0.f ? s.grad_scale : 1.f;   // g * 1 == g bit for bit
    const bool aligned = ((reinterpret_cast<uintptr_t>(s.p) | reinterpret_cast<uintptr_t>(s.g) |
                           reinterpret_cast<uintptr_t>(s.m) | reinterpret_cast<uintptr_t>(s.v)) & 15) == 0;
    if (aligned && i0 + kRAdamVec <= s.n) {
        float4 p = *reinterpret_cast<const float4*>(s.p + i0);
        float4 g = *reinterpret_cast<const float4*>(s.g + i0);
        g.x *= gs; g.y *= gs; g.z *= gs; g.w *= gs;
        float4 m = *reinterpret_cast<const float4*>(s.m + i0);
        float4 v = *reinterpret_cast<const float4*>(s.v + i0);
        radam_elem(s, p.x, g.x, m.x, v.x);
        radam_elem(s, p.y, g.y, m.y, v.y);
        radam_elem(s, p.z, g.z, m.z, v.z);
        radam_elem(s, p.w, g.w, m.w, v.w);
        *reinterpret_cast<float4*>(s.m + i0) = m;
        *reinterpret_cast<float4*>(s.v + i0) = v;
        if (s.mode != 0) *reinterpret_cast<float4*>(s.p + i0) = p;
    } else {
        for (int64_t i = i0; i < i0 + kRAdamVec && i < s.n; ++i) {
            float p = s.p[i], m = s.m[i], v = s.v[i];
            radam_elem(s, p, s.g[i] * gs, m, v);
            s.m[i] = m;
            s.v[i] = v;
            if (s.mode != 0) s.p[i] = p;
        }
    }
}

// ---------------------------------------------------------------- TV loss
// Grid (kTVBlocks, L): block (b, l) strides over level l's (cube+1)^3 vertices, so a level's partial
// sums meet in one LDS reduction per block and one atomic per block (the atomics of one level
// serialise at its address: a one-vertex-per-thread grid of ~2,300 blocks took 41 instead of 21 us).
// tv_fwd issues the gathers of up to kTVUnroll of a thread's vertices before the first add (the
// finest levels' 51^3 cuboids are ~5.4 vertices per thread: one round trip instead of five).
constexpr uint32_t kTVSkip = 0xFFFFFFFFu;

__global__ void __launch_bounds__(256) tv_fwd_kernel(TVParams P) {
    tv_fwd_block(P, blockIdx.y, blockIdx.x, gridDim.x);
}

__global__ void __launch_bounds__(256) tv_bwd_kernel(TVParams P) {
    const int l = blockIdx.y;
    const int c = P.cube[l], n1 = c + 1;
    const uint32_t nv = (uint32_t)(P.vstart[l + 1] - P.vstart[l]);
    const float2* tab = reinterpret_cast<const float2*>(P.tables[l]);
    int mvd[3];
    tv_corner(P, l, mvd);
    const int* mv = mvd;
    float* dt = P.dtables[l];
    const float s = P.scale[l] / (float)c;
    const int lane = threadIdx.x & 63;
    // uniform trip count per wave (the re-issue below shuffles across the wave)
    for (uint32_t base = blockIdx.x * 256u + (threadIdx.x & ~63u); base < nv; base += gridDim.x * 256u) {
        const uint32_t lv = base + lane;
        const bool ok = lv < nv;
        int i = 0, j = 0, k = 0;
        if (ok) tv_vertex(lv, n1, i, j, k);
        const float2 e = ok ? tv_fetch(tab, mv, i, j, k, P.mask) : make_float2(0.f, 0.f);
        float gx = 0.f, gy = 0.f;   // sum over pairs of d/de_v of (e_hi - e_lo)^2
#define NERF_TV_PAIR(cond, di, dj, dk)                                           \
        if (ok && (cond)) {                                                              \
            const float2 f = tv_fetch(tab, mv, i + (di), j + (dj), k + (dk), P.mask); \
            gx += 2.0f * (e.x - f.x);                                            \
            gy += 2.0f * (e.y - f.y);                                            \
        }
        NERF_TV_PAIR(i > 0, -1, 0, 0)
        NERF_TV_PAIR(i < c, 1, 0, 0)
        NERF_TV_PAIR(j > 0, 0, -1, 0)
        NERF_TV_PAIR(j < c, 0, 1, 0)
        NERF_TV_PAIR(k > 0, 0, 0, -1)
        NERF_TV_PAIR(k < c, 0, 0, 1)
#undef NERF_TV_PAIR
        const uint32_t h = ok ? spatial_hash3((uint32_t)(mv[0] + i), (uint32_t)(mv[1] + j), (uint32_t)(mv[2] + k), P.mask)
                              : kTVSkip;
        // Re-issue so that lanes (2t, 2t+1) add vertex t's two features: one 8-B row per lane pair,
        // one memory-side atomic request instead of two.
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int src = 32 * r + (lane >> 1);
            const uint32_t hs = (uint32_t)__shfl((int)h, src, 64);
            const float vx = __shfl(gx, src, 64), vy = __shfl(gy, src, 64);
            const float v = (lane & 1) ? vy : vx;
            if (hs != kTVSkip) __hip_atomic_fetch_add(dt + 2 * hs + (lane & 1), v * s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}


}  // namespace nerf

using namespace nerf;

extern "C" int nerf_radam_step(const nerf_radam_segment* segs, int n_segs, const float* d_coef, void* stream) {
    NERF_REQUIRE(segs && n_segs >= 0 && n_segs <= kMaxSegs, "radam_step: n_segs %d (max %d)", n_segs, kMaxSegs);
    RAdamSegs S{};
    S.n = 0;
    S.coef = d_coef;
    int64_t blocks = 0;
    for (int i = 0; i < n_segs; ++i) {
        NERF_REQUIRE(!d_coef || segs[i].n > 0, "radam_step: empty segment %d with device coefficients", i);
        if (segs[i].n <= 0) continue;
        NERF_REQUIRE(segs[i].p && segs[i].g && segs[i].m && segs[i].v, "radam_step: segment %d has a null pointer", i);
        NERF_REQUIRE(segs[i].mode >= 0 && segs[i].mode <= 2, "radam_step: segment %d mode %d", i, segs[i].mode);
        S.seg[S.n] = segs[i];
        S.block_start[S.n] = blocks;
        blocks += (segs[i].n + (int64_t)kRAdamThreads * kRAdamVec - 1) / ((int64_t)kRAdamThreads * kRAdamVec);
        S.n++;
    }
    S.block_start[S.n] = blocks;
    if (blocks == 0) return NERF_OK;
    hipLaunchKernelGGL(radam_kernel, dim3((unsigned)blocks), dim3(kRAdamThreads), 0, as_stream(stream), S);
    NERF_CHECK_LAUNCH("radam_step");
    return NERF_OK;
}

extern "C" int nerf_tv_fwd(const float* const* d_tables, int n_levels, int log2_T, const int64_t* min_vertex,
                           const int64_t* d_min_vertex, const int* cube, float* d_loss, float* d_verts,
                           void* stream) {
    TVParams P{};
    int rc = fill_tv(P, n_levels, log2_T, min_vertex, d_min_vertex, cube);
    if (rc) return rc;
    NERF_REQUIRE(d_tables && d_loss, "tv_fwd: null arg");
    for (int l = 0; l < n_levels; ++l) {
        NERF_REQUIRE(d_tables[l], "tv_fwd: table %d null", l);
        P.tables[l] = d_tables[l];
    }
    P.loss = d_loss;
    P.verts = reinterpret_cast<float2*>(d_verts);
    hipLaunchKernelGGL(tv_fwd_kernel, dim3(kTVBlocks, n_levels), dim3(256), 0, as_stream(stream), P);
    NERF_CHECK_LAUNCH("tv_fwd");
    return NERF_OK;
}

extern "C" int nerf_tv_bwd(const float* const* d_tables, int n_levels, int log2_T, const int64_t* min_vertex,
                           const int64_t* d_min_vertex, const int* cube, const float* d_scale,
                           float* const* d_dtables, void* stream) {
    TVParams P{};
    int rc = fill_tv(P, n_levels, log2_T, min_vertex, d_min_vertex, cube);
    if (rc) return rc;
    NERF_REQUIRE(d_tables && d_dtables && d_scale, "tv_bwd: null arg");
    for (int l = 0; l < n_levels; ++l) {
        NERF_REQUIRE(d_tables[l] && d_dtables[l], "tv_bwd: table %d null", l);
        P.tables[l] = d_tables[l];
        P.dtables[l] = d_dtables[l];
    }
    P.scale = d_scale;
    hipLaunchKernelGGL(tv_bwd_kernel, dim3(kTVBlocks, n_levels), dim3(256), 0, as_stream(stream), P);
    NERF_CHECK_LAUNCH("tv_bwd");
    return NERF_OK;
}
