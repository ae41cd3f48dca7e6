// Active points of a field backward: the points whose upstream gradient row is not all zero.
//
// raw2outputs' autograd (PocketNeRF/run_nerf.py:364-386) gives a sample with relu(sigma + noise) = 0
// (empty space, and every point run_network masks outside the box, run_nerf.py:66) alpha = 0, weight 0
// and a zero sigma gradient, so its whole raw-gradient row is 0 — and so are its MLP weight-gradient
// terms and its hash-feature gradient (NeRFSmall's backward is linear in the upstream gradient). The
// MLP backward and the hash bins can therefore walk only the active points: the same sums, exactly,
// without the zero terms.
//
// Stable compaction in two launches: (1) per block of kBlockPts points, the number of active points
// (and of active ones among the first n_first points); (2) each block sums
// the counts of the blocks before it and writes its active indices in ascending order (wave ballots,
// an LDS scan over the block's waves). Ascending order keeps the samples of a ray adjacent, which the
// hash bins' run merge relies on, and makes the lists (and so every sum over them) deterministic.
#include "common.h"

namespace nerf {

constexpr int kActThreads = 256;
constexpr int kActPer = 16;                          // points per thread
constexpr int kBlockPts = kActThreads * kActPer;     // 4096 points per block

struct ActiveArgs {
    const float* graw;      // [P, 4]
    const float* dgeo;      // optional [P, 16] (normals head: rows 1..15 are the upstream d geo)
    int64_t P;
    const int32_t* graw_rows;   // optional [P]: row of point p in graw / dgeo (the reuse's point order)
    int64_t n_first;        // active points < n_first are counted apart (the list's prefix)
    int32_t* rows;          // out [P]: active points, ascending
    int32_t* counts;        // out [2]: number of active points, of those < n_first
    int32_t* block_counts;  // workspace [2][n_blocks]
    // optional: zero the feature-gradient rows the backward will not write but a bin will read —
    // row p >= n_first of an INACTIVE point p
    float* zero; int64_t zero_sl; int n_levels;
};

__device__ __forceinline__ bool row_active(const ActiveArgs& a, int64_t p) {
    if (a.graw_rows) p = a.graw_rows[p];
    const float4 g = *reinterpret_cast<const float4*>(a.graw + 4 * p);
    bool on = g.x != 0.f || g.y != 0.f || g.z != 0.f || g.w != 0.f;
    if (a.dgeo && !on) {
        const float4* d = reinterpret_cast<const float4*>(a.dgeo + 16 * p);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float4 v = d[k];
            if (k == 0) v.x = 0.f;   // row 0 of d geo is not an input of the field (normals.hip)
            on = on || v.x != 0.f || v.y != 0.f || v.z != 0.f || v.w != 0.f;
        }
    }
    return on;
}

// point k of thread t of block b: b * kBlockPts + k * kActThreads + t (consecutive threads, consecutive points)
__global__ void __launch_bounds__(kActThreads) active_count_kernel(ActiveArgs a) {
    const int64_t base = (int64_t)blockIdx.x * kBlockPts;
    int n0 = 0, n1 = 0;
#pragma unroll 4
    for (int k = 0; k < kActPer; ++k) {
        const int64_t p = base + k * kActThreads + threadIdx.x;
        if (p < a.P && row_active(a, p)) {
            ++n0;
            if (p < a.n_first) ++n1;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        n0 += __shfl_xor(n0, o, 64);
        n1 += __shfl_xor(n1, o, 64);
    }
    __shared__ int s[2][kActThreads / 64];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { s[0][w] = n0; s[1][w] = n1; }
    __syncthreads();
    if (threadIdx.x == 0) {
        int t0 = 0, t1 = 0;
        for (int i = 0; i < kActThreads / 64; ++i) { t0 += s[0][i]; t1 += s[1][i]; }
        a.block_counts[blockIdx.x] = t0;
        a.block_counts[gridDim.x + blockIdx.x] = t1;
    }
}

__global__ void __launch_bounds__(kActThreads) active_scatter_kernel(ActiveArgs a) {
    const int b = blockIdx.x, nb = gridDim.x;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // this block's offsets: the counts of the blocks before it
    int o0 = 0, o1 = 0;
    for (int i = threadIdx.x; i < b; i += kActThreads) {
        o0 += a.block_counts[i];
        o1 += a.block_counts[nb + i];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        o0 += __shfl_xor(o0, o, 64);
        o1 += __shfl_xor(o1, o, 64);
    }
    __shared__ int s_off[2][kActThreads / 64];
    __shared__ int s_cnt[2][kActThreads / 64];
    if (lane == 0) { s_off[0][w] = o0; s_off[1][w] = o1; }
    __syncthreads();
    int base0 = 0, base1 = 0;
    for (int i = 0; i < kActThreads / 64; ++i) { base0 += s_off[0][i]; base1 += s_off[1][i]; }
    __syncthreads();
    const int64_t pbase = (int64_t)b * kBlockPts;
    for (int k = 0; k < kActPer; ++k) {
        const int64_t p = pbase + k * kActThreads + threadIdx.x;
        const bool on = p < a.P && row_active(a, p);
        if (a.zero && p < a.P && !on && p >= a.n_first)
            for (int l = 0; l < a.n_levels; ++l)
                *reinterpret_cast<float2*>(a.zero + 2 * p + l * a.zero_sl) = make_float2(0.f, 0.f);
        const bool on1 = on && p < a.n_first;
        const uint64_t m0 = __ballot(on), m1 = __ballot(on1);
        const uint64_t below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
        if (lane == 0) { s_cnt[0][w] = __popcll(m0); s_cnt[1][w] = __popcll(m1); }
        __syncthreads();
        int w0 = base0;
        for (int i = 0; i < w; ++i) w0 += s_cnt[0][i];
        if (on) a.rows[w0 + __popcll(m0 & below)] = (int32_t)p;
        for (int i = 0; i < kActThreads / 64; ++i) { base0 += s_cnt[0][i]; base1 += s_cnt[1][i]; }
        __syncthreads();
    }
    if (b == nb - 1 && threadIdx.x == 0) {   // the last block knows both totals
        a.counts[0] = base0;
        a.counts[1] = base1;
    }
}

}  // namespace nerf

using namespace nerf;

extern "C" size_t nerf_active_rows_workspace_bytes(int64_t n_points) {
    if (n_points < 0) return 0;
    return (size_t)2 * (size_t)std::max<int64_t>(1, (n_points + kBlockPts - 1) / kBlockPts) * sizeof(int32_t);
}

extern "C" int nerf_active_rows(const float* d_graw, const float* d_dgeo, int64_t n_points,
                                const int32_t* d_graw_rows, int64_t n_first, int32_t* d_rows, int32_t* d_counts,
                                float* d_zero_feat, int64_t zero_stride_level, int n_levels, void* d_workspace,
                                size_t workspace_bytes, void* stream) {
    NERF_REQUIRE(n_points >= 0 && n_points <= INT32_MAX, "active_rows: n_points %lld", (long long)n_points);
    NERF_REQUIRE(d_counts && d_workspace && workspace_bytes >= nerf_active_rows_workspace_bytes(n_points),
                 "active_rows: null counts / workspace, or workspace %zu B < %zu B", workspace_bytes,
                 nerf_active_rows_workspace_bytes(n_points));
    NERF_REQUIRE(n_first >= 0, "active_rows: n_first %lld", (long long)n_first);
    NERF_REQUIRE(!d_zero_feat || (n_levels >= 1 && n_levels <= NERF_MAX_LEVELS && zero_stride_level % 2 == 0 &&
                                  ((uintptr_t)d_zero_feat & 7) == 0),
                 "active_rows: zeroed feature rows need 1..16 levels and 8-B aligned pairs");
    if (n_points == 0) {
        if (hipMemsetAsync(d_counts, 0, 2 * sizeof(int32_t), as_stream(stream)) != hipSuccess) {
            set_error("active_rows: hipMemsetAsync failed");
            return NERF_E_LAUNCH;
        }
        return NERF_OK;
    }
    NERF_REQUIRE(d_graw && d_rows, "active_rows: null arg");
    NERF_REQUIRE(((uintptr_t)d_graw & 15) == 0 && (!d_dgeo || ((uintptr_t)d_dgeo & 15) == 0),
                 "active_rows: graw / dgeo rows must be 16-B aligned");
    ActiveArgs a{d_graw, d_dgeo, n_points, d_graw_rows, n_first, d_rows, d_counts,
                 static_cast<int32_t*>(d_workspace), d_zero_feat, zero_stride_level, n_levels};
    const unsigned nb = blocks_for(n_points, kBlockPts);
    hipLaunchKernelGGL(active_count_kernel, dim3(nb), dim3(kActThreads), 0, as_stream(stream), a);
    hipLaunchKernelGGL(active_scatter_kernel, dim3(nb), dim3(kActThreads), 0, as_stream(stream), a);
    NERF_CHECK_LAUNCH("active_rows");
    return NERF_OK;
}
