// Structural priors (PocketNeRF/structural_priors.py): the one O(N * Q) step of the loss, the
// spatial nearest neighbour of spatial_normal_consistency_loss (:333-346):
//     distances = torch.cdist(coords[idx1], coords); distances[q, idx1[q]] = inf; idx2 = argmin
// One block per query point: each thread scans a strided slice of the N candidates (squared
// distance in fp32, self excluded), a wave then a block arg-min with the lowest index winning ties
// (torch.argmin's first occurrence), and the winner's distance sqrt(d2). For the integer pixel
// coordinates train() passes (select_coords), d2 is exact, so this equals cdist's mm-based value.
#include "common.h"

namespace nerf {

__global__ void __launch_bounds__(256) nearest_kernel(const float* __restrict__ xy, int64_t n,
                                                      const int64_t* __restrict__ idx1, int64_t* __restrict__ idx2,
                                                      float* __restrict__ dist) {
    const int64_t q = blockIdx.x;
    const int64_t self = idx1[q];
    const float qx = xy[2 * self], qy = xy[2 * self + 1];
    float best = INFINITY;
    int64_t bi = n;   // "no candidate" sorts after every real index
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
        const float dx = xy[2 * i] - qx, dy = xy[2 * i + 1] - qy;
        const float d2 = i == self ? INFINITY : dx * dx + dy * dy;
        if (d2 < best) { best = d2; bi = i; }   // strided ascending scan: first minimum per thread
    }
    for (int o = 32; o > 0; o >>= 1) {
        const float ob = __shfl_xor(best, o, 64);
        const int64_t oi = __shfl_xor(bi, o, 64);
        if (ob < best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    __shared__ float s_b[4];
    __shared__ int64_t s_i[4];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { s_b[w] = best; s_i[w] = bi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < 4; ++k)
            if (s_b[k] < best || (s_b[k] == best && s_i[k] < bi)) { best = s_b[k]; bi = s_i[k]; }
        if (bi >= n) bi = self == 0 ? (n > 1 ? 1 : 0) : 0;   // all candidates infinite: argmin -> index 0 unless self
        idx2[q] = bi;
        dist[q] = sqrtf(best);
    }
}

}  // namespace nerf

using namespace nerf;

extern "C" int nerf_nearest_pixel(const float* d_xy, int64_t n, const int64_t* d_idx1, int64_t n_query,
                                  int64_t* d_idx2, float* d_dist, void* stream) {
    NERF_REQUIRE(n >= 2 && n_query >= 0 && n_query < (1ll << 31), "nearest_pixel: n=%lld queries=%lld",
                 (long long)n, (long long)n_query);
    NERF_REQUIRE(d_xy && d_idx1 && d_idx2 && d_dist, "nearest_pixel: null arg");
    if (n_query == 0) return NERF_OK;
    hipLaunchKernelGGL(nearest_kernel, dim3((unsigned)n_query), dim3(256), 0, as_stream(stream), d_xy, n, d_idx1,
                       d_idx2, d_dist);
    NERF_CHECK_LAUNCH("nearest_pixel");
    return NERF_OK;
}
