// Numerical check of render_rays' outputs (run_nerf.py:545-547: with DEBUG set, every returned
// tensor is tested for NaN/Inf). One launch for all of a call's tensors: block (b, t) scans a
// grid-strided part of tensor t and adds its count of non-finite values to d_counts[t] (integer
// atomics: the counts are exact). The host reads the counts once, only in debug mode.
#include "common.h"

namespace nerf {

struct FiniteArgs {
    const float* ptr[NERF_MAX_CHECK];
    int64_t n[NERF_MAX_CHECK];
};

__global__ void __launch_bounds__(256) count_nonfinite_kernel(FiniteArgs a, int* __restrict__ counts) {
    const int t = blockIdx.y;
    const float* __restrict__ p = a.ptr[t];
    const int64_t n = a.n[t];
    int c = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        c += isfinite(p[i]) ? 0 : 1;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(counts + t, c);
}

}  // namespace nerf

using namespace nerf;

extern "C" int nerf_count_nonfinite(const float* const* d_ptrs, const int64_t* sizes, int n_tensors, int* d_counts,
                                    void* stream) {
    NERF_REQUIRE(n_tensors >= 0 && n_tensors <= NERF_MAX_CHECK, "count_nonfinite: %d tensors (0..%d)", n_tensors,
                 NERF_MAX_CHECK);
    NERF_REQUIRE(n_tensors == 0 || (d_ptrs && sizes && d_counts), "count_nonfinite: null arg");
    if (n_tensors == 0) return NERF_OK;
    FiniteArgs a{};
    int64_t most = 1;
    for (int t = 0; t < n_tensors; ++t) {
        NERF_REQUIRE(sizes[t] >= 0 && (sizes[t] == 0 || d_ptrs[t]), "count_nonfinite: tensor %d", t);
        a.ptr[t] = d_ptrs[t];
        a.n[t] = sizes[t];
        most = sizes[t] > most ? sizes[t] : most;
    }
    const hipError_t e = hipMemsetAsync(d_counts, 0, n_tensors * sizeof(int), as_stream(stream));
    if (e != hipSuccess) {
        set_error("count_nonfinite: hipMemsetAsync: %s", hipGetErrorString(e));
        return NERF_E_LAUNCH;
    }
    const unsigned bx = (unsigned)std::min<int64_t>(blocks_for(most, 256), 1024);
    hipLaunchKernelGGL(count_nonfinite_kernel, dim3(bx, n_tensors), dim3(256), 0, as_stream(stream), a, d_counts);
    NERF_CHECK_LAUNCH("count_nonfinite");
    return NERF_OK;
}
