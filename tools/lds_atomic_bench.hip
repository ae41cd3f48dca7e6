// Micro-benchmark: LDS atomic throughput on gfx950 (one 1024-thread block per CU, random or
// conflict-free addresses into a 16K-row table). Informs the owner pass of the binned hash
// backward (csrc/hashgrid.hip). Build: hipcc --offload-arch=gfx950 -O3 tools/lds_atomic_bench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

constexpr int kRows = 1 << 14;
constexpr int kIters = 256;

__device__ __forceinline__ uint32_t rnd(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

template <int KIND, bool RANDOM>
__global__ void __launch_bounds__(1024) lds_kernel(float* out) {
    __shared__ __attribute__((aligned(16))) float s[2 * kRows];
    for (int i = threadIdx.x; i < 2 * kRows; i += 1024) s[i] = 0.f;
    __syncthreads();
    uint32_t st = rnd(blockIdx.x * 1024 + threadIdx.x);
    for (int it = 0; it < kIters; ++it) {
        st = rnd(st + it);
        const uint32_t r = RANDOM ? (st & (kRows - 1)) : ((threadIdx.x + it * 1024) & (kRows - 1));
        const float v = (float)(st & 255) * 0.01f;
        if constexpr (KIND == 0) {          // 2 x ds_add_f32 (x, y of a float2 row)
            atomicAdd(&s[2 * r], v);
            atomicAdd(&s[2 * r + 1], v);
        } else if constexpr (KIND == 1) {   // 2 x ds_add_u32
            atomicAdd(reinterpret_cast<uint32_t*>(&s[2 * r]), (uint32_t)st);
            atomicAdd(reinterpret_cast<uint32_t*>(&s[2 * r + 1]), (uint32_t)st);
        } else if constexpr (KIND == 2) {   // 1 x ds_add_f64 on the 8-B row
            atomicAdd(reinterpret_cast<double*>(&s[2 * r]), (double)v);
        } else if constexpr (KIND == 3) {   // plain read-modify-write (racy; cost floor)
            float2* p = reinterpret_cast<float2*>(&s[2 * r]);
            float2 t = *p;
            t.x += v; t.y += v;
            *p = t;
        } else {                            // 2 x ds_add_f32, rows split x/y planes
            atomicAdd(&s[r], v);
            atomicAdd(&s[kRows + r], v);
        }
    }
    __syncthreads();
    float acc = 0.f;
    for (int i = threadIdx.x; i < 2 * kRows; i += 1024) acc += s[i];
    if (acc == 12345.f) out[blockIdx.x] = acc;
}

template <int KIND, bool RANDOM>
static float run(float* d, const char* name) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int w = 0; w < 2; ++w) lds_kernel<KIND, RANDOM><<<256, 1024>>>(d);
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) lds_kernel<KIND, RANDOM><<<256, 1024>>>(d);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    ms /= 5.f;
    const double ops = 256.0 * 1024 * kIters;   // row updates
    printf("{\"kind\": \"%s\", \"random\": %d, \"us\": %.1f, \"row_updates_per_clk_per_cu\": %.3f}\n", name,
           (int)RANDOM, ms * 1e3, ops / (ms * 1e-3) / 256 / 2.4e9);
    return ms;
}

int main() {
    float* d;
    hipMalloc(&d, 1024 * sizeof(float));
    run<0, true>(d, "ds_add_f32 x2");
    run<0, false>(d, "ds_add_f32 x2");
    run<4, true>(d, "ds_add_f32 x2 planar");
    run<1, true>(d, "ds_add_u32 x2");
    run<2, true>(d, "ds_add_f64");
    run<3, true>(d, "plain rmw float2");
    run<3, false>(d, "plain rmw float2");
    hipFree(d);
    return 0;
}
