// Shared device/host helpers for libnerfhip (gfx950, wave64). Not part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>

#include "../../include/nerf_hip.h"

namespace nerf {

// ---------------------------------------------------------------- host-side error reporting
void set_error(const char* fmt, ...);

#define NERF_REQUIRE(cond, ...)                 \
    do {                                        \
        if (!(cond)) {                          \
            ::nerf::set_error(__VA_ARGS__);     \
            return NERF_E_ARG;                  \
        }                                       \
    } while (0)

#define NERF_CHECK_LAUNCH(what)                                                             \
    do {                                                                                    \
        hipError_t e_ = hipGetLastError();                                                  \
        if (e_ != hipSuccess) {                                                             \
            ::nerf::set_error("%s: %s", what, hipGetErrorString(e_));                       \
            return NERF_E_LAUNCH;                                                           \
        }                                                                                   \
    } while (0)

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

constexpr int kWave = 64;

inline unsigned blocks_for(int64_t n, int threads) {
    return (unsigned)((n + threads - 1) / threads);
}

// ---------------------------------------------------------------- device helpers
// Philox4x32-10 (Salmon et al. 2011): counter = (index lo, index hi, offset lo, offset hi),
// key = seed. Returns 4 uniforms in [0,1) with 24-bit resolution.
struct U4 { float x, y, z, w; };

__device__ __forceinline__ uint32_t mulhilo(uint32_t a, uint32_t b, uint32_t& hi) {
    uint64_t p = (uint64_t)a * (uint64_t)b;
    hi = (uint32_t)(p >> 32);
    return (uint32_t)p;
}

__device__ __forceinline__ U4 philox_uniform4(uint64_t seed, uint64_t offset, uint64_t index) {
    uint32_t c0 = (uint32_t)index, c1 = (uint32_t)(index >> 32);
    uint32_t c2 = (uint32_t)offset, c3 = (uint32_t)(offset >> 32);
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint32_t hi0, hi1;
        uint32_t lo0 = mulhilo(0xD2511F53u, c0, hi0);
        uint32_t lo1 = mulhilo(0xCD9E8D57u, c2, hi1);
        uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    const float s = 1.0f / 16777216.0f;
    return U4{(c0 >> 8) * s, (c1 >> 8) * s, (c2 >> 8) * s, (c3 >> 8) * s};
}

__device__ __forceinline__ float philox_uniform(uint64_t seed, uint64_t offset, uint64_t index) {
    U4 u = philox_uniform4(seed, offset, index >> 2);
    switch (index & 3) {
        case 0: return u.x;
        case 1: return u.y;
        case 2: return u.z;
        default: return u.w;
    }
}

// Spatial hash of utils.py:13-24 for 3-D integer corners (uint32 wrap == the reference's int64
// arithmetic modulo the 2^log2_T mask).
__device__ __forceinline__ uint32_t spatial_hash3(uint32_t x, uint32_t y, uint32_t z, uint32_t mask) {
    return (x * 1u ^ y * 2654435761u ^ z * 805459861u) & mask;
}

// DPP lane move (VALU, no LDS crossbar): CTRL 0x110+n = row_shr:n, 0x142 = row_bcast:15,
// 0x143 = row_bcast:31 (GFX9 encodings, valid on gfx950). Lanes with no source / masked rows read 0.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_move(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROW_MASK, 0xF, false));
}

// Segmented inclusive wave64 sums of N values per lane, runs = lanes [start, lane] (start: first lane
// of the lane's run). Intra-row Hillis-Steele (row_shr 1,2,4,8) then the row_bcast 15 / 31 carries
// of the classic DPP scan, each applied only where the source lane lies in the same run. STEPS: the
// intra-row distances 1 .. 2^(STEPS-1) are applied (enough when every run is shorter than 2^STEPS
// lanes); CROSS: the carries across rows.
template <int N, int STEPS, bool CROSS>
__device__ __forceinline__ void wave_segmented_scan_steps(float (&v)[N], int lane, int start) {
    const int r16 = lane & 15, row = lane >> 4, span = lane - start;
    const bool t1 = r16 >= 1 && span >= 1;
    const bool t2 = r16 >= 2 && span >= 2;
    const bool t4 = r16 >= 4 && span >= 4;
    const bool t8 = r16 >= 8 && span >= 8;
    const bool tb15 = (row & 1) && start <= 16 * row - 1;
    const bool tb31 = row >= 2 && start <= 31;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        float x = v[i], t;
        t = dpp_move<0x111, 0xF>(x); if (t1) x += t;
        if constexpr (STEPS >= 2) { t = dpp_move<0x112, 0xF>(x); if (t2) x += t; }
        if constexpr (STEPS >= 3) { t = dpp_move<0x114, 0xF>(x); if (t4) x += t; }
        if constexpr (STEPS >= 4) { t = dpp_move<0x118, 0xF>(x); if (t8) x += t; }
        if constexpr (CROSS) {
            t = dpp_move<0x142, 0xA>(x); if (tb15) x += t;
            t = dpp_move<0x143, 0xC>(x); if (tb31) x += t;
        }
        v[i] = x;
    }
}

// The full scan, or a shorter one chosen once per wave (ballots): runs of consecutive samples in
// one voxel are mostly 2-4 lanes long and seldom cross a 16-lane row, so most waves need one or two
// of the six steps.
template <int N>
__device__ __forceinline__ void wave_segmented_inclusive_sum(float (&v)[N], int lane, int start) {
    const int span = lane - start;
    const bool cross = __ballot(start < (lane & ~15)) != 0ull;   // a run continues across a row boundary
    if (!cross && __ballot(span >= 2) == 0ull) wave_segmented_scan_steps<N, 1, false>(v, lane, start);
    else if (!cross && __ballot(span >= 4) == 0ull) wave_segmented_scan_steps<N, 2, false>(v, lane, start);
    else wave_segmented_scan_steps<N, 4, true>(v, lane, start);
}

// Wave64 reductions / scans through DPP-capable shuffles.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

}  // namespace nerf
