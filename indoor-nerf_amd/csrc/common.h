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

// n / d for 0 <= n < 2^31 as mulhi(n, m) >> s (Granlund-Montgomery: l = ceil(log2 d),
// m = ceil(2^(31+l) / d) < 2^32, s = l - 1; m = 0 encodes d = 1): a runtime-invariant divisor costs
// two VALU ops instead of the ~15 of an integer division (v_rcp_iflag + correction steps)
__device__ __forceinline__ uint32_t udiv_magic(uint32_t n, uint32_t m, int s) {
    return m ? (__umulhi(n, m) >> s) : n;
}

inline void ray_div_magic(int64_t d, uint32_t& m, int& s) {
    if (d <= 1) { m = 0; s = 0; return; }
    int l = 0;
    while ((int64_t(1) << l) < d) ++l;
    m = (uint32_t)(((uint64_t(1) << (31 + l)) + (uint64_t)d - 1) / (uint64_t)d);
    s = l - 1;
}

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
// Step-major: each step runs over all N values before the next, so a DPP read never follows the
// VALU write of its source register within the 2-wait-state hazard window (value-major order put
// an s_nop in front of nearly every DPP step).
template <int N, int CTRL, int ROW_MASK>
__device__ __forceinline__ void seg_scan_step(float (&v)[N], bool take) {
    float t[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        if constexpr (ROW_MASK == 0xF) {
            t[i] = v[i] + dpp_move<CTRL, ROW_MASK>(v[i]);
        } else {   // masked-out rows never take the step: their lanes' t may be anything (mov_dpp: old undef)
            t[i] = v[i] + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v[i]), CTRL, ROW_MASK, 0xF, false));
        }
    }
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = take ? t[i] : v[i];   // a select, not a branch
}

template <int N, int STEPS, bool CROSS>
__device__ __forceinline__ void wave_segmented_scan_steps(float (&v)[N], int lane, int start) {
    const int r16 = lane & 15, row = lane >> 4, span = lane - start;
    const bool t1 = r16 >= 1 && span >= 1;
    const bool t2 = r16 >= 2 && span >= 2;
    const bool t4 = r16 >= 4 && span >= 4;
    const bool t8 = r16 >= 8 && span >= 8;
    const bool tb15 = (row & 1) && start <= 16 * row - 1;
    const bool tb31 = row >= 2 && start <= 31;
    seg_scan_step<N, 0x111, 0xF>(v, t1);
    if constexpr (STEPS >= 2) seg_scan_step<N, 0x112, 0xF>(v, t2);
    if constexpr (STEPS >= 3) seg_scan_step<N, 0x114, 0xF>(v, t4);
    if constexpr (STEPS >= 4) seg_scan_step<N, 0x118, 0xF>(v, t8);
    if constexpr (CROSS) {
        seg_scan_step<N, 0x142, 0xA>(v, tb15);
        seg_scan_step<N, 0x143, 0xC>(v, tb31);
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

// ---- fp64 wave64 scans and reductions on DPP (VALU lane moves; no LDS crossbar round trips) ----
// A double moves as its two dwords; lanes without a source (or in masked rows) keep `old`.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ double dpp_d(double v, double old) {
    const uint64_t u = __double_as_longlong(v), o = __double_as_longlong(old);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)o, (int)(uint32_t)u, CTRL, ROW_MASK, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(o >> 32), (int)(uint32_t)(u >> 32), CTRL,
                                                              ROW_MASK, 0xF, false);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

__device__ __forceinline__ double readlane_d(double v, int l) {
    const uint64_t u = __double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// Sum over the wave, returned to every lane: quad, half-row and row mirrors, then the row_bcast 15 /
// 31 carries leave the total in lane 63, read back as a uniform value. Fixed order (deterministic).
__device__ __forceinline__ double wave_sum_dpp(double v) {
    v += dpp_d<0xB1>(v, 0.0);        // quad_perm [1,0,3,2]
    v += dpp_d<0x4E>(v, 0.0);        // quad_perm [2,3,0,1]
    v += dpp_d<0x141>(v, 0.0);       // row_half_mirror: the other quad of the 8
    v += dpp_d<0x140>(v, 0.0);       // row_mirror: the other 8 of the row
    v += dpp_d<0x142, 0xA>(v, 0.0);  // row_bcast:15 into rows 1, 3
    v += dpp_d<0x143, 0xC>(v, 0.0);  // row_bcast:31 into rows 2, 3
    return readlane_d(v, 63);
}

// Inclusive prefix sum over lanes: row_shr 1, 2, 4, 8 inside each row, then the row_bcast carries.
__device__ __forceinline__ double wave_incl_sum_dpp(double v) {
    v += dpp_d<0x111>(v, 0.0);
    v += dpp_d<0x112>(v, 0.0);
    v += dpp_d<0x114>(v, 0.0);
    v += dpp_d<0x118>(v, 0.0);
    v += dpp_d<0x142, 0xA>(v, 0.0);
    v += dpp_d<0x143, 0xC>(v, 0.0);
    return v;
}

// Exclusive product scan over lanes (lane 0 gets 1): Hillis-Steele row_shr 1, 2, 4, 8 inside each
// row, the row_bcast 15 / 31 carries across rows, then wave_shr:1.
__device__ __forceinline__ double wave_excl_prod_dpp(double v) {
    v *= dpp_d<0x111>(v, 1.0);
    v *= dpp_d<0x112>(v, 1.0);
    v *= dpp_d<0x114>(v, 1.0);
    v *= dpp_d<0x118>(v, 1.0);
    v *= dpp_d<0x142, 0xA>(v, 1.0);
    v *= dpp_d<0x143, 0xC>(v, 1.0);
    return dpp_d<0x138>(v, 1.0);     // wave_shr:1
}

// Exclusive suffix scan of affine maps f_b(U) = X_b + P_b U over lanes (lane b gets the composition
// of lanes b+1 .. 63 applied to U = 0, i.e. its X; lane 63 gets 0): row_shl 1, 2, 4, 8 inside each
// row (a missing source is the identity (0, 1)), the row totals (lane 16r) read back and composed
// across rows, then wave_shl:1.
__device__ __forceinline__ double wave_excl_suffix_affine_dpp(double X, double P, int lane) {
#define NERF_AFFINE_STEP(CTRL)                             {                                                          const double Xn = dpp_d<CTRL>(X, 0.0);                 const double Pn = dpp_d<CTRL>(P, 1.0);                 X = X + P * Xn;                                        P = P * Pn;                                        }
    NERF_AFFINE_STEP(0x101)
    NERF_AFFINE_STEP(0x102)
    NERF_AFFINE_STEP(0x104)
    NERF_AFFINE_STEP(0x108)
#undef NERF_AFFINE_STEP
    // suffix over the rows after this lane's: S3 = id, S2 = C3, S1 = C2 o C3, S0 = C1 o S1
    const double X1 = readlane_d(X, 16), P1 = readlane_d(P, 16);
    const double X2 = readlane_d(X, 32), P2 = readlane_d(P, 32);
    const double X3 = readlane_d(X, 48);
    const double S2x = X3;
    const double S1x = X2 + P2 * S2x;
    const double S0x = X1 + P1 * S1x;
    const int row = lane >> 4;
    const double Sx = row == 0 ? S0x : row == 1 ? S1x : row == 2 ? S2x : 0.0;
    X = X + P * Sx;
    return dpp_d<0x130>(X, 0.0);     // wave_shl:1: lane b reads lane b + 1; lane 63 keeps 0
}

}  // namespace nerf
