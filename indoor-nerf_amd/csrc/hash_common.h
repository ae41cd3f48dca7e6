// Shared per-point voxel math of the hash-grid kernels (hashgrid.hip, quant.hip).
#pragma once

#include "common.h"

namespace nerf {

struct HashParams {
    const float* tables[NERF_MAX_LEVELS];
    float cell[NERF_MAX_LEVELS][3];   // grid_size = (box_max - box_min) / res, fp32 on the host
    float bmin[3];
    float bmax[3];
    uint32_t mask;
    uint32_t fastdiv;                 // fill_cells: the box and cells admit div_rn<true> (below)
};

// Correctly rounded fp32 n / d. FAST is the core of the compiler's IEEE division sequence
// (v_rcp, one Newton step on the reciprocal, quotient, two residual corrections) without its
// v_div_scale / v_div_fmas scaling and v_div_fixup special-case steps (11 -> 8 VALU): those change
// nothing when n = 0 or 2^-96 <= |n| <= 2^42 and 2^-41 <= d <= 2^41 (no operand or residual
// leaves the normal range), so FAST returns the bits of n / d there. axis_cell's callers take
// FAST only when fill_cells accepted the box and cells and every coordinate of the wave passes
// fastdiv_point_ok, which together bound both numerators and denominators to that range.
template <bool FAST>
__device__ __forceinline__ float div_rn(float n, float d) {
    if constexpr (FAST) {
        float r = __builtin_amdgcn_rcpf(d);
        r = fmaf(fmaf(-d, r, 1.0f), r, r);
        float q = n * r;
        q = fmaf(fmaf(-d, q, n), r, q);
        return fmaf(fmaf(-d, q, n), r, q);
    } else {
        return n / d;
    }
}

// A point admits the fast division when every |coordinate| is in [2^-72, 2^40] (NaN/Inf fail):
// then x - vmin and clamp(x) - lo are 0 or >= 2^-95 in magnitude (vmin = base * cell + lo is 0
// or >= 2^-63 given fill_cells' bounds on lo and cell) and both quotients stay normal.
__device__ __forceinline__ bool fastdiv_point_ok(float x, float y, float z) {
    const float m = fminf(fminf(fabsf(x), fabsf(y)), fabsf(z));
    const float s = fabsf(x) + fabsf(y) + fabsf(z);
    return m >= 0x1p-72f && s <= 0x1p40f;
}

// Per-axis voxel math of utils.py:103-112, fp32, exact op order.
struct AxisCell {
    int base;      // bottom_left_idx
    float w;       // (x - vmin) / (vmax - vmin), on the UNclamped x (hash_encoding.py:64)
    bool inside;   // x == max(min(x, bmax), bmin)
};

template <bool FAST = false>
__device__ __forceinline__ AxisCell axis_cell(float x, float lo, float hi, float cell) {
    AxisCell a;
    a.inside = (x == fmaxf(fminf(x, hi), lo));
    float xc = fminf(fmaxf(x, lo), hi);                   // torch.clamp(min=lo, max=hi)
    a.base = (int)floorf(div_rn<FAST>(xc - lo, cell));    // floor(...).int()
    float vmin = (float)a.base * cell + lo;               // bottom_left_idx*grid_size + box_min
    float vmax = vmin + cell;                             // + 1.0*grid_size
    a.w = div_rn<FAST>(x - vmin, vmax - vmin);
    return a;
}

// grid_size = (box_max - box_min) / resolution (utils.py:106): the same two fp32 operations,
// correctly rounded, on the host once per launch instead of per point. Returns whether the box and
// the cells admit div_rn<true>: |box bounds| 0 or in [2^-40, 2^40], cells in [2^-40, 2^40] and at
// least 2^-16 of the largest |bound| (so vmax - vmin stays within 2^-7 of the cell).
static bool fill_cells(float (*cell)[3], const float* bmin, const float* bmax, const float* res, int n_levels) {
    bool ok = true;
    float big = 0.f;
    for (int a = 0; a < 3; ++a)
        for (const float b : {bmin[a], bmax[a]}) {
            const float m = b < 0.f ? -b : b;
            ok = ok && (m == 0.f || (m >= 0x1p-40f && m <= 0x1p40f));
            big = m > big ? m : big;
        }
    for (int l = 0; l < n_levels; ++l)
        for (int a = 0; a < 3; ++a) {
            const volatile float d = bmax[a] - bmin[a];
            cell[l][a] = d / res[l];
            const float c = cell[l][a];
            ok = ok && c >= 0x1p-40f && c <= 0x1p40f && c >= big * 0x1p-16f;
        }
    return ok;
}

// ---- A-CAQ quantizer record (quantization.py:144-187), written by nerf_quant_params -------------
// {scale, scale + 1e-8, zero_point, qmin, qmax, ste, integer bits, 0}: the scalars
// LearnedBitwidthQuantizer.forward derives from (soft_bits, range_scale, v_max) before touching x.
struct QuantRec {
    float scale, scale_eps, zp, qmin, qmax, ste, bits, pad;
};

// x -> round(x / (scale + 1e-8) + zp) clamped to [qmin, qmax] -> (q - zp) * scale, returned in the
// training-mode STE form x + (deq - x) (:176-181) or as deq (eval, :183-186); fp32, same op order.
__device__ __forceinline__ float quant_code(float x, const QuantRec& q) {
    const float xq = rintf(x / q.scale_eps + q.zp);       // torch.round: half to even
    return fminf(fmaxf(xq, q.qmin), q.qmax);              // torch.clamp(min, max)
}

__device__ __forceinline__ float fake_quant(float x, const QuantRec& q) {
    const float deq = (quant_code(x, q) - q.zp) * q.scale;
    return q.ste != 0.f ? x + (deq - x) : deq;
}

// Order-preserving float <-> uint32 map for atomicMin/atomicMax calibration statistics.
__device__ __forceinline__ uint32_t f2ord(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}

// Trilinear blend of hash_encoding.py:56-80 for one feature (x, then y, then z pairs).
__device__ __forceinline__ float trilerp(const float (&e)[8], float wx, float wy, float wz) {
    const float ox = 1.0f - wx, oy = 1.0f - wy, oz = 1.0f - wz;
    const float c00 = e[0] * ox + e[4] * wx;
    const float c01 = e[1] * ox + e[5] * wx;
    const float c10 = e[2] * ox + e[6] * wx;
    const float c11 = e[3] * ox + e[7] * wx;
    const float c0 = c00 * oy + c10 * wy;
    const float c1 = c01 * oy + c11 * wy;
    return c0 * oz + c1 * wz;
}

// ---- TV loss over a hashed cuboid per level (loss.py:11-43): optim.hip (forward, atomic backward)
// and hashgrid.hip (binned backward) -----------------------------------------------------------
struct TVParams {
    const float* tables[NERF_MAX_LEVELS];
    float* dtables[NERF_MAX_LEVELS];
    int mv[NERF_MAX_LEVELS][3];
    int cube[NERF_MAX_LEVELS];
    int64_t vstart[NERF_MAX_LEVELS + 1];   // first vertex of each level in the flattened launch
    int L;
    uint32_t mask;
    const int64_t* dmv;   // optional device [L][3] cuboid corners (graph replays draw new ones)
    const float* scale;   // bwd: device [L] upstream gradient per level
    float* loss;          // fwd: device [L]
    float2* verts;        // optional: the cuboid vertices' table rows, level l at verts + vstart[l]
                          // (written by tv_fwd, read by tv_bwd_bin in place of the hashed gathers)
};

__device__ __forceinline__ float2 tv_fetch(const float2* tab, const int* mv, int i, int j, int k, uint32_t mask) {
    return tab[spatial_hash3((uint32_t)(mv[0] + i), (uint32_t)(mv[1] + j), (uint32_t)(mv[2] + k), mask)];
}

// level l's cuboid corner: the device slots (graph replays draw new ones) or the launch's copy
__device__ __forceinline__ void tv_corner(const TVParams& P, int l, int (&mv)[3]) {
    if (P.dmv) {
        mv[0] = (int)P.dmv[3 * l]; mv[1] = (int)P.dmv[3 * l + 1]; mv[2] = (int)P.dmv[3 * l + 2];
    } else {
        mv[0] = P.mv[l][0]; mv[1] = P.mv[l][1]; mv[2] = P.mv[l][2];
    }
}

__device__ __forceinline__ void tv_vertex(uint32_t lv, int n1, int& i, int& j, int& k) {
    const uint32_t q = lv / (uint32_t)n1;      // < 1025^3: 32-bit index math
    k = (int)(lv - q * (uint32_t)n1);
    j = (int)(q % (uint32_t)n1);
    i = (int)(q / (uint32_t)n1);
}

static int fill_tv(TVParams& P, int n_levels, int log2_T, const int64_t* min_vertex, const int64_t* d_min_vertex,
                   const int* cube) {
    NERF_REQUIRE(n_levels >= 1 && n_levels <= NERF_MAX_LEVELS, "tv: n_levels %d", n_levels);
    NERF_REQUIRE(log2_T >= 1 && log2_T <= 30, "tv: log2_T %d", log2_T);
    NERF_REQUIRE((min_vertex || d_min_vertex) && cube, "tv: null arg");
    P.dmv = d_min_vertex;
    P.L = n_levels;
    P.mask = (uint32_t)((1u << log2_T) - 1u);
    P.vstart[0] = 0;
    for (int l = 0; l < n_levels; ++l) {
        NERF_REQUIRE(cube[l] >= 1 && cube[l] <= 1024, "tv: cube[%d] = %d", l, cube[l]);
        for (int a = 0; a < 3; ++a) P.mv[l][a] = min_vertex ? (int)min_vertex[3 * l + a] : 0;
        P.cube[l] = cube[l];
        const int64_t n1 = cube[l] + 1;
        P.vstart[l + 1] = P.vstart[l] + n1 * n1 * n1;
    }

    return NERF_OK;
}

}  // namespace nerf
