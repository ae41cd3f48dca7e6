// Shared per-point voxel math of the hash-grid kernels (hashgrid.hip, quant.hip).
#pragma once

#include "common.h"

namespace nerf {

// RAdam's elementwise update (radam.py:49-79), in the reference's op order (compiled with
// -ffp-contract=off); shared by the fused optimizer launch (optim.hip) and the owner pass's fused table
// step (hashgrid.hip), which therefore update a table element bit for bit alike:
//   v = v*b2 + ((1-b2)*g)*g            exp_avg_sq.mul_(beta2).addcmul_(1 - beta2, grad, grad)
//   m = m*b1 + (1-b1)*g                exp_avg.mul_(beta1).add_(1 - beta1, grad)
//   p = p + (-wd*lr)*p                 weight decay (when wd != 0)
//   p = p + ((-step*lr)*m)/(sqrt(v)+eps)   addcdiv_ (mode 2), or p + (-step*lr)*m (mode 1)
__device__ __forceinline__ void radam_elem(const nerf_radam_segment& s, float& p, float g, float& m, float& v) {
    v = v * s.beta2 + (s.one_minus_beta2 * g) * g;
    m = m * s.beta1 + s.one_minus_beta1 * g;
    if (s.mode == 0) return;
    if (s.decay_coef != 0.f) p = p + s.decay_coef * p;
    if (s.mode == 2) p = p + (s.step_coef * m) / (sqrtf(v) + s.eps);
    else p = p + s.step_coef * m;
}

struct HashParams {
    const float* tables[NERF_MAX_LEVELS];
    float cell[NERF_MAX_LEVELS][3];   // grid_size = (box_max - box_min) / res, fp32 on the host
    float rcell[NERF_MAX_LEVELS][3];  // RN(1 / grid_size) (fill_cells): div_rn<true>'s reciprocal of the cell
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

// div_rn<true> with the reciprocal given: r = RN(1 / d), computed once per launch on the host for a
// uniform divisor (the cell size of a level and axis). Quotient then two residual corrections: with
// r correctly rounded and no operand or residual leaving the normal range (the FAST conditions), the
// last correction returns RN(n / d) (Markstein's correction theorem); the refined hardware
// reciprocal this replaces (v_rcp_f32 + two FMAs per axis) is no closer to 1 / d than r.
__device__ __forceinline__ float div_rn_recip(float n, float d, float r) {
    float q = n * r;
    q = fmaf(fmaf(-d, q, n), r, q);
    return fmaf(fmaf(-d, q, n), r, q);
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

// FAST (finite coordinates, fastdiv_point_ok): the clamp as one v_med3_f32 (the median of x, lo, hi
// IS clamp(x, lo, hi) for lo <= hi; a zero's sign it may pick differently cannot move the floor) and
// the cell division with the host's reciprocal rcell.
template <bool FAST = false>
__device__ __forceinline__ AxisCell axis_cell(float x, float lo, float hi, float cell, float rcell = 0.f) {
    AxisCell a;
    a.inside = (x == fmaxf(fminf(x, hi), lo));
    if constexpr (FAST) {
        const float xc = __builtin_amdgcn_fmed3f(x, lo, hi);
        a.base = (int)floorf(div_rn_recip(xc - lo, cell, rcell));
    } else {
        float xc = fminf(fmaxf(x, lo), hi);                   // torch.clamp(min=lo, max=hi)
        a.base = (int)floorf(div_rn<false>(xc - lo, cell));   // floor(...).int()
    }
    float vmin = (float)a.base * cell + lo;               // bottom_left_idx*grid_size + box_min
    float vmax = vmin + cell;                             // + 1.0*grid_size
    a.w = div_rn<FAST>(x - vmin, vmax - vmin);
    return a;
}

// RN(1 / c) for a positive normal float c: the double quotient rounded to float, then the float
// neighbour whose error is smaller, if any (the error 1 - c r is exact in double: c r has <= 48
// significant bits), so a double rounding of 1 / c cannot leave it off by one.
static float recip_rn(float c) {
    float r = (float)(1.0 / (double)c);
    auto err = [c](float q) { const double e = 1.0 - (double)c * (double)q; return e < 0 ? -e : e; };
    for (const float q : {nextafterf(r, 0.f), nextafterf(r, 1e30f)}) {
        const double eq = err(q), er = err(r);
        if (eq < er || (eq == er && (__builtin_bit_cast(uint32_t, q) & 1u) == 0u)) r = q;
    }
    return r;
}

// grid_size = (box_max - box_min) / resolution (utils.py:106): the same two fp32 operations,
// correctly rounded, on the host once per launch instead of per point. Returns whether the box and
// the cells admit div_rn<true>: |box bounds| 0 or in [2^-40, 2^40], cells in [2^-40, 2^40] and at
// least 2^-16 of the largest |bound| (so vmax - vmin stays within 2^-7 of the cell).
static bool fill_cells(float (*cell)[3], float (*rcell)[3], const float* bmin, const float* bmax, const float* res,
                       int n_levels) {
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
            rcell[l][a] = recip_rn(c);
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

// ---- lane-pair forward gather (hashgrid.hip hash_encode_fwd_pair_kernel, quant.hip packed gather) ----
constexpr int kFwdGroupRound = 2;   // grouped coarse levels: gathers of two levels in flight per thread
constexpr int kFwdGroupMax = 8;
// QUANT: every gathered corner feature goes through the level's A-CAQ quantizer first
// (hash_encoding.py:97-101: quantizers[i](voxel_embedds), elementwise on the [P,8,2] gather).
// Lane-pair forward: lanes 2m and 2m+1 share point m of the wave and gather the x = 0 and x = 1
// corners of its voxel. Corners (x,y,z) and (x+1,y,z) hash to h and h ^ (x ^ (x+1)), the same 64-B
// line for 15 of 16 x, so each gather instruction touches ~32 lines instead of 64 (the vector
// memory path processes a wave instruction's distinct lines one after another). The x blend
// c_jk = e(0,j,k)(1-wx) + e(1,j,k)wx becomes a + partner's b (IEEE addition commutes: bit-exact).
// value of the other lane of the pair (lanes 2m <-> 2m+1): DPP quad_perm [1,0,3,2], no LDS round
// trip (ds_bpermute)
__device__ __forceinline__ int pair_swap_i(int v) { return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false); }
__device__ __forceinline__ float pair_swap(float v) { return __int_as_float(pair_swap_i(__float_as_int(v))); }

// The three axes of a point for lane xb of its pair: both lanes need all three, so lane 0 computes
// (x, y) and lane 1 (x, z) and they swap the y / z results (4 divisions per lane, not 6).
template <bool FAST>
__device__ __forceinline__ void fwd_axes(float x, float y, float z, const HashParams& hp, int lvl, int xb,
                                         AxisCell& ax, AxisCell& ay, AxisCell& az) {
    ax = axis_cell<FAST>(x, hp.bmin[0], hp.bmax[0], hp.cell[lvl][0], hp.rcell[lvl][0]);
    const AxisCell a2 = axis_cell<FAST>(xb ? z : y, xb ? hp.bmin[2] : hp.bmin[1], xb ? hp.bmax[2] : hp.bmax[1],
                                        xb ? hp.cell[lvl][2] : hp.cell[lvl][1],
                                        xb ? hp.rcell[lvl][2] : hp.rcell[lvl][1]);
    const int pk = a2.base | (a2.inside ? 0x40000000 : 0);   // 0 <= base <= res < 2^30
    const int opk = pair_swap_i(pk);
    const float ow = pair_swap(a2.w);
    AxisCell o;
    o.base = opk & 0x3FFFFFFF;
    o.inside = (opk & 0x40000000) != 0;
    o.w = ow;
    ay = xb ? o : a2;
    az = xb ? a2 : o;
}

// One (point, level) of a lane pair: the axes and the four gathers are issued first (fwd_gather),
// the blend and the store follow (fwd_finish), so a thread can keep several levels' gathers in flight.
struct FwdLvl {
    float wx, wy, wz;
    bool inside;
    float2 e[4];   // corners (xb, j, k), index 2j + k
};

template <bool FAST>
__device__ __forceinline__ void fwd_gather(float x, float y, float z, const HashParams& hp, int lvl, int xb,
                                           FwdLvl& s) {
    AxisCell ax, ay, az;
    fwd_axes<FAST>(x, y, z, hp, lvl, xb, ax, ay, az);
    s.wx = ax.w; s.wy = ay.w; s.wz = az.w;
    s.inside = ax.inside && ay.inside && az.inside;
    const float2* __restrict__ tab = reinterpret_cast<const float2*>(hp.tables[lvl]);
    const uint32_t bx = (uint32_t)ax.base + (uint32_t)xb, by = (uint32_t)ay.base, bz = (uint32_t)az.base;
#pragma unroll
    for (int c = 0; c < 4; ++c) s.e[c] = tab[spatial_hash3(bx, by + ((c >> 1) & 1), bz + (c & 1), hp.mask)];
}

template <bool QUANT>
__device__ __forceinline__ void fwd_finish(FwdLvl& s, int lvl, int xb, bool valid, int64_t p,
                                           float* __restrict__ feat, int64_t sp, int64_t sl,
                                           uint8_t* __restrict__ keep, const QuantRec* __restrict__ qrec) {
    if constexpr (QUANT) {
        const QuantRec q = qrec[lvl];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            s.e[c].x = fake_quant(s.e[c].x, q);
            s.e[c].y = fake_quant(s.e[c].y, q);
        }
    }
    const float wx = s.wx, wy = s.wy, wz = s.wz;
    const float fx = xb ? wx : 1.0f - wx;
    float cx[4], cy[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float ax_ = s.e[c].x * fx, ay_ = s.e[c].y * fx;
        cx[c] = ax_ + pair_swap(ax_);
        cy[c] = ay_ + pair_swap(ay_);
    }
    const float oy = 1.0f - wy, oz = 1.0f - wz;
    // c00 = cx[0], c01 = cx[1], c10 = cx[2], c11 = cx[3]
    const float c0x = cx[0] * oy + cx[2] * wy, c1x = cx[1] * oy + cx[3] * wy;
    const float c0y = cy[0] * oy + cy[2] * wy, c1y = cy[1] * oy + cy[3] * wy;
    const float ox_ = c0x * oz + c1x * wz, oy_ = c0y * oz + c1y * wz;
    if (!valid) return;
    if (lvl == 0 && keep && xb == 0) keep[p] = s.inside ? 1 : 0;
    float* dst = feat + p * sp + (int64_t)lvl * sl;
    dst[xb] = xb ? oy_ : ox_;
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

// ---- TV loss forward (loss.py:11-43), one block of tv_fwd_kernel (optim.hip) or of the TV blocks of
// hash_encode_fwd_tv_kernel (hashgrid.hip)
constexpr int kTVBlocks = 96;
constexpr int kTVUnroll = 8;

// cube vertex (i,j,k) = min_vertex + (i,j,k) in meshgrid 'ij' order (loss.py:25-27)
template <int UNROLL = kTVUnroll>
__device__ __forceinline__ void tv_fwd_block(const TVParams& P, int l, unsigned bx, unsigned nbx) {
    const int c = P.cube[l], n1 = c + 1;
    const uint32_t nv = (uint32_t)(P.vstart[l + 1] - P.vstart[l]);
    const float2* tab = reinterpret_cast<const float2*>(P.tables[l]);
    int mvd[3];
    tv_corner(P, l, mvd);
    const int* mv = mvd;
    const uint32_t stride = nbx * 256u;
    float part = 0.f;
    for (uint32_t lv0 = bx * 256u + threadIdx.x; lv0 < nv; lv0 += UNROLL * stride) {
        float2 e[UNROLL], f[UNROLL][3];
        bool nb[UNROLL][3];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint32_t lv = lv0 + u * stride;
            const bool ok = lv < nv;
            int i = 0, j = 0, k = 0;
            if (ok) tv_vertex(lv, n1, i, j, k);
            nb[u][0] = ok && i < c; nb[u][1] = ok && j < c; nb[u][2] = ok && k < c;
            e[u] = ok ? tv_fetch(tab, mv, i, j, k, P.mask) : make_float2(0.f, 0.f);
            f[u][0] = nb[u][0] ? tv_fetch(tab, mv, i + 1, j, k, P.mask) : e[u];
            f[u][1] = nb[u][1] ? tv_fetch(tab, mv, i, j + 1, k, P.mask) : e[u];
            f[u][2] = nb[u][2] ? tv_fetch(tab, mv, i, j, k + 1, P.mask) : e[u];
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const uint32_t lv = lv0 + u * stride;
            if (lv < nv) {
                if (P.verts) P.verts[P.vstart[l] + lv] = e[u];
                float acc = 0.f;
#pragma unroll
                for (int d = 0; d < 3; ++d)
                    if (nb[u][d]) { const float dx = f[u][d].x - e[u].x, dy = f[u][d].y - e[u].y; acc += dx * dx + dy * dy; }
                part += acc / (float)c;
            }
        }
    }
    __shared__ float s_part[4];
    const float w = wave_sum(part);
    if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = w;
    __syncthreads();
    if (threadIdx.x == 0) {
        const float t = (s_part[0] + s_part[1]) + (s_part[2] + s_part[3]);
        if (t != 0.f) atomicAdd(P.loss + l, t);
    }
}


}  // namespace nerf
