#include <stdlib.h>
// Field MLP on the bf16 matrix cores with fp32 accuracy ("x6", the default MLP path).
//
// gfx950 has no tf32/xf32 MFMA and its f32-input MFMA (v_mfma_f32_32x32x2_f32) runs at 1/16 of
// the bf16 rate. Every fp32 operand v is therefore split EXACTLY into three bf16 pieces
//     v = v0 + v1 + v2,   v0 = bf16_rne(v), v1 = bf16_rne(v - v0), v2 = bf16_rne(v - v0 - v1)
// (|v1| <= 2^-8 |v|, |v2| <= 2^-16 |v|; nothing is left after v2 for normal fp32) and a product
// a*b is formed by six v_mfma_f32_32x32x16_bf16 terms
//     a0b0 + a0b1 + a1b0 + a1b1 + a0b2 + a2b0
// whose dropped terms a1b2 + a2b1 + a2b2 are <= 2^-23 |ab|: the per-product error of an fp32
// multiply (2^-24 |ab|) within a factor of two, accumulated in fp32 like the f32 MFMA chain.
// Six 32-cycle bf16 MFMAs per 32x32x16 step replace eight 64-cycle f32 MFMAs (2.7x fewer cycles).
//
// Orientation (as field_frag.hip): a layer's activations are a 32x32 accumulator tile
// X[neuron][point], lane = point. The next layer Y = W X takes X as the B operand with no data
// movement: the k-chunk c (0, 1) of a 32-row tile is registers 8c..8c+7, element i of lane half
// h <-> neuron row 16c + 4h + (i&3) + 8(i>>2), and the weight A operand is read with the same
// permutation from an LDS image of W (two ds_read_b64 per piece). The transposed chain
// (gX = W^T gY) reads the SAME image with ds_read_b64_tr_b16 (gfx950's transposing LDS read).
// Weight gradients dW = gY X^T sum over points (the lane index of both tiles): both tiles are
// staged per wave as [point][neuron] bf16 images and read back transposed, then 6 MFMAs per
// 16-point chunk accumulate into register-resident dW tiles (reduced once per block).
//
// LDS images (bf16, per piece, rows padded by 4 elements so that the 32 row reads of a lane half
// hit 64 distinct banks): W0 [64][32], W1 [16][64], C0' [64][32] (cols: 0 sigma slot = 0,
// 1..15 = C0 geo cols 16..30, 16..31 = C0 SH cols 0..15), C1 [64][64], C2 [16][64] (rows 3..15
// zero).
#include "field_common.h"

namespace nerf {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

// 8 values of an operand fragment as three bf16 pieces; element i = half (i & 1) of dword i >> 1.
struct S3 {
    u32x4 p[3];
};

#define X6_MFMA(a, b, c) \
    __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, (a)), __builtin_bit_cast(bf16x8, (b)), (c), 0, 0, 0)

__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
    const bf16x2 v = {(__bf16)a, (__bf16)b};   // v_cvt_pk_bf16_f32: round to nearest even
    return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ float lo_f(uint32_t p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float hi_f(uint32_t p) { return __uint_as_float(p & 0xffff0000u); }

// The empty asm statements keep each packed word opaque: otherwise the compiler rewrites
// lo_f(pk(a, b)) as a second, single-value conversion of a (one extra VALU op per pair).
__device__ __forceinline__ void split2(float a, float b, uint32_t& p0, uint32_t& p1, uint32_t& p2) {
    p0 = pk_bf16(a, b);
    asm("" : "+v"(p0));
    const float ra = a - lo_f(p0), rb = b - hi_f(p0);      // exact
    p1 = pk_bf16(ra, rb);
    asm("" : "+v"(p1));
    const float sa = ra - lo_f(p1), sb = rb - hi_f(p1);    // exact
    p2 = pk_bf16(sa, sb);
}

// ReLU as ONE integer op per element, v_max_i32(bits, 0): a negative float (and -0, and a negative
// NaN) is a negative int and becomes +0, a positive one keeps its bits. A float max compiles to two
// v_max_f32 per element on MFMA results (a canonicalising max first), the shift-and-mask form to two.
__device__ __forceinline__ void relu16i(floatx16& v) {
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = __int_as_float(max(__float_as_int(v[r]), 0));
}

// bit k of m |= (v > 0) for a ReLU output v >= 0 (its bits are nonzero iff v > 0): v_min_u32 +
// v_lshl_or_b32, two ops instead of compare, select and or
__device__ __forceinline__ uint32_t relu_bit(uint32_t m, float v, int k) {
    return m | (min(__float_as_uint(v), 1u) << k);
}

__device__ __forceinline__ S3 split8(float v0, float v1, float v2, float v3, float v4, float v5, float v6, float v7) {
    uint32_t a[4], b[4], c[4];
    split2(v0, v1, a[0], b[0], c[0]);
    split2(v2, v3, a[1], b[1], c[1]);
    split2(v4, v5, a[2], b[2], c[2]);
    split2(v6, v7, a[3], b[3], c[3]);
    S3 s;
    s.p[0] = u32x4{a[0], a[1], a[2], a[3]};
    s.p[1] = u32x4{b[0], b[1], b[2], b[3]};
    s.p[2] = u32x4{c[0], c[1], c[2], c[3]};
    return s;
}

// chunk c of a 32-row accumulator tile: registers 8c .. 8c+7
__device__ __forceinline__ S3 split_chunk(const floatx16& v, int c) {
    return split8(v[8 * c], v[8 * c + 1], v[8 * c + 2], v[8 * c + 3], v[8 * c + 4], v[8 * c + 5], v[8 * c + 6],
                  v[8 * c + 7]);
}

__device__ __forceinline__ S3 split_arr(const float* v) {
    return split8(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]);
}

// acc += A B over one 16-deep k-chunk, fp32-accurate (six bf16 products; small terms first)
__device__ __forceinline__ floatx16 mma6(const S3& A, const S3& B, floatx16 c) {
    c = X6_MFMA(A.p[0], B.p[2], c);
    c = X6_MFMA(A.p[2], B.p[0], c);
    c = X6_MFMA(A.p[1], B.p[1], c);
    c = X6_MFMA(A.p[0], B.p[1], c);
    c = X6_MFMA(A.p[1], B.p[0], c);
    c = X6_MFMA(A.p[0], B.p[0], c);
    return c;
}

// ---- LDS images (bf16 elements) ----------------------------------------------------------------
constexpr int S64 = 68, S32 = 36;            // padded row strides of 64- and 32-column matrices
constexpr int IM_W0 = 0;                     // [64][S32]
constexpr int IM_W1 = IM_W0 + 64 * S32;      // [16][S64]
constexpr int IM_C0 = IM_W1 + 16 * S64;      // [64][S32]
constexpr int IM_C1 = IM_C0 + 64 * S32;      // [64][S64]
constexpr int IM_C2 = IM_C1 + 64 * S64;      // [16][S64]
constexpr int IM_PIECE = IM_C2 + 16 * S64;   // 11,136 elements per piece
constexpr int IM_BYTES = 3 * IM_PIECE * 2;   // 66,816 B
// logical (unpadded) element index ranges of the five matrices, for the fill loop
constexpr int L_W1 = 2048, L_C0 = 3072, L_C1 = 5120, L_C2 = 9216, L_END = 10240;
// backward staging of one 32-row gradient tile [32 points][32], three bf16 pieces
constexpr int STG_PIECE = 32 * S32;

__device__ __forceinline__ float image_value(int idx, const nerf_mlp_weights& W) {
    if (idx < L_W1) return W.w0[idx];                                     // [64][32]
    if (idx < L_C0) return W.w1[idx - L_W1];                              // [16][64]
    if (idx < L_C1) {
        const int k = idx - L_C0, r = k >> 5, c = k & 31;
        if (c == 0) return 0.f;                                           // sigma slot
        return c < 16 ? W.c0[r * 31 + 15 + c] : W.c0[r * 31 + c - 16];    // geo 1..15 | SH 0..15
    }
    if (idx < L_C2) return W.c1[idx - L_C1];
    const int k = idx - L_C2;
    return (k >> 6) < 3 ? W.c2[k] : 0.f;
}

// Every block's prologue. The loads of a round (kFillRound per thread) are issued before the first
// split / store: one memory round trip per round instead of one per element (a thread of a 512-wide
// block has 20 elements; one at a time, their L2 latencies were serial).
constexpr int kFillRound = 10;
__device__ inline void fill_images(__bf16* img, const nerf_mlp_weights& W) {
    for (int base = threadIdx.x; base < L_END; base += kFillRound * blockDim.x) {
        float v[kFillRound];
#pragma unroll
        for (int u = 0; u < kFillRound; ++u) {
            const int idx = base + u * (int)blockDim.x;
            v[u] = idx < L_END ? image_value(idx, W) : 0.f;
        }
#pragma unroll
        for (int u = 0; u < kFillRound; ++u) {
            const int idx = base + u * (int)blockDim.x;
            if (idx >= L_END) continue;
            int off;
            if (idx < L_W1) off = IM_W0 + (idx >> 5) * S32 + (idx & 31);
            else if (idx < L_C0) { const int k = idx - L_W1; off = IM_W1 + (k >> 6) * S64 + (k & 63); }
            else if (idx < L_C1) { const int k = idx - L_C0; off = IM_C0 + (k >> 5) * S32 + (k & 31); }
            else if (idx < L_C2) { const int k = idx - L_C1; off = IM_C1 + (k >> 6) * S64 + (k & 63); }
            else { const int k = idx - L_C2; off = IM_C2 + (k >> 6) * S64 + (k & 63); }
            const __bf16 a0 = (__bf16)v[u];
            const float r1 = v[u] - (float)a0;
            const __bf16 a1 = (__bf16)r1;
            const __bf16 a2 = (__bf16)(r1 - (float)a1);
            img[off] = a0;
            img[IM_PIECE + off] = a1;
            img[2 * IM_PIECE + off] = a2;
        }
    }
}

// A operand of Y = M X for the output row r of lane m: elements i <-> columns
// col0 + (i&3) + 8(i>>2), col0 = 32t + 16c + 4h (two ds_read_b64 per piece).
__device__ __forceinline__ S3 row_read(const __bf16* img, int base, int S, int r, int col0) {
    S3 s;
    const int o0 = base + r * S + col0;
#pragma unroll
    for (int p = 0; p < 3; ++p) {
        const u32x2 a = *reinterpret_cast<const u32x2*>(img + p * IM_PIECE + o0);
        const u32x2 b = *reinterpret_cast<const u32x2*>(img + p * IM_PIECE + o0 + 8);
        s.p[p] = u32x4{a.x, a.y, b.x, b.y};
    }
    return s;
}

// row_read over a staging image (piece stride `piece`)
__device__ __forceinline__ S3 row_read_st(const __bf16* st, int piece, int S, int r, int col0) {
    S3 s;
    const int o0 = r * S + col0;
#pragma unroll
    for (int p = 0; p < 3; ++p) {
        const u32x2 a = *reinterpret_cast<const u32x2*>(st + p * piece + o0);
        const u32x2 b = *reinterpret_cast<const u32x2*>(st + p * piece + o0 + 8);
        s.p[p] = u32x4{a.x, a.y, b.x, b.y};
    }
    return s;
}

// Operand whose k index runs over the ROWS of a row-major image: lane (m = lane&31, h = lane>>5)
// gets column col0 + m at rows row0 + 4h + (i&3) + 8(i>>2) (row0 = 16 x chunk, col0 = 32 x tile).
// Two ds_read_b64_tr_b16 per piece: 16-lane group g reads the 4 x 16 block at rows row0 + 4h
// (+8), columns col0 + 16(g&1); lane 4q+p supplies row q, columns 4p..4p+3, and lane i of the
// group receives column i of the 4 rows.
__device__ __forceinline__ S3 tr_read(const __bf16* img, int piece, int base, int S, int row0, int col0, int lane) {
    const int g = lane >> 4, il = lane & 15, q = il >> 2, p = il & 3, h = g >> 1;
    const int oa = base + (row0 + 4 * h + q) * S + col0 + 16 * (g & 1) + 4 * p;
    S3 s;
#pragma unroll
    for (int pc = 0; pc < 3; ++pc) {
        const bf16x4 ta = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(img + pc * piece + oa));
        const bf16x4 tb = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(img + pc * piece + oa + 8 * S));
        const u32x2 a = __builtin_bit_cast(u32x2, ta), b = __builtin_bit_cast(u32x2, tb);
        s.p[pc] = u32x4{a.x, a.y, b.x, b.y};
    }
    return s;
}

// tr_read for a row-stacked A operand (stride S32 images): lanes m < 16 (16-lane groups 0 and 2)
// take columns 0..15 of the block starting at element base_lo, lanes m >= 16 (groups 1 and 3) the
// same columns of the block at base_hi, k over the block's 16 rows (one piece each)
__device__ __forceinline__ u32x4 tr_read_pair(const __bf16* img, int base_lo, int base_hi, int lane) {
    const int g = lane >> 4, il = lane & 15, q = il >> 2, p = il & 3, h = g >> 1;
    const int oa = ((g & 1) ? base_hi : base_lo) + (4 * h + q) * S32 + 4 * p;
    const bf16x4 ta = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(img + oa));
    const bf16x4 tb = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(img + oa + 8 * S32));
    const u32x2 a = __builtin_bit_cast(u32x2, ta), b = __builtin_bit_cast(u32x2, tb);
    return u32x4{a.x, a.y, b.x, b.y};
}

// Stage chunk c of a 32-row tile (lane = point j) into a [32 points][S] staging image at
// columns col_t + 16c + 4h + (i&3) + 8(i>>2).
__device__ __forceinline__ void stage(__bf16* st, int piece, int S, const S3& s, int col_t, int c, int j, int h) {
    const int o0 = j * S + col_t + 16 * c + 4 * h;
#pragma unroll
    for (int p = 0; p < 3; ++p) {
        *reinterpret_cast<u32x2*>(st + p * piece + o0) = u32x2{s.p[p][0], s.p[p][1]};
        *reinterpret_cast<u32x2*>(st + p * piece + o0 + 8) = u32x2{s.p[p][2], s.p[p][3]};
    }
}

__device__ __forceinline__ void stage_grad(__bf16* stG, const S3& s, int c, int j, int h) {
    stage(stG, STG_PIECE, S32, s, 0, c, j, h);
}

// An opaque zero, redefined every tile: the weight images are loop-invariant, and without it the
// compiler hoists every fragment read out of the tile loop (288 registers of fragments -> spills).
__device__ __forceinline__ int opaque_zero() {
    int z = 0;
    asm volatile("" : "+v"(z));
    return z;
}

// ---- per-tile inputs ---------------------------------------------------------------------------
// x[8c + i] = feature 16c + 4h + (i&3) + 8(i>>2); SH = the three bf16 pieces of SH 4h + (i&3) + 8(i>>2)
struct InX6 {
    float x[16];
    S3 SH;
    uint32_t pt;    // 32-bit indexing (launch_* checks the sizes): one VGPR per address, saddr forms
    bool valid;
};

// NT: nontemporal loads (the backward's re-read of the features, the last use of the ~100 MB a
// step's hash forward writes: they no longer displace the tables and moments in the Infinity Cache;
// with the bins' d feat loads the same way, bins 202 -> 177 us and step 1.216 -> 1.187 ms on one box,
// profiles/r05v_ab_nt_feature_loads.jsonl)
#ifndef NERF_X6_BWD_NT_FEAT
#define NERF_X6_BWD_NT_FEAT 1
#endif
#ifndef NERF_X6_BWD_PREFETCH
#define NERF_X6_BWD_PREFETCH 1
#endif
typedef float f32x2_nt __attribute__((ext_vector_type(2)));
template <bool NT = false>
__device__ __forceinline__ void load_x6(const MlpArgs& a, uint32_t pt, bool valid, int h, float (&x)[16], int zero) {
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int q = 0; q < 2; ++q)
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int level = 8 * c + 4 * q + 2 * h + e;   // features 2 level, 2 level + 1
                // branch-free: a tail lane computes on the last point's features. Its column of every
                // tile is its own (Y = W X mixes no columns), the forward stores nothing for it, and in
                // the backward its upstream gradient is zero, so every weight-gradient term it forms is
                // 0 x (finite) — no zeroing of the inputs (28 selects per tile) is needed
                const uint32_t pc = valid ? pt : (uint32_t)(a.P - 1);
                const float* src = a.feat + (uint32_t)(pc * (uint32_t)a.sp + level * (uint32_t)a.sl + zero);
                if constexpr (NT) {
                    const f32x2_nt v = __builtin_nontemporal_load(reinterpret_cast<const f32x2_nt*>(src));
                    x[8 * c + 4 * q + 2 * e] = v.x;
                    x[8 * c + 4 * q + 2 * e + 1] = v.y;
                } else {
                    const float2 v = *reinterpret_cast<const float2*>(src);
                    x[8 * c + 4 * q + 2 * e] = v.x;
                    x[8 * c + 4 * q + 2 * e + 1] = v.y;
                }
            }
}

// shv[i] = SH coefficient 4h + (i&3) + 8(i>>2) of the point's view direction
__device__ __forceinline__ void load_sh6(const MlpArgs& a, uint32_t pt, bool valid, int h, float (&shv)[8], int zero) {
    float o[16];
    const uint32_t pc = valid ? pt : (uint32_t)(a.P - 1);
    if (!a.viewdirs && a.sh_stride == 0) {
        // per-ray SH rows (written by the stratified sampler): two 16-B loads, no evaluation
        const uint32_t ray = ray_of(a, pc) * (uint32_t)kShRecord + zero;
        const float4 u = *reinterpret_cast<const float4*>(a.sh + ray + 4 * h);
        const float4 v = *reinterpret_cast<const float4*>(a.sh + ray + 8 + 4 * h);
        shv[0] = u.x; shv[1] = u.y; shv[2] = u.z; shv[3] = u.w;   // tail lanes: the last point's (load_x6)
        shv[4] = v.x; shv[5] = v.y; shv[6] = v.z; shv[7] = v.w;
        return;
    }
    if (a.viewdirs) {
        const uint32_t ray = (pc < (uint32_t)a.seg_split ? pc / (uint32_t)a.spr
                                                         : (pc - (uint32_t)a.seg_split) / (uint32_t)a.spr2) * 3u + zero;
        sh4_eval(a.viewdirs[ray], a.viewdirs[ray + 1], a.viewdirs[ray + 2], o);
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) o[k] = a.sh[(uint32_t)(pc * (uint32_t)a.sh_stride + k + zero)];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {   // static indices + one select (a dynamic o[4h + k] is a 16-way select chain)
        const int k = (i & 3) + 8 * (i >> 2);
        shv[i] = h ? o[k + 4] : o[k];
    }
}

// The C0 operand of the point's SH: from the per-ray records' pre-split pieces (kShRecord layout:
// 16 fp32 coefficients, then pieces 0, 1, 2 of the 16 as bf16; two 8-B loads per piece), else split here
__device__ __forceinline__ S3 load_sh_split(const MlpArgs& a, uint32_t pt, bool valid, int h) {
    if (!a.viewdirs && a.sh_stride == 0) {
        const uint32_t pc = valid ? pt : (uint32_t)(a.P - 1);
        const uint16_t* rec = reinterpret_cast<const uint16_t*>(a.sh + ray_of(a, pc) * (uint32_t)kShRecord) + 32;
        S3 s;
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const u32x2 g0 = *reinterpret_cast<const u32x2*>(rec + 16 * q + 4 * h);
            const u32x2 g1 = *reinterpret_cast<const u32x2*>(rec + 16 * q + 8 + 4 * h);
            s.p[q] = u32x4{g0.x, g0.y, g1.x, g1.y};   // tail lanes: the last point's (load_x6)
        }
        return s;
    }
    float shv[8];
    load_sh6(a, pt, valid, h, shv, 0);
    return split_arr(shv);
}

__device__ __forceinline__ void load_in_x6(const MlpArgs& a, int64_t tile, int j, int h, InX6& in) {
    in.pt = (uint32_t)(tile * 32 + j);
    in.valid = tile * 32 + j < a.P;
    load_x6(a, in.pt, in.valid, h, in.x, 0);   // (nontemporal here too: bins +3 us, r05w — rejected)
    in.SH = load_sh_split(a, in.pt, in.valid, h);
}

// Row of point pt in raw / geo / graw / dgeo / dsh (MlpArgs point order)
__device__ __forceinline__ uint32_t io_row(const MlpArgs& a, uint32_t pt) {
    return a.io_rows ? (uint32_t)a.io_rows[pt] : pt;
}

// Backward tiles over the active points only (a.rows, MlpArgs): tile slot idx is point rows[idx]; the
// number of points is read on the device (graph-capturable: the list is built in the same stream).
__device__ __forceinline__ int64_t bwd_points(const MlpArgs& a) {
    return a.rows ? (int64_t)*a.count : a.P;
}

__device__ __forceinline__ void bwd_point(const MlpArgs& a, int64_t n, int64_t tile, int j, uint32_t& pt, bool& valid) {
    const int64_t idx = tile * 32 + j;
    valid = idx < n;
    if (a.rows) {
        pt = (uint32_t)a.rows[valid ? idx : n - 1];
    } else {
        pt = (uint32_t)idx;
    }
}

__device__ __forceinline__ void load_in_x6_bwd(const MlpArgs& a, int64_t n, int64_t tile, int j, int h, InX6& in) {
    bwd_point(a, n, tile, j, in.pt, in.valid);
    load_x6<NERF_X6_BWD_NT_FEAT != 0>(a, in.pt, in.valid, h, in.x, 0);
    in.SH = load_sh_split(a, in.pt, in.valid, h);
}

struct ActX6 {
    S3 xb[2];       // x's pieces (layer 0's B operand)
    floatx16 h1[2];
    floatx16 o;
    floatx16 h2[2];
    floatx16 h3[2];
    uint32_t m1;    // A-CAQ: ReLU mask of layer 0 before the activation quantizer
};

// layer 0: h1 = relu(W0 x) (A-CAQ: Q(relu(.)), m1 = its ReLU mask); lane = point j, half h
// (on the pieces of x, split by the caller: the backward stages them for dW0 as well)
template <bool QUANT>
__device__ __forceinline__ void layer0_split(const __bf16* img, const S3 (&xb)[2], floatx16 (&h1)[2], uint32_t& m1,
                                             int lane, const QuantRec& aq) {
    const int m = lane & 31, h = lane >> 5;
    h1[0] = h1[1] = zero16();
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int t = 0; t < 2; ++t) h1[t] = mma6(row_read(img, IM_W0, S32, 32 * t + m, 16 * c + 4 * h), xb[c], h1[t]);
    m1 = 0;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        relu16i(h1[t]);
        if constexpr (QUANT) {
#pragma unroll
            for (int r = 0; r < 16; ++r) m1 = relu_bit(m1, h1[t][r], 16 * t + r);
            fake_quant16(h1[t], aq);
        }
    }
}

template <bool QUANT>
__device__ __forceinline__ void layer0(const __bf16* img, const float (&x)[16], floatx16 (&h1)[2], uint32_t& m1,
                                       int lane, const QuantRec& aq) {
    const S3 xb[2] = {split_arr(x), split_arr(x + 8)};
    layer0_split<QUANT>(img, xb, h1, m1, lane, aq);
}

// One weight piece per row half of a 32-row A operand: lane m reads the row starting at element
// row_lo (m < 16) or row_hi (m >= 16), columns col0 + (i&3) + 8(i>>2)
__device__ __forceinline__ u32x4 row_read_pair(const __bf16* img, int row_lo, int row_hi, int m, int col0) {
    const int o0 = (m < 16 ? row_lo : row_hi) + col0;
    const u32x2 a = *reinterpret_cast<const u32x2*>(img + o0);
    const u32x2 b = *reinterpret_cast<const u32x2*>(img + o0 + 8);
    return u32x4{a.x, a.y, b.x, b.y};
}

// A 16-row layer (W1: o = W1 h1) on 32x32x16 tiles with the two row halves carrying different weight
// pieces: A01 = [a0 ; a1] and A2z = [a2 ; 0], so four MFMAs per k-chunk form the six x6 terms (and
// a1 b2): rows r and r + 16 of the accumulator hold the two partial sums (the caller adds them).
// The half-empty tile took six MFMAs per k-chunk.
__device__ __forceinline__ floatx16 mma4_rows16(const u32x4& A01, const u32x4& A2z, const S3& B, floatx16 c) {
    c = X6_MFMA(A2z, B.p[0], c);   // a2 b0 | 0
    c = X6_MFMA(A01, B.p[2], c);   // a0 b2 | a1 b2
    c = X6_MFMA(A01, B.p[1], c);   // a0 b1 | a1 b1
    c = X6_MFMA(A01, B.p[0], c);   // a0 b0 | a1 b0
    return c;
}

// rows 0..15 of a row-stacked accumulator: registers r and r + 8 of a lane hold rows R and R + 16
__device__ __forceinline__ floatx16 fold_rows16(const floatx16& acc) {
    floatx16 o = zero16();
#pragma unroll
    for (int r = 0; r < 8; ++r) o[r] = acc[r] + acc[r + 8];
    return o;
}

// forward chain up to h3 (the output layer C2 is the caller's: forward kernel rgb_c2); C1 = false: up to
// h2 only (the backward with the forward's saved h3)
struct NoHook {
    __device__ __forceinline__ void operator()() const {}
};
template <bool QUANT, bool C1 = true, typename BeforeC0 = NoHook>
__device__ __forceinline__ void fwd_chain(const __bf16* img, const InX6& in, ActX6& f, int lane, const QuantRec& aq,
                                          const BeforeC0& before_c0 = BeforeC0{}) {
    const int m = lane & 31, h = lane >> 5;
    f.xb[0] = split_arr(in.x);
    f.xb[1] = split_arr(in.x + 8);
    layer0_split<QUANT>(img, f.xb, f.h1, f.m1, lane, aq);
    // L1: o = W1 h1, row-stacked pieces; the zero half reads rows of C2's zero padding (rows 3..15)
    {
        floatx16 acc = zero16();
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const int col0 = 32 * t + 16 * c + 4 * h;
                const int r = IM_W1 + (m & 15) * S64;
                const u32x4 A01 = row_read_pair(img, r, IM_PIECE + r, m, col0);
                const u32x4 A2z = row_read_pair(img, 2 * IM_PIECE + r, IM_C2 + 8 * S64, m, col0);
                acc = mma4_rows16(A01, A2z, split_chunk(f.h1[t], c), acc);
            }
        f.o = fold_rows16(acc);
    }
    before_c0();
    // C0: h2 = relu(C0' [o rows 0..15 ; sh])
    f.h2[0] = f.h2[1] = zero16();
    {
        const S3 O0 = split_chunk(f.o, 0);
#pragma unroll
        for (int t = 0; t < 2; ++t) f.h2[t] = mma6(row_read(img, IM_C0, S32, 32 * t + m, 4 * h), O0, f.h2[t]);
    }
    {
#pragma unroll
        for (int t = 0; t < 2; ++t) f.h2[t] = mma6(row_read(img, IM_C0, S32, 32 * t + m, 16 + 4 * h), in.SH, f.h2[t]);
    }
    relu16i(f.h2[0]); relu16i(f.h2[1]);
    if constexpr (!C1) return;
    // C1: h3 = relu(C1 h2)
    f.h3[0] = f.h3[1] = zero16();
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const S3 hb = split_chunk(f.h2[t], c);
#pragma unroll
            for (int to = 0; to < 2; ++to)
                f.h3[to] = mma6(row_read(img, IM_C1, S64, 32 * to + m, 32 * t + 16 * c + 4 * h), hb, f.h3[to]);
        }
    relu16i(f.h3[0]); relu16i(f.h3[1]);
}

// Output layer rgb = C2 h3 (3 rows) in exact fp32 VALU: on 32-row tiles it used 3 of 32 rows and
// needed the h3 split (24 MFMAs + 176 VALU per tile). Lane (j, h) holds h3 at neurons
// 32t + row_of(r, h): it forms the three partial dot products over those 32 neurons (fp32 FMA chains,
// weights from an fp32 LDS image [h][o][32]: ds_read_b128 broadcasts), and two v_permlane32_swap
// exchanges add the lane halves' partials. Every lane ends with all three outputs of its point.
constexpr int C2F_FLOATS = 2 * 3 * 32;

__device__ inline void fill_c2f(float* c2f, const nerf_mlp_weights& W) {
    for (int idx = threadIdx.x; idx < C2F_FLOATS; idx += blockDim.x) {
        const int hh = idx / 96, o = (idx / 32) % 3, k = idx & 31;
        c2f[idx] = W.c2[o * 64 + 32 * (k >> 4) + row_of(k & 15, hh)];
    }
}

__device__ __forceinline__ float swap_half_sum(float lo, float hi, float& other) {
    // lanes 32..63 of `lo` trade places with lanes 0..31 of `hi`: afterwards lanes 0..31 hold
    // (lo_lo, lo_hi) and lanes 32..63 (hi_lo, hi_hi), so one add gives lo's half sum in the lower
    // lanes and hi's in the upper lanes
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(lo), __float_as_uint(hi), false, false);
    other = __uint_as_float(r[1]);
    return __uint_as_float(r[0]);
}

__device__ __forceinline__ void rgb_c2(const float* c2f, const floatx16 (&h3)[2], int h, float (&rgb)[3]) {
    const float4* w4 = reinterpret_cast<const float4*>(c2f + 96 * h);
    float p[3];
#pragma unroll
    for (int o = 0; o < 3; ++o) {
        float acc = 0.f;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const float4 w = w4[8 * o + q];
            const int k = 4 * q;
            acc = __builtin_fmaf(w.x, h3[k >> 4][k & 15], acc);
            acc = __builtin_fmaf(w.y, h3[(k + 1) >> 4][(k + 1) & 15], acc);
            acc = __builtin_fmaf(w.z, h3[(k + 2) >> 4][(k + 2) & 15], acc);
            acc = __builtin_fmaf(w.w, h3[(k + 3) >> 4][(k + 3) & 15], acc);
        }
        p[o] = acc;
    }
    float b, d;
    const float a = swap_half_sum(p[0], p[1], b);
    const float s01 = a + b;                       // lanes 0..31: rgb0, lanes 32..63: rgb1
    const float c = swap_half_sum(p[2], p[2], d);
    rgb[2] = c + d;                                // every lane
    float e;
    rgb[0] = swap_half_sum(s01, s01, e);           // the lower lanes' value, in every lane
    rgb[1] = e;
}

// Stage 1's ga3 = C2^T g_rgb (3 live k rows) on the exact fp32 matrix core (v_mfma_f32_32x32x2_f32):
// two k = 2 MFMAs per 32-row tile (k = r, g | b, 0) replace six x6 MFMAs of a 16-deep k-chunk, and
// no operand is split. A operand of tile t, MFMA m: lane (i, h) holds C2[2m + h][32t + i] (0 past
// the three rows), stored [t][lane][m] so one ds_read_b64 per tile fetches both; B operand: lane
// (j, h) holds g_rgb[2m + h] of point j. The accumulator layout equals the bf16 MFMA's.
#ifndef NERF_X6_GA3_F32
#define NERF_X6_GA3_F32 1
#endif
constexpr int C2B_FLOATS = 2 * 64 * 2;

__device__ inline void fill_c2b(float* c2b, const nerf_mlp_weights& W) {
    for (int idx = threadIdx.x; idx < C2B_FLOATS; idx += blockDim.x) {
        const int t = idx >> 7, ln = (idx >> 1) & 63, m = idx & 1, k = 2 * m + (ln >> 5);
        c2b[idx] = k < 3 ? W.c2[k * 64 + 32 * t + (ln & 31)] : 0.f;
    }
}

__device__ __forceinline__ floatx16 ga3_f32(const float* c2b, int t, float b0, float b1, int lane) {
    const float2 a = *reinterpret_cast<const float2*>(c2b + 2 * (64 * t + lane));
    floatx16 c = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b0, zero16(), 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b1, c, 0, 0, 0);
}

// Saved C1 outputs (training forward -> backward): per 32-point tile the 2 x 16 h3 registers of every lane
// as float4 groups, [tile][t][q][lane][4] (one coalesced 16-B access per lane and group; 256 B per
// point). The backward then skips C1's recompute (48 of the chain wave's MFMAs and the h2 split, 176
// VALU, per tile). Nontemporal both ways: the buffer is written once and read once.
typedef float f32x4_nt __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t h3_off(int64_t tile, int t, int q, int lane) {
    return (((((uint32_t)tile * 2u + (uint32_t)t) * 4u + (uint32_t)q) * 64u) + (uint32_t)lane) * 4u;
}

// ================================================================ forward kernel
template <bool QUANT>
// 512-thread blocks: the 66.8 KB weight image is shared by 8 waves, so two blocks per CU give 4
// waves per SIMD (105 VGPRs) instead of 2 with 256-thread blocks
__global__ void __launch_bounds__(512, 2) mlp_fwd_x6_kernel(MlpArgs a) {
    __shared__ __attribute__((aligned(16))) __bf16 img[3 * IM_PIECE];
    __shared__ __attribute__((aligned(16))) float c2f[C2F_FLOATS];
    fill_images(img, a.W);
    fill_c2f(c2f, a.W);
    __syncthreads();
    const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
    QuantRec aq{};
    if constexpr (QUANT) aq = *a.aq;
    const int64_t n_tiles = (a.P + 31) / 32;
    const int wpb = blockDim.x >> 6;
    for (int64_t tile = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6); tile < n_tiles; tile += (int64_t)gridDim.x * wpb) {
        InX6 in;
        load_in_x6(a, tile, j, h, in);
        ActX6 f;
        const int z = opaque_zero();
        fwd_chain<QUANT>(img + z, in, f, lane, aq);
        if constexpr (!QUANT) {
            if (a.h3) {
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        __builtin_nontemporal_store(f32x4_nt{f.h3[t][4 * q], f.h3[t][4 * q + 1], f.h3[t][4 * q + 2],
                                                             f.h3[t][4 * q + 3]},
                                                    reinterpret_cast<f32x4_nt*>(a.h3 + h3_off(tile, t, q, lane)));
            }
        }
        float rgb[3];
        rgb_c2(c2f + z, f.h3, h, rgb);
        const uint32_t orow = in.valid ? io_row(a, in.pt) : 0u;
        if (h == 0 && in.valid) {
            const bool keep = a.keep ? a.keep[in.pt] != 0 : true;
            *reinterpret_cast<float4*>(a.raw + 4u * orow) = make_float4(rgb[0], rgb[1], rgb[2], keep ? f.o[0] : 0.f);
        }
        if (a.geo_out && in.valid) {
#pragma unroll
            for (int r = 0; r < 8; ++r) a.geo_out[16u * orow + row_of(r, h)] = f.o[r];
        }
    }
}

// Calibration-only launch of the activation quantizer (quantization.py:97-119 on the first
// netchunk's h = relu(x W0^T), run_nerf_helpers.py:280-284): layer 0 per tile, wave min/max, one
// atomic pair per wave (order-preserving u32 images of the floats).
__global__ void __launch_bounds__(512, 2) mlp_act_minmax_x6_kernel(MlpArgs a) {
    __shared__ __attribute__((aligned(16))) __bf16 img[3 * IM_PIECE];
    fill_images(img, a.W);
    __syncthreads();
    const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
    const int64_t n = a.calib_points < a.P ? a.calib_points : a.P;
    const int64_t n_tiles = (n + 31) / 32;
    const int wpb = blockDim.x >> 6;
    float lo = INFINITY, hi = -INFINITY;
    for (int64_t tile = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6); tile < n_tiles; tile += (int64_t)gridDim.x * wpb) {
        const uint32_t pt = (uint32_t)(tile * 32 + j);
        const bool valid = tile * 32 + j < n;
        float x[16];
        load_x6(a, pt, valid, h, x, 0);
        floatx16 h1[2];
        uint32_t m1;
        layer0<false>(img + opaque_zero(), x, h1, m1, lane, QuantRec{});
        if (valid) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                lo = fminf(lo, fminf(h1[0][r], h1[1][r]));
                hi = fmaxf(hi, fmaxf(h1[0][r], h1[1][r]));
            }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        lo = fminf(lo, __shfl_xor(lo, o, 64));
        hi = fmaxf(hi, __shfl_xor(hi, o, 64));
    }
    if (lane == 0 && lo <= hi) {
        atomicMin(a.act_minmax, f2ord(lo));
        atomicMax(a.act_minmax + 1, f2ord(hi));
    }
}

// ================================================================ backward, split roles
// The one-wave-per-tile backward above runs at one wave per SIMD (its chain state and the twelve
// dW accumulator tiles need ~470 registers), so every VALU split, LDS latency and dependent MFMA
// of the tile is exposed. Here each tile is shared by a PAIR of waves on the same SIMD (waves p
// and p + 4 of a 512-thread block): the chain wave runs the forward recompute and the transposed
// chain and stages each (gradient tile, activation tile) pair; the wgrad wave holds the dW tiles
// and turns each staged pair into six-MFMA products. Two waves per SIMD (256 registers each) let
// one wave's VALU work hide under the other's MFMAs.
// Hand-off per pair, over the pair's single staging buffer, with two LDS sequence counters:
// the chain wave waits for ack == k - 1 before it writes stage k and then stores ready = k
// (release: its staging writes are complete first); the wgrad wave waits for ready == k, reads
// the stage and stores ack = k (release: its reads have returned). Both waves walk the same tile
// list with the same seven stages per tile, so every wait is matched and the loop ends together.
constexpr int CG_STAGES = 7;

#ifdef NERF_X6CG_PROF   // diagnostic build only: wait / loop cycles of the chain and wgrad waves
__device__ unsigned long long cg_prof[4];
__device__ unsigned long long cg_stage_wait[8];   // chain wave's wait before each stage of a tile
#define CG_T() __builtin_amdgcn_s_memtime()
#endif

__device__ __forceinline__ void flag_wait(int* f, int v, unsigned long long* waited = nullptr) {
#ifdef NERF_X6CG_PROF
    const unsigned long long t0 = CG_T();
#endif
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < v) __builtin_amdgcn_s_sleep(1);
#ifdef NERF_X6CG_PROF
    *waited += CG_T() - t0;
#else
    (void)waited;
#endif
}
__device__ __forceinline__ void flag_set(int* f, int v) {
    __hip_atomic_store(f, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// ... and with a scheduling barrier behind it, so that the compiler cannot hoist the MFMAs that
// follow above the store (they do not depend on it), which would hold the partner wave for
// their whole duration.
__device__ __forceinline__ void flag_set_now(int* f, int v) {
    __hip_atomic_store(f, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    __builtin_amdgcn_sched_barrier(0);
}

// fp32 activation staging of the split-role backward: [64 neurons][SPF] fp32, column = point.
// The chain wave stores its activation tiles unsplit (one ds_write_b32 per value); the wgrad wave
// reads each operand fragment with two ds_read_b128, releases the buffer and only then splits it
// into bf16 pieces, so the split of every staged activation runs on the wave that otherwise waits
// (measured with NERF_X6CG_PROF before: chain wave busy 75 %, wgrad wave 28 %).
constexpr int SPF = 36;                                   // row stride: conflict-free b128 reads
constexpr int ACTF_FLOATS = 64 * SPF;                     // 9,216 B
// per wave pair: the activation image and TWO gradient buffers (stage k uses buffer k & 1)
constexpr int ST_CG = 2 * ACTF_FLOATS + 6 * STG_PIECE;    // bf16 elements (23,040 B)
constexpr int X6_CG_LDS = IM_BYTES + 4 * ST_CG * 2;       // 158,976 B
// and behind it a zero block of 16 rows x S32 (1,152 B): the zero half of row-stacked transposed
// A operands (tr_read_pair)
constexpr int X6_ZBLK = X6_CG_LDS / 2;                    // element offset from the image
constexpr int X6_ZBLK_ELEMS = 16 * S32;

__device__ __forceinline__ void stage_tileF(float* actF, const floatx16& v, int row0, int j, int h) {
#pragma unroll
    for (int r = 0; r < 16; ++r) actF[(row0 + row_of(r, h)) * SPF + j] = v[r];
}

// element i of v <-> neuron row0 + 4h + (i&3) + 8(i>>2)
__device__ __forceinline__ void stage_arrF(float* actF, const float* v, int row0, int j, int h) {
#pragma unroll
    for (int i = 0; i < 8; ++i) actF[(row0 + 4 * h + (i & 3) + 8 * (i >> 2)) * SPF + j] = v[i];
}

template <bool QUANT, bool SAVED>
__device__ __forceinline__ void bwd_chain_role(const MlpArgs& a, const __bf16* img, __bf16* stA, __bf16* stG,
                                               int* ready, int* ack, int p, int lane, const QuantRec& aq, int blk,
                                               int nblk, const float* c2b) {
    const int j = lane & 31, h = lane >> 5;
    float* actF = reinterpret_cast<float*>(stA);
    int seq = 0;
    unsigned long long waited = 0;
#ifdef NERF_X6CG_PROF
    const unsigned long long t_start = CG_T();
#endif
    // stage k writes gradient buffer k & 1 (and, when it stages activations, the one activation
    // buffer): it may start once the wgrad wave has released stage k - 2 (k - 1 with activations)
#ifdef NERF_X6CG_PROF
    unsigned long long sw[CG_STAGES] = {};
    auto open = [&](bool act, int k) {   // k: the stage (1..7) of the tile, a constant after unrolling
        unsigned long long w = 0;
        flag_wait(ack, act ? seq : seq - 1, &w);
        waited += w;
        sw[k - 1] += w;
    };
#else
    auto open = [&](bool act, int) { flag_wait(ack, act ? seq : seq - 1, &waited); };
#endif
    __bf16* const stGb[2] = {stG, stG + 3 * STG_PIECE};
    auto publish = [&]() { flag_set(ready, ++seq); };
    const int64_t n_pts = bwd_points(a);
    const int64_t n_tiles = (n_pts + 31) / 32;
#if NERF_X6_BWD_PREFETCH
    // the next tile's inputs are loaded after stage 5 (the forward state is dead by then) and are in
    // flight during stages 6 and 7 instead of stalling the next tile's forward recompute
    InX6 in_next;
    if ((int64_t)blk * 4 + p < n_tiles) load_in_x6_bwd(a, n_pts, (int64_t)blk * 4 + p, j, h, in_next);
#endif
    for (int64_t tile = (int64_t)blk * 4 + p; tile < n_tiles; tile += (int64_t)nblk * 4) {
        const __bf16* imt = img + opaque_zero();
#if NERF_X6_BWD_PREFETCH
        InX6 in = in_next;
#else
        InX6 in;
        load_in_x6_bwd(a, n_pts, tile, j, h, in);
#endif
        ActX6 f;
        if constexpr (SAVED) {   // h3 from the forward, the loads in flight during layer C0 (issued before
            f32x4_nt h3v[8];     // layer 0 or after the chain instead: the same time, profiles/r06d_ab_saved_h3.jsonl;
                                 // one tile ahead with the inputs: spills, 360 -> 452 us, tools/variants/)
            auto load_h3 = [&]() {
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    h3v[k] = __builtin_nontemporal_load(
                        reinterpret_cast<const f32x4_nt*>(a.h3 + h3_off(tile, k >> 2, k & 3, lane)));
            };
            fwd_chain<QUANT, false>(imt, in, f, lane, aq, load_h3);
#pragma unroll
            for (int k = 0; k < 8; ++k)
#pragma unroll
                for (int e = 0; e < 4; ++e) f.h3[k >> 2][4 * (k & 3) + e] = h3v[k][e];
        } else {
            fwd_chain<QUANT>(imt, in, f, lane, aq);
        }

        const uint32_t orow = io_row(a, in.valid ? in.pt : (uint32_t)(a.P - 1));
        float4 g4 = *reinterpret_cast<const float4*>(a.graw + 4u * orow);
        if (!in.valid) g4 = make_float4(0.f, 0.f, 0.f, 0.f);
        const bool keep = in.valid && (a.keep ? a.keep[in.pt] != 0 : true);
        const float gsig = keep ? g4.w : 0.f;

        // stage 1 (dC2): g_rgb, h3
        floatx16 ga3[2];
        {
            const S3 GR = h ? split8(0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f)
                            : split8(g4.x, g4.y, g4.z, 0.f, 0.f, 0.f, 0.f, 0.f);
            open(true, 1);
            stage_grad(stGb[1], GR, 0, j, h);      // columns 16..31 stale: they only reach dC2 rows >= 16
#pragma unroll
            for (int t = 0; t < 2; ++t) stage_tileF(actF, f.h3[t], 32 * t, j, h);
            publish();
#if NERF_X6_GA3_F32
            const float b0 = h ? g4.y : g4.x, b1 = h ? 0.f : g4.z;
            (void)imt;
#endif
#pragma unroll
            for (int t = 0; t < 2; ++t) {
#if NERF_X6_GA3_F32
                ga3[t] = ga3_f32(c2b + opaque_zero(), t, b0, b1, lane);
#else
                ga3[t] = mma6(tr_read(imt, IM_PIECE, IM_C2, S64, 0, 32 * t, lane), GR, zero16());
#endif
#pragma unroll
                for (int r = 0; r < 16; ++r) ga3[t][r] = f.h3[t][r] > 0.f ? ga3[t][r] : 0.f;
            }
        }
        // stages 2, 3 (dC1 rows 32t..): ga3 tile t, h2
        floatx16 ga2[2];
        ga2[0] = ga2[1] = zero16();
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const S3 g0 = split_chunk(ga3[t], 0), g1 = split_chunk(ga3[t], 1);
            open(t == 0, 2 + t);
            if (t == 0) {
#pragma unroll
                for (int ta = 0; ta < 2; ++ta) stage_tileF(actF, f.h2[ta], 32 * ta, j, h);
            }
            stage_grad(stGb[t], g0, 0, j, h);
            stage_grad(stGb[t], g1, 1, j, h);
            publish();
#pragma unroll
            for (int ti = 0; ti < 2; ++ti) {
                ga2[ti] = mma6(tr_read(imt, IM_PIECE, IM_C1, S64, 32 * t, 32 * ti, lane), g0, ga2[ti]);
                ga2[ti] = mma6(tr_read(imt, IM_PIECE, IM_C1, S64, 32 * t + 16, 32 * ti, lane), g1, ga2[ti]);
            }
        }
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) ga2[t][r] = f.h2[t][r] > 0.f ? ga2[t][r] : 0.f;

        // stages 4, 5 (dC0 rows 32t..): ga2 tile t, [o ; sh]
        floatx16 go = zero16();
        if (h == 0) go[0] = gsig;
        if (a.dgeo && in.valid) {
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int row = row_of(r, h);
                if (row >= 1) go[r] = a.dgeo[16u * orow + row];
            }
        }
        // without an SH gradient only rows 0..15 of go (sigma, geo) are live: their A operand C0'^T
        // is row-stacked as in fwd_chain's W1 layer (four MFMAs per k-chunk instead of six)
        const bool stack = a.dsh == nullptr;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const S3 g0 = split_chunk(ga2[t], 0), g1 = split_chunk(ga2[t], 1);
            open(t == 0, 4 + t);
            if (t == 0) {
#pragma unroll
                for (int r = 0; r < 8; ++r) actF[row_of(r, h) * SPF + j] = f.o[r];
                float shv[8];
                load_sh6(a, in.pt, in.valid, h, shv, opaque_zero());   // re-evaluated: nothing is kept across stages
                stage_arrF(actF, shv, 16, j, h);
            }
            stage_grad(stGb[t], g0, 0, j, h);
            stage_grad(stGb[t], g1, 1, j, h);
            publish();
            if (stack) {
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const int row0 = IM_C0 + (32 * t + 16 * c) * S32;
                    const u32x4 A01 = tr_read_pair(imt, row0, IM_PIECE + row0, lane);
                    const u32x4 A2z = tr_read_pair(imt, 2 * IM_PIECE + row0, X6_ZBLK, lane);
                    go = mma4_rows16(A01, A2z, c ? g1 : g0, go);
                }
            } else {
                go = mma6(tr_read(imt, IM_PIECE, IM_C0, S32, 32 * t, 0, lane), g0, go);
                go = mma6(tr_read(imt, IM_PIECE, IM_C0, S32, 32 * t + 16, 0, lane), g1, go);
            }
        }
        if (stack) go = fold_rows16(go);
        if (a.dsh && in.valid) {
#pragma unroll
            for (int r = 8; r < 16; ++r) a.dsh[16u * orow + row_of(r, h) - 16] = go[r];
        }

#if NERF_X6_BWD_PREFETCH
        if (tile + (int64_t)nblk * 4 < n_tiles) load_in_x6_bwd(a, n_pts, tile + (int64_t)nblk * 4, j, h, in_next);
#endif
        // stage 6 (dW1): go, h1 (held in registers since the forward recompute; with QUANT recomputed
        // from x's pieces) and layer 0's ReLU mask m1 (with QUANT: before the activation quantizer)
        // in the unused columns 16.. of the gradient tile.
        // The wgrad wave forms ga1 = mask(W1^T go) itself (it waits on the chain wave otherwise).
        // x's bf16 pieces, split once by fwd_chain and held since, are staged at stage 7 (the wgrad
        // wave does not split x; no reload of the features: 4 B/lane of spills, MLP backward 380 ->
        // 375 us per launch, profiles/r05d_ab_bench.jsonl)
        S3 xb[2] = {f.xb[0], f.xb[1]};
        {
            floatx16 h1[2];
            uint32_t m1;
            if constexpr (QUANT) {
                layer0_split<QUANT>(imt, xb, h1, m1, lane, aq);   // kept live, the quantizer state spills
            } else {
                h1[0] = f.h1[0];   // layer 0's output of the forward recompute, live since (24 MFMAs and
                h1[1] = f.h1[1];   // the ReLUs fewer than recomputing it here; no spills without QUANT)
                m1 = 0;
            }
            const S3 GO = split_chunk(go, 0);
            open(true, 6);
#pragma unroll
            for (int t = 0; t < 2; ++t) stage_tileF(actF, h1[t], 32 * t, j, h);
            stage_grad(stGb[0], GO, 0, j, h);      // columns 16..31 stale: they only reach dW1 rows >= 16
            if constexpr (!QUANT) {
                m1 = 0;
#pragma unroll
                for (int t = 0; t < 2; ++t)
#pragma unroll
                    for (int r = 0; r < 16; ++r) m1 = relu_bit(m1, h1[t][r], 16 * t + r);
            }
            *reinterpret_cast<uint32_t*>(stGb[0] + j * S32 + 16 + 2 * h) = m1;
            publish();
        }
        // stage 7 (dW0): x, as its bf16 pieces in a [32 points][S32] image in the activation buffer
        open(true, 7);
        stage(stA, STG_PIECE, S32, xb[0], 0, 0, j, h);
        stage(stA, STG_PIECE, S32, xb[1], 0, 1, j, h);
        publish();
    }
#ifdef NERF_X6CG_PROF
    if (lane == 0) {
        atomicAdd(&cg_prof[0], waited);
        atomicAdd(&cg_prof[1], CG_T() - t_start);
        for (int k = 0; k < CG_STAGES; ++k) atomicAdd(&cg_stage_wait[k], sw[k]);
    }
#endif
}

// The wgrad wave's operands. C2 (3 rows) and W1 (16 rows) use v_mfma_f32_16x16x32_bf16 tiles
// (16 rows x 16 columns, all 32 points in one k step): half the matrix-pipe time and half the
// accumulator registers of 32-row tiles. For a 16x16x32 operand lane l holds row/column
// col0 + (l & 15) at the 8 points 4g + (i & 3) + 16(i >> 2), g = l >> 4 (any point permutation
// works as long as both operands use the same one).
typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ S3 tr_read16(const __bf16* st, int piece, int S, int col0, int lane) {
    const int g = lane >> 4, il = lane & 15, q = il >> 2, p = il & 3;
    const int oa = (4 * g + q) * S + col0 + 4 * p;
    S3 s;
#pragma unroll
    for (int pc = 0; pc < 3; ++pc) {
        const bf16x4 ta = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(st + pc * piece + oa));
        const bf16x4 tb = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(st + pc * piece + oa + 16 * S));
        const u32x2 a = __builtin_bit_cast(u32x2, ta), b = __builtin_bit_cast(u32x2, tb);
        s.p[pc] = u32x4{a.x, a.y, b.x, b.y};
    }
    return s;
}

#define X6_MFMA16(a, b, c) \
    __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, (a)), __builtin_bit_cast(bf16x8, (b)), (c), 0, 0, 0)

__device__ __forceinline__ floatx4 mma6_16(const S3& A, const S3& B, floatx4 c) {
    c = X6_MFMA16(A.p[0], B.p[2], c);
    c = X6_MFMA16(A.p[2], B.p[0], c);
    c = X6_MFMA16(A.p[1], B.p[1], c);
    c = X6_MFMA16(A.p[0], B.p[1], c);
    c = X6_MFMA16(A.p[1], B.p[0], c);
    c = X6_MFMA16(A.p[0], B.p[0], c);
    return c;
}

struct WgradX6 {
    floatx4 dC2[4], dW1[4];                      // 16x16 tiles: rows 0..15, columns 16u..16u+15
    floatx16 dC1[2][2], dC0[2][1], dW0[2][1];    // 32x32 tiles
};

// A 16-row stage: G columns 0..15 against the 64 staged activation columns.
// Raw fp32 activation fragments (8 values), split into pieces after the buffer is released.
struct Raw8 {
    float4 a, b;
};
__device__ __forceinline__ S3 split_raw(const Raw8& v) {
    return split8(v.a.x, v.a.y, v.a.z, v.a.w, v.b.x, v.b.y, v.b.z, v.b.w);
}
// 32x32x16 B operand: lane (m, h) <-> neuron col0 + m at points row0 + 4h + (i&3) + 8(i>>2)
__device__ __forceinline__ Raw8 act_read32(const float* actF, int row0, int col0, int lane) {
    const float* q = actF + (col0 + (lane & 31)) * SPF + row0 + 4 * (lane >> 5);
    return Raw8{*reinterpret_cast<const float4*>(q), *reinterpret_cast<const float4*>(q + 8)};
}
// 16x16x32 B operand: lane l <-> neuron col0 + (l & 15) at points 4(l >> 4) + (i&3) + 16(i>>2)
__device__ __forceinline__ Raw8 act_read16(const float* actF, int col0, int lane) {
    const float* q = actF + (col0 + (lane & 15)) * SPF + 4 * (lane >> 4);
    return Raw8{*reinterpret_cast<const float4*>(q), *reinterpret_cast<const float4*>(q + 16)};
}

struct Ops16 {
    S3 A;
    Raw8 B[4];
};
__device__ __forceinline__ void read16(Ops16& o, const __bf16* stG, const float* actF, int lane) {
    o.A = tr_read16(stG, STG_PIECE, S32, 0, lane);
#pragma unroll
    for (int u = 0; u < 4; ++u) o.B[u] = act_read16(actF, 16 * u, lane);
}
__device__ __forceinline__ void mma16(floatx4 (&acc)[4], const Ops16& o) {
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = mma6_16(o.A, split_raw(o.B[u]), acc[u]);
}

// A 32-row stage (NU activation tiles of 32 columns), operands for both 16-point chunks.
template <int NU>
struct Ops32 {
    S3 A[2];
    Raw8 B[2][NU];
};
template <int NU>
__device__ __forceinline__ void read32(Ops32<NU>& o, const __bf16* stG, const float* actF, int lane) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        o.A[c] = tr_read(stG, STG_PIECE, 0, S32, 16 * c, 0, lane);
#pragma unroll
        for (int u = 0; u < NU; ++u) o.B[c][u] = act_read32(actF, 16 * c, 32 * u, lane);
    }
}
template <int NU>
__device__ __forceinline__ void mma32(floatx16 (&acc)[NU], const Ops32<NU>& o) {
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int u = 0; u < NU; ++u) acc[u] = mma6(o.A[c], split_raw(o.B[c][u]), acc[u]);
}

// Every stage: wait for it, read all of its operands, release the buffer (ack), then run the MFMAs,
// so the chain wave's next staging overlaps them.
template <bool QUANT>
__device__ __forceinline__ void bwd_wgrad_role(const MlpArgs& a, const __bf16* img, const __bf16* stA,
                                               __bf16* stG, int* ready, int* ack, int p, int lane, WgradX6& g,
                                               int blk, int nblk) {
    const int j = lane & 31, h = lane >> 5;
    const float* actF = reinterpret_cast<const float*>(stA);
#pragma unroll
    for (int u = 0; u < 4; ++u) { g.dC2[u] = floatx4{0.f, 0.f, 0.f, 0.f}; g.dW1[u] = floatx4{0.f, 0.f, 0.f, 0.f}; }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        g.dC0[i][0] = zero16(); g.dW0[i][0] = zero16();
        g.dC1[i][0] = zero16(); g.dC1[i][1] = zero16();
    }
    int seq = 0;
    unsigned long long waited = 0;
#ifdef NERF_X6CG_PROF
    const unsigned long long t_start = CG_T();
#endif
    auto take = [&]() { flag_wait(ready, seq + 1, &waited); };
    auto release = [&]() { flag_set_now(ack, ++seq); };
    const int64_t n_pts = bwd_points(a);
    const int64_t n_tiles = (n_pts + 31) / 32;
    for (int64_t tile = (int64_t)blk * 4 + p; tile < n_tiles; tile += (int64_t)nblk * 4) {
        {   // 1: dC2
            Ops16 o;
            take(); read16(o, stG + 3 * STG_PIECE, actF, lane); release();
            mma16(g.dC2, o);
        }
        // 2 + 3: dC1 for both ga3 tiles against ONE split of h2 (per 16-point chunk c: the two h2
        // fragments split once, both gradient tiles' fragments read), released after the last reads.
        // Splitting h2 once instead of once per ga3 tile: 413 -> 401 us per launch (tools/mlp_ab.py).
        // The same merge of stages 4 + 5 (dC0) is slower (the later release holds the chain wave:
        // 414 -> 422 us), and x split once for both dW0 tiles does not move the launch.
        seq += 1;
        take();
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            Raw8 hr[2];
            S3 A[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) hr[u] = act_read32(actF, 16 * c, 32 * u, lane);
#pragma unroll
            for (int t = 0; t < 2; ++t) A[t] = tr_read(stG + t * 3 * STG_PIECE, STG_PIECE, 0, S32, 16 * c, 0, lane);
            if (c == 1) release();
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const S3 hb = split_raw(hr[u]);
#pragma unroll
                for (int t = 0; t < 2; ++t) g.dC1[t][u] = mma6(A[t], hb, g.dC1[t][u]);
            }
        }
        {   // 4, 5: dC0 for both ga2 tiles against ONE split of [o ; sh] (staged once, at stage 4)
            S3 B[2], A[2];
            take();
#pragma unroll
            for (int c = 0; c < 2; ++c) A[c] = tr_read(stG, STG_PIECE, 0, S32, 16 * c, 0, lane);
            Raw8 br[2];
#pragma unroll
            for (int c = 0; c < 2; ++c) br[c] = act_read32(actF, 16 * c, 0, lane);
            release();
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                B[c] = split_raw(br[c]);
                g.dC0[0][0] = mma6(A[c], B[c], g.dC0[0][0]);
            }
            take();
#pragma unroll
            for (int c = 0; c < 2; ++c) A[c] = tr_read(stG + 3 * STG_PIECE, STG_PIECE, 0, S32, 16 * c, 0, lane);
            release();
#pragma unroll
            for (int c = 0; c < 2; ++c) g.dC0[1][0] = mma6(A[c], B[c], g.dC0[1][0]);
        }
        // 6: dW1, and ga1 = W1^T go masked by layer 0's ReLU (go read in the B layout: lane = point).
        // From here until stage 7 is released both gradient buffers are this wave's (the chain wave
        // stages only x at stage 7, and its next gradient write waits for stage 7's release): ga1 is
        // staged there, tile t in buffer 1 - t, for dW0 and gx = W0^T ga1 (the d features).
        floatx16 gx = zero16();
        {
            Ops16 o;
            take();
            read16(o, stG, actF, lane);   // stage 6: gradient buffer 0
            const S3 GOb = row_read_st(stG, STG_PIECE, S32, j, 4 * h);
            const uint32_t m1 = *reinterpret_cast<const uint32_t*>(stG + j * S32 + 16 + 2 * h);
            release();
            mma16(g.dW1, o);
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                floatx16 ga1 = mma6(tr_read(img, IM_PIECE, IM_W1, S64, 0, 32 * t, lane), GOb, zero16());
#pragma unroll
                for (int r = 0; r < 16; ++r) ga1[r] = ((m1 >> (16 * t + r)) & 1u) ? ga1[r] : 0.f;
                stage_grad(stG + (1 - t) * 3 * STG_PIECE, split_chunk(ga1, 0), 0, j, h);
                stage_grad(stG + (1 - t) * 3 * STG_PIECE, split_chunk(ga1, 1), 1, j, h);
            }
        }
        take();   // 7: dW0 = ga1 x^T and gx = W0^T ga1 (B = the staged ga1, lane = point)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            S3 A[2], X[2], gb[2];
            const __bf16* sg = stG + (1 - t) * 3 * STG_PIECE;
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                A[c] = tr_read(sg, STG_PIECE, 0, S32, 16 * c, 0, lane);
                X[c] = tr_read(stA, STG_PIECE, 0, S32, 16 * c, 0, lane);   // x pieces (k = point)
                gb[c] = row_read_st(sg, STG_PIECE, S32, j, 16 * c + 4 * h);
            }
            if (t == 1) flag_set(ack, ++seq);
#pragma unroll
            for (int c = 0; c < 2; ++c) g.dW0[t][0] = mma6(A[c], X[c], g.dW0[t][0]);
#pragma unroll
            for (int c = 0; c < 2; ++c) gx = mma6(tr_read(img, IM_PIECE, IM_W0, S32, 32 * t + 16 * c, 0, lane), gb[c], gx);
        }
        uint32_t pt;
        bool pvalid;
        bwd_point(a, n_pts, tile, j, pt, pvalid);
        if (a.dfeat && pvalid) {
            // offsets formed per tile (opaque stride): hoisted out of the loop they pin 16 registers
            const uint32_t sl = (uint32_t)a.dsl + (uint32_t)opaque_zero(), base = pt * (uint32_t)a.dsp;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int fi = row_of(r, h);
                a.dfeat[base + (fi >> 1) * sl + (fi & 1)] = gx[r];   // default policy: the bins read it next
                                                                       // (nontemporal: bins 176 -> 205 us, r05x)
            }
        }
    }
    static_assert(CG_STAGES == 7, "stage list above");
#ifdef NERF_X6CG_PROF
    if (lane == 0) { atomicAdd(&cg_prof[2], waited); atomicAdd(&cg_prof[3], CG_T() - t_start); }
#endif
}

// Up to two nets per launch: the coarse and the fine pass of an iteration are separate NeRFSmall
// instances (run_nerf.py:254-259) whose backwards are both ready when autograd reaches the first of
// them (field.py defers them to the end of the pass). Blocks [0, split) run job 0 and the others
// job 1, each block on its own net's weight image and tiles, so the per-launch fixed costs (weight
// image build, chain / wgrad pipeline fill and drain, block reduction tail) are paid once per step.
struct MlpBwdJobs {
    MlpArgs a[2];
    int split;       // blocks of job 0
    float* det_ws;   // deterministic mode: per-block weight-gradient images [gridDim.x][GW_TOTAL]
};

template <bool QUANT, bool SAVED>
__global__ void __launch_bounds__(512, 1) mlp_bwd_x6cg_kernel(MlpBwdJobs jobs) {
    __shared__ __attribute__((aligned(16))) __bf16 lds[X6_CG_LDS / 2 + X6_ZBLK_ELEMS];
    __shared__ int flags[8];   // ready[0..3], ack[0..3]
    __shared__ __attribute__((aligned(16))) float c2b[C2B_FLOATS];
    const bool second = (int)blockIdx.x >= jobs.split;
    const MlpArgs& a = second ? jobs.a[1] : jobs.a[0];
    const int blk = second ? (int)blockIdx.x - jobs.split : (int)blockIdx.x;
    const int nblk = second ? (int)gridDim.x - jobs.split : jobs.split;
    __bf16* img = lds;
    const int wv = threadIdx.x >> 6, p = wv & 3;
    const bool wgrad_wave = wv >= 4;
    __bf16* stA = lds + 3 * IM_PIECE + p * ST_CG;   // fp32 activation image (actF)
    __bf16* stG = stA + 2 * ACTF_FLOATS;
    fill_images(img, a.W);
    fill_c2b(c2b, a.W);
    for (int i = threadIdx.x; i < X6_ZBLK_ELEMS / 2; i += blockDim.x) reinterpret_cast<uint32_t*>(img + X6_ZBLK)[i] = 0u;
    if (threadIdx.x < 8) flags[threadIdx.x] = 0;
    __syncthreads();

    const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
    WgradX6 g;   // defined (and live) on the wgrad waves only
    if (wgrad_wave) {
        bwd_wgrad_role<QUANT>(a, img, stA, stG, flags + p, flags + 4 + p, p, lane, g, blk, nblk);
    } else {
        QuantRec aq{};
        if constexpr (QUANT) aq = *a.aq;
        bwd_chain_role<QUANT, SAVED>(a, img, stA, stG, flags + p, flags + 4 + p, p, lane, aq, blk, nblk, c2b);
    }

    // ---- block reduction of the wgrad waves' tiles, one global flush per block. Each wgrad wave
    // writes its full weight-gradient image (every index exactly once: the tile maps are fixed) into
    // its own LDS copy with plain stores; then all 512 threads sum the four copies in a fixed order.
    // LDS fp32 atomics here (one ds_add_f32 per value and wave into a shared image) cost 49 us per
    // launch.
    static_assert(4 * GW_TOTAL * (int)sizeof(float) <= X6_CG_LDS, "four weight-gradient images must fit the LDS");
    __syncthreads();
    float* gw = reinterpret_cast<float*>(lds);
    if (wgrad_wave) {
        float* mine = gw + p * GW_TOTAL;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int rr = row_of(r, h);
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const int row = 32 * t + rr;
#pragma unroll
                for (int u = 0; u < 2; ++u) mine[GW_C1 + row * 64 + 32 * u + j] = g.dC1[t][u][r];
                if (j != 0) mine[GW_C0 + row * 31 + (j < 16 ? 15 + j : j - 16)] = g.dC0[t][0][r];
                mine[GW_W0 + row * 32 + j] = g.dW0[t][0][r];
            }
        }
        // 16x16 tiles: lane l holds rows 4(l >> 4) + i, column 16u + (l & 15)
        const int r0 = 4 * (lane >> 4), n = lane & 15;
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (r0 + i < 3) mine[GW_C2 + (r0 + i) * 64 + 16 * u + n] = g.dC2[u][i];
                mine[GW_W1 + (r0 + i) * 64 + 16 * u + n] = g.dW1[u][i];
            }
    }
    __syncthreads();
    auto sum4 = [&](int i) { return (gw[i] + gw[GW_TOTAL + i]) + (gw[2 * GW_TOTAL + i] + gw[3 * GW_TOTAL + i]); };
    if (jobs.det_ws) {   // deterministic: the block's image, reduced over blocks in order by mlp_wgrad_reduce
        float* dst = jobs.det_ws + (size_t)blockIdx.x * GW_TOTAL;
        for (int i = threadIdx.x; i < GW_TOTAL; i += blockDim.x) dst[i] = sum4(i);
        return;
    }
    // one loop per matrix: a pointer chosen per index would be a dynamically indexed private array
    auto flush = [&](float* dst, int off, int n) {
        for (int k = threadIdx.x; k < n; k += blockDim.x) {
            const float v = sum4(off + k);
            if (v != 0.f) __hip_atomic_fetch_add(dst + k, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    flush(a.G.w0, GW_W0, GW_W1 - GW_W0);
    flush(a.G.w1, GW_W1, GW_C0 - GW_W1);
    flush(a.G.c0, GW_C0, GW_C1 - GW_C0);
    flush(a.G.c1, GW_C1, GW_C2 - GW_C1);
    flush(a.G.c2, GW_C2, GW_TOTAL - GW_C2);
}

// Deterministic weight-gradient reduction: value i of a net's gradient image summed over the net's
// blocks [b0, b0 + nb) — one wave per value, lane l taking blocks l, l + 64, ... in order, then a
// fixed-order wave tree — and added to .grad (the sole writer: no atomics).
__global__ void __launch_bounds__(256) mlp_wgrad_reduce_kernel(const float* __restrict__ ws, int b0, int nb,
                                                               nerf_mlp_grads G) {
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (i >= GW_TOTAL) return;
    float s = 0.f;
    for (int b = lane; b < nb; b += 64) s += ws[(size_t)(b0 + b) * GW_TOTAL + i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane != 0) return;
    if (i < GW_W1) G.w0[i - GW_W0] += s;
    else if (i < GW_C0) G.w1[i - GW_W1] += s;
    else if (i < GW_C1) G.c0[i - GW_C0] += s;
    else if (i < GW_C2) G.c1[i - GW_C1] += s;
    else G.c2[i - GW_C2] += s;
}

// every element index the kernels form (feat, sh, raw/graw, geo/dgeo/dsh, dfeat) stays below 2^31
static bool fits_u32(const MlpArgs& a) {
    const int64_t lim = (int64_t)1 << 31;
    return a.P * a.sp + 16 * a.sl < lim && a.P * a.dsp + 16 * a.dsl < lim && a.P * a.sh_stride + 16 < lim &&
           16 * (a.P + 32) < lim && (!a.h3 || 64 * (a.P + 31) < lim);
}

int launch_mlp_fwd_x6(const MlpArgs& a, hipStream_t stream) {
    NERF_REQUIRE(fits_u32(a), "mlp_fwd(x6): %lld points exceed 32-bit indexing", (long long)a.P);
    NERF_REQUIRE(!a.h3 || !a.aq, "mlp_fwd(x6): saved h3 with A-CAQ (its backward recomputes)");
    const int64_t tiles = (a.P + 31) / 32;
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((tiles + 7) / 8, 256 * 2));
    if (a.aq)
        hipLaunchKernelGGL(mlp_fwd_x6_kernel<true>, dim3((unsigned)blocks), dim3(512), 0, stream, a);
    else
        hipLaunchKernelGGL(mlp_fwd_x6_kernel<false>, dim3((unsigned)blocks), dim3(512), 0, stream, a);
    NERF_CHECK_LAUNCH("mlp_fwd(x6)");
    return NERF_OK;
}

int launch_mlp_act_minmax_x6(const MlpArgs& a, hipStream_t stream) {
    NERF_REQUIRE(fits_u32(a), "mlp_act_minmax(x6): %lld points exceed 32-bit indexing", (long long)a.P);
    const int64_t n = a.calib_points < a.P ? a.calib_points : a.P;
    if (n <= 0) return NERF_OK;
    const int64_t tiles = (n + 31) / 32;
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((tiles + 7) / 8, 256 * 2));
    hipLaunchKernelGGL(mlp_act_minmax_x6_kernel, dim3((unsigned)blocks), dim3(512), 0, stream, a);
    NERF_CHECK_LAUNCH("mlp_act_minmax(x6)");
    return NERF_OK;
}

// jobs: 1 or 2 nets (P > 0 each, the same quantizer mode); det_ws (deterministic mode) holds
// kMlpBwdMaxBlocks x GW_TOTAL floats.
int launch_mlp_bwd_x6(const MlpArgs* jobs, int n_jobs, float* det_ws, hipStream_t stream) {
    NERF_REQUIRE(n_jobs == 1 || n_jobs == 2, "mlp_bwd(x6): %d jobs", n_jobs);
    int64_t want[2] = {0, 0}, tiles[2] = {0, 0};
    for (int k = 0; k < n_jobs; ++k) {
        NERF_REQUIRE(fits_u32(jobs[k]), "mlp_bwd(x6): %lld points exceed 32-bit indexing", (long long)jobs[k].P);
        NERF_REQUIRE(jobs[k].P > 0, "mlp_bwd(x6): empty job");
        NERF_REQUIRE((jobs[k].aq != nullptr) == (jobs[0].aq != nullptr), "mlp_bwd(x6): mixed quantizer modes");
        NERF_REQUIRE((jobs[k].h3 != nullptr) == (jobs[0].h3 != nullptr), "mlp_bwd(x6): saved h3 on some jobs only");
        NERF_REQUIRE(!jobs[k].h3 || (!jobs[k].aq && !jobs[k].rows), "mlp_bwd(x6): saved h3 with A-CAQ or active rows");
        tiles[k] = (jobs[k].P + 31) / 32;
        want[k] = (tiles[k] + 3) / 4;   // blocks of 4 wave pairs, one tile per pair
    }
    MlpBwdJobs J{};
    J.a[0] = jobs[0];
    J.a[1] = n_jobs == 2 ? jobs[1] : jobs[0];
    J.det_ws = det_ws;
    int64_t blocks;
    if (n_jobs == 1) {
        blocks = std::max<int64_t>(1, std::min<int64_t>(want[0], kMlpBwdMaxBlocks));
        J.split = (int)blocks;
    } else if (want[0] + want[1] <= kMlpBwdMaxBlocks) {
        blocks = want[0] + want[1];
        J.split = (int)want[0];
    } else {   // one block per CU: blocks in proportion to the tiles, so both nets finish together
        blocks = kMlpBwdMaxBlocks;
        const int64_t b0 = (kMlpBwdMaxBlocks * tiles[0] + (tiles[0] + tiles[1]) / 2) / (tiles[0] + tiles[1]);
        J.split = (int)std::min<int64_t>(std::max<int64_t>(b0, 1), kMlpBwdMaxBlocks - 1);
    }
    if (jobs[0].aq)
        hipLaunchKernelGGL((mlp_bwd_x6cg_kernel<true, false>), dim3((unsigned)blocks), dim3(512), 0, stream, J);
    else if (jobs[0].h3)
        hipLaunchKernelGGL((mlp_bwd_x6cg_kernel<false, true>), dim3((unsigned)blocks), dim3(512), 0, stream, J);
    else
        hipLaunchKernelGGL((mlp_bwd_x6cg_kernel<false, false>), dim3((unsigned)blocks), dim3(512), 0, stream, J);
    NERF_CHECK_LAUNCH("mlp_bwd(x6)");
    if (det_ws) {
        for (int k = 0; k < n_jobs; ++k) {
            const int b0 = k == 0 ? 0 : J.split, nb = k == 0 ? J.split : (int)blocks - J.split;
            hipLaunchKernelGGL(mlp_wgrad_reduce_kernel, dim3((GW_TOTAL + 3) / 4), dim3(256), 0, stream, det_ws, b0, nb,
                               jobs[k].G);
        }
        NERF_CHECK_LAUNCH("mlp_bwd(x6) deterministic reduction");
    }
    return NERF_OK;
}

#ifdef NERF_X6CG_PROF
// diagnostic builds only: the chain / wgrad waves' wait and loop cycles summed over all waves since
// the last call (s_memtime units), then the chain wave's waits per stage; all reset
extern "C" int nerf_x6cg_prof(unsigned long long* out12) {
    if (hipMemcpyFromSymbol(out12, HIP_SYMBOL(cg_prof), sizeof(cg_prof)) != hipSuccess) return 1;
    if (hipMemcpyFromSymbol(out12 + 4, HIP_SYMBOL(cg_stage_wait), sizeof(cg_stage_wait)) != hipSuccess) return 1;
    const unsigned long long zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(cg_prof), zero, sizeof(cg_prof)) != hipSuccess) return 1;
    return hipMemcpyToSymbol(HIP_SYMBOL(cg_stage_wait), zero, sizeof(cg_stage_wait)) == hipSuccess ? 0 : 1;
}
#endif

}  // namespace nerf
