// Shared device helpers of the field (MLP) kernels: argument block, MFMA layout helpers, SH4,
// per-tile input loads. See field.hip for the layout conventions.
#pragma once

#include <stdlib.h>

#include <algorithm>

#include "hash_common.h"

namespace nerf {

typedef float floatx16 __attribute__((ext_vector_type(16)));

#define NERF_MFMA(a, b, c) __builtin_amdgcn_mfma_f32_32x32x2f32((a), (b), (c), 0, 0, 0)

__device__ __forceinline__ int row_of(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// ---- LDS weight images (floats)
constexpr int RS_W0 = 33;   // W0  [64][32]
constexpr int RS_W1 = 65;   // W1  [32][64], rows 16..31 zero
constexpr int RS_C0 = 33;   // C0y [64][32]: cols 0..15 = C0[:,0..15] (SH), col 16 = 0 (sigma slot),
                            //               cols 17..31 = C0[:,16..30] (geo feature 1..15)
constexpr int RS_C1 = 65;   // C1  [64][64]
constexpr int RS_C2 = 65;   // C2  [32][64], rows 3..31 zero
constexpr int OFF_W0 = 0;
constexpr int OFF_W1 = OFF_W0 + 64 * RS_W0;
constexpr int OFF_C0 = OFF_W1 + 32 * RS_W1;
constexpr int OFF_C1 = OFF_C0 + 64 * RS_C0;
constexpr int OFF_C2 = OFF_C1 + 64 * RS_C1;
constexpr int LDS_W = OFF_C2 + 32 * RS_C2;          // 12544 floats = 49 KiB

// ---- backward LDS: per-wave activation / gradient staging, per-block weight-grad accumulator
constexpr int RS_T = 68;                            // [32 points][64 (+4 pad)]
constexpr int STAGE = 32 * RS_T;
constexpr int GW_W0 = 0, GW_W1 = 2048, GW_C0 = 3072, GW_C1 = 5056, GW_C2 = 9152, GW_TOTAL = 9344;
constexpr int BWD_WAVES = 4;
constexpr int LDS_BWD = LDS_W + BWD_WAVES * 2 * STAGE + GW_TOTAL;   // 157,184 B

struct MlpArgs {
    const float* feat; int64_t sp, sl;
    const float* sh; int64_t sh_stride;
    const float* viewdirs; int64_t spr;
    const uint8_t* keep;
    int64_t P;
    nerf_mlp_weights W;
    float* raw;
    const float* graw;
    nerf_mlp_grads G;
    float* dfeat;
    float* dsh;
    float* geo_out;       // fwd, optional: o = [sigma, geo 15] per point, [P,16] (normals head input)
    const float* dgeo;    // bwd, optional: upstream d o from the normals head, [P,16] (row 0 ignored)
    const QuantRec* aq;   // optional A-CAQ record of the layer-0 activation quantizer
    uint32_t* act_minmax; // calibration-only launch: min/max of relu(x W0^T) (order-preserving u32)
    int64_t calib_points;
    int flush_skip;       // A/B timing only (NERF_X6CG_FLUSH): 1 = no global flush, 2 = no block reduction either
};

// A-CAQ activation quantizer on a layer-0 accumulator tile (sigma_act_quantizers[0],
// run_nerf_helpers.py:280-284).
__device__ __forceinline__ void fake_quant16(floatx16& v, const QuantRec& q) {
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = fake_quant(v[r], q);
}

__device__ inline void load_weight_images(float* lds, const nerf_mlp_weights& W) {
    for (int i = threadIdx.x; i < LDS_W; i += blockDim.x) {
        float v = 0.f;
        if (i < OFF_W1) {
            const int r = i / RS_W0, c = i % RS_W0;
            if (c < 32) v = W.w0[r * 32 + c];
        } else if (i < OFF_C0) {
            const int k = i - OFF_W1, r = k / RS_W1, c = k % RS_W1;
            if (r < 16 && c < 64) v = W.w1[r * 64 + c];
        } else if (i < OFF_C1) {
            const int k = i - OFF_C0, r = k / RS_C0, c = k % RS_C0;
            if (c < 16) v = W.c0[r * 31 + c];
            else if (c >= 17 && c < 32) v = W.c0[r * 31 + c - 1];
        } else if (i < OFF_C2) {
            const int k = i - OFF_C1, r = k / RS_C1, c = k % RS_C1;
            if (c < 64) v = W.c1[r * 64 + c];
        } else {
            const int k = i - OFF_C2, r = k / RS_C2, c = k % RS_C2;
            if (r < 3 && c < 64) v = W.c2[r * 64 + c];
        }
        lds[i] = v;
    }
}

// SHEncoder degree 4, fp32, the reference's operand order (hash_encoding.py:158-179).
__device__ __forceinline__ void sh4_eval(float x, float y, float z, float* o) {
    const float xx = x * x, yy = y * y, zz = z * z;
    const float xy = x * y, yz = y * z, xz = x * z;
    o[0] = 0.28209479177387814f;
    o[1] = -0.4886025119029199f * y;
    o[2] = 0.4886025119029199f * z;
    o[3] = -0.4886025119029199f * x;
    o[4] = 1.0925484305920792f * xy;
    o[5] = -1.0925484305920792f * yz;
    o[6] = 0.31539156525252005f * ((2.0f * zz - xx) - yy);
    o[7] = -1.0925484305920792f * xz;
    o[8] = 0.5462742152960396f * (xx - yy);
    o[9] = (-0.5900435899266435f * y) * (3.0f * xx - yy);
    o[10] = (2.890611442640554f * xy) * z;
    o[11] = (-0.4570457994644658f * y) * ((4.0f * zz - xx) - yy);
    o[12] = (0.3731763325901154f * z) * ((2.0f * zz - 3.0f * xx) - 3.0f * yy);
    o[13] = (-0.4570457994644658f * x) * ((4.0f * zz - xx) - yy);
    o[14] = (1.445305721320277f * z) * (xx - yy);
    o[15] = (-0.5900435899266435f * x) * (xx - 3.0f * yy);
}

// ---- per-tile inputs: lane (j, h) holds x[pt][2s+h] (s<16) and sh[pt][2s+h] (s<8)
__device__ __forceinline__ void load_tile_inputs(const MlpArgs& a, int64_t pt, bool valid, int h, float (&x)[16],
                                                 float (&shv)[8]) {
#pragma unroll
    for (int s = 0; s < 16; ++s) x[s] = valid ? a.feat[pt * a.sp + (int64_t)s * a.sl + h] : 0.f;
    if (a.viewdirs) {
        float o[16];
        if (valid) {
            const int64_t ray = pt / a.spr;
            sh4_eval(a.viewdirs[3 * ray], a.viewdirs[3 * ray + 1], a.viewdirs[3 * ray + 2], o);
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) o[k] = 0.f;
        }
#pragma unroll
        for (int s = 0; s < 8; ++s) shv[s] = h ? o[2 * s + 1] : o[2 * s];
    } else {
#pragma unroll
        for (int s = 0; s < 8; ++s) shv[s] = valid ? a.sh[pt * a.sh_stride + 2 * s + h] : 0.f;
    }
}

__device__ __forceinline__ floatx16 zero16() {
    floatx16 z;
#pragma unroll
    for (int r = 0; r < 16; ++r) z[r] = 0.f;
    return z;
}

__device__ __forceinline__ void relu16(floatx16& v) {
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = v[r] > 0.f ? v[r] : 0.f;
}

// Write a C-layout tile (rows = neurons 32*t + row(r,h), col = point j) to a [point][RS_T] stage.
__device__ __forceinline__ void stage_tile(float* st, const floatx16& v, int t, int j, int h) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        float4 q = make_float4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]);
        *reinterpret_cast<float4*>(st + j * RS_T + 32 * t + 8 * g + 4 * h) = q;
    }
}

}  // namespace nerf
