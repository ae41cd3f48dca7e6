// Shared device helpers of the field (MLP) kernels: argument block, MFMA layout helpers, SH4,
// per-tile input loads. See field.hip for the layout conventions.
#pragma once

#include <stdlib.h>

#include <algorithm>

#include "hash_common.h"

namespace nerf {

typedef float floatx16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int row_of(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// weight-gradient image of one net (GW_TOTAL floats): W0 [64][32], W1 [16][64], C0 [64][31],
// C1 [64][64], C2 [3][64]
constexpr int GW_W0 = 0, GW_W1 = 2048, GW_C0 = 3072, GW_C1 = 5056, GW_C2 = 9152, GW_TOTAL = 9344;

// MLP backward grid cap: one 512-thread block per CU (159 KB of LDS each)
constexpr int kMlpBwdMaxBlocks = 256;

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
    int64_t dsp, dsl;            // bwd: d feat strides (fill_args: the feature strides)
    // point order (nerf_point_order): point p's row in raw / geo / graw / dgeo / dsh is io_rows[p] (NULL:
    // p); its ray is p / spr below seg_split, (p - seg_split) / spr2 from there on
    const int32_t* io_rows;
    int64_t seg_split, spr2;
    // n / spr and n / spr2 for n < 2^31 as mulhi(n, m) >> s (m = 0: divisor 1), set by fill_args /
    // fill_order (Granlund-Montgomery: m = ceil(2^(31+l) / d), l = ceil(log2 d), s = l - 1)
    uint32_t rd_m1, rd_m2;
    int rd_s1, rd_s2;
    const int32_t* rows;         // bwd, optional: walk only the points rows[0 .. *count) (active points)
    const int32_t* count;
    float* dsh;
    float* geo_out;       // fwd, optional: o = [sigma, geo 15] per point, [P,16] (normals head input)
    const float* dgeo;    // bwd, optional: upstream d o from the normals head, [P,16] (row 0 ignored)
    const QuantRec* aq;   // optional A-CAQ record of the layer-0 activation quantizer
    uint32_t* act_minmax; // calibration-only launch: min/max of relu(x W0^T) (order-preserving u32)
    int64_t calib_points;
    float* h3;            // optional: layer C1's ReLU outputs per 32-point tile (field_x6.hip h3_at): the
                          // forward stores them, the backward reads them instead of recomputing C1
};

// A-CAQ activation quantizer on a layer-0 accumulator tile (sigma_act_quantizers[0],
// run_nerf_helpers.py:280-284).
__device__ __forceinline__ void fake_quant16(floatx16& v, const QuantRec& q) {
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = fake_quant(v[r], q);
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

// Per-ray SH record (sh_stride 0, nerf_sample_stratified_sh): 16 fp32 coefficients, then the three
// exact bf16 pieces (v0 = bf16(v), v1 = bf16(v - v0), v2 = bf16(v - v0 - v1)) of each, 160 B
constexpr int kShRecord = 40;   // floats

// The ray of point pc (the point order's two segments, MlpArgs)
__device__ __forceinline__ uint32_t ray_of(const MlpArgs& a, uint32_t pc) {
    return pc < (uint32_t)a.seg_split ? udiv_magic(pc, a.rd_m1, a.rd_s1)
                                      : udiv_magic(pc - (uint32_t)a.seg_split, a.rd_m2, a.rd_s2);
}

__device__ __forceinline__ floatx16 zero16() {
    floatx16 z;
#pragma unroll
    for (int r = 0; r < 16; ++r) z[r] = 0.f;
    return z;
}

}  // namespace nerf
