// Normals head of NeRFSmall (run_nerf_helpers.py:259-263, :298-302; ScanNet configuration):
//   n = normalize(N1 relu(N0 geo + b0) + b1)        N0 [32,15], b0 [32], N1 [3,32], b1 [3]
// appended to the MLP's raw as channels 4..6 (raw [P,7] = rgb, sigma, n). run_network's mask
// `outputs_flat[~keep_mask, -1] = 0` (run_nerf.py:66) then zeroes the LAST channel, which with
// normals is n_z, not sigma: the reference's behaviour, reproduced here (the MLP runs without its
// sigma mask when the head is on).
//
// One thread per point; the 611 head parameters sit in LDS (wave-uniform broadcast reads). The
// backward also forms the head's weight gradients, sums over all points (dN0 = dh^T geo, db0 = sum
// dh, dN1 = dn^T relu(h), db1 = sum dn): a persistent grid of 128-point tiles stages each tile's
// per-point factors in LDS, every thread owns ~5 of the 611 gradient values and accumulates them
// over the tiles in registers, each block stores its totals, and a small kernel sums the blocks in
// order into .grad (no [P,32] buffers in HBM, no K = P library GEMMs, no same-address atomics).
#include "common.h"

namespace nerf {

constexpr int NH_HID = 32, NH_GEO = 15;
constexpr int NH_N0 = 0, NH_B0 = NH_N0 + NH_HID * NH_GEO, NH_N1 = NH_B0 + NH_HID, NH_B1 = NH_N1 + 3 * NH_HID,
              NH_ALL = NH_B1 + 3;   // 611 floats

struct NormalArgs {
    const float* o16;      // [P,16] = [sigma, geo 15] (MLP geo output)
    const float* raw4;     // [P,4]
    const uint8_t* keep;   // [P] or null (fwd with rows: indexed in the source order)
    const int32_t* rows;   // fwd: null, or the merged row of each source-order point (a permutation of [0, P))
    uint8_t* keep_out;     // fwd with rows: keep scattered to the merged rows (what the backward reads)
    int64_t P;
    nerf_normal_head W;
    float* raw7;           // fwd out [P,7]
    const float* graw7;    // bwd in [P,7]
    float* graw4;          // bwd out [P,4]
    float* dgeo;           // bwd out [P,16] (row 0 = 0)
    nerf_normal_head_grads G;   // bwd: accumulated weight gradients
    float* partials;       // bwd: [gridDim.x][NH_ALL] per-block sums (reduced by normal_head_wgrad_reduce)
};

// LDS image of the head, rows padded to 16 floats so that a row is four ds_read_b128 (broadcast
// reads: every lane of a wave reads the same weights): N0 [32][16] (column 15 = 0), b0 [32],
// N1 [3][32], b1 [3].
constexpr int LH_N0 = 0, LH_B0 = 32 * 16, LH_N1 = LH_B0 + 32, LH_B1 = LH_N1 + 96, LH_ALL = LH_B1 + 4;

__device__ __forceinline__ void load_head(float* s, const nerf_normal_head& W) {
    for (int i = threadIdx.x; i < LH_ALL; i += blockDim.x) {
        float v = 0.f;
        if (i < LH_B0) v = (i & 15) < NH_GEO ? W.n0[(i >> 4) * NH_GEO + (i & 15)] : 0.f;
        else if (i < LH_N1) v = W.b0[i - LH_B0];
        else if (i < LH_B1) v = W.n1[i - LH_N1];
        else if (i < LH_B1 + 3) v = W.b1[i - LH_B1];
        s[i] = v;
    }
    __syncthreads();
}

__device__ __forceinline__ float4 ld4(const float* s, int i) { return *reinterpret_cast<const float4*>(s + i); }

__global__ void __launch_bounds__(256) normal_head_fwd_kernel(NormalArgs a) {
    __shared__ __attribute__((aligned(16))) float s[LH_ALL];
    load_head(s, a.W);
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= a.P) return;
    // with rows, thread q takes source point q at its merged row p (the fine pass's importance-first
    // walk): its keep flag lands at p for the backward, replacing a scatter of its own
    const int64_t p = a.rows ? (int64_t)a.rows[q] : q;
    float geo[NH_GEO], n[3];
    {   // o16 = [sigma, geo 0..14]: four 16-B loads instead of fifteen 4-B ones
        const float4* src = reinterpret_cast<const float4*>(a.o16 + p * 16);
        const float4 v0 = src[0], v1 = src[1], v2 = src[2], v3 = src[3];
        geo[0] = v0.y; geo[1] = v0.z; geo[2] = v0.w;
        geo[3] = v1.x; geo[4] = v1.y; geo[5] = v1.z; geo[6] = v1.w;
        geo[7] = v2.x; geo[8] = v2.y; geo[9] = v2.z; geo[10] = v2.w;
        geo[11] = v3.x; geo[12] = v3.y; geo[13] = v3.z; geo[14] = v3.w;
    }
    // F.linear with bias (addmm: bias + x W^T), fp32 dot products in input order; one hidden unit's N1
    // terms added as it is formed: no [32] hidden array, four units per loop trip (unrolled whole, the compiler held every
    // weight in registers: 174 VGPRs, two waves per SIMD)
    {
        float nacc[3] = {0.f, 0.f, 0.f};
#pragma unroll 1
        for (int i4 = 0; i4 < NH_HID; i4 += 4) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int i = i4 + e;
                float acc = 0.f;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 t = ld4(s, LH_N0 + 16 * i + 4 * q);
                    acc = fmaf(t.x, geo[4 * q], acc);
                    acc = fmaf(t.y, geo[4 * q + 1], acc);
                    acc = fmaf(t.z, geo[4 * q + 2], acc);
                    if (q < 3) acc = fmaf(t.w, geo[4 * q + 3], acc);
                }
                const float r = fmaxf(acc + s[LH_B0 + i], 0.f);
#pragma unroll
                for (int c = 0; c < 3; ++c) nacc[c] = fmaf(s[LH_N1 + c * NH_HID + i], r, nacc[c]);
            }
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) n[c] = nacc[c] + s[LH_B1 + c];
    }
    // F.normalize(x, dim=-1): x / max(||x||_2, 1e-12)
    const float nrm = fmaxf(sqrtf(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]), 1e-12f);
    const float4 r = *reinterpret_cast<const float4*>(a.raw4 + 4 * p);
    const bool keep = a.keep ? a.keep[q] != 0 : true;
    if (a.keep_out) a.keep_out[p] = keep ? 1 : 0;
    float* o = a.raw7 + 7 * p;
    o[0] = r.x; o[1] = r.y; o[2] = r.z; o[3] = r.w;
    o[4] = n[0] / nrm;
    o[5] = n[1] / nrm;
    o[6] = keep ? n[2] / nrm : 0.f;
}

constexpr int NH_TILE = 128;
// LDS row strides (floats): d hidden and relu(hidden) rows of 32 + 4 (relu's column 32 = 1: db1 as one
// more product column), geo rows of 16 + 4 (column 15 = 1: db0 as N0's 16th column; stride 20 keeps the
// ds_write_b128 of eight consecutive rows on 32 distinct banks), d n rows of 4 (column 3 = 0)
constexpr int NH_SDH = 36, NH_SR = 36, NH_SG = 20;
constexpr int NH_R1 = 36;   // columns of the d N1 image (32 hidden + the ones column + 3 pad)

// One thread per point for the per-point part (the head's forward recompute, the normalize backward,
// d hidden, d geo); then the tile's weight gradients as register-blocked outer products: each of the
// 128 threads owns a 4 x 4 block of [dN0 | db0] (32 x 16) over a quarter of the tile's points (two
// ds_read_b128 feed 16 FMAs), threads 0..71 also a 4 x 4 block of [dN1 | db1] (4 x 36) over 16 points.
// Blocks keep their sums in registers over all their tiles; at the end the quarters / point groups are
// added in a fixed order and each block stores its 611 totals (normal_head_wgrad_reduce_kernel sums
// the blocks in order: deterministic). The earlier form (every thread 5 gradient values, each a
// 128-step dot product of two LDS reads per FMA) ran 248 us per launch at the ScanNet config, latency-
// bound on its 1,280 dependent LDS reads per wave and tile.
__global__ void __launch_bounds__(NH_TILE) __attribute__((amdgpu_waves_per_eu(2))) normal_head_bwd_kernel(NormalArgs a) {
    __shared__ __attribute__((aligned(16))) float s[LH_ALL];
    __shared__ __attribute__((aligned(16))) float s_dh[NH_TILE * NH_SDH];   // d pre-ReLU hidden
    __shared__ __attribute__((aligned(16))) float s_r[NH_TILE * NH_SR];     // relu(hidden), column 32 = 1
    __shared__ __attribute__((aligned(16))) float s_geo[NH_TILE * NH_SG];   // geo, column 15 = 1
    __shared__ __attribute__((aligned(16))) float s_dn[NH_TILE * 4];        // d pre-normalize n, column 3 = 0
    load_head(s, a.W);
    const int tid = threadIdx.x;
    const int blk0 = tid & 31, quarter = tid >> 5, rg = blk0 >> 2, cg = blk0 & 3;   // [dN0 | db0] block
    const bool own1 = tid < 72;
    const int blk1 = tid % 9, grp1 = tid / 9;                                      // [dN1 | db1] block
    float acc0[16], acc1[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) { acc0[j] = 0.f; acc1[j] = 0.f; }
    for (int64_t base = (int64_t)blockIdx.x * NH_TILE; base < a.P; base += (int64_t)gridDim.x * NH_TILE) {
        const int64_t p = base + tid;
        const bool valid = p < a.P;
        float geo[16];
        {
            const float4* src = reinterpret_cast<const float4*>(a.o16 + (valid ? p : 0) * 16);
            float4 v[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = valid ? src[q] : make_float4(0.f, 0.f, 0.f, 0.f);
            // o16 = [sigma, geo 0..14]: geo k at element k + 1
            geo[0] = v[0].y; geo[1] = v[0].z; geo[2] = v[0].w;
            geo[3] = v[1].x; geo[4] = v[1].y; geo[5] = v[1].z; geo[6] = v[1].w;
            geo[7] = v[2].x; geo[8] = v[2].y; geo[9] = v[2].z; geo[10] = v[2].w;
            geo[11] = v[3].x; geo[12] = v[3].y; geo[13] = v[3].z; geo[14] = v[3].w;
            geo[15] = 1.f;
        }
        // forward, four hidden units at a time (relu(hidden) to this thread's LDS row: its sign is the
        // ReLU mask of the backward below), the same fp32 op order as normal_head_fwd_kernel
        float* rdh = s_dh + tid * NH_SDH;
        float* rr = s_r + tid * NH_SR;
        float nacc[3] = {0.f, 0.f, 0.f};
#pragma unroll 1
        for (int i4 = 0; i4 < NH_HID; i4 += 4) {
            float r4[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int i = i4 + e;
                float hi = 0.f;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 t = ld4(s, LH_N0 + 16 * i + 4 * q);
                    hi = fmaf(t.x, geo[4 * q], hi);
                    hi = fmaf(t.y, geo[4 * q + 1], hi);
                    hi = fmaf(t.z, geo[4 * q + 2], hi);
                    if (q < 3) hi = fmaf(t.w, geo[4 * q + 3], hi);
                }
                hi = hi + s[LH_B0 + i];
                r4[e] = fmaxf(hi, 0.f);
#pragma unroll
                for (int c = 0; c < 3; ++c) nacc[c] = fmaf(s[LH_N1 + c * NH_HID + i], r4[e], nacc[c]);
            }
            *reinterpret_cast<float4*>(rr + i4) = make_float4(r4[0], r4[1], r4[2], r4[3]);
        }
        float n[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) n[c] = nacc[c] + s[LH_B1 + c];
        float dn[3] = {0.f, 0.f, 0.f};
        if (valid) {
            const float* g7 = a.graw7 + 7 * p;
            *reinterpret_cast<float4*>(a.graw4 + 4 * p) = make_float4(g7[0], g7[1], g7[2], g7[3]);
            const bool keep = a.keep ? a.keep[p] != 0 : true;
            const float g[3] = {g7[4], g7[5], keep ? g7[6] : 0.f};
            // y = x / m, m = max(||x||, eps): dx = g / m - x (g.x) / (m^2 ||x||)  (the norm term only
            // while ||x|| > eps, where the clamp passes the gradient)
            const float len = sqrtf(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
            const float m = fmaxf(len, 1e-12f);
            const float gx = g[0] * n[0] + g[1] * n[1] + g[2] * n[2];
#pragma unroll
            for (int c = 0; c < 3; ++c) dn[c] = g[c] / m - (len > 1e-12f ? n[c] * (gx / (m * m * len)) : 0.f);
        }
        float dg[NH_GEO];
#pragma unroll
        for (int k = 0; k < NH_GEO; ++k) dg[k] = 0.f;
#pragma unroll 1
        for (int i4 = 0; i4 < NH_HID; i4 += 4) {
            const float4 rv = *reinterpret_cast<const float4*>(rr + i4);
            const float r4[4] = {rv.x, rv.y, rv.z, rv.w};
            float dh4[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int i = i4 + e;
                dh4[e] = r4[e] > 0.f ? (s[LH_N1 + i] * dn[0] + s[LH_N1 + NH_HID + i] * dn[1]) +
                                           s[LH_N1 + 2 * NH_HID + i] * dn[2]
                                     : 0.f;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 t = ld4(s, LH_N0 + 16 * i + 4 * q);
                    dg[4 * q] = fmaf(t.x, dh4[e], dg[4 * q]);
                    dg[4 * q + 1] = fmaf(t.y, dh4[e], dg[4 * q + 1]);
                    dg[4 * q + 2] = fmaf(t.z, dh4[e], dg[4 * q + 2]);
                    if (q < 3) dg[4 * q + 3] = fmaf(t.w, dh4[e], dg[4 * q + 3]);
                }
            }
            *reinterpret_cast<float4*>(rdh + i4) = make_float4(dh4[0], dh4[1], dh4[2], dh4[3]);
        }
        *reinterpret_cast<float4*>(rr + NH_HID) = make_float4(1.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int q = 0; q < 4; ++q)
            *reinterpret_cast<float4*>(s_geo + tid * NH_SG + 4 * q) =
                make_float4(geo[4 * q], geo[4 * q + 1], geo[4 * q + 2], geo[4 * q + 3]);
        *reinterpret_cast<float4*>(s_dn + tid * 4) = make_float4(dn[0], dn[1], dn[2], 0.f);
        if (valid) {
            float4* d = reinterpret_cast<float4*>(a.dgeo + p * 16);
            d[0] = make_float4(0.f, dg[0], dg[1], dg[2]);
            d[1] = make_float4(dg[3], dg[4], dg[5], dg[6]);
            d[2] = make_float4(dg[7], dg[8], dg[9], dg[10]);
            d[3] = make_float4(dg[11], dg[12], dg[13], dg[14]);
        }
        __syncthreads();
        // [dN0 | db0] += d hidden^T [geo | 1] over this thread's quarter of the tile
#pragma unroll 4
        for (int u = 0; u < NH_TILE / 4; ++u) {
            const int q = quarter * (NH_TILE / 4) + u;
            const float4 d4 = *reinterpret_cast<const float4*>(s_dh + q * NH_SDH + 4 * rg);
            const float4 g4 = *reinterpret_cast<const float4*>(s_geo + q * NH_SG + 4 * cg);
            const float dv[4] = {d4.x, d4.y, d4.z, d4.w}, gv[4] = {g4.x, g4.y, g4.z, g4.w};
#pragma unroll
            for (int x = 0; x < 4; ++x)
#pragma unroll
                for (int y = 0; y < 4; ++y) acc0[4 * x + y] = fmaf(dv[x], gv[y], acc0[4 * x + y]);
        }
        if (own1) {   // [dN1 | db1] += d n^T [relu(hidden) | 1] over 16 points
#pragma unroll 4
            for (int u = 0; u < 16; ++u) {
                const int q = grp1 * 16 + u;
                const float4 n4 = *reinterpret_cast<const float4*>(s_dn + q * 4);
                const float4 r4 = *reinterpret_cast<const float4*>(s_r + q * NH_SR + 4 * blk1);
                const float nv[4] = {n4.x, n4.y, n4.z, n4.w}, rv[4] = {r4.x, r4.y, r4.z, r4.w};
#pragma unroll
                for (int x = 0; x < 4; ++x)
#pragma unroll
                    for (int y = 0; y < 4; ++y) acc1[4 * x + y] = fmaf(nv[x], rv[y], acc1[4 * x + y]);
            }
        }
        __syncthreads();
    }
    // the block's totals: quarters / point groups added in a fixed order (the LDS tiles reused)
    float* part0 = s_dh;   // [4 quarters][32 x 16]
    float* part1 = s_r;    // [8 groups][4 x 36]
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) part0[quarter * 512 + (4 * rg + x) * 16 + 4 * cg + y] = acc0[4 * x + y];
    if (own1) {
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int y = 0; y < 4; ++y) part1[grp1 * 144 + x * NH_R1 + 4 * blk1 + y] = acc1[4 * x + y];
    }
    __syncthreads();
    for (int v = tid; v < NH_ALL; v += NH_TILE) {
        float t = 0.f;
        if (v < NH_N1) {   // N0 [i][k] | b0 [i] = column 15
            const int idx = v < NH_B0 ? (v / NH_GEO) * 16 + v % NH_GEO : (v - NH_B0) * 16 + 15;
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) t += part0[qq * 512 + idx];
        } else {           // N1 [c][i] | b1 [c] = column 32
            const int idx = v < NH_B1 ? ((v - NH_N1) / NH_HID) * NH_R1 + (v - NH_N1) % NH_HID : (v - NH_B1) * NH_R1 + NH_HID;
#pragma unroll
            for (int gg = 0; gg < 8; ++gg) t += part1[gg * 144 + idx];
        }
        a.partials[(size_t)blockIdx.x * NH_ALL + v] = t;
    }
}

// one wave per gradient value: lane l sums blocks l, l + 64, ... in order, then a fixed-order wave
// tree (deterministic), and lane 0 adds the total into .grad
__global__ void __launch_bounds__(256) normal_head_wgrad_reduce_kernel(const float* __restrict__ partials, int nb,
                                                                       nerf_normal_head_grads G) {
    const int v = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (v >= NH_ALL) return;
    float t = 0.f;
    for (int b = lane; b < nb; b += 64) t += partials[(size_t)b * NH_ALL + v];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
    if (lane != 0) return;
    if (v < NH_B0) G.n0[v] += t;
    else if (v < NH_N1) G.b0[v - NH_B0] += t;
    else if (v < NH_B1) G.n1[v - NH_N1] += t;
    else G.b1[v - NH_B1] += t;
}

constexpr int kHeadBwdBlocks = 1024;
constexpr int kHeadBwdResident = 768;
static_assert(kHeadBwdResident <= kHeadBwdBlocks, "workspace");

static int fill_normal(NormalArgs& a, const float* o16, const uint8_t* keep, int64_t P, const nerf_normal_head* W) {
    NERF_REQUIRE(P >= 0, "normal_head: n_points < 0");
    NERF_REQUIRE((P == 0 || o16) && W && W->n0 && W->b0 && W->n1 && W->b1, "normal_head: null argument");
    NERF_REQUIRE(((uintptr_t)o16 & 15) == 0, "normal_head: geo rows must be 16-B aligned (16-float rows)");
    a.o16 = o16;
    a.keep = keep;
    a.P = P;
    a.W = *W;
    return NERF_OK;
}

}  // namespace nerf

using namespace nerf;

extern "C" int nerf_normal_head_fwd_rows(const float* d_o16, const float* d_raw4, const uint8_t* d_keep,
                                         const int32_t* d_rows, int64_t n_points, const nerf_normal_head* head,
                                         float* d_raw7, uint8_t* d_keep_out, void* stream) {
    NormalArgs a{};
    int rc = fill_normal(a, d_o16, d_keep, n_points, head);
    if (rc) return rc;
    NERF_REQUIRE(n_points == 0 || (d_raw4 && d_raw7), "normal_head_fwd: null buffer");
    NERF_REQUIRE(!d_rows || n_points <= INT32_MAX, "normal_head_fwd: rows are int32");
    NERF_REQUIRE(!d_keep_out || d_keep, "normal_head_fwd: keep_out needs keep");
    if (n_points == 0) return NERF_OK;
    a.rows = d_rows;
    a.keep_out = d_keep_out;
    a.raw4 = d_raw4;
    a.raw7 = d_raw7;
    hipLaunchKernelGGL(normal_head_fwd_kernel, dim3(blocks_for(n_points, 256)), dim3(256), 0, as_stream(stream), a);
    NERF_CHECK_LAUNCH("normal_head_fwd");
    return NERF_OK;
}

extern "C" int nerf_normal_head_fwd(const float* d_o16, const float* d_raw4, const uint8_t* d_keep, int64_t n_points,
                                    const nerf_normal_head* head, float* d_raw7, void* stream) {
    return nerf_normal_head_fwd_rows(d_o16, d_raw4, d_keep, nullptr, n_points, head, d_raw7, nullptr, stream);
}

extern "C" size_t nerf_normal_head_bwd_workspace_bytes(void) {
    return (size_t)kHeadBwdBlocks * NH_ALL * sizeof(float);
}

extern "C" int nerf_normal_head_bwd(const float* d_o16, const uint8_t* d_keep, int64_t n_points,
                                    const nerf_normal_head* head, const float* d_graw7, float* d_graw4, float* d_dgeo,
                                    const nerf_normal_head_grads* grads, float* d_workspace, size_t workspace_bytes,
                                    void* stream) {
    NormalArgs a{};
    int rc = fill_normal(a, d_o16, d_keep, n_points, head);
    if (rc) return rc;
    NERF_REQUIRE((n_points == 0 || (d_graw7 && d_graw4 && d_dgeo)) && grads && grads->n0 && grads->b0 && grads->n1 && grads->b1,
                 "normal_head_bwd: null buffer");
    NERF_REQUIRE((((uintptr_t)d_graw4 | (uintptr_t)d_dgeo) & 15) == 0, "normal_head_bwd: d raw4 / d geo must be 16-B aligned");
    NERF_REQUIRE(d_workspace && workspace_bytes >= nerf_normal_head_bwd_workspace_bytes(),
                 "normal_head_bwd: workspace %zu B < %zu B", workspace_bytes, nerf_normal_head_bwd_workspace_bytes());
    if (n_points == 0) return NERF_OK;
    a.graw7 = d_graw7;
    a.graw4 = d_graw4;
    a.dgeo = d_dgeo;
    a.G = *grads;
    a.partials = d_workspace;
    // one round of resident blocks (51.6 KB of LDS each: 3 per CU on 256 CUs), at most the workspace's
    const unsigned blocks = (unsigned)std::min<int64_t>(blocks_for(n_points, NH_TILE), kHeadBwdResident);
    hipLaunchKernelGGL(normal_head_bwd_kernel, dim3(blocks), dim3(NH_TILE), 0, as_stream(stream), a);
    NERF_CHECK_LAUNCH("normal_head_bwd");
    hipLaunchKernelGGL(normal_head_wgrad_reduce_kernel, dim3((NH_ALL + 3) / 4), dim3(256), 0, as_stream(stream),
                       d_workspace, (int)blocks, *grads);
    NERF_CHECK_LAUNCH("normal_head_bwd");
    return NERF_OK;
}
