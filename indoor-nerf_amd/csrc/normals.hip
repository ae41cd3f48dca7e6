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
    const uint8_t* keep;   // [P] or null
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

// F.linear with bias (addmm: bias + x W^T); fp32 dot products in input order
__device__ __forceinline__ void head_forward(const float* s, const float* geo, float* h, float* n) {
#pragma unroll 4
    for (int i = 0; i < NH_HID; ++i) {
        float w[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float4 t = ld4(s, LH_N0 + 16 * i + 4 * q);
            w[4 * q] = t.x; w[4 * q + 1] = t.y; w[4 * q + 2] = t.z; w[4 * q + 3] = t.w;
        }
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < NH_GEO; ++k) acc = fmaf(w[k], geo[k], acc);
        h[i] = acc + s[LH_B0 + i];
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < NH_HID; i += 4) {
            const float4 t = ld4(s, LH_N1 + c * NH_HID + i);
            acc = fmaf(t.x, fmaxf(h[i], 0.f), acc);
            acc = fmaf(t.y, fmaxf(h[i + 1], 0.f), acc);
            acc = fmaf(t.z, fmaxf(h[i + 2], 0.f), acc);
            acc = fmaf(t.w, fmaxf(h[i + 3], 0.f), acc);
        }
        n[c] = acc + s[LH_B1 + c];
    }
}

__global__ void __launch_bounds__(256) normal_head_fwd_kernel(NormalArgs a) {
    __shared__ __attribute__((aligned(16))) float s[LH_ALL];
    load_head(s, a.W);
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= a.P) return;
    float geo[NH_GEO], h[NH_HID], n[3];
#pragma unroll
    for (int k = 0; k < NH_GEO; ++k) geo[k] = a.o16[p * 16 + 1 + k];
    head_forward(s, geo, h, n);
    // F.normalize(x, dim=-1): x / max(||x||_2, 1e-12)
    const float nrm = fmaxf(sqrtf(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]), 1e-12f);
    const float4 r = *reinterpret_cast<const float4*>(a.raw4 + 4 * p);
    const bool keep = a.keep ? a.keep[p] != 0 : true;
    float* o = a.raw7 + 7 * p;
    o[0] = r.x; o[1] = r.y; o[2] = r.z; o[3] = r.w;
    o[4] = n[0] / nrm;
    o[5] = n[1] / nrm;
    o[6] = keep ? n[2] / nrm : 0.f;
}

constexpr int NH_TILE = 128;
constexpr int NH_OWN = (NH_ALL + NH_TILE - 1) / NH_TILE;   // gradient values per thread (5)

// at most 128 VGPRs (the LDS allows 3 blocks of 128 threads per CU; unconstrained, the compiler
// unrolls everything into 256 registers and runs one wave per SIMD)
__global__ void __launch_bounds__(NH_TILE) __attribute__((amdgpu_waves_per_eu(4))) normal_head_bwd_kernel(NormalArgs a) {
    __shared__ __attribute__((aligned(16))) float s[LH_ALL];
    __shared__ float s_dh[NH_TILE][NH_HID + 1];   // d pre-ReLU hidden
    __shared__ float s_hr[NH_TILE][NH_HID + 1];   // pre-ReLU hidden (relu applied where read)
    __shared__ float s_geo[NH_TILE][NH_GEO + 1];
    __shared__ float s_dn[NH_TILE][4];            // d pre-normalize n
    load_head(s, a.W);
    const int tid = threadIdx.x;
    float acc[NH_OWN];
#pragma unroll
    for (int j = 0; j < NH_OWN; ++j) acc[j] = 0.f;
    for (int64_t base = (int64_t)blockIdx.x * NH_TILE; base < a.P; base += (int64_t)gridDim.x * NH_TILE) {
        const int64_t p = base + tid;
        const bool valid = p < a.P;
        float geo[NH_GEO];
#pragma unroll
        for (int k = 0; k < NH_GEO; ++k) geo[k] = valid ? a.o16[p * 16 + 1 + k] : 0.f;
        // forward, one hidden unit at a time (the hidden layer goes to LDS, not registers)
        float n[3] = {s[LH_B1], s[LH_B1 + 1], s[LH_B1 + 2]}, nacc[3] = {0.f, 0.f, 0.f};
#pragma unroll 2
        for (int i = 0; i < NH_HID; ++i) {
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
            s_hr[tid][i] = hi;
            const float r = fmaxf(hi, 0.f);
#pragma unroll
            for (int c = 0; c < 3; ++c) nacc[c] = fmaf(s[LH_N1 + c * NH_HID + i], r, nacc[c]);
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) n[c] = nacc[c] + n[c];
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
#pragma unroll 2
        for (int i = 0; i < NH_HID; ++i) {
            const float dh = s_hr[tid][i] > 0.f ? (s[LH_N1 + i] * dn[0] + s[LH_N1 + NH_HID + i] * dn[1]) +
                                                       s[LH_N1 + 2 * NH_HID + i] * dn[2]
                                                : 0.f;
            s_dh[tid][i] = dh;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 t = ld4(s, LH_N0 + 16 * i + 4 * q);
                dg[4 * q] = fmaf(t.x, dh, dg[4 * q]);
                dg[4 * q + 1] = fmaf(t.y, dh, dg[4 * q + 1]);
                dg[4 * q + 2] = fmaf(t.z, dh, dg[4 * q + 2]);
                if (q < 3) dg[4 * q + 3] = fmaf(t.w, dh, dg[4 * q + 3]);
            }
        }
#pragma unroll
        for (int k = 0; k < NH_GEO; ++k) s_geo[tid][k] = geo[k];
#pragma unroll
        for (int c = 0; c < 3; ++c) s_dn[tid][c] = dn[c];
        if (valid) {
            float* d = a.dgeo + p * 16;
            d[0] = 0.f;
#pragma unroll
            for (int k = 0; k < NH_GEO; ++k) d[1 + k] = dg[k];
        }
    __syncthreads();
        // gradient value v = tid + NH_TILE j: N0 [i][k] | b0 [i] | N1 [c][i] | b1 [c], summed over the tile
#pragma unroll
        for (int j = 0; j < NH_OWN; ++j) {
            const int v = tid + NH_TILE * j;
            float t = 0.f;
            if (v < NH_B0) {
                const int i = v / NH_GEO, k = v % NH_GEO;
#pragma unroll 8
                for (int q = 0; q < NH_TILE; ++q) t = fmaf(s_dh[q][i], s_geo[q][k], t);
            } else if (v < NH_N1) {
#pragma unroll 8
                for (int q = 0; q < NH_TILE; ++q) t += s_dh[q][v - NH_B0];
            } else if (v < NH_B1) {
                const int c = (v - NH_N1) / NH_HID, i = (v - NH_N1) % NH_HID;
#pragma unroll 8
                for (int q = 0; q < NH_TILE; ++q) t = fmaf(s_dn[q][c], fmaxf(s_hr[q][i], 0.f), t);
            } else if (v < NH_ALL) {
#pragma unroll 8
                for (int q = 0; q < NH_TILE; ++q) t += s_dn[q][v - NH_B1];
            }
            acc[j] += t;
        }
        __syncthreads();
    }
    // per-block sums, reduced over blocks in order by normal_head_wgrad_reduce_kernel: every block
    // adding its 611 values with atomics serialises ~1000 adds on each address at the L2
#pragma unroll
    for (int j = 0; j < NH_OWN; ++j) {
        const int v = tid + NH_TILE * j;
        if (v < NH_ALL) a.partials[(size_t)blockIdx.x * NH_ALL + v] = acc[j];
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

static int fill_normal(NormalArgs& a, const float* o16, const uint8_t* keep, int64_t P, const nerf_normal_head* W) {
    NERF_REQUIRE(P >= 0, "normal_head: n_points < 0");
    NERF_REQUIRE((P == 0 || o16) && W && W->n0 && W->b0 && W->n1 && W->b1, "normal_head: null argument");
    a.o16 = o16;
    a.keep = keep;
    a.P = P;
    a.W = *W;
    return NERF_OK;
}

}  // namespace nerf

using namespace nerf;

extern "C" int nerf_normal_head_fwd(const float* d_o16, const float* d_raw4, const uint8_t* d_keep, int64_t n_points,
                                    const nerf_normal_head* head, float* d_raw7, void* stream) {
    NormalArgs a{};
    int rc = fill_normal(a, d_o16, d_keep, n_points, head);
    if (rc) return rc;
    NERF_REQUIRE(n_points == 0 || (d_raw4 && d_raw7), "normal_head_fwd: null buffer");
    if (n_points == 0) return NERF_OK;
    a.raw4 = d_raw4;
    a.raw7 = d_raw7;
    hipLaunchKernelGGL(normal_head_fwd_kernel, dim3(blocks_for(n_points, 256)), dim3(256), 0, as_stream(stream), a);
    NERF_CHECK_LAUNCH("normal_head_fwd");
    return NERF_OK;
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
    NERF_REQUIRE(d_workspace && workspace_bytes >= nerf_normal_head_bwd_workspace_bytes(),
                 "normal_head_bwd: workspace %zu B < %zu B", workspace_bytes, nerf_normal_head_bwd_workspace_bytes());
    if (n_points == 0) return NERF_OK;
    a.graw7 = d_graw7;
    a.graw4 = d_graw4;
    a.dgeo = d_dgeo;
    a.G = *grads;
    a.partials = d_workspace;
    const unsigned blocks = (unsigned)std::min<int64_t>(blocks_for(n_points, NH_TILE), kHeadBwdBlocks);
    hipLaunchKernelGGL(normal_head_bwd_kernel, dim3(blocks), dim3(NH_TILE), 0, as_stream(stream), a);
    NERF_CHECK_LAUNCH("normal_head_bwd");
    hipLaunchKernelGGL(normal_head_wgrad_reduce_kernel, dim3((NH_ALL + 3) / 4), dim3(256), 0, as_stream(stream),
                       d_workspace, (int)blocks, *grads);
    NERF_CHECK_LAUNCH("normal_head_bwd");
    return NERF_OK;
}
