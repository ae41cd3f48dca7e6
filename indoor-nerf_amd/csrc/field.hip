// Radiance field MLP of NeRFSmall (PocketNeRF/run_nerf_helpers.py:169-306, as create_nerf builds
// it, run_nerf.py:240-247): sigma net 32 -> 64 -> 16, colour net [SH16 | geo15] -> 64 -> 64 -> 3,
// no biases, ReLU between layers, no output activation; plus run_network's sigma := 0 outside the
// bbox (run_nerf.py:66) and SHEncoder degree 4 (hash_encoding.py:153-191) in the prologue.
//
// fp32 MFMA: v_mfma_f32_32x32x2_f32 (exact f32 fma chain in k order). One wave computes a 32-point
// tile in the TRANSPOSED orientation  Y^T[neuron][point] = W[neuron][in] * X^T[in][point]:
//   A operand (32x2):  lane l -> A[i = l&31][k = l>>5]       (weights, read from LDS)
//   B operand (2x32):  lane l -> B[k = l>>5][j = l&31]       (activations, point j = lane&31)
//   C/D (32x32):       lane l, reg r -> [row (r&3)+8(r>>2)+4(l>>5)][col l&31]
// so every layer's accumulator register r is directly the next layer's B operand for the k-pair
// {row(r,0), row(r,1)}; the A operand is read from the weight image at those (permuted) columns.
// Weight images live in LDS with odd row strides, so a 32-lane column read is conflict-free.
//
// Backward recomputes the forward tile in registers, runs the transposed chain
// (g_h3 = C2^T g_rgb, g_h2 = C1^T g_a3, g_geo = C0^T g_a2, g_h1 = W1^T g_o, g_x = W0^T g_a1), and
// forms weight gradients as MFMAs over the tile's points (K = points) with both operands staged
// through per-wave LDS in [point][neuron] layout; per-tile partial sums go to a per-block LDS
// accumulator (ds_add_f32) that is flushed to global memory once per block with fp32 atomics.
#include "field_common.h"

namespace nerf {

__global__ void __launch_bounds__(256) sh4_fwd_kernel(const float* __restrict__ d, int64_t n, float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float o[16];
    sh4_eval(d[3 * i], d[3 * i + 1], d[3 * i + 2], o);
#pragma unroll
    for (int k = 0; k < 16; k += 4)
        *reinterpret_cast<float4*>(out + 16 * i + k) = make_float4(o[k], o[k + 1], o[k + 2], o[k + 3]);
}

// Forward of one 32-point tile. Outputs: h1 (relu), o (sigma/geo rows 0..15), h2, h3 (relu), rgb.
struct FwdTile {
    floatx16 h1[2];
    floatx16 o;
    floatx16 h2[2];
    floatx16 h3[2];
    floatx16 rgb;
};

__device__ __forceinline__ void forward_tile(const float* __restrict__ lds, const float (&x)[16], const float (&shv)[8],
                                             int j, int h, FwdTile& f, bool need_rgb) {
    // L0: h1 = relu(W0 x)
    f.h1[0] = zero16();
    f.h1[1] = zero16();
#pragma unroll
    for (int s = 0; s < 16; ++s) {
        const int k = 2 * s + h;
        f.h1[0] = NERF_MFMA(lds[OFF_W0 + j * RS_W0 + k], x[s], f.h1[0]);
        f.h1[1] = NERF_MFMA(lds[OFF_W0 + (j + 32) * RS_W0 + k], x[s], f.h1[1]);
    }
    relu16(f.h1[0]);
    relu16(f.h1[1]);
    // L1: o = W1 h1 (rows 0..15 valid)
    f.o = zero16();
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r)
            f.o = NERF_MFMA(lds[OFF_W1 + j * RS_W1 + 32 * t + row_of(r, h)], f.h1[t][r], f.o);
    // C0: h2 = relu(C0y [sh ; o])
    f.h2[0] = zero16();
    f.h2[1] = zero16();
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        const int k = 2 * s + h;
        f.h2[0] = NERF_MFMA(lds[OFF_C0 + j * RS_C0 + k], shv[s], f.h2[0]);
        f.h2[1] = NERF_MFMA(lds[OFF_C0 + (j + 32) * RS_C0 + k], shv[s], f.h2[1]);
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const int k = 16 + row_of(r, h);
        f.h2[0] = NERF_MFMA(lds[OFF_C0 + j * RS_C0 + k], f.o[r], f.h2[0]);
        f.h2[1] = NERF_MFMA(lds[OFF_C0 + (j + 32) * RS_C0 + k], f.o[r], f.h2[1]);
    }
    relu16(f.h2[0]);
    relu16(f.h2[1]);
    // C1: h3 = relu(C1 h2)
    f.h3[0] = zero16();
    f.h3[1] = zero16();
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int k = 32 * t + row_of(r, h);
            f.h3[0] = NERF_MFMA(lds[OFF_C1 + j * RS_C1 + k], f.h2[t][r], f.h3[0]);
            f.h3[1] = NERF_MFMA(lds[OFF_C1 + (j + 32) * RS_C1 + k], f.h2[t][r], f.h3[1]);
        }
    relu16(f.h3[0]);
    relu16(f.h3[1]);
    if (!need_rgb) return;
    // C2: rgb = C2 h3 (rows 0..2 valid)
    f.rgb = zero16();
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r)
            f.rgb = NERF_MFMA(lds[OFF_C2 + j * RS_C2 + 32 * t + row_of(r, h)], f.h3[t][r], f.rgb);
}

__global__ void __launch_bounds__(256) mlp_fwd_kernel(MlpArgs a) {
    __shared__ float lds[LDS_W];
    load_weight_images(lds, a.W);
    __syncthreads();
    const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
    const int64_t n_tiles = (a.P + 31) / 32;
    for (int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); tile < n_tiles; tile += (int64_t)gridDim.x * 4) {
        const int64_t pt = tile * 32 + j;
        const bool valid = pt < a.P;
        float x[16], shv[8];
        load_tile_inputs(a, pt, valid, h, x, shv);
        FwdTile f;
        forward_tile(lds, x, shv, j, h, f, true);
        if (h == 0 && valid) {
            const bool keep = a.keep ? a.keep[pt] != 0 : true;
            *reinterpret_cast<float4*>(a.raw + 4 * pt) = make_float4(f.rgb[0], f.rgb[1], f.rgb[2], keep ? f.o[0] : 0.f);
        }
    }
}

// ---------------------------------------------------------------- backward
// dW[i][n] (+)= sum over the tile's 32 points of A_stage[pt][i0 + i] * B_stage[pt][n0 + n]: one
// 32x32 output tile, 16 k-steps of two points; accumulate into the block's LDS gradient image at
// gw[(i0 + i) * ld + n0 + n] for i < rows, n < cols.
__device__ __forceinline__ void wgrad_tile(const float* A, int ai0, const float* B, int bn0, float* gw, int ld,
                                           int rows, int cols, int j, int h) {
    floatx16 acc = zero16();
#pragma unroll
    for (int s = 0; s < 16; ++s) {
        const int pt = 2 * s + h;
        acc = NERF_MFMA(A[pt * RS_T + ai0 + j], B[pt * RS_T + bn0 + j], acc);
    }
    if (j < cols) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int i = row_of(r, h);
            if (i < rows) atomicAdd(gw + i * ld + j, acc[r]);
        }
    }
}

__global__ void __launch_bounds__(256) mlp_bwd_kernel(MlpArgs a) {
    __shared__ __attribute__((aligned(16))) float lds[LDS_BWD];
    float* wimg = lds;
    const int wv = threadIdx.x >> 6;
    float* stA = lds + LDS_W + wv * 2 * STAGE;     // activations [pt][neuron]
    float* stG = stA + STAGE;                       // gradients   [pt][neuron]
    float* gw = lds + LDS_W + BWD_WAVES * 2 * STAGE;
    load_weight_images(wimg, a.W);
    for (int i = threadIdx.x; i < GW_TOTAL; i += blockDim.x) gw[i] = 0.f;
    __syncthreads();

    const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
    const int64_t n_tiles = (a.P + 31) / 32;
    for (int64_t tile = (int64_t)blockIdx.x * BWD_WAVES + wv; tile < n_tiles; tile += (int64_t)gridDim.x * BWD_WAVES) {
        const int64_t p0 = tile * 32;
        const int64_t pt = p0 + j;
        const bool valid = pt < a.P;
        float x[16], shv[8];
        load_tile_inputs(a, pt, valid, h, x, shv);
        FwdTile f;
        forward_tile(wimg, x, shv, j, h, f, false);

        // upstream: g_rgb (k-pairs {0,1}, {2,-}) and g_sigma
        const float4 g4 = valid ? *reinterpret_cast<const float4*>(a.graw + 4 * pt) : make_float4(0.f, 0.f, 0.f, 0.f);
        const bool keep = valid && (a.keep ? a.keep[pt] != 0 : true);
        const float gsig = keep ? g4.w : 0.f;

        // ---- C2: g_h3 = C2^T g_rgb ; g_a3 = g_h3 * (h3 > 0)
        floatx16 ga3[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            ga3[t] = zero16();
            ga3[t] = NERF_MFMA(wimg[OFF_C2 + h * RS_C2 + 32 * t + j], h ? g4.y : g4.x, ga3[t]);
            ga3[t] = NERF_MFMA(wimg[OFF_C2 + (2 + h) * RS_C2 + 32 * t + j], h ? 0.f : g4.z, ga3[t]);
#pragma unroll
            for (int r = 0; r < 16; ++r) ga3[t][r] = f.h3[t][r] > 0.f ? ga3[t][r] : 0.f;
        }
        // dC2[i][n] = sum_pt g_rgb[pt][i] h3[pt][n]  (A = g_rgb staged in stG cols 0..2)
        stage_tile(stA, f.h3[0], 0, j, h);
        stage_tile(stA, f.h3[1], 1, j, h);
        if (h == 0) {
            stG[j * RS_T + 0] = g4.x; stG[j * RS_T + 1] = g4.y; stG[j * RS_T + 2] = g4.z;
#pragma unroll
            for (int c = 3; c < 32; ++c) stG[j * RS_T + c] = 0.f;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        wgrad_tile(stG, 0, stA, 0, gw + GW_C2, 64, 3, 32, j, h);
        wgrad_tile(stG, 0, stA, 32, gw + GW_C2 + 32, 64, 3, 32, j, h);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");

        // ---- C1: g_h2 = C1^T g_a3 ; g_a2 = g_h2 * (h2 > 0) ; dC1 = g_a3^T h2
        floatx16 ga2[2];
        ga2[0] = zero16();
        ga2[1] = zero16();
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int k = 32 * t + row_of(r, h);     // C1 output neuron = h3 neuron
                ga2[0] = NERF_MFMA(wimg[OFF_C1 + k * RS_C1 + j], ga3[t][r], ga2[0]);
                ga2[1] = NERF_MFMA(wimg[OFF_C1 + k * RS_C1 + 32 + j], ga3[t][r], ga2[1]);
            }
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) ga2[t][r] = f.h2[t][r] > 0.f ? ga2[t][r] : 0.f;
        stage_tile(stA, f.h2[0], 0, j, h);
        stage_tile(stA, f.h2[1], 1, j, h);
        stage_tile(stG, ga3[0], 0, j, h);
        stage_tile(stG, ga3[1], 1, j, h);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int u = 0; u < 2; ++u)
                wgrad_tile(stG, 32 * ti, stA, 32 * u, gw + GW_C1 + 32 * ti * 64 + 32 * u, 64, 32, 32, j, h);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");

        // ---- C0: g_y0[geo] = C0y^T g_a2 (rows i <-> o-row i, i < 16) ; dC0y = g_a2^T y0
        floatx16 go = zero16();
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int k = 32 * t + row_of(r, h);     // h2 neuron
                const float w = j < 16 ? wimg[OFF_C0 + k * RS_C0 + 16 + j] : 0.f;
                go = NERF_MFMA(w, ga2[t][r], go);
            }
        if (h == 0) go[0] = gsig;                      // o-row 0 = sigma
        // y0 stage: [pt][0..15] = sh, [pt][16..31] = o rows
#pragma unroll
        for (int s = 0; s < 8; ++s) stA[j * RS_T + 2 * s + h] = shv[s];
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            float4 q = make_float4(f.o[4 * g], f.o[4 * g + 1], f.o[4 * g + 2], f.o[4 * g + 3]);
            *reinterpret_cast<float4*>(stA + j * RS_T + 16 + 8 * g + 4 * h) = q;
        }
        stage_tile(stG, ga2[0], 0, j, h);
        stage_tile(stG, ga2[1], 1, j, h);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        // dC0 columns: y0 col c < 16 -> C0 col c; y0 col 17..31 -> C0 col c-1 (col 16 = sigma: dropped)
#pragma unroll
        for (int ti = 0; ti < 2; ++ti) {
            floatx16 acc = zero16();
#pragma unroll
            for (int s = 0; s < 16; ++s) {
                const int p = 2 * s + h;
                acc = NERF_MFMA(stG[p * RS_T + 32 * ti + j], stA[p * RS_T + j], acc);
            }
            if (j != 16) {
                const int col = j < 16 ? j : j - 1;
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    atomicAdd(gw + GW_C0 + (32 * ti + row_of(r, h)) * 31 + col, acc[r]);
            }
        }
        // optional d(SH input): g_sh = C0y[:, 0..15]^T g_a2
        if (a.dsh) {
            floatx16 gs = zero16();
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int k = 32 * t + row_of(r, h);
                    const float w = j < 16 ? wimg[OFF_C0 + k * RS_C0 + j] : 0.f;
                    gs = NERF_MFMA(w, ga2[t][r], gs);
                }
            if (valid) {
#pragma unroll
                for (int r = 0; r < 8; ++r) a.dsh[pt * 16 + row_of(r, h)] = gs[r];
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");

        // ---- W1: g_h1 = W1^T g_o ; g_a1 = g_h1 * (h1 > 0) ; dW1 = g_o^T h1
        floatx16 ga1[2];
        ga1[0] = zero16();
        ga1[1] = zero16();
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const int k = row_of(r, h);                  // o-row 0..15
            ga1[0] = NERF_MFMA(wimg[OFF_W1 + k * RS_W1 + j], go[r], ga1[0]);
            ga1[1] = NERF_MFMA(wimg[OFF_W1 + k * RS_W1 + 32 + j], go[r], ga1[1]);
        }
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) ga1[t][r] = f.h1[t][r] > 0.f ? ga1[t][r] : 0.f;
        stage_tile(stA, f.h1[0], 0, j, h);
        stage_tile(stA, f.h1[1], 1, j, h);
        stage_tile(stG, go, 0, j, h);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        wgrad_tile(stG, 0, stA, 0, gw + GW_W1, 64, 16, 32, j, h);
        wgrad_tile(stG, 0, stA, 32, gw + GW_W1 + 32, 64, 16, 32, j, h);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");

        // ---- W0: g_x = W0^T g_a1 ; dW0 = g_a1^T x
        floatx16 gx = zero16();
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int k = 32 * t + row_of(r, h);     // h1 neuron
                gx = NERF_MFMA(wimg[OFF_W0 + k * RS_W0 + j], ga1[t][r], gx);
            }
        if (a.dfeat && valid) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int fidx = row_of(r, h);           // feature 0..31
                a.dfeat[pt * a.sp + (int64_t)(fidx >> 1) * a.sl + (fidx & 1)] = gx[r];
            }
        }
        // x stage [pt][0..31]
#pragma unroll
        for (int s = 0; s < 16; ++s) stA[j * RS_T + 2 * s + h] = x[s];
        stage_tile(stG, ga1[0], 0, j, h);
        stage_tile(stG, ga1[1], 1, j, h);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        wgrad_tile(stG, 0, stA, 0, gw + GW_W0, 32, 32, 32, j, h);
        wgrad_tile(stG, 32, stA, 0, gw + GW_W0 + 32 * 32, 32, 32, 32, j, h);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    __syncthreads();
    // flush the block's weight gradients
    for (int i = threadIdx.x; i < GW_TOTAL; i += blockDim.x) {
        float* dst;
        int k;
        if (i < GW_W1) { dst = a.G.w0; k = i; }
        else if (i < GW_C0) { dst = a.G.w1; k = i - GW_W1; }
        else if (i < GW_C1) { dst = a.G.c0; k = i - GW_C0; }
        else if (i < GW_C2) { dst = a.G.c1; k = i - GW_C1; }
        else { dst = a.G.c2; k = i - GW_C2; }
        const float v = gw[i];
        if (v != 0.f) __hip_atomic_fetch_add(dst + k, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

int launch_mlp_fwd_frag(const MlpArgs& a, hipStream_t stream);   // field_frag.hip
int launch_mlp_bwd_frag(const MlpArgs& a, hipStream_t stream);

int launch_mlp_fwd_x6(const MlpArgs& a, hipStream_t stream);     // field_x6.hip
int launch_mlp_bwd_x6(const MlpArgs& a, hipStream_t stream, bool split_roles);

// MLP kernel generation, for A/B runs: NERF_MLP=1 the first version (f32 MFMA, LDS weight
// images), NERF_MLP=2 the fragment-stationary f32-MFMA version (field_frag.hip), NERF_MLP=3 the
// fp32-accurate bf16x6 version (field_x6.hip) with one wave per tile in the backward; default (4):
// bf16x6 with the backward split into chain / weight-gradient wave pairs (1.27x the one-wave x6
// backward on the lego fine pass).
static int mlp_version() {
    const char* e = getenv("NERF_MLP");
    if (e && e[0] >= '1' && e[0] <= '4') return e[0] - '0';
    return 4;
}

static bool use_frag_mlp() { return mlp_version() != 1; }

static int launch_mlp_fwd_default(const MlpArgs& a, hipStream_t stream) {
    // the activation-quantizer calibration launch (layer 0 only) stays on the f32 path
    const int v = mlp_version();
    if (v >= 3 && !a.act_minmax) return launch_mlp_fwd_x6(a, stream);
    return launch_mlp_fwd_frag(a, stream);
}

static int launch_mlp_bwd_default(const MlpArgs& a, hipStream_t stream) {
    const int v = mlp_version();
    if (v >= 3) return launch_mlp_bwd_x6(a, stream, v == 4);
    return launch_mlp_bwd_frag(a, stream);
}

static int fill_args(MlpArgs& a, const float* d_feat, int64_t sp, int64_t sl, const float* d_sh, int64_t sh_stride,
                     const float* d_viewdirs, int64_t spr, const uint8_t* d_keep, int64_t n,
                     const nerf_mlp_weights* w) {
    NERF_REQUIRE(n >= 0, "mlp: n_points < 0");
    NERF_REQUIRE(d_feat && w && w->w0 && w->w1 && w->c0 && w->c1 && w->c2, "mlp: null feature/weight pointer");
    NERF_REQUIRE(d_viewdirs || d_sh, "mlp: need d_sh or d_viewdirs");
    NERF_REQUIRE(!d_viewdirs || spr >= 1, "mlp: samples_per_ray must be >= 1");
    a.feat = d_feat; a.sp = sp; a.sl = sl; a.sh = d_sh; a.sh_stride = sh_stride;
    a.viewdirs = d_viewdirs; a.spr = spr; a.keep = d_keep; a.P = n; a.W = *w;
    return NERF_OK;
}

}  // namespace nerf

using namespace nerf;

extern "C" int nerf_sh4_fwd(const float* d_dirs, int64_t n, float* d_out, void* stream) {
    NERF_REQUIRE(n >= 0 && d_dirs && d_out, "sh4_fwd: bad args");
    if (n == 0) return NERF_OK;
    hipLaunchKernelGGL(sh4_fwd_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, as_stream(stream), d_dirs, n, d_out);
    NERF_CHECK_LAUNCH("sh4_fwd");
    return NERF_OK;
}

extern "C" int nerf_mlp_fwd_q(const float* d_feat, int64_t feat_stride_point, int64_t feat_stride_level,
                              const float* d_sh, int64_t sh_stride, const float* d_viewdirs, int64_t samples_per_ray,
                              const uint8_t* d_keep, int64_t n_points, const nerf_mlp_weights* weights, float* d_raw,
                              float* d_geo, const float* d_act_qrec, uint32_t* d_act_minmax, int64_t act_calib_points,
                              void* stream) {
    MlpArgs a{};
    int rc = fill_args(a, d_feat, feat_stride_point, feat_stride_level, d_sh, sh_stride, d_viewdirs, samples_per_ray,
                       d_keep, n_points, weights);
    if (rc) return rc;
    NERF_REQUIRE(d_raw || d_act_minmax, "mlp_fwd: null output");
    if (n_points == 0) return NERF_OK;
    a.raw = d_raw;
    a.geo_out = d_geo;
    a.aq = reinterpret_cast<const QuantRec*>(d_act_qrec);
    a.act_minmax = d_act_minmax;
    a.calib_points = act_calib_points;
    if (use_frag_mlp()) return launch_mlp_fwd_default(a, as_stream(stream));
    NERF_REQUIRE(!d_geo, "mlp_fwd: the geo output needs the default (fragment) MLP kernels");
    NERF_REQUIRE(!d_act_qrec && !d_act_minmax, "mlp_fwd: quantization needs the default (fragment) MLP kernels");
    const int64_t tiles = (n_points + 31) / 32;
    const int64_t blocks = std::min<int64_t>((tiles + 3) / 4, 256 * 3);
    hipLaunchKernelGGL(mlp_fwd_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), a);
    NERF_CHECK_LAUNCH("mlp_fwd");
    return NERF_OK;
}

extern "C" int nerf_mlp_fwd(const float* d_feat, int64_t feat_stride_point, int64_t feat_stride_level,
                            const float* d_sh, int64_t sh_stride, const float* d_viewdirs, int64_t samples_per_ray,
                            const uint8_t* d_keep, int64_t n_points, const nerf_mlp_weights* weights, float* d_raw,
                            float* d_geo, void* stream) {
    return nerf_mlp_fwd_q(d_feat, feat_stride_point, feat_stride_level, d_sh, sh_stride, d_viewdirs, samples_per_ray,
                          d_keep, n_points, weights, d_raw, d_geo, nullptr, nullptr, 0, stream);
}

extern "C" int nerf_mlp_bwd_q(const float* d_feat, int64_t feat_stride_point, int64_t feat_stride_level,
                              const float* d_sh, int64_t sh_stride, const float* d_viewdirs, int64_t samples_per_ray,
                              const uint8_t* d_keep, int64_t n_points, const nerf_mlp_weights* weights,
                              const float* d_graw, const nerf_mlp_grads* grads, float* d_dfeat, float* d_dsh,
                              const float* d_dgeo, const float* d_act_qrec, void* stream) {
    MlpArgs a{};
    int rc = fill_args(a, d_feat, feat_stride_point, feat_stride_level, d_sh, sh_stride, d_viewdirs, samples_per_ray,
                       d_keep, n_points, weights);
    if (rc) return rc;
    NERF_REQUIRE(d_graw && grads && grads->w0 && grads->w1 && grads->c0 && grads->c1 && grads->c2,
                 "mlp_bwd: null gradient pointer");
    if (n_points == 0) return NERF_OK;
    a.graw = d_graw; a.G = *grads; a.dfeat = d_dfeat; a.dsh = d_dsh; a.dgeo = d_dgeo;
    a.aq = reinterpret_cast<const QuantRec*>(d_act_qrec);
    if (use_frag_mlp()) return launch_mlp_bwd_default(a, as_stream(stream));
    NERF_REQUIRE(!d_dgeo, "mlp_bwd: the geo gradient input needs the default (fragment) MLP kernels");
    NERF_REQUIRE(!d_act_qrec, "mlp_bwd: quantization needs the default (fragment) MLP kernels");
    const int64_t tiles = (n_points + 31) / 32;
    const int64_t blocks = std::min<int64_t>((tiles + BWD_WAVES - 1) / BWD_WAVES, 256);
    hipLaunchKernelGGL(mlp_bwd_kernel, dim3((unsigned)blocks), dim3(64 * BWD_WAVES), 0, as_stream(stream), a);
    NERF_CHECK_LAUNCH("mlp_bwd");
    return NERF_OK;
}

extern "C" int nerf_mlp_bwd(const float* d_feat, int64_t feat_stride_point, int64_t feat_stride_level,
                            const float* d_sh, int64_t sh_stride, const float* d_viewdirs, int64_t samples_per_ray,
                            const uint8_t* d_keep, int64_t n_points, const nerf_mlp_weights* weights,
                            const float* d_graw, const nerf_mlp_grads* grads, float* d_dfeat, float* d_dsh,
                            const float* d_dgeo, void* stream) {
    return nerf_mlp_bwd_q(d_feat, feat_stride_point, feat_stride_level, d_sh, sh_stride, d_viewdirs, samples_per_ray,
                          d_keep, n_points, weights, d_graw, grads, d_dfeat, d_dsh, d_dgeo, nullptr, stream);
}
