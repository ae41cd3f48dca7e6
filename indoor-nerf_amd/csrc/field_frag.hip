// Field MLP, fragment-stationary version (the default; field.hip holds the first version, kept for
// A/B runs with NERF_MLP=1).
//
// Every MFMA of the chain takes its A operand (a weight) from a per-lane "fragment": fragment f of
// lane l is the one float that lane must feed to the f-th MFMA of the fixed instruction sequence
// (layouts and orientation: field.hip header). The fragment table below lists all 372 of them.
//   forward : the 192 forward fragments are an LDS image laid out [group of 4][lane][4]: one
//             conflict-free ds_read_b128 feeds four consecutive MFMAs (48 per tile instead of 192
//             ds_read_b32). Holding them in registers instead does not fit beside the activations
//             in the 256 architectural VGPRs (hipcc spills 784 B/lane).
//   backward: the 340 fragments it needs (forward recompute + transposed chain) form the same kind
//             of LDS image; the
//             weight-gradient accumulators (12 tiles of 32x32 = 192 registers) stay in registers
//             across all tiles a wave processes and are reduced once per block at the end.
#include "field_common.h"

namespace nerf {

// ---- fragment table (lane l: j = l & 31, h = l >> 5; row(r,h) = (r&3) + 8(r>>2) + 4h)
constexpr int F_L0 = 0;       // 32  t*16+s      W0[j+32t][2s+h]
constexpr int F_L1 = 32;      // 32  t*16+r      j<16 ? W1[j][32t+row] : 0
constexpr int F_C0S = 64;     // 16  t*8+s       C0[j+32t][2s+h]                      (SH inputs)
constexpr int F_C0O = 80;     // 16  t*8+r       rho=row: rho ? C0[j+32t][15+rho] : 0  (o rows; rho 0 = sigma)
constexpr int F_C1 = 96;      // 64  to*32+ti*16+r   C1[j+32to][32ti+row]
constexpr int F_C2 = 160;     // 32  ti*16+r     j<3 ? C2[j][32ti+row] : 0
constexpr int F_FWD = 192;
constexpr int F_C2T = 192;    // 4   t*2+q       k=2q+h: k<3 ? C2[k][32t+j] : 0
constexpr int F_C1T = 196;    // 64  to*32+ti*16+r   k=32ti+row: C1[k][32to+j]
constexpr int F_C0GT = 260;   // 32  ti*16+r     k=32ti+row: 1<=j<16 ? C0[k][15+j] : 0
constexpr int F_W1T = 292;    // 16  t*8+r       k=row (<16): W1[k][32t+j]
constexpr int F_W0T = 308;    // 32  ti*16+r     k=32ti+row: W0[k][j]
constexpr int F_C0ST = 340;   // 32  ti*16+r     k=32ti+row: j<16 ? C0[k][j] : 0
constexpr int F_ALL = 372;

__device__ inline float frag_value(int f, int lane, const nerf_mlp_weights& W) {
    const int j = lane & 31, h = lane >> 5;
    if (f < F_L1) { const int t = (f - F_L0) >> 4, s = (f - F_L0) & 15; return W.w0[(j + 32 * t) * 32 + 2 * s + h]; }
    if (f < F_C0S) {
        const int t = (f - F_L1) >> 4, r = (f - F_L1) & 15;
        return j < 16 ? W.w1[j * 64 + 32 * t + row_of(r, h)] : 0.f;
    }
    if (f < F_C0O) { const int t = (f - F_C0S) >> 3, s = (f - F_C0S) & 7; return W.c0[(j + 32 * t) * 31 + 2 * s + h]; }
    if (f < F_C1) {
        const int t = (f - F_C0O) >> 3, r = (f - F_C0O) & 7, rho = row_of(r, h);
        return rho ? W.c0[(j + 32 * t) * 31 + 15 + rho] : 0.f;
    }
    if (f < F_C2) {
        const int q = f - F_C1, to = q >> 5, ti = (q >> 4) & 1, r = q & 15;
        return W.c1[(j + 32 * to) * 64 + 32 * ti + row_of(r, h)];
    }
    if (f < F_C2T) {
        const int ti = (f - F_C2) >> 4, r = (f - F_C2) & 15;
        return j < 3 ? W.c2[j * 64 + 32 * ti + row_of(r, h)] : 0.f;
    }
    if (f < F_C1T) {
        const int q = f - F_C2T, t = q >> 1, k = 2 * (q & 1) + h;
        return k < 3 ? W.c2[k * 64 + 32 * t + j] : 0.f;
    }
    if (f < F_C0GT) {
        const int q = f - F_C1T, to = q >> 5, ti = (q >> 4) & 1, r = q & 15;
        return W.c1[(32 * ti + row_of(r, h)) * 64 + 32 * to + j];
    }
    if (f < F_W1T) {
        const int ti = (f - F_C0GT) >> 4, r = (f - F_C0GT) & 15;
        return (j >= 1 && j < 16) ? W.c0[(32 * ti + row_of(r, h)) * 31 + 15 + j] : 0.f;
    }
    if (f < F_W0T) {
        const int t = (f - F_W1T) >> 3, r = (f - F_W1T) & 7;
        return W.w1[row_of(r, h) * 64 + 32 * t + j];
    }
    if (f < F_C0ST) {
        const int ti = (f - F_W0T) >> 4, r = (f - F_W0T) & 15;
        return W.w0[(32 * ti + row_of(r, h)) * 32 + j];
    }
    const int ti = (f - F_C0ST) >> 4, r = (f - F_C0ST) & 15;
    return j < 16 ? W.c0[(32 * ti + row_of(r, h)) * 31 + j] : 0.f;
}

struct TileIn {
    float x[16];
    float shv[8];
    int64_t pt;
    bool valid;
};

__device__ __forceinline__ void load_in(const MlpArgs& a, int64_t tile, int j, int h, TileIn& in) {
    in.pt = tile * 32 + j;
    in.valid = in.pt < a.P;
    load_tile_inputs(a, in.pt, in.valid, h, in.x, in.shv);
}

struct Acts {
    floatx16 h1[2];
    floatx16 o;
    floatx16 h2[2];
    floatx16 h3[2];
    floatx16 rgb;
};

// ================================================================ forward
// Forward fragments [0, 192) as an LDS image [group of 4][lane][4]: one ds_read_b128 feeds four
// consecutive MFMAs of a layer (v1 issued one ds_read_b32 per MFMA).
constexpr int LDS_FWD_FR = F_FWD * 64;   // 12,288 floats = 48 KiB

__device__ __forceinline__ float4 frag4f(const float* img, int f, int lane) {
    return *reinterpret_cast<const float4*>(img + (f >> 2) * 256 + lane * 4);
}

__device__ __forceinline__ float q4f(const float4& v, int q) { return q == 0 ? v.x : q == 1 ? v.y : q == 2 ? v.z : v.w; }

template <bool QUANT>
__device__ __forceinline__ void fwd_tile(const float* img, const TileIn& A, Acts& a, int lane, bool need_rgb,
                                         const QuantRec& aq) {
    a.h1[0] = a.h1[1] = zero16();
#pragma unroll
    for (int sg = 0; sg < 4; ++sg) {
        const float4 w0 = frag4f(img, F_L0 + 4 * sg, lane), w1 = frag4f(img, F_L0 + 16 + 4 * sg, lane);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            a.h1[0] = NERF_MFMA(q4f(w0, q), A.x[4 * sg + q], a.h1[0]);
            a.h1[1] = NERF_MFMA(q4f(w1, q), A.x[4 * sg + q], a.h1[1]);
        }
    }
    relu16(a.h1[0]); relu16(a.h1[1]);
    if constexpr (QUANT) { fake_quant16(a.h1[0], aq); fake_quant16(a.h1[1], aq); }
    __builtin_amdgcn_sched_barrier(0);
    a.o = zero16();
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) {
            const float4 w = frag4f(img, F_L1 + t * 16 + 4 * rg, lane);
#pragma unroll
            for (int q = 0; q < 4; ++q) a.o = NERF_MFMA(q4f(w, q), a.h1[t][4 * rg + q], a.o);
        }
    __builtin_amdgcn_sched_barrier(0);
    a.h2[0] = a.h2[1] = zero16();
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            const float4 ws = frag4f(img, F_C0S + t * 8 + 4 * g, lane);
            const float4 wo = frag4f(img, F_C0O + t * 8 + 4 * g, lane);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                a.h2[t] = NERF_MFMA(q4f(ws, q), A.shv[4 * g + q], a.h2[t]);
                a.h2[t] = NERF_MFMA(q4f(wo, q), a.o[4 * g + q], a.h2[t]);
            }
        }
    relu16(a.h2[0]); relu16(a.h2[1]);
    __builtin_amdgcn_sched_barrier(0);
    a.h3[0] = a.h3[1] = zero16();
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) {
            const float4 w0 = frag4f(img, F_C1 + 0 * 32 + ti * 16 + 4 * rg, lane);
            const float4 w1 = frag4f(img, F_C1 + 1 * 32 + ti * 16 + 4 * rg, lane);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                a.h3[0] = NERF_MFMA(q4f(w0, q), a.h2[ti][4 * rg + q], a.h3[0]);
                a.h3[1] = NERF_MFMA(q4f(w1, q), a.h2[ti][4 * rg + q], a.h3[1]);
            }
        }
    relu16(a.h3[0]); relu16(a.h3[1]);
    if (!need_rgb) return;
    __builtin_amdgcn_sched_barrier(0);
    a.rgb = zero16();
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) {
            const float4 w = frag4f(img, F_C2 + ti * 16 + 4 * rg, lane);
#pragma unroll
            for (int q = 0; q < 4; ++q) a.rgb = NERF_MFMA(q4f(w, q), a.h3[ti][4 * rg + q], a.rgb);
        }
}

__device__ __forceinline__ void store_raw(const MlpArgs& a, const TileIn& in, const Acts& v, int h) {
    if (h == 0 && in.valid) {
        const bool keep = a.keep ? a.keep[in.pt] != 0 : true;
        *reinterpret_cast<float4*>(a.raw + 4 * in.pt) = make_float4(v.rgb[0], v.rgb[1], v.rgb[2], keep ? v.o[0] : 0.f);
    }
    if (a.geo_out && in.valid) {   // o rows 0..15 of this point: registers r with row_of(r, h) < 16
#pragma unroll
        for (int r = 0; r < 8; ++r) a.geo_out[in.pt * 16 + row_of(r, h)] = v.o[r];
    }
}

template <bool QUANT>
__global__ void __launch_bounds__(256, 2) mlp_fwd_frag_kernel(MlpArgs a) {
    __shared__ __attribute__((aligned(16))) float img[LDS_FWD_FR];
    for (int idx = threadIdx.x; idx < LDS_FWD_FR; idx += blockDim.x) {
        const int f = idx >> 6, ln = idx & 63;
        img[(f >> 2) * 256 + ln * 4 + (f & 3)] = frag_value(f, ln, a.W);
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
    QuantRec aq{};
    if constexpr (QUANT) aq = *a.aq;
    const int64_t n_tiles = (a.P + 31) / 32;
    for (int64_t t0 = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); t0 < n_tiles; t0 += (int64_t)gridDim.x * 4) {
        TileIn A;
        load_in(a, t0, j, h, A);
        Acts va;
        fwd_tile<QUANT>(img, A, va, lane, true, aq);
        store_raw(a, A, va, h);
    }
}

// Calibration-only launch of the activation quantizer (quantization.py:97-119 on the first
// netchunk's h = relu(x W0^T)): layer 0 per tile, wave min/max, one atomic pair per wave.
__global__ void __launch_bounds__(256) mlp_act_minmax_kernel(MlpArgs a) {
    __shared__ __attribute__((aligned(16))) float img[32 * 64];
    for (int idx = threadIdx.x; idx < 32 * 64; idx += blockDim.x) {
        const int f = idx >> 6, ln = idx & 63;
        img[(f >> 2) * 256 + ln * 4 + (f & 3)] = frag_value(F_L0 + f, ln, a.W);
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
    const int64_t n = a.calib_points < a.P ? a.calib_points : a.P;
    const int64_t n_tiles = (n + 31) / 32;
    float lo = INFINITY, hi = -INFINITY;
    for (int64_t t0 = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); t0 < n_tiles; t0 += (int64_t)gridDim.x * 4) {
        TileIn A;
        load_in(a, t0, j, h, A);
        floatx16 h1[2];
        h1[0] = h1[1] = zero16();
#pragma unroll
        for (int sg = 0; sg < 4; ++sg) {
            const float4 w0 = frag4f(img, F_L0 + 4 * sg, lane), w1 = frag4f(img, F_L0 + 16 + 4 * sg, lane);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                h1[0] = NERF_MFMA(q4f(w0, q), A.x[4 * sg + q], h1[0]);
                h1[1] = NERF_MFMA(q4f(w1, q), A.x[4 * sg + q], h1[1]);
            }
        }
        relu16(h1[0]); relu16(h1[1]);
        if (A.pt < n) {
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

// ================================================================ backward
constexpr int BWD_FRAGS = F_C2 + (F_ALL - F_C2T);   // 160 + 180 = 340 (C2 forward fragments not needed)
constexpr int LDS_FR = BWD_FRAGS * 64;              // 21,760 floats
constexpr int LDS_BWD2 = LDS_FR + 4 * 2 * STAGE;    // 39,168 floats = 156,672 B

__device__ __forceinline__ int compact_frag(int f) { return f < F_C2 ? f : f - (F_C2T - F_C2); }

__device__ __forceinline__ float4 frag4(const float* img, int f, int lane) {
    return *reinterpret_cast<const float4*>(img + (compact_frag(f) >> 2) * 256 + lane * 4);
}

__device__ __forceinline__ float q4(const float4& v, int q) { return q == 0 ? v.x : q == 1 ? v.y : q == 2 ? v.z : v.w; }

#define NERF_WAVE_SYNC()                                       \
    do {                                                       \
        __builtin_amdgcn_wave_barrier();                       \
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); \
        __builtin_amdgcn_sched_barrier(0);                     \
    } while (0)

// dst += sum over the tile's 32 points of A_stage[pt][ai0 + i] * B_stage[pt][bn0 + n]
__device__ __forceinline__ void wgrad_acc(floatx16& acc, const float* A, int ai0, const float* B, int bn0, int j, int h) {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
        const int p = 2 * s + h;
        acc = NERF_MFMA(A[p * RS_T + ai0 + j], B[p * RS_T + bn0 + j], acc);
    }
}

template <bool QUANT>
__global__ void __launch_bounds__(256, 1) mlp_bwd_frag_kernel(MlpArgs a) {
    __shared__ __attribute__((aligned(16))) float lds[LDS_BWD2];
    float* img = lds;
    const int wv = threadIdx.x >> 6;
    float* stA = lds + LDS_FR + wv * 2 * STAGE;
    float* stG = stA + STAGE;
    for (int idx = threadIdx.x; idx < LDS_FR; idx += blockDim.x) {
        const int c = idx >> 6, ln = idx & 63;                 // compacted fragment, lane
        const int f = c < F_C2 ? c : c + (F_C2T - F_C2);
        img[(c >> 2) * 256 + ln * 4 + (c & 3)] = frag_value(f, ln, a.W);
    }
    __syncthreads();

    const int lane = threadIdx.x & 63, j = lane & 31, h = lane >> 5;
    QuantRec aq{};
    if constexpr (QUANT) aq = *a.aq;
    floatx16 dC2[2], dC1[4], dC0[2], dW1[2], dW0[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) { dC2[i] = zero16(); dC0[i] = zero16(); dW1[i] = zero16(); dW0[i] = zero16(); }
#pragma unroll
    for (int i = 0; i < 4; ++i) dC1[i] = zero16();

    const int64_t n_tiles = (a.P + 31) / 32;
    for (int64_t tile = (int64_t)blockIdx.x * 4 + wv; tile < n_tiles; tile += (int64_t)gridDim.x * 4) {
        TileIn in;
        load_in(a, tile, j, h, in);
        // ---- forward recompute (fragments from LDS, 4 per ds_read_b128)
        Acts f;
        f.h1[0] = f.h1[1] = zero16();
#pragma unroll
        for (int sg = 0; sg < 4; ++sg) {
            const float4 w0 = frag4(img, F_L0 + 4 * sg, lane), w1 = frag4(img, F_L0 + 16 + 4 * sg, lane);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                f.h1[0] = NERF_MFMA(q4(w0, q), in.x[4 * sg + q], f.h1[0]);
                f.h1[1] = NERF_MFMA(q4(w1, q), in.x[4 * sg + q], f.h1[1]);
            }
        }
        relu16(f.h1[0]); relu16(f.h1[1]);
        // with the activation quantizer, h1 holds Q(relu(pre)) and the ReLU mask is kept as bits
        uint32_t m1 = 0;
        if constexpr (QUANT) {
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) m1 |= (f.h1[t][r] > 0.f ? 1u : 0u) << (16 * t + r);
            fake_quant16(f.h1[0], aq); fake_quant16(f.h1[1], aq);
        }
        __builtin_amdgcn_sched_barrier(0);
        f.o = zero16();
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int rg = 0; rg < 4; ++rg) {
                const float4 w = frag4(img, F_L1 + t * 16 + 4 * rg, lane);
#pragma unroll
                for (int q = 0; q < 4; ++q) f.o = NERF_MFMA(q4(w, q), f.h1[t][4 * rg + q], f.o);
            }
        __builtin_amdgcn_sched_barrier(0);
        f.h2[0] = f.h2[1] = zero16();
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int g = 0; g < 2; ++g) {
                const float4 ws = frag4(img, F_C0S + t * 8 + 4 * g, lane);
                const float4 wo = frag4(img, F_C0O + t * 8 + 4 * g, lane);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    f.h2[t] = NERF_MFMA(q4(ws, q), in.shv[4 * g + q], f.h2[t]);
                    f.h2[t] = NERF_MFMA(q4(wo, q), f.o[4 * g + q], f.h2[t]);
                }
            }
        relu16(f.h2[0]); relu16(f.h2[1]);
        __builtin_amdgcn_sched_barrier(0);
        f.h3[0] = f.h3[1] = zero16();
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int rg = 0; rg < 4; ++rg) {
                const float4 w0 = frag4(img, F_C1 + 0 * 32 + ti * 16 + 4 * rg, lane);
                const float4 w1 = frag4(img, F_C1 + 1 * 32 + ti * 16 + 4 * rg, lane);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    f.h3[0] = NERF_MFMA(q4(w0, q), f.h2[ti][4 * rg + q], f.h3[0]);
                    f.h3[1] = NERF_MFMA(q4(w1, q), f.h2[ti][4 * rg + q], f.h3[1]);
                }
            }
        relu16(f.h3[0]); relu16(f.h3[1]);
        __builtin_amdgcn_sched_barrier(0);

        // ---- upstream gradients
        const float4 g4 = in.valid ? *reinterpret_cast<const float4*>(a.graw + 4 * in.pt) : make_float4(0.f, 0.f, 0.f, 0.f);
        const bool keep = in.valid && (a.keep ? a.keep[in.pt] != 0 : true);
        const float gsig = keep ? g4.w : 0.f;

        // ---- C2: g_a3 = (C2^T g_rgb) * (h3 > 0)
        floatx16 ga3[2];
        {
            const float4 w = frag4(img, F_C2T, lane);   // [t0q0, t0q1, t1q0, t1q1]
            const float b0 = h ? g4.y : g4.x, b1 = h ? 0.f : g4.z;
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                ga3[t] = zero16();
                ga3[t] = NERF_MFMA(q4(w, 2 * t), b0, ga3[t]);
                ga3[t] = NERF_MFMA(q4(w, 2 * t + 1), b1, ga3[t]);
#pragma unroll
                for (int r = 0; r < 16; ++r) ga3[t][r] = f.h3[t][r] > 0.f ? ga3[t][r] : 0.f;
            }
        }
        stage_tile(stA, f.h3[0], 0, j, h);
        stage_tile(stA, f.h3[1], 1, j, h);
        if (h == 0) {
            *reinterpret_cast<float4*>(stG + j * RS_T) = make_float4(g4.x, g4.y, g4.z, 0.f);
#pragma unroll
            for (int c = 4; c < 32; c += 4) *reinterpret_cast<float4*>(stG + j * RS_T + c) = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        NERF_WAVE_SYNC();
        wgrad_acc(dC2[0], stG, 0, stA, 0, j, h);
        wgrad_acc(dC2[1], stG, 0, stA, 32, j, h);
        NERF_WAVE_SYNC();

        // ---- C1: g_a2 = (C1^T g_a3) * (h2 > 0) ; dC1 += g_a3^T h2
        floatx16 ga2[2];
        ga2[0] = ga2[1] = zero16();
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int rg = 0; rg < 4; ++rg) {
                const float4 w0 = frag4(img, F_C1T + 0 * 32 + ti * 16 + 4 * rg, lane);
                const float4 w1 = frag4(img, F_C1T + 1 * 32 + ti * 16 + 4 * rg, lane);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    ga2[0] = NERF_MFMA(q4(w0, q), ga3[ti][4 * rg + q], ga2[0]);
                    ga2[1] = NERF_MFMA(q4(w1, q), ga3[ti][4 * rg + q], ga2[1]);
                }
            }
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) ga2[t][r] = f.h2[t][r] > 0.f ? ga2[t][r] : 0.f;
        stage_tile(stA, f.h2[0], 0, j, h);
        stage_tile(stA, f.h2[1], 1, j, h);
        stage_tile(stG, ga3[0], 0, j, h);
        stage_tile(stG, ga3[1], 1, j, h);
        NERF_WAVE_SYNC();
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int u = 0; u < 2; ++u) wgrad_acc(dC1[ti * 2 + u], stG, 32 * ti, stA, 32 * u, j, h);
        NERF_WAVE_SYNC();

        // ---- C0: g_o(geo rows) = C0y^T g_a2 ; o-row 0 = g_sigma ; dC0y += g_a2^T y0
        // The accumulator is seeded rather than patched after the MFMAs: row 0 (sigma) with g_sigma
        // (the C0GT fragments are zero for row 0) and, with the normals head, rows 1..15 with its
        // d geo. A VALU read-modify-write of these accumulator registers right after the MFMA chain
        // produced wrong sums when both terms were non-zero (ROCm 7.2, gfx950).
        floatx16 go = zero16();
        if (h == 0) go[0] = gsig;
        if (a.dgeo && in.valid) {
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int row = row_of(r, h);
                if (row >= 1) go[r] = a.dgeo[in.pt * 16 + row];
            }
        }
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int rg = 0; rg < 4; ++rg) {
                const float4 w = frag4(img, F_C0GT + ti * 16 + 4 * rg, lane);
#pragma unroll
                for (int q = 0; q < 4; ++q) go = NERF_MFMA(q4(w, q), ga2[ti][4 * rg + q], go);
            }
#pragma unroll
        for (int s = 0; s < 8; ++s) stA[j * RS_T + 2 * s + h] = in.shv[s];
#pragma unroll
        for (int g = 0; g < 2; ++g)
            *reinterpret_cast<float4*>(stA + j * RS_T + 16 + 8 * g + 4 * h) =
                make_float4(f.o[4 * g], f.o[4 * g + 1], f.o[4 * g + 2], f.o[4 * g + 3]);
        stage_tile(stG, ga2[0], 0, j, h);
        stage_tile(stG, ga2[1], 1, j, h);
        NERF_WAVE_SYNC();
        wgrad_acc(dC0[0], stG, 0, stA, 0, j, h);
        wgrad_acc(dC0[1], stG, 32, stA, 0, j, h);
        if (a.dsh) {
            floatx16 gs = zero16();
#pragma unroll
            for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                for (int rg = 0; rg < 4; ++rg) {
                    const float4 w = frag4(img, F_C0ST + ti * 16 + 4 * rg, lane);
#pragma unroll
                    for (int q = 0; q < 4; ++q) gs = NERF_MFMA(q4(w, q), ga2[ti][4 * rg + q], gs);
                }
            if (in.valid) {
#pragma unroll
                for (int r = 0; r < 8; ++r) a.dsh[in.pt * 16 + row_of(r, h)] = gs[r];
            }
        }
        NERF_WAVE_SYNC();

        // ---- W1: g_a1 = (W1^T g_o) * (h1 > 0) ; dW1 += g_o^T h1
        floatx16 ga1[2];
        ga1[0] = ga1[1] = zero16();
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int g = 0; g < 2; ++g) {
                const float4 w = frag4(img, F_W1T + t * 8 + 4 * g, lane);
#pragma unroll
                for (int q = 0; q < 4; ++q) ga1[t] = NERF_MFMA(q4(w, q), go[4 * g + q], ga1[t]);
            }
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const bool on = QUANT ? ((m1 >> (16 * t + r)) & 1u) != 0u : f.h1[t][r] > 0.f;
                ga1[t][r] = on ? ga1[t][r] : 0.f;
            }
        stage_tile(stA, f.h1[0], 0, j, h);
        stage_tile(stA, f.h1[1], 1, j, h);
        stage_tile(stG, go, 0, j, h);
        NERF_WAVE_SYNC();
        wgrad_acc(dW1[0], stG, 0, stA, 0, j, h);
        wgrad_acc(dW1[1], stG, 0, stA, 32, j, h);
        NERF_WAVE_SYNC();

        // ---- W0: g_x = W0^T g_a1 ; dW0 += g_a1^T x
        floatx16 gx = zero16();
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
            for (int rg = 0; rg < 4; ++rg) {
                const float4 w = frag4(img, F_W0T + ti * 16 + 4 * rg, lane);
#pragma unroll
                for (int q = 0; q < 4; ++q) gx = NERF_MFMA(q4(w, q), ga1[ti][4 * rg + q], gx);
            }
        if (a.dfeat && in.valid) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int fi = row_of(r, h);
                a.dfeat[in.pt * a.sp + (int64_t)(fi >> 1) * a.sl + (fi & 1)] = gx[r];
            }
        }
#pragma unroll
        for (int s = 0; s < 16; ++s) stA[j * RS_T + 2 * s + h] = in.x[s];
        stage_tile(stG, ga1[0], 0, j, h);
        stage_tile(stG, ga1[1], 1, j, h);
        NERF_WAVE_SYNC();
        wgrad_acc(dW0[0], stG, 0, stA, 0, j, h);
        wgrad_acc(dW0[1], stG, 32, stA, 0, j, h);
        NERF_WAVE_SYNC();
    }

    // ---- block reduction of the weight gradients, then one atomic flush per block
    __syncthreads();
    float* gw = lds;                                   // the fragment image is no longer needed
    for (int i = threadIdx.x; i < GW_TOTAL; i += blockDim.x) gw[i] = 0.f;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int rr = row_of(r, h);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            if (rr < 3) atomicAdd(gw + GW_C2 + rr * 64 + 32 * u + j, dC2[u][r]);
            if (rr < 16) atomicAdd(gw + GW_W1 + rr * 64 + 32 * u + j, dW1[u][r]);
        }
#pragma unroll
        for (int ti = 0; ti < 2; ++ti) {
            const int row = 32 * ti + rr;
#pragma unroll
            for (int u = 0; u < 2; ++u) atomicAdd(gw + GW_C1 + row * 64 + 32 * u + j, dC1[ti * 2 + u][r]);
            if (j != 16) atomicAdd(gw + GW_C0 + row * 31 + (j < 16 ? j : j - 1), dC0[ti][r]);
            atomicAdd(gw + GW_W0 + row * 32 + j, dW0[ti][r]);
        }
    }
    __syncthreads();
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

int launch_mlp_fwd_frag(const MlpArgs& a, hipStream_t stream) {
    const int64_t tiles = (a.P + 31) / 32;
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((tiles + 3) / 4, 256 * 3));
    if (a.act_minmax) {
        const int64_t n = a.calib_points < a.P ? a.calib_points : a.P;
        if (n <= 0) return NERF_OK;
        const int64_t cb = std::max<int64_t>(1, std::min<int64_t>(((n + 31) / 32 + 3) / 4, 256 * 4));
        hipLaunchKernelGGL(mlp_act_minmax_kernel, dim3((unsigned)cb), dim3(256), 0, stream, a);
        NERF_CHECK_LAUNCH("mlp_fwd(act calibration)");
        return NERF_OK;
    }
    if (a.aq)
        hipLaunchKernelGGL(mlp_fwd_frag_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, stream, a);
    else
        hipLaunchKernelGGL(mlp_fwd_frag_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, stream, a);
    NERF_CHECK_LAUNCH("mlp_fwd(frag)");
    return NERF_OK;
}

int launch_mlp_bwd_frag(const MlpArgs& a, hipStream_t stream) {
    const int64_t tiles = (a.P + 31) / 32;
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((tiles + 3) / 4, 256));
    if (a.aq)
        hipLaunchKernelGGL(mlp_bwd_frag_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, stream, a);
    else
        hipLaunchKernelGGL(mlp_bwd_frag_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, stream, a);
    NERF_CHECK_LAUNCH("mlp_bwd(frag)");
    return NERF_OK;
}

}  // namespace nerf
