// A-CAQ learned-bitwidth quantization (PocketNeRF/quantization.py:63-187) on the hash-grid path.
//
//   nerf_quant_params        LearnedBitwidthQuantizer.forward's scalar algebra (:158-178) for up to
//                            32 quantizers in one launch (no host sync: the reference's .item() of
//                            the integer bit width is evaluated on the device, exactly)
//   nerf_quant_minmax*       calibration statistics (order-preserving uint32 atomics)
//   nerf_hash_gather_minmax  the [P,8,2] corner gather of every level, reduced to min/max (the x
//                            the level quantizer calibrates on, hash_encoding.py:94-101)
//   nerf_quant_calibrate     calibrate() (:97-119)
//   nerf_fake_quant          the elementwise quantizer (W0 weight quantizer, standalone modules)
//   packed tables            eval-mode quantizer output (q - zp) * scale depends only on the code
//                            q, so the tables are stored as 4/8/16-bit codes and the gather reads
//                            1/2/4 bytes per corner instead of 8 (nerf_hash_encode_fwd_packed).
#include <math.h>

#include "hash_common.h"

namespace nerf {

struct QuantizerSet {
    nerf_quantizer q[NERF_MAX_QUANTIZERS];
};

// 2 ** B for a float tensor exponent: evaluated in double and rounded once, the correctly rounded
// value glibc's powf returns (torch CPU pow of a 0-dim tensor).
__device__ __forceinline__ float pow2f_exact(float b) { return (float)exp2((double)b); }

// float(python int) for 2^k - 1 and -(2^(k-1)): int64 -> float32 rounding, as torch casts scalars.
__device__ __forceinline__ float int_to_f32(int64_t v) { return (float)v; }

__global__ void quant_params_kernel(QuantizerSet set, int n, int training, QuantRec* __restrict__ out) {
    const int i = threadIdx.x;
    if (i >= n) return;
    const nerf_quantizer& d = set.q[i];
    const bool sym = d.v_max == nullptr;
    const float bw = fminf(fmaxf(*d.soft_bits, d.min_bits), d.max_bits);   // torch.clamp(soft_bits, min, max)
    const int bi = (int)rintf(bw);                                           // int(torch.round(bit_width))
    QuantRec r;
    if (sym) {
        r.qmin = int_to_f32(-(int64_t(1) << (bi - 1)));
        r.qmax = int_to_f32((int64_t(1) << (bi - 1)) - 1);
    } else {
        r.qmin = 0.f;
        r.qmax = int_to_f32((int64_t(1) << bi) - 1);
    }
    const float range = *d.range_scale;
    float scale;
    if (sym) {
        // training: range / 2 ** (B - 1) with B a tensor; eval: range / (python int 2 ** (B - 1))
        const float den = training ? pow2f_exact(bw - 1.0f) : int_to_f32(int64_t(1) << (bi - 1));
        scale = range / den;
        r.zp = 0.f;
    } else {
        const float rv = fmaxf(range, 1e-8f);                                // clamp(range_scale, min=1e-8)
        const float den = training ? (pow2f_exact(bw) - 1.0f) : int_to_f32((int64_t(1) << bi) - 1);
        scale = rv / den;
        const float z = fminf(fmaxf(*d.v_max / scale, r.qmin), r.qmax);    // clamp(v_max / scale, qmin, qmax)
        r.zp = rintf(z);
    }
    r.scale = scale;
    r.scale_eps = scale + 1e-8f;
    r.ste = training ? 1.f : 0.f;
    r.bits = (float)bi;
    r.pad = 0.f;
    out[i] = r;
}

__global__ void minmax_reset_kernel(uint32_t* mm, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        mm[2 * i] = 0xFFFFFFFFu;   // encodes the largest value (NaN payloads sort above +inf; none expected)
        mm[2 * i + 1] = 0u;
    }
}

__device__ __forceinline__ void block_minmax_commit(float lo, float hi, uint32_t* mm) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        lo = fminf(lo, __shfl_xor(lo, o, 64));
        hi = fmaxf(hi, __shfl_xor(hi, o, 64));
    }
    if ((threadIdx.x & 63) == 0 && lo <= hi) {
        atomicMin(mm, f2ord(lo));
        atomicMax(mm + 1, f2ord(hi));
    }
}

__global__ void __launch_bounds__(256) minmax_kernel(const float* __restrict__ x, int64_t n, uint32_t* mm) {
    float lo = INFINITY, hi = -INFINITY;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float v = x[i];
        lo = fminf(lo, v);
        hi = fmaxf(hi, v);
    }
    block_minmax_commit(lo, hi, mm);
}

__global__ void __launch_bounds__(256) hash_gather_minmax_kernel(const float* __restrict__ xyz, int64_t n,
                                                                 HashParams hp, uint32_t* mm) {
    const int lvl = blockIdx.y;
    const float2* __restrict__ tab = reinterpret_cast<const float2*>(hp.tables[lvl]);
    float lo = INFINITY, hi = -INFINITY;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x) {
        const AxisCell ax = axis_cell(xyz[3 * p + 0], hp.bmin[0], hp.bmax[0], hp.cell[lvl][0]);
        const AxisCell ay = axis_cell(xyz[3 * p + 1], hp.bmin[1], hp.bmax[1], hp.cell[lvl][1]);
        const AxisCell az = axis_cell(xyz[3 * p + 2], hp.bmin[2], hp.bmax[2], hp.cell[lvl][2]);
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const uint32_t h = spatial_hash3((uint32_t)ax.base + ((c >> 2) & 1), (uint32_t)ay.base + ((c >> 1) & 1),
                                             (uint32_t)az.base + (c & 1), hp.mask);
            const float2 e = tab[h];
            lo = fminf(lo, fminf(e.x, e.y));
            hi = fmaxf(hi, fmaxf(e.x, e.y));
        }
    }
    block_minmax_commit(lo, hi, mm + 2 * lvl);
}

__global__ void quant_calibrate_kernel(QuantizerSet set, int n, const uint32_t* __restrict__ mm) {
    const int i = threadIdx.x;
    if (i >= n) return;
    const nerf_quantizer& d = set.q[i];
    const float bmin = ord2f(mm[2 * i]), bmax = ord2f(mm[2 * i + 1]);
    const float rmin = fminf(*d.running_min, bmin), rmax = fmaxf(*d.running_max, bmax);
    *d.running_min = rmin;
    *d.running_max = rmax;
    if (d.v_max == nullptr) {
        *d.range_scale = 2.0f * fmaxf(fabsf(rmin), fabsf(rmax));
    } else {
        *d.range_scale = rmax - rmin;
        *d.v_max = rmax;
    }
}

__global__ void __launch_bounds__(256) fake_quant_kernel(const float* __restrict__ x, int64_t n,
                                                         const QuantRec* __restrict__ rec, float* __restrict__ y) {
    const QuantRec q = *rec;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        y[i] = fake_quant(x[i], q);
}

// A-CAQ bit-width controller of train() (run_nerf.py:1207-1250), every 10th iteration, on the
// device (the reference reads img_loss and every soft_bits with .item()): the same double-precision
// algebra on the float32 values, then the float32 in-place add and clamp of soft_bits.
__global__ void acaq_update_kernel(QuantizerSet set, int n, const float* __restrict__ img_loss,
                                   double* __restrict__ best, int has_target, double target_metric,
                                   double bit_penalty, double* __restrict__ report) {
    if (threadIdx.x != 0) return;
    const double cur = (double)*img_loss;
    double target;
    if (has_target) {
        target = target_metric;
    } else {
        const double b = isnan(*best) ? cur : fmin(*best, cur);     // train.best_loss (:1218-1221)
        *best = b;
        target = b * 1.2;
    }
    const double ratio = cur / target;
    for (int i = 0; i < n; ++i) {
        float* sb = const_cast<float*>(set.q[i].soft_bits);
        const double bits = (double)*sb;
        double delta = ratio < 0.95 ? -0.3 : (ratio < 1.05 ? -0.1 : 0.2);
        delta -= bit_penalty * bits / 8.0;
        delta *= 1.0 + ((double)i - (double)n / 2.0) * 0.02;       // layer_factor
        const float nb = *sb + (float)delta;                         // soft_bits.data += bit_delta (fp32)
        *sb = fminf(fmaxf(nb, set.q[i].min_bits), set.q[i].max_bits);
    }
    if (report) {
        report[0] = target;
        report[1] = ratio;
    }
}

// ---- int-packed tables ----------------------------------------------------------------------
// Level l occupies bytes [l * T * 8, (l+1) * T * 8) of the packed buffer (the fp32 table's size, so
// the layout never depends on the bit widths and needs no host round trip); its entries are stored
// densely from the region start with the code width of the level's record: B <= 4 -> 1 byte per
// entry (two 4-bit codes), B <= 8 -> 2 bytes, B <= 16 -> 4 bytes, else the fp32 deq pair (8 bytes).
__device__ __forceinline__ int code_width(const QuantRec& q) {
    const int b = (int)q.bits;
    return b <= 4 ? 4 : b <= 8 ? 8 : b <= 16 ? 16 : 32;
}

struct PackTables {
    const float* tables[NERF_MAX_LEVELS];
};

// dirty[l] = force || record l differs from the one the level was last packed with; prev := rec.
__global__ void pack_dirty_kernel(const QuantRec* __restrict__ rec, QuantRec* __restrict__ prev, int n, int force,
                                  int* __restrict__ dirty) {
    const int l = threadIdx.x;
    if (l >= n) return;
    const float* a = reinterpret_cast<const float*>(rec + l);
    float* b = reinterpret_cast<float*>(prev + l);
    bool same = !force;
#pragma unroll
    for (int k = 0; k < 8; ++k) same = same && (__float_as_uint(a[k]) == __float_as_uint(b[k]));
    dirty[l] = same ? 0 : 1;
#pragma unroll
    for (int k = 0; k < 8; ++k) b[k] = a[k];
}

// One thread per table entry (2 features). Codes are stored unsigned: q - qmin (qmin = 0 for the
// asymmetric hash quantizers; symmetric codes are offset so they stay non-negative).
__global__ void __launch_bounds__(256) pack_tables_kernel(PackTables pt, int64_t T, const QuantRec* __restrict__ qrec,
                                                          const int* __restrict__ dirty, uint8_t* __restrict__ packed) {
    const int lvl = blockIdx.y;
    if (!dirty[lvl]) return;
    const QuantRec q = qrec[lvl];
    const int bits = code_width(q);
    uint8_t* base = packed + (size_t)lvl * (size_t)T * 8;
    const float2* tab = reinterpret_cast<const float2*>(pt.tables[lvl]);
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < T; r += (int64_t)gridDim.x * blockDim.x) {
        const float2 e = tab[r];
        if (bits == 32) {
            reinterpret_cast<float2*>(base)[r] = make_float2((quant_code(e.x, q) - q.zp) * q.scale,
                                                             (quant_code(e.y, q) - q.zp) * q.scale);
            continue;
        }
        const uint32_t c0 = (uint32_t)(quant_code(e.x, q) - q.qmin), c1 = (uint32_t)(quant_code(e.y, q) - q.qmin);
        if (bits == 4) base[r] = (uint8_t)(c0 | (c1 << 4));
        else if (bits == 8) reinterpret_cast<uint16_t*>(base)[r] = (uint16_t)(c0 | (c1 << 8));
        else reinterpret_cast<uint32_t*>(base)[r] = c0 | (c1 << 16);
    }
}

template <int BITS>
__device__ __forceinline__ void load_codes(const uint8_t* base, uint32_t h, const QuantRec& q, float& f0, float& f1) {
    uint32_t c0, c1;
    if constexpr (BITS == 4) {
        const uint32_t v = base[h];
        c0 = v & 15u; c1 = v >> 4;
    } else if constexpr (BITS == 8) {
        const uint32_t v = reinterpret_cast<const uint16_t*>(base)[h];
        c0 = v & 255u; c1 = v >> 8;
    } else {
        const uint32_t v = reinterpret_cast<const uint32_t*>(base)[h];
        c0 = v & 65535u; c1 = v >> 16;
    }
    // q = code + qmin is an exact float integer (|q| < 2^17); deq = (q - zp) * scale as :186
    f0 = (((float)c0 + q.qmin) - q.zp) * q.scale;
    f1 = (((float)c1 + q.qmin) - q.zp) * q.scale;
}

// Lane-pair packed gather (the fp32 forward's structure, hashgrid.hip hash_encode_fwd_pair_kernel):
// lanes 2m and 2m+1 share point m and gather the x = 0 / x = 1 corners of its voxel, so corners
// (x, y, z) and (x+1, y, z), which hash to h and h ^ (x ^ (x+1)), leave in one instruction's line;
// level-major grid rows (one level's packed table hot in each XCD's L2), the coarse levels whose
// (res + 1)^3 vertices fit the table grouped into row 0, and the fast division of the voxel math.
// The dequantized corners blend exactly as the fp32 forward (bit-identical to nerf_hash_encode_fwd_q with the same eval-mode records).
template <int BITS>
__device__ __forceinline__ float2 packed_entry(const uint8_t* base, uint32_t h, const QuantRec& q) {
    if constexpr (BITS == 32) {
        return reinterpret_cast<const float2*>(base)[h];
    } else {
        float f0, f1;
        load_codes<BITS>(base, h, q, f0, f1);
        return make_float2(f0, f1);
    }
}

template <int BITS, bool FAST>
__device__ __forceinline__ void packed_gather(float x, float y, float z, const HashParams& hp, int lvl, int xb,
                                              const uint8_t* base, const QuantRec& q, FwdLvl& s) {
    AxisCell ax, ay, az;
    fwd_axes<FAST>(x, y, z, hp, lvl, xb, ax, ay, az);
    s.wx = ax.w; s.wy = ay.w; s.wz = az.w;
    s.inside = ax.inside && ay.inside && az.inside;
    const uint32_t bx = (uint32_t)ax.base + (uint32_t)xb, by = (uint32_t)ay.base, bz = (uint32_t)az.base;
#pragma unroll
    for (int c = 0; c < 4; ++c)
        s.e[c] = packed_entry<BITS>(base, spatial_hash3(bx, by + ((c >> 1) & 1), bz + (c & 1), hp.mask), q);
}

__device__ __forceinline__ void packed_level(float x, float y, float z, const HashParams& hp, int lvl, int xb,
                                             bool fast, int64_t T, const uint8_t* __restrict__ packed,
                                             const QuantRec* __restrict__ qrec, FwdLvl& s) {
    const QuantRec q = qrec[lvl];
    const uint8_t* base = packed + (size_t)lvl * (size_t)T * 8;
    const int w = code_width(q);   // uniform: one level per call
#define NERF_PK(B)                                                          \
    if (fast) packed_gather<B, true>(x, y, z, hp, lvl, xb, base, q, s);    \
    else packed_gather<B, false>(x, y, z, hp, lvl, xb, base, q, s);
    if (w == 4) { NERF_PK(4) } else if (w == 8) { NERF_PK(8) } else if (w == 16) { NERF_PK(16) } else { NERF_PK(32) }
#undef NERF_PK
}


__global__ void __launch_bounds__(256) hash_encode_fwd_packed_pair_kernel(
    const float* __restrict__ xyz, int64_t n, HashParams hp, int group, int64_t T, const uint8_t* __restrict__ packed,
    const QuantRec* __restrict__ qrec, float* __restrict__ feat, int64_t sp, int64_t sl, uint8_t* __restrict__ keep) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int row = blockIdx.y;
    const int64_t p = t >> 1;
    const int xb = (int)(t & 1);
    const bool valid = p < n;
    const int64_t pc = valid ? p : n - 1;             // invalid lanes mirror a valid point (no stores)
    const float x = xyz[3 * pc + 0], y = xyz[3 * pc + 1], z = xyz[3 * pc + 2];
    const bool fast = hp.fastdiv && __ballot(!fastdiv_point_ok(x, y, z)) == 0ull;   // wave-uniform
    if (group > 0 && row == 0) {
        for (int l0 = 0; l0 < group; l0 += kFwdGroupRound) {
            FwdLvl s[kFwdGroupRound];
#pragma unroll
            for (int g = 0; g < kFwdGroupRound; ++g)
                if (l0 + g < group) packed_level(x, y, z, hp, l0 + g, xb, fast, T, packed, qrec, s[g]);
#pragma unroll
            for (int g = 0; g < kFwdGroupRound; ++g)
                if (l0 + g < group) fwd_finish<false>(s[g], l0 + g, xb, valid, p, feat, sp, sl, keep, nullptr);
        }
        return;
    }
    const int lvl = group > 0 ? group + row - 1 : row;
    FwdLvl s;
    packed_level(x, y, z, hp, lvl, xb, fast, T, packed, qrec, s);
    fwd_finish<false>(s, lvl, xb, valid, p, feat, sp, sl, keep, nullptr);
}

static int fill_set(QuantizerSet& s, const nerf_quantizer* qs, int n, bool need_stats) {
    NERF_REQUIRE(qs && n >= 1 && n <= NERF_MAX_QUANTIZERS, "quant: n = %d quantizers (1..%d)", n, NERF_MAX_QUANTIZERS);
    for (int i = 0; i < n; ++i) {
        NERF_REQUIRE(qs[i].soft_bits && qs[i].range_scale, "quant: quantizer %d has null parameters", i);
        NERF_REQUIRE(!need_stats || (qs[i].running_min && qs[i].running_max), "quant: quantizer %d has null buffers", i);
        NERF_REQUIRE(qs[i].min_bits >= 1.f && qs[i].max_bits <= 32.f && qs[i].min_bits <= qs[i].max_bits,
                     "quant: quantizer %d bit range [%g, %g]", i, qs[i].min_bits, qs[i].max_bits);
        s.q[i] = qs[i];
    }
    return NERF_OK;
}

static int hash_params(HashParams& hp, const float* bmin, const float* bmax, const float* res, int n_levels,
                       int log2_T, const float* const* tables) {
    NERF_REQUIRE(n_levels >= 1 && n_levels <= NERF_MAX_LEVELS, "quant: n_levels %d", n_levels);
    NERF_REQUIRE(log2_T >= 1 && log2_T <= 30, "quant: log2_T %d", log2_T);
    NERF_REQUIRE(bmin && bmax && res, "quant: null bbox / resolutions");
    for (int l = 0; l < n_levels; ++l) hp.tables[l] = tables ? tables[l] : nullptr;
    for (int a = 0; a < 3; ++a) { hp.bmin[a] = bmin[a]; hp.bmax[a] = bmax[a]; }
    hp.fastdiv = fill_cells(hp.cell, hp.rcell, bmin, bmax, res, n_levels) ? 1u : 0u;
    hp.mask = (uint32_t)((1u << log2_T) - 1u);
    return NERF_OK;
}

}  // namespace nerf

using namespace nerf;

extern "C" int nerf_quant_params(const nerf_quantizer* qs, int n, int training, float* d_rec, void* stream) {
    QuantizerSet s;
    int rc = fill_set(s, qs, n, false);
    if (rc) return rc;
    NERF_REQUIRE(d_rec, "quant_params: null output");
    hipLaunchKernelGGL(quant_params_kernel, dim3(1), dim3(64), 0, as_stream(stream), s, n, training ? 1 : 0,
                       reinterpret_cast<QuantRec*>(d_rec));
    NERF_CHECK_LAUNCH("quant_params");
    return NERF_OK;
}

extern "C" int nerf_quant_minmax_reset(uint32_t* d_minmax, int n, void* stream) {
    NERF_REQUIRE(d_minmax && n >= 1, "quant_minmax_reset: bad args");
    hipLaunchKernelGGL(minmax_reset_kernel, dim3(blocks_for(n, 64)), dim3(64), 0, as_stream(stream), d_minmax, n);
    NERF_CHECK_LAUNCH("quant_minmax_reset");
    return NERF_OK;
}

extern "C" int nerf_quant_minmax(const float* d_x, int64_t count, uint32_t* d_minmax, void* stream) {
    NERF_REQUIRE(d_minmax && count >= 0 && (d_x || count == 0), "quant_minmax: bad args");
    if (count == 0) return NERF_OK;
    const unsigned blocks = (unsigned)std::min<int64_t>(blocks_for(count, 256), 1024);
    hipLaunchKernelGGL(minmax_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), d_x, count, d_minmax);
    NERF_CHECK_LAUNCH("quant_minmax");
    return NERF_OK;
}

extern "C" int nerf_hash_gather_minmax(const float* d_xyz, int64_t n_points, const float* bbox_min3,
                                       const float* bbox_max3, const float* level_res, int n_levels, int log2_T,
                                       const float* const* d_tables, uint32_t* d_minmax, void* stream) {
    NERF_REQUIRE(d_tables && d_minmax && n_points >= 0 && (n_points == 0 || d_xyz), "hash_gather_minmax: bad args");
    HashParams hp{};
    int rc = hash_params(hp, bbox_min3, bbox_max3, level_res, n_levels, log2_T, d_tables);
    if (rc) return rc;
    for (int l = 0; l < n_levels; ++l) NERF_REQUIRE(d_tables[l], "hash_gather_minmax: table %d is null", l);
    if (n_points == 0) return NERF_OK;
    const unsigned bx = (unsigned)std::min<int64_t>(blocks_for(n_points, 256), 512);
    hipLaunchKernelGGL(hash_gather_minmax_kernel, dim3(bx, n_levels), dim3(256), 0, as_stream(stream), d_xyz,
                       n_points, hp, d_minmax);
    NERF_CHECK_LAUNCH("hash_gather_minmax");
    return NERF_OK;
}

extern "C" int nerf_quant_calibrate(const nerf_quantizer* qs, int n, const uint32_t* d_minmax, void* stream) {
    QuantizerSet s;
    int rc = fill_set(s, qs, n, true);
    if (rc) return rc;
    NERF_REQUIRE(d_minmax, "quant_calibrate: null statistics");
    hipLaunchKernelGGL(quant_calibrate_kernel, dim3(1), dim3(64), 0, as_stream(stream), s, n, d_minmax);
    NERF_CHECK_LAUNCH("quant_calibrate");
    return NERF_OK;
}

extern "C" int nerf_fake_quant(const float* d_x, int64_t count, const float* d_rec, float* d_y, void* stream) {
    NERF_REQUIRE(count >= 0 && d_rec && ((d_x && d_y) || count == 0), "fake_quant: bad args");
    if (count == 0) return NERF_OK;
    const unsigned blocks = (unsigned)std::min<int64_t>(blocks_for(count, 256), 4096);
    hipLaunchKernelGGL(fake_quant_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), d_x, count,
                       reinterpret_cast<const QuantRec*>(d_rec), d_y);
    NERF_CHECK_LAUNCH("fake_quant");
    return NERF_OK;
}

extern "C" size_t nerf_quant_packed_bytes(int n_levels, int log2_T) {
    if (n_levels < 1 || n_levels > NERF_MAX_LEVELS || log2_T < 1 || log2_T > 30) return 0;
    return (size_t)n_levels * ((size_t)1 << log2_T) * 8;
}

extern "C" int nerf_quant_pack_tables(const float* const* d_tables, int n_levels, int log2_T, const float* d_qrec,
                                      float* d_prev_rec, int force, int* d_dirty, void* d_packed, void* stream) {
    NERF_REQUIRE(d_tables && d_qrec && d_prev_rec && d_dirty && d_packed && n_levels >= 1 &&
                 n_levels <= NERF_MAX_LEVELS && log2_T >= 1 && log2_T <= 30, "quant_pack_tables: bad args");
    PackTables pt{};
    for (int l = 0; l < n_levels; ++l) {
        NERF_REQUIRE(d_tables[l], "quant_pack_tables: table %d is null", l);
        pt.tables[l] = d_tables[l];
    }
    hipLaunchKernelGGL(pack_dirty_kernel, dim3(1), dim3(64), 0, as_stream(stream),
                       reinterpret_cast<const QuantRec*>(d_qrec), reinterpret_cast<QuantRec*>(d_prev_rec), n_levels,
                       force ? 1 : 0, d_dirty);
    NERF_CHECK_LAUNCH("quant_pack_tables(dirty)");
    const int64_t T = int64_t(1) << log2_T;
    const unsigned bx = (unsigned)std::min<int64_t>(blocks_for(T, 256), 512);
    hipLaunchKernelGGL(pack_tables_kernel, dim3(bx, n_levels), dim3(256), 0, as_stream(stream), pt, T,
                       reinterpret_cast<const QuantRec*>(d_qrec), d_dirty, reinterpret_cast<uint8_t*>(d_packed));
    NERF_CHECK_LAUNCH("quant_pack_tables");
    return NERF_OK;
}

extern "C" int nerf_hash_encode_fwd_packed(const float* d_xyz, int64_t n_points, const float* bbox_min3,
                                           const float* bbox_max3, const float* level_res, int n_levels, int log2_T,
                                           const void* d_packed, const float* d_qrec, float* d_feat,
                                           int64_t feat_stride_point, int64_t feat_stride_level, uint8_t* d_keep,
                                           void* stream) {
    NERF_REQUIRE(n_points >= 0 && d_packed && d_qrec && (n_points == 0 || (d_xyz && d_feat)),
                 "hash_encode_fwd_packed: bad args");
    HashParams hp{};
    int rc = hash_params(hp, bbox_min3, bbox_max3, level_res, n_levels, log2_T, nullptr);
    if (rc) return rc;
    if (n_points == 0) return NERF_OK;
    int group = 0;   // coarse levels whose (res + 1)^3 vertices fit the table share grid row 0
    while (group < std::min(n_levels, kFwdGroupMax)) {
        const double v = (double)level_res[group] + 1.0;
        if (v * v * v > (double)(1u << log2_T)) break;
        ++group;
    }
    if (group < 2) group = 0;
    const int rows = group > 0 ? n_levels - group + 1 : n_levels;
    hipLaunchKernelGGL(hash_encode_fwd_packed_pair_kernel, dim3(blocks_for(2 * n_points, 256), rows), dim3(256), 0,
                       as_stream(stream), d_xyz, n_points, hp, group, int64_t(1) << log2_T,
                       reinterpret_cast<const uint8_t*>(d_packed), reinterpret_cast<const QuantRec*>(d_qrec), d_feat,
                       feat_stride_point, feat_stride_level, d_keep);
    NERF_CHECK_LAUNCH("hash_encode_fwd_packed");
    return NERF_OK;
}

extern "C" int nerf_acaq_update(const nerf_quantizer* qs, int n, const float* d_img_loss, double* d_best_loss,
                                int has_target, double target_metric, double bit_penalty, double* d_report,
                                void* stream) {
    QuantizerSet set;
    int rc = fill_set(set, qs, n, false);
    if (rc) return rc;
    NERF_REQUIRE(d_img_loss && (has_target || d_best_loss), "acaq_update: null loss / best-loss pointer");
    hipLaunchKernelGGL(acaq_update_kernel, dim3(1), dim3(64), 0, as_stream(stream), set, n, d_img_loss, d_best_loss,
                       has_target ? 1 : 0, target_metric, bit_penalty, d_report);
    NERF_CHECK_LAUNCH("acaq_update");
    return NERF_OK;
}
