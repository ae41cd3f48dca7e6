// Multi-resolution hash grid: forward gather + trilinear, backward scatter-add.
//
// Restates, per (point, level), the reference's eager-op chain
//   get_voxel_vertices  PocketNeRF/utils.py:95-117  (keep mask, clamp, cell, floor, corners)
//   hash                PocketNeRF/utils.py:13-24   (x*1 ^ y*2654435761 ^ z*805459861, masked)
//   nn.Embedding gather PocketNeRF/hash_encoding.py:94
//   trilinear_interp    PocketNeRF/hash_encoding.py:56-80 (x, then y, then z blends)
// in one thread, with the reference's op order and no contraction (-ffp-contract=off), so indices,
// keep mask and features are bit-identical to the fp32 reference.
//
// Launch geometry: rows of blocks in one grid dimension: row 0 runs the G coarse levels of its points
// (hash_encode_fwd_pair_kernel), every other row one level. Blocks are dispatched in order, so at
// any moment the whole chip works on one or two levels and each XCD's 4 MiB L2 holds the level's
// table lines that the current point range touches (tables are 4 MiB per level at log2_T = 19).
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "hash_common.h"

namespace nerf {

struct HashGradParams {
    float* dtables[NERF_MAX_LEVELS];
    float cell[NERF_MAX_LEVELS][3];
    float rcell[NERF_MAX_LEVELS][3];   // RN(1 / cell): div_rn_recip (hash_common.h)
    float bmin[3];
    float bmax[3];
    uint32_t mask;
    uint32_t fastdiv;     // fill_cells accepted the box and cells for div_rn<true>
    // binned path (MODE 3): per (level, 256-point chunk) a region of kChunkCap entries sorted by
    // owner slice, plus the slice offsets of each region.
    uint16_t* bin_h;      // entry row within its owner slice
    float2* bin_g;        // entry (d feat0, d feat1)
    uint32_t* bin_seg;    // [L][n_owner][nchunks]: segment start | count << 16 within the chunk region
    int nchunks;          // chunks the owner pass walks
    int chunk_base;       // bin pass: chunk index of this launch's first kChunkPts points
    int chunk_stride;     // chunk capacity of the workspace (the layout stride)
    int slice_log2;       // owner slice = 2^slice_log2 rows (LDS: 16 B per row, 32 B deterministic)
    int owner_log2;       // owners per level = 2^owner_log2
    float* chunk_max;     // deterministic mode: [L][chunk_stride] max |entry| of each chunk, else null
    int overwrite;        // owner pass: store every row (the gradients are logically zero), no loads
    int level0;           // owner pass: first level of the launch's level range (grid rows = its levels)
    // owner pass, optional: the optimizer step of the tables fused into the flush (overwrite mode):
    // each row's gradient, once stored, updates the row's parameters and moments (radam_elem)
    float* st_p[NERF_MAX_LEVELS];
    float* st_m[NERF_MAX_LEVELS];
    float* st_v[NERF_MAX_LEVELS];
    nerf_radam_segment st;   // scalars (pointers unused)
    const float* st_coef;    // optional device (decay_coef, step_coef, mode, -): graph replays
    int st_on;
};

// The flush of an owner block with the fused table step: rows [0, S) of the slice at `row0` of level lvl;
// g(i) gives row i's gradient, which is stored to dt[i] (overwrite mode) and then updates the row's
// parameters and moments. A batch's parameter / moment loads are issued before its first gradient, so
// they are in flight while the gradients are formed and stored.
// A row that never received a gradient (its moments are +0) and gets none now: without weight decay
// RAdam leaves its parameter and moments bit for bit as they are (+0 * beta + (+0 * g) * g = +0, and
// p + (c * +0) / (sqrt(+0) + eps) = p), so only its gradient row is stored. Most rows of the coarse
// levels' 2^19-row tables are never hashed to: the table step skips their 24 B of writes.
// With eps == 0 the adaptive step of such a row is (c * 0) / (sqrt(0) + 0) = NaN in the reference
// (radam.py:85), so mode 2 with eps == 0 takes the full update.
__device__ __forceinline__ bool radam_idle(const nerf_radam_segment& s, float2 g, float2 m, float2 v) {
    return s.decay_coef == 0.f && (s.mode != 2 || s.eps > 0.f) &&
           (__float_as_uint(g.x) | __float_as_uint(g.y) | __float_as_uint(m.x) |
                                   __float_as_uint(m.y) | __float_as_uint(v.x) | __float_as_uint(v.y)) == 0u;
}

template <int THREADS, int ROWS, typename G>
__device__ __forceinline__ void owner_table_step(const HashGradParams& hp, int lvl, size_t row0, int S, float2* dt,
                                                 G g) {
    nerf_radam_segment s = hp.st;
    if (hp.st_coef) {
        s.decay_coef = hp.st_coef[0];
        s.step_coef = hp.st_coef[1];
        s.mode = (int)hp.st_coef[2];
    }
    float2* P = reinterpret_cast<float2*>(hp.st_p[lvl]) + row0;
    float2* M = reinterpret_cast<float2*>(hp.st_m[lvl]) + row0;
    float2* V = reinterpret_cast<float2*>(hp.st_v[lvl]) + row0;
    for (int b = threadIdx.x; b < S; b += ROWS * THREADS) {
        float2 p[ROWS], m[ROWS], v[ROWS];
#pragma unroll
        for (int k = 0; k < ROWS; ++k) {
            const int i = b + k * THREADS;
            if (i < S) { p[k] = P[i]; m[k] = M[i]; v[k] = V[i]; }
        }
#pragma unroll
        for (int k = 0; k < ROWS; ++k) {
            const int i = b + k * THREADS;
            if (i >= S) continue;
            const float2 gi = g(i);
            dt[i] = gi;
            if (radam_idle(s, gi, m[k], v[k])) continue;
            radam_elem(s, p[k].x, gi.x, m[k].x, v[k].x);
            radam_elem(s, p[k].y, gi.y, m[k].y, v[k].y);
            M[i] = m[k];
            V[i] = v[k];
            if (s.mode != 0) P[i] = p[k];
        }
    }
}

// Grouped coarse levels: blockIdx.y == 0 runs levels [0, group) of its points, two levels' gathers
// in flight at a time; the other rows run one level each (level-major: one table hot in each XCD's
// L2). A coarse level alone is latency-bound (few, hot table lines; a single round trip per wave per
// level): grouping the 6 coarse levels of the lego config took the forward from 121 to 107 us per
// launch (same box; 3 or 6 levels in flight: 114 / 154 us, the registers cost occupancy).

#ifdef NERF_FWD_PROF   // diagnostic build only (tools/fwd_prof.py): per-block start / end (100 MHz real
                       // time) and the XCC / hardware ids of the block's first wave
constexpr int kFwdProfBlocks = 65536;
__device__ unsigned long long fwd_prof[kFwdProfBlocks * 3];
#endif

// Points per thread on the single-level rows (the grouped row keeps one: its levels are its
// memory-level parallelism). Two points (p and p + 128 of the block's 256) put 8 gathers in flight
// per thread instead of 4: per-block timelines (tools/fwd_prof.py, profiles/r05p_fwd_prof_pts*.json)
// show each level row running as ~1.5 waves of latency-bound blocks; 92.6 -> 88.2 us per launch in
// the bench, bit-identical (profiles/r05p_ab_fwd_row_pts2.jsonl)
#ifndef NERF_FWD_ROW_PTS
#define NERF_FWD_ROW_PTS 2
#endif
constexpr int kFwdRowPts = NERF_FWD_ROW_PTS;

// Grid: one dimension, rows in order — blocks [0, gx0) the grouped row (128 points each), then gx1
// blocks (128 kFwdRowPts points each) per single-level row (group == 0: gx1 per level from block 0).
template <bool QUANT>
__global__ void __launch_bounds__(256) hash_encode_fwd_pair_kernel(
    const float* __restrict__ xyz, int64_t n, HashParams hp, int group, unsigned gx0, unsigned gx1,
    float* __restrict__ feat, int64_t sp, int64_t sl, uint8_t* __restrict__ keep,
    const QuantRec* __restrict__ qrec) {
#ifdef NERF_FWD_PROF
    const size_t prof_blk = blockIdx.x;
    if (threadIdx.x == 0 && prof_blk < kFwdProfBlocks) {
        fwd_prof[prof_blk * 3 + 0] = __builtin_amdgcn_s_memrealtime();
        // XCC_ID (hwreg 20, 4 bits) << 32 | HW_ID (hwreg 4: wave, SIMD, CU, SE ids)
        const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (3 << 11));
        const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));
        fwd_prof[prof_blk * 3 + 2] = ((unsigned long long)xcc << 32) | hw;
    }
    struct Done {
        size_t b;
        __device__ ~Done() {
            __syncthreads();
            if (threadIdx.x == 0 && b < kFwdProfBlocks) fwd_prof[b * 3 + 1] = __builtin_amdgcn_s_memrealtime();
        }
    } done{prof_blk};
#endif
    const unsigned b = blockIdx.x;
    const int xb = (int)(threadIdx.x & 1);
    if (group > 0 && b < gx0) {
        const int64_t p = ((int64_t)b * blockDim.x + threadIdx.x) >> 1;
        const bool valid = p < n;
        const int64_t pc = valid ? p : n - 1;         // invalid lanes mirror a valid point (no stores)
        const float x = xyz[3 * pc + 0], y = xyz[3 * pc + 1], z = xyz[3 * pc + 2];
        const bool fast = hp.fastdiv && __ballot(!fastdiv_point_ok(x, y, z)) == 0ull;   // wave-uniform
        for (int l0 = 0; l0 < group; l0 += kFwdGroupRound) {
            FwdLvl s[kFwdGroupRound];
#pragma unroll
            for (int g = 0; g < kFwdGroupRound; ++g) {
                if (l0 + g < group) {
                    if (fast) fwd_gather<true>(x, y, z, hp, l0 + g, xb, s[g]);
                    else fwd_gather<false>(x, y, z, hp, l0 + g, xb, s[g]);
                }
            }
#pragma unroll
            for (int g = 0; g < kFwdGroupRound; ++g)
                if (l0 + g < group) fwd_finish<QUANT>(s[g], l0 + g, xb, valid, pc, feat, sp, sl, keep, qrec);
        }
        return;
    }
    const unsigned r = group > 0 ? b - gx0 : b;
    const int lvl = (group > 0 ? group : 0) + (int)(r / gx1);
    const int64_t p0 = (int64_t)(r % gx1) * (128 * kFwdRowPts) + (threadIdx.x >> 1);
    int64_t pc[kFwdRowPts];
    bool valid[kFwdRowPts];
    float x[kFwdRowPts], y[kFwdRowPts], z[kFwdRowPts];
    bool ok = true;
#pragma unroll
    for (int k = 0; k < kFwdRowPts; ++k) {
        const int64_t p = p0 + 128 * k;
        valid[k] = p < n;
        pc[k] = valid[k] ? p : n - 1;
        x[k] = xyz[3 * pc[k] + 0]; y[k] = xyz[3 * pc[k] + 1]; z[k] = xyz[3 * pc[k] + 2];
        ok = ok && fastdiv_point_ok(x[k], y[k], z[k]);
    }
    const bool fast = hp.fastdiv && __ballot(!ok) == 0ull;
    FwdLvl s[kFwdRowPts];
#pragma unroll
    for (int k = 0; k < kFwdRowPts; ++k) {
        if (fast) fwd_gather<true>(x[k], y[k], z[k], hp, lvl, xb, s[k]);
        else fwd_gather<false>(x[k], y[k], z[k], hp, lvl, xb, s[k]);
    }
#pragma unroll
    for (int k = 0; k < kFwdRowPts; ++k) fwd_finish<QUANT>(s[k], lvl, xb, valid[k], pc[k], feat, sp, sl, keep, qrec);
}


// Backward: dL/de_c = ((g*(1-wz or wz))*(1-wy or wy))*(1-wx or wx), the order autograd applies the
// three blend steps in reverse; scatter-added with fp32 atomics (no-return global_atomic_add_f32).
// Consecutive threads are consecutive samples of one ray: at coarse levels they usually share the
// voxel, so a thread first merges runs of equal voxels inside its wave (see below).
__device__ __forceinline__ void atomic_add_f32(float* p, float v) {
    __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// MODE 1 (no workspace): the per-item contributions are staged in LDS and re-issued as float
// atomics so that one wave instruction covers 4 items x 16 dwords, ordered (item, corner pair
// (j,k), i, feature). Corners (x, y, z) and (x+1, y, z) hash to h and h ^ (x ^ (x+1)) (x only
// touches the low 11 bits), so the 4 dwords of a pair usually share one 64-B segment and leave as
// ONE atomic request.
constexpr uint32_t kSkip = 0xFFFFFFFFu;

// MODE 3 (binned, "owner computes"): float atomics execute at the memory side at one chip-wide
// rate of 64-B requests (MI355X_MICROARCH.md, Global float atomics), and the hash scatters every
// corner pair to its own line, so the atomic path is request-bound (plus same-line serialisation
// at the coarse levels, where every ray crosses the same few thousand voxels). The binned path
// replaces the memory-side atomics: this kernel writes each (row, d feat) entry into a per-chunk
// region sorted by owner slice (plain stores), and hash_bwd_owner_kernel sums each slice in LDS.
constexpr int kChunkPts = NERF_HASH_CHUNK_POINTS;   // points per chunk = threads per bin block
constexpr int kChunkCap = kChunkPts * 8;            // entries per chunk (8 corners per point)
constexpr int kChunkCapLog2 = kChunkPts == 256 ? 11 : kChunkPts == 512 ? 12 : 13;
static_assert(kChunkPts == 256 || kChunkPts == 512 || kChunkPts == 1024, "chunk of 256, 512 or 1024 points");
#ifndef NERF_OWNER_ACC32
#define NERF_OWNER_ACC32 0
#endif
#ifndef NERF_OWNER_SLICE_LOG2
#define NERF_OWNER_SLICE_LOG2 13
#endif
constexpr bool kOwnerAcc32 = NERF_OWNER_ACC32 != 0;   // fp32 LDS accumulators (ds_add_f32) instead of fp64
constexpr int kSliceLog2 = NERF_OWNER_SLICE_LOG2;     // owner slice: 2^13 rows x 16 B (fp64 pair) = 128 KiB of LDS
#ifndef NERF_OWNER_THREADS
#define NERF_OWNER_THREADS 1024
#endif
constexpr int kOwnerThreadsDefault = NERF_OWNER_THREADS;
#ifndef NERF_BIN_NT_STORES
#define NERF_BIN_NT_STORES 1
#endif



constexpr int kSliceLog2Det = 12;         // deterministic: 2^12 rows x 32 B (two int64 words per feature)
constexpr int kMaxOwnersLog2 = 7;
constexpr int kMaxOwners = 1 << kMaxOwnersLog2;

// Bin one chunk: count the block's entries per owner slice (LDS atomics), scan, place every entry
// at its slot of an LDS image of the chunk's region, then write the image out with 16-B coalesced
// stores (scattered per-lane stores were TA-bound: 64 lines per instruction). Every (level, chunk)
// in [0, n_chunks) gets its n_owner segment words, empty ones included. NE entries per thread
// (8 corners of a point; 1 TV vertex), at most kChunkCap per chunk. PAIRED: entries (2p, 2p+1) usually
// share an owner slice (a point's corners (x, y, z) and (x+1, y, z) hash to h and h ^ (x ^ (x+1)),
// which differ below bit 13 whenever x < 8191): such a pair takes its two slots with ONE counting
// atomic — the contended LDS counters are a quarter of the bin pass's time.
// The LDS of bin_chunk: one object per kernel whatever instantiations of bin_chunk it inlines (the
// hash bins and the TV bins in one launch, hash_encode_bwd_tv_pair_kernel: 42 KB, not 84 KB and a
// third of the occupancy).
struct BinLds {
    uint32_t cnt[kMaxOwners];
    uint32_t start[kMaxOwners + 1];
    __attribute__((aligned(16))) uint16_t eh[kChunkCap];
    __attribute__((aligned(16))) float2 eg[kChunkCap];
};
__device__ __forceinline__ BinLds& bin_lds() {
    __shared__ BinLds s;
    return s;
}

template <int THREADS, int NE, bool PAIRED = false>
__device__ __forceinline__ void bin_chunk(const HashGradParams& hp, int lvl, int chunk, const uint32_t (&hh)[NE],
                                          const float (&vx)[NE], const float (&vy)[NE], const bool (&on)[NE]) {
    constexpr int CAP = THREADS * NE;
    static_assert(CAP <= kChunkCap, "chunk region");
    BinLds& lds = bin_lds();
    uint32_t* const s_cnt = lds.cnt;
    uint32_t* const s_start = lds.start;
    uint16_t* const s_eh = lds.eh;
    float2* const s_eg = lds.eg;
    const int lane = threadIdx.x & 63;
    const int n_own = 1 << hp.owner_log2;
    // (zeroing the counters at the block's start instead, so that a wave counts as soon as its own
    // point math is done, measured slower: bins 207 -> 212 us per step, profiles/r05d_ab_bench.jsonl)
    if (threadIdx.x < n_own) s_cnt[threadIdx.x] = 0;
    __syncthreads();
    uint32_t pos[NE];
    if constexpr (PAIRED) {
        static_assert(NE % 2 == 0, "pairs");
#pragma unroll
        for (int c = 0; c < NE; c += 2) {
            const uint32_t o0 = hh[c] >> hp.slice_log2, o1 = hh[c + 1] >> hp.slice_log2;
            const bool same = o0 == o1;
            const uint32_t n0 = (on[c] ? 1u : 0u) + (on[c + 1] && same ? 1u : 0u);
            const uint32_t b0 = n0 ? atomicAdd(&s_cnt[on[c] ? o0 : o1], n0) : 0u;
            const uint32_t b1 = (on[c + 1] && !same) ? atomicAdd(&s_cnt[o1], 1u) : 0u;
            pos[c] = on[c] ? b0 : kSkip;
            pos[c + 1] = on[c + 1] ? (same ? b0 + (on[c] ? 1u : 0u) : b1) : kSkip;
        }
    } else {
#pragma unroll
        for (int c = 0; c < NE; ++c) pos[c] = on[c] ? atomicAdd(&s_cnt[hh[c] >> hp.slice_log2], 1u) : kSkip;
    }
    __syncthreads();
    if (threadIdx.x < 64) {   // exclusive scan of <= 128 counters in wave 0, two per lane
        const int o0 = 2 * lane, o1 = 2 * lane + 1;
        const uint32_t v0 = o0 < n_own ? s_cnt[o0] : 0u, v1 = o1 < n_own ? s_cnt[o1] : 0u;
        uint32_t inc = v0 + v1;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(inc, o, 64);
            if (lane >= o) inc += t;
        }
        const uint32_t ex0 = inc - v0 - v1, ex1 = ex0 + v0;
        if (o0 < n_own) {
            s_start[o0] = ex0;
            hp.bin_seg[((size_t)lvl * n_own + o0) * hp.chunk_stride + chunk] = ex0 | (v0 << 16);
        }
        if (o1 < n_own) {
            s_start[o1] = ex1;
            hp.bin_seg[((size_t)lvl * n_own + o1) * hp.chunk_stride + chunk] = ex1 | (v1 << 16);
        }
        if (o0 == n_own - 1) s_start[n_own] = ex1;
        if (o1 == n_own - 1) s_start[n_own] = ex1 + v1;
    }
    __syncthreads();
    const uint32_t smask = (1u << hp.slice_log2) - 1u;
#pragma unroll
    for (int c = 0; c < NE; ++c) {
        if (pos[c] != kSkip) {
            const uint32_t k = s_start[hh[c] >> hp.slice_log2] + pos[c];
            s_eh[k] = (uint16_t)(hh[c] & smask);
            s_eg[k] = make_float2(vx[c], vy[c]);
        }
    }
    if (hp.chunk_max) {   // deterministic mode: the level's largest |entry| sets the owners' fixed-point scale
        float m = 0.f;
#pragma unroll
        for (int c = 0; c < NE; ++c)
            if (pos[c] != kSkip) m = fmaxf(m, fmaxf(fabsf(vx[c]), fabsf(vy[c])));
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
        __shared__ float s_wmax[THREADS / 64];
        if (lane == 0) s_wmax[threadIdx.x >> 6] = m;
        __syncthreads();
        if (threadIdx.x == 0) {   // one plain store per chunk (per-level atomics serialise the blocks)
            for (int w = 1; w < THREADS / 64; ++w) m = fmaxf(m, s_wmax[w]);
            hp.chunk_max[(size_t)lvl * hp.chunk_stride + chunk] = m;
        }
    }
    __syncthreads();
    const uint32_t total = s_start[n_own];
    const size_t base = ((size_t)lvl * hp.chunk_stride + chunk) * kChunkCap;
    // two entries per lane: rows as one dword, (d feat) x 2 as one dwordx4; a trailing odd
    // slot carries stale LDS bytes that no owner reads (owners read < count per segment).
    // Nontemporal stores: the ~0.5 GB of entries a step writes would otherwise stream through the
    // 256 MB Infinity Cache and evict the tables and moments (192 MB) the fused table step and the
    // next forward read: owner 258 -> 239 us, step 1.332 -> 1.311 ms on one box
    // (profiles/r05t_ab_bin_nt_stores.jsonl). Nontemporal entry LOADS in the owner on top: owner
    // 236 -> 280 us; nontemporal gradient-row stores in the fused step: +-0 (r05u) — both rejected.
    for (uint32_t i = 2 * threadIdx.x; i < total; i += 2 * THREADS) {
#if NERF_BIN_NT_STORES
        __builtin_nontemporal_store(*reinterpret_cast<const uint32_t*>(&s_eh[i]), reinterpret_cast<uint32_t*>(hp.bin_h + base + i));
        typedef float nt_f4 __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(*reinterpret_cast<const nt_f4*>(&s_eg[i]), reinterpret_cast<nt_f4*>(hp.bin_g + base + i));
#else
        *reinterpret_cast<uint32_t*>(hp.bin_h + base + i) = *reinterpret_cast<const uint32_t*>(&s_eh[i]);
        *reinterpret_cast<float4*>(hp.bin_g + base + i) = *reinterpret_cast<const float4*>(&s_eg[i]);
#endif
    }
}

// Optional row maps of a bin launch (coarse-feature reuse): point p reads xyz and dfeat
// at row rows[p] (NULL: p), and adds dfeat2 at row rows2[p] (NULL: p; NULL dfeat2: nothing) to its
// gradient.
struct BinRows {
    const int32_t* rows;
    const float* dfeat2;
    const int32_t* rows2;
    int64_t sp2, sl2;
    const int32_t* count;   // optional device int: only points p < *count are binned (an active-point list)
};

// MODE 1: coalesced float atomics (no workspace); 3: binned (default). blk: the block's chunk within the
// launch's points (blockIdx.x, or its offset in a two-job launch).
template <int MODE, int THREADS>
__device__ __forceinline__ void bwd_bin_block(const float* __restrict__ xyz, int64_t n, const HashGradParams& hp,
                                              const float* __restrict__ dfeat, int64_t sp, int64_t sl,
                                              const BinRows& br, int blk) {
    const int64_t p = (int64_t)blk * blockDim.x + threadIdx.x;
    const int lvl = blockIdx.y;
    if (br.count) n = min(n, (int64_t)*br.count);
    if constexpr (MODE == 3) {
        if ((int64_t)blk * blockDim.x >= n) {   // a chunk past the active points: empty segments
            const int chunk = hp.chunk_base + blk;
            const int n_own = 1 << hp.owner_log2;
            for (int o = threadIdx.x; o < n_own; o += blockDim.x)
                hp.bin_seg[((size_t)lvl * n_own + o) * hp.chunk_stride + chunk] = 0u;
            if (hp.chunk_max && threadIdx.x == 0) hp.chunk_max[(size_t)lvl * hp.chunk_stride + chunk] = 0.f;
            return;
        }
    }
    const bool valid = p < n;
    float x = 0.f, y = 0.f, z = 0.f, gx = 0.f, gy = 0.f;
    if (valid) {
        const int64_t r = br.rows ? (int64_t)br.rows[p] : p;
        x = xyz[3 * r + 0]; y = xyz[3 * r + 1]; z = xyz[3 * r + 2];
        // d feat is read once: nontemporal loads keep it from displacing the tables and moments in the
        // Infinity Cache (with the MLP backward's feature loads: bins 202 -> 177 us per step,
        // profiles/r05v_ab_nt_feature_loads.jsonl)
        if (dfeat) {
            const float* src = dfeat + r * sp + (int64_t)lvl * sl;
            gx = __builtin_nontemporal_load(src);
            gy = __builtin_nontemporal_load(src + 1);
        }
        if (br.dfeat2) {   // the same point's gradient from a second pass (coarse-feature reuse)
            const int64_t r2 = br.rows2 ? (int64_t)br.rows2[p] : p;
            const float* s2 = br.dfeat2 + r2 * br.sp2 + (int64_t)lvl * br.sl2;
            gx += __builtin_nontemporal_load(s2);
            gy += __builtin_nontemporal_load(s2 + 1);
        }
    }
    AxisCell ax, ay, az;
    if (hp.fastdiv && __ballot(valid && !fastdiv_point_ok(x, y, z)) == 0ull) {   // wave-uniform
        ax = axis_cell<true>(x, hp.bmin[0], hp.bmax[0], hp.cell[lvl][0], hp.rcell[lvl][0]);
        ay = axis_cell<true>(y, hp.bmin[1], hp.bmax[1], hp.cell[lvl][1], hp.rcell[lvl][1]);
        az = axis_cell<true>(z, hp.bmin[2], hp.bmax[2], hp.cell[lvl][2], hp.rcell[lvl][2]);
    } else {
        ax = axis_cell(x, hp.bmin[0], hp.bmax[0], hp.cell[lvl][0]);
        ay = axis_cell(y, hp.bmin[1], hp.bmax[1], hp.cell[lvl][1]);
        az = axis_cell(z, hp.bmin[2], hp.bmax[2], hp.cell[lvl][2]);
    }
    const float wx = ax.w, wy = ay.w, wz = az.w;
    const float ox = 1.0f - wx, oy = 1.0f - wy, oz = 1.0f - wz;

    // Per-corner contributions, corner c = 4i+2j+k.
    float cgx[8], cgy[8];
    {
        const float b0x = gx * oz, b1x = gx * wz, b0y = gy * oz, b1y = gy * wz;  // d c0, d c1
        const float a00x = b0x * oy, a10x = b0x * wy, a01x = b1x * oy, a11x = b1x * wy;
        const float a00y = b0y * oy, a10y = b0y * wy, a01y = b1y * oy, a11y = b1y * wy;
        // c00 <- e0,e4 ; c01 <- e1,e5 ; c10 <- e2,e6 ; c11 <- e3,e7
        cgx[0] = a00x * ox; cgx[4] = a00x * wx; cgy[0] = a00y * ox; cgy[4] = a00y * wx;
        cgx[1] = a01x * ox; cgx[5] = a01x * wx; cgy[1] = a01y * ox; cgy[5] = a01y * wx;
        cgx[2] = a10x * ox; cgx[6] = a10x * wx; cgy[2] = a10y * ox; cgy[6] = a10y * wx;
        cgx[3] = a11x * ox; cgx[7] = a11x * wx; cgy[3] = a11y * ox; cgy[7] = a11y * wx;
    }

    // Wave-level run merge: a voxel key equal to the previous lane's continues a run; segmented
    // inclusive sums leave each run's total on its LAST lane, which alone emits the run's entries.
    // Run starts / tails come from the ballot of run heads; the sums use DPP (wave_segmented_
    // inclusive_sum), not the LDS crossbar.
    const uint32_t key_lo = (uint32_t)ax.base | ((uint32_t)ay.base << 16);
    const uint32_t key_hi = (uint32_t)az.base | (valid ? 0u : 0x80000000u);
    const int lane = threadIdx.x & 63;
    const uint32_t prev_lo = __shfl_up(key_lo, 1, 64), prev_hi = __shfl_up(key_hi, 1, 64);
    const bool head = (lane == 0) || prev_lo != key_lo || prev_hi != key_hi;
    const uint64_t heads = __ballot(head);
    const bool tail = (lane == 63) || ((heads >> (lane + 1)) & 1ull);
    if (heads != ~0ull) {  // some run has length > 1 in this wave
        const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
        const int start = 63 - __clzll(heads & upto);
        float cg[16];   // one scan over both features: the step choice is made once
#pragma unroll
        for (int c = 0; c < 8; ++c) { cg[c] = cgx[c]; cg[8 + c] = cgy[c]; }
        wave_segmented_inclusive_sum(cg, lane, start);
#pragma unroll
        for (int c = 0; c < 8; ++c) { cgx[c] = cg[c]; cgy[c] = cg[8 + c]; }
    }
    const bool emit = valid && tail;
    float* tab = hp.dtables[lvl];
    const uint32_t bx = (uint32_t)ax.base, by = (uint32_t)ay.base, bz = (uint32_t)az.base;
    if constexpr (MODE == 3) {
        // entries in x-pairs: slot 2q + i holds corner 4i + q ((x, y, z) then (x+1, y, z))
        uint32_t hh[8];
        bool on[8];
        float ex[8], ey[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int c = 4 * (e & 1) + (e >> 1);
            hh[e] = spatial_hash3(bx + ((c >> 2) & 1), by + ((c >> 1) & 1), bz + (c & 1), hp.mask);
            ex[e] = cgx[c];
            ey[e] = cgy[c];
            on[e] = emit && (ex[e] != 0.f || ey[e] != 0.f);
        }
        bin_chunk<THREADS, 8, true>(hp, lvl, hp.chunk_base + blk, hh, ex, ey, on);
    } else {
        __shared__ float s_val[4][64][17];
        __shared__ uint32_t s_h[4][64][9];
        const int wv = threadIdx.x >> 6;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            s_h[wv][lane][c] = emit ? spatial_hash3(bx + ((c >> 2) & 1), by + ((c >> 1) & 1), bz + (c & 1), hp.mask)
                                    : kSkip;
            s_val[wv][lane][2 * c + 0] = cgx[c];
            s_val[wv][lane][2 * c + 1] = cgy[c];
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll 4
        for (int r = 0; r < 16; ++r) {
            const int d = r * 64 + lane;
            const int item = d >> 4, within = d & 15;
            const int c = ((within >> 1) & 1) * 4 + (within >> 2);   // i*4 + pair(j,k)
            const int f = within & 1;
            const uint32_t h = s_h[wv][item][c];
            const float v = s_val[wv][item][2 * c + f];
            if (h != kSkip && v != 0.f) atomic_add_f32(tab + 2 * h + f, v);
        }
    }
}

template <int MODE, int THREADS>
__global__ void __launch_bounds__(THREADS) hash_encode_bwd_kernel(
    const float* __restrict__ xyz, int64_t n, HashGradParams hp,
    const float* __restrict__ dfeat, int64_t sp, int64_t sl, BinRows br) {
    bwd_bin_block<MODE, THREADS>(xyz, n, hp, dfeat, sp, sl, br, (int)blockIdx.x);
}

// Two bin jobs in one launch (the fine and the coarse pass of an iteration, side by side in one
// workspace): blocks [0, split) bin job a's chunks, the rest job b's — no drain / ramp between them.
struct BinJob {
    const float* xyz;
    int64_t n;
    HashGradParams hp;
    const float* dfeat;
    int64_t sp, sl;
    BinRows br;
};

template <int THREADS>
__global__ void __launch_bounds__(THREADS) hash_encode_bwd_pair_kernel(BinJob a, BinJob b, unsigned split) {
    if (blockIdx.x < split) bwd_bin_block<3, THREADS>(a.xyz, a.n, a.hp, a.dfeat, a.sp, a.sl, a.br, (int)blockIdx.x);
    else bwd_bin_block<3, THREADS>(b.xyz, b.n, b.hp, b.dfeat, b.sp, b.sl, b.br, (int)(blockIdx.x - split));
}

// TV backward (loss.py:11-43 autograd) into the binned workspace, summed by the same owner pass as
// the hash backward: no memory-side float atomics, and deterministic with it. Chunk k of level l
// holds vertices [k C, (k + 1) C) of the level's (cube + 1)^3 cuboid (C = kChunkCap, 8 vertices per
// thread; chunks past a level's last vertex are empty), one entry per vertex: row hash(min_vertex +
// (i, j, k)), value (sum over the in-cuboid neighbours n of 2 (e_v - e_n)) x scale[l] / cube — the
// per-vertex terms and op order of the atomic tv_bwd_kernel (optim.hip).
// Block bx of level l's TV chunks, binned as chunk `chunk` of hp's workspace.
template <int THREADS>
__device__ __forceinline__ void tv_bin_block(const TVParams& P, const HashGradParams& hp, int l, int chunk,
                                             unsigned bx) {
    constexpr int NE = 8;   // vertices per thread: chunks of kChunkCap entries, like the hash bins
    const int c = P.cube[l], n1 = c + 1;
    const uint32_t nv = (uint32_t)(P.vstart[l + 1] - P.vstart[l]);
    const float2* tab = reinterpret_cast<const float2*>(P.tables[l]);
    int mv[3];
    tv_corner(P, l, mv);
    const float s = P.scale[l] / (float)c;
    uint32_t hh[NE];
    float vx[NE], vy[NE];
    bool on[NE];
#pragma unroll
    for (int q = 0; q < NE; ++q) {
        const uint32_t lv = bx * (uint32_t)(NE * THREADS) + q * THREADS + threadIdx.x;
        float gx = 0.f, gy = 0.f;
        hh[q] = 0;
        on[q] = false;
        if (lv < nv) {
            int i, j, k;
            tv_vertex(lv, n1, i, j, k);
            // the forward's gathered rows (dense, vertex order: neighbours are lv +- 1, n1, n1^2), or
            // the hashed table rows
            const float2* V = P.verts ? P.verts + P.vstart[l] : nullptr;
            const float2 e = V ? V[lv] : tv_fetch(tab, mv, i, j, k, P.mask);
            auto pair = [&](bool cond, int di, int dj, int dk) {
                if (!cond) return;
                const float2 f = V ? V[(int)lv + (di * n1 + dj) * n1 + dk] : tv_fetch(tab, mv, i + di, j + dj, k + dk, P.mask);
                gx += 2.0f * (e.x - f.x);
                gy += 2.0f * (e.y - f.y);
            };
            pair(i > 0, -1, 0, 0);
            pair(i < c, 1, 0, 0);
            pair(j > 0, 0, -1, 0);
            pair(j < c, 0, 1, 0);
            pair(k > 0, 0, 0, -1);
            pair(k < c, 0, 0, 1);
            hh[q] = spatial_hash3((uint32_t)(mv[0] + i), (uint32_t)(mv[1] + j), (uint32_t)(mv[2] + k), P.mask);
        }
        vx[q] = gx * s;
        vy[q] = gy * s;
        on[q] = lv < nv && (vx[q] != 0.f || vy[q] != 0.f);
    }
    bin_chunk<THREADS, NE>(hp, l, chunk, hh, vx, vy, on);
}

template <int THREADS>
__global__ void __launch_bounds__(THREADS) tv_bwd_bin_kernel(TVParams P, HashGradParams hp) {
    tv_bin_block<THREADS>(P, hp, blockIdx.y, hp.chunk_base + (int)blockIdx.x, blockIdx.x);
}

// The hash bins of up to two jobs with the pass's TV bins in front (nerf_hash_encode_bwd_bin_batch_tv):
// blocks [0, tv_blocks) are TV chunks tv_base + x in job a's workspace layout (one workspace per
// batch), the rest the hash_encode_bwd_pair_kernel blocks (split: job a's chunks; b may repeat a with
// no blocks of its own). The TV's 4,224 waves ran 19.8 us as a launch of their own (rocprof r06h).
template <int THREADS>
__global__ void __launch_bounds__(THREADS) hash_encode_bwd_tv_pair_kernel(BinJob a, BinJob b, unsigned split,
                                                                          TVParams tv, int tv_base,
                                                                          unsigned tv_blocks) {
    if (blockIdx.x < tv_blocks) {
        tv_bin_block<THREADS>(tv, a.hp, blockIdx.y, tv_base + (int)blockIdx.x, blockIdx.x);
        return;
    }
    const unsigned x = blockIdx.x - tv_blocks;
    if (x < split) bwd_bin_block<3, THREADS>(a.xyz, a.n, a.hp, a.dfeat, a.sp, a.sl, a.br, (int)x);
    else bwd_bin_block<3, THREADS>(b.xyz, b.n, b.hp, b.dfeat, b.sp, b.sl, b.br, (int)(x - split));
}
static_assert(2 * sizeof(BinJob) + sizeof(TVParams) + 16 <= 4096, "hash_encode_bwd_tv_pair_kernel: kernel arguments over 4 KiB");

// ---- owner pass of the binned backward ----------------------------------------------------
// Block (o, l) owns rows [o * 2^slice_log2, (o+1) * 2^slice_log2) of level l's gradient table. It
// walks every chunk's segment for that slice, sums the entries into LDS (ds_add_f64: no
// memory-side requests) and adds the slice into the table once with plain coalesced loads/stores
// (it is the slice's only writer). Segments are ~64 entries, so instead of one segment per wave
// step the entries of a window of chunks are numbered consecutively (exclusive scan of the segment
// counts in LDS) and every lane takes every 64th entry, 8 per batch: 16 global loads in flight per
// lane, all lanes busy whatever the segment lengths.
// SLICE_LOG2 / THREADS: 2^13-row slices with one 1024-thread block per CU (128 KiB of LDS); 2^12-row
// slices with two 512-thread blocks per CU measured slower (0.41 vs 0.34 ms per backward: the
// doubled per-owner segment scans outweigh the overlap); again in round 5 with the fused table step
// in the flush (one block's flush beside the other's sums): owner 256.5 -> 269.4 us, bins +3 us
// (-DNERF_OWNER_SLICE_LOG2=12 -DNERF_OWNER_THREADS=512, profiles/r05r_ab_owner_slice12_rejected.jsonl).
//
// DET (deterministic mode): integer accumulation is associative, so the sums do not depend on the
// order in which waves add entries. Each entry v becomes two int64 fixed-point words at the level's
// scale 2^s (s from the level's largest |entry| and the entry-count bound, so no sum can overflow):
// hi = rint(v 2^s), lo = rint((v 2^s - hi) 2^L); the slice is summed with ds_add_u64 and the row
// total hi 2^-s + lo 2^-(s+L) (about 2^-75 of the level's largest entry per term) is rounded to fp32
// once. Slices are 2^12 rows (32 B of LDS per row).
#ifdef NERF_OWNER_PROF   // diagnostic build only (tools/owner_prof.py): per-block timestamps (100 MHz real
                        // time): start, first window scanned, entries summed, flushed
__device__ unsigned long long owner_prof[NERF_MAX_LEVELS * kMaxOwners * 4];
#define OWNER_T(k)                                                                                         \
    do {                                                                                                   \
        if (threadIdx.x == 0)                                                                              \
            owner_prof[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 4 + (k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define OWNER_T(k) do { } while (0)
#endif

template <int SLICE_LOG2, int THREADS, bool DET>
__global__ void __launch_bounds__(THREADS) hash_bwd_owner_kernel(HashGradParams hp) {
    OWNER_T(0);
    constexpr int kOwnerThreads = THREADS;
#ifndef NERF_OWNER_BATCH
#define NERF_OWNER_BATCH 8
#endif
    constexpr int NB = NERF_OWNER_BATCH;                   // steps per software-pipelined batch
                                                           // (12: owner 234 -> 241 us; 16: 271 us with
                                                           // spills; profiles/r05af_ab_owner_batch_rejected.jsonl)
    constexpr int kScanPer = 4;                            // chunks per thread in the window scan
    constexpr int kOwnerWindow = kScanPer * THREADS;       // chunks per window (the fine + coarse + TV
                                                           // chunks of a 4096-ray step fit one window)
    // fp64 accumulators: ds_add_f64 runs ~14x the rate of ds_add_f32 on gfx950 (tools/
    // lds_atomic_bench.hip: 2.24 vs 0.165 row updates per clock per CU, random rows), and the
    // slice total is rounded to fp32 once.
    constexpr bool A32 = kOwnerAcc32 && !DET;
    using Acc = typename std::conditional<A32, float2, double2>::type;
    __shared__ __attribute__((aligned(16))) Acc s_slice[(DET ? 2 : 1) << SLICE_LOG2];
    static_assert(sizeof(s_slice) <= 128 * 1024, "owner slice accumulators");
    // DET: four fixed-point word arrays [hi x | hi y | lo x | lo y][S] (8-B row stride per array: random
    // rows spread over all 32 bank pairs; one [row][4] record put every add on 8 of them)
    unsigned long long* s_fix = reinterpret_cast<unsigned long long*>(s_slice);
    __shared__ uint32_t s_pre[kOwnerWindow + 1];
    __shared__ uint16_t s_beg[kOwnerWindow];
    __shared__ uint32_t s_wsum[kOwnerThreads / 64];
    // Dispatch order of the levels: finest, coarsest, next finest, ... The finest levels carry the
    // most entries (a level-15 block ~74 us, a level-0 block ~25 us, tools/owner_prof.py): dispatched
    // level-major they start last and leave a tail of 64 long blocks on a quarter of the CUs
    // (makespan 244 us vs 202 us of block time per CU); interleaved, light blocks fill in behind the
    // heavy ones (235 us; owner launch 255 -> 248 us on one box, profiles/r03i_ab_owner_order.jsonl).
    // Finest first alone is slower (273 us): the coarse pass's bins, written last, are partly still
    // in the Infinity Cache when the early blocks read them. Re-measured in round 5 with the entries
    // stored nontemporally (no bins in the Infinity Cache) as a longest-first order: 234.7 -> 249.9 us
    // (profiles/r05ac_ab_fill_prologue_owner_lpt.jsonl) — the interleaving stays.
    const int o = blockIdx.x, y = blockIdx.y;
    const int lvl = hp.level0 + ((y & 1) ? (y >> 1) : (int)gridDim.y - 1 - (y >> 1));
    const int S = 1 << hp.slice_log2, n_own = 1 << hp.owner_log2;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    for (int i = tid; i < (DET ? 2 : 1) * S; i += kOwnerThreads) s_slice[i] = Acc{0, 0};
    // the two features' sums as separate arrays: an 8-B add to row h of one array lands on banks
    // (2h, 2h + 1) mod 64, all 32 bank pairs, where the interleaved (x, y) rows put every x add on
    // banks 4h, 4h + 1 (16 pairs) and doubled the conflicts of the random-row scatter
    using Sc = typename std::conditional<A32, float, double>::type;
    Sc* const s_ax = reinterpret_cast<Sc*>(s_slice);
    Sc* const s_ay = s_ax + S;
    // DET: scale exponents (hi: 2^sh, lo: 2^(sh + L)) from the level's largest |entry| (the max of
    // the chunks' maxima; a level without entries has max 0)
    int sh = 0, sl_ = 0;
    if constexpr (DET) {
        float m = 0.f;
        for (int c = tid; c < hp.nchunks; c += kOwnerThreads) m = fmaxf(m, hp.chunk_max[(size_t)lvl * hp.chunk_stride + c]);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
        if (lane == 0) s_wsum[wave] = __float_as_uint(m);
        __syncthreads();
        for (int w = 0; w < kOwnerThreads / 64; ++w) m = fmaxf(m, __uint_as_float(s_wsum[w]));
        __syncthreads();   // s_wsum is reused by the window scans
        int E;
        (void)frexpf(m, &E);                                                // max |entry| < 2^E
        const int b = kChunkCapLog2 + (32 - __clz((unsigned)max(hp.nchunks - 1, 1)));  // entries <= 2^b
        sh = 62 - E - b;
        sl_ = sh + (61 - b);
    }
    const uint32_t* seg = hp.bin_seg + ((size_t)lvl * n_own + o) * hp.chunk_stride;
    for (int w0 = 0; w0 < hp.nchunks; w0 += kOwnerWindow) {
        const int nw = min(kOwnerWindow, hp.nchunks - w0);
        // segment counts of the window -> exclusive prefix s_pre (kScanPer consecutive chunks per thread)
        uint32_t cnt[kScanPer], part = 0;
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) {
            const int i = kScanPer * tid + k;
            cnt[k] = 0;
            if (i < nw) { const uint32_t v = seg[w0 + i]; cnt[k] = v >> 16; s_beg[i] = (uint16_t)(v & 0xFFFFu); }
            part += cnt[k];
        }
        uint32_t inc = part;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t t = __shfl_up(inc, d, 64);
            if (lane >= d) inc += t;
        }
        if (lane == 63) s_wsum[wave] = inc;
        __syncthreads();
        uint32_t ex = inc - part;
        for (int w = 0; w < wave; ++w) ex += s_wsum[w];
#pragma unroll
        for (int k = 0; k < kScanPer; ++k) {
            const int i = kScanPer * tid + k;
            if (i <= nw) s_pre[i] = ex;      // i == nw: the window total
            ex += cnt[k];
        }
        if (nw == kOwnerWindow && tid == kOwnerThreads - 1) s_pre[nw] = ex;   // no thread holds i == nw
        __syncthreads();
        if (w0 == 0) OWNER_T(1);
        // The window's entries split evenly across the waves; a wave walks its range 64 entries
        // (one per lane) per step. Chunk lookup is wave-cooperative, with no per-lane walk: lane l
        // holds the boundary s_pre[cw + l] of a 64-chunk window; the chunk of entry e is the last
        // boundary <= e: a ballot gives the step's first chunk, and the few boundaries that fall
        // inside the step (read with readlane) move the lanes past them. A step ends at the
        // window's last boundary; a step starting beyond it reloads the window (binary search).
        constexpr int kWaves = kOwnerThreads / 64;
        const uint32_t tot = s_pre[nw];
        const uint32_t e_beg = (uint32_t)((uint64_t)tot * wave / kWaves);
        const uint32_t e_end = (uint32_t)((uint64_t)tot * (wave + 1) / kWaves);
        // entry offsets fit 32 bits (make_bin_plan: < 2^32 entries), one VGPR per address
        const uint32_t region0 = (uint32_t)(((size_t)lvl * hp.chunk_stride + w0) * kChunkCap);
        int cw = 0;
        uint32_t Bw = 0, Gw = 0, B63 = 0;   // B63: first entry beyond the window's chunks cw .. cw+62
        auto reload = [&](uint32_t E) {
            int lo = 0, hi = nw;   // s_pre[lo] <= E < s_pre[hi]
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (s_pre[mid] <= E) lo = mid; else hi = mid;
            }
            cw = lo;
            const int ci = cw + lane;
            Bw = ci <= nw ? s_pre[ci] : 0xFFFFFFFFu;
            Gw = ci < nw ? (uint32_t)s_beg[ci] : 0u;
            B63 = __builtin_amdgcn_readlane(Bw, 63);
        };
        // address of entry E + lane (ok: inside [E, end of step)); returns the next step's start
        auto step = [&](uint32_t E, uint32_t& addr, bool& ok) -> uint32_t {
            if (E >= e_end) { addr = region0; ok = false; return E; }
            if (E >= B63) reload(E);
            const uint32_t lim = min(min(E + 64u, B63), e_end);
            const uint32_t e = E + lane;
            int idx = __popcll(__ballot(Bw <= E)) - 1;
            uint64_t inner = __ballot(Bw > E && Bw < lim);
            while (inner) {
                const int b = __ffsll((unsigned long long)inner) - 1;
                inner &= inner - 1;
                idx += e >= (uint32_t)__builtin_amdgcn_readlane(Bw, b) ? 1 : 0;
            }
            const uint32_t cur = (uint32_t)__builtin_amdgcn_ds_bpermute(idx << 2, (int)Bw);
            const uint32_t beg = (uint32_t)__builtin_amdgcn_ds_bpermute(idx << 2, (int)Gw);
            ok = e < lim;
            addr = ok ? region0 + (uint32_t)(cw + idx) * kChunkCap + beg + (e - cur) : region0;
            return lim;
        };
        auto track = [&](uint32_t& E, uint32_t (&addr)[NB], uint32_t& valid) {
            valid = 0;
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                bool ok;
                E = step(E, addr[j], ok);
                valid |= (ok ? 1u : 0u) << j;
            }
        };
        auto fetch = [&](const uint32_t (&addr)[NB], uint16_t (&h)[NB], float2 (&g)[NB]) {
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                // default-policy loads: the coarse pass's bins were written just before this launch and part
                // of them is still in the Infinity Cache (nontemporal loads: 0.39 vs 0.33 ms per step)
                h[j] = hp.bin_h[addr[j]];
                const uint64_t gv = *reinterpret_cast<const uint64_t*>(hp.bin_g + addr[j]);   // (d feat0, d feat1)
                g[j] = make_float2(__uint_as_float((uint32_t)gv), __uint_as_float((uint32_t)(gv >> 32)));
            }
        };
        // software pipeline: the next batch's loads are in flight while this batch's adds run
        uint32_t addr[NB];
        uint16_t h[NB];
        float2 g[NB];
        uint32_t valid;
        uint32_t E = e_beg;
        if (E < e_end) reload(E);
        track(E, addr, valid);
        fetch(addr, h, g);
        // the loop and step() (ballots, readlane, bpermute) stay wave-uniform: exit only when no
        // lane of the wave has an entry left
        while (__ballot(valid != 0u) != 0ull) {
            uint32_t addr2[NB];
            uint16_t h2[NB];
            float2 g2[NB];
            uint32_t valid2;
            track(E, addr2, valid2);
            fetch(addr2, h2, g2);
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                if (valid & (1u << j)) {
                    if constexpr (DET) {
                        const double tx = ldexp((double)g[j].x, sh), ty = ldexp((double)g[j].y, sh);
                        const double hx = rint(tx), hy = rint(ty);
                        const long long lx = (long long)rint(ldexp(tx - hx, sl_ - sh));
                        const long long ly = (long long)rint(ldexp(ty - hy, sl_ - sh));
                        unsigned long long* r = s_fix + h[j];
                        atomicAdd(r, (unsigned long long)(long long)hx);
                        atomicAdd(r + S, (unsigned long long)(long long)hy);
                        atomicAdd(r + 2 * S, (unsigned long long)lx);
                        atomicAdd(r + 3 * S, (unsigned long long)ly);
                    } else {
                        atomicAdd(&s_ax[h[j]], (Sc)g[j].x);
                        atomicAdd(&s_ay[h[j]], (Sc)g[j].y);
                    }
                }
            }
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                h[j] = h2[j];
                g[j] = g2[j];
            }
            valid = valid2;
        }
        if (w0 + kOwnerWindow < hp.nchunks) __syncthreads();   // s_pre / s_beg reused by the next window
    }
    // fused table step, full slices (the lego hot path): the last window's barrier is the flush barrier
    // below, and a thread done with its entries issues its rows' parameter / moment loads before it
    // waits there for the block's slower waves
    // (half of a thread's rows here, the other half at the flush: all of them would spill)
    constexpr int kRowsP = (1 << SLICE_LOG2) / THREADS, kHalf = kRowsP / 2;
    const bool pre = !DET && hp.st_on && hp.overwrite && S == (1 << SLICE_LOG2);
    float2 pp[kRowsP], pm[kRowsP], pv[kRowsP];
    const size_t prow0 = (size_t)o * S;
    auto pload = [&](int k) {
        pp[k] = reinterpret_cast<const float2*>(hp.st_p[lvl])[prow0 + tid + k * THREADS];
        pm[k] = reinterpret_cast<const float2*>(hp.st_m[lvl])[prow0 + tid + k * THREADS];
        pv[k] = reinterpret_cast<const float2*>(hp.st_v[lvl])[prow0 + tid + k * THREADS];
    };
    if (pre) {
#pragma unroll
        for (int k = 0; k < kHalf; ++k) pload(k);
    }
    // Flush: every row's table load is issued before any add (one memory round trip per block,
    // not one per row batch: a load behind the previous batch's store left 8 serial round trips).
    __syncthreads();
    OWNER_T(2);
#ifdef NERF_OWNER_PROF
    struct Done {
        __device__ ~Done() { __syncthreads(); OWNER_T(3); }
    } done;
#endif
    float2* dt = reinterpret_cast<float2*>(hp.dtables[lvl]) + (size_t)o * S;
    constexpr int kRows = (1 << SLICE_LOG2) / kOwnerThreads;
    if constexpr (DET) {
        auto fixed = [&](int row, int f) {
            const long long hi = (long long)s_fix[f * S + row], lo = (long long)s_fix[(2 + f) * S + row];
            return ldexp((double)hi, -sh) + ldexp((double)lo, -sl_);
        };
        if (hp.st_on) {   // overwrite mode (the entry point checks): the stored row is the step's gradient
            owner_table_step<kOwnerThreads, kRows>(hp, lvl, (size_t)o * S, S, dt, [&](int i) {
                return make_float2((float)fixed(i, 0), (float)fixed(i, 1));
            });
            return;
        }
        for (int i = tid; i < S; i += kOwnerThreads) {
            const double vx = fixed(i, 0), vy = fixed(i, 1);
            if (hp.overwrite) {
                dt[i] = make_float2((float)vx, (float)vy);   // == (float)(0.0 + v), and +0 where v == 0
            } else if (vx != 0.0 || vy != 0.0) {
                const float2 t = dt[i];
                dt[i] = make_float2((float)((double)t.x + vx), (float)((double)t.y + vy));
            }
        }
        return;
    }
    if (hp.overwrite) {   // rows without entries become +0, as after a memset
        if (pre) {
            nerf_radam_segment s = hp.st;
            if (hp.st_coef) {
                s.decay_coef = hp.st_coef[0];
                s.step_coef = hp.st_coef[1];
                s.mode = (int)hp.st_coef[2];
            }
            float2* P = reinterpret_cast<float2*>(hp.st_p[lvl]) + (size_t)o * S;
            float2* M = reinterpret_cast<float2*>(hp.st_m[lvl]) + (size_t)o * S;
            float2* V = reinterpret_cast<float2*>(hp.st_v[lvl]) + (size_t)o * S;
#pragma unroll
            for (int k = kHalf; k < kRowsP; ++k) pload(k);
#pragma unroll
            for (int k = 0; k < kRowsP; ++k) {
                const int i = tid + k * kOwnerThreads;
                const Acc v{s_ax[i], s_ay[i]};
                const float2 g = make_float2((float)v.x, (float)v.y);
                dt[i] = g;
                if (radam_idle(s, g, pm[k], pv[k])) continue;
                radam_elem(s, pp[k].x, g.x, pm[k].x, pv[k].x);
                radam_elem(s, pp[k].y, g.y, pm[k].y, pv[k].y);
                M[i] = pm[k];
                V[i] = pv[k];
                if (s.mode != 0) P[i] = pp[k];
            }
            return;
        }
        if (hp.st_on) {
            owner_table_step<kOwnerThreads, kRows>(hp, lvl, (size_t)o * S, S, dt, [&](int i) {
                const Acc v{s_ax[i], s_ay[i]};
                return make_float2((float)v.x, (float)v.y);
            });
            return;
        }
        for (int i = tid; i < S; i += kOwnerThreads) {
            const Acc v{s_ax[i], s_ay[i]};
            dt[i] = make_float2((float)v.x, (float)v.y);
        }
        return;
    }
    // the row's prior gradient plus the slice's sum: in fp32 (A32, as the reference's accumulating
    // .grad) or with the fp64 sum rounded once
    auto plus = [](float t, auto v) { return A32 ? (float)(t + v) : (float)((double)t + (double)v); };
    if (S == (1 << SLICE_LOG2)) {
        float2 t[kRows];
#pragma unroll
        for (int k = 0; k < kRows; ++k) t[k] = dt[tid + k * kOwnerThreads];
#pragma unroll
        for (int k = 0; k < kRows; ++k) {
            const Acc v{s_ax[tid + k * kOwnerThreads], s_ay[tid + k * kOwnerThreads]};
            if (v.x != 0 || v.y != 0) dt[tid + k * kOwnerThreads] = make_float2(plus(t[k].x, v.x), plus(t[k].y, v.y));
        }
    } else {   // small tables (log2_T < slice): one partial slice per level
        for (int i = tid; i < S; i += kOwnerThreads) {
            const Acc v{s_ax[i], s_ay[i]};
            if (v.x != 0 || v.y != 0) {
                const float2 t = dt[i];
                dt[i] = make_float2(plus(t.x, v.x), plus(t.y, v.y));
            }
        }
    }
}

// Entries a step's bin launches emitted (the counts of every segment word of chunks [0, n_chunks)):
// a measurement for bench.py's pricing of the hash backward (bins drop zero entries and merge runs).
__global__ void __launch_bounds__(1024) bin_entry_count_kernel(const uint32_t* __restrict__ seg, int64_t n_words_per_lvl,
                                                               int64_t stride, int n_chunks, int L,
                                                               unsigned long long* __restrict__ count) {
    unsigned long long part = 0;
    const int64_t total = (int64_t)L * n_words_per_lvl * n_chunks;
    for (int64_t i = threadIdx.x; i < total; i += blockDim.x) {
        const int64_t row = i / n_chunks, c = i - row * n_chunks;
        part += seg[row * stride + c] >> 16;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
    __shared__ unsigned long long s_part[16];
    if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = part;
    __syncthreads();
    if (threadIdx.x == 0) {   // one block: a plain store, in a fixed order
        unsigned long long t = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += s_part[w];
        *count = t;
    }
}

struct BinPlan {
    int slice_log2, owner_log2, nchunks;
    size_t off_h, off_g, off_off, off_max, total;   // byte offsets in the workspace
};

// Binned path for log2_T in [1, slice + log2(kMaxOwners)]: slices of min(2^slice, T) rows.
static bool make_bin_plan(int n_levels, int log2_T, int64_t n_points, BinPlan& B, bool det = false) {
    const int slice = det ? kSliceLog2Det : kSliceLog2;
    if (log2_T < 1 || log2_T > slice + kMaxOwnersLog2 || n_points < 0) return false;
    B.slice_log2 = log2_T < slice ? log2_T : slice;
    B.owner_log2 = log2_T - B.slice_log2;
    B.nchunks = (int)((n_points + kChunkPts - 1) / kChunkPts);
    const size_t entries = (size_t)n_levels * B.nchunks * kChunkCap;
    if (entries >= ((size_t)1 << 32)) return false;   // the owner pass indexes entries with 32 bits
    const size_t offs = (size_t)n_levels * B.nchunks * (1 << B.owner_log2);
    auto up = [](size_t v) { return (v + 255) & ~(size_t)255; };
    B.off_g = 0;
    B.off_h = up(entries * sizeof(float2));
    B.off_off = B.off_h + up(entries * sizeof(uint16_t));
    B.off_max = B.off_off + up(offs * sizeof(uint32_t));
    B.total = B.off_max + (det ? up((size_t)n_levels * B.nchunks * sizeof(float)) : 0);
    return true;
}

}  // namespace nerf

using namespace nerf;

extern "C" int nerf_hash_encode_fwd_q(const float* d_xyz, int64_t n_points, const float* bbox_min3,
                                      const float* bbox_max3, const float* level_res, int n_levels, int log2_T,
                                      const float* const* d_tables, const float* d_qrec, float* d_feat,
                                      int64_t feat_stride_point, int64_t feat_stride_level, uint8_t* d_keep,
                                      void* stream) {
    NERF_REQUIRE(n_points >= 0, "hash_encode_fwd: n_points < 0");
    NERF_REQUIRE(n_levels >= 1 && n_levels <= NERF_MAX_LEVELS, "hash_encode_fwd: n_levels %d", n_levels);
    NERF_REQUIRE(log2_T >= 1 && log2_T <= 30, "hash_encode_fwd: log2_T %d", log2_T);
    NERF_REQUIRE((n_points == 0 || (d_xyz && d_feat)) && d_tables && level_res && bbox_min3 && bbox_max3, "hash_encode_fwd: null arg");
    if (n_points == 0) return NERF_OK;
    HashParams hp{};
    for (int l = 0; l < n_levels; ++l) {
        NERF_REQUIRE(d_tables[l], "hash_encode_fwd: table %d is null", l);
        hp.tables[l] = d_tables[l];
    }
    for (int a = 0; a < 3; ++a) { hp.bmin[a] = bbox_min3[a]; hp.bmax[a] = bbox_max3[a]; }
    hp.fastdiv = fill_cells(hp.cell, hp.rcell, bbox_min3, bbox_max3, level_res, n_levels) ? 1u : 0u;
    hp.mask = (uint32_t)((1u << log2_T) - 1u);
    const QuantRec* q = reinterpret_cast<const QuantRec*>(d_qrec);
    // coarse levels grouped into one grid row: the leading levels whose (res + 1)^3 vertices fit the
    // table (no hash collisions, a small set of hot lines)
    int group = 0;
    while (group < std::min(n_levels, kFwdGroupMax)) {
        const double v = (double)level_res[group] + 1.0;
        if (v * v * v > (double)(1u << log2_T)) break;
        ++group;
    }
    if (group < 2) group = 0;
    // one-dimensional grid over every level row: gridDim.x * 256 work-items must stay below 2^32, so a
    // call of more points than one launch holds runs as consecutive point ranges (rows stay
    // level-major inside each)
    auto blocks = [&](int64_t n, unsigned& gx0, unsigned& gx1) {
        gx0 = group > 0 ? (unsigned)blocks_for(2 * n, 256) : 0u;
        gx1 = (unsigned)blocks_for(2 * n, 256 * kFwdRowPts);
        return (uint64_t)gx0 + (uint64_t)gx1 * (uint64_t)(n_levels - (group > 0 ? group : 0));
    };
    constexpr uint64_t kMaxBlocks = 0xFFFFFFFFull / 256;
    int64_t span = n_points;
    unsigned gx0, gx1;
    while (blocks(span, gx0, gx1) > kMaxBlocks) span = ((span / 2) + 255) & ~(int64_t)255;
    for (int64_t p0 = 0; p0 < n_points; p0 += span) {
        const int64_t n = std::min(span, n_points - p0);
        const dim3 grid((unsigned)blocks(n, gx0, gx1));
        uint8_t* kp = d_keep ? d_keep + p0 : nullptr;
        float* fp = d_feat + p0 * feat_stride_point;
        if (q)
            hipLaunchKernelGGL(hash_encode_fwd_pair_kernel<true>, grid, dim3(256), 0, as_stream(stream), d_xyz + 3 * p0,
                               n, hp, group, gx0, gx1, fp, feat_stride_point, feat_stride_level, kp, q);
        else
            hipLaunchKernelGGL(hash_encode_fwd_pair_kernel<false>, grid, dim3(256), 0, as_stream(stream), d_xyz + 3 * p0,
                               n, hp, group, gx0, gx1, fp, feat_stride_point, feat_stride_level, kp, q);
        NERF_CHECK_LAUNCH("hash_encode_fwd");
    }
    return NERF_OK;
}

extern "C" int nerf_hash_encode_fwd(const float* d_xyz, int64_t n_points, const float* bbox_min3,
                                    const float* bbox_max3, const float* level_res, int n_levels, int log2_T,
                                    const float* const* d_tables, float* d_feat, int64_t feat_stride_point,
                                    int64_t feat_stride_level, uint8_t* d_keep, void* stream) {
    return nerf_hash_encode_fwd_q(d_xyz, n_points, bbox_min3, bbox_max3, level_res, n_levels, log2_T, d_tables,
                                  nullptr, d_feat, feat_stride_point, feat_stride_level, d_keep, stream);
}

// ---- binned backward: bin launches + one owner launch ---------------------------------------
// The fine and the coarse pass of a training iteration scatter into the same tables; binning both
// into one workspace (side by side, chunk_base apart) and summing them with ONE owner launch pays
// the owner's per-launch costs (LDS clear, slice flush = a read-modify-write of every table row)
// once per iteration instead of once per pass.
static int bin_layout(const char* who, int n_levels, int log2_T, int64_t chunk_capacity, int det, void* d_workspace,
                      size_t workspace_bytes, HashGradParams& hp) {
    NERF_REQUIRE(n_levels >= 1 && n_levels <= NERF_MAX_LEVELS, "%s: n_levels %d", who, n_levels);
    NERF_REQUIRE(chunk_capacity >= 1 && chunk_capacity <= (int64_t)1 << 26, "%s: chunk_capacity %lld", who,
                 (long long)chunk_capacity);
    BinPlan B{};
    NERF_REQUIRE(make_bin_plan(n_levels, log2_T, chunk_capacity * kChunkPts, B, det != 0),
                 "%s: no binned path for log2_T %d%s", who, log2_T, det ? " (deterministic)" : "");
    NERF_REQUIRE(d_workspace != nullptr && workspace_bytes >= B.total,
                 "%s: workspace %zu B < %zu B (nerf_hash_encode_bwd_workspace_bytes(L, log2_T, NERF_HASH_CHUNK_POINTS * capacity, det))",
                 who, workspace_bytes, B.total);
    char* ws = static_cast<char*>(d_workspace);
    hp.bin_g = reinterpret_cast<float2*>(ws + B.off_g);
    hp.bin_h = reinterpret_cast<uint16_t*>(ws + B.off_h);
    hp.bin_seg = reinterpret_cast<uint32_t*>(ws + B.off_off);
    hp.chunk_max = det ? reinterpret_cast<float*>(ws + B.off_max) : nullptr;
    hp.chunk_stride = B.nchunks;
    hp.slice_log2 = B.slice_log2;
    hp.owner_log2 = B.owner_log2;
    hp.mask = (uint32_t)((1u << log2_T) - 1u);
    return NERF_OK;
}

extern "C" int nerf_hash_bwd_chunk_points(void) { return kChunkPts; }

#ifdef NERF_FWD_PROF
extern "C" int nerf_fwd_prof_read(unsigned long long* host, int n) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(fwd_prof), sizeof(unsigned long long) * (size_t)n);
}
#endif

#ifdef NERF_OWNER_PROF
extern "C" int nerf_owner_prof_read(unsigned long long* host, int n) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(owner_prof), sizeof(unsigned long long) * (size_t)n);
}
#endif

extern "C" size_t nerf_hash_encode_bwd_workspace_bytes(int n_levels, int log2_T, int64_t n_points, int deterministic) {
    BinPlan B{};
    if (n_levels < 1 || n_levels > NERF_MAX_LEVELS || !make_bin_plan(n_levels, log2_T, n_points, B, deterministic != 0))
        return 0;
    return B.total;
}

extern "C" int nerf_hash_encode_bwd_bin_rows(const float* d_xyz, const int32_t* d_rows, const int32_t* d_count,
                                             int64_t n_points,
                                             const float* bbox_min3, const float* bbox_max3, const float* level_res,
                                             int n_levels, int log2_T, const float* d_dfeat, int64_t feat_stride_point,
                                             int64_t feat_stride_level, const float* d_dfeat2, const int32_t* d_rows2,
                                             int64_t feat2_stride_point, int64_t feat2_stride_level,
                                             int64_t chunk_base, int64_t chunk_capacity, int deterministic,
                                             void* d_workspace, size_t workspace_bytes, void* stream) {
    const nerf_bin_job j{d_xyz, d_rows, d_count, n_points, d_dfeat, feat_stride_point, feat_stride_level, d_dfeat2,
                         d_rows2, feat2_stride_point, feat2_stride_level, chunk_base};
    return nerf_hash_encode_bwd_bin_batch(&j, 1, bbox_min3, bbox_max3, level_res, n_levels, log2_T, chunk_capacity,
                                          deterministic, d_workspace, workspace_bytes, stream);
}

static int bin_job(const nerf_bin_job& j, const float* bbox_min3, const float* bbox_max3, const float* level_res,
                   int n_levels, int log2_T, int64_t chunk_capacity, int deterministic, void* d_workspace,
                   size_t workspace_bytes, BinJob& out, int64_t& nch) {
    NERF_REQUIRE(j.n_points >= 0, "hash_encode_bwd_bin: n_points < 0");
    NERF_REQUIRE((j.n_points == 0 || (j.xyz && (j.dfeat || j.dfeat2))) && level_res && bbox_min3 && bbox_max3,
                 "hash_encode_bwd_bin: null arg");
    NERF_REQUIRE(j.n_points == 0 || !j.dfeat2 || (((uintptr_t)j.dfeat2 & 7) == 0 && j.feat2_stride_point % 2 == 0 &&
                                                  j.feat2_stride_level % 2 == 0),
                 "hash_encode_bwd_bin: dfeat2 needs 8-B aligned feature pairs");
    HashGradParams hp{};
    const int rc = bin_layout("hash_encode_bwd_bin", n_levels, log2_T, chunk_capacity, deterministic, d_workspace,
                              workspace_bytes, hp);
    if (rc) return rc;
    nch = (j.n_points + kChunkPts - 1) / kChunkPts;
    NERF_REQUIRE(j.chunk_base >= 0 && j.chunk_base + nch <= chunk_capacity,
                 "hash_encode_bwd_bin: chunks [%lld, %lld) exceed the capacity %lld", (long long)j.chunk_base,
                 (long long)(j.chunk_base + nch), (long long)chunk_capacity);
    for (int a = 0; a < 3; ++a) { hp.bmin[a] = bbox_min3[a]; hp.bmax[a] = bbox_max3[a]; }
    hp.fastdiv = fill_cells(hp.cell, hp.rcell, bbox_min3, bbox_max3, level_res, n_levels) ? 1u : 0u;
    hp.chunk_base = (int)j.chunk_base;
    hp.nchunks = (int)(j.chunk_base + nch);
    out = BinJob{j.xyz, j.n_points, hp, j.dfeat, j.feat_stride_point, j.feat_stride_level,
                 BinRows{j.rows, j.dfeat2, j.rows2, j.feat2_stride_point, j.feat2_stride_level, j.count}};
    return NERF_OK;
}

static int64_t tv_bin_chunks(int n_levels, const int* cube) {
    int64_t most = 0;
    for (int l = 0; l < n_levels; ++l) {
        const int64_t n1 = (int64_t)cube[l] + 1;
        most = std::max<int64_t>(most, (n1 * n1 * n1 + kChunkCap - 1) / kChunkCap);
    }
    return most;
}

extern "C" int64_t nerf_tv_bwd_bin_chunks(int n_levels, const int* cube) {
    if (n_levels < 1 || n_levels > NERF_MAX_LEVELS || !cube) return 0;
    for (int l = 0; l < n_levels; ++l)
        if (cube[l] < 1 || cube[l] > 1024) return 0;
    return tv_bin_chunks(n_levels, cube);
}

static int launch_bin_jobs(const nerf_bin_job* jobs, int n_jobs, const BinJob* bj, const int64_t* nch, int i,
                           int n_levels, hipStream_t st) {
    while (i < n_jobs) {
        if (jobs[i].n_points == 0) { ++i; continue; }
        int k = i + 1;
        while (k < n_jobs && jobs[k].n_points == 0) ++k;
        if (k < n_jobs) {   // two jobs: one launch
            hipLaunchKernelGGL((hash_encode_bwd_pair_kernel<kChunkPts>), dim3((unsigned)(nch[i] + nch[k]), n_levels),
                               dim3(kChunkPts), 0, st, bj[i], bj[k], (unsigned)nch[i]);
            i = k + 1;
        } else {
            const BinJob& b = bj[i];
            hipLaunchKernelGGL((hash_encode_bwd_kernel<3, kChunkPts>), dim3((unsigned)nch[i], n_levels), dim3(kChunkPts),
                               0, st, b.xyz, b.n, b.hp, b.dfeat, b.sp, b.sl, b.br);
            i = k;
        }
    }
    NERF_CHECK_LAUNCH("hash_encode_bwd_bin");
    return NERF_OK;
}

static int tv_bin_params(const char* fn, const nerf_tv_bin_job& j, int n_levels, int log2_T, int64_t chunk_capacity,
                         TVParams& P, int64_t& nch) {
    int rc = fill_tv(P, n_levels, log2_T, j.min_vertex, j.d_min_vertex, j.cube);
    if (rc) return rc;
    NERF_REQUIRE(j.d_tables && j.d_scale, "%s: null arg", fn);
    for (int l = 0; l < n_levels; ++l) {
        NERF_REQUIRE(j.d_tables[l], "%s: table %d null", fn, l);
        P.tables[l] = j.d_tables[l];
    }
    P.scale = j.d_scale;
    P.verts = const_cast<float2*>(reinterpret_cast<const float2*>(j.d_verts));
    nch = tv_bin_chunks(n_levels, j.cube);
    NERF_REQUIRE(j.chunk_base >= 0 && j.chunk_base + nch <= chunk_capacity, "%s: chunks [%lld, %lld) exceed the capacity %lld",
                 fn, (long long)j.chunk_base, (long long)(j.chunk_base + nch), (long long)chunk_capacity);
    return NERF_OK;
}

extern "C" int nerf_hash_encode_bwd_bin_batch(const nerf_bin_job* jobs, int n_jobs, const float* bbox_min3,
                                              const float* bbox_max3, const float* level_res, int n_levels,
                                              int log2_T, int64_t chunk_capacity, int deterministic,
                                              void* d_workspace, size_t workspace_bytes, void* stream) {
    return nerf_hash_encode_bwd_bin_batch_tv(jobs, n_jobs, bbox_min3, bbox_max3, level_res, n_levels, log2_T,
                                             chunk_capacity, deterministic, d_workspace, workspace_bytes, nullptr,
                                             stream);
}

extern "C" int nerf_hash_encode_bwd_bin_batch_tv(const nerf_bin_job* jobs, int n_jobs, const float* bbox_min3,
                                                 const float* bbox_max3, const float* level_res, int n_levels,
                                                 int log2_T, int64_t chunk_capacity, int deterministic,
                                                 void* d_workspace, size_t workspace_bytes, const nerf_tv_bin_job* tv,
                                                 void* stream) {
    NERF_REQUIRE(n_jobs >= 0 && n_jobs <= 8 && (n_jobs == 0 || jobs), "hash_encode_bwd_bin_batch: %d jobs", n_jobs);
    BinJob bj[8];
    int64_t nch[8];
    for (int i = 0; i < n_jobs; ++i) {   // every job validated before anything is launched
        const int rc = bin_job(jobs[i], bbox_min3, bbox_max3, level_res, n_levels, log2_T, chunk_capacity,
                               deterministic, d_workspace, workspace_bytes, bj[i], nch[i]);
        if (rc) return rc;
    }
    hipStream_t st = as_stream(stream);
    TVParams P{};
    int64_t tv_nch = 0;
    if (tv) {
        NERF_REQUIRE(tv->d_verts, "hash_encode_bwd_bin_batch_tv: d_verts required");
        const int rc = tv_bin_params("hash_encode_bwd_bin_batch_tv", *tv, n_levels, log2_T, chunk_capacity, P, tv_nch);
        if (rc) return rc;
        int first = 0;
        while (first < n_jobs && jobs[first].n_points == 0) ++first;
        if (first == n_jobs) {   // no hash points: the TV bins alone
            HashGradParams hp{};
            const int rc2 = bin_layout("hash_encode_bwd_bin_batch_tv", n_levels, log2_T, chunk_capacity, deterministic,
                                       d_workspace, workspace_bytes, hp);
            if (rc2) return rc2;
            hp.chunk_base = (int)tv->chunk_base;
            hipLaunchKernelGGL((tv_bwd_bin_kernel<kChunkPts>), dim3((unsigned)tv_nch, n_levels), dim3(kChunkPts), 0, st,
                               P, hp);
            NERF_CHECK_LAUNCH("hash_encode_bwd_bin_batch_tv");
            return NERF_OK;
        }
        int second = first + 1;
        while (second < n_jobs && jobs[second].n_points == 0) ++second;
        const bool pair = second < n_jobs;
        hipLaunchKernelGGL((hash_encode_bwd_tv_pair_kernel<kChunkPts>),
                           dim3((unsigned)(tv_nch + nch[first] + (pair ? nch[second] : 0)), n_levels), dim3(kChunkPts),
                           0, st, bj[first], pair ? bj[second] : bj[first], (unsigned)nch[first], P,
                           (int)tv->chunk_base, (unsigned)tv_nch);
        NERF_CHECK_LAUNCH("hash_encode_bwd_bin_batch_tv");
        return launch_bin_jobs(jobs, n_jobs, bj, nch, pair ? second + 1 : second, n_levels, st);   // any further jobs
    }
    return launch_bin_jobs(jobs, n_jobs, bj, nch, 0, n_levels, st);
}

extern "C" int nerf_hash_encode_bwd_bin(const float* d_xyz, int64_t n_points, const float* bbox_min3,
                                        const float* bbox_max3, const float* level_res, int n_levels, int log2_T,
                                        const float* d_dfeat, int64_t feat_stride_point, int64_t feat_stride_level,
                                        int64_t chunk_base, int64_t chunk_capacity, int deterministic,
                                        void* d_workspace, size_t workspace_bytes, void* stream) {
    NERF_REQUIRE(n_points == 0 || d_dfeat, "hash_encode_bwd_bin: null arg");
    return nerf_hash_encode_bwd_bin_rows(d_xyz, nullptr, nullptr, n_points, bbox_min3, bbox_max3, level_res, n_levels,
                                         log2_T,
                                         d_dfeat, feat_stride_point, feat_stride_level, nullptr, nullptr, 0, 0,
                                         chunk_base, chunk_capacity, deterministic, d_workspace, workspace_bytes,
                                         stream);
}

extern "C" int nerf_tv_bwd_bin(const float* const* d_tables, int n_levels, int log2_T, const int64_t* min_vertex,
                               const int64_t* d_min_vertex, const int* cube, const float* d_scale,
                               const float* d_verts, int64_t chunk_base, int64_t chunk_capacity, int deterministic,
                               void* d_workspace, size_t workspace_bytes, void* stream) {
    TVParams P{};
    int rc = fill_tv(P, n_levels, log2_T, min_vertex, d_min_vertex, cube);
    if (rc) return rc;
    NERF_REQUIRE(d_tables && d_scale, "tv_bwd_bin: null arg");
    for (int l = 0; l < n_levels; ++l) {
        NERF_REQUIRE(d_tables[l], "tv_bwd_bin: table %d null", l);
        P.tables[l] = d_tables[l];
    }
    P.scale = d_scale;
    P.verts = const_cast<float2*>(reinterpret_cast<const float2*>(d_verts));
    HashGradParams hp{};
    rc = bin_layout("tv_bwd_bin", n_levels, log2_T, chunk_capacity, deterministic, d_workspace, workspace_bytes, hp);
    if (rc) return rc;
    const int64_t nch = tv_bin_chunks(n_levels, cube);
    NERF_REQUIRE(chunk_base >= 0 && chunk_base + nch <= chunk_capacity,
                 "tv_bwd_bin: chunks [%lld, %lld) exceed the capacity %lld", (long long)chunk_base,
                 (long long)(chunk_base + nch), (long long)chunk_capacity);
    hp.chunk_base = (int)chunk_base;
    hipLaunchKernelGGL((tv_bwd_bin_kernel<kChunkPts>), dim3((unsigned)nch, n_levels), dim3(kChunkPts), 0,
                       as_stream(stream), P, hp);
    NERF_CHECK_LAUNCH("tv_bwd_bin");
    return NERF_OK;
}

extern "C" int nerf_hash_encode_bwd_owner_step(int n_levels, int level_begin, int level_end, int log2_T,
                                               int64_t n_chunks, int64_t chunk_capacity, float* const* d_dtables,
                                               int deterministic, void* d_workspace, size_t workspace_bytes,
                                               const nerf_radam_table_step* step, void* stream) {
    NERF_REQUIRE((deterministic & ~(1 | NERF_OWNER_OVERWRITE)) == 0, "hash_encode_bwd_owner: flags %d", deterministic);
    NERF_REQUIRE(0 <= level_begin && level_begin <= level_end && level_end <= n_levels,
                 "hash_encode_bwd_owner: level range [%d, %d) of %d", level_begin, level_end, n_levels);
    const bool overwrite = (deterministic & NERF_OWNER_OVERWRITE) != 0;
    deterministic &= 1;
    HashGradParams hp{};
    const int rc = bin_layout("hash_encode_bwd_owner", n_levels, log2_T, chunk_capacity, deterministic, d_workspace,
                              workspace_bytes, hp);
    if (rc) return rc;
    hp.overwrite = overwrite ? 1 : 0;
    NERF_REQUIRE(n_chunks >= 0 && n_chunks <= chunk_capacity, "hash_encode_bwd_owner: n_chunks %lld of %lld",
                 (long long)n_chunks, (long long)chunk_capacity);
    if (step) {
        NERF_REQUIRE(overwrite, "hash_encode_bwd_owner: the fused table step needs NERF_OWNER_OVERWRITE (the "
                                "stored row is the whole gradient)");
        NERF_REQUIRE(step->d_params && step->d_exp_avg && step->d_exp_avg_sq && step->mode >= 0 && step->mode <= 2,
                     "hash_encode_bwd_owner: bad table step");
        for (int l = level_begin; l < level_end; ++l) {
            NERF_REQUIRE(step->d_params[l] && step->d_exp_avg[l] && step->d_exp_avg_sq[l] &&
                             (((uintptr_t)step->d_params[l] | (uintptr_t)step->d_exp_avg[l] |
                               (uintptr_t)step->d_exp_avg_sq[l]) & 7) == 0,
                         "hash_encode_bwd_owner: table step level %d: null or unaligned tensor", l);
            hp.st_p[l] = step->d_params[l];
            hp.st_m[l] = step->d_exp_avg[l];
            hp.st_v[l] = step->d_exp_avg_sq[l];
        }
        hp.st.beta1 = step->beta1; hp.st.beta2 = step->beta2;
        hp.st.one_minus_beta1 = step->one_minus_beta1; hp.st.one_minus_beta2 = step->one_minus_beta2;
        hp.st.eps = step->eps; hp.st.decay_coef = step->decay_coef; hp.st.step_coef = step->step_coef;
        hp.st.mode = step->mode;
        hp.st_coef = step->d_coef;
        hp.st_on = 1;
    }
    NERF_REQUIRE(d_dtables, "hash_encode_bwd_owner: null grad tables");
    for (int l = 0; l < n_levels; ++l) {
        NERF_REQUIRE(d_dtables[l], "hash_encode_bwd_owner: grad table %d is null", l);
        hp.dtables[l] = d_dtables[l];
    }
    if ((n_chunks == 0 && !overwrite) || level_end == level_begin) return NERF_OK;
    hp.nchunks = (int)n_chunks;
    hp.level0 = level_begin;
    const dim3 grid(1u << hp.owner_log2, level_end - level_begin);
    if (deterministic)
        hipLaunchKernelGGL((hash_bwd_owner_kernel<kSliceLog2Det, 1024, true>), grid, dim3(1024), 0, as_stream(stream),
                           hp);
    else
        hipLaunchKernelGGL((hash_bwd_owner_kernel<kSliceLog2, kOwnerThreadsDefault, false>), grid,
                           dim3(kOwnerThreadsDefault), 0, as_stream(stream), hp);
    NERF_CHECK_LAUNCH("hash_encode_bwd_owner");
    return NERF_OK;
}

extern "C" int nerf_hash_encode_bwd_owner_range(int n_levels, int level_begin, int level_end, int log2_T,
                                                int64_t n_chunks, int64_t chunk_capacity, float* const* d_dtables,
                                                int deterministic, void* d_workspace, size_t workspace_bytes,
                                                void* stream) {
    return nerf_hash_encode_bwd_owner_step(n_levels, level_begin, level_end, log2_T, n_chunks, chunk_capacity,
                                           d_dtables, deterministic, d_workspace, workspace_bytes, nullptr, stream);
}

extern "C" int nerf_hash_bwd_entry_count(int n_levels, int log2_T, int64_t n_chunks, int64_t chunk_capacity,
                                         int deterministic, const void* d_workspace, size_t workspace_bytes,
                                         unsigned long long* d_count, void* stream) {
    HashGradParams hp{};
    const int rc = bin_layout("hash_bwd_entry_count", n_levels, log2_T, chunk_capacity, deterministic & 1,
                              const_cast<void*>(d_workspace), workspace_bytes, hp);
    if (rc) return rc;
    NERF_REQUIRE(n_chunks >= 0 && n_chunks <= chunk_capacity && d_count, "hash_bwd_entry_count: n_chunks %lld of %lld",
                 (long long)n_chunks, (long long)chunk_capacity);
    hipLaunchKernelGGL(bin_entry_count_kernel, dim3(1), dim3(1024), 0, as_stream(stream), hp.bin_seg,
                       (int64_t)1 << hp.owner_log2, (int64_t)hp.chunk_stride, (int)n_chunks, n_levels, d_count);
    NERF_CHECK_LAUNCH("hash_bwd_entry_count");
    return NERF_OK;
}

extern "C" int nerf_hash_encode_bwd_owner(int n_levels, int log2_T, int64_t n_chunks, int64_t chunk_capacity,
                                          float* const* d_dtables, int deterministic, void* d_workspace,
                                          size_t workspace_bytes, void* stream) {
    return nerf_hash_encode_bwd_owner_range(n_levels, 0, n_levels, log2_T, n_chunks, chunk_capacity, d_dtables,
                                            deterministic, d_workspace, workspace_bytes, stream);
}

// No workspace: coalesced memory-side float atomics (never deterministic).
extern "C" int nerf_hash_encode_bwd(const float* d_xyz, int64_t n_points, const float* bbox_min3,
                                    const float* bbox_max3, const float* level_res, int n_levels, int log2_T,
                                    const float* d_dfeat, int64_t feat_stride_point, int64_t feat_stride_level,
                                    float* const* d_dtables, void* stream) {
    NERF_REQUIRE(n_points >= 0, "hash_encode_bwd: n_points < 0");
    NERF_REQUIRE(n_levels >= 1 && n_levels <= NERF_MAX_LEVELS, "hash_encode_bwd: n_levels %d", n_levels);
    NERF_REQUIRE(log2_T >= 1 && log2_T <= 30, "hash_encode_bwd: log2_T %d", log2_T);
    NERF_REQUIRE((n_points == 0 || (d_xyz && d_dfeat)) && d_dtables && level_res && bbox_min3 && bbox_max3, "hash_encode_bwd: null arg");
    if (n_points == 0) return NERF_OK;
    HashGradParams hp{};
    for (int l = 0; l < n_levels; ++l) {
        NERF_REQUIRE(d_dtables[l], "hash_encode_bwd: grad table %d is null", l);
        hp.dtables[l] = d_dtables[l];
    }
    for (int a = 0; a < 3; ++a) { hp.bmin[a] = bbox_min3[a]; hp.bmax[a] = bbox_max3[a]; }
    hp.fastdiv = fill_cells(hp.cell, hp.rcell, bbox_min3, bbox_max3, level_res, n_levels) ? 1u : 0u;
    hp.mask = (uint32_t)((1u << log2_T) - 1u);
    hipLaunchKernelGGL((hash_encode_bwd_kernel<1, 256>), dim3(blocks_for(n_points, 256), n_levels), dim3(256), 0,
                       as_stream(stream), d_xyz, n_points, hp, d_dfeat, feat_stride_point, feat_stride_level,
                       BinRows{nullptr, nullptr, nullptr, 0, 0, nullptr});
    NERF_CHECK_LAUNCH("hash_encode_bwd");
    return NERF_OK;
}

// Binned path in one call: bin chunks [0, n) then the owner pass over them. A NULL workspace (or a
// log2_T without a binned path and deterministic == 0) falls back to nerf_hash_encode_bwd.
extern "C" int nerf_hash_encode_bwd_ws(const float* d_xyz, int64_t n_points, const float* bbox_min3,
                                       const float* bbox_max3, const float* level_res, int n_levels, int log2_T,
                                       const float* d_dfeat, int64_t feat_stride_point, int64_t feat_stride_level,
                                       float* const* d_dtables, int deterministic, void* d_workspace,
                                       size_t workspace_bytes, void* stream) {
    NERF_REQUIRE(n_points >= 0, "hash_encode_bwd: n_points < 0");
    NERF_REQUIRE(n_levels >= 1 && n_levels <= NERF_MAX_LEVELS, "hash_encode_bwd: n_levels %d", n_levels);
    NERF_REQUIRE(log2_T >= 1 && log2_T <= 30, "hash_encode_bwd: log2_T %d", log2_T);
    NERF_REQUIRE(d_dtables && level_res && bbox_min3 && bbox_max3, "hash_encode_bwd: null arg");
    for (int l = 0; l < n_levels; ++l) NERF_REQUIRE(d_dtables[l], "hash_encode_bwd: grad table %d is null", l);
    if (n_points == 0) return NERF_OK;
    BinPlan B{};
    const bool binned = d_workspace != nullptr && n_levels >= 1 && n_levels <= NERF_MAX_LEVELS &&
                        make_bin_plan(n_levels, log2_T, n_points, B, deterministic != 0);
    if (!binned) {
        NERF_REQUIRE(!deterministic, "hash_encode_bwd: the deterministic mode needs the binned path (a workspace of "
                                     "nerf_hash_encode_bwd_workspace_bytes(L, log2_T, P, 1) > 0 bytes)");
        return nerf_hash_encode_bwd(d_xyz, n_points, bbox_min3, bbox_max3, level_res, n_levels, log2_T, d_dfeat,
                                    feat_stride_point, feat_stride_level, d_dtables, stream);
    }
    const int64_t nch = (n_points + kChunkPts - 1) / kChunkPts;
    int rc = nerf_hash_encode_bwd_bin(d_xyz, n_points, bbox_min3, bbox_max3, level_res, n_levels, log2_T, d_dfeat,
                                      feat_stride_point, feat_stride_level, 0, nch, deterministic, d_workspace,
                                      workspace_bytes, stream);
    if (rc) return rc;
    return nerf_hash_encode_bwd_owner(n_levels, log2_T, nch, nch, d_dtables, deterministic, d_workspace,
                                      workspace_bytes, stream);
}
