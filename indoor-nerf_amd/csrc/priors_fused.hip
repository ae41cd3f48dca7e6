// Structural priors of the ScanNet configuration on the device, without host synchronisation, so
// the training iteration that includes them can be captured in a HIP graph.
//
// combine_structural_losses_v2 (PocketNeRF/structural_priors.py:374-451) with its parts
//   SemanticPlaneDetector.detect_planes            :86-155  (floor / wall masks; the wall clusters
//                                                            are logging only and not computed)
//   ManhattanFrameEstimator.estimate_frame         :16-45   (10-round spherical k-means :48-77,
//                                                            frame = U @ V of svd(centres^T))
//   manhattan_sdf_loss                             :194-256
//   structured_planarity_loss                      :259-318
//   spatial_normal_consistency_loss                :321-371
// and its backward (the reference's autograd graph: through F.normalize, the k-means means, the
// 3x3 SVD and the det flip). Every data-dependent branch of the reference (`if n_floor > 50`, ...)
// is evaluated on the device from block-wide counts; a term whose condition fails contributes 0.
//
// Three single-workgroup launches (N <= 8192 rays, one 1024-thread block):
//   priors_prep_kernel : normals -> masks, counts, k-means (assignments of every round kept for the
//                        backward);
//   priors_loss_kernel : (device mode) the 3x3 SVD of the centres on one thread (fp64 registers, no
//                        scratch at this kernel's 70 VGPRs), frame, the three losses, their sum;
//   priors_bwd_kernel  : d depth, d normals from d loss.
// With pixel coordinates the loss launch stops after the consistency queries: the nearest-pixel
// search runs one block per query (priors_nearest_kernel) and priors_loss_tail_kernel finishes.
// Randomness: the reference draws torch.randn (k-means init), torch.randperm (planarity pairs) and
// torch.randint (consistency queries). Replay mode takes those draws as inputs (the Python layer
// makes them with torch's generators in the reference's order); device mode draws them from
// Philox (seed, offset) — randperm as a sort of the class members by random keys (bitonic, LDS).
// The SVD: device mode computes it here (Jacobi on A^T A in fp64, singular values descending, each
// V column's largest-magnitude component made positive); replay mode takes U, S, V from the host
// (torch.svd, LAPACK), because the frame U @ V depends on the singular-vector sign convention.
#include "common.h"

namespace nerf {

constexpr int kPT = 1024;                  // threads per block
constexpr int kPriorsMaxRays = NERF_PRIORS_MAX_RAYS;
constexpr int kCapPairs[3] = {100, 100, 50};
constexpr float kClassScale[3] = {2.0f, 1.5f, 0.1f};
constexpr int kMaxCons = 200;
constexpr int kSelSeg = 512;               // selected keys per class (>= 2 x the largest pair cap)
static_assert(kSelSeg >= 2 * 100 && (kSelSeg & (kSelSeg - 1)) == 0, "segment");

// Device state shared by the three launches (lives at the start of the workspace).
struct PriorsState {
    int n_stable, n_floor, n_wall, n_other, n_keep, n_sure, kmeans, flip;
    int pair_n[3], n_cons, pad0, pad1;
    float M;                  // Manhattan total before the clamp
    float parts[7];           // floor, wall, general, manhattan, planarity, consistency, total
    float centres[9];         // final k-means centres (rows)
    float means[9];           // the mean vector each centre was last normalised from
    int centre_iter[3];       // round of that update (-1: still the random init)
    int centre_count[3];
    float U[9], S[3], V[9];   // svd(centres^T) = U diag(S) V^T
    float frame[9];           // U @ V, last column negated when det < 0
    int pair_a[250], pair_b[250];
    int idx1[kMaxCons], idx2[kMaxCons];
    float dist[kMaxCons];
};

struct PriorsArgs {
    const float* depth;       // [N]
    const float* normals;     // [N, 3]
    const float* coords;      // [N, 2] or null (sequential-neighbour fallback)
    int N;
    int use_m, use_p, use_c;  // which weights the caller's dict holds
    float w_m, w_p, w_c;
    const float* d_scale;     // optional device multiplier of the three weights (the ramp), null = 1
    float conf_thr, normal_thr;
    // replay inputs (null = draw on the device)
    const float* centres0;    // [3,3] torch.randn
    const int32_t* perm;      // [3][2 * cap] randperm positions, first 2 n_pairs used per class
    const int32_t* idx1;      // [n_cons] torch.randint
    const float* usv;         // [21] U (3x3), S (3), V (3x3) from the host SVD (replay mode)
    uint64_t seed, offset;
    const uint64_t* d_rng;
    PriorsState* st;
    uint8_t* cls;             // [N] bit0 floor, bit1 wall, bit2 stable, bit3 kept by the frame estimator
    int8_t* assign;           // [10][N] k-means assignment per round (-1: not kept)
    int32_t* members;         // [3][N] class members in index order
    float* loss;              // [1]
    const float* addend;      // loss: optional [1] added to the total in the loss word (the iteration's other losses)
    float* parts_out;         // loss: optional [7] copy of PriorsState::parts
    const float* d_loss;      // bwd: [1] upstream gradient
    float* d_depth;           // bwd: [N]
    float* d_normals;         // bwd: [N, 3]
};

__device__ __forceinline__ void rng_of(const PriorsArgs& a, uint64_t& s, uint64_t& o) {
    s = a.d_rng ? a.d_rng[0] : a.seed;
    o = a.d_rng ? a.d_rng[1] : a.offset;
}

// ---- block-wide reductions (1024 threads = 16 waves) -----------------------------------------
template <typename T>
__device__ T block_sum(T v, T* red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    T t = 0;
    for (int k = 0; k < kPT / 64; ++k) t += red[k];   // same order in every thread
    return t;
}

// wave64 total through DPP (row_shr 1/2/4/8 scan, then row_bcast 15/31: lane 63 holds the sum),
// read back as a wave-uniform value: no LDS crossbar and no per-step lane-address registers
__device__ __forceinline__ float wave_total(float x) {
    x += dpp_move<0x111, 0xF>(x);
    x += dpp_move<0x112, 0xF>(x);
    x += dpp_move<0x114, 0xF>(x);
    x += dpp_move<0x118, 0xF>(x);
    x += dpp_move<0x142, 0xA>(x);
    x += dpp_move<0x143, 0xC>(x);
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63));
}

// K sums at once (two barriers instead of two per sum): red holds 16 x K + K floats; thread k < K
// adds the 16 wave totals of value k, then every thread reads the K block totals
template <int K>
__device__ void block_sum_vec(float (&v)[K], float* red) {
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = wave_total(v[k]);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int k = 0; k < K; ++k) red[w * K + k] = v[k];
    __syncthreads();
    if (threadIdx.x < K) {
        float t = 0.f;
        for (int j = 0; j < kPT / 64; ++j) t += red[j * K + threadIdx.x];
        red[16 * K + threadIdx.x] = t;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = red[16 * K + k];
}

// exclusive prefix of a 0/1 flag over the block's ray range [base, base + kPT), + block total
__device__ int block_excl_scan(int f, int* red, int& total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t b = __ballot(f);
    const int in_wave = __popcll(b & ((1ull << lane) - 1ull));
    __syncthreads();
    if (lane == 0) red[w] = __popcll(b);
    __syncthreads();
    int before = 0;
    total = 0;
    for (int k = 0; k < kPT / 64; ++k) {
        before += k < w ? red[k] : 0;
        total += red[k];
    }
    return before + in_wave;
}

// F.normalize(x, dim=-1): x / max(||x||, 1e-12), the norm as torch.linalg.vector_norm (fp32)
__device__ __forceinline__ float norm3(float x, float y, float z) { return sqrtf((x * x + y * y) + z * z); }

__device__ __forceinline__ void load_nz(const PriorsArgs& a, int i, float (&n)[3], float& len) {
    const float x = a.normals[3 * i], y = a.normals[3 * i + 1], z = a.normals[3 * i + 2];
    len = norm3(x, y, z);
    const float d = fmaxf(len, 1e-12f);
    n[0] = x / d; n[1] = y / d; n[2] = z / d;
}

__device__ __forceinline__ float dot3(const float* a, const float* b) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }

// ---- 3x3 SVD (device mode), fp64 -----------------------------------------------------------------
__device__ void svd3(const float* A_, float* U, float* S, float* V) {
    double A[3][3], B[3][3], Q[3][3];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) A[r][c] = A_[3 * r + c];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            B[r][c] = A[0][r] * A[0][c] + A[1][r] * A[1][c] + A[2][r] * A[2][c];
            Q[r][c] = r == c ? 1.0 : 0.0;
        }
    for (int sweep = 0; sweep < 30; ++sweep) {   // cyclic Jacobi on B = A^T A
        double off = fabs(B[0][1]) + fabs(B[0][2]) + fabs(B[1][2]);
        if (off < 1e-30) break;
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int q = p + 1; q < 3; ++q) {
                if (fabs(B[p][q]) < 1e-300) continue;
                const double th = (B[q][q] - B[p][p]) / (2.0 * B[p][q]);
                const double t = (th >= 0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
#pragma unroll
                for (int k = 0; k < 3; ++k) {   // B <- J^T B J
                    const double bkp = B[k][p], bkq = B[k][q];
                    B[k][p] = c * bkp - s * bkq;
                    B[k][q] = s * bkp + c * bkq;
                }
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const double bpk = B[p][k], bqk = B[q][k];
                    B[p][k] = c * bpk - s * bqk;
                    B[q][k] = s * bpk + c * bqk;
                }
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const double qkp = Q[k][p], qkq = Q[k][q];
                    Q[k][p] = c * qkp - s * qkq;
                    Q[k][q] = s * qkp + c * qkq;
                }
            }
    }
    // descending eigenvalues: a 3-element sorting network of column swaps (constant indices only,
    // so the matrices stay in registers)
    double e[3] = {B[0][0], B[1][1], B[2][2]};
    auto swapcol = [&](int i, int j) {
        const double t = e[i]; e[i] = e[j]; e[j] = t;
#pragma unroll
        for (int r = 0; r < 3; ++r) { const double q = Q[r][i]; Q[r][i] = Q[r][j]; Q[r][j] = q; }
    };
    if (e[1] > e[0]) swapcol(0, 1);
    if (e[2] > e[0]) swapcol(0, 2);
    if (e[2] > e[1]) swapcol(1, 2);
    double v[3][3], u[3][3], s[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double a0 = fabs(Q[0][k]), a1 = fabs(Q[1][k]), a2 = fabs(Q[2][k]);
        const double pick = (a0 >= a1 && a0 >= a2) ? Q[0][k] : (a1 >= a2 ? Q[1][k] : Q[2][k]);
        const double sg = pick < 0 ? -1.0 : 1.0;   // sign convention: largest |component| positive
#pragma unroll
        for (int r = 0; r < 3; ++r) v[r][k] = sg * Q[r][k];
        s[k] = sqrt(fmax(e[k], 0.0));
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
#pragma unroll
        for (int r = 0; r < 3; ++r) u[r][k] = A[r][0] * v[0][k] + A[r][1] * v[1][k] + A[r][2] * v[2][k];
        const double l = sqrt(u[0][k] * u[0][k] + u[1][k] * u[1][k] + u[2][k] * u[2][k]);
        if (s[k] > 1e-12 * fmax(s[0], 1e-300) && l > 0) {
            for (int r = 0; r < 3; ++r) u[r][k] /= l;
        } else {   // rank deficient: complete the basis (u_k orthogonal to the previous columns)
            double w[3];
            if (k == 2) {
                w[0] = u[1][0] * u[2][1] - u[2][0] * u[1][1];
                w[1] = u[2][0] * u[0][1] - u[0][0] * u[2][1];
                w[2] = u[0][0] * u[1][1] - u[1][0] * u[0][1];
            } else {   // any unit vector orthogonal to u_0
                const double e[3] = {fabs(u[0][0]) < 0.9 ? 1.0 : 0.0, fabs(u[0][0]) < 0.9 ? 0.0 : 1.0, 0.0};
                const double d = e[0] * u[0][0] + e[1] * u[1][0] + e[2] * u[2][0];
                for (int r = 0; r < 3; ++r) w[r] = e[r] - d * u[r][0];
            }
            const double wl = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
            for (int r = 0; r < 3; ++r) u[r][k] = w[r] / wl;
        }
    }
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            U[3 * r + c] = (float)u[r][c];
            V[3 * r + c] = (float)v[r][c];
        }
    for (int k = 0; k < 3; ++k) S[k] = (float)s[k];
}

// ================================================================ prep: masks, counts, k-means, SVD
__global__ void __launch_bounds__(kPT) priors_prep_kernel(PriorsArgs a) {
    __shared__ float s_red[17 * 12];
    __shared__ float s_c[9];
    extern __shared__ float s_nz[];   // [N][3] normalised normals: the 10 k-means rounds read them from LDS
    PriorsState& st = *a.st;
    const int N = a.N, tid = threadIdx.x;
    int ns = 0, nf = 0, nw = 0, nk = 0;
    for (int i = tid; i < N; i += kPT) {
        float n[3], len;
        load_nz(a, i, n, len);
        const bool stable = len > 0.1f;
        const float az = fabsf(n[2]);
        const bool fl = stable && az > a.normal_thr, wa = stable && az < 1.0f - a.normal_thr;
        const bool keep = len > a.conf_thr;
        a.cls[i] = (uint8_t)((fl ? 1 : 0) | (wa ? 2 : 0) | (stable ? 4 : 0) | (keep ? 8 : 0));
        s_nz[3 * i] = n[0]; s_nz[3 * i + 1] = n[1]; s_nz[3 * i + 2] = keep ? n[2] : NAN;   // NaN z: not kept
        ns += stable; nf += fl; nw += wa; nk += keep;
    }
    {
        float c4[4] = {(float)ns, (float)nf, (float)nw, (float)nk};
        block_sum_vec<4>(c4, s_red);
        ns = (int)c4[0]; nf = (int)c4[1]; nw = (int)c4[2]; nk = (int)c4[3];
    }
    if (ns < 10) {   // detect_planes: too few stable normals -> empty masks (:105-112)
        for (int i = tid; i < N; i += kPT) a.cls[i] &= (uint8_t)~3u;
        nf = nw = 0;
    }
    // frame estimator: < 20 confident or < 30 kept normals -> identity (:20-27)
    const bool run_km = nk >= 30;
    if (tid == 0) {
        st.n_stable = ns; st.n_floor = nf; st.n_wall = nw; st.n_other = N - nf - nw; st.n_keep = nk;
        st.kmeans = run_km ? 1 : 0;
        for (int k = 0; k < 3; ++k) { st.centre_iter[k] = -1; st.centre_count[k] = 0; }
    }
    if (!run_km) return;
    // k-means init: F.normalize(torch.randn(3, 3)) rows
    if (tid < 3) {
        float r[3];
        if (a.centres0) {
            for (int c = 0; c < 3; ++c) r[c] = a.centres0[3 * tid + c];
        } else {   // Box-Muller from Philox: normals 3 tid .. 3 tid + 2
            uint64_t sd, of;
            rng_of(a, sd, of);
            const U4 u0 = philox_uniform4(sd, of, 2 * tid), u1 = philox_uniform4(sd, of, 2 * tid + 1);
            const float uu[4] = {u0.x, u0.y, u0.z, u0.w}, vv[4] = {u1.x, u1.y, u1.z, u1.w};
            for (int c = 0; c < 3; ++c) {
                // v_cos_f32 takes revolutions: cos(2 pi v) without the full-range reduction of cosf
                const float m = sqrtf(-2.0f * __logf(fmaxf(uu[c], 1e-12f)));
                r[c] = m * __builtin_amdgcn_cosf(vv[c]);
            }
        }
        const float d = fmaxf(norm3(r[0], r[1], r[2]), 1e-12f);
        for (int c = 0; c < 3; ++c) s_c[3 * tid + c] = r[c] / d;
    }
    __syncthreads();
    for (int it = 0; it < 10; ++it) {
        float red[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};   // 9 coordinate sums + 3 counts (exact in fp32)
        const float c00 = s_c[0], c01 = s_c[1], c02 = s_c[2], c10 = s_c[3], c11 = s_c[4], c12 = s_c[5],
                    c20 = s_c[6], c21 = s_c[7], c22 = s_c[8];
        for (int i = tid; i < N; i += kPT) {
            const float x = s_nz[3 * i], y = s_nz[3 * i + 1], z = s_nz[3 * i + 2];
            int8_t asg = -1;
            if (z == z) {   // kept
                const float d0 = (x * c00 + y * c01) + z * c02, d1 = (x * c10 + y * c11) + z * c12,
                            d2 = (x * c20 + y * c21) + z * c22;
                asg = 0;   // torch.argmax: first maximum
                float best = d0;
                if (d1 > best) { best = d1; asg = 1; }
                if (d2 > best) asg = 2;
#pragma unroll
                for (int k = 0; k < 3; ++k)
                    if (asg == k) { red[3 * k] += x; red[3 * k + 1] += y; red[3 * k + 2] += z; red[9 + k] += 1.f; }
            }
            a.assign[(size_t)it * N + i] = asg;
        }
        // the 16 waves' partials to LDS; thread k < 3 alone adds centre k's four (in block_sum_vec's
        // order, the same bits) and updates it: two block barriers per round instead of five
#pragma unroll
        for (int k = 0; k < 12; ++k) red[k] = wave_total(red[k]);
        if ((tid & 63) == 0)
#pragma unroll
            for (int k = 0; k < 12; ++k) s_red[(tid >> 6) * 12 + k] = red[k];
        __syncthreads();
        if (tid < 3) {   // centre = F.normalize(mean); an empty cluster keeps its centre
            const int k = tid;
            const int col[4] = {3 * k, 3 * k + 1, 3 * k + 2, 9 + k};
            float t4[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float t = 0.f;
                for (int j = 0; j < kPT / 64; ++j) t += s_red[j * 12 + col[q]];
                t4[q] = t;
            }
            if (t4[3] > 0.f) {
                const float m[3] = {t4[0] / t4[3], t4[1] / t4[3], t4[2] / t4[3]};
                const float d = fmaxf(norm3(m[0], m[1], m[2]), 1e-12f);
                for (int c = 0; c < 3; ++c) {
                    s_c[3 * k + c] = m[c] / d;
                    st.means[3 * k + c] = m[c];
                }
                st.centre_iter[k] = it;
                st.centre_count[k] = (int)t4[3];
            }
        }
        __syncthreads();
    }
    if (tid < 9) st.centres[tid] = s_c[tid];
}

// ---- bitonic sort of up to 8192 64-bit keys in LDS (device-mode randperm) ------------------------
// A stage of stride <= 64 pairs keys inside 128-key runs, and thread t's pairs lie in run t >> 6 (and
// t >> 6 + 16, ... for t + kPT): every wave touches only its own runs, so such a stage after another
// one needs a wave barrier, not a block barrier (4,096 keys: 15 block barriers instead of 78; the same
// compare-swaps, so the same order bit for bit).
// seg < M: each seg-key segment sorted ascending on its own (the merge directions of the last stage
// all ascending), the same network as a sort of seg keys per segment.
__device__ void bitonic_sort(uint64_t* k, int M, int seg) {
    int prev = 1 << 30;   // stride of the previous stage (the first stage follows the keys' stores)
    for (int size = 2; size <= seg; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            if (stride >= 128 || prev >= 128) {
                __syncthreads();
            } else {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            prev = stride;
            for (int t = threadIdx.x; t < M / 2; t += kPT) {
                const int lo = 2 * t - (t & (stride - 1));
                const int hi = lo + stride;
                const bool up = size == seg || (lo & size) == 0;
                const uint64_t x = k[lo], y = k[hi];
                if ((x > y) == up) { k[lo] = y; k[hi] = x; }
            }
        }
    __syncthreads();
}

// ================================================================ losses
// normal consistency over the ncons (idx1, idx2, dist) triples of st, then the total, the loss word
// (+ the caller's addend) and the parts; every thread of the block calls it
__device__ void consistency_and_total(const PriorsArgs& a, PriorsState& st, int ncons, float scale, float mloss,
                                      float ploss, float pf, float pw, float pg, float* s_red) {
    const bool xy = a.coords != nullptr;
    float cs = 0.f;
    for (int q = threadIdx.x; q < ncons; q += kPT) {
        float n1[3], n2[3], l1, l2;
        const int i1 = st.idx1[q], i2 = st.idx2[q];
        load_nz(a, i1, n1, l1);
        load_nz(a, i2, n2, l2);
        const float dsim = expf(-fabsf(a.depth[i1] - a.depth[i2]));
        const float wq = xy ? expf(-st.dist[q] * 0.1f) * dsim : dsim;
        cs += wq * (1.0f - dot3(n1, n2));
    }
    cs = block_sum(cs, s_red);
    const float closs = (a.use_c && ncons > 0) ? a.w_c * scale * (cs / (float)ncons) : 0.f;
    if (threadIdx.x == 0) {
        const float total = ((0.f + mloss) + ploss) + closs;
        st.parts[5] = closs; st.parts[6] = total;
        *a.loss = a.addend ? *a.addend + total : total;   // the caller's `loss + total`, one fp32 add
        if (a.parts_out) {
            const float pv[7] = {pf, pw, pg, mloss, ploss, closs, total};
            for (int k = 0; k < 7; ++k) a.parts_out[k] = pv[k];
        }
    }
}

__global__ void __launch_bounds__(kPT) priors_loss_kernel(PriorsArgs a) {
    __shared__ float s_red[17 * 4];
    __shared__ int s_ired[16];
    __shared__ float s_f[9];
    __shared__ int s_cnt[3];
    __shared__ int s_hist[3 * 256];
    __shared__ int s_bin[3];
    extern __shared__ uint64_t s_keys[];   // device mode: max(M2, 4 x 512) sort keys
    PriorsState& st = *a.st;
    const int N = a.N, tid = threadIdx.x;
    const float scale = a.d_scale ? *a.d_scale : 1.0f;
    // ---- frame
    if (tid == 0) {
        float f[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        int flip = 0;
        if (st.kmeans) {
            if (!a.usv) {   // device mode: the SVD of A = centres^T (fp64 Jacobi) here, not a launch of its own
                float A[9];
                for (int r = 0; r < 3; ++r)
                    for (int c = 0; c < 3; ++c) A[3 * r + c] = st.centres[3 * c + r];
                svd3(A, st.U, st.S, st.V);
            } else {
                for (int k = 0; k < 9; ++k) { st.U[k] = a.usv[k]; st.V[k] = a.usv[12 + k]; }
                for (int k = 0; k < 3; ++k) st.S[k] = a.usv[9 + k];
            }
            for (int r = 0; r < 3; ++r)   // U @ V (the reference multiplies by torch.svd's V itself)
                for (int c = 0; c < 3; ++c)
                    f[3 * r + c] = (st.U[3 * r] * st.V[c] + st.U[3 * r + 1] * st.V[3 + c]) + st.U[3 * r + 2] * st.V[6 + c];
            const float det = f[0] * (f[4] * f[8] - f[5] * f[7]) - f[1] * (f[3] * f[8] - f[5] * f[6]) +
                              f[2] * (f[3] * f[7] - f[4] * f[6]);
            if (det < 0.f) {
                flip = 1;
                for (int r = 0; r < 3; ++r) f[3 * r + 2] = -f[3 * r + 2];
            }
        }
        for (int k = 0; k < 9; ++k) { st.frame[k] = f[k]; s_f[k] = f[k]; }
        st.flip = flip;
    }
    __syncthreads();
    // ---- Manhattan (:194-256)
    float sf = 0.f, sw = 0.f, sg = 0.f;
    int nsure = 0;
    for (int i = tid; i < N; i += kPT) {
        float n[3], len;
        load_nz(a, i, n, len);
        const uint8_t c = a.cls[i];
        float al[3];
        for (int k = 0; k < 3; ++k) al[k] = fabsf((n[0] * s_f[k] + n[1] * s_f[3 + k]) + n[2] * s_f[6 + k]);
        if (c & 1) sf += fminf(fmaxf(1.0f - al[2], 0.f), 1.f);
        if (c & 2) sw += fminf(fmaxf(1.0f - fmaxf(al[0], al[1]), 0.f), 1.f);
        const float best = fmaxf(fmaxf(al[0], al[1]), al[2]);
        if (best > 0.5f) { sg += fminf(fmaxf(1.0f - best, 0.f), 1.f); ++nsure; }
    }
    {
        float r4[4] = {sf, sw, sg, (float)nsure};
        block_sum_vec<4>(r4, s_red);
        sf = r4[0]; sw = r4[1]; sg = r4[2]; nsure = (int)r4[3];
    }
    float M = 0.f, pf = 0.f, pw = 0.f, pg = 0.f;
    if (st.n_floor > 50) { pf = sf / (float)st.n_floor; M = M + pf * 0.5f; }
    if (st.n_wall > 30) { pw = sw / (float)st.n_wall; M = M + pw * 0.3f; }
    if (nsure > 20) { pg = sg / (float)nsure; M = M + pg * 0.02f; }
    const float mloss = a.use_m ? a.w_m * scale * fminf(fmaxf(M, 0.f), 0.1f) : 0.f;
    // ---- planarity (:259-318): class members in index order, random pairs
    int ncls[3] = {st.n_floor, st.n_wall, st.n_other};
    if (a.perm) {   // replay: randperm positions index the class members in index order (torch.where)
        if (tid < 3) s_cnt[tid] = 0;
        for (int base = 0; base < N; base += kPT) {
            const int i = base + tid;
            const uint8_t c = i < N ? a.cls[i] : 0;
            for (int k = 0; k < 3; ++k) {
                const int f = i < N && (k == 2 ? (c & 3) == 0 : ((c >> k) & 1) != 0);
                int total;
                const int pos = block_excl_scan(f, s_ired, total);   // (synchronises before reading s_cnt)
                if (f) a.members[(size_t)k * N + s_cnt[k] + pos] = i;
                __syncthreads();
                if (tid == 0) s_cnt[k] += total;
            }
        }
    }
    __syncthreads();
    int npair[3];
    for (int k = 0; k < 3; ++k) {
        const bool on = N >= 10 && ncls[k] > 5 && ncls[k] > 1;
        npair[k] = on ? min(kCapPairs[k], ncls[k] / 2) : 0;
    }
    if (!a.perm && (npair[0] | npair[1] | npair[2])) {   // device randperm: members ordered by random key
        // key = class << 40 | 24 random bits << 14 | index; a class's pairs are the 2 npair smallest keys
        // of the class. Selected, then sorted: a histogram of the random bits' top 8 per class finds the
        // bin holding the (2 npair)-th smallest, the keys up to that bin (~2 npair + N / 256) go to a
        // 512-key segment per class, and the segments are sorted — the same keys in the same order as
        // the sort of all M2 keys (which remains the path when a segment would overflow).
        int M2 = 1;
        while (M2 < N) M2 <<= 1;
        uint64_t sd, of;
        rng_of(a, sd, of);
        auto key_of = [&](int i) -> uint64_t {
            const uint8_t c = a.cls[i];
            const uint64_t k = (c & 1) ? 0 : (c & 2) ? 1 : 2;
            const uint32_t r = (uint32_t)(philox_uniform(sd, of, 64 + (uint64_t)i) * 16777216.0f);
            return (k << 40) | ((uint64_t)r << 14) | (uint64_t)i;
        };
        for (int i = tid; i < 3 * 256; i += kPT) s_hist[i] = 0;
        if (tid < 3) s_cnt[tid] = 0;
        __syncthreads();
        for (int i = tid; i < N; i += kPT) {
            const uint64_t key = key_of(i);
            atomicAdd(&s_hist[(int)(key >> 40) * 256 + (int)((key >> 30) & 255)], 1);
        }
        __syncthreads();
        if (tid < 3 * 64) {   // wave k: the bin of class k's (2 npair)-th smallest key (-1: no pairs)
            const int k = tid >> 6, lane = tid & 63, need = 2 * npair[k];
            int c4[4], run = 0;
            for (int j = 0; j < 4; ++j) { c4[j] = s_hist[k * 256 + 4 * lane + j]; run += c4[j]; }
            int incl = run;   // inclusive scan of the lanes' 4-bin sums
            for (int o = 1; o < 64; o <<= 1) {
                const int v = __shfl_up(incl, o, 64);
                if (lane >= o) incl += v;
            }
            int below = incl - run, bin = 1 << 30;
            for (int j = 0; j < 4; ++j) {
                if (below < need && below + c4[j] >= need) bin = 4 * lane + j;
                below += c4[j];
            }
            for (int o = 32; o > 0; o >>= 1) bin = min(bin, __shfl_xor(bin, o, 64));
            if (lane == 0) s_bin[k] = need > 0 ? bin : -1;
        }
        __syncthreads();
        uint64_t* seg = s_keys;   // [4][512]: classes 0..2, the fourth all padding
        for (int i = tid; i < N; i += kPT) {
            const uint64_t key = key_of(i);
            const int k = (int)(key >> 40);
            if ((int)((key >> 30) & 255) <= s_bin[k]) {
                const int pos = atomicAdd(&s_cnt[k], 1);
                if (pos < kSelSeg) seg[k * kSelSeg + pos] = key;
            }
        }
        __syncthreads();
        const bool fits = s_cnt[0] <= kSelSeg && s_cnt[1] <= kSelSeg && s_cnt[2] <= kSelSeg;
        if (fits) {
            for (int i = tid; i < 4 * kSelSeg; i += kPT)
                if (i >= 3 * kSelSeg || (i & (kSelSeg - 1)) >= s_cnt[i / kSelSeg]) seg[i] = ~0ull;
            bitonic_sort(seg, 4 * kSelSeg, kSelSeg);
        } else {   // a bin too full for its segment: every key, one sort
            __syncthreads();
            for (int i = tid; i < M2; i += kPT) s_keys[i] = i < N ? key_of(i) : ~0ull;
            bitonic_sort(s_keys, M2, M2);
        }
        int off = 0, start = 0;   // sorted: class 0 (floor), 1 (wall), 2 (other), random order inside a class
        for (int k = 0; k < 3; ++k) {
            const int s0 = fits ? k * kSelSeg : start;
            for (int t = tid; t < npair[k]; t += kPT) {
                st.pair_a[off + t] = (int)(s_keys[s0 + t] & 0x3FFF);
                st.pair_b[off + t] = (int)(s_keys[s0 + npair[k] + t] & 0x3FFF);
            }
            off += kCapPairs[k];
            start += ncls[k];
        }
    } else if (a.perm) {
        int off = 0;
        for (int k = 0; k < 3; ++k) {
            for (int t = tid; t < npair[k]; t += kPT) {
                st.pair_a[off + t] = a.members[(size_t)k * N + a.perm[2 * off + t]];
                st.pair_b[off + t] = a.members[(size_t)k * N + a.perm[2 * off + npair[k] + t]];
            }
            off += kCapPairs[k];
        }
    }
    __syncthreads();
    float ploss = 0.f;
    {
        int off = 0;
        float part[3];
        for (int k = 0; k < 3; ++k) {
            float s = 0.f;
            for (int t = tid; t < npair[k]; t += kPT)
                s += fabsf(a.depth[st.pair_a[off + t]] - a.depth[st.pair_b[off + t]]);
            part[k] = s;
            off += kCapPairs[k];
        }
        block_sum_vec<3>(part, s_red);
        float tot = 0.f;
        for (int k = 0; k < 3; ++k)
            if (npair[k] > 0) tot = tot + (part[k] / (float)npair[k]) * kClassScale[k];
        ploss = a.use_p ? a.w_p * scale * tot : 0.f;
    }
    // ---- normal consistency (:321-371)
    const bool xy = a.coords != nullptr;
    const int ncons = N < 10 ? 0 : (xy ? min(kMaxCons, N / 2) : min(100, N - 1));
    {
        uint64_t sd, of;
        rng_of(a, sd, of);
        for (int q = tid; q < ncons; q += kPT) {
            int i1;
            if (a.idx1) {
                i1 = a.idx1[q];
            } else {
                const int hi = xy ? N : N - 1;
                i1 = min((int)(philox_uniform(sd, of, 64 + (uint64_t)kPriorsMaxRays + q) * (float)hi), hi - 1);
            }
            st.idx1[q] = i1;
        }
    }
    __syncthreads();
    if (tid == 0) {   // the tail's inputs (priors_loss_tail_kernel reads them back with pixel coordinates)
        st.M = M;
        st.n_sure = nsure;
        st.pair_n[0] = npair[0]; st.pair_n[1] = npair[1]; st.pair_n[2] = npair[2];
        st.n_cons = ncons;
        st.parts[0] = pf; st.parts[1] = pw; st.parts[2] = pg;
        st.parts[3] = mloss; st.parts[4] = ploss;
    }
    if (xy) return;   // nearest pixels: priors_nearest_kernel (one block per query), then the tail
    for (int q = tid; q < ncons; q += kPT) { st.idx2[q] = st.idx1[q] + 1; st.dist[q] = 0.f; }
    __syncthreads();
    consistency_and_total(a, st, ncons, scale, mloss, ploss, pf, pw, pg, s_red);
}

// Pixel-coordinate mode (spatial_coords given, :333-346): the nearest other pixel of query q, one
// block per query over all N candidates (a single workgroup scanning 200 x N took ~90 us on one CU),
// the lowest index on ties (torch.argmin), the same comparisons as nerf_nearest_pixel.
__global__ void __launch_bounds__(256) priors_nearest_kernel(PriorsArgs a) {
    PriorsState& st = *a.st;
    const int q = blockIdx.x, N = a.N;
    if (q >= st.n_cons) return;
    const int self = st.idx1[q];
    const float qx = a.coords[2 * self], qy = a.coords[2 * self + 1];
    float best = INFINITY;
    int bi = N;
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
        const float dx = a.coords[2 * i] - qx, dy = a.coords[2 * i + 1] - qy;
        const float d2 = i == self ? INFINITY : dx * dx + dy * dy;
        if (d2 < best) { best = d2; bi = i; }   // strided ascending scan: first minimum per thread
    }
    for (int o = 32; o > 0; o >>= 1) {
        const float ob = __shfl_xor(best, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ob < best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    __shared__ float s_b[4];
    __shared__ int s_i[4];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { s_b[w] = best; s_i[w] = bi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < 4; ++k)
            if (s_b[k] < best || (s_b[k] == best && s_i[k] < bi)) { best = s_b[k]; bi = s_i[k]; }
        if (bi >= N) bi = self == 0 ? 1 : 0;
        st.idx2[q] = bi;
        st.dist[q] = sqrtf(best);
    }
}

__global__ void __launch_bounds__(kPT) priors_loss_tail_kernel(PriorsArgs a) {
    __shared__ float s_red[17 * 4];
    PriorsState& st = *a.st;
    const float scale = a.d_scale ? *a.d_scale : 1.0f;
    consistency_and_total(a, st, st.n_cons, scale, st.parts[3], st.parts[4], st.parts[0], st.parts[1], st.parts[2],
                          s_red);
}

// ================================================================ backward
// 3x3 helpers (row-major)
__device__ __forceinline__ void mm3(const double* A, const double* B, double* C) {
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) C[3 * r + c] = A[3 * r] * B[c] + A[3 * r + 1] * B[3 + c] + A[3 * r + 2] * B[6 + c];
}
__device__ __forceinline__ void tr3(const double* A, double* T) {
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) T[3 * c + r] = A[3 * r + c];
}

__global__ void __launch_bounds__(kPT) priors_bwd_kernel(PriorsArgs a) {
    extern __shared__ float s_g[];    // [N][4]: d nz (3), d depth
    __shared__ float s_red[17 * 9];
    __shared__ float s_gF[9];
    __shared__ float s_gmean[9];
    const PriorsState& st = *a.st;
    const int N = a.N, tid = threadIdx.x;
    const float g = *a.d_loss;
    const float scale = a.d_scale ? *a.d_scale : 1.0f;
    for (int i = tid; i < 4 * N; i += kPT) s_g[i] = 0.f;
    __syncthreads();
    // ---- Manhattan: d M = g w_m [0 <= M <= 0.1] (torch.clamp passes the gradient inclusively)
    const float gM = (a.use_m && st.M >= 0.f && st.M <= 0.1f) ? g * a.w_m * scale : 0.f;
    const float* f = st.frame;
    float gF[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (gM != 0.f) {
        const float cf = st.n_floor > 50 ? gM * 0.5f / (float)st.n_floor : 0.f;
        const float cw = st.n_wall > 30 ? gM * 0.3f / (float)st.n_wall : 0.f;
        const float cg = st.n_sure > 20 ? gM * 0.02f / (float)st.n_sure : 0.f;
        for (int i = tid; i < N; i += kPT) {
            float n[3], len;
            load_nz(a, i, n, len);
            const uint8_t c = a.cls[i];
            float d[3], al[3];
            for (int k = 0; k < 3; ++k) {
                d[k] = (n[0] * f[k] + n[1] * f[3 + k]) + n[2] * f[6 + k];
                al[k] = fabsf(d[k]);
            }
            auto sgn = [](float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); };
            float gd[3] = {0.f, 0.f, 0.f};   // d loss / d (n . f_k)
            if ((c & 1) && cf != 0.f) {
                const float v = 1.0f - al[2];
                if (v >= 0.f && v <= 1.f) gd[2] += -cf * sgn(d[2]);
            }
            if ((c & 2) && cw != 0.f) {
                const float mx = fmaxf(al[0], al[1]), v = 1.0f - mx;
                if (v >= 0.f && v <= 1.f) {   // torch.maximum: ties split the gradient
                    const float w0 = al[0] > al[1] ? 1.f : (al[0] == al[1] ? 0.5f : 0.f);
                    gd[0] += -cw * w0 * sgn(d[0]);
                    gd[1] += -cw * (1.f - w0) * sgn(d[1]);
                }
            }
            if (cg != 0.f) {
                int k = 0;   // torch.max(dim): the first maximum
                for (int j = 1; j < 3; ++j)
                    if (al[j] > al[k]) k = j;
                const float v = 1.0f - al[k];
                if (al[k] > 0.5f && v >= 0.f && v <= 1.f) gd[k] += -cg * sgn(d[k]);
            }
            for (int k = 0; k < 3; ++k) {
                if (gd[k] == 0.f) continue;
                for (int r = 0; r < 3; ++r) {
                    s_g[4 * i + r] += gd[k] * f[3 * r + k];
                    gF[3 * r + k] += gd[k] * n[r];
                }
            }
        }
    }
    block_sum_vec<9>(gF, s_red);
    // ---- through the frame: det flip, F = U V, svd backward, normalize, mean (single thread)
    if (tid == 0) {
        for (int k = 0; k < 9; ++k) s_gmean[k] = 0.f;
        if (st.kmeans && gM != 0.f) {
            double GF[9], U[9], V[9], Ut[9], Vt[9], gU[9], gV[9];
            for (int k = 0; k < 9; ++k) { GF[k] = gF[k]; U[k] = st.U[k]; V[k] = st.V[k]; }
            if (st.flip)
                for (int r = 0; r < 3; ++r) GF[3 * r + 2] = -GF[3 * r + 2];
            tr3(U, Ut);
            tr3(V, Vt);
            mm3(GF, Vt, gU);   // F = U V: dU = dF V^T, dV = U^T dF
            mm3(Ut, GF, gV);
            // A = U S V^T (square, full rank): dA = U [ (Fm o (U^T dU - dU^T U)) S + S (Fm o (V^T dV - dV^T V)) ] V^T
            double s[3] = {st.S[0], st.S[1], st.S[2]};
            double UtgU[9], gUtU[9], VtgV[9], gVtV[9], gUt[9], gVt[9];
            mm3(Ut, gU, UtgU);
            tr3(gU, gUt);
            mm3(gUt, U, gUtU);
            mm3(Vt, gV, VtgV);
            tr3(gV, gVt);
            mm3(gVt, V, gVtV);
            double inner[9];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) {
                    double Fm = 0.0;
                    if (i != j) {
                        const double den = s[j] * s[j] - s[i] * s[i];
                        Fm = fabs(den) > 1e-30 ? 1.0 / den : 0.0;
                    }
                    inner[3 * i + j] = Fm * (UtgU[3 * i + j] - gUtU[3 * i + j]) * s[j] +
                                       s[i] * Fm * (VtgV[3 * i + j] - gVtV[3 * i + j]);
                }
            double t1[9], gA[9];
            mm3(U, inner, t1);
            mm3(t1, Vt, gA);
            // A = centres^T: d centres[k][c] = dA[c][k]; centre = m / max(|m|, eps)
            for (int k = 0; k < 3; ++k) {
                if (st.centre_iter[k] < 0) continue;
                const double gc[3] = {gA[k], gA[3 + k], gA[6 + k]};
                const double m[3] = {st.means[3 * k], st.means[3 * k + 1], st.means[3 * k + 2]};
                const double len = sqrt(m[0] * m[0] + m[1] * m[1] + m[2] * m[2]);
                double gm[3];
                if (len > 1e-12) {
                    const double c[3] = {m[0] / len, m[1] / len, m[2] / len};
                    const double dc = c[0] * gc[0] + c[1] * gc[1] + c[2] * gc[2];
                    for (int r = 0; r < 3; ++r) gm[r] = (gc[r] - c[r] * dc) / len;
                } else {
                    for (int r = 0; r < 3; ++r) gm[r] = gc[r] / 1e-12;
                }
                for (int r = 0; r < 3; ++r) s_gmean[3 * k + r] = (float)(gm[r] / (double)st.centre_count[k]);
            }
        }
    }
    __syncthreads();
    if (st.kmeans && gM != 0.f) {   // mean backward: every member of the centre's last update round
        for (int i = tid; i < N; i += kPT) {
            for (int k = 0; k < 3; ++k) {
                const int it = st.centre_iter[k];
                if (it >= 0 && a.assign[(size_t)it * N + i] == k)
                    for (int r = 0; r < 3; ++r) s_g[4 * i + r] += s_gmean[3 * k + r];
            }
        }
    }
    __syncthreads();
    // ---- planarity: d |d_a - d_b| / n_pairs x class scale
    if (a.use_p) {
        int off = 0;
        for (int k = 0; k < 3; ++k) {
            const int np = st.pair_n[k];
            const float c = np > 0 ? g * a.w_p * scale * kClassScale[k] / (float)np : 0.f;
            for (int t = tid; t < np; t += kPT) {
                const int ia = st.pair_a[off + t], ib = st.pair_b[off + t];
                const float d = a.depth[ia] - a.depth[ib];
                const float sg = d > 0.f ? c : (d < 0.f ? -c : 0.f);
                atomicAdd(&s_g[4 * ia + 3], sg);
                atomicAdd(&s_g[4 * ib + 3], -sg);
            }
            off += kCapPairs[k];
        }
    }
    // ---- consistency: mean over queries of w (1 - n1 . n2)
    if (a.use_c && st.n_cons > 0) {
        const bool xy = a.coords != nullptr;
        const float c = g * a.w_c * scale / (float)st.n_cons;
        for (int q = tid; q < st.n_cons; q += kPT) {
            const int i1 = st.idx1[q], i2 = st.idx2[q];
            float n1[3], n2[3], l1, l2;
            load_nz(a, i1, n1, l1);
            load_nz(a, i2, n2, l2);
            const float dd = a.depth[i1] - a.depth[i2];
            const float dsim = expf(-fabsf(dd));
            const float sw = xy ? expf(-st.dist[q] * 0.1f) : 1.f;
            const float wq = sw * dsim, cosv = dot3(n1, n2);
            const float gw = c * (1.0f - cosv);                    // d loss / d w
            const float gdd = gw * sw * dsim * (dd > 0.f ? -1.f : (dd < 0.f ? 1.f : 0.f));   // through exp(-|dd|)
            atomicAdd(&s_g[4 * i1 + 3], gdd);
            atomicAdd(&s_g[4 * i2 + 3], -gdd);
            for (int r = 0; r < 3; ++r) {
                atomicAdd(&s_g[4 * i1 + r], -c * wq * n2[r]);
                atomicAdd(&s_g[4 * i2 + r], -c * wq * n1[r]);
            }
        }
    }
    __syncthreads();
    // ---- F.normalize backward and outputs
    for (int i = tid; i < N; i += kPT) {
        float n[3], len;
        load_nz(a, i, n, len);
        const float gx = s_g[4 * i], gy = s_g[4 * i + 1], gz = s_g[4 * i + 2];
        float o[3];
        if (len > 1e-12f) {
            const float dp = (n[0] * gx + n[1] * gy) + n[2] * gz;
            o[0] = (gx - n[0] * dp) / len;
            o[1] = (gy - n[1] * dp) / len;
            o[2] = (gz - n[2] * dp) / len;
        } else {
            o[0] = gx / 1e-12f; o[1] = gy / 1e-12f; o[2] = gz / 1e-12f;
        }
        a.d_normals[3 * i] = o[0];
        a.d_normals[3 * i + 1] = o[1];
        a.d_normals[3 * i + 2] = o[2];
        a.d_depth[i] = s_g[4 * i + 3];
    }
}

}  // namespace nerf

using namespace nerf;

// workspace: PriorsState | cls [N] | assign [10][N] | members [3][N]
static size_t priors_ws_bytes(int64_t n) {
    auto up = [](size_t v) { return (v + 255) & ~(size_t)255; };
    return up(sizeof(PriorsState)) + up((size_t)n) + up((size_t)10 * n) + up((size_t)3 * n * sizeof(int32_t));
}

extern "C" size_t nerf_priors_workspace_bytes(int64_t n_rays) {
    return n_rays < 1 || n_rays > kPriorsMaxRays ? 0 : priors_ws_bytes(n_rays);
}

static int priors_args(PriorsArgs& a, const float* d_depth, const float* d_normals, const float* d_coords, int64_t n,
                       const nerf_priors_config* cfg, void* d_ws, size_t ws_bytes) {
    NERF_REQUIRE(n >= 1 && n <= kPriorsMaxRays, "priors: %lld rays (1..%d)", (long long)n, kPriorsMaxRays);
    NERF_REQUIRE(d_depth && d_normals && cfg && d_ws, "priors: null arg");
    NERF_REQUIRE(cfg->perm || cfg->normal_threshold >= 0.5f,
                 "priors: device-drawn pairs need disjoint floor / wall classes (normal_threshold >= 0.5)");
    NERF_REQUIRE(ws_bytes >= priors_ws_bytes(n), "priors: workspace %zu B < %zu B", ws_bytes, priors_ws_bytes(n));
    auto up = [](size_t v) { return (v + 255) & ~(size_t)255; };
    char* w = static_cast<char*>(d_ws);
    a.depth = d_depth; a.normals = d_normals; a.coords = d_coords; a.N = (int)n;
    a.use_m = cfg->use_manhattan; a.use_p = cfg->use_planarity; a.use_c = cfg->use_consistency;
    a.w_m = cfg->w_manhattan; a.w_p = cfg->w_planarity; a.w_c = cfg->w_consistency;
    a.d_scale = cfg->d_scale;
    a.conf_thr = cfg->confidence_threshold; a.normal_thr = cfg->normal_threshold;
    a.centres0 = cfg->centres0; a.perm = cfg->perm; a.idx1 = cfg->idx1; a.usv = cfg->usv;
    a.seed = cfg->seed; a.offset = cfg->offset; a.d_rng = reinterpret_cast<const uint64_t*>(cfg->d_rng);
    a.st = reinterpret_cast<PriorsState*>(w);
    w += up(sizeof(PriorsState));
    a.cls = reinterpret_cast<uint8_t*>(w);
    w += up((size_t)n);
    a.assign = reinterpret_cast<int8_t*>(w);
    w += up((size_t)10 * n);
    a.members = reinterpret_cast<int32_t*>(w);
    return NERF_OK;
}

extern "C" int nerf_priors_prep(const float* d_depth, const float* d_normals, const float* d_coords, int64_t n_rays,
                                const nerf_priors_config* cfg, void* d_workspace, size_t workspace_bytes,
                                float* d_centres_out, void* stream) {
    PriorsArgs a{};
    int rc = priors_args(a, d_depth, d_normals, d_coords, n_rays, cfg, d_workspace, workspace_bytes);
    if (rc) return rc;
    hipLaunchKernelGGL(priors_prep_kernel, dim3(1), dim3(kPT), (size_t)3 * n_rays * sizeof(float), as_stream(stream), a);
    NERF_CHECK_LAUNCH("priors_prep");
    if (d_centres_out) {   // the final k-means centres [3,3] (rows), for the host SVD of replay mode
        const hipError_t e = hipMemcpyAsync(d_centres_out, a.st->centres, 9 * sizeof(float), hipMemcpyDeviceToDevice,
                                            as_stream(stream));
        if (e != hipSuccess) {
            set_error("priors_prep: hipMemcpyAsync failed");
            return NERF_E_LAUNCH;
        }
    }
    return NERF_OK;
}

extern "C" int nerf_priors_loss_add(const float* d_depth, const float* d_normals, const float* d_coords,
                                    int64_t n_rays, const nerf_priors_config* cfg, void* d_workspace,
                                    size_t workspace_bytes, const float* d_addend, float* d_loss, float* d_parts,
                                    void* stream) {
    PriorsArgs a{};
    int rc = priors_args(a, d_depth, d_normals, d_coords, n_rays, cfg, d_workspace, workspace_bytes);
    if (rc) return rc;
    NERF_REQUIRE(d_loss, "priors_loss: null loss");
    a.loss = d_loss;
    a.addend = d_addend;
    a.parts_out = d_parts;   // floor, wall, general, manhattan, planarity, consistency, total: stored by the kernel
    int M2 = 1;
    while (M2 < n_rays) M2 <<= 1;
    const size_t lds = cfg->perm ? 0 : (size_t)std::max(M2, 4 * kSelSeg) * sizeof(uint64_t);
    hipLaunchKernelGGL(priors_loss_kernel, dim3(1), dim3(kPT), lds, as_stream(stream), a);
    NERF_CHECK_LAUNCH("priors_loss");
    if (d_coords) {   // the nearest-pixel queries (n_cons <= kMaxCons, read by each block) and the tail
        hipLaunchKernelGGL(priors_nearest_kernel, dim3(kMaxCons), dim3(256), 0, as_stream(stream), a);
        NERF_CHECK_LAUNCH("priors_loss (nearest)");
        hipLaunchKernelGGL(priors_loss_tail_kernel, dim3(1), dim3(kPT), 0, as_stream(stream), a);
        NERF_CHECK_LAUNCH("priors_loss (tail)");
    }
    return NERF_OK;
}

extern "C" int nerf_priors_loss(const float* d_depth, const float* d_normals, const float* d_coords, int64_t n_rays,
                                const nerf_priors_config* cfg, void* d_workspace, size_t workspace_bytes,
                                float* d_loss, float* d_parts, void* stream) {
    return nerf_priors_loss_add(d_depth, d_normals, d_coords, n_rays, cfg, d_workspace, workspace_bytes, nullptr,
                                d_loss, d_parts, stream);
}

extern "C" int nerf_priors_bwd(const float* d_depth, const float* d_normals, const float* d_coords, int64_t n_rays,
                               const nerf_priors_config* cfg, void* d_workspace, size_t workspace_bytes,
                               const float* d_grad_loss, float* d_grad_depth, float* d_grad_normals, void* stream) {
    PriorsArgs a{};
    int rc = priors_args(a, d_depth, d_normals, d_coords, n_rays, cfg, d_workspace, workspace_bytes);
    if (rc) return rc;
    NERF_REQUIRE(d_grad_loss && d_grad_depth && d_grad_normals, "priors_bwd: null arg");
    a.d_loss = d_grad_loss;
    a.d_depth = d_grad_depth;
    a.d_normals = d_grad_normals;
    hipLaunchKernelGGL(priors_bwd_kernel, dim3(1), dim3(kPT), (size_t)4 * n_rays * sizeof(float), as_stream(stream), a);
    NERF_CHECK_LAUNCH("priors_bwd");
    return NERF_OK;
}
