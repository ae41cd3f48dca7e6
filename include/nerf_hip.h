/*
 * nerf_hip.h — C ABI of libnerfhip.so, the MI355X (gfx950) kernels of the render_rays hot path.
 *
 * Boundary: the reference is pure PyTorch; every function below replaces one
 * implicit eager-op sequence of its Python API. The Python host layer (indoor-nerf_amd/, imported
 * as indoor_nerf_amd) binds these with ctypes and keeps the reference's module/function names.
 *
 * Conventions
 *   - Every pointer argument named d_* is DEVICE memory, caller-owned, contiguous, float32 unless
 *     typed otherwise; outputs are caller-allocated. The library allocates nothing (except
 *     nerf_host_ring_alloc's host ring) and keeps no state between calls (reentrant; safe under
 *     stream capture).
 *   - Host arrays (level resolutions, table pointer lists, bbox) are read during the call only.
 *   - `stream` is a hipStream_t passed as void* (torch.cuda.current_stream().cuda_stream).
 *   - Return 0 on success, else a NERF_E_* code; nerf_last_error() gives the message (per thread).
 *   - Empty batches (0 rays / points) return 0 without launching, and their per-ray / per-point
 *     buffers may be NULL (torch's empty tensors have data_ptr 0), as the reference's torch ops
 *     accept empty tensors; weights, tables and host arrays are still validated.
 *   - Random draws: a NULL d_u* argument means "draw in-kernel" from Philox4x32-10 keyed by
 *     (seed, offset); a non-NULL one supplies the uniforms (the reference's pytest=True path).
 *     A non-NULL d_rng (device uint64[2]) overrides (seed, offset) — used when a whole training
 *     step is captured in a HIP graph and every replay must draw new numbers.
 *   - Likewise nerf_tv_* take the cuboid corners from d_min_vertex (device int64[L][3]) and
 *     nerf_radam_step its per-step scalars from d_coef (device float[n][4]) when non-NULL.
 */
#ifndef NERF_HIP_H
#define NERF_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NERF_OK 0
#define NERF_E_ARG 1        /* bad shape / size / null pointer            */
#define NERF_E_LAUNCH 2     /* hipLaunchKernel / hipGetLastError failed     */
#define NERF_E_UNSUPPORTED 3

#define NERF_MAX_LEVELS 16

const char* nerf_last_error(void);
int nerf_abi_version(void);

/* ---- numerical check (render_rays' DEBUG test, run_nerf.py:545-547) ----------------------------
 * d_counts[t] = number of NaN/Inf values among the sizes[t] floats at d_ptrs[t] (host arrays of
 * n_tensors <= NERF_MAX_CHECK entries; d_counts device int[n_tensors], overwritten). */
#define NERF_MAX_CHECK 32
int nerf_count_nonfinite(const float* const* d_ptrs, const int64_t* sizes, int n_tensors, int* d_counts,
                         void* stream);

/* ---- multi-resolution hash grid -------------------------------------------------------------
 * Replaces HashEmbedder.forward (PocketNeRF/hash_encoding.py:82-107) = per level
 * get_voxel_vertices + hash (utils.py:95-117, :13-24), nn.Embedding gather (hash_encoding.py:94)
 * and trilinear_interp (:56-80); and its autograd backward (embedding_dense_backward).
 * Feature output element (point p, level l, feature f) is written at
 *   d_feat[p*feat_stride_point + l*feat_stride_level + f]     (f in {0,1}; n_features == 2)
 * so [P, 2L] point-major (stride_point=2L, stride_level=2) and [L, P, 2] level-major
 * (stride_point=2, stride_level=2P) are both supported. d_keep[p] = point inside the bbox on
 * all three axes (hash_encoding.py:106). level_res: host float[n_levels] = floor(16*b^l) (:89).
 * Tables: host array of n_levels device pointers, each [2^log2_T, 2] float32.
 */
int nerf_hash_encode_fwd(const float* d_xyz, int64_t n_points,
                         const float* bbox_min3, const float* bbox_max3,
                         const float* level_res, int n_levels, int log2_T,
                         const float* const* d_tables,
                         float* d_feat, int64_t feat_stride_point, int64_t feat_stride_level,
                         uint8_t* d_keep, void* stream);

/* Same with the A-CAQ quantizers applied to every gathered corner feature before the trilinear
 * blend (hash_encoding.py:97-101, LearnedBitwidthQuantizer.forward quantization.py:144-187).
 * d_qrec: device float[n_levels][8] records from nerf_quant_params (NULL = no quantization). The
 * backward is unchanged: the quantizer's straight-through estimator passes d feat through. */
int nerf_hash_encode_fwd_q(const float* d_xyz, int64_t n_points,
                           const float* bbox_min3, const float* bbox_max3,
                           const float* level_res, int n_levels, int log2_T,
                           const float* const* d_tables, const float* d_qrec,
                           float* d_feat, int64_t feat_stride_point, int64_t feat_stride_level,
                           uint8_t* d_keep, void* stream);

/* d_dtables: host array of n_levels device pointers; gradients are ACCUMULATED (atomic adds). */
int nerf_hash_encode_bwd(const float* d_xyz, int64_t n_points,
                         const float* bbox_min3, const float* bbox_max3,
                         const float* level_res, int n_levels, int log2_T,
                         const float* d_dfeat, int64_t feat_stride_point, int64_t feat_stride_level,
                         float* const* d_dtables, void* stream);

/* Same, on the binned ("owner computes") path: the entries are first written, sorted by table
 * slice, into a caller-owned device workspace (plain stores), then one workgroup per table slice
 * sums them in LDS and adds the slice into d_dtables once. Replaces the memory-side float atomics
 * of nerf_hash_encode_bwd, whose request rate bounds that path. The workspace needs no
 * initialisation; calls sharing one must be stream-ordered. workspace_bytes >=
 * nerf_hash_encode_bwd_workspace_bytes(n_levels, log2_T, n_points, deterministic) (0: path
 * unavailable for this log2_T; a NULL workspace gives nerf_hash_encode_bwd, which is never
 * deterministic).
 * deterministic != 0: SURVEY.md §8(b)'s `deterministic` flag. The owner pass sums in exact
 * integer fixed point (two int64 words per value at a per-level scale from the level's largest
 * entry; ~2^-75 of that entry per term), which is associative, so identical inputs give
 * bit-identical gradients whatever the scheduling. Needs log2_T <= 19 (2^12-row slices). */
size_t nerf_hash_encode_bwd_workspace_bytes(int n_levels, int log2_T, int64_t n_points, int deterministic);
int nerf_hash_encode_bwd_ws(const float* d_xyz, int64_t n_points,
                            const float* bbox_min3, const float* bbox_max3,
                            const float* level_res, int n_levels, int log2_T,
                            const float* d_dfeat, int64_t feat_stride_point, int64_t feat_stride_level,
                            float* const* d_dtables, int deterministic, void* d_workspace, size_t workspace_bytes,
                            void* stream);

/* The binned path split in two, so that several backwards into the same tables (the fine and the
 * coarse pass of one iteration: two autograd nodes of HashEmbedder.forward, hash_encoding.py:82-107)
 * share ONE owner pass. The workspace holds chunk_capacity chunks of C = nerf_hash_bwd_chunk_points()
 * (= NERF_HASH_CHUNK_POINTS) points (workspace_bytes >= nerf_hash_encode_bwd_workspace_bytes(n_levels,
 * log2_T, C * chunk_capacity, deterministic)); a bin call writes its ceil(n_points / C) chunks from
 * chunk_base on, and the owner call sums chunks
 * [0, n_chunks) into d_dtables (ACCUMULATED). Calls sharing a workspace must be stream-ordered and
 * use the same n_levels, log2_T, chunk_capacity and deterministic.
 * The owner's `deterministic` argument is a bit set: bit 0 = deterministic (as above), bit 1 =
 * NERF_OWNER_OVERWRITE: the tables' prior contents are ignored and every row of all n_levels
 * tables is STORED (its sum, or 0 where no entry lands), also when n_chunks == 0 — the result of
 * zeroing the gradients and accumulating, bit for bit, without the memset and without the owner's
 * row loads (the caller promises the gradients are logically zero: GradArena's deferred zero). */
#define NERF_OWNER_OVERWRITE 2
#ifndef NERF_HASH_CHUNK_POINTS
#define NERF_HASH_CHUNK_POINTS 512
#endif
int nerf_hash_bwd_chunk_points(void);
int nerf_hash_encode_bwd_bin(const float* d_xyz, int64_t n_points,
                             const float* bbox_min3, const float* bbox_max3,
                             const float* level_res, int n_levels, int log2_T,
                             const float* d_dfeat, int64_t feat_stride_point, int64_t feat_stride_level,
                             int64_t chunk_base, int64_t chunk_capacity, int deterministic,
                             void* d_workspace, size_t workspace_bytes, void* stream);
/* Row-mapped bin (coarse-feature reuse): point p reads d_xyz and d_dfeat at row d_rows[p] (NULL: p);
 * with d_dfeat2 != NULL it adds d_dfeat2 at row d_rows2[p] (NULL: p; strides feat2_*) to its
 * gradient, so a point shared by two passes is binned once with the sum of both gradients (d_dfeat
 * may then be NULL: the point's gradient is the d_dfeat2 term alone). d_count (device int, NULL = all
 * n_points): only points p < *d_count are binned (d_rows = an active-point list of nerf_active_rows);
 * the launch covers the chunks of n_points, those past the count get empty segments. */
int nerf_hash_encode_bwd_bin_rows(const float* d_xyz, const int32_t* d_rows, const int32_t* d_count, int64_t n_points,
                                  const float* bbox_min3, const float* bbox_max3,
                                  const float* level_res, int n_levels, int log2_T,
                                  const float* d_dfeat, int64_t feat_stride_point, int64_t feat_stride_level,
                                  const float* d_dfeat2, const int32_t* d_rows2,
                                  int64_t feat2_stride_point, int64_t feat2_stride_level,
                                  int64_t chunk_base, int64_t chunk_capacity, int deterministic,
                                  void* d_workspace, size_t workspace_bytes, void* stream);

/* Several bin launches of one workspace as ONE call (the fine and the coarse pass of an iteration): each
 * job's fields as the nerf_hash_encode_bwd_bin_rows arguments of the same name; the shared arguments
 * (box, levels, workspace) as there. Two non-empty jobs run as one launch (no drain / ramp between
 * them), more as one launch per further pair. Every job is validated before anything is launched;
 * the workspace contents are those of the separate calls. */
typedef struct nerf_bin_job {
    const float* xyz; const int32_t* rows; const int32_t* count; int64_t n_points;
    const float* dfeat; int64_t feat_stride_point, feat_stride_level;
    const float* dfeat2; const int32_t* rows2; int64_t feat2_stride_point, feat2_stride_level;
    int64_t chunk_base;
} nerf_bin_job;
int nerf_hash_encode_bwd_bin_batch(const nerf_bin_job* jobs, int n_jobs, const float* bbox_min3,
                                   const float* bbox_max3, const float* level_res, int n_levels, int log2_T,
                                   int64_t chunk_capacity, int deterministic, void* d_workspace,
                                   size_t workspace_bytes, void* stream);
int nerf_hash_encode_bwd_owner(int n_levels, int log2_T, int64_t n_chunks, int64_t chunk_capacity,
                               float* const* d_dtables, int deterministic, void* d_workspace,
                               size_t workspace_bytes, void* stream);
/* The owner pass of levels [level_begin, level_end) only (the same workspace and tables): a data-
 * parallel step launches the levels of each gradient bucket separately and starts the bucket's
 * reduce-scatter as soon as its levels are summed (dist.ShardedOptimizer buckets). */
int nerf_hash_encode_bwd_owner_range(int n_levels, int level_begin, int level_end, int log2_T, int64_t n_chunks,
                                     int64_t chunk_capacity, float* const* d_dtables, int deterministic,
                                     void* d_workspace, size_t workspace_bytes, void* stream);

/* The owner pass of levels [level_begin, level_end) with the tables' optimizer step fused into it: after
 * a block stores its slice's gradient rows (NERF_OWNER_OVERWRITE required: the stored row is then the
 * whole gradient of the step), it applies RAdam to those rows of d_params[l] / d_exp_avg[l] /
 * d_exp_avg_sq[l] — the elementwise update of nerf_radam_step, bit for bit, with the segment scalars
 * below (or, with d_coef, (decay_coef, step_coef, mode) read from device memory: graph replays). The
 * gradients stay stored (optimizer.step() leaves .grad in place). One launch instead of the owner pass
 * plus the tables' share of nerf_radam_step (16.8 M of its 16.8 M elements at the lego config): the
 * gradient is not read back, and the parameter rows stream while the owner blocks sum. NULL step: the
 * plain owner pass. */
typedef struct {
    float* const* d_params;       /* host arrays of n_levels device pointers, [2^log2_T][2] fp32 each */
    float* const* d_exp_avg;
    float* const* d_exp_avg_sq;
    float beta1, beta2, one_minus_beta1, one_minus_beta2, eps, decay_coef, step_coef;
    int mode;                     /* 0: moments only, 1: SGD-like, 2: adaptive (radam.py:49-79) */
    const float* d_coef;          /* optional device float[4]: (decay_coef, step_coef, mode, unused) */
} nerf_radam_table_step;
int nerf_hash_encode_bwd_owner_step(int n_levels, int level_begin, int level_end, int log2_T, int64_t n_chunks,
                                    int64_t chunk_capacity, float* const* d_dtables, int deterministic,
                                    void* d_workspace, size_t workspace_bytes, const nerf_radam_table_step* step,
                                    void* stream);

/* Entries the bin launches of chunks [0, n_chunks) of a workspace emitted (sum of their segment counts:
 * after the run merge, without zero entries), stored to d_count (device uint64). A measurement for the
 * bench's pricing of the hash backward; same workspace rules as the owner pass. */
int nerf_hash_bwd_entry_count(int n_levels, int log2_T, int64_t n_chunks, int64_t chunk_capacity, int deterministic,
                              const void* d_workspace, size_t workspace_bytes, unsigned long long* d_count,
                              void* stream);

/* ---- active points of a field backward -----------------------------------------------------------
 * raw2outputs' autograd (run_nerf.py:364-386) gives every sample with relu(sigma + noise) = 0 an all-
 * zero raw-gradient row, and NeRFSmall's backward is linear in it: such points add nothing to the MLP
 * weight gradients or the hash-table gradients. nerf_active_rows lists, in ascending order, the points
 * p whose row d_graw_rows[p] (NULL: p) of d_graw [P,4] (or of d_dgeo [P,16], rows 1..15, when given)
 * is not all zero: d_rows [P], d_counts[0]; d_counts[1] = how many of them are < n_first (the list's
 * prefix). d_zero_feat (optional, level-major, n_levels x 2 floats per row at stride
 * zero_stride_level): rows p >= n_first of the INACTIVE points are zeroed (feature-gradient rows a bin
 * reads but the active-point backward does not write). Two launches, no host sync; the workspace is
 * nerf_active_rows_workspace_bytes(P). */
size_t nerf_active_rows_workspace_bytes(int64_t n_points);
int nerf_active_rows(const float* d_graw, const float* d_dgeo, int64_t n_points, const int32_t* d_graw_rows,
                     int64_t n_first, int32_t* d_rows, int32_t* d_counts,
                     float* d_zero_feat, int64_t zero_stride_level, int n_levels, void* d_workspace,
                     size_t workspace_bytes, void* stream);

/* ---- spherical harmonics, degree 4 (SHEncoder.forward, hash_encoding.py:153-191) ---------- */
int nerf_sh4_fwd(const float* d_dirs, int64_t n, float* d_out /* [n,16] */, void* stream);

/* ---- fused tiny MLP (NeRFSmall.forward, run_nerf_helpers.py:265-306, + run_network's
 *      sigma := 0 outside the bbox, run_nerf.py:66), fp32-accurate on the bf16 matrix cores
 *      (each fp32 operand split into three bf16 pieces, six v_mfma_f32_32x32x16_bf16 per product) -----
 * Weights are nn.Linear layouts [out][in], no bias: w0 [64,32], w1 [16,64], c0 [64,31],
 * c1 [64,64], c2 [3,64] (create_nerf's NeRFSmall(num_layers=2, num_layers_color=3)).
 * Input point p: hash features x[p][k] = d_feat[p*feat_stride_point + (k/2)*feat_stride_level + k%2]
 * (k < 32); view encoding: if d_viewdirs != NULL, SH4 of d_viewdirs[p / samples_per_ray] is
 * computed in-kernel, else sh[p][k] = d_sh[p*sh_stride + k] (k < 16) — or, with sh_stride == 0, the
 * per-RAY records of 40 floats: sh[p][k] = d_sh[40*(p / samples_per_ray) + k], followed by the three
 * exact bf16 pieces of the 16 values (piece q of k at bf16 index 32 + 16q + k of the record) that
 * the MLP kernels use as the pre-split matrix operand (16-B aligned; the point order's two segments
 * as for d_viewdirs), i.e. nerf_sample_stratified_sh's d_sh.
 * d_keep may be NULL (keep all). Output d_raw [P,4] = [rgb_raw(3), sigma_raw].
 */
typedef struct {
    const float* w0;
    const float* w1;
    const float* c0;
    const float* c1;
    const float* c2;
} nerf_mlp_weights;

typedef struct {
    float* w0;
    float* w1;
    float* c0;
    float* c1;
    float* c2;
} nerf_mlp_grads;

/* d_geo (may be NULL): also write o = [sigma, geo_feat 15] per point, [P,16] — the normals head's
 * input (run_nerf_helpers.py:287, :300). */
int nerf_mlp_fwd(const float* d_feat, int64_t feat_stride_point, int64_t feat_stride_level,
                 const float* d_sh, int64_t sh_stride,
                 const float* d_viewdirs, int64_t samples_per_ray,
                 const uint8_t* d_keep, int64_t n_points,
                 const nerf_mlp_weights* weights, float* d_raw, float* d_geo, void* stream);

/* Backward: recomputes the forward, then ACCUMULATES weight grads into *grads (atomic adds) and
 * WRITES d_dfeat (same strides as d_feat; may be NULL) and d_dsh ([P,16], may be NULL).
 * d_dgeo (may be NULL): extra upstream gradient of o rows 1..15 ([P,16], from the normals head). */
int nerf_mlp_bwd(const float* d_feat, int64_t feat_stride_point, int64_t feat_stride_level,
                 const float* d_sh, int64_t sh_stride,
                 const float* d_viewdirs, int64_t samples_per_ray,
                 const uint8_t* d_keep, int64_t n_points,
                 const nerf_mlp_weights* weights, const float* d_graw /* [P,4] */,
                 const nerf_mlp_grads* grads, float* d_dfeat, float* d_dsh, const float* d_dgeo, void* stream);

/* A-CAQ variants (NeRFSmall(use_quantization=True), run_nerf_helpers.py:268-284). The caller passes
 * the fake-quantized W0 (nerf_fake_quant with sigma_weight_quantizer's record) as weights->w0, and
 * gradients land in the unquantized W0's grad (straight-through). d_act_qrec (NULL = none): record
 * of sigma_act_quantizers[0], applied to h = relu(x W0^T) before the second sigma layer; the
 * backward keeps relu'(pre) as the mask and Q(h) as the activation, as the reference's autograd.
 * fwd with d_act_minmax != NULL is a calibration-only launch: it folds min/max of relu(x W0^T)
 * over the first act_calib_points points into d_act_minmax (uint32[2], see nerf_quant_minmax)
 * and writes no outputs. */
int nerf_mlp_fwd_q(const float* d_feat, int64_t feat_stride_point, int64_t feat_stride_level,
                   const float* d_sh, int64_t sh_stride,
                   const float* d_viewdirs, int64_t samples_per_ray,
                   const uint8_t* d_keep, int64_t n_points,
                   const nerf_mlp_weights* weights, float* d_raw, float* d_geo,
                   const float* d_act_qrec, uint32_t* d_act_minmax, int64_t act_calib_points, void* stream);
/* Point order of a fine pass with the coarse-feature reuse: the features are in the
 * importance-first order of the reuse (rows [0, seg_split): importance sample k of ray r at r*N + k;
 * then coarse sample i of ray r at seg_split + r*S + i) while raw / geo (fwd) and graw / dgeo / dsh
 * (bwd) stay in the merged order render_rays composites (run_nerf.py:512-516). Point p's row there is
 * io_rows[p] (NULL: p; nerf_sample_fine_rows' d_imp_rows followed by its d_coarse_rows); its view
 * direction is ray p / samples_per_ray below seg_split and (p - seg_split) / spr2 from there on. */
typedef struct {
    const int32_t* io_rows;
    int64_t seg_split;
    int64_t spr2;
} nerf_point_order;

/* nerf_mlp_fwd_q in a point order (NULL order: the identity, seg_split = n_points). */
/* Training forward (ABI 10): also stores layer C1's ReLU outputs into d_h3 (>= nerf_mlp_h3_bytes(n_points),
 * 256 B per point, an opaque per-tile layout) for the backward job's `h3`, which then reads them
 * instead of recomputing C1; bit-identical to the recompute. Not with A-CAQ (d_act_qrec). */
size_t nerf_mlp_h3_bytes(int64_t n_points);
int nerf_mlp_fwd_h3(const float* d_feat, int64_t feat_stride_point, int64_t feat_stride_level,
                    const float* d_sh, int64_t sh_stride,
                    const float* d_viewdirs, int64_t samples_per_ray,
                    const uint8_t* d_keep, int64_t n_points,
                    const nerf_mlp_weights* weights, float* d_raw, float* d_geo,
                    const float* d_act_qrec, uint32_t* d_act_minmax, int64_t act_calib_points,
                    const nerf_point_order* order, float* d_h3, void* stream);
int nerf_mlp_fwd_ord(const float* d_feat, int64_t feat_stride_point, int64_t feat_stride_level,
                     const float* d_sh, int64_t sh_stride,
                     const float* d_viewdirs, int64_t samples_per_ray,
                     const uint8_t* d_keep, int64_t n_points,
                     const nerf_mlp_weights* weights, float* d_raw, float* d_geo,
                     const float* d_act_qrec, uint32_t* d_act_minmax, int64_t act_calib_points,
                     const nerf_point_order* order, void* stream);
int nerf_mlp_bwd_q(const float* d_feat, int64_t feat_stride_point, int64_t feat_stride_level,
                   const float* d_sh, int64_t sh_stride,
                   const float* d_viewdirs, int64_t samples_per_ray,
                   const uint8_t* d_keep, int64_t n_points,
                   const nerf_mlp_weights* weights, const float* d_graw,
                   const nerf_mlp_grads* grads, float* d_dfeat, float* d_dsh, const float* d_dgeo,
                   const float* d_act_qrec, void* stream);

/* Batched backward of up to NERF_MLP_MAX_JOBS nets in ONE launch (the coarse and the fine NeRFSmall
 * of a training iteration: run_nerf.py:1007-1035 backpropagates both; the reference runs them as
 * separate autograd subgraphs). Each job carries the arguments of nerf_mlp_bwd_q. Empty jobs are
 * skipped. d_det_workspace (NULL = off; >= nerf_mlp_bwd_det_workspace_bytes()) selects the
 * DETERMINISTIC mode: every block's weight-gradient partial sum is stored and reduced over blocks in
 * a fixed order (no float atomics), so identical inputs give bit-identical gradients.
 * Stateless: the kernels keep everything between the stages of a tile in registers and LDS, so
 * calls on different streams of one device may run concurrently (only calls that share a
 * d_det_workspace must be stream-ordered). */
#define NERF_MLP_MAX_JOBS 2
typedef struct {
    const float* feat;
    int64_t feat_stride_point, feat_stride_level;
    const float* sh;
    int64_t sh_stride;
    const float* viewdirs;
    int64_t samples_per_ray;
    const uint8_t* keep;
    int64_t n_points;
    nerf_mlp_weights weights;
    const float* graw;
    nerf_mlp_grads grads;
    float* dfeat;
    float* dsh;
    const float* dgeo;
    const float* act_qrec;
    nerf_point_order order;      /* spr2 == 0 (zero-filled): one segment, rows io_rows (NULL: the identity) */
    int64_t dfeat_stride_point, dfeat_stride_level;   /* 0: the feature strides */
    const int32_t* rows;         /* optional (with d_count): walk only the points rows[0 .. *d_count) — the active
                                    points of nerf_active_rows; the other points' d feat / d sh are not written */
    const int32_t* d_count;      /* device int: the number of rows */
    const float* h3;             /* optional (ABI 10): the h3 the same points' nerf_mlp_fwd_h3 stored (NULL:
                                    recomputed); not with act_qrec or rows; all jobs of a launch alike or split */
} nerf_mlp_bwd_job;

size_t nerf_mlp_bwd_det_workspace_bytes(void);
int nerf_mlp_bwd_batch(const nerf_mlp_bwd_job* jobs, int n_jobs, float* d_det_workspace,
                       size_t det_workspace_bytes, void* stream);

/* ---- normals head (run_nerf_helpers.py:259-263, :298-302): n = normalize(N1 relu(N0 geo + b0) + b1)
 * nn.Linear layouts: n0 [32,15], b0 [32], n1 [3,32], b1 [3].
 * fwd: raw7 [P,7] = [raw4, n]; with d_keep, n_z := 0 where !keep (run_network's mask hits the LAST
 *      channel, run_nerf.py:66). bwd: from graw7 writes graw4 [P,4] (the MLP's upstream grad) and
 *      dgeo [P,16] (row 0 = 0), and ACCUMULATES the head's weight gradients into *grads
 *      (dN0 = dhid^T geo, db0 = sum dhid, dN1 = dn^T hid, db1 = sum dn, summed in-kernel; per-block
 *      sums in d_workspace (>= nerf_normal_head_bwd_workspace_bytes()) reduced in a fixed order). */
typedef struct {
    const float* n0;
    const float* b0;
    const float* n1;
    const float* b1;
} nerf_normal_head;

typedef struct {
    float* n0;
    float* b0;
    float* n1;
    float* b1;
} nerf_normal_head_grads;

int nerf_normal_head_fwd(const float* d_o16, const float* d_raw4, const uint8_t* d_keep, int64_t n_points,
                         const nerf_normal_head* head, float* d_raw7, void* stream);
/* ABI 12: the forward over a permuted point order — source point q (its keep flag d_keep[q]) sits at
 * merged row d_rows[q] of d_o16 / d_raw4 / d_raw7, and its keep flag is scattered to d_keep_out[d_rows[q]]
 * (the merged-order mask nerf_normal_head_bwd reads). d_rows must be a permutation of [0, n_points);
 * NULL rows = nerf_normal_head_fwd (d_keep_out NULL too). Replaces FieldFn's keep scatter on the fine
 * pass with coarse-feature reuse (render.CoarseReuse: the MLP walks the importance-first order). */
int nerf_normal_head_fwd_rows(const float* d_o16, const float* d_raw4, const uint8_t* d_keep, const int32_t* d_rows,
                              int64_t n_points, const nerf_normal_head* head, float* d_raw7, uint8_t* d_keep_out,
                              void* stream);
size_t nerf_normal_head_bwd_workspace_bytes(void);
int nerf_normal_head_bwd(const float* d_o16, const uint8_t* d_keep, int64_t n_points,
                         const nerf_normal_head* head, const float* d_graw7, float* d_graw4, float* d_dgeo,
                         const nerf_normal_head_grads* grads, float* d_workspace, size_t workspace_bytes,
                         void* stream);

/* ---- volume compositing (raw2outputs, run_nerf.py:347-411), one wavefront per ray ----------
 * d_raw [R,S,raw_channels] (4, or 7 with normals), d_z [R,S], d_rays_d [R,3] (unnormalised),
 * d_noise [R,S] added to sigma (NULL = none). Outputs (any may be NULL except d_weights):
 * rgb [R,3], disp [R], acc [R], weights [R,S], depth [R], entropy [R], normal [R,3].
 */
int nerf_composite_fwd(const float* d_raw, int raw_channels, const float* d_z, const float* d_rays_d,
                       const float* d_noise, int64_t n_rays, int n_samples, int white_bkgd,
                       float* d_rgb, float* d_disp, float* d_acc, float* d_weights, float* d_depth,
                       float* d_entropy, float* d_normal, void* stream);

/* Upstream grads (any may be NULL = zero): g_rgb [R,3], g_disp, g_acc [R], g_weights [R,S],
 * g_depth, g_entropy [R], g_normal [R,3]. Writes d_graw [R,S,raw_channels]. */
int nerf_composite_bwd(const float* d_raw, int raw_channels, const float* d_z, const float* d_rays_d,
                       const float* d_noise, int64_t n_rays, int n_samples, int white_bkgd,
                       const float* d_g_rgb, const float* d_g_disp, const float* d_g_acc,
                       const float* d_g_weights, const float* d_g_depth, const float* d_g_entropy,
                       const float* d_g_normal, float* d_graw, void* stream);

/* Several compositing backwards in one call (the fine and the coarse pass of a training iteration):
 * each job's fields as the nerf_composite_bwd arguments of the same name. Two jobs with
 * ceil(S/64) in {(1,1),(2,1),(3,1),(4,1),(2,2),(3,2),(4,2),(3,3)} (either order) run as ONE launch;
 * otherwise one launch per job. Every job is validated before anything is launched; results are
 * bit-identical to nerf_composite_bwd per job. */
typedef struct nerf_composite_bwd_job {
    const float* raw; int raw_channels; const float* z; const float* rays_d; const float* noise;
    int64_t n_rays; int n_samples; int white_bkgd;
    const float* g_rgb; const float* g_disp; const float* g_acc; const float* g_weights; const float* g_depth;
    const float* g_entropy; const float* g_normal;
    float* graw;
} nerf_composite_bwd_job;
int nerf_composite_bwd_batch(const nerf_composite_bwd_job* jobs, int n_jobs, void* stream);

/* ---- ray sampling (render_rays, run_nerf.py:460-490) --------------------------------------
 * d_rays: packed ray batch [R, ray_stride] = [o(3), d(3), near, far, (viewdir(3))] as render()
 * builds it (run_nerf.py:134-140). d_t: [S] = torch.linspace(0,1,S) values. perturb != 0 jitters
 * with d_u [R,S] (NULL = Philox(seed, offset)). Writes d_z [R,S] and d_pts [R,S,3] (may be NULL).
 */
int nerf_sample_stratified(const float* d_rays, int64_t ray_stride, int64_t n_rays, int n_samples,
                           const float* d_t, int lindisp, int perturb, const float* d_u,
                           uint64_t seed, uint64_t offset, const uint64_t* d_rng,
                           float* d_z, float* d_pts,
                           float* d_dirs /* optional [R,3]: ray columns 3..5, contiguous */,
                           float* d_viewdirs /* optional [R,3]: the last 3 ray columns (stride > 8) */,
                           void* stream);

/* Same, also writing d_sh [R,40] = per ray SH4 of its view direction (the last 3 columns; needs
 * ray_stride > 8; hash_encoding.py:153-191), 16 fp32 values and their three bf16 pieces: the per-ray
 * records the MLP entries take with sh_stride 0. */
int nerf_sample_stratified_sh(const float* d_rays, int64_t ray_stride, int64_t n_rays, int n_samples,
                              const float* d_t, int lindisp, int perturb, const float* d_u,
                              uint64_t seed, uint64_t offset, const uint64_t* d_rng,
                              float* d_z, float* d_pts, float* d_dirs, float* d_viewdirs, float* d_sh,
                              void* stream);

/* sample_pdf (run_nerf_helpers.py:354-397) on bins [R,n_bins], weights [R,n_bins-1];
 * det: u = d_t_imp (torch.linspace(0,1,N) values, [N]); else u = d_u [R,N] or Philox. */
int nerf_sample_pdf(const float* d_bins, int64_t bins_stride, const float* d_weights, int64_t weights_stride,
                    int64_t n_rays, int n_bins, int n_importance, int det, const float* d_t_imp,
                    const float* d_u, uint64_t seed, uint64_t offset, const uint64_t* d_rng,
                    float* d_samples, void* stream);

/* Hierarchical step of render_rays (run_nerf.py:508-513, :541) in one launch: z_mid of the
 * coarse z, sample_pdf on weights[...,1:-1], sort(cat(z, z_samples)), fine points, z_std.
 * Outputs d_z_fine [R,S+N], d_pts_fine [R,S+N,3] (may be NULL), d_z_std [R] (may be NULL),
 * d_samples [R,N] (may be NULL). */
int nerf_sample_fine(const float* d_rays, int64_t ray_stride, const float* d_z, const float* d_weights,
                     int64_t n_rays, int n_samples, int n_importance, int det, const float* d_t_imp,
                     const float* d_u, uint64_t seed, uint64_t offset, const uint64_t* d_rng,
                     float* d_z_fine, float* d_pts_fine, float* d_z_std, float* d_samples, void* stream);
/* Same, also writing the maps of the merge (NULL = skip; coarse-feature reuse):
 * d_coarse_rows [R,S] int32 = the absolute fine row r*(S+N) + rank of coarse sample i of ray r;
 * d_imp_rows [R,N] int32 = the fine rows of the ray's importance samples, ascending; d_imp_pts [R,N,3]
 * their points (the same bits as d_pts_fine at those rows); d_perm [R*(S+N)] int32 = fine row ->
 * position in the importance-first order (importance k of ray r: r*N + k; coarse i: R*N + r*S + i).
 * Needs R*(S+N) <= INT32_MAX when a map is set. */
int nerf_sample_fine_rows(const float* d_rays, int64_t ray_stride, const float* d_z, const float* d_weights,
                          int64_t n_rays, int n_samples, int n_importance, int det, const float* d_t_imp,
                          const float* d_u, uint64_t seed, uint64_t offset, const uint64_t* d_rng,
                          float* d_z_fine, float* d_pts_fine, float* d_z_std, float* d_samples,
                          int32_t* d_coarse_rows, int32_t* d_imp_rows, float* d_imp_pts, int32_t* d_perm,
                          void* stream);

/* The coarse pass of render_rays in one launch: nerf_composite_fwd (arguments as there; d_z, d_weights
 * and n_rays / n_samples are shared with the sampler) followed by nerf_sample_fine_rows on its weights
 * (the remaining arguments as there). Bit-identical to the two calls, which it makes itself when
 * n_samples > 128 (the fused launch holds the weights of a ray in LDS, one wave per ray). */
int nerf_composite_sample_fine(const float* d_raw, int raw_channels, const float* d_z, const float* d_rays_d,
                               const float* d_noise, int64_t n_rays, int n_samples, int white_bkgd,
                               float* d_rgb, float* d_disp, float* d_acc, float* d_weights, float* d_depth,
                               float* d_entropy, float* d_normal,
                               const float* d_rays, int64_t ray_stride, int n_importance, int det,
                               const float* d_t_imp, const float* d_u, uint64_t seed, uint64_t offset,
                               const uint64_t* d_rng, float* d_z_fine, float* d_pts_fine, float* d_z_std,
                               float* d_samples, int32_t* d_coarse_rows, int32_t* d_imp_rows, float* d_imp_pts,
                               int32_t* d_perm, void* stream);

/* ---- rays of the training batch / of a whole image (run_nerf.py:973-1004, run_nerf_helpers.py:311-320)
 * Camera: c2w = the pose [3,4] as float32 (torch.Tensor(pose)), fx = K[0][0], fy = K[1][1],
 * cx = K[0][2], cy = K[1][2] rounded to float32 (the scalars get_rays' tensor ops see).
 * Pixel (row, col) -> dirs = ((col - cx)/fx, -(row - cy)/fy, -1), rays_d = c2w[:3,:3] dirs,
 * rays_o = c2w[:3,3]. Cells of the crop window [r0, r0+h) x [c0, c0+w) are numbered row-major.
 * random != 0: n_rays DISTINCT cells drawn uniformly without replacement (np.random.choice(...,
 * replace=False) of train(); a keyed Feistel permutation from (seed, offset)); random == 0: cells
 * 0..n_rays-1 in order (the whole image when the window is the image). d_image [H,W,channels]
 * float32 (may be NULL if d_target is NULL): d_target [n,3] = its first three channels at the
 * pixel. d_coords [n,2] int32 (row, col), may be NULL. */
typedef struct {
    float c2w[12];
    float fx, fy, cx, cy;
} nerf_camera;

int nerf_sample_rays(const nerf_camera* cam, int H, int W, int crop_r0, int crop_c0, int crop_h, int crop_w,
                     int64_t n_rays, int random, uint64_t seed, uint64_t offset,
                     const float* d_image, int channels, float* d_rays_o, float* d_rays_d, float* d_target,
                     int32_t* d_coords, void* stream);
/* nerf_sample_rays (random = 1) with the image chosen on the device: d_sel = {image index, seed,
 * offset} (device int64[3], read by the launch — a captured training step's per-replay slots: train()
 * draws a new image and pixel batch every iteration, run_nerf.py:975-1004); d_cams [n_images]
 * nerf_camera and d_images [n_images, H, W, channels] float32 (may be NULL if d_target is NULL)
 * resident on the device; the image index is taken mod n_images. Bit-identical to nerf_sample_rays
 * with that image's camera and image, the same seed and offset. */
int nerf_sample_rays_sel(const nerf_camera* d_cams, const float* d_images, int64_t n_images, int H, int W,
                         int channels, int crop_r0, int crop_c0, int crop_h, int crop_w, int64_t n_rays,
                         const int64_t* d_sel, float* d_rays_o, float* d_rays_d, float* d_target,
                         int32_t* d_coords, void* stream);

/* render()'s ray batch (run_nerf.py:115-140): viewdir = d/|d| of the world direction, optional
 * ndc_rays with near plane 1 (run_nerf_helpers.py:333-350; ndc_coef_w/h = float32 of
 * -1/(W/(2 focal)) and -1/(H/(2 focal))), then [o(3), d(3), near, far, viewdir(3)] per ray
 * (8 floats without viewdirs). d_rays_o/d [n,3]; d_out [n, 11 | 8]. */
int nerf_rays_pack(const float* d_rays_o, const float* d_rays_d, int64_t n_rays, float near, float far,
                   int ndc, float ndc_coef_w, float ndc_coef_h, int use_viewdirs, float* d_out, void* stream);
/* Same, also storing 0.0f over up to NERF_MAX_ZERO_RANGES float ranges in the same launch: a training
 * step's gradient / loss-accumulator zero fills, folded into its first launch (_lib.defer_fill_zero). */
#define NERF_MAX_ZERO_RANGES 4
typedef struct nerf_zero_range { float* ptr; int64_t n; } nerf_zero_range;
int nerf_rays_pack_z(const float* d_rays_o, const float* d_rays_d, int64_t n_rays, float near, float far,
                     int ndc, float ndc_coef_w, float ndc_coef_h, int use_viewdirs, float* d_out,
                     const nerf_zero_range* zeros, int n_zeros, void* stream);

/* ---- RAdam (PocketNeRF/radam.py:28-94), one launch over up to 32 tensor segments ----------
 * Per segment: p, g, m (exp_avg), v (exp_avg_sq) of n elements. The host evaluates the scalar
 * algebra of radam.py:56-79 in double, exactly as the reference's Python does, and passes the
 * float32 roundings of the scalars the tensor ops see:
 *   beta1, beta2            multipliers of exp_avg / exp_avg_sq (mul_(beta))
 *   one_minus_beta1/2       float(1 - beta)          (add_/addcmul_ value)
 *   decay_coef              float(-weight_decay*lr)   (0 = no decay)
 *   step_coef               float(-step_size*lr)
 *   mode 2: N_sma >= 5 (p += step_coef*m/(sqrt(v)+eps)), 1: step_size > 0 (p += step_coef*m),
 *   0: moments only.
 * d_coef (may be NULL): device [n_segs][4] = (decay_coef, step_coef, mode, 0) overriding the
 * by-value ones (a step captured in a HIP graph reads this step's scalars from memory).
 * grad_scale (ABI 9): g is read as g * grad_scale (0 = 1: unscaled) — a ZeRO-1 shard steps on the
 * reduce-scatter's SUM of the ranks' gradients with grad_scale = float(1 / world), the mean the
 * replicated path forms with a separate multiply, without that extra pass over the shard.
 */
typedef struct {
    float* p;
    const float* g;
    float* m;
    float* v;
    int64_t n;
    float beta1, beta2, one_minus_beta1, one_minus_beta2, eps, decay_coef, step_coef;
    int mode;
    float grad_scale;
} nerf_radam_segment;

int nerf_radam_step(const nerf_radam_segment* segs, int n_segs, const float* d_coef, void* stream);

/* ---- per-step scalars of a captured training step (graphs.StepScalars) ------------------------
 * The one exception to "the library allocates nothing": nerf_host_ring_alloc returns n_bytes of
 * pinned, device-mapped, coherent host memory (hipHostMalloc Mapped|Coherent); free it with
 * nerf_host_ring_free after the last replay that reads it has completed.
 * nerf_scalars_fetch (one block, the first launch of a captured step) copies slot
 * (d_ctl[0] mod n_slots) of that ring (n_slots x slot_bytes) into d_dst and advances d_ctl[0]; only
 * the 4-byte words [0, d_ctl[1]) and [d_ctl[2], d_ctl[2] + d_ctl[3]) are copied. d_ctl: device
 * int64[4]. done_offset >= 0: the int64 at that byte offset of the ring (past the slots) receives
 * the new d_ctl[0] once the slot is read, so the host knows which slots it may rewrite; the last 8
 * bytes of every slot then hold the index (int64) of the replay the host wrote the slot for, and a
 * fetch that finds another index than its d_ctl[0] stores d_ctl[0] + 1 into the int64 at
 * done_offset + 8 (sticky: only while that word is 0; the ring holds done_offset + 16 bytes or more).
 * Replaces the host->device copy and event queued before every replay (graphs.py StepScalars.upload). */
int nerf_host_ring_alloc(int64_t n_bytes, void** host);
int nerf_host_ring_free(void* host);
int nerf_scalars_fetch(const void* host_ring, int64_t slot_bytes, int n_slots, int64_t done_offset, int64_t* d_ctl,
                       void* d_dst, void* stream);

/* ---- total-variation loss on one hashed cuboid per level (loss.py:11-43) ------------------
 * min_vertex: host int64[n_levels][3] (the reference draws it with torch.randint);
 * cube: host int[n_levels] cuboid edge. fwd: d_loss[l] += TV_l (ACCUMULATED; zero it first).
 * bwd: d_dtables[l] += d(scale_l * TV_l)/d table, scale: host float[n_levels]. */
int nerf_tv_fwd(const float* const* d_tables, int n_levels, int log2_T, const int64_t* min_vertex,
                const int64_t* d_min_vertex, const int* cube, float* d_loss,
                float* d_verts /* optional out: float2[sum_l (cube_l+1)^3], the vertices' table rows */,
                void* stream);
int nerf_tv_bwd(const float* const* d_tables, int n_levels, int log2_T, const int64_t* min_vertex,
                const int64_t* d_min_vertex, const int* cube, const float* d_scale /* device [n_levels] */,
                float* const* d_dtables, void* stream);
/* Binned TV backward: the same gradient as nerf_tv_bwd, written as entries into a binned hash-backward
 * workspace (chunks [chunk_base, chunk_base + nerf_tv_bwd_bin_chunks(n_levels, cube)), one entry per
 * cuboid vertex) and summed into the tables by nerf_hash_encode_bwd_owner together with the hash
 * backwards binned beside it: no float atomics, bit-reproducible under deterministic = 1. Workspace
 * rules as nerf_hash_encode_bwd_bin. nerf_tv_bwd_bin_chunks returns 0 for invalid arguments. */
int64_t nerf_tv_bwd_bin_chunks(int n_levels, const int* cube);
int nerf_tv_bwd_bin(const float* const* d_tables, int n_levels, int log2_T, const int64_t* min_vertex,
                    const int64_t* d_min_vertex, const int* cube, const float* d_scale /* device [n_levels] */,
                    const float* d_verts /* optional: nerf_tv_fwd's d_verts of the same tables and cuboids */,
                    int64_t chunk_base, int64_t chunk_capacity, int deterministic, void* d_workspace,
                    size_t workspace_bytes, void* stream);
/* ABI 11: nerf_composite_fwd with the iteration's TV forward (nerf_tv_fwd) in the same launch: the TV's
 * gather blocks run beside the fine pass's one-wave rays instead of as a launch of their own. tv: the
 * nerf_tv_fwd arguments of the same name for n_levels tables of 2^log2_T rows (d_loss accumulates as
 * there, d_verts optional); NULL tv = nerf_composite_fwd. Outputs are those of the two separate calls
 * (the TV loss up to its float atomics' order). */
typedef struct nerf_tv_fwd_job {
    const float* const* d_tables; const int64_t* min_vertex; const int64_t* d_min_vertex; const int* cube;
    float* d_loss; float* d_verts;
} nerf_tv_fwd_job;
int nerf_composite_fwd_tv(const float* d_raw, int raw_channels, const float* d_z, const float* d_rays_d,
                          const float* d_noise, int64_t n_rays, int n_samples, int white_bkgd, float* d_rgb,
                          float* d_disp, float* d_acc, float* d_weights, float* d_depth, float* d_entropy,
                          float* d_normal, const nerf_tv_fwd_job* tv, int n_levels, int log2_T, void* stream);
/* ABI 11: nerf_hash_encode_bwd_bin_batch with the pass's binned TV backward in the same launch (its
 * blocks first: the TV's few, gather-latency-bound blocks run beside the hash bins instead of as a
 * launch of their own). tv: the nerf_tv_bwd_bin arguments of the same name (d_verts required; the
 * levels and workspace are the batch's); NULL tv = nerf_hash_encode_bwd_bin_batch. The workspace
 * contents are those of the separate calls, bit for bit. */
typedef struct nerf_tv_bin_job {
    const float* const* d_tables; const int64_t* min_vertex; const int64_t* d_min_vertex; const int* cube;
    const float* d_scale; const float* d_verts; int64_t chunk_base;
} nerf_tv_bin_job;
int nerf_hash_encode_bwd_bin_batch_tv(const nerf_bin_job* jobs, int n_jobs, const float* bbox_min3,
                                      const float* bbox_max3, const float* level_res, int n_levels, int log2_T,
                                      int64_t chunk_capacity, int deterministic, void* d_workspace,
                                      size_t workspace_bytes, const nerf_tv_bin_job* tv, void* stream);

/* ---- training-loss head (run_nerf.py:1011-1037: img2mse of both passes, sparsity, TV, mse2psnr) ----
 * fwd: device scalars loss, img_loss (fine-pass MSE), psnr; rgb0 / sparsity / sparsity0 / tv may be NULL.
 *      loss = img + mse(rgb0) + sparse_w * (sum(sp) + sum(sp0)) + tv_w * sum_l tv[l]
 * bwd: d_grad_loss is a device scalar; outputs d rgb = (g/3R) * 2 (rgb - t), d sp = sparse_w g,
 *      d tv[l] = tv_w g (NULL outputs are skipped). */
int nerf_train_loss_fwd(const float* d_rgb, const float* d_rgb0, const float* d_target, int64_t n_rays,
                        const float* d_sparsity, const float* d_sparsity0, float sparse_w, const float* d_tv,
                        int n_tv, float tv_w, float* d_loss, float* d_img_loss, float* d_psnr, void* stream);
int nerf_train_loss_bwd(const float* d_rgb, const float* d_rgb0, const float* d_target, int64_t n_rays,
                        float sparse_w, int n_tv, float tv_w, const float* d_grad_loss, float* d_grad_rgb,
                        float* d_grad_rgb0, float* d_grad_sparsity, float* d_grad_sparsity0, float* d_grad_tv,
                        void* stream);

/* ---- A-CAQ learned-bitwidth quantization (PocketNeRF/quantization.py:63-187, config 5) --------
 * A quantizer's state is the reference module's tensors, as caller-owned device scalars (fp32):
 * soft_bits, range_scale, v_max (NULL for a symmetric quantizer) and the running_min/max buffers.
 * Quantization record (device float[8]): {scale, scale + 1e-8, zero_point, qmin, qmax, ste, bits, 0}.
 */
typedef struct {
    const float* soft_bits;
    float* range_scale;
    float* v_max;          /* NULL: symmetric */
    float* running_min;
    float* running_max;
    float min_bits, max_bits;
} nerf_quantizer;

#define NERF_MAX_QUANTIZERS 32

/* Records of n quantizers (<= NERF_MAX_QUANTIZERS), as LearnedBitwidthQuantizer.forward derives them
 * (:158-178): B = clamp(soft_bits) (training) or round(B) (eval); qmin/qmax from round(B);
 * symmetric scale = range/2^(B-1), zp = 0; asymmetric scale = max(range,1e-8)/(2^B-1),
 * zp = round(clamp(v_max/scale, qmin, qmax)). ste = training. */
int nerf_quant_params(const nerf_quantizer* qs, int n, int training, float* d_rec, void* stream);

/* Calibration statistics: d_minmax is device uint32[n][2] holding order-preserving encodings of
 * (min, max). reset sets n slots to (+inf, -inf); minmax folds d_x[0..count) into slot 0. */
int nerf_quant_minmax_reset(uint32_t* d_minmax, int n, void* stream);
int nerf_quant_minmax(const float* d_x, int64_t count, uint32_t* d_minmax, void* stream);

/* Per-level min/max of the gathered corner features [P,8,2] of the hash encoding (the x
 * LearnedBitwidthQuantizer.calibrate sees, quantization.py:97-119), folded into d_minmax[level]. */
int nerf_hash_gather_minmax(const float* d_xyz, int64_t n_points, const float* bbox_min3, const float* bbox_max3,
                            const float* level_res, int n_levels, int log2_T, const float* const* d_tables,
                            uint32_t* d_minmax, void* stream);

/* calibrate() (:97-119) of n quantizers from the batch statistics d_minmax[n][2]: running min/max,
 * then range_scale (= max - min, or 2 max|.| when symmetric) and v_max (= running max). */
int nerf_quant_calibrate(const nerf_quantizer* qs, int n, const uint32_t* d_minmax, void* stream);

/* Elementwise fake quantization y = Q(x) with one record (d_rec); in training mode the STE form
 * x + (deq - x), whose gradient is the identity. d_y may alias d_x. */
int nerf_fake_quant(const float* d_x, int64_t count, const float* d_rec, float* d_y, void* stream);

/* A-CAQ bit-width controller of train() (run_nerf.py:1207-1250), run every 10th iteration from
 * acaq_start_iter: loss_ratio = img_loss / target (target = target_metric, or 1.2 x the best
 * img_loss so far, kept in d_best_loss, NaN = unset); per quantizer idx of n:
 * delta = {-0.3 | -0.1 | +0.2 by ratio < 0.95 / < 1.05 / else} - bit_penalty*bits/8, times
 * 1 + (idx - n/2)*0.02; soft_bits = clamp(soft_bits + delta, min_bits, max_bits). Writes each
 * quantizer's soft_bits; d_report (may be NULL): double[2] = (target, ratio). */
int nerf_acaq_update(const nerf_quantizer* qs, int n, const float* d_img_loss, double* d_best_loss,
                     int has_target, double target_metric, double bit_penalty, double* d_report, void* stream);

/* Int-packed hash tables for eval-mode rendering (quantizer in eval mode: value = (q - zp) * scale
 * with q the integer code, quantization.py:183-186). Level l occupies bytes [l*T*8, (l+1)*T*8) of
 * d_packed (nerf_quant_packed_bytes); its entries are stored densely from the region start with
 * the width of the level's record bits: <= 4 -> 1 byte per entry (two 4-bit codes), <= 8 -> 2,
 * <= 16 -> 4, else the dequantized fp32 pair (8). The layout never depends on the bit widths, so
 * no host round trip is needed.
 * pack: repacks exactly the levels whose record differs from d_prev_rec ([n_levels][8], device;
 *       initialise with NaNs or pass force=1 when the tables changed), then stores the records
 *       there; d_dirty: device int[n_levels] scratch.
 * fwd:  the gather + trilinear of nerf_hash_encode_fwd_q reading codes; bit-identical to it with
 *       the same eval-mode records. */
size_t nerf_quant_packed_bytes(int n_levels, int log2_T);
int nerf_quant_pack_tables(const float* const* d_tables, int n_levels, int log2_T, const float* d_qrec,
                           float* d_prev_rec, int force, int* d_dirty, void* d_packed, void* stream);
int nerf_hash_encode_fwd_packed(const float* d_xyz, int64_t n_points, const float* bbox_min3, const float* bbox_max3,
                                const float* level_res, int n_levels, int log2_T, const void* d_packed,
                                const float* d_qrec, float* d_feat, int64_t feat_stride_point,
                                int64_t feat_stride_level, uint8_t* d_keep, void* stream);

/* ---- structural priors on the device (combine_structural_losses_v2, structural_priors.py:374-451,
 *      with detect_planes :86-155, estimate_frame :16-77, manhattan_sdf_loss :194-256,
 *      structured_planarity_loss :259-318, spatial_normal_consistency_loss :321-371) -----------------
 * Three single-workgroup launches over n_rays <= NERF_PRIORS_MAX_RAYS rays, no host synchronisation
 * (capturable): prep (masks, counts, 10-round k-means, device 3x3 SVD unless cfg->usv), loss (frame,
 * the three losses; d_loss [1], d_parts [7] = floor, wall, general, manhattan, planarity,
 * consistency, total, may be NULL), bwd (d depth [n], d normals [n,3] from d_grad_loss [1]). The
 * workspace (nerf_priors_workspace_bytes) carries the state between the three calls.
 * Randomness: cfg->centres0 ([3,3] torch.randn), cfg->perm ([3][2*cap] randperm positions per class,
 * caps 100/100/50) and cfg->idx1 (torch.randint queries) replay the reference's draws; NULL draws them
 * from Philox (seed, offset | d_rng). cfg->usv ([21]: U, S, V of svd(centres^T)) replaces the device
 * SVD (prep's d_centres_out [9] gives the centres for it). d_coords NULL = sequential neighbours. */
#define NERF_PRIORS_MAX_RAYS 8192
typedef struct {
    int use_manhattan, use_planarity, use_consistency;
    float w_manhattan, w_planarity, w_consistency;
    const float* d_scale;              /* device multiplier of the weights (the ramp), NULL = 1 */
    float confidence_threshold;        /* ManhattanFrameEstimator (0.4 in combine) */
    float normal_threshold;            /* SemanticPlaneDetector (0.5 in combine) */
    const float* centres0;
    const int32_t* perm;
    const int32_t* idx1;
    const float* usv;
    uint64_t seed, offset;
    const uint64_t* d_rng;
} nerf_priors_config;

size_t nerf_priors_workspace_bytes(int64_t n_rays);
int nerf_priors_prep(const float* d_depth, const float* d_normals, const float* d_coords, int64_t n_rays,
                     const nerf_priors_config* cfg, void* d_workspace, size_t workspace_bytes, float* d_centres_out,
                     void* stream);
int nerf_priors_loss(const float* d_depth, const float* d_normals, const float* d_coords, int64_t n_rays,
                     const nerf_priors_config* cfg, void* d_workspace, size_t workspace_bytes, float* d_loss,
                     float* d_parts, void* stream);
/* ABI 12: nerf_priors_loss with *d_loss = *d_addend + total (one fp32 add: the training step's
 * `loss + structural_loss`, run_nerf.py:1131, without a launch of its own); d_addend NULL = total.
 * d_parts of both entries is written by the loss launch itself (no device copy after it). */
int nerf_priors_loss_add(const float* d_depth, const float* d_normals, const float* d_coords, int64_t n_rays,
                         const nerf_priors_config* cfg, void* d_workspace, size_t workspace_bytes,
                         const float* d_addend, float* d_loss, float* d_parts, void* stream);
int nerf_priors_bwd(const float* d_depth, const float* d_normals, const float* d_coords, int64_t n_rays,
                    const nerf_priors_config* cfg, void* d_workspace, size_t workspace_bytes,
                    const float* d_grad_loss, float* d_grad_depth, float* d_grad_normals, void* stream);

/* ---- structural priors (PocketNeRF/structural_priors.py:333-346, the ScanNet configuration) -----
 * For each query ray q (d_idx1[q], int64), the nearest OTHER ray in pixel space: d_xy [n,2] fp32
 * pixel coordinates (train()'s select_coords), self excluded, ties to the lowest index
 * (torch.argmin), d_idx2[q] its index (int64) and d_dist[q] = sqrt of the squared distance. */
int nerf_nearest_pixel(const float* d_xy, int64_t n, const int64_t* d_idx1, int64_t n_query, int64_t* d_idx2,
                       float* d_dist, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* NERF_HIP_H */
