// Ray generation and train()'s per-iteration pixel batch on the device.
//
//   nerf_sample_rays  run_nerf.py:973-1004 (use_batching = False): N_rand distinct pixels of one
//                     training image (optionally inside the precrop window), their rays
//                     (run_nerf_helpers.get_rays :311-320, evaluated only at those pixels) and
//                     target colours, in one launch. The reference rebuilds every ray of the
//                     image, draws np.random.choice(H*W, N_rand, replace=False) on the host and
//                     gathers (plus a 7.7 MB host->device copy of the image) per iteration.
//   random = 0        rays of grid cells 0..n-1 in row-major order: get_rays of a whole image
//                     (render(c2w=...) / render_path) or of the crop window.
//
// Sampling without replacement: cell index = pi(t) for lane t, where pi is a keyed 4-round
// Feistel permutation of [0, 2^(2k)) restricted to [0, n_cells) by cycle walking (a bijection on
// [0, n_cells), so the N_rand cells are distinct by construction); keys from (seed, offset).
#include "common.h"

namespace nerf {

struct Cam {
    float c2w[12];
    float fx, fy, cx, cy;
};

__device__ __forceinline__ uint32_t mix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x7feb352du;
    h ^= h >> 15;
    h *= 0x846ca68bu;
    h ^= h >> 16;
    return h;
}

__device__ __forceinline__ uint32_t feistel_perm(uint32_t x, int half_bits, const uint32_t (&key)[4]) {
    const uint32_t mask = (1u << half_bits) - 1u;
    uint32_t L = x >> half_bits, R = x & mask;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t nl = R;
        R = (L ^ mix32(R ^ key[r])) & mask;
        L = nl;
    }
    return (L << half_bits) | R;
}

__global__ void __launch_bounds__(256) sample_rays_kernel(Cam cam, int W_img, int r0, int c0, int cw, int64_t n_cells,
                                                          int64_t n_rays, int random, int half_bits, uint32_t k0,
                                                          uint32_t k1, uint32_t k2, uint32_t k3,
                                                          const float* __restrict__ image, int channels,
                                                          float* __restrict__ rays_o, float* __restrict__ rays_d,
                                                          float* __restrict__ target, int32_t* __restrict__ coords) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_rays) return;
    int64_t cell = t;
    if (random) {
        const uint32_t key[4] = {k0, k1, k2, k3};
        uint32_t x = (uint32_t)t;
        do {
            x = feistel_perm(x, half_bits, key);
        } while ((int64_t)x >= n_cells);
        cell = x;
    }
    const int row = r0 + (int)(cell / cw), col = c0 + (int)(cell % cw);
    // dirs = [(i - cx)/fx, -(j - cy)/fy, -1]; rays_d = sum(dirs[..., None, :] * c2w[:3,:3], -1)
    const float i = (float)col, j = (float)row;
    const float d0 = (i - cam.cx) / cam.fx;
    const float d1 = -(j - cam.cy) / cam.fy;
    const float d2 = -1.0f;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float p0 = d0 * cam.c2w[4 * a + 0], p1 = d1 * cam.c2w[4 * a + 1], p2 = d2 * cam.c2w[4 * a + 2];
        rays_d[3 * t + a] = (p0 + p1) + p2;
        rays_o[3 * t + a] = cam.c2w[4 * a + 3];
    }
    if (target) {
        const float* px = image + ((int64_t)row * W_img + col) * channels;
#pragma unroll
        for (int a = 0; a < 3; ++a) target[3 * t + a] = px[a];
    }
    if (coords) {
        coords[2 * t] = row;
        coords[2 * t + 1] = col;
    }
}

// render()'s prologue (run_nerf.py:115-140): viewdirs = d / |d| (before NDC), optional ndc_rays
// (run_nerf_helpers.py:333-350, near plane 1), and the packed ray batch [o, d, near, far, viewdir].
// The NDC coefficients -1/(W/(2f)), -1/(H/(2f)) are python doubles in the reference that torch
// rounds to float32 before the tensor ops; the host passes them that way.
struct PackArgs {
    const float* o;
    const float* d;
    int64_t n;
    float near, far;
    int ndc, viewdirs;
    float cw, ch;          // float32(-1/(W/(2 focal))), float32(-1/(H/(2 focal)))
    float* out;
    int stride;            // 8 or 11
    nerf_zero_range zero[NERF_MAX_ZERO_RANGES];   // fills folded into this launch (render's first)
    int n_zero;
};

__device__ __forceinline__ void pack_ray(const PackArgs& a, int64_t r) {
    float ox = a.o[3 * r], oy = a.o[3 * r + 1], oz = a.o[3 * r + 2];
    float dx = a.d[3 * r], dy = a.d[3 * r + 1], dz = a.d[3 * r + 2];
    float* dst = a.out + r * a.stride;
    if (a.viewdirs) {
        const float nrm = sqrtf((dx * dx + dy * dy) + dz * dz);
        dst[8] = dx / nrm;
        dst[9] = dy / nrm;
        dst[10] = dz / nrm;
    }
    if (a.ndc) {
        const float t = -(1.0f + oz) / dz;
        ox = ox + t * dx;
        oy = oy + t * dy;
        oz = oz + t * dz;
        const float o0 = a.cw * ox / oz, o1 = a.ch * oy / oz, o2 = 1.0f + 2.0f / oz;
        const float d0 = a.cw * (dx / dz - ox / oz), d1 = a.ch * (dy / dz - oy / oz), d2 = -2.0f / oz;
        ox = o0; oy = o1; oz = o2;
        dx = d0; dy = d1; dz = d2;
    }
    dst[0] = ox; dst[1] = oy; dst[2] = oz;
    dst[3] = dx; dst[4] = dy; dst[5] = dz;
    dst[6] = a.near;
    dst[7] = a.far;
}

__global__ void __launch_bounds__(256) rays_pack_kernel(PackArgs a) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < a.n) pack_ray(a, t);
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int k = 0; k < a.n_zero; ++k) {
        float* z = a.zero[k].ptr;
        for (int64_t i = t; i < a.zero[k].n; i += stride) z[i] = 0.0f;
    }
}

__host__ __device__ __forceinline__ uint32_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return (uint32_t)((z ^ (z >> 31)) >> 16);
}

// nerf_sample_rays with the image, its camera and the draw's (seed, offset) chosen on the device:
// sel = {image index, seed, offset} (int64, e.g. a captured step's per-replay slots), so one
// captured launch draws a new batch every replay. Same keys, permutation and ray arithmetic as the
// host-argument launch (bit-identical for the same image, seed and offset).
__global__ void __launch_bounds__(256) sample_rays_sel_kernel(const nerf_camera* __restrict__ cams,
                                                              const float* __restrict__ images, int64_t n_images,
                                                              int64_t image_elems, int W_img, int r0, int c0, int cw,
                                                              int64_t n_cells, int64_t n_rays, int half_bits,
                                                              const int64_t* __restrict__ sel, int channels,
                                                              float* __restrict__ rays_o, float* __restrict__ rays_d,
                                                              float* __restrict__ target, int32_t* __restrict__ coords) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_rays) return;
    int64_t img = sel[0] % n_images;
    if (img < 0) img += n_images;
    uint64_t s = (uint64_t)sel[1] ^ ((uint64_t)sel[2] * 0xD1B54A32D192ED03ull);
    const uint32_t k0 = splitmix(s), k1 = splitmix(s), k2 = splitmix(s), k3 = splitmix(s);
    const nerf_camera& cm = cams[img];
    Cam c;
#pragma unroll
    for (int k = 0; k < 12; ++k) c.c2w[k] = cm.c2w[k];
    c.fx = cm.fx; c.fy = cm.fy; c.cx = cm.cx; c.cy = cm.cy;
    // one body with the host-argument kernel: a thread of a one-ray grid at ray t
    const uint32_t key[4] = {k0, k1, k2, k3};
    uint32_t x = (uint32_t)t;
    do {
        x = feistel_perm(x, half_bits, key);
    } while ((int64_t)x >= n_cells);
    const int64_t cell = x;
    const int row = r0 + (int)(cell / cw), col = c0 + (int)(cell % cw);
    const float i = (float)col, j = (float)row;
    const float d0 = (i - c.cx) / c.fx;
    const float d1 = -(j - c.cy) / c.fy;
    const float d2 = -1.0f;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float p0 = d0 * c.c2w[4 * a + 0], p1 = d1 * c.c2w[4 * a + 1], p2 = d2 * c.c2w[4 * a + 2];
        rays_d[3 * t + a] = (p0 + p1) + p2;
        rays_o[3 * t + a] = c.c2w[4 * a + 3];
    }
    if (target) {
        const float* px = images + img * image_elems + ((int64_t)row * W_img + col) * channels;
#pragma unroll
        for (int a = 0; a < 3; ++a) target[3 * t + a] = px[a];
    }
    if (coords) {
        coords[2 * t] = row;
        coords[2 * t + 1] = col;
    }
}

}  // namespace nerf

using namespace nerf;

extern "C" int nerf_sample_rays_sel(const nerf_camera* d_cams, const float* d_images, int64_t n_images, int H, int W,
                                    int channels, int crop_r0, int crop_c0, int crop_h, int crop_w, int64_t n_rays,
                                    const int64_t* d_sel, float* d_rays_o, float* d_rays_d, float* d_target,
                                    int32_t* d_coords, void* stream) {
    NERF_REQUIRE(d_cams && d_sel && d_rays_o && d_rays_d && n_images > 0, "sample_rays_sel: null argument");
    NERF_REQUIRE(H > 0 && W > 0 && crop_r0 >= 0 && crop_c0 >= 0 && crop_h > 0 && crop_w > 0 &&
                 crop_r0 + crop_h <= H && crop_c0 + crop_w <= W, "sample_rays_sel: crop window outside the %dx%d image",
                 H, W);
    const int64_t n_cells = (int64_t)crop_h * crop_w;
    NERF_REQUIRE(n_rays >= 0 && n_rays <= n_cells, "sample_rays_sel: %lld rays from %lld pixels (no replacement)",
                 (long long)n_rays, (long long)n_cells);
    NERF_REQUIRE(n_cells <= (int64_t(1) << 30), "sample_rays_sel: crop window too large");
    NERF_REQUIRE(!d_target || (d_images && channels >= 3), "sample_rays_sel: target needs images with >= 3 channels");
    if (n_rays == 0) return NERF_OK;
    int bits = 2;
    while ((int64_t(1) << bits) < n_cells) bits += 2;
    hipLaunchKernelGGL(sample_rays_sel_kernel, dim3(blocks_for(n_rays, 256)), dim3(256), 0, as_stream(stream), d_cams,
                       d_images, n_images, (int64_t)H * W * channels, W, crop_r0, crop_c0, crop_w, n_cells, n_rays,
                       bits / 2, d_sel, channels, d_rays_o, d_rays_d, d_target, d_coords);
    NERF_CHECK_LAUNCH("sample_rays_sel");
    return NERF_OK;
}

extern "C" int nerf_sample_rays(const nerf_camera* cam, int H, int W, int crop_r0, int crop_c0, int crop_h,
                                int crop_w, int64_t n_rays, int random, uint64_t seed, uint64_t offset,
                                const float* d_image, int channels, float* d_rays_o, float* d_rays_d, float* d_target,
                                int32_t* d_coords, void* stream) {
    NERF_REQUIRE(cam && d_rays_o && d_rays_d, "sample_rays: null argument");
    NERF_REQUIRE(H > 0 && W > 0 && crop_r0 >= 0 && crop_c0 >= 0 && crop_h > 0 && crop_w > 0 &&
                 crop_r0 + crop_h <= H && crop_c0 + crop_w <= W, "sample_rays: crop window outside the %dx%d image", H, W);
    const int64_t n_cells = (int64_t)crop_h * crop_w;
    NERF_REQUIRE(n_rays >= 0 && n_rays <= n_cells, "sample_rays: %lld rays from %lld pixels (no replacement)",
                 (long long)n_rays, (long long)n_cells);
    NERF_REQUIRE(n_cells <= (int64_t(1) << 30), "sample_rays: crop window too large");
    NERF_REQUIRE(!d_target || (d_image && channels >= 3), "sample_rays: target needs an image with >= 3 channels");
    if (n_rays == 0) return NERF_OK;
    int bits = 2;
    while ((int64_t(1) << bits) < n_cells) bits += 2;   // even width: two halves of bits/2
    uint64_t s = seed ^ (offset * 0xD1B54A32D192ED03ull);
    const uint32_t k0 = splitmix(s), k1 = splitmix(s), k2 = splitmix(s), k3 = splitmix(s);
    Cam c;
    for (int k = 0; k < 12; ++k) c.c2w[k] = cam->c2w[k];
    c.fx = cam->fx; c.fy = cam->fy; c.cx = cam->cx; c.cy = cam->cy;
    hipLaunchKernelGGL(sample_rays_kernel, dim3(blocks_for(n_rays, 256)), dim3(256), 0, as_stream(stream), c, W,
                       crop_r0, crop_c0, crop_w, n_cells, n_rays, random ? 1 : 0, bits / 2, k0, k1, k2, k3, d_image,
                       channels, d_rays_o, d_rays_d, d_target, d_coords);
    NERF_CHECK_LAUNCH("sample_rays");
    return NERF_OK;
}

extern "C" int nerf_rays_pack_z(const float* d_rays_o, const float* d_rays_d, int64_t n_rays, float near, float far,
                                int ndc, float ndc_coef_w, float ndc_coef_h, int use_viewdirs, float* d_out,
                                const nerf_zero_range* zeros, int n_zeros, void* stream) {
    NERF_REQUIRE(n_rays >= 0 && (n_rays == 0 || (d_rays_o && d_rays_d && d_out)), "rays_pack: bad args");
    NERF_REQUIRE(n_zeros >= 0 && n_zeros <= NERF_MAX_ZERO_RANGES && (n_zeros == 0 || zeros),
                 "rays_pack: %d zero ranges (at most %d)", n_zeros, NERF_MAX_ZERO_RANGES);
    PackArgs a{d_rays_o, d_rays_d, n_rays, near, far, ndc ? 1 : 0, use_viewdirs ? 1 : 0, ndc_coef_w, ndc_coef_h,
               d_out, use_viewdirs ? 11 : 8, {}, 0};
    int64_t most = 0;
    for (int k = 0; k < n_zeros; ++k) {
        NERF_REQUIRE(zeros[k].n >= 0 && (zeros[k].n == 0 || zeros[k].ptr), "rays_pack: zero range %d", k);
        if (zeros[k].n == 0) continue;
        a.zero[a.n_zero++] = zeros[k];
        most = std::max(most, zeros[k].n);
    }
    if (n_rays == 0 && a.n_zero == 0) return NERF_OK;
    // the rays' threads, or enough for 16 values each of the largest range (at most 1024 blocks)
    const unsigned blocks = std::max(blocks_for(n_rays, 256), std::min(1024u, blocks_for(most, 256 * 16)));
    hipLaunchKernelGGL(rays_pack_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), a);
    NERF_CHECK_LAUNCH("rays_pack");
    return NERF_OK;
}

extern "C" int nerf_rays_pack(const float* d_rays_o, const float* d_rays_d, int64_t n_rays, float near, float far,
                              int ndc, float ndc_coef_w, float ndc_coef_h, int use_viewdirs, float* d_out,
                              void* stream) {
    return nerf_rays_pack_z(d_rays_o, d_rays_d, n_rays, near, far, ndc, ndc_coef_w, ndc_coef_h, use_viewdirs, d_out,
                            nullptr, 0, stream);
}
