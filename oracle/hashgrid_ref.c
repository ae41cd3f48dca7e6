/*
 * hashgrid_ref.c — plain-C CPU restatement of the hash-grid encoding, TEST INFRASTRUCTURE ONLY.
 *
 * Bit-exact restatement of the integer/index path and the fp32 trilinear blend of
 *   get_voxel_vertices  PocketNeRF/utils.py:95-117
 *   hash                PocketNeRF/utils.py:13-24
 *   trilinear_interp    PocketNeRF/hash_encoding.py:56-80
 *   HashEmbedder.forward PocketNeRF/hash_encoding.py:82-107
 * Compiled by __graft_entry__.build() with gcc -O2 -ffp-contract=off (no FMA contraction) into
 * oracle/_build/libhashgrid_ref.so; pinned against tests/golden/f2_voxel.npz and f3_hash_fwd.npz by
 * tests/test_abi.py. Only tests and bench.py's cpu_baseline may load it.
 */
#include <math.h>
#include <stdint.h>

static uint32_t spatial_hash3(uint32_t x, uint32_t y, uint32_t z, uint32_t mask) {
    return (x * 1u ^ y * 2654435761u ^ z * 805459861u) & mask;
}

/* xyz [n,3]; tables [L][2^log2_T][2]; feat [n][2L]; keep [n]; idx [n][L][8] (may be NULL);
 * vmin/vmax [n][L][3] (may be NULL). */
void hashgrid_ref_fwd(const float* xyz, int64_t n, const float* bmin, const float* bmax, const float* res, int L,
                      int log2_T, const float* tables, float* feat, uint8_t* keep, int32_t* idx, float* vmin_out,
                      float* vmax_out) {
    const uint32_t mask = (uint32_t)((1u << log2_T) - 1u);
    const int64_t T = (int64_t)1 << log2_T;
    for (int64_t p = 0; p < n; ++p) {
        const float* x = xyz + 3 * p;
        int inside = 1;
        for (int lvl = 0; lvl < L; ++lvl) {
            int base[3];
            float w[3];
            for (int a = 0; a < 3; ++a) {
                const float lo = bmin[a], hi = bmax[a];
                float mn = x[a] < hi ? x[a] : hi;
                float mx = mn > lo ? mn : lo;
                if (lvl == 0 && !(x[a] == mx)) inside = 0;
                float xc = x[a] < lo ? lo : (x[a] > hi ? hi : x[a]);
                volatile float cell = (hi - lo) / res[lvl];
                volatile float q = (xc - lo) / cell;
                base[a] = (int)floorf(q);
                volatile float prod = (float)base[a] * cell;
                volatile float v0 = prod + lo;
                volatile float v1 = v0 + cell;
                volatile float num = x[a] - v0;
                volatile float den = v1 - v0;
                w[a] = num / den;
                if (vmin_out) vmin_out[(p * L + lvl) * 3 + a] = v0;
                if (vmax_out) vmax_out[(p * L + lvl) * 3 + a] = v1;
            }
            const float* tab = tables + (int64_t)lvl * T * 2;
            float e[8][2];
            for (int c = 0; c < 8; ++c) {
                const uint32_t h = spatial_hash3((uint32_t)base[0] + ((c >> 2) & 1), (uint32_t)base[1] + ((c >> 1) & 1),
                                                 (uint32_t)base[2] + (c & 1), mask);
                if (idx) idx[(p * L + lvl) * 8 + c] = (int32_t)h;
                e[c][0] = tab[2 * h];
                e[c][1] = tab[2 * h + 1];
            }
            const float ox = 1.0f - w[0], oy = 1.0f - w[1], oz = 1.0f - w[2];
            for (int f = 0; f < 2; ++f) {
                volatile float t0, t1;
                float c00, c01, c10, c11, c0, c1;
                t0 = e[0][f] * ox; t1 = e[4][f] * w[0]; c00 = t0 + t1;
                t0 = e[1][f] * ox; t1 = e[5][f] * w[0]; c01 = t0 + t1;
                t0 = e[2][f] * ox; t1 = e[6][f] * w[0]; c10 = t0 + t1;
                t0 = e[3][f] * ox; t1 = e[7][f] * w[0]; c11 = t0 + t1;
                t0 = c00 * oy; t1 = c10 * w[1]; c0 = t0 + t1;
                t0 = c01 * oy; t1 = c11 * w[1]; c1 = t0 + t1;
                t0 = c0 * oz; t1 = c1 * w[2];
                feat[p * 2 * L + 2 * lvl + f] = t0 + t1;
            }
        }
        keep[p] = (uint8_t)inside;
    }
}
