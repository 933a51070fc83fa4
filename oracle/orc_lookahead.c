/* CPU oracle (test infrastructure only): the importance propagation of
 * compute_block_importances (src/api/internal.rs:823-1010), one (frame,
 * reference) pass.  f32 arithmetic in the reference's operation order; the
 * library is built with -ffp-contract=off, so no product-sum is fused
 * (Rust never fuses). */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "orc_common.h"

#define IMP_B 8                       /* IMPORTANCE_BLOCK_SIZE */
#define MV_UNITS 8                    /* MV_UNITS_PER_PIXEL */
#define B_MV (IMP_B * MV_UNITS)       /* BLOCK_SIZE_IN_MV_UNITS */
#define AREA_MV (B_MV * B_MV)         /* BLOCK_AREA_IN_MV_UNITS */

/* One (frame, reference) pass over precomputed inter costs: mvs,
 * inter_costs, intra_costs, importances: [h_imp][w_imp] of the frame
 * (lookahead_mvs sampled at [2y][2x], get_satd of the source block against
 * the reference block at the MV, lookahead_intra_costs, block_importances);
 * ref_importances: the reference frame's block_importances, accumulated in
 * place in source-block raster order, each source's four targets in the
 * order top-left, top-right, bottom-left, bottom-right (:900-1045). */
void orc_propagate_importances_costs(int w_imp, int h_imp, const orc_mv *mvs,
                                     const uint32_t *inter_costs, const uint32_t *intra_costs,
                                     const float *importances, int n_unique,
                                     float *ref_importances) {
  for (int y = 0; y < h_imp; y++)
    for (int x = 0; x < w_imp; x++) {
      const orc_mv mv = mvs[y * w_imp + x];
      const int64_t rx = (int64_t)x * B_MV + mv.col;
      const int64_t ry = (int64_t)y * B_MV + mv.row;
      const float inter_cost = (float)inter_costs[y * w_imp + x];
      const float intra_cost = (float)intra_costs[y * w_imp + x];
      const float future = importances[y * w_imp + x];
      /* f32::max returns the other operand when one is NaN (0/0), as fmaxf */
      const float fraction = fmaxf(1.0f - inter_cost / intra_cost, 0.0f);
      const float amount = (intra_cost + future) * fraction / (float)n_unique;
      const int64_t tlx = (rx - (rx < 0 ? B_MV - 1 : 0)) / B_MV * B_MV;
      const int64_t tly = (ry - (ry < 0 ? B_MV - 1 : 0)) / B_MV * B_MV;
      const int64_t trx = tlx + B_MV, bly = tly + B_MV;
      const int64_t tx[4] = {tlx, trx, tlx, trx}, ty[4] = {tly, tly, bly, bly};
      const int64_t fx[4] = {trx - rx, rx + B_MV - trx, trx - rx, rx + B_MV - trx};
      const int64_t fy[4] = {bly - ry, bly - ry, ry + B_MV - bly, ry + B_MV - bly};
      for (int k = 0; k < 4; k++) {
        const float f = (float)(fx[k] * fy[k]) / (float)AREA_MV;
        const int64_t bx = tx[k] / B_MV, by = ty[k] / B_MV;
        if (bx >= 0 && by >= 0 && bx < w_imp && by < h_imp)
          ref_importances[by * w_imp + bx] += amount * f;
      }
    }
}

/* get_satd of every source block against the reference block at its MV
 * (region at (rx / 8, ry / 8): isize division truncates toward zero). */
void orc_importance_inter_costs(const void *org, ptrdiff_t org_stride, const void *ref,
                                ptrdiff_t ref_stride, int w_imp, int h_imp, int hbd,
                                const orc_mv *mvs, uint32_t *inter_costs) {
  const size_t px = hbd ? 2 : 1;
  for (int y = 0; y < h_imp; y++)
    for (int x = 0; x < w_imp; x++) {
      const orc_mv mv = mvs[y * w_imp + x];
      const int64_t px_x = ((int64_t)x * B_MV + mv.col) / MV_UNITS;
      const int64_t px_y = ((int64_t)y * B_MV + mv.row) / MV_UNITS;
      const uint8_t *o = (const uint8_t *)org + ((ptrdiff_t)y * IMP_B * org_stride + x * IMP_B) * px;
      const uint8_t *r = (const uint8_t *)ref + ((ptrdiff_t)px_y * ref_stride + px_x) * px;
      inter_costs[y * w_imp + x] = orc_get_satd(o, org_stride, r, ref_stride, IMP_B, IMP_B, hbd, 0);
    }
}

/* org / ref: the planes' pixel (0, 0), strides in elements; the rest as
 * orc_propagate_importances_costs. */
void orc_propagate_importances(const void *org, ptrdiff_t org_stride, const void *ref,
                               ptrdiff_t ref_stride, int w_imp, int h_imp, int hbd,
                               const orc_mv *mvs, const uint32_t *intra_costs,
                               const float *importances, int n_unique,
                               float *ref_importances) {
  uint32_t *inter = malloc((size_t)w_imp * h_imp * sizeof(uint32_t));
  if (!inter) return;
  orc_importance_inter_costs(org, org_stride, ref, ref_stride, w_imp, h_imp, hbd, mvs, inter);
  orc_propagate_importances_costs(w_imp, h_imp, mvs, inter, intra_costs, importances, n_unique,
                                  ref_importances);
  free(inter);
}

/* f32::log2 as the reference gets it on x86-64 Linux: glibc's log2f
 * (sysdeps/ieee754/flt-32/e_log2f.c, its published algorithm): x = 2^k z,
 * z in [0x3f330000, 2 * that) as a float, one of 16 subintervals i by the top
 * mantissa bits, r = z / c_i - 1 with the table's (1 / c_i, log2 c_i), and
 * log2 x = k + log2 c_i + a degree-4 polynomial in r, all in double, rounded
 * once to float.  The table and coefficients are glibc's (__log2f_data);
 * tests/test_lookahead.py checks this function against the host's log2f.
 * The importance argument 1 + imp / intra is >= 1, finite or +inf. */
static const double LOG2F_T[16][2] = {
    {0x1.661ec79f8f3bep+0, -0x1.efec65b963019p-2}, {0x1.571ed4aaf883dp+0, -0x1.b0b6832d4fca4p-2},
    {0x1.49539f0f010b0p+0, -0x1.7418b0a1fb77bp-2}, {0x1.3c995b0b80385p+0, -0x1.39de91a6dcf7bp-2},
    {0x1.30d190c8864a5p+0, -0x1.01d9bf3f2b631p-2}, {0x1.25e227b0b8ea0p+0, -0x1.97c1d1b3b7af0p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.2f9e393af3c9fp-3}, {0x1.12358f08ae5bap+0, -0x1.960cbbf788d5cp-4},
    {0x1.0953f419900a7p+0, -0x1.a6f9db6475fcep-5}, {0x1.0000000000000p+0, 0x0.0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.338ca9f24f53dp-4}, {0x1.ca4b31f026aa0p-1, 0x1.476a9543891bap-3},
    {0x1.b2036576afce6p-1, 0x1.e840b4ac4e4d2p-3}, {0x1.9c2d163a1aa2dp-1, 0x1.40645f0c6651cp-2},
    {0x1.886e6037841edp-1, 0x1.88e9c2c1b9ff8p-2}, {0x1.767dcf5534862p-1, 0x1.ce0a44eb17bccp-2}};
static const double LOG2F_A[4] = {-0x1.712b6f70a7e4dp-2, 0x1.ecabf496832e0p-2,
                                  -0x1.715479ffae3dep-1, 0x1.715475f35c8b8p+0};

float orc_log2f(float x) {
  uint32_t ix;
  memcpy(&ix, &x, 4);
  if (ix == 0x3f800000u) return 0.0f;
  if (ix >= 0x7f800000u || ix == 0) return log2f(x); /* inf, NaN, negatives, zero */
  if (ix < 0x00800000u) { /* subnormal: normalise */
    const float y = x * 0x1p23f;
    memcpy(&ix, &y, 4);
    ix -= 23u << 23;
  }
  const uint32_t tmp = ix - 0x3f330000u;
  const int i = (int)((tmp >> 19) % 16);
  const uint32_t iz = ix - (tmp & 0xff800000u);
  const int k = (int32_t)tmp >> 23;
  float zf;
  memcpy(&zf, &iz, 4);
  const double z = zf, invc = LOG2F_T[i][0], logc = LOG2F_T[i][1];
  const double r = fma(z, invc, -1.0);
  const double y0 = logc + (double)k, r2 = r * r;
  double y = fma(LOG2F_A[1], r, LOG2F_A[2]);
  y = fma(LOG2F_A[0], r2, y);
  const double p = fma(LOG2F_A[3], r, y0);
  return (float)fma(y, r2, p);
}

/* Test hook: the floats lo, lo + step, ... < hi where orc_log2f differs from
 * the host's log2f (bit patterns); returns the count. */
uint64_t orc_log2f_mismatches(uint32_t lo, uint32_t hi, uint32_t step) {
  uint64_t bad = 0;
  for (uint64_t u = lo; u < hi; u += step) {
    const uint32_t v = (uint32_t)u;
    float x, a, b;
    memcpy(&x, &v, 4);
    a = orc_log2f(x);
    b = log2f(x);
    if (memcmp(&a, &b, 4)) bad++;
  }
  return bad;
}
