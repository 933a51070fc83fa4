/* CPU oracle (test infrastructure only): the importance propagation of
 * compute_block_importances (src/api/internal.rs:823-1010), one (frame,
 * reference) pass.  f32 arithmetic in the reference's operation order; the
 * library is built with -ffp-contract=off, so no product-sum is fused
 * (Rust never fuses). */
#include <math.h>

#include "orc_common.h"

#define IMP_B 8                       /* IMPORTANCE_BLOCK_SIZE */
#define MV_UNITS 8                    /* MV_UNITS_PER_PIXEL */
#define B_MV (IMP_B * MV_UNITS)       /* BLOCK_SIZE_IN_MV_UNITS */
#define AREA_MV (B_MV * B_MV)         /* BLOCK_AREA_IN_MV_UNITS */

/* org / ref: the planes' pixel (0, 0), strides in elements; mvs,
 * intra_costs, importances: [h_imp][w_imp] of the frame (lookahead_mvs
 * sampled at [2y][2x], lookahead_intra_costs, block_importances);
 * ref_importances: the reference frame's block_importances, accumulated in
 * place in source-block raster order, each source's four targets in the
 * order top-left, top-right, bottom-left, bottom-right. */
void orc_propagate_importances(const void *org, ptrdiff_t org_stride, const void *ref,
                               ptrdiff_t ref_stride, int w_imp, int h_imp, int hbd,
                               const orc_mv *mvs, const uint32_t *intra_costs,
                               const float *importances, int n_unique,
                               float *ref_importances) {
  const size_t px = hbd ? 2 : 1;
  for (int y = 0; y < h_imp; y++)
    for (int x = 0; x < w_imp; x++) {
      const orc_mv mv = mvs[y * w_imp + x];
      const int64_t rx = (int64_t)x * B_MV + mv.col;
      const int64_t ry = (int64_t)y * B_MV + mv.row;
      /* region at (rx / 8, ry / 8): isize division truncates toward zero */
      const int64_t px_x = rx / MV_UNITS, px_y = ry / MV_UNITS;
      const uint8_t *o = (const uint8_t *)org + ((ptrdiff_t)y * IMP_B * org_stride + x * IMP_B) * px;
      const uint8_t *r = (const uint8_t *)ref + ((ptrdiff_t)px_y * ref_stride + px_x) * px;
      const float inter_cost = (float)orc_get_satd(o, org_stride, r, ref_stride, IMP_B, IMP_B, hbd, 0);
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
