/* Motion-search restatements (test infrastructure only), src/me.rs. */
#include "orc_common.h"

/* get_mv_rate / diff_to_rate, src/me.rs:1006-1021 */
static uint32_t diff_to_rate(int16_t diff, int allow_hp) {
  int16_t d = allow_hp ? diff : (int16_t)(diff >> 1);
  if (d == 0) return 0;
  uint16_t a = (uint16_t)(d < 0 ? -d : d);
  return 2u * (16u - (uint32_t)(__builtin_clz((uint32_t)a) - 16));
}
uint32_t orc_get_mv_rate(orc_mv a, orc_mv b, int allow_hp) {
  return diff_to_rate((int16_t)(a.row - b.row), allow_hp) +
         diff_to_rate((int16_t)(a.col - b.col), allow_hp);
}

/* full_search, src/me.rs:943-990: candidate windows at (x, y) for
 * y = y_lo, y_lo+step, ... <= y_hi (outer) and x likewise (inner);
 * cost = 256*sad + rate*lambda, strict `<` keeps the first minimum. */
void orc_full_search(const void *org, ptrdiff_t org_stride, const void *ref,
                     ptrdiff_t ref_stride, int hbd, int po_x, int po_y,
                     int x_lo, int x_hi, int y_lo, int y_hi, int blk_w,
                     int blk_h, int step, uint32_t lambda, orc_mv pmv0,
                     orc_mv pmv1, int allow_hp, orc_mv *best_mv,
                     uint64_t *lowest_cost) {
  size_t px = hbd ? 2 : 1;
  const char *o = (const char *)org + (po_y * org_stride + po_x) * (ptrdiff_t)px;
  for (int y = y_lo; y <= y_hi; y += step)
    for (int x = x_lo; x <= x_hi; x += step) {
      const char *r = (const char *)ref + (y * ref_stride + x) * (ptrdiff_t)px;
      uint32_t sad =
          orc_get_sad(o, org_stride, r, ref_stride, blk_w, blk_h, hbd);
      orc_mv mv = {(int16_t)(8 * (y - po_y)), (int16_t)(8 * (x - po_x))};
      uint32_t r1 = orc_get_mv_rate(mv, pmv0, allow_hp);
      uint32_t r2 = orc_get_mv_rate(mv, pmv1, allow_hp);
      uint32_t rate = r1 < r2 + 1 ? r1 : r2 + 1;
      uint64_t cost = 256ull * sad + (uint64_t)rate * lambda;
      if (cost < *lowest_cost) {
        *lowest_cost = cost;
        *best_mv = mv;
      }
    }
}

/* get_mv_rd_cost + compute_mv_rd_cost, src/me.rs:787-856. */
static uint64_t mv_rd_cost(const orc_ds_ctx *c, orc_mv mv) {
  if (mv.col < c->mvx_min || mv.col > c->mvx_max || mv.row < c->mvy_min ||
      mv.row > c->mvy_max)
    return UINT64_MAX;
  size_t px = c->hbd ? 2 : 1;
  const char *o = (const char *)c->org +
                  ((ptrdiff_t)c->po_y * c->org_stride + c->po_x) * (ptrdiff_t)px;
  uint32_t dist;
  if (!c->subpel) {
    /* Rust i16 `/` truncates toward zero, as C does */
    const char *r = (const char *)c->ref +
                    ((ptrdiff_t)(c->po_y + mv.row / 8) * c->ref_stride +
                     (c->po_x + mv.col / 8)) * (ptrdiff_t)px;
    dist = c->satd ? orc_get_satd(o, c->org_stride, r, c->ref_stride, c->w,
                                  c->h, c->hbd, 0)
                   : orc_get_sad(o, c->org_stride, r, c->ref_stride, c->w,
                                 c->h, c->hbd);
  } else {
    /* predict_inter / get_params, src/predict.rs:267-283 (luma: dec 0) */
    int ys = 3 + c->ref_ydec, xs = 3 + c->ref_xdec;
    int roff = (int)mv.row >> ys, coff = (int)mv.col >> xs;
    int rf = ((int)mv.row - roff * (1 << ys)) << (4 - ys);
    int cf = ((int)mv.col - coff * (1 << xs)) << (4 - xs);
    /* PlaneSlice::clamp, src/frame/plane.rs:521-533 */
    int qx = c->po_x + coff - 3, qy = c->po_y + roff - 3;
    if (qx > c->ref_width) qx = c->ref_width;
    if (qx < -c->ref_xorigin) qx = -c->ref_xorigin;
    if (qy > c->ref_height) qy = c->ref_height;
    if (qy < -c->ref_yorigin) qy = -c->ref_yorigin;
    const char *s = (const char *)c->ref +
                    ((ptrdiff_t)(qy + 3) * c->ref_stride + (qx + 3)) * (ptrdiff_t)px;
    uint16_t tmp[128 * 128];
    orc_put_8tap(tmp, c->w, s, c->ref_stride, c->w, c->h, cf, rf, 0, 0,
                 c->bit_depth, c->hbd, 0);
    dist = c->satd ? orc_get_satd(o, c->org_stride, tmp, c->w, c->w, c->h,
                                  c->hbd, 0)
                   : orc_get_sad(o, c->org_stride, tmp, c->w, c->w, c->h,
                                 c->hbd);
  }
  uint32_t r1 = orc_get_mv_rate(mv, c->pmv[0], c->allow_hp);
  uint32_t r2 = orc_get_mv_rate(mv, c->pmv[1], c->allow_hp);
  uint32_t rate = r1 < r2 + 1 ? r1 : r2 + 1;
  return 256ull * dist + (uint64_t)rate * c->lambda;
}

/* diamond_me_search + get_best_predictor, src/me.rs:655-785. */
void orc_diamond_search(const orc_ds_ctx *c, const orc_mv *pred, int n_pred,
                        orc_mv *best_mv, uint64_t *best_cost) {
  orc_mv center = {0, 0};
  uint64_t center_cost = UINT64_MAX;
  for (int p = 0; p < n_pred; p++) {
    uint64_t cost = mv_rd_cost(c, pred[p]);
    if (cost < center_cost) {
      center = pred[p];
      center_cost = cost;
    }
  }
  static const int16_t pat[4][2] = {{1, 0}, {0, 1}, {-1, 0}, {0, -1}};
  int16_t radius = c->subpel ? 4 : 16;
  int16_t radius_end = c->subpel ? (c->allow_hp ? 1 : 2) : 8;
  for (;;) {
    uint64_t best = UINT64_MAX;
    orc_mv bmv = {0, 0};
    for (int p = 0; p < 4; p++) {
      orc_mv cand = {(int16_t)(center.row + radius * pat[p][0]),
                     (int16_t)(center.col + radius * pat[p][1])};
      uint64_t cost = mv_rd_cost(c, cand);
      if (cost < best) {
        best = cost;
        bmv = cand;
      }
    }
    if (center_cost <= best) {
      if (radius == radius_end) break;
      radius /= 2;
    } else {
      center = bmv;
      center_cost = best;
    }
  }
  *best_mv = center;
  *best_cost = center_cost;
}

/* telescopic_subpel_search (src/me.rs:858-941): 3x3 grids around the
 * running best at steps 8, 4, 2 (and 1 with allow_hp); the grid centre
 * of a step is fixed, every candidate in (i, j) raster order updates the
 * best on a strict '<'. */
void orc_telescopic_subpel(const orc_ds_ctx *c, orc_mv *best_mv, uint64_t *lowest_cost) {
  const int nsteps = c->allow_hp ? 4 : 3;
  for (int st = 0; st < nsteps; st++) {
    const int16_t step = (int16_t)(8 >> st);
    const orc_mv center = *best_mv;
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        if (i == 1 && j == 1) continue;
        orc_mv cand = {(int16_t)(center.row + step * (i - 1)), (int16_t)(center.col + step * (j - 1))};
        /* out-of-range candidates are skipped (mv_rd_cost returns MAX) */
        uint64_t cost = mv_rd_cost(c, cand);
        if (cost < *lowest_cost) {
          *lowest_cost = cost;
          *best_mv = cand;
        }
      }
  }
}

/* tx-domain distortion of encode_tx_block (src/encoder.rs:1210-1224):
 * sum over the coded area of ((c - rc) * (c - rc)) as u64 -- i32 wrapping
 * square, sign-extended -- then rounded by 2 * (3 - get_log_tx_scale)
 * (src/quantize.rs:34-39) bits. */
uint64_t orc_tx_dist(const int32_t *coeffs, const int32_t *rcoeffs, int coded_area,
                     int tx_w, int tx_h) {
  uint64_t d = 0;
  for (int i = 0; i < coded_area; i++) {
    int32_t e = (int32_t)((uint32_t)coeffs[i] - (uint32_t)rcoeffs[i]);
    int32_t sq = (int32_t)((uint32_t)e * (uint32_t)e);
    d += (uint64_t)(int64_t)sq;
  }
  const int area = tx_w * tx_h;
  const int log_scale = (area > 256) + (area > 1024);
  const int bits = 2 * (3 - log_scale);
  return (d + (1ull << (bits - 1))) >> bits;
}

/* get_subset_predictors, src/me.rs:82-174: zero; the coarse MVs
 * quantize_to_fullpel'd; subsets A and B from the tile's motion field
 * (left, top, top-right, each pushed when non-zero, then their mean
 * quantize_to_fullpel'd when non-zero); subset C from the reference frame's
 * field (left, top, right, bottom, co-located, each when non-zero).
 * tile: the tile's field (4x4 units, row pitch tp, tc columns), the block
 * at (bx, by) in it; prev: the frame-size field of the reference frame
 * (pitch pp, fc x fr 4x4 units; NULL: none), the block at frame (fx, fy).
 * Returns the count (<= ORC_MAX_PRED). */
int orc_subset_predictors(int bx, int by, const orc_mv *cmvs, int ncmv, const orc_mv *tile,
                          int tp, int tc, const orc_mv *prev, int pp, int fc, int fr, int fx,
                          int fy, orc_mv *out) {
  int n = 0;
  out[n++] = (orc_mv){0, 0};
  for (int i = 0; i < ncmv; i++)
    out[n++] = (orc_mv){(int16_t)((cmvs[i].row / 8) * 8), (int16_t)((cmvs[i].col / 8) * 8)};
  orc_mv med[3];
  int nm = 0;
  if (bx > 0) {
    const orc_mv l = tile[(size_t)by * tp + bx - 1];
    med[nm++] = l;
    if (l.row || l.col) out[n++] = l;
  }
  if (by > 0) {
    const orc_mv t = tile[(size_t)(by - 1) * tp + bx];
    med[nm++] = t;
    if (t.row || t.col) out[n++] = t;
    if (bx < tc - 1) {
      const orc_mv tr = tile[(size_t)(by - 1) * tp + bx + 1];
      med[nm++] = tr;
      if (tr.row || tr.col) out[n++] = tr;
    }
  }
  if (nm) {
    /* MotionVector Add / Div<i16>: i16 arithmetic, truncating division */
    int16_t sr = 0, sc = 0;
    for (int i = 0; i < nm; i++) {
      sr = (int16_t)(sr + med[i].row);
      sc = (int16_t)(sc + med[i].col);
    }
    sr = (int16_t)(sr / nm);
    sc = (int16_t)(sc / nm);
    const orc_mv q = {(int16_t)((sr / 8) * 8), (int16_t)((sc / 8) * 8)};
    if (q.row || q.col) out[n++] = q;
  }
  if (prev) {
#define ORC_PREV(x, y)                                  \
  do {                                                  \
    const orc_mv v_ = prev[(size_t)(y) * pp + (x)];     \
    if (v_.row || v_.col) out[n++] = v_;                \
  } while (0)
    if (fx > 0) ORC_PREV(fx - 1, fy);
    if (fy > 0) ORC_PREV(fx, fy - 1);
    if (fx < fc - 1) ORC_PREV(fx + 1, fy);
    if (fy < fr - 1) ORC_PREV(fx, fy + 1);
    ORC_PREV(fx, fy);
#undef ORC_PREV
  }
  return n;
}
