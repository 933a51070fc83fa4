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
