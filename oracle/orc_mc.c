/* Motion-compensation restatements (test infrastructure only).
 * Follows src/mc.rs:70-408 (put_8tap_ref / prep_8tap_ref / mc_avg_ref). */
#include "orc_common.h"

/* SUBPEL_FILTERS, src/mc.rs:70-179 (6 sets x 16 fracs x 8 taps). */
static const int32_t SUBPEL[6][16][8] = {
    {{0, 0, 0, 128, 0, 0, 0, 0},     {0, 2, -6, 126, 8, -2, 0, 0},
     {0, 2, -10, 122, 18, -4, 0, 0}, {0, 2, -12, 116, 28, -8, 2, 0},
     {0, 2, -14, 110, 38, -10, 2, 0}, {0, 2, -14, 102, 48, -12, 2, 0},
     {0, 2, -16, 94, 58, -12, 2, 0}, {0, 2, -14, 84, 66, -12, 2, 0},
     {0, 2, -14, 76, 76, -14, 2, 0}, {0, 2, -12, 66, 84, -14, 2, 0},
     {0, 2, -12, 58, 94, -16, 2, 0}, {0, 2, -12, 48, 102, -14, 2, 0},
     {0, 2, -10, 38, 110, -14, 2, 0}, {0, 2, -8, 28, 116, -12, 2, 0},
     {0, 0, -4, 18, 122, -10, 2, 0}, {0, 0, -2, 8, 126, -6, 2, 0}},
    {{0, 0, 0, 128, 0, 0, 0, 0},   {0, 2, 28, 62, 34, 2, 0, 0},
     {0, 0, 26, 62, 36, 4, 0, 0},  {0, 0, 22, 62, 40, 4, 0, 0},
     {0, 0, 20, 60, 42, 6, 0, 0},  {0, 0, 18, 58, 44, 8, 0, 0},
     {0, 0, 16, 56, 46, 10, 0, 0}, {0, -2, 16, 54, 48, 12, 0, 0},
     {0, -2, 14, 52, 52, 14, -2, 0}, {0, 0, 12, 48, 54, 16, -2, 0},
     {0, 0, 10, 46, 56, 16, 0, 0}, {0, 0, 8, 44, 58, 18, 0, 0},
     {0, 0, 6, 42, 60, 20, 0, 0},  {0, 0, 4, 40, 62, 22, 0, 0},
     {0, 0, 4, 36, 62, 26, 0, 0},  {0, 0, 2, 34, 62, 28, 2, 0}},
    {{0, 0, 0, 128, 0, 0, 0, 0},         {-2, 2, -6, 126, 8, -2, 2, 0},
     {-2, 6, -12, 124, 16, -6, 4, -2},   {-2, 8, -18, 120, 26, -10, 6, -2},
     {-4, 10, -22, 116, 38, -14, 6, -2}, {-4, 10, -22, 108, 48, -18, 8, -2},
     {-4, 10, -24, 100, 60, -20, 8, -2}, {-4, 10, -24, 90, 70, -22, 10, -2},
     {-4, 12, -24, 80, 80, -24, 12, -4}, {-2, 10, -22, 70, 90, -24, 10, -4},
     {-2, 8, -20, 60, 100, -24, 10, -4}, {-2, 8, -18, 48, 108, -22, 10, -4},
     {-2, 6, -14, 38, 116, -22, 10, -4}, {-2, 6, -10, 26, 120, -18, 8, -2},
     {-2, 4, -6, 16, 124, -12, 6, -2},   {0, 2, -2, 8, 126, -6, 2, -2}},
    {{0, 0, 0, 128, 0, 0, 0, 0},  {0, 0, 0, 120, 8, 0, 0, 0},
     {0, 0, 0, 112, 16, 0, 0, 0}, {0, 0, 0, 104, 24, 0, 0, 0},
     {0, 0, 0, 96, 32, 0, 0, 0},  {0, 0, 0, 88, 40, 0, 0, 0},
     {0, 0, 0, 80, 48, 0, 0, 0},  {0, 0, 0, 72, 56, 0, 0, 0},
     {0, 0, 0, 64, 64, 0, 0, 0},  {0, 0, 0, 56, 72, 0, 0, 0},
     {0, 0, 0, 48, 80, 0, 0, 0},  {0, 0, 0, 40, 88, 0, 0, 0},
     {0, 0, 0, 32, 96, 0, 0, 0},  {0, 0, 0, 24, 104, 0, 0, 0},
     {0, 0, 0, 16, 112, 0, 0, 0}, {0, 0, 0, 8, 120, 0, 0, 0}},
    {{0, 0, 0, 128, 0, 0, 0, 0},     {0, 0, -4, 126, 8, -2, 0, 0},
     {0, 0, -8, 122, 18, -4, 0, 0},  {0, 0, -10, 116, 28, -6, 0, 0},
     {0, 0, -12, 110, 38, -8, 0, 0}, {0, 0, -12, 102, 48, -10, 0, 0},
     {0, 0, -14, 94, 58, -10, 0, 0}, {0, 0, -12, 84, 66, -10, 0, 0},
     {0, 0, -12, 76, 76, -12, 0, 0}, {0, 0, -10, 66, 84, -12, 0, 0},
     {0, 0, -10, 58, 94, -14, 0, 0}, {0, 0, -10, 48, 102, -12, 0, 0},
     {0, 0, -8, 38, 110, -12, 0, 0}, {0, 0, -6, 28, 116, -10, 0, 0},
     {0, 0, -4, 18, 122, -8, 0, 0},  {0, 0, -2, 8, 126, -4, 0, 0}},
    {{0, 0, 0, 128, 0, 0, 0, 0},   {0, 0, 30, 62, 34, 2, 0, 0},
     {0, 0, 26, 62, 36, 4, 0, 0},  {0, 0, 22, 62, 40, 4, 0, 0},
     {0, 0, 20, 60, 42, 6, 0, 0},  {0, 0, 18, 58, 44, 8, 0, 0},
     {0, 0, 16, 56, 46, 10, 0, 0}, {0, 0, 14, 54, 48, 12, 0, 0},
     {0, 0, 12, 52, 52, 12, 0, 0}, {0, 0, 12, 48, 54, 14, 0, 0},
     {0, 0, 10, 46, 56, 16, 0, 0}, {0, 0, 8, 44, 58, 18, 0, 0},
     {0, 0, 6, 42, 60, 20, 0, 0},  {0, 0, 4, 40, 62, 22, 0, 0},
     {0, 0, 4, 36, 62, 26, 0, 0},  {0, 0, 2, 34, 62, 30, 0, 0}}};

/* get_filter, src/mc.rs:201-210: BILINEAR (3) or length > 4 keep the mode,
 * otherwise the 4-tap set min(mode,1)+4. */
const int32_t *orc_get_filter(int mode, int frac, int length) {
  int idx = (mode == 3 || length > 4) ? mode : ((mode < 1 ? mode : 1) + 4);
  return SUBPEL[idx][frac];
}

/* run_filter, src/mc.rs:187-198: sum_i f[i] * src[i*stride]. */
static int32_t run_filter(const void *src, int hbd, ptrdiff_t base,
                          ptrdiff_t stride, const int32_t *f) {
  int32_t s = 0;
  for (int i = 0; i < 8; i++)
    s = w_add(s, w_mul(f[i], orc_px(src, hbd, base + i * stride)));
  return s;
}
static int32_t run_filter_i16(const int16_t *p, ptrdiff_t stride,
                              const int32_t *f) {
  int32_t s = 0;
  for (int i = 0; i < 8; i++) s = w_add(s, w_mul(f[i], p[i * stride]));
  return s;
}

/* Final pixel conversion. Reference: clamp to [0, max] (src/mc.rs:244-245).
 * Generated u8 kernels: max(0) then `as u8` (wraps mod 256). */
static inline int32_t to_pixel(int32_t v, int32_t maxv, int hbd, int emu) {
  if (emu && !hbd) return v < 0 ? 0 : (v & 0xff);
  return clamp_i32(v, 0, maxv);
}

/* put_8tap_ref, src/mc.rs:213-307.  The (x,y) case filters 8-column
 * groups through an i16 intermediate of height h+7 (:271-304); that is
 * column-wise identical to a full-width intermediate, which is used here. */
void orc_put_8tap(void *dst, ptrdiff_t dst_stride, const void *src,
                  ptrdiff_t src_stride, int w, int h, int col_frac,
                  int row_frac, int mode_x, int mode_y, int bit_depth,
                  int hbd, int emulate_gen) {
  const int32_t *yf = orc_get_filter(mode_y, row_frac, h);
  const int32_t *xf = orc_get_filter(mode_x, col_frac, w);
  int32_t maxv = (1 << bit_depth) - 1;
  int ib = 4 - (bit_depth == 12 ? 2 : 0);
  if (col_frac == 0 && row_frac == 0) {
    for (int r = 0; r < h; r++)
      for (int c = 0; c < w; c++)
        orc_px_store(dst, hbd, r * dst_stride + c,
                     orc_px(src, hbd, r * src_stride + c));
  } else if (col_frac == 0) {
    for (int r = 0; r < h; r++)
      for (int c = 0; c < w; c++) {
        int32_t v = run_filter(src, hbd, (r - 3) * src_stride + c,
                               src_stride, yf);
        orc_px_store(dst, hbd, r * dst_stride + c,
                     to_pixel(round_shift(v, 7), maxv, hbd, emulate_gen));
      }
  } else if (row_frac == 0) {
    for (int r = 0; r < h; r++)
      for (int c = 0; c < w; c++) {
        int32_t v = run_filter(src, hbd, r * src_stride + c - 3, 1, xf);
        v = round_shift(round_shift(v, 7 - ib), ib);
        orc_px_store(dst, hbd, r * dst_stride + c,
                     to_pixel(v, maxv, hbd, emulate_gen));
      }
  } else {
    int16_t mid[(128 + 7) * 128];
    for (int r = 0; r < h + 7; r++)
      for (int c = 0; c < w; c++)
        mid[r * w + c] = (int16_t)round_shift(
            run_filter(src, hbd, (r - 3) * src_stride + c - 3, 1, xf),
            7 - ib);
    for (int r = 0; r < h; r++)
      for (int c = 0; c < w; c++) {
        int32_t v = round_shift(run_filter_i16(mid + r * w + c, w, yf),
                                7 + ib);
        orc_px_store(dst, hbd, r * dst_stride + c,
                     to_pixel(v, maxv, hbd, emulate_gen));
      }
  }
}

/* prep_8tap_ref, src/mc.rs:310-387: i16 intermediates, stride w, no clamp. */
void orc_prep_8tap(int16_t *tmp, const void *src, ptrdiff_t src_stride, int w,
                   int h, int col_frac, int row_frac, int mode_x, int mode_y,
                   int bit_depth, int hbd) {
  const int32_t *yf = orc_get_filter(mode_y, row_frac, h);
  const int32_t *xf = orc_get_filter(mode_x, col_frac, w);
  int ib = 4 - (bit_depth == 12 ? 2 : 0);
  if (col_frac == 0 && row_frac == 0) {
    for (int r = 0; r < h; r++)
      for (int c = 0; c < w; c++)
        tmp[r * w + c] =
            (int16_t)((int16_t)orc_px(src, hbd, r * src_stride + c) << ib);
  } else if (col_frac == 0) {
    for (int r = 0; r < h; r++)
      for (int c = 0; c < w; c++)
        tmp[r * w + c] = (int16_t)round_shift(
            run_filter(src, hbd, (r - 3) * src_stride + c, src_stride, yf),
            7 - ib);
  } else if (row_frac == 0) {
    for (int r = 0; r < h; r++)
      for (int c = 0; c < w; c++)
        tmp[r * w + c] = (int16_t)round_shift(
            run_filter(src, hbd, r * src_stride + c - 3, 1, xf), 7 - ib);
  } else {
    int16_t mid[(128 + 7) * 128];
    for (int r = 0; r < h + 7; r++)
      for (int c = 0; c < w; c++)
        mid[r * w + c] = (int16_t)round_shift(
            run_filter(src, hbd, (r - 3) * src_stride + c - 3, 1, xf),
            7 - ib);
    for (int r = 0; r < h; r++)
      for (int c = 0; c < w; c++)
        tmp[r * w + c] =
            (int16_t)round_shift(run_filter_i16(mid + r * w + c, w, yf), 7);
  }
}

/* mc_avg_ref, src/mc.rs:389-408 (+ generated u8 quirk, gen/mc.rs:815-823). */
void orc_mc_avg(void *dst, ptrdiff_t dst_stride, const int16_t *tmp1,
                const int16_t *tmp2, int w, int h, int bit_depth, int hbd,
                int emulate_gen) {
  int32_t maxv = (1 << bit_depth) - 1;
  int ib = 4 - (bit_depth == 12 ? 2 : 0);
  for (int r = 0; r < h; r++)
    for (int c = 0; c < w; c++) {
      int32_t v = round_shift((int32_t)tmp1[r * w + c] + tmp2[r * w + c],
                              ib + 1);
      orc_px_store(dst, hbd, r * dst_stride + c,
                   to_pixel(v, maxv, hbd, emulate_gen));
    }
}
