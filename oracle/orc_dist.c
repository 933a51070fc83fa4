/* Distortion restatements (test infrastructure only).
 * SAD/SATD: src/dist.rs; SSE and cdef-dist: src/rdo.rs. */
#include <math.h>
#include <string.h>

#include "orc_common.h"

/* get_sad_ref, src/dist.rs:25-46: sum over rows of sum |a-b| as u32. */
uint32_t orc_get_sad(const void *org, ptrdiff_t org_stride, const void *ref,
                     ptrdiff_t ref_stride, int w, int h, int hbd) {
  uint32_t sum = 0;
  for (int r = 0; r < h; r++)
    for (int c = 0; c < w; c++) {
      int32_t d = orc_px(org, hbd, r * org_stride + c) -
                  orc_px(ref, hbd, r * ref_stride + c);
      sum += (uint32_t)(d < 0 ? -d : d);
    }
  return sum;
}

/* ---- SATD, reference form (src/dist.rs:197-328) ---------------------- */

/* One 1-D Hadamard over `n` points (n = 4 or 8) at element stride `s`,
 * butterfly order of hadamard4_1d / hadamard8_1d (src/dist.rs:208-256). */
static void had1d_i32(int32_t *d, int n, int s) {
  int32_t v[8];
  for (int k = 0; k < n; k++) v[k] = d[k * s];
  /* stage 1: pairs (0,1) (2,3) (4,5) (6,7) */
  for (int k = 0; k < n; k += 2) {
    int32_t a = v[k], b = v[k + 1];
    v[k] = a + b;
    v[k + 1] = a - b;
  }
  /* stage 2: pairs (0,2) (1,3) (4,6) (5,7) */
  for (int g = 0; g < n; g += 4)
    for (int k = 0; k < 2; k++) {
      int32_t a = v[g + k], b = v[g + k + 2];
      v[g + k] = a + b;
      v[g + k + 2] = a - b;
    }
  /* stage 3 (8-point only): pairs (k, k+4) */
  if (n == 8)
    for (int k = 0; k < 4; k++) {
      int32_t a = v[k], b = v[k + 4];
      v[k] = a + b;
      v[k + 4] = a - b;
    }
  for (int k = 0; k < n; k++) d[k * s] = v[k];
}

/* ---- SATD, generated-kernel emulation (build/kernel/gen/dist.rs) -----
 * Same butterfly network, but every lane is i16 (wrapping) even for u16
 * pixels (:193, :256), |x| is the (t+m)^m form (src/util/simd.rs:81-91),
 * the last horizontal stage is replaced by max(|a|,|b|)*2 in i16 (:234-240,
 * :337-341), lanes are cast i16 -> u32 with sign extension and summed with
 * u32 wrapping (:242-243, :343-352). */
static inline int16_t i16w(int32_t v) { return (int16_t)(uint16_t)(uint32_t)v; }
static inline int16_t i16abs(int16_t t) {
  int16_t m = (int16_t)(t >> 15);
  return i16w((int32_t)(int16_t)i16w(t + m) ^ m);
}

static uint32_t satd_chunk_gen(const int32_t *diff, int n) {
  int16_t d[64];
  for (int i = 0; i < n * n; i++) d[i] = i16w(diff[i]);
  /* vertical: all stages, over every column */
  for (int c = 0; c < n; c++) {
    int16_t v[8];
    for (int k = 0; k < n; k++) v[k] = d[k * n + c];
    for (int k = 0; k < n; k += 2) {
      int16_t a = v[k], b = v[k + 1];
      v[k] = i16w(a + b);
      v[k + 1] = i16w(a - b);
    }
    for (int g = 0; g < n; g += 4)
      for (int k = 0; k < 2; k++) {
        int16_t a = v[g + k], b = v[g + k + 2];
        v[g + k] = i16w(a + b);
        v[g + k + 2] = i16w(a - b);
      }
    if (n == 8)
      for (int k = 0; k < 4; k++) {
        int16_t a = v[k], b = v[k + 4];
        v[k] = i16w(a + b);
        v[k + 4] = i16w(a - b);
      }
    for (int k = 0; k < n; k++) d[k * n + c] = v[k];
  }
  /* horizontal: all but the last stage, then max(|a|,|b|)*2 */
  uint32_t sum = 0;
  for (int r = 0; r < n; r++) {
    int16_t v[8];
    for (int k = 0; k < n; k++) v[k] = d[r * n + k];
    for (int k = 0; k < n; k += 2) {
      int16_t a = v[k], b = v[k + 1];
      v[k] = i16w(a + b);
      v[k + 1] = i16w(a - b);
    }
    int half = n / 2;
    if (n == 8)
      for (int g = 0; g < n; g += 4)
        for (int k = 0; k < 2; k++) {
          int16_t a = v[g + k], b = v[g + k + 2];
          v[g + k] = i16w(a + b);
          v[g + k + 2] = i16w(a - b);
        }
    for (int k = 0; k < half; k++) {
      int16_t a = i16abs(v[k]), b = i16abs(v[k + half]);
      int16_t m = a > b ? a : b;
      int16_t t = i16w((int32_t)m * 2);
      sum += (uint32_t)(int32_t)t; /* i16 -> u32 `as`: sign-extends */
    }
  }
  return sum;
}

uint32_t orc_get_satd(const void *org, ptrdiff_t org_stride, const void *ref,
                      ptrdiff_t ref_stride, int w, int h, int hbd,
                      int emulate_gen) {
  int size = w < h ? w : h;
  if (size > 8) size = 8;
  uint64_t sum64 = 0;
  uint32_t sum32 = 0;
  int32_t buf[64];
  for (int cy = 0; cy < h; cy += size)
    for (int cx = 0; cx < w; cx += size) {
      for (int r = 0; r < size; r++)
        for (int c = 0; c < size; c++)
          buf[r * size + c] =
              orc_px(org, hbd, (cy + r) * org_stride + cx + c) -
              orc_px(ref, hbd, (cy + r) * ref_stride + cx + c);
      if (emulate_gen) {
        sum32 += satd_chunk_gen(buf, size);
      } else {
        /* hadamard2d: vertical (columns, stride = size) then horizontal */
        for (int c = 0; c < size; c++) had1d_i32(buf + c, size, size);
        for (int r = 0; r < size; r++) had1d_i32(buf + r * size, size, 1);
        for (int i = 0; i < size * size; i++)
          sum64 += (uint64_t)(buf[i] < 0 ? -(int64_t)buf[i] : buf[i]);
      }
    }
  int ln = orc_msb(size);
  if (emulate_gen) /* u32 arithmetic, build/kernel/gen/dist.rs:555-557 */
    return (sum32 + (uint32_t)((1u << ln) >> 1)) >> ln;
  return (uint32_t)((sum64 + ((1ull << ln) >> 1)) >> ln);
}

/* sse_wxh, src/rdo.rs:286-335 (raw per-importance-block values; the f64
 * bias multiplication stays with the caller, src/rdo.rs:325-331). */
int orc_sse_wxh(const void *a, ptrdiff_t sa, const void *b, ptrdiff_t sb,
                int w, int h, int xdec, int ydec, int hbd, uint64_t *out) {
  if ((w & 3) || (h & 3)) return -1; /* assert!(w & (MI_SIZE-1) == 0) */
  int imp_w = w < 8 ? w : 8, imp_h = h < 8 ? h : 8;
  int bw = imp_w >> xdec, bh = imp_h >> ydec;
  if (bw == 0 || bh == 0) return -1;
  int n = 0;
  for (int by = 0; by < h / bh; by++)
    for (int bx = 0; bx < w / bw; bx++) {
      uint64_t value = 0;
      for (int j = 0; j < bh; j++) {
        uint32_t row = 0;
        for (int i = 0; i < bw; i++) {
          ptrdiff_t r = by * bh + j, c = bx * bw + i;
          /* (i16(a) - i16(b)) as i32, squared as u32 */
          int32_t d = (int32_t)(int16_t)orc_px(a, hbd, r * sa + c) -
                      (int32_t)(int16_t)orc_px(b, hbd, r * sb + c);
          row += (uint32_t)w_mul(d, d);
        }
        value += row;
      }
      out[n++] = value;
    }
  return n;
}

/* cdef_dist_wxh_8x8 moments, src/rdo.rs:219-241. */
void orc_cdef_moments_8x8(const void *a, ptrdiff_t sa, const void *b,
                          ptrdiff_t sb, int hbd, int64_t out[5]) {
  int32_t sum_s = 0, sum_d = 0;
  int64_t sum_s2 = 0, sum_d2 = 0, sum_sd = 0;
  for (int j = 0; j < 8; j++)
    for (int i = 0; i < 8; i++) {
      int32_t s = orc_px(a, hbd, j * sa + i);
      int32_t d = orc_px(b, hbd, j * sb + i);
      sum_s += s;
      sum_d += d;
      sum_s2 += (int64_t)w_mul(s, s);
      sum_d2 += (int64_t)w_mul(d, d);
      sum_sd += (int64_t)w_mul(s, d);
    }
  out[0] = sum_s;
  out[1] = sum_d;
  out[2] = sum_s2;
  out[3] = sum_d2;
  out[4] = sum_sd;
}

/* f64 tail, src/rdo.rs:242-252. */
uint64_t orc_cdef_dist_from_moments(const int64_t m[5], int bit_depth) {
  int coeff_shift = bit_depth - 8;
  int64_t sum_s = m[0], sum_d = m[1];
  double svar = (double)(m[2] - ((sum_s * sum_s + 32) >> 6));
  double dvar = (double)(m[3] - ((sum_d * sum_d + 32) >> 6));
  double sse = (double)(m[3] + m[2] - 2 * m[4]);
  double ssim_boost =
      (4033.0 / 16384.0) *
      (svar + dvar + (double)(16384ll << (2 * coeff_shift))) /
      sqrt((double)(16265089ull << (4 * coeff_shift)) + svar * dvar);
  double v = sse * ssim_boost + 0.5;
  if (!(v > 0.0)) return 0; /* Rust `as u64`: NaN and negatives -> 0 */
  if (v >= 18446744073709551615.0) return UINT64_MAX;
  return (uint64_t)v;
}

/* compute_lookahead_intra_costs (src/api/internal.rs:680-765): per 8x8
 * importance block (w_in_imp_b = ceil(w / 8), src/encoder.rs:624-625),
 * PredictionMode::DC_PRED.predict_intra into a copy of the plane with the
 * tile rect at the block itself, so relative position (0, 0) ->
 * PredictionVariant::NONE -> pred_dc_128 (src/predict.rs:214-221, 552-557,
 * 623-633), then get_satd (src/dist.rs:197-328) of source vs prediction.
 * org: the plane's pixel (0, 0); stride in elements. */
void orc_lookahead_intra_costs(const void *org, ptrdiff_t stride, int w, int h, int hbd, int bd,
                               uint32_t *out) {
  const int nbx = (w + 7) / 8, nby = (h + 7) / 8;
  uint16_t pred16[64];
  uint8_t pred8[64];
  for (int i = 0; i < 64; i++) {  /* pred_dc_128: 128 << (bit_depth - 8) */
    pred16[i] = (uint16_t)(128u << (bd - 8));
    pred8[i] = (uint8_t)(128u << (bd - 8));
  }
  const size_t px = hbd ? 2 : 1;
  for (int by = 0; by < nby; by++)
    for (int bx = 0; bx < nbx; bx++) {
      const uint8_t *o = (const uint8_t *)org + ((ptrdiff_t)by * 8 * stride + bx * 8) * px;
      out[by * nbx + bx] =
          orc_get_satd(o, stride, hbd ? (const void *)pred16 : (const void *)pred8, 8, 8, 8, hbd, 0);
    }
}
