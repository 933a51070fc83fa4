/* Loop restoration, self-guided filter only (test infrastructure only):
 * the CPU restatement the HIP path (rav1e_amd/csrc/rv_lrf.hip) is checked
 * against.
 *
 *   RestorationState::new          src/lrf.rs:1197-1343   orc_lrf_config
 *   setup_integral_image           src/lrf.rs:483-580     orc_lrf_integral
 *     (VertPaddedIter / HorzPaddedIter, :336-481)
 *   sgrproj_sum_finish / get_integral_square  :305-334
 *   native::sgrproj_box_ab_r1/_r2, box_f_r0/_r1/_r2  :156-302
 *   sgrproj_stripe_filter          src/lrf.rs:582-748     orc_sgr_stripe_filter
 *   sgrproj_solve                  src/lrf.rs:764-965     orc_sgr_solve
 *   lrf_filter_frame               src/lrf.rs:1345-1444   orc_lrf_filter_frame
 *   count_lrf_switchable           src/context.rs:3560-3594  orc_lrf_rate
 *   write_lrf's state updates      src/context.rs:3596-3659  orc_lrf_commit
 *   symbol_bits / frac_compute / count_subexp(_with_ref)
 *                                  src/ec.rs:366-388, 559-590, 632-725
 *
 * rav1e evaluates the Wiener filter nowhere (`unreachable!()` in
 * rdo_loop_decision and count_lrf_switchable): units are None or Sgrproj.
 * Integer arithmetic wraps like the reference's release build (u32 sums of
 * the integral image, u32 products in sgrproj_sum_finish); sgrproj_solve's
 * f64 sums of integer products are exact, so they are kept in int64 and
 * converted once, then the reference's f64 operations follow in order. */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "orc_common.h"

#define SGRPROJ_RST_BITS 4
#define SGRPROJ_PRJ_BITS 7
#define SGRPROJ_SGR_BITS 8
#define SGRPROJ_MTABLE_BITS 20
#define SGRPROJ_RECIP_BITS 12
#define SGRPROJ_PARAMS_BITS 4
#define SGRPROJ_PRJ_SUBEXP_K 4
#define OD_BITRES 3

/* SGRPROJ_PARAMS_S (src/lrf.rs:61-78): (r2 strength, r1 strength) per set */
const uint32_t ORC_SGRPROJ_PARAMS_S[16][2] = {
    {140, 3236}, {112, 2158}, {93, 1618}, {80, 1438}, {70, 1295}, {58, 1177},
    {47, 1079},  {37, 996},   {30, 925},  {25, 863},  {0, 2589},  {0, 1618},
    {0, 1177},   {0, 925},    {56, 0},    {22, 0}};
static const int XQD_MIN[2] = {-96, -32}, XQD_MID[2] = {-32, 31}, XQD_MAX[2] = {31, 95};

static int imin(int a, int b) { return a < b ? a : b; }
static int imax(int a, int b) { return a > b ? a : b; }
static int iclamp(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }
static int ilog_sz(size_t v) { int n = 0; while (v) { n++; v >>= 1; } return n; }

/* ---- RestorationState::new (src/lrf.rs:1197-1343) ------------------------
 * tiled: the frame has more than one tile (fi.tiling.cols > 1 || rows > 1);
 * 64x64 superblocks.  Per plane: unit size, the unit's superblock shifts,
 * the stripe height, units across and down. */
void orc_lrf_config(int width, int height, int xdec, int ydec, int base_q_idx, int tiled,
                    int tile_w_sb, int tile_h_sb, orc_lrf_plane_cfg out[3]) {
  const int stripe_uv_decimate = xdec > 0 && ydec > 0;
  const int y_sb_log2 = 6, uv_sb_h_log2 = y_sb_log2 - xdec, uv_sb_v_log2 = y_sb_log2 - ydec;
  /* enable_large_lru && enable_restoration */
  const int lrf_base_shift = base_q_idx > 200 ? 0 : base_q_idx > 160 ? 1 : 2;
  int lrf_chroma_shift = 0;
  if (stripe_uv_decimate) {
    if (lrf_base_shift == 2) {
      lrf_chroma_shift = 1;
    } else {
      const int u = 1 << (8 - lrf_base_shift);
      const int unshifted = ((width >> xdec) - 1) % u <= u / 2 || ((height >> ydec) - 1) % u <= u / 2;
      const int shifted =
          ((width >> xdec) - 1) % (u >> 1) <= u / 4 || ((height >> ydec) - 1) % (u >> 1) <= u / 4;
      lrf_chroma_shift = unshifted && !shifted ? 1 : 0;
    }
  }
  int y_unit = 1 << (8 - lrf_base_shift), uv_unit = 1 << (8 - (lrf_base_shift + lrf_chroma_shift));
  if (tiled) {
    const int tzh = __builtin_ctz((unsigned)tile_w_sb), tzv = __builtin_ctz((unsigned)tile_h_sb);
    y_unit = imin(y_unit, 1 << (y_sb_log2 + imin(tzh, tzv)));
    uv_unit = imin(uv_unit, imin(1 << (uv_sb_h_log2 + tzh), 1 << (uv_sb_v_log2 + tzv)));
  }
  const int y_log2 = ilog_sz((size_t)y_unit) - 1, uv_log2 = ilog_sz((size_t)uv_unit) - 1;
  const int y_cols = imax((width + (y_unit >> 1)) / y_unit, 1);
  const int y_rows = imax((height + (y_unit >> 1)) / y_unit, 1);
  const int uv_cols = imax((((width + ((1 << xdec) >> 1)) >> xdec) + (uv_unit >> 1)) / uv_unit, 1);
  const int uv_rows = imax((((height + ((1 << ydec) >> 1)) >> ydec) + (uv_unit >> 1)) / uv_unit, 1);
  out[0] = (orc_lrf_plane_cfg){y_unit, y_log2 - y_sb_log2, y_log2 - y_sb_log2, 64, y_cols, y_rows};
  for (int p = 1; p < 3; p++)
    out[p] = (orc_lrf_plane_cfg){uv_unit,  uv_log2 - uv_sb_h_log2, uv_log2 - uv_sb_v_log2,
                                 stripe_uv_decimate ? 32 : 64, uv_cols, uv_rows};
}

/* ---- setup_integral_image (src/lrf.rs:483-580) ---------------------------
 * Plane coordinates: the stripe starts at (x0, y0) of its planes (cdeffed
 * and deblocked share the geometry; pixel (x, y) at base[y * stride + x],
 * strides cs / ds);
 * crop_w / crop_h: the width / height left from (x0, y0) to the crop
 * (frame) edge.  Image row r reads plane row y0 - 4 + r clamped to the crop
 * ([0, y0 + crop_h)) and to the stripe's extension [y0 - 2, y0 + sh + 1]
 * (sh = stripe_h rounded up to even): cdeffed inside [y0, y0 + sh),
 * deblocked outside (VertPaddedIter).  Image column c reads plane column
 * x0 - 4 + c clamped to [0, x0 + stripe_w + min(3, crop_w - stripe_w))
 * (HorzPaddedIter over the row's unique elements).  ii / sq: (sh + 6) rows
 * x (stripe_w + 7) columns at pitch iis, u32 wrapping prefix sums. */
void orc_lrf_integral(const void *cdeffed, ptrdiff_t cs, const void *deblocked, ptrdiff_t ds,
                      int hbd, int x0, int y0, int crop_w, int crop_h, int stripe_w, int stripe_h,
                      uint32_t *ii, uint32_t *sq, int iis) {
  const int sh = stripe_h + (stripe_h & 1);
  const int rows = 4 + sh + 2, cols = 4 + stripe_w + 3;
  const int xmax = x0 + stripe_w + imin(3, crop_w - stripe_w) - 1;
  const int crop = crop_h + y0;
  for (int r = 0; r < rows; r++) {
    const int cy = iclamp(y0 - 4 + r, 0, crop - 1);
    const int ly = iclamp(cy, y0 - 2, y0 + sh + 1);
    const int inside = ly >= y0 && ly < y0 + sh;
    const void *src = inside ? cdeffed : deblocked;
    const ptrdiff_t stride = inside ? cs : ds;
    uint32_t sum = 0, ssum = 0;
    for (int c = 0; c < cols; c++) {
      const int x = iclamp(x0 - 4 + c, 0, xmax);
      const uint32_t v = (uint32_t)orc_px(src, hbd, (ptrdiff_t)ly * stride + x);
      sum += v;
      ssum += v * v;
      ii[r * iis + c] = sum + (r ? ii[(r - 1) * iis + c] : 0);
      sq[r * iis + c] = ssum + (r ? sq[(r - 1) * iis + c] : 0);
    }
  }
}

/* get_integral_square (:326-334): rows (y, y + d], columns (x, x + d] */
static uint32_t isq(const uint32_t *ii, int s, int x, int y, int d) {
  return ii[y * s + x] + ii[(y + d) * s + x + d] - ii[(y + d) * s + x] - ii[y * s + x + d];
}
/* sgrproj_sum_finish (:305-323) */
static void sum_finish(uint32_t ssq, uint32_t sum, uint32_t n, uint32_t one_over_n, uint32_t s,
                       int bdm8, uint32_t *a_out, uint32_t *b_out) {
  const uint32_t scaled_ssq = (ssq + ((1u << (2 * bdm8)) >> 1)) >> (2 * bdm8);
  const uint32_t scaled_sum = (sum + ((1u << bdm8) >> 1)) >> bdm8;
  const int32_t pd = w_sub((int32_t)(scaled_ssq * n), (int32_t)(scaled_sum * scaled_sum));
  const uint32_t p = (uint32_t)(pd > 0 ? pd : 0);
  const uint32_t z = (p * s + ((1u << SGRPROJ_MTABLE_BITS) >> 1)) >> SGRPROJ_MTABLE_BITS;
  const uint32_t a = z >= 255 ? 256 : z == 0 ? 1 : ((z << SGRPROJ_SGR_BITS) + z / 2) / (z + 1);
  const uint32_t b = ((1u << SGRPROJ_SGR_BITS) - a) * sum * one_over_n;
  *a_out = a;
  *b_out = (b + ((1u << SGRPROJ_RECIP_BITS) >> 1)) >> SGRPROJ_RECIP_BITS;
}
/* sgrproj_box_ab_r1 / _r2 (:167-226): an (a, b) row for w + 2 columns at
 * image row y; r1 reads the image from (1, 1) on (the caller's offset) */
static void box_ab(int r, uint32_t *af, uint32_t *bf, const uint32_t *ii, const uint32_t *sq,
                   int iis, int y, int w, uint32_t s, int bdm8) {
  const int off = r == 1 ? iis + 1 : 0, d = 2 * r + 1;
  for (int x = 0; x < w + 2; x++)
    sum_finish(isq(sq + off, iis, x, y, d), isq(ii + off, iis, x, y, d), (uint32_t)(d * d),
               r == 1 ? 455 : 164, s, bdm8, &af[x], &bf[x]);
}

/* The f rows of one row pair (the body shared by sgrproj_stripe_filter and
 * sgrproj_solve, :611-733 / :796-905): for every row y of the stripe,
 * f_r2 (every other row computed, both rows of a pair from it) and f_r1,
 * into f2 / f1 ([h][w]); rows clipped to h. */
static void sgr_f(int set, int bdm8, const uint32_t *ii, const uint32_t *sq, int iis, int w, int h,
                  const void *cd, ptrdiff_t cs, int hbd, uint32_t *f2, uint32_t *f1) {
  const uint32_t s2 = ORC_SGRPROJ_PARAMS_S[set][0], s1 = ORC_SGRPROJ_PARAMS_S[set][1];
  const int W2 = w + 2;
  uint32_t *a2 = calloc(2 * (size_t)W2, 4), *b2 = calloc(2 * (size_t)W2, 4);
  uint32_t *a1 = calloc(3 * (size_t)W2, 4), *b1 = calloc(3 * (size_t)W2, 4);
  const int shift = 5 + SGRPROJ_SGR_BITS - SGRPROJ_RST_BITS, shifto = 4 + SGRPROJ_SGR_BITS - SGRPROJ_RST_BITS;
  const int sr = SGRPROJ_RST_BITS;
#define PX(x, y) ((uint32_t)orc_px(cd, hbd, (ptrdiff_t)(y) * cs + (x)))
  if (s2) box_ab(2, a2, b2, ii, sq, iis, 0, w, s2, bdm8);
  if (s1) {
    box_ab(1, a1, b1, ii, sq, iis, 0, w, s1, bdm8);
    box_ab(1, a1 + W2, b1 + W2, ii, sq, iis, 1, w, s1, bdm8);
  }
  for (int y = 0; y < h; y += 2) {
    uint32_t *fr2[2] = {f2 + (size_t)y * w, f2 + (size_t)imin(y + 1, h - 1) * w};
    if (s2) {
      uint32_t *an = a2 + ((y / 2 + 1) % 2) * W2, *bn = b2 + ((y / 2 + 1) % 2) * W2;
      box_ab(2, an, bn, ii, sq, iis, y + 2, w, s2, bdm8);
      const uint32_t *ap0 = a2 + ((y / 2) % 2) * W2, *bp0 = b2 + ((y / 2) % 2) * W2;
      const uint32_t *ap1 = an, *bp1 = bn;
      for (int x = 0; x < w; x++) {
        const uint32_t a = 5 * (ap0[x] + ap0[x + 2]) + 6 * ap0[x + 1];
        const uint32_t b = 5 * (bp0[x] + bp0[x + 2]) + 6 * bp0[x + 1];
        const uint32_t ao = 5 * (ap1[x] + ap1[x + 2]) + 6 * ap1[x + 1];
        const uint32_t bo = 5 * (bp1[x] + bp1[x + 2]) + 6 * bp1[x + 1];
        const uint32_t v = (a + ao) * PX(x, y) + b + bo;
        const uint32_t f0 = (v + ((1u << shift) >> 1)) >> shift;
        /* (box_f_r2 also forms row y + 1 past an odd stripe's end; unused) */
        const uint32_t vo = ao * (y + 1 < h ? PX(x, y + 1) : 0) + bo;
        const uint32_t fo = (vo + ((1u << shifto) >> 1)) >> shifto;
        fr2[0][x] = f0;
        if (y + 1 < h) fr2[1][x] = fo;
      }
    } else {
      for (int x = 0; x < w; x++) {
        fr2[0][x] = PX(x, y) << sr;  /* box_f_r0, shared by both rows */
        if (y + 1 < h) fr2[1][x] = PX(x, y) << sr;
      }
    }
    for (int dy = 0; dy < imin(2, h - y); dy++) {
      const int yy = y + dy;
      uint32_t *fo = f1 + (size_t)yy * w;
      if (s1) {
        box_ab(1, a1 + ((yy + 2) % 3) * W2, b1 + ((yy + 2) % 3) * W2, ii, sq, iis, yy + 2, w, s1, bdm8);
        const uint32_t *A[3] = {a1 + (yy % 3) * W2, a1 + ((yy + 1) % 3) * W2, a1 + ((yy + 2) % 3) * W2};
        const uint32_t *B[3] = {b1 + (yy % 3) * W2, b1 + ((yy + 1) % 3) * W2, b1 + ((yy + 2) % 3) * W2};
        for (int x = 0; x < w; x++) {
          const uint32_t a = 3 * (A[0][x] + A[2][x] + A[0][x + 2] + A[2][x + 2]) +
                             4 * (A[1][x] + A[0][x + 1] + A[1][x + 1] + A[2][x + 1] + A[1][x + 2]);
          const uint32_t b = 3 * (B[0][x] + B[2][x] + B[0][x + 2] + B[2][x + 2]) +
                             4 * (B[1][x] + B[0][x + 1] + B[1][x + 1] + B[2][x + 1] + B[1][x + 2]);
          const uint32_t v = a * PX(x, yy) + b;
          fo[x] = (v + ((1u << shift) >> 1)) >> shift;
        }
      } else {
        for (int x = 0; x < w; x++) fo[x] = PX(x, yy) << sr;
      }
    }
  }
#undef PX
  free(a2);
  free(b2);
  free(a1);
  free(b1);
}

/* sgrproj_stripe_filter (:582-748): the stripe (w x h at cd) filtered with
 * set / xqd into out */
void orc_sgr_stripe_filter(int set, const int8_t xqd[2], int bd, const uint32_t *ii,
                           const uint32_t *sq, int iis, int w, int h, const void *cd, ptrdiff_t cs,
                           void *out, ptrdiff_t os, int hbd) {
  uint32_t *f2 = malloc(sizeof(uint32_t) * (size_t)w * h), *f1 = malloc(sizeof(uint32_t) * (size_t)w * h);
  sgr_f(set, bd - 8, ii, sq, iis, w, h, cd, cs, hbd, f2, f1);
  const int w0 = xqd[0], w1 = xqd[1], w2 = (1 << SGRPROJ_PRJ_BITS) - w0 - w1;
  const int sh = SGRPROJ_RST_BITS + SGRPROJ_PRJ_BITS, mx = (1 << bd) - 1;
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      const int32_t u = orc_px(cd, hbd, (ptrdiff_t)y * cs + x) << SGRPROJ_RST_BITS;
      const int32_t v = w0 * (int32_t)f2[(size_t)y * w + x] + w1 * u + w2 * (int32_t)f1[(size_t)y * w + x];
      const int32_t s = (v + ((1 << sh) >> 1)) >> sh;
      orc_px_store(out, hbd, (ptrdiff_t)y * os + x, iclamp(s, 0, mx));
    }
  free(f2);
  free(f1);
}

/* sgrproj_solve (:764-965): the least-squares (xqd0, xqd1) of the unit
 * (w x h at cd, the source at in) */
void orc_sgr_solve(int set, int bd, const uint32_t *ii, const uint32_t *sq, int iis,
                   const void *in, ptrdiff_t is, const void *cd, ptrdiff_t cs, int hbd, int w, int h,
                   int8_t xqd[2]) {
  uint32_t *f2 = malloc(sizeof(uint32_t) * (size_t)w * h), *f1 = malloc(sizeof(uint32_t) * (size_t)w * h);
  sgr_f(set, bd - 8, ii, sq, iis, w, h, cd, cs, hbd, f2, f1);
  int64_t H00 = 0, H11 = 0, H01 = 0, C0 = 0, C1 = 0;
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      const int64_t u = (int64_t)orc_px(cd, hbd, (ptrdiff_t)y * cs + x) << SGRPROJ_RST_BITS;
      const int64_t s = ((int64_t)orc_px(in, hbd, (ptrdiff_t)y * is + x) << SGRPROJ_RST_BITS) - u;
      const int64_t a2 = (int64_t)(int32_t)f2[(size_t)y * w + x] - u;
      const int64_t a1 = (int64_t)(int32_t)f1[(size_t)y * w + x] - u;
      H00 += a2 * a2;
      H11 += a1 * a1;
      H01 += a1 * a2;
      C0 += a2 * s;
      C1 += a1 * s;
    }
  free(f2);
  free(f1);
  orc_sgr_solve_finish(set, w, h, H00, H01, H11, C0, C1, xqd);
}

/* The f64 tail of sgrproj_solve (:920-964) from the exact sums */
void orc_sgr_solve_finish(int set, int w, int h, int64_t H00, int64_t H01, int64_t H11, int64_t C0,
                          int64_t C1, int8_t xqd[2]) {
  const uint32_t s2 = ORC_SGRPROJ_PARAMS_S[set][0], s1 = ORC_SGRPROJ_PARAMS_S[set][1];
  const double n = (double)w * (double)h;
  double h00 = (double)H00, h01 = (double)H01, h11 = (double)H11, c0 = (double)C0, c1 = (double)C1;
  h00 /= n;
  h01 /= n;
  h11 /= n;
  const double h10 = h01;
  const double sc = (double)(1 << SGRPROJ_PRJ_BITS) / n;
  c0 *= sc;
  c1 *= sc;
  int xq0, xq1;
  if (s2 == 0) {
    xq0 = 0;
    xq1 = h11 == 0. ? 0 : (int)round(c1 / h11);
  } else if (s1 == 0) {
    xq0 = h00 == 0. ? 0 : (int)round(c0 / h00);
    xq1 = 0;
  } else {
    const double det = h00 * h11 - h01 * h10;
    if (det == 0.) {
      xq0 = xq1 = 0;
    } else {
      const double div1 = h11 * c0 - h01 * c1, div2 = h00 * c1 - h10 * c0;
      xq0 = (int)round(div1 / det);
      xq1 = (int)round(div2 / det);
    }
  }
  const int x0 = iclamp(xq0, XQD_MIN[0], XQD_MAX[0]);
  const int x1 = iclamp((1 << SGRPROJ_PRJ_BITS) - x0 - xq1, XQD_MIN[1], XQD_MAX[1]);
  xqd[0] = (int8_t)x0;
  xqd[1] = (int8_t)x1;
}

/* ---- lrf_filter_frame (src/lrf.rs:1345-1444), Sgrproj and None units ----
 * out[p] holds the CDEF output (cdeffed, read from a copy) and receives the
 * restored plane; pre[p] the deblocked planes; plane p is (width + xdec_p)
 * >> xdec_p wide.  units[p][row * cols + col]: set (-1: None) and xqd.
 * enable_cdef = 0: Sgrproj units are skipped (:1406-1408). */
void orc_lrf_filter_frame(void *const out[3], const void *const pre[3], const ptrdiff_t stride[3],
                          int hbd, int bd, int width, int height, int xdec, int ydec,
                          const orc_lrf_plane_cfg cfg[3], const orc_lrf_unit *const units[3],
                          int enable_cdef) {
  const int stripe_n = (height + 7) / 64 + 1;
  const int iis = 256 + 6 + 2;  /* STRIPE_IMAGE_STRIDE */
  uint32_t *ii = malloc(sizeof(uint32_t) * iis * (64 + 6 + 2 + 2));
  uint32_t *sq = malloc(sizeof(uint32_t) * iis * (64 + 6 + 2 + 2));
  for (int p = 0; p < 3; p++) {
    const int xd = p ? xdec : 0, yd = p ? ydec : 0;
    const int crop_w = (width + ((1 << xd) >> 1)) >> xd, crop_h = (height + ((1 << yd) >> 1)) >> yd;
    const int B = hbd ? 2 : 1;
    uint8_t *cdeffed = malloc((size_t)crop_w * crop_h * B);  /* out.clone() (:1349) */
    for (int y = 0; y < crop_h; y++)
      memcpy(cdeffed + (size_t)y * crop_w * B, (const uint8_t *)out[p] + (size_t)y * stride[p] * B,
             (size_t)crop_w * B);
    for (int si = 0; si < stripe_n; si++) {
      int y0, sz;
      if (si == 0) {
        y0 = 0;
        sz = (64 - 8) >> yd;
      } else {
        y0 = (si * 64 - 8) >> yd;
        sz = imin(64 >> yd, crop_h - y0);
      }
      if (sz <= 0) continue;
      for (int rux = 0; rux < cfg[p].cols; rux++) {
        const int x = rux * cfg[p].unit_size;
        const int size = rux == cfg[p].cols - 1 ? crop_w - x : cfg[p].unit_size;
        /* restoration_unit_index_by_stripe (:1172-1182) */
        const int ry = imin(si * cfg[p].stripe_h / cfg[p].unit_size, cfg[p].rows - 1);
        const orc_lrf_unit u = units[p][ry * cfg[p].cols + imin(rux, cfg[p].cols - 1)];
        if (u.set < 0 || !enable_cdef) continue;
        orc_lrf_integral(cdeffed, crop_w, pre[p], stride[p], hbd, x, y0, crop_w - x, crop_h - y0,
                         size, sz, ii, sq, iis);
        const int8_t xqd[2] = {u.xqd[0], u.xqd[1]};
        orc_sgr_stripe_filter(u.set, xqd, bd, ii, sq, iis, size, sz,
                              cdeffed + ((size_t)y0 * crop_w + x) * B, crop_w,
                              (uint8_t *)out[p] + ((size_t)y0 * stride[p] + x) * B, stride[p], hbd);
      }
    }
    free(cdeffed);
  }
  free(ii);
  free(sq);
}

/* ---- rates (src/ec.rs, src/context.rs:3560-3659) --------------------------
 * symbol_bits (src/ec.rs:559-590) priced at a writer in its initial state
 * (WriterBase::new: rng 0x8000, cnt -9): the replay codes no symbol besides
 * the coefficients, so the range coder's state at a unit is
 * not the reference's; every price uses this one state. */
static uint32_t frac_compute(uint32_t nbits_total, uint32_t rng) {
  const uint32_t nbits = nbits_total << OD_BITRES;
  uint32_t l = 0;
  for (int i = 0; i < OD_BITRES; i++) {
    rng = (rng * rng) >> 15;
    const uint32_t b = rng >> 16;
    l = (l << 1) | b;
    rng >>= b;
  }
  return nbits - l;
}
uint32_t orc_symbol_bits(uint32_t s, const uint16_t *cdf, int nsym) {
  const uint32_t rng_full = 0x8000;
  const int cnt = -9;
  const uint32_t rng = rng_full >> 8;
  const uint32_t fh = (uint32_t)cdf[s] >> 6;
  uint32_t r;
  if (s > 0) {
    const uint32_t fl = (uint32_t)cdf[s - 1] >> 6;
    r = ((rng * fl) >> 1) - ((rng * fh) >> 1) + 4;
  } else {
    const uint32_t nms1 = (uint32_t)nsym - s - 1;
    r = rng_full - ((rng * fh) >> 1) - nms1 * 4;
  }
  const uint32_t pre = frac_compute((uint32_t)(cnt + 9), rng_full);
  const int d = 16 - ilog_sz(r);
  int c = cnt, bits = 0, sh = c + d;
  if (sh >= 0) {
    c += 16;
    if (sh >= 8) {
      bits += 8;
      c -= 8;
    }
    bits += 8;
    sh = c + d - 24;
  }
  return frac_compute((uint32_t)(bits + sh + 9), r << d) - pre;
}
static uint32_t count_quniform(uint32_t n, uint32_t v) {
  uint32_t bits = 0;
  if (n > 1) {
    const uint32_t l = (uint32_t)orc_msb((int32_t)n) + 1, m = (1u << l) - n;
    bits += (l - 1) << OD_BITRES;
    if (v >= m) bits += 1 << OD_BITRES;
  }
  return bits;
}
static uint32_t count_subexp(uint32_t n, uint32_t k, uint32_t v) {
  uint32_t i = 0, mk = 0, bits = 0;
  for (;;) {
    const uint32_t b = i ? k + i - 1 : k, a = 1u << b;
    if (n <= mk + 3 * a) {
      bits += count_quniform(n - mk, v - mk);
      break;
    }
    const int t = v >= mk + a;
    bits += 1 << OD_BITRES;
    if (t) {
      i++;
      mk += a;
    } else {
      bits += b << OD_BITRES;
      break;
    }
  }
  return bits;
}
static uint32_t recenter(uint32_t r, uint32_t v) {
  return v > (r << 1) ? v : v >= r ? (v - r) << 1 : ((r - v) << 1) - 1;
}
static uint32_t count_signed_subexp_with_ref(int v, int low, int high, uint32_t k, int r) {
  const uint32_t x = (uint32_t)(v - low), n = (uint32_t)(high - low), rr = (uint32_t)(r - low);
  return (rr << 1) <= n ? count_subexp(n, k, recenter(rr, x))
                        : count_subexp(n, k, recenter(n - 1 - rr, n - 1 - x));
}

/* count_lrf_switchable (src/context.rs:3560-3594), RESTORE_SWITCHABLE:
 * set < 0 = RestorationFilter::None */
uint32_t orc_lrf_rate(const uint16_t cdf[4], const int8_t ref[2], int set, const int8_t xqd[2]) {
  if (set < 0) return orc_symbol_bits(0, cdf, 3);
  uint32_t bits = orc_symbol_bits(2, cdf, 3) + (SGRPROJ_PARAMS_BITS << OD_BITRES);
  for (int i = 0; i < 2; i++)
    if (ORC_SGRPROJ_PARAMS_S[set][i] > 0)
      bits += count_signed_subexp_with_ref(xqd[i], XQD_MIN[i], XQD_MAX[i] + 1, SGRPROJ_PRJ_SUBEXP_K,
                                           ref[i]);
  return bits;
}
/* write_lrf's state updates (:3596-3659): the CDF (symbol_with_update) and
 * the plane's sgrproj_ref */
void orc_lrf_commit(uint16_t cdf[4], int8_t ref[2], int set, const int8_t xqd[2]) {
  orc_update_cdf(cdf, 4, set < 0 ? 0 : 2);
  if (set < 0) return;
  for (int i = 0; i < 2; i++)
    if (ORC_SGRPROJ_PARAMS_S[set][i] > 0)
      ref[i] = xqd[i];
    else
      ref[i] = i == 0 ? 0 : 95;
}
/* the tile's initial state: default_switchable_restore_cdf
 * (src/entropymode.rs:1427-1428, cdf!(9413, 22581)) and SGRPROJ_XQD_MID */
void orc_lrf_tile_init(uint16_t cdf[4], int8_t ref[3][2]) {
  cdf[0] = 32768 - 9413;
  cdf[1] = 32768 - 22581;
  cdf[2] = 0;
  cdf[3] = 0;
  for (int p = 0; p < 3; p++) {
    ref[p][0] = (int8_t)XQD_MID[0];
    ref[p][1] = (int8_t)XQD_MID[1];
  }
}
