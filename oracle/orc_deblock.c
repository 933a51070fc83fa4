/* Deblocking filter (test infrastructure only): deblock_plane
 * (src/deblock.rs:1174-1335) with the edge drivers filter_v_edge /
 * filter_h_edge (:1001-1041, 1087-1127), deblock_size / deblock_level
 * (:115-163) and the 4 / 6 / 8 / 14-tap filters with their masks
 * (:165-995).  rav1e interleaves the vertical and horizontal edges, the
 * horizontal lagging one 4x4 row and two columns; no horizontal edge reads
 * a pixel a later vertical edge writes and vice versa, so this restatement
 * runs every vertical edge of the plane, then every horizontal one.
 *
 * Blocks: per luma 4x4 block (mi) of the frame, `lg` = log2 of the square
 * block's width in 4x4 units (1 = 8x8 .. 4 = 64x64; the transform is the
 * block's size, rdo_tx_decision off) and `skip`.  Every block is inter
 * (the replay codes no intra blocks); loop-filter deltas are off
 * (DeblockState::default, src/encoder.rs:420-434). */
#include <stdlib.h>

#include "orc_common.h"

static int iabs(int v) { return v < 0 ? -v : v; }
static int imax(int a, int b) { return a > b ? a : b; }
static int imin(int a, int b) { return a < b ? a : b; }

/* filter_narrow2_4 / filter_narrow4_4 (:165-240) */
static void narrow2(int32_t *v, int shift) { /* v = p1 p0 q0 q1 */
  const int lo = -(128 << shift), hi = (128 << shift) - 1, mx = (256 << shift) - 1;
  int f0 = clamp_i32(v[0] - v[3], lo, hi);
  int f1 = clamp_i32(f0 + 3 * (v[2] - v[1]) + 4, lo, hi) >> 3;
  int f2 = clamp_i32(f0 + 3 * (v[2] - v[1]) + 3, lo, hi) >> 3;
  v[1] = clamp_i32(v[1] + f2, 0, mx);
  v[2] = clamp_i32(v[2] - f1, 0, mx);
}
static void narrow4(int32_t *v, int shift) {
  const int lo = -(128 << shift), hi = (128 << shift) - 1, mx = (256 << shift) - 1;
  int f1 = clamp_i32(3 * (v[2] - v[1]) + 4, lo, hi) >> 3;
  int f2 = clamp_i32(3 * (v[2] - v[1]) + 3, lo, hi) >> 3;
  int f3 = (f1 + 1) >> 1;
  v[0] = clamp_i32(v[0] + f3, 0, mx);
  v[1] = clamp_i32(v[1] + f2, 0, mx);
  v[2] = clamp_i32(v[2] - f1, 0, mx);
  v[3] = clamp_i32(v[3] - f3, 0, mx);
}
/* the level-domain tests (:337-380) */
static int limit_to_level(int limit, int shift) { return (limit + (1 << shift) - 1) >> shift; }
static int blimit_to_level(int blimit, int shift) {
  return (((blimit + (1 << shift) - 1) >> shift) - 2) / 3;
}
static int thresh_to_level(int thresh, int shift) {
  return (thresh + (1 << shift) - 1) >> shift << 4;
}
static int nhev4(const int32_t *v, int shift) { /* p1 p0 q0 q1 */
  return thresh_to_level(imax(iabs(v[0] - v[1]), iabs(v[3] - v[2])), shift);
}
static int blim(const int32_t *v, int shift) {
  return blimit_to_level(iabs(v[1] - v[2]) * 2 + iabs(v[0] - v[3]) / 2, shift);
}

/* deblock_size{4,6,8,14}_inner on the taps t[0..n) across the edge (in
 * place): n = 4, 6, 8 or 14 */
static void filter_taps(int32_t *t, int n, int level, int bd) {
  const int s = bd - 8, flat = 1 << s;
  if (n == 4) {
    int m = imax(limit_to_level(imax(iabs(t[0] - t[1]), iabs(t[3] - t[2])), s), blim(t, s));
    if (m > level) return;
    if (nhev4(t, s) <= level) narrow4(t, s); else narrow2(t, s);
    return;
  }
  if (n == 6) { /* p2 p1 p0 q0 q1 q2 */
    const int32_t *c = t + 1;
    int m = imax(limit_to_level(imax(iabs(t[0] - t[1]), imax(iabs(t[1] - t[2]),
                                 imax(iabs(t[5] - t[4]), iabs(t[4] - t[3])))), s), blim(c, s));
    if (m > level) return;
    int f = imax(iabs(t[1] - t[2]), imax(iabs(t[4] - t[3]), imax(iabs(t[0] - t[2]), iabs(t[5] - t[3]))));
    if (f <= flat) { /* filter_wide6_4 */
      const int p2 = t[0], p1 = t[1], p0 = t[2], q0 = t[3], q1 = t[4], q2 = t[5];
      t[1] = (p2 * 3 + p1 * 2 + p0 * 2 + q0 + 4) >> 3;
      t[2] = (p2 + p1 * 2 + p0 * 2 + q0 * 2 + q1 + 4) >> 3;
      t[3] = (p1 + p0 * 2 + q0 * 2 + q1 * 2 + q2 + 4) >> 3;
      t[4] = (p0 + q0 * 2 + q1 * 2 + q2 * 3 + 4) >> 3;
    } else if (nhev4(c, s) <= level) {
      narrow4(t + 1, s);
    } else {
      narrow2(t + 1, s);
    }
    return;
  }
  /* 8 and 14: the inner 8 taps p3..q3 */
  int32_t *in = n == 8 ? t : t + 3;
  const int32_t *c = in + 2;
  int m = imax(limit_to_level(imax(iabs(in[0] - in[1]), imax(iabs(in[1] - in[2]),
               imax(iabs(in[2] - in[3]), imax(iabs(in[7] - in[6]),
               imax(iabs(in[6] - in[5]), iabs(in[5] - in[4])))))), s), blim(c, s));
  if (m > level) return;
  int f8 = imax(iabs(in[2] - in[3]), imax(iabs(in[5] - in[4]), imax(iabs(in[1] - in[3]),
           imax(iabs(in[6] - in[4]), imax(iabs(in[0] - in[3]), iabs(in[7] - in[4]))))));
  if (f8 <= flat) {
    int wide14 = 0;
    if (n == 14) {
      int f14 = imax(iabs(t[2] - t[6]), imax(iabs(t[11] - t[7]), imax(iabs(t[1] - t[6]),
                imax(iabs(t[12] - t[7]), imax(iabs(t[0] - t[6]), iabs(t[13] - t[7]))))));
      wide14 = f14 <= flat;
    }
    if (wide14) { /* filter_wide14_12 */
      const int p6 = t[0], p5 = t[1], p4 = t[2], p3 = t[3], p2 = t[4], p1 = t[5], p0 = t[6];
      const int q0 = t[7], q1 = t[8], q2 = t[9], q3 = t[10], q4 = t[11], q5 = t[12], q6 = t[13];
      int o[12];
      o[0] = (p6 * 7 + p5 * 2 + p4 * 2 + p3 + p2 + p1 + p0 + q0 + 8) >> 4;
      o[1] = (p6 * 5 + p5 * 2 + p4 * 2 + p3 * 2 + p2 + p1 + p0 + q0 + q1 + 8) >> 4;
      o[2] = (p6 * 4 + p5 + p4 * 2 + p3 * 2 + p2 * 2 + p1 + p0 + q0 + q1 + q2 + 8) >> 4;
      o[3] = (p6 * 3 + p5 + p4 + p3 * 2 + p2 * 2 + p1 * 2 + p0 + q0 + q1 + q2 + q3 + 8) >> 4;
      o[4] = (p6 * 2 + p5 + p4 + p3 + p2 * 2 + p1 * 2 + p0 * 2 + q0 + q1 + q2 + q3 + q4 + 8) >> 4;
      o[5] = (p6 + p5 + p4 + p3 + p2 + p1 * 2 + p0 * 2 + q0 * 2 + q1 + q2 + q3 + q4 + q5 + 8) >> 4;
      o[6] = (p5 + p4 + p3 + p2 + p1 + p0 * 2 + q0 * 2 + q1 * 2 + q2 + q3 + q4 + q5 + q6 + 8) >> 4;
      o[7] = (p4 + p3 + p2 + p1 + p0 + q0 * 2 + q1 * 2 + q2 * 2 + q3 + q4 + q5 + q6 * 2 + 8) >> 4;
      o[8] = (p3 + p2 + p1 + p0 + q0 + q1 * 2 + q2 * 2 + q3 * 2 + q4 + q5 + q6 * 3 + 8) >> 4;
      o[9] = (p2 + p1 + p0 + q0 + q1 + q2 * 2 + q3 * 2 + q4 * 2 + q5 + q6 * 4 + 8) >> 4;
      o[10] = (p1 + p0 + q0 + q1 + q2 + q3 * 2 + q4 * 2 + q5 * 2 + q6 * 5 + 8) >> 4;
      o[11] = (p0 + q0 + q1 + q2 + q3 + q4 * 2 + q5 * 2 + q6 * 7 + 8) >> 4;
      for (int i = 0; i < 12; i++) t[1 + i] = o[i];
    } else { /* filter_wide8_6 on p3..q3 */
      const int p3 = in[0], p2 = in[1], p1 = in[2], p0 = in[3], q0 = in[4], q1 = in[5], q2 = in[6], q3 = in[7];
      in[1] = (p3 * 3 + p2 * 2 + p1 + p0 + q0 + 4) >> 3;
      in[2] = (p3 * 2 + p2 + p1 * 2 + p0 + q0 + q1 + 4) >> 3;
      in[3] = (p3 + p2 + p1 + p0 * 2 + q0 + q1 + q2 + 4) >> 3;
      in[4] = (p2 + p1 + p0 + q0 * 2 + q1 + q2 + q3 + 4) >> 3;
      in[5] = (p1 + p0 + q0 + q1 * 2 + q2 + q3 * 2 + 4) >> 3;
      in[6] = (p0 + q0 + q1 + q2 * 2 + q3 * 3 + 4) >> 3;
    }
  } else if (nhev4(c, s) <= level) {
    narrow4(in + 2, s);
  } else {
    narrow2(in + 2, s);
  }
}

/* The transform width (vertical) / height in 4x4 units of the block with
 * log2 size lg in plane pli: the luma transform is the block's size, the
 * chroma one largest_chroma_tx_size (partition.rs:288-297), coded size
 * capped at 32. */
static int tx_mi(int lg, int pli, int dec) {
  if (pli == 0) return 1 << lg;
  int px = (4 << lg) >> dec;
  if (px > 32) px = 32;
  return px >= 4 ? px / 4 : 1;
}

void orc_deblock_plane(void *origin, ptrdiff_t stride, int hbd, int bd, int width, int height,
                       int xdec, int ydec, int pli, const uint8_t *lg, const uint8_t *skip,
                       int mi_stride, const uint8_t levels[4]) {
  if (pli == 0 ? (levels[0] == 0 && levels[1] == 0) : levels[pli + 1] == 0) return;
  const int cols = ((((width + 3) >> 2) + ((1 << xdec) >> 1)) >> xdec) << xdec;
  const int rows = ((((height + 3) >> 2) + ((1 << ydec) >> 1)) >> ydec) << ydec;
  const int cap = pli == 0 ? 14 : 6;
  for (int pass = 0; pass < 2; pass++) {
    const int vert = pass == 0;
    const int dec = vert ? xdec : ydec;
    const int level = pli == 0 ? levels[vert ? 0 : 1] : levels[pli + 1];
    if (level == 0) continue;
    for (int y = vert ? 0 : 1 << ydec; y < rows; y += 1 << ydec)
      for (int x = vert ? 1 << xdec : 0; x < cols; x += 1 << xdec) {
        const int b = y * mi_stride + x;
        const int n4 = 1 << lg[b];
        const int pos = vert ? x : y;
        if (((pos >> dec) & (tx_mi(lg[b], pli, dec) - 1)) != 0) continue; /* tx edge */
        /* deblock_left / deblock_up: odd mi for subsampled chroma */
        const int px_ = (x | xdec) - (vert ? 1 << xdec : 0);
        const int py_ = (y | ydec) - (vert ? 0 : 1 << ydec);
        const int pb = py_ * mi_stride + px_;
        const int block_edge = (pos & (n4 - 1)) == 0;
        if (!(block_edge || !skip[b] || !skip[pb])) continue;
        const int size = imin(cap, imin(tx_mi(lg[b], pli, dec), tx_mi(lg[pb], pli, dec)) << 2);
        const int ox = (x * 4) >> xdec, oy = (y * 4) >> ydec;
        for (int k = 0; k < 4; k++) {
          int32_t t[14];
          const int h = size >> 1;
          for (int i = 0; i < size; i++) {
            const ptrdiff_t at = vert ? (ptrdiff_t)(oy + k) * stride + ox - h + i
                                      : (ptrdiff_t)(oy - h + i) * stride + ox + k;
            t[i] = orc_px(origin, hbd, at);
          }
          filter_taps(t, size, level, bd);
          for (int i = 0; i < size; i++) {
            const ptrdiff_t at = vert ? (ptrdiff_t)(oy + k) * stride + ox - h + i
                                      : (ptrdiff_t)(oy - h + i) * stride + ox + k;
            orc_px_store(origin, hbd, at, t[i]);
          }
        }
      }
  }
}

/* ---- sse_optimize (src/deblock.rs:1418-1475): the level search of
 * deblock_filter_optimize below speed 8.  Every edge segment row is measured
 * unfiltered against the source: the tally at index L gains the SSE change
 * of the filter a level-L pass would apply, so the prefix sum at L is the
 * plane's SSE at level L (each edge filtered from the unfiltered
 * reconstruction, the directions separable). */

/* the mask / flat / nhev decisions of sse_size{4,6,8,14} (:425-999) on the
 * n taps of one row: mask clamped to [1, 64], nhev to [mask, 64]; flat: 0 =
 * narrow, 1 = wide (6 / 8), 2 = wide14 */
static void sse_decide(const int32_t *t, int n, int s, int *mask, int *nhev, int *flat) {
  const int fl = 1 << s;
  int m, f = 0;
  const int32_t *c; /* p1 p0 q0 q1 */
  if (n == 4) {
    c = t;
    m = imax(limit_to_level(imax(iabs(t[0] - t[1]), iabs(t[3] - t[2])), s), blim(t, s));
  } else if (n == 6) {
    c = t + 1;
    m = imax(limit_to_level(imax(iabs(t[0] - t[1]), imax(iabs(t[1] - t[2]),
                            imax(iabs(t[5] - t[4]), iabs(t[4] - t[3])))), s), blim(c, s));
    f = imax(iabs(t[1] - t[2]), imax(iabs(t[4] - t[3]), imax(iabs(t[0] - t[2]), iabs(t[5] - t[3])))) <= fl;
  } else {
    const int32_t *in = n == 8 ? t : t + 3;
    c = in + 2;
    m = imax(limit_to_level(imax(iabs(in[0] - in[1]), imax(iabs(in[1] - in[2]),
             imax(iabs(in[2] - in[3]), imax(iabs(in[7] - in[6]),
             imax(iabs(in[6] - in[5]), iabs(in[5] - in[4])))))), s), blim(c, s));
    f = imax(iabs(in[2] - in[3]), imax(iabs(in[5] - in[4]), imax(iabs(in[1] - in[3]),
        imax(iabs(in[6] - in[4]), imax(iabs(in[0] - in[3]), iabs(in[7] - in[4])))))) <= fl;
    if (f && n == 14 &&
        imax(iabs(t[2] - t[6]), imax(iabs(t[11] - t[7]), imax(iabs(t[1] - t[6]),
        imax(iabs(t[12] - t[7]), imax(iabs(t[0] - t[6]), iabs(t[13] - t[7])))))) <= fl)
      f = 2;
  }
  *mask = m < 1 ? 1 : m > 64 ? 64 : m;
  const int h = nhev4(c, s);
  *nhev = h < *mask ? *mask : h > 64 ? 64 : h;
  *flat = f;
}

/* one variant of the row: the taps after filter `kind` (0 none, 1 narrow2,
 * 2 narrow4, 3 wide), then the SSE of the compared outputs (taps [o, n-o),
 * o = 0 for 4 taps else 1) against the source (stride_sse, :337-344) */
static int64_t sse_variant(const int32_t *taps, const int32_t *a, int n, int kind, int flat, int s) {
  int32_t t[14];
  for (int i = 0; i < n; i++) t[i] = taps[i];
  int32_t *c = t + (n == 4 ? 0 : n == 6 ? 1 : n == 8 ? 2 : 5);
  if (kind == 1) narrow2(c, s);
  if (kind == 2) narrow4(c, s);
  if (kind == 3) {
    /* the wide filters of filter_taps: level 63 passes every mask and the
     * flatness decides (the caller only asks for wide when flat) */
    filter_taps(t, n, 63, s + 8);
    (void)flat;
  }
  const int o = n == 4 ? 0 : 1;
  int64_t acc = 0;
  for (int i = o; i < n - o; i++) acc += (int64_t)(a[i] - t[i]) * (a[i] - t[i]);
  return acc;
}

/* the tally updates of one row (sse_size4 .. sse_size14's accumulation) */
static void sse_row(const int32_t *t, const int32_t *a, int n, int bd, int64_t *tally) {
  const int s = bd - 8;
  int mask, nhev, flat;
  sse_decide(t, n, s, &mask, &nhev, &flat);
  const int64_t none = sse_variant(t, a, n, 0, 0, s);
  tally[0] += none;
  tally[mask] -= none;
  if (flat) {
    tally[mask] += mask <= 63 ? sse_variant(t, a, n, 3, flat, s) : none;
  } else {
    const int64_t n2 = nhev != mask ? sse_variant(t, a, n, 1, 0, s) : none;
    const int64_t n4 = nhev <= 63 ? sse_variant(t, a, n, 2, 0, s) : none;
    tally[mask] += n2;
    tally[nhev] -= n2;
    tally[nhev] += n4;
  }
}

/* pixel x of row y, 128 outside [0, pw): the fill of a fresh plane
 * (src/frame/plane.rs:130-134); neither the reconstruction nor the input
 * frame is padded before the loop filters (src/encoder.rs:2789-2793) */
static int32_t px_or_128(const void *o, ptrdiff_t stride, int hbd, int pw, int x, int y) {
  return x < 0 || x >= pw ? 128 : orc_px(o, hbd, (ptrdiff_t)y * stride + x);
}

void orc_deblock_sse_plane(const void *rec, ptrdiff_t rstride, const void *src, ptrdiff_t sstride,
                           int hbd, int bd, int width, int height, int xdec, int ydec, int pli,
                           const uint8_t *lg, const uint8_t *skip, int mi_stride,
                           int64_t v_tally[65], int64_t h_tally[65]) {
  const int cols = (width + 3) >> 2, rows = (height + 3) >> 2;
  const int pw = (width + xdec) >> xdec;
  const int cap = pli == 0 ? 14 : 6;
  for (int k = 0; k < 65; k++) v_tally[k] = h_tally[k] = 0;
  /* sse_plane's edge walk (:1351-1406): vertical edges x >= 1 << xdec on
   * every row, horizontal edges y >= 1 << ydec on every column */
  for (int pass = 0; pass < 2; pass++) {
    const int vert = pass == 0;
    const int dec = vert ? xdec : ydec;
    int64_t *tally = vert ? v_tally : h_tally;
    for (int y = vert ? 0 : 1 << ydec; y < rows; y += 1 << ydec)
      for (int x = vert ? 1 << xdec : 0; x < cols; x += 1 << xdec) {
        const int b = y * mi_stride + x;
        const int pos = vert ? x : y;
        if (((pos >> dec) & (tx_mi(lg[b], pli, dec) - 1)) != 0) continue;
        const int px_ = (x | xdec) - (vert ? 1 << xdec : 0);
        const int py_ = (y | ydec) - (vert ? 0 : 1 << ydec);
        const int pb = py_ * mi_stride + px_;
        if (!((pos & ((1 << lg[b]) - 1)) == 0 || !skip[b] || !skip[pb])) continue;
        /* sse_h_edge (:1129-1171) sizes the filter with deblock_size(...,
         * vertical = true, ...) and measures the rows across the column
         * po.x - size / 2 (pitch 1), as sse_v_edge does: both directions
         * tally horizontal taps */
        const int size = imin(cap, imin(tx_mi(lg[b], pli, xdec), tx_mi(lg[pb], pli, xdec)) << 2);
        const int ox = (x * 4) >> xdec, oy = (y * 4) >> ydec;
        for (int k = 0; k < 4; k++) {
          int32_t t[14], a[14];
          for (int i = 0; i < size; i++) {
            t[i] = px_or_128(rec, rstride, hbd, pw, ox - size / 2 + i, oy + k);
            a[i] = px_or_128(src, sstride, hbd, pw, ox - size / 2 + i, oy + k);
          }
          sse_row(t, a, size, bd, tally);
        }
      }
  }
}

/* sse_optimize's choice (:1441-1473): prefix sums to MAX_LOOP_FILTER, the
 * first minimum; luma per direction, chroma over both directions */
void orc_deblock_sse_levels(const int64_t v_tally[3][65], const int64_t h_tally[3][65],
                            uint8_t levels[4]) {
  for (int p = 0; p < 3; p++) {
    int64_t v[64], h[64];
    v[0] = v_tally[p][0];
    h[0] = h_tally[p][0];
    for (int i = 1; i < 64; i++) {
      v[i] = v[i - 1] + v_tally[p][i];
      h[i] = h[i - 1] + h_tally[p][i];
    }
    int bv = 0, bh = 0, bc = 0;
    for (int i = 1; i < 64; i++) {
      if (v[bv] > v[i]) bv = i;
      if (h[bh] > h[i]) bh = i;
      if (v[bc] + h[bc] > v[i] + h[i]) bc = i;
    }
    if (p == 0) {
      levels[0] = (uint8_t)bv;
      levels[1] = (uint8_t)bh;
    } else {
      levels[p + 1] = (uint8_t)bc;
    }
  }
}

/* deblock_filter_optimize's fast path (src/deblock.rs:1477-1517,
 * speed >= 8): one level for every plane and direction from the frame's
 * ac quantizer. */
int orc_deblock_fast_level(int ac_q, int bd, int is_key) {
  int v;
  if (bd == 8)
    v = is_key ? (ac_q * 17563 - 421574 + (1 << 17)) >> 18 : (ac_q * 6017 + 650707 + (1 << 17)) >> 18;
  else if (bd == 10)
    v = ((ac_q * 20723 + 4060632 + (1 << 19)) >> 20) - (is_key ? 4 : 0);
  else
    v = ((ac_q * 20723 + 16242526 + (1 << 21)) >> 22) - (is_key ? 4 : 0);
  return v < 0 ? 0 : v > 63 ? 63 : v;
}
