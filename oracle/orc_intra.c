/* Intra prediction (test infrastructure only): PredictionMode::predict_intra
 * without CfL (src/predict.rs:202-241) and the native Intra trait
 * (src/predict.rs:538-1035).
 *
 * edge: rav1e's edge_buf of 4 * MAX_TX_SIZE + 1 pixels (src/predict.rs:
 * 545-551): left pixels bottom-to-top, right-aligned in [0, 128); the
 * top-left pixel at 128; the above row (and above-right) from 129.
 * variant: PredictionVariant (0 NONE, 1 LEFT, 2 TOP, 3 BOTH) of the block's
 * tile position (src/predict.rs:175-184). */
#include <stdlib.h>

#include "orc_common.h"

#define MAXTX 64

/* sm_weight_arrays (src/predict.rs:406-424), indexed from the block size */
static const uint8_t SM_W[2 * MAXTX] = {
    0,   0,   255, 128, 255, 149, 85,  64,  255, 197, 146, 105, 73,  50,  37,  32,
    255, 225, 196, 170, 145, 123, 102, 84,  68,  54,  43,  33,  26,  20,  17,  16,
    255, 240, 225, 210, 196, 182, 169, 157, 145, 133, 122, 111, 101, 92,  83,  74,
    66,  59,  52,  45,  39,  34,  29,  25,  21,  17,  14,  12,  10,  9,   8,   8,
    255, 248, 240, 233, 225, 218, 210, 203, 196, 189, 182, 176, 169, 163, 156, 150,
    144, 138, 133, 127, 121, 116, 111, 106, 101, 96,  91,  86,  82,  77,  73,  69,
    65,  61,  57,  54,  50,  47,  44,  41,  38,  35,  32,  29,  27,  25,  22,  20,
    18,  16,  15,  13,  12,  10,  9,   8,   7,   6,   6,   5,   5,   4,   4,   4};

/* dr_intra_derivative (src/predict.rs:912-944) */
static int dr_deriv(int a) {
  switch (a) {
    case 4: return 1023; case 7: return 547; case 10: return 372; case 14: return 273;
    case 17: return 215; case 20: return 178; case 23: return 151; case 26: return 132;
    case 29: return 116; case 32: return 102; case 36: return 90; case 39: return 80;
    case 42: return 71; case 45: return 64; case 48: return 57; case 51: return 51;
    case 54: return 45; case 58: return 40; case 61: return 35; case 64: return 31;
    case 67: return 27; case 70: return 23; case 73: return 19; case 76: return 15;
    case 81: return 11; case 84: return 7; case 87: return 3;
    default: return 0;
  }
}

void orc_predict_intra(int mode, int variant, void *dst, ptrdiff_t stride, int w, int h,
                       int bit_depth, int hbd, const void *edge) {
  const int32_t maxv = (1 << bit_depth) - 1;
#define E(i) orc_px(edge, hbd, (i))
#define OUT(r, c, v) orc_px_store(dst, hbd, (ptrdiff_t)(r) * stride + (c), (v))
  /* predict_intra's remaps (src/predict.rs:214-233) */
  if (mode == 12) /* PAETH_PRED */
    mode = variant == 0 ? 0 : variant == 1 ? 2 : variant == 2 ? 1 : 12;
  int angle = 0;
  switch (mode) {
    case 3: angle = 45; break;
    case 4: angle = 135; break;
    case 5: angle = 113; break;
    case 6: angle = 157; break;
    case 7: angle = 203; break;
    case 8: angle = 67; break;
  }
  const int L0 = 2 * MAXTX - h;         /* left_slice start */
  const int LB = 2 * MAXTX - h - w;     /* left_and_left_below start */
  const int A0 = 2 * MAXTX + 1;         /* above */
  const int32_t top_left = E(2 * MAXTX);
#define LEFT(k) E(L0 + (k))
#define LEFTB(k) E(LB + (k))
#define ABOVE(k) E(A0 + (k))
  if (mode == 0) { /* DC_PRED by variant */
    uint32_t v;
    if (variant == 0) {
      v = 128u << (bit_depth - 8);
    } else if (variant == 1) {
      uint32_t s = 0;
      for (int k = 0; k < h; k++) s += (uint32_t)LEFT(k);
      v = (s + (uint32_t)(h >> 1)) / (uint32_t)h;
    } else if (variant == 2) {
      uint32_t s = 0;
      for (int k = 0; k < w; k++) s += (uint32_t)ABOVE(k);
      v = (s + (uint32_t)(w >> 1)) / (uint32_t)w;
    } else {
      uint32_t s = 0;
      for (int k = 0; k < h; k++) s += (uint32_t)LEFT(k);
      for (int k = 0; k < w; k++) s += (uint32_t)ABOVE(k);
      const uint32_t len = (uint32_t)(w + h);
      v = (s + (len >> 1)) / len;
    }
    for (int r = 0; r < h; r++)
      for (int c = 0; c < w; c++) OUT(r, c, (int32_t)v);
    return;
  }
  for (int r = 0; r < h; r++)
    for (int c = 0; c < w; c++) {
      int32_t v = 0;
      switch (mode) {
        case 1: v = ABOVE(c); break;            /* V_PRED */
        case 2: v = LEFT(h - 1 - r); break;     /* H_PRED */
        case 12: {                              /* PAETH_PRED */
          const int32_t l = LEFT(h - 1 - r), t = ABOVE(c);
          const int32_t base = t + l - top_left;
          const int32_t pl = abs(base - l), pt = abs(base - t), ptl = abs(base - top_left);
          v = (pl <= pt && pl <= ptl) ? l : (pt <= ptl ? t : top_left);
          break;
        }
        case 9: { /* SMOOTH_PRED */
          const uint32_t below = (uint32_t)LEFT(0), right = (uint32_t)ABOVE(w - 1);
          const uint32_t wh = SM_W[h + r], ww = SM_W[w + c];
          uint32_t s = wh * (uint32_t)ABOVE(c) + (256 - wh) * below +
                       ww * (uint32_t)LEFT(h - 1 - r) + (256 - ww) * right;
          v = (int32_t)((s + (1u << 8)) >> 9);
          break;
        }
        case 11: { /* SMOOTH_H_PRED */
          const uint32_t right = (uint32_t)ABOVE(w - 1), ww = SM_W[w + c];
          uint32_t s = ww * (uint32_t)LEFT(h - 1 - r) + (256 - ww) * right;
          v = (int32_t)((s + (1u << 7)) >> 8);
          break;
        }
        case 10: { /* SMOOTH_V_PRED */
          const uint32_t below = (uint32_t)LEFT(0), wh = SM_W[h + r];
          uint32_t s = wh * (uint32_t)ABOVE(c) + (256 - wh) * below;
          v = (int32_t)((s + (1u << 7)) >> 8);
          break;
        }
        default: { /* directional, pred_directional (src/predict.rs:894-1034) */
          const int dx = angle < 90 ? dr_deriv(angle)
                                    : (angle > 90 && angle < 180 ? dr_deriv(180 - angle) : 0);
          const int dy = (angle > 90 && angle < 180) ? dr_deriv(angle - 90)
                                                     : (angle > 180 ? dr_deriv(270 - angle) : 0);
          if (angle < 90) {
            const int idx = (r + 1) * dx;
            const int base = (idx >> 6) + c, shift = (idx >> 1) & 31;
            const int max_base_x = h + w - 1;
            v = base < max_base_x
                    ? round_shift(ABOVE(base) * (32 - shift) + ABOVE(base + 1) * shift, 5)
                    : ABOVE(max_base_x);
          } else if (angle < 180) {
            const int idx = (c << 6) - (r + 1) * dx;
            const int base = idx >> 6;
            if (base >= -1) {
              const int shift = (idx >> 1) & 31;
              const int32_t a = base < 0 ? top_left : ABOVE(base);
              const int32_t b = ABOVE(base + 1);
              v = round_shift(a * (32 - shift) + b * shift, 5);
            } else {
              const int idy = (r << 6) - (c + 1) * dy;
              const int bl = idy >> 6, shift = (idy >> 1) & 31;
              const int32_t a = bl < 0 ? top_left : LEFTB(w + h - 1 - bl);
              const int32_t b = LEFTB(w + h - (2 + bl));
              v = round_shift(a * (32 - shift) + b * shift, 5);
            }
          } else {
            const int idx = (c + 1) * dy;
            const int base = (idx >> 6) + r, shift = (idx >> 1) & 31;
            v = round_shift(LEFTB(w + h - 1 - base) * (32 - shift) +
                                LEFTB(w + h - 2 - base) * shift,
                            5);
          }
          v = v < 0 ? 0 : (v > maxv ? maxv : v);
          break;
        }
      }
      OUT(r, c, v);
    }
#undef E
#undef OUT
#undef LEFT
#undef LEFTB
#undef ABOVE
}

/* get_intra_edges (src/partition.rs:500-693) with opt_mode None (every
 * edge: left, top-left, top, top-right, bottom-left) for the first (only)
 * transform block of a superblock-level partition: an n x n block at
 * tile-relative pixel (x, y) of a plane region of tw x th pixels whose pixel
 * (0, 0) is `tile` (stride in elements).  The partition is the 64x64
 * superblock, so has_top_right (src/recon_intra.rs:174-241) holds iff the
 * top row and the right neighbour exist (the block sits in the top row of
 * its superblock) and has_bottom_left (:376-470) never does (the bottom-left
 * superblock is coded later).  have_top / have_left: partition_bo.y / .x >
 * 0 (> 1 for a decimated plane), i.e. not the tile's first superblock row /
 * column.  Entries no branch writes stay zero (rav1e leaves them
 * uninitialized; no predictor reads them).  edge: 4 * 64 + 1 pixels. */
void orc_intra_edges_sb(const void *tile, ptrdiff_t stride, int hbd, int bd, int tw, int th,
                        int x, int y, int n, int have_top, int have_left, void *edge) {
  (void)th;
  (void)have_left;
  const int base = 128 << (bd - 8);
#define D(r, c) orc_px(tile, hbd, (ptrdiff_t)(r) * stride + (c))
#define S(i, v) orc_px_store(edge, hbd, (i), (v))
#define G(i) orc_px(edge, hbd, (i))
  for (int i = 0; i < 4 * MAXTX + 1; i++) S(i, 0);
  const int L = 2 * MAXTX, A = 2 * MAXTX + 1;
  /* left, bottom to top, right-aligned */
  if (x != 0) {
    for (int i = 0; i < n; i++) S(L - n + i, D(y + n - 1 - i, x - 1));
  } else {
    const int32_t v = y != 0 ? D(y - 1, 0) : base + 1;
    for (int i = L - n; i < L; i++) S(i, v);
  }
  /* top-left */
  S(L, x == 0 && y == 0 ? base : y == 0 ? D(0, x - 1) : x == 0 ? D(y - 1, 0) : D(y - 1, x - 1));
  /* top */
  if (y != 0) {
    for (int i = 0; i < n; i++) S(A + i, D(y - 1, x + i));
  } else {
    const int32_t v = x != 0 ? D(0, x - 1) : base - 1;
    for (int i = 0; i < n; i++) S(A + i, v);
  }
  /* top-right */
  const int right_available = x + n < tw;
  int na = 0;
  if (y != 0 && have_top && right_available) na = n < tw - x - n ? n : tw - x - n;
  for (int i = 0; i < na; i++) S(A + n + i, D(y - 1, x + n + i));
  if (na < n) {
    const int32_t v = G(A + n + na - 1);
    for (int i = n + na; i < 2 * n; i++) S(A + i, v);
  }
  /* bottom-left: none available; replicate the bottom-most left pixel */
  {
    const int32_t v = G(L - n);
    for (int i = L - 2 * n; i < L - n; i++) S(i, v);
  }
#undef D
#undef S
#undef G
}
