// rv_intra.h -- intra prediction and get_intra_edges on the device, shared by
// the batched predictor (rv_intra.hip), the intra-mode screening of the
// replay (rv_intra_pass.hip) and the intra RDO chains (rv_rdo.hip).
//
// Edge buffer (rav1e's edge_buf, 4 * MAX_TX_SIZE + 1 pixels, built by
// get_intra_edges, src/partition.rs:500-693): left pixels bottom-to-top and
// right-aligned in [0, 128), the top-left pixel at 128, the above row (and
// above-right) from 129.  On the device it lives in LDS as i32.
#pragma once

#include "rv_device.h"

namespace rv {

constexpr int kIntraEdge = 4 * 64 + 1;
constexpr int kIntraModes = 13;
// RAV1E_INTRA_MODES (src/predict.rs:32-46) as PredictionMode values
static __constant__ uint8_t kIntraModeOrder[kIntraModes] = {0, 2, 1, 9, 11, 10, 12,
                                                             3, 4, 5, 6, 7, 8};

// sm_weight_arrays (src/predict.rs:406-424)
static __constant__ uint8_t kSmW[128] = {
    0,   0,   255, 128, 255, 149, 85,  64,  255, 197, 146, 105, 73,  50,  37,  32,
    255, 225, 196, 170, 145, 123, 102, 84,  68,  54,  43,  33,  26,  20,  17,  16,
    255, 240, 225, 210, 196, 182, 169, 157, 145, 133, 122, 111, 101, 92,  83,  74,
    66,  59,  52,  45,  39,  34,  29,  25,  21,  17,  14,  12,  10,  9,   8,   8,
    255, 248, 240, 233, 225, 218, 210, 203, 196, 189, 182, 176, 169, 163, 156, 150,
    144, 138, 133, 127, 121, 116, 111, 106, 101, 96,  91,  86,  82,  77,  73,  69,
    65,  61,  57,  54,  50,  47,  44,  41,  38,  35,  32,  29,  27,  25,  22,  20,
    18,  16,  15,  13,  12,  10,  9,   8,   7,   6,   6,   5,   5,   4,   4,   4};

// dr_intra_derivative (src/predict.rs:912-944) of the angles rav1e's six
// directional modes reach (45, 23, 67)
__device__ __forceinline__ int intra_dr_deriv(int a) {
  return a == 45 ? 64 : a == 23 ? 151 : a == 67 ? 27 : 0;
}

// predict_intra's remaps (src/predict.rs:214-236): PAETH by variant, and the
// directional angle of a mode.  variant: PredictionVariant (0 NONE, 1 LEFT,
// 2 TOP, 3 BOTH) of the block's tile position.
__device__ __forceinline__ int intra_remap(int mode, int variant) {
  return mode == 12 ? (variant == 0 ? 0 : variant == 1 ? 2 : variant == 2 ? 1 : 12) : mode;
}
__device__ __forceinline__ int intra_angle(int mode) {
  return mode == 3 ? 45 : mode == 4 ? 135 : mode == 5 ? 113 : mode == 6 ? 157
       : mode == 7 ? 203 : mode == 8 ? 67 : 0;
}

// Per-block constants of a (remapped) mode: DC value (needs the edge sums),
// derivatives.
struct IntraSetup {
  int mode, angle, dx, dy;
  int32_t dcv;
};

// The DC value of the remapped DC_PRED (pred_dc / _top / _left / _128,
// src/predict.rs:603-661): sums over the first h left / w above pixels,
// reduced over the G lanes of this lane's group.
template <int G>
__device__ __forceinline__ int32_t intra_dc(const int32_t *e, int variant, int w, int h, int bd,
                                            int lane) {
  const int L0 = 128 - h, A0 = 129;
  uint32_t s = 0;
  if (variant & 1)
    for (int k = lane; k < h; k += G) s += (uint32_t)e[L0 + k];
  if (variant & 2)
    for (int k = lane; k < w; k += G) s += (uint32_t)e[A0 + k];
  s = group_sum<G>(s);
  const uint32_t len = (variant & 1 ? h : 0) + (variant & 2 ? w : 0);
  return variant == 0 ? (128 << (bd - 8)) : (int32_t)((s + (len >> 1)) / len);
}

__device__ __forceinline__ IntraSetup intra_setup(int mode, int variant) {
  IntraSetup s;
  s.mode = intra_remap(mode, variant);
  s.angle = intra_angle(s.mode);
  const int a = s.angle;
  s.dx = a < 90 ? intra_dr_deriv(a) : (a > 90 && a < 180 ? intra_dr_deriv(180 - a) : 0);
  s.dy = (a > 90 && a < 180) ? intra_dr_deriv(a - 90) : (a > 180 ? intra_dr_deriv(270 - a) : 0);
  s.dcv = 0;
  return s;
}

// Pixel (r, c) of the w x h prediction (the native Intra trait,
// src/predict.rs:599-1034; no edge filter or upsampling, as rav1e).
__device__ __forceinline__ int32_t intra_px(const IntraSetup &s, const int32_t *e, int w, int h,
                                            int r, int c, int maxv) {
  const int L0 = 128 - h, LB = 128 - h - w, A0 = 129;
  switch (s.mode) {
    case 0: return s.dcv;                          // DC_PRED
    case 1: return e[A0 + c];                      // V_PRED
    case 2: return e[L0 + h - 1 - r];              // H_PRED
    case 12: {                                     // PAETH_PRED
      const int32_t tl = e[128], l = e[L0 + h - 1 - r], t = e[A0 + c];
      const int32_t base = t + l - tl;
      const int32_t pl = abs(base - l), pt = abs(base - t), ptl = abs(base - tl);
      return (pl <= pt && pl <= ptl) ? l : (pt <= ptl ? t : tl);
    }
    case 9: {  // SMOOTH_PRED: weights scaled by 2^8, log2_scale 9
      const uint32_t wh = kSmW[h + r], ww = kSmW[w + c];
      const uint32_t v = wh * (uint32_t)e[A0 + c] + (256 - wh) * (uint32_t)e[L0] +
                         ww * (uint32_t)e[L0 + h - 1 - r] + (256 - ww) * (uint32_t)e[A0 + w - 1];
      return (int32_t)((v + 256) >> 9);
    }
    case 11: {  // SMOOTH_H_PRED
      const uint32_t ww = kSmW[w + c];
      return (int32_t)((ww * (uint32_t)e[L0 + h - 1 - r] + (256 - ww) * (uint32_t)e[A0 + w - 1] +
                        128) >> 8);
    }
    case 10: {  // SMOOTH_V_PRED
      const uint32_t wh = kSmW[h + r];
      return (int32_t)((wh * (uint32_t)e[A0 + c] + (256 - wh) * (uint32_t)e[L0] + 128) >> 8);
    }
    default: {  // pred_directional (src/predict.rs:894-1034)
      int32_t v;
      if (s.angle < 90) {
        const int idx = (r + 1) * s.dx, base = (idx >> 6) + c, sh = (idx >> 1) & 31;
        const int mb = h + w - 1;
        v = base < mb ? round_shift(e[A0 + base] * (32 - sh) + e[A0 + base + 1] * sh, 5) : e[A0 + mb];
      } else if (s.angle < 180) {
        const int idx = (c << 6) - (r + 1) * s.dx, base = idx >> 6;
        if (base >= -1) {
          const int sh = (idx >> 1) & 31;
          const int32_t a = base < 0 ? e[128] : e[A0 + base];
          v = round_shift(a * (32 - sh) + e[A0 + base + 1] * sh, 5);
        } else {
          const int idy = (r << 6) - (c + 1) * s.dy, bl = idy >> 6, sh = (idy >> 1) & 31;
          const int32_t a = bl < 0 ? e[128] : e[LB + w + h - 1 - bl];
          v = round_shift(a * (32 - sh) + e[LB + w + h - 2 - bl] * sh, 5);
        }
      } else {
        const int idx = (c + 1) * s.dy, base = (idx >> 6) + r, sh = (idx >> 1) & 31;
        v = round_shift(e[LB + w + h - 1 - base] * (32 - sh) + e[LB + w + h - 2 - base] * sh, 5);
      }
      return v < 0 ? 0 : (v > maxv ? maxv : v);
    }
  }
}

// get_intra_edges (src/partition.rs:500-693) with opt_mode None for the
// transform block of a superblock-level partition (an n x n block at
// tile-relative pixel (x, y) of a tw-wide tile region whose pixel (0, 0) is
// plane pixel (tx, ty)): has_top_right holds iff the top row and the right
// neighbour exist, has_bottom_left never (src/recon_intra.rs:174-470 for
// the first transform block of a 64x64 partition).  The G lanes of a group
// fill e (i32, LDS); entries no branch of the reference writes are zero.
// The caller orders the writes before any read (a barrier).
template <typename Px, int G>
__device__ __forceinline__ void intra_edges_sb(const rv_plane &p, int tx, int ty, int tw, int x,
                                               int y, int n, int have_top, int bd, int32_t *e,
                                               int lane) {
  const int base = 128 << (bd - 8);
  const int L = 128, A = 129;
  auto D = [&](int r, int c) -> int32_t { return (int32_t)*plane_ptr<Px>(p, tx + c, ty + r); };
  const int na = (y != 0 && have_top && x + n < tw) ? (n < tw - x - n ? n : tw - x - n) : 0;
  for (int i = lane; i < kIntraEdge; i += G) {
    int32_t v = 0;
    if (i >= L - n && i < L) {  // left
      const int k = i - (L - n);
      v = x != 0 ? D(y + n - 1 - k, x - 1) : (y != 0 ? D(y - 1, 0) : base + 1);
    } else if (i == L) {  // top-left
      v = x == 0 && y == 0 ? base : y == 0 ? D(0, x - 1) : x == 0 ? D(y - 1, 0) : D(y - 1, x - 1);
    } else if (i >= A && i < A + n) {  // top
      const int k = i - A;
      v = y != 0 ? D(y - 1, x + k) : (x != 0 ? D(0, x - 1) : base - 1);
    } else if (i >= A + n && i < A + 2 * n) {  // top-right: available, else the last one
      const int k = i - A - n;
      const int kk = k < na ? k : na - 1;
      if (kk >= 0)
        v = D(y - 1, x + n + kk);
      else  // none available: above[n - 1]
        v = y != 0 ? D(y - 1, x + n - 1) : (x != 0 ? D(0, x - 1) : base - 1);
    } else if (i >= L - 2 * n && i < L - n) {  // bottom-left: left[L - n] replicated
      v = x != 0 ? D(y + n - 1, x - 1) : (y != 0 ? D(y - 1, 0) : base + 1);
    }
    e[i] = v;
  }
}

}  // namespace rv
