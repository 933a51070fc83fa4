// rv_lrf.h -- loop restoration's geometry, rates and the solve's f64 tail,
// shared by the decision kernel and the host (rv_lrf.hip, rv_replay.hip).
#pragma once

#include <math.h>
#include <stdint.h>

#include "rv_device.h"

// RestorationState::new's per-plane result (src/lrf.rs:1197-1343)
struct LrfPlaneCfg {
  int unit_size, sb_h_shift, sb_v_shift, stripe_h, cols, rows;
};

// the frame as the loop-restoration kernels see it (units of one superblock)
struct LrfGeo {
  int W, H, xdec, ydec, bd;
  int sbc, sbr, nsb, tws, ths;          // superblocks, tile size in superblocks
  int unit[3], cols[3], rows[3], stripe_h[3];
  int ucols_max, urows_max;             // the unit arrays' pitch / rows
};

// RestorationState::new (src/lrf.rs:1197-1343); tiled: more than one tile
__host__ inline void lrf_config(int width, int height, int xdec, int ydec, int base_q_idx, int tiled,
                                int tile_w_sb, int tile_h_sb, LrfPlaneCfg out[3]) {
  auto ilog = [](int v) {
    int n = 0;
    while (v) {
      n++;
      v >>= 1;
    }
    return n;
  };
  const int dec = xdec > 0 && ydec > 0;
  const int y_sb_log2 = 6, uv_h_log2 = y_sb_log2 - xdec, uv_v_log2 = y_sb_log2 - ydec;
  const int base = base_q_idx > 200 ? 0 : base_q_idx > 160 ? 1 : 2;
  int chroma = 0;
  if (dec) {
    if (base == 2) {
      chroma = 1;
    } else {
      const int u = 1 << (8 - base);
      const bool unshifted = ((width >> xdec) - 1) % u <= u / 2 || ((height >> ydec) - 1) % u <= u / 2;
      const bool shifted =
          ((width >> xdec) - 1) % (u >> 1) <= u / 4 || ((height >> ydec) - 1) % (u >> 1) <= u / 4;
      chroma = unshifted && !shifted ? 1 : 0;
    }
  }
  int yu = 1 << (8 - base), uvu = 1 << (8 - (base + chroma));
  if (tiled) {
    const int tzh = __builtin_ctz((unsigned)tile_w_sb), tzv = __builtin_ctz((unsigned)tile_h_sb);
    const int ya = 1 << (y_sb_log2 + (tzh < tzv ? tzh : tzv));
    const int ha = 1 << (uv_h_log2 + tzh), va = 1 << (uv_v_log2 + tzv);
    yu = yu < ya ? yu : ya;
    uvu = uvu < (ha < va ? ha : va) ? uvu : (ha < va ? ha : va);
  }
  const int yl = ilog(yu) - 1, uvl = ilog(uvu) - 1;
  auto atleast1 = [](int v) { return v > 1 ? v : 1; };
  out[0] = {yu, yl - y_sb_log2, yl - y_sb_log2, 64, atleast1((width + (yu >> 1)) / yu),
            atleast1((height + (yu >> 1)) / yu)};
  const int cw = (width + ((1 << xdec) >> 1)) >> xdec, ch = (height + ((1 << ydec) >> 1)) >> ydec;
  for (int p = 1; p < 3; p++)
    out[p] = {uvu, uvl - uv_h_log2, uvl - uv_v_log2, dec ? 32 : 64, atleast1((cw + (uvu >> 1)) / uvu),
              atleast1((ch + (uvu >> 1)) / uvu)};
}

// ---- rates: count_lrf_switchable (src/context.rs:3560-3594) ---------------------
// symbol_bits (src/ec.rs:559-590) at a writer in its initial state (rng
// 0x8000, cnt -9): the replay codes no symbol besides the coefficients
// (DESIGN.md §7), so every price uses this one state.
__host__ __device__ inline uint32_t lrf_frac_compute(uint32_t nbits_total, uint32_t rng) {
  const uint32_t nbits = nbits_total << 3;
  uint32_t l = 0;
  for (int i = 0; i < 3; i++) {
    rng = (rng * rng) >> 15;
    const uint32_t b = rng >> 16;
    l = (l << 1) | b;
    rng >>= b;
  }
  return nbits - l;
}
__host__ __device__ inline uint32_t lrf_symbol_bits(uint32_t s, const uint16_t *cdf, int nsym) {
  const uint32_t full = 0x8000, rng = full >> 8;
  const int cnt = -9;
  const uint32_t fh = (uint32_t)cdf[s] >> 6;
  uint32_t r;
  if (s > 0) {
    const uint32_t fl = (uint32_t)cdf[s - 1] >> 6;
    r = ((rng * fl) >> 1) - ((rng * fh) >> 1) + 4;
  } else {
    r = full - ((rng * fh) >> 1) - ((uint32_t)nsym - s - 1) * 4;
  }
  const uint32_t pre = lrf_frac_compute((uint32_t)(cnt + 9), full);
  const int lg = 32 - __builtin_clz(r);  // r >= 4
  const int d = 16 - lg;
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
  return lrf_frac_compute((uint32_t)(bits + sh + 9), r << d) - pre;
}
// count_quniform / count_subexp / count_signed_subexp_with_ref (src/ec.rs:632-725)
__host__ __device__ inline uint32_t lrf_count_subexp(uint32_t n, uint32_t k, uint32_t v) {
  uint32_t i = 0, mk = 0, bits = 0;
  for (;;) {
    const uint32_t b = i ? k + i - 1 : k, a = 1u << b;
    if (n <= mk + 3 * a) {
      const uint32_t nn = n - mk, vv = v - mk;
      if (nn > 1) {
        int m = 0;
        for (uint32_t t = nn; t > 1; t >>= 1) m++;  // msb
        const uint32_t l = (uint32_t)m + 1, mm = (1u << l) - nn;
        bits += (l - 1) << 3;
        if (vv >= mm) bits += 1 << 3;
      }
      break;
    }
    bits += 1 << 3;
    if (v >= mk + a) {
      i++;
      mk += a;
    } else {
      bits += b << 3;
      break;
    }
  }
  return bits;
}
__host__ __device__ inline uint32_t lrf_recenter(uint32_t r, uint32_t v) {
  return v > (r << 1) ? v : v >= r ? (v - r) << 1 : ((r - v) << 1) - 1;
}
__host__ __device__ inline uint32_t lrf_subexp_ref(int v, int low, int high, uint32_t k, int r) {
  const uint32_t x = (uint32_t)(v - low), n = (uint32_t)(high - low), rr = (uint32_t)(r - low);
  return (rr << 1) <= n ? lrf_count_subexp(n, k, lrf_recenter(rr, x))
                        : lrf_count_subexp(n, k, lrf_recenter(n - 1 - rr, n - 1 - x));
}

// a tile's restoration coding state: lrf_switchable_cdf (shared by the
// planes) and each plane's sgrproj_ref
struct LrfTileState {
  uint16_t cdf[4];
  int8_t ref[3][2];
};
__host__ __device__ inline void lrf_tile_init(LrfTileState &s) {
  s.cdf[0] = 32768 - 9413;  // default_switchable_restore_cdf (src/entropymode.rs:1427-1428)
  s.cdf[1] = 32768 - 22581;
  s.cdf[2] = 0;
  s.cdf[3] = 0;
  for (int p = 0; p < 3; p++) {
    s.ref[p][0] = -32;  // SGRPROJ_XQD_MID
    s.ref[p][1] = 31;
  }
}
__host__ __device__ inline bool lrf_set_has(int set, int i);
// count_lrf_switchable at restoration CDF cdf and the plane's sgrproj_ref
// (r0, r1); set < 0: None
__host__ __device__ inline uint32_t lrf_rate_at(const uint16_t *cdf, int r0, int r1, int set, int x0, int x1) {
  if (set < 0) return lrf_symbol_bits(0, cdf, 3);
  uint32_t bits = lrf_symbol_bits(2, cdf, 3) + (4u << 3);  // + SGRPROJ_PARAMS_BITS
  if (lrf_set_has(set, 0)) bits += lrf_subexp_ref(x0, -96, 32, 4, r0);
  if (lrf_set_has(set, 1)) bits += lrf_subexp_ref(x1, -32, 96, 4, r1);
  return bits;
}
__host__ __device__ inline uint32_t lrf_rate(const LrfTileState &s, int p, int set, const int8_t *xqd) {
  return set < 0 ? lrf_rate_at(s.cdf, 0, 0, -1, 0, 0)
                 : lrf_rate_at(s.cdf, s.ref[p][0], s.ref[p][1], set, xqd[0], xqd[1]);
}
// write_lrf's updates (src/context.rs:3596-3659): symbol_with_update's
// update_cdf (src/ec.rs:891-905) and the plane's sgrproj_ref
__host__ __device__ inline void lrf_commit(LrfTileState &s, int p, int set, const int8_t *xqd) {
  const uint32_t val = set < 0 ? 0 : 2;
  const int ns = 3, rate = 3 + 1 + (s.cdf[ns] >> 4);
  s.cdf[ns] = (uint16_t)(s.cdf[ns] + 1 - (s.cdf[ns] >> 5));
  for (int i = 0; i < ns - 1; i++)
    s.cdf[i] = (uint32_t)i >= val ? (uint16_t)(s.cdf[i] - (s.cdf[i] >> rate))
                                  : (uint16_t)(s.cdf[i] + ((32768 - s.cdf[i]) >> rate));
  if (set < 0) return;
  for (int i = 0; i < 2; i++) s.ref[p][i] = lrf_set_has(set, i) ? xqd[i] : (i == 0 ? 0 : 95);
}
// the sets with a radius-2 / radius-1 filter (SGRPROJ_PARAMS_S non-zero)
__host__ __device__ inline bool lrf_set_has(int set, int i) {
  return i == 0 ? set < 10 || set > 13 : set < 14;
}

// sgrproj_solve's tail (src/lrf.rs:920-964) from the exact sums
__host__ __device__ inline void lrf_solve_finish(int set, int w, int h, int64_t H00, int64_t H01,
                                                 int64_t H11, int64_t C0, int64_t C1, int8_t xqd[2]) {
  const bool r2 = lrf_set_has(set, 0), r1 = lrf_set_has(set, 1);
  const double n = (double)w * (double)h;
  double h00 = (double)H00, h01 = (double)H01, h11 = (double)H11, c0 = (double)C0, c1 = (double)C1;
  h00 /= n;
  h01 /= n;
  h11 /= n;
  const double h10 = h01;
  const double sc = 128.0 / n;
  c0 *= sc;
  c1 *= sc;
  int xq0, xq1;
  if (!r2) {
    xq0 = 0;
    xq1 = h11 == 0. ? 0 : (int)round(c1 / h11);
  } else if (!r1) {
    xq0 = h00 == 0. ? 0 : (int)round(c0 / h00);
    xq1 = 0;
  } else {
    const double det = h00 * h11 - h01 * h10;
    if (det == 0.) {
      xq0 = xq1 = 0;
    } else {
      const double d1 = h11 * c0 - h01 * c1, d2 = h00 * c1 - h10 * c0;
      xq0 = (int)round(d1 / det);
      xq1 = (int)round(d2 / det);
    }
  }
  const int x0 = xq0 < -96 ? -96 : xq0 > 31 ? 31 : xq0;
  const int t = 128 - x0 - xq1, x1 = t < -32 ? -32 : t > 95 ? 95 : t;
  xqd[0] = (int8_t)x0;
  xqd[1] = (int8_t)x1;
}

// rv_lrf.hip
int lrf_geometry(int width, int height, int xdec, int ydec, int bit_depth, int base_q_idx, int tile_w_sb,
                 int tile_h_sb, LrfGeo *g);
int lrf_rdo_launch(const rv_plane rec[3], const rv_plane src[3], const uint8_t *skip, int mi_stride,
                   const float *imp, int w_imp, int w_in_b, int h_in_b, const LrfGeo &g, int cdef,
                   const uint8_t *dir, const int32_t *var, const uint8_t cdef_str[2], const double ds[3],
                   uint64_t *err, int8_t *xqd, const int32_t *rect, hipStream_t s);
int lrf_decide_launch(const LrfGeo &g, const uint64_t *err, const int8_t *xqd, double lambda, int8_t *units,
                      const int32_t *rect, int fix_passes, hipStream_t s);
int lrf_filter_launch(const rv_plane cd[3], const rv_plane db[3], const rv_plane out[3], const LrfGeo &g,
                      const int8_t *units, int enable_cdef, hipStream_t s);
