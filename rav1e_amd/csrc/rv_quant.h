// rv_quant.h -- quantize / dequantize (src/quantize.rs) for one transform
// block per group of LPB lanes (a wavefront or a half), on coefficients in
// LDS.  Shared by the standalone batch launch (rv_quant.hip) and the fused
// RDO kernel (rv_rdo.hip).
//
// QuantizationContext::quantize (src/quantize.rs:255-316) is a scan-order
// loop whose rounding offset depends on a 2-state `level_mode` carried from
// coefficient to coefficient.  Here every lane takes a contiguous chunk of
// scan indices:
//   1. eob = the last scan index >= 1 whose |coeff| reaches the deadzone:
//      the value held by the highest lane with one (a ballot);
//   2. each lane composes, over its chunk, the state transition the loop
//      applies from level_mode 0 and from level_mode 1 -- a map {0,1} ->
//      {0,1}, always the identity or a constant;
//   3. the level_mode entering a lane's chunk is the constant of the last
//      constant map below it (two ballots), else the initial 1;
//   4. each lane re-runs its chunk from that state and writes the levels.
// The result is the reference's sequential loop, position for position.
// Every lane of the wavefront calls it together (ballots are wave-wide).
#pragma once

#include "rv_device.h"
#include "rv_quant_tables.h"
#include "rv_rate_table.h"

namespace rv {

struct QCtx {  // QuantizationContext (src/quantize.rs:108-120)
  int log_tx_scale;
  int32_t dc_quant, dc_offset, ac_quant, ac_offset0, ac_offset1, deadzone;
  uint32_t dc_a, dc_b, dc_s, ac_a, ac_b, ac_s;  // divu_gen
};

// get_log_tx_scale (src/quantize.rs:35-40) from the transform area
__host__ __device__ __forceinline__ int q_log_tx_scale(int area) {
  return (area > 256) + (area > 1024);
}

__device__ __forceinline__ int q_lookup(int ac, int qindex, int delta_q, int bd) {
  int i = qindex + delta_q;
  i = i < 0 ? 0 : i > 255 ? 255 : i;
  return RV_QLOOKUP[(3 * ac + (bd - 8) / 2) * 256 + i];
}

// divu_gen (src/quantize.rs:122-137)
__device__ __forceinline__ void q_divu_gen(uint32_t d, uint32_t &a, uint32_t &b, uint32_t &s) {
  const uint32_t m = 31u - (uint32_t)__builtin_clz(d);
  s = m;
  if ((d & (d - 1)) == 0) {
    a = b = 0xFFFFFFFFu;
  } else {
    const uint64_t t = (1ull << (m + 32)) / d;
    const uint64_t r = (t * d + d) & 0xFFFFFFFFull;
    if (r <= (1ull << m)) {
      a = (uint32_t)t + 1;
      b = 0;
    } else {
      a = b = (uint32_t)t;
    }
  }
}

// divu_pair (src/quantize.rs:139-153): ((a * |x| + b) >> 32) >> s, signed
__device__ __forceinline__ int32_t q_divu(int32_t x, uint32_t a, uint32_t b, uint32_t s) {
  const uint32_t y = (uint32_t)(x < 0 ? wsub(0, x) : x);
  const uint32_t lo = a * y, hi = __umulhi(a, y);
  const uint32_t sum = lo + b;
  const uint32_t q = (hi + (sum < lo ? 1u : 0u)) >> s;
  return x < 0 ? wsub(0, (int32_t)q) : (int32_t)q;
}

// QuantizationContext::update (src/quantize.rs:205-253)
__device__ __forceinline__ QCtx q_ctx(int qindex, int area, int is_intra, int bd, int dc_delta_q,
                                      int ac_delta_q) {
  QCtx c;
  c.log_tx_scale = q_log_tx_scale(area);
  c.dc_quant = q_lookup(0, qindex, dc_delta_q, bd);
  c.ac_quant = q_lookup(1, qindex, ac_delta_q, bd);
  q_divu_gen((uint32_t)c.dc_quant, c.dc_a, c.dc_b, c.dc_s);
  q_divu_gen((uint32_t)c.ac_quant, c.ac_a, c.ac_b, c.ac_s);
  c.dc_offset = c.dc_quant * (is_intra ? 109 : 108) / 256;
  c.ac_offset0 = c.ac_quant * (is_intra ? 98 : 97) / 256;
  c.ac_offset1 = c.ac_quant * (is_intra ? 109 : 108) / 256;
  const int32_t off_eob = c.ac_quant * (is_intra ? 88 : 44) / 256;
  c.deadzone = (c.ac_quant - off_eob + (1 << c.log_tx_scale) - 1) >> c.log_tx_scale;
  return c;
}

__device__ __forceinline__ int32_t q_signum(int32_t v) { return (v > 0) - (v < 0); }

// Quantize + dequantize one block of N = coded_tx_area positions: `co(pos)`
// reads the forward transform's coefficient at scan position pos; `put(pos,
// q, r)` receives the level (qcoeffs[pos]) and the dequantized value
// (rcoeffs[pos], src/quantize.rs:319-333).  Every position is written
// exactly once, by the lane that read it (so `put` may overwrite `co`'s
// storage in place).  All LPB lanes of the group call it; returns eob.
//
// divu_pair is exact truncating division (its construction, and the
// reference's own test, src/quantize.rs:160-168), and the coefficient and
// its rounding offset have the same sign, so with a = |coeff << scale| and
// the offset o the loop picks (src/quantize.rs:293-311):
//   level0 > 1 - mode   <=>  coeff > 0 and a >= (mode ? 1 : 2) * ac_quant
//   level == 0          <=>  a + o < ac_quant
//   level > 1           <=>  coeff > 0 and a + o >= 2 * ac_quant
// so the level_mode transitions need comparisons only and each coefficient
// is divided once, in the final pass.  Valid for |coefficient| < 2^28 (the
// forward transforms stay below 2^21, tools/txbounds).
template <int N, int LPB, typename Co, typename Put>
__device__ __forceinline__ int quantize_block(const QCtx &c, const uint16_t *scan, Co co,
                                              Put put) {
  constexpr int K = N >= LPB ? N / LPB : 1;  // scan indices per lane
  const int lane = rv_tid() & (LPB - 1);
  const int i0 = lane * K;
  const bool live = i0 < N;
  const int s = c.log_tx_scale;
  const int32_t acq = c.ac_quant, acq2 = 2 * c.ac_quant;
  // coefficients << log_tx_scale: held in registers for up to 16 per lane,
  // re-read from `co` per pass beyond that (register budget of the fused
  // kernels)
  constexpr bool kCache = K <= 16;
  constexpr int kUnroll = kCache ? K : 2;
  int32_t cf[kCache ? K : 1];
  if constexpr (kCache) {
#pragma unroll
    for (int k = 0; k < K; k++) cf[k] = live ? (int32_t)((uint32_t)co(scan[i0 + k]) << s) : 0;
  }
  auto coef = [&](int k) __attribute__((always_inline)) -> int32_t {
    if constexpr (kCache) return cf[k];
    return live ? (int32_t)((uint32_t)co(scan[i0 + k]) << s) : 0;
  };
  // 1. eob: the deadzone test is on the unscaled magnitude
  int last = 0;
#pragma unroll kUnroll
  for (int k = 0; k < K; k++) {
    const int32_t v = coef(k) >> s;
    if (i0 + k >= 1 && (v < 0 ? -v : v) >= c.deadzone) last = i0 + k;
  }
  // lanes of this group in the wavefront's 64-bit masks
  const int wl = rv_tid() & 63;
  const uint64_t gmask = LPB == 64 ? ~0ull : (((1ull << LPB) - 1) << (wl & ~(LPB - 1)));
  const uint64_t sig = __ballot(last >= 1) & gmask;
  // chunks ascend with the lane, so the highest lane holding a significant
  // coefficient holds the eob
  const int eob = sig ? __shfl(last, 63 - __builtin_clzll(sig), 64) : 1;
  // 2. this lane's transition map over its indices in [1, eob]:
  // T(0) = [level under mode 0 > 1], T(1) = [level under mode 1 != 0].
  // T(0) <= T(1) always (mode 1 never picks the smaller offset), so every
  // map and composition is the identity (2), constant 0 (0) or constant 1 (3).
  int map = 2;  // f(st) = (map >> st) & 1
#pragma unroll kUnroll
  for (int k = 0; k < K; k++) {
    const int i = i0 + k;
    if (i >= 1 && i <= eob) {
      const int32_t v = coef(k), a = v < 0 ? -v : v;
      const int32_t o0 = v > 0 && a >= acq2 ? c.ac_offset1 : c.ac_offset0;
      const int32_t o1 = v > 0 && a >= acq ? c.ac_offset1 : c.ac_offset0;
      const int t0 = v > 0 && a + o0 >= acq2;
      const int t1 = a + o1 >= acq;
      const int f0 = map & 1, f1 = (map >> 1) & 1;
      map = (f0 ? t1 : t0) | ((f1 ? t1 : t0) << 1);
    }
  }
  // 3. the level_mode entering this lane's chunk: the constant of the last
  // non-identity map below this lane in the group, else the initial 1
  const uint64_t nonid = __ballot(map != 2) & gmask;
  const uint64_t ones = __ballot(map == 3) & gmask;
  const uint64_t below = nonid & ((1ull << wl) - 1);
  int mode = below ? (int)((ones >> (63 - __builtin_clzll(below))) & 1) : 1;
  // 4. levels (one division each) and dequantized values
  const int32_t roff = (1 << s) - 1;
#pragma unroll kUnroll
  for (int k = 0; k < K; k++) {
    const int i = i0 + k;
    if (!live) break;
    const int32_t v = coef(k);
    int32_t q;
    if (i == 0) {
      q = q_divu(wadd(v, q_signum(v) * c.dc_offset), c.dc_a, c.dc_b, c.dc_s);
    } else if (i <= eob) {
      const int32_t a = v < 0 ? -v : v;
      const int32_t o = v > 0 && a >= (mode ? acq : acq2) ? c.ac_offset1 : c.ac_offset0;
      q = q_divu(wadd(v, q_signum(v) * o), c.ac_a, c.ac_b, c.ac_s);
      mode = (mode != 0 && q == 0) ? 0 : (q > 1 ? 1 : mode);
    } else {
      q = 0;
    }
    const int32_t r = wadd(wmul(q, i == 0 ? c.dc_quant : c.ac_quant), (q >> 31) & roff) >> s;
    put(scan[i], q, r);
  }
  return eob;
}

// dequantize (src/quantize.rs:319-333) of the level at raster index i
__device__ __forceinline__ int32_t q_dequant(const QCtx &c, int32_t q, int i) {
  return wadd(wmul(q, i == 0 ? c.dc_quant : c.ac_quant), (q >> 31) & ((1 << c.log_tx_scale) - 1)) >>
         c.log_tx_scale;
}

// estimate_rate (src/rdo.rs:204-216): the rate read off the trained table,
// linearly interpolated between the two distortion bins around the block's
// tx-domain distortion; i64 as in the reference (the bins differ by one, so
// the divisor is RATE_EST_BIN_SIZE and the division truncates toward zero).
__device__ __forceinline__ uint64_t q_estimate_rate(int qindex, int tx_size, uint64_t fd) {
  const uint32_t *row =
      RV_RDO_RATE_TABLE + ((qindex / RV_RDO_QUANT_DIV) * 19 + tx_size) * RV_RDO_NUM_BINS;
  uint64_t down = fd / RV_RATE_EST_BIN_SIZE;
  down = down < RV_RDO_NUM_BINS - 2 ? down : RV_RDO_NUM_BINS - 2;
  const uint64_t up = down + 1;
  const int64_t x0 = (int64_t)(down * RV_RATE_EST_BIN_SIZE);
  const int64_t y0 = row[down], y1 = row[up];
  const int64_t slope = (int64_t)((uint64_t)(y1 - y0) << 8) / RV_RATE_EST_BIN_SIZE;
  const int64_t r = y0 + ((int64_t)((uint64_t)((int64_t)fd - x0) * (uint64_t)slope) >> 8);
  return r > 0 ? (uint64_t)r : 0;
}

}  // namespace rv
