// rv_quant.h -- quantize / dequantize (src/quantize.rs) for one transform
// block per group of LPB lanes (a wavefront or a half), on coefficients in
// LDS.  Shared by the standalone batch launch (rv_quant.hip) and the fused
// RDO kernel (rv_rdo.hip).
//
// QuantizationContext::quantize (src/quantize.rs:255-316) is a scan-order
// loop whose rounding offset depends on a 2-state `level_mode` carried from
// coefficient to coefficient.  Here every lane takes a contiguous chunk of
// scan indices:
//   1. eob = the last scan index >= 1 whose |coeff| reaches the deadzone
//      (a max over the lanes);
//   2. each lane composes, over its chunk, the state transition the loop
//      applies from level_mode 0 and from level_mode 1 -- a map {0,1} ->
//      {0,1} in two bits;
//   3. an exclusive prefix composition of the lanes' maps (log2(LPB)
//      shuffle steps, starting from level_mode = 1) gives every lane the
//      level_mode entering its chunk;
//   4. each lane re-runs its chunk from that state and writes the levels.
// The result is the reference's sequential loop, position for position.
#pragma once

#include "rv_device.h"
#include "rv_quant_tables.h"

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

// The level of one AC coefficient under level_mode `mode`; *next = the
// level_mode after it (src/quantize.rs:293-311).
__device__ __forceinline__ int32_t q_ac_level(const QCtx &c, int32_t raw, int mode, int *next) {
  const int32_t coeff = (int32_t)((uint32_t)raw << c.log_tx_scale);
  const int32_t level0 = q_divu(coeff, c.ac_a, c.ac_b, c.ac_s);
  const int32_t offset = level0 > 1 - mode ? c.ac_offset1 : c.ac_offset0;
  const int32_t q = q_divu(wadd(coeff, q_signum(coeff) * offset), c.ac_a, c.ac_b, c.ac_s);
  *next = (mode != 0 && q == 0) ? 0 : (q > 1 ? 1 : mode);
  return q;
}

// Quantize + dequantize one block: `co(pos)` reads the forward transform's
// coefficient at scan position pos (< n = coded_tx_area); `put(pos, q, r)`
// receives the level (qcoeffs[pos]) and the dequantized value
// (rcoeffs[pos], src/quantize.rs:319-333).  Every position is written
// exactly once, by the lane that read it (so `put` may overwrite `co`'s
// storage in place).  All LPB lanes of the group call it; returns eob.
template <int LPB, typename Co, typename Put>
__device__ __forceinline__ int quantize_block(const QCtx &c, const uint16_t *scan, int n, Co co,
                                              Put put) {
  const int lane = threadIdx.x & (LPB - 1);
  const int K = (n + LPB - 1) / LPB;  // scan indices per lane (n is a power of 2 >= 16)
  const int i0 = lane * K, i1 = i0 + K < n ? i0 + K : n;
  // 1. eob
  int last = 0;
  for (int i = i0; i < i1; i++) {
    const int32_t v = co(scan[i]);
    if (i >= 1 && (v < 0 ? wsub(0, v) : v) >= c.deadzone) last = i;
  }
#pragma unroll
  for (int o = LPB / 2; o > 0; o >>= 1) {
    const int w = __shfl_xor(last, o, LPB);
    last = w > last ? w : last;
  }
  const int eob = last >= 1 ? last : 1;
  // 2. this lane's transition map over scan indices [max(i0,1), min(i1, eob + 1))
  int map = 2;  // identity: (f(0), f(1)) = (0, 1), f(s) = (map >> s) & 1
  for (int i = i0 < 1 ? 1 : i0; i < i1 && i <= eob; i++) {
    const int32_t raw = co(scan[i]);
    int n0, n1;
    q_ac_level(c, raw, 0, &n0);
    q_ac_level(c, raw, 1, &n1);
    const int f0 = (map >> 0) & 1, f1 = (map >> 1) & 1;  // compose: T o map
    map = (f0 ? n1 : n0) | ((f1 ? n1 : n0) << 1);
  }
  // 3. inclusive prefix of maps in lane order (P_l = M_l o ... o M_0), then
  // the state entering this lane's chunk = P_{l-1}(1)
  int pre = map;
#pragma unroll
  for (int d = 1; d < LPB; d <<= 1) {
    const int other = __shfl_up(pre, d, LPB);
    if (lane >= d) {
      const int a0 = (other >> 0) & 1, a1 = (other >> 1) & 1;  // pre o other
      pre = ((pre >> a0) & 1) | (((pre >> a1) & 1) << 1);
    }
  }
  int prev = __shfl_up(pre, 1, LPB);
  int mode = lane == 0 ? 1 : (prev >> 1) & 1;
  // 4. levels and dequantized values
  const int32_t roff = (1 << c.log_tx_scale) - 1;
  for (int i = i0; i < i1; i++) {
    const int pos = scan[i];
    int32_t q;
    if (i == 0) {
      int32_t dc = (int32_t)((uint32_t)co(0) << c.log_tx_scale);
      dc = wadd(dc, q_signum(dc) * c.dc_offset);
      q = q_divu(dc, c.dc_a, c.dc_b, c.dc_s);
    } else if (i <= eob) {
      int nx;
      q = q_ac_level(c, co(pos), mode, &nx);
      mode = nx;
    } else {
      q = 0;
    }
    const int32_t r = wadd(wmul(q, i == 0 ? c.dc_quant : c.ac_quant), (q >> 31) & roff) >> c.log_tx_scale;
    put(pos, q, r);
  }
  return eob;
}

}  // namespace rv
