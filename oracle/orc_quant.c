/* CPU oracle (test infrastructure only): quantize / dequantize of
 * src/quantize.rs, the step of encode_tx_block (src/encoder.rs:1170, 1192)
 * between the forward and the inverse transform.
 *
 * i32 coefficients as in encode_tx_block (qcoeffs: [i32; 32 * 32]); i32
 * arithmetic wraps (Rust release).  Tables: orc_quant_tables.h (generated,
 * checked against the reference's). */
#include <stdlib.h>

#include "orc_common.h"
#include "orc_quant_tables.h"

/* get_log_tx_scale (src/quantize.rs:35-40) */
int orc_get_log_tx_scale(int tx_size) {
  const int area = 1 << (ORC_TX_W_LOG2[tx_size] + ORC_TX_H_LOG2[tx_size]);
  return (area > 256) + (area > 1024);
}

/* av1_get_coded_tx_size(tx_size).area() (src/context.rs:1949-1956) */
int orc_coded_tx_area(int tx_size) {
  const int w = 1 << ORC_TX_W_LOG2[tx_size], h = 1 << ORC_TX_H_LOG2[tx_size];
  return (w < 32 ? w : 32) * (h < 32 ? h : 32);
}

static int qtab(int ac, int qindex, int delta_q, int bd) {
  int i = qindex + delta_q;
  i = i < 0 ? 0 : i > 255 ? 255 : i;
  return ORC_QLOOKUP[(3 * ac + (bd - 8) / 2) * 256 + i];
}
/* dc_q / ac_q (src/quantize.rs:42-62) */
int orc_dc_q(int qindex, int delta_q, int bd) { return qtab(0, qindex, delta_q, bd); }
int orc_ac_q(int qindex, int delta_q, int bd) { return qtab(1, qindex, delta_q, bd); }

/* divu_gen (src/quantize.rs:122-137): (a, b, shift) with
 * x / d == ((a * |x| + b) >> 32) >> shift */
void orc_divu_gen(uint32_t d, uint32_t out[3]) {
  const uint64_t m = 31 - (uint64_t)__builtin_clz(d);
  if ((d & (d - 1)) == 0) {
    out[0] = 0xFFFFFFFFu;
    out[1] = 0xFFFFFFFFu;
    out[2] = (uint32_t)m;
  } else {
    const uint64_t t = (1ull << (m + 32)) / d;
    const uint64_t r = (t * d + d) & 0xFFFFFFFFull;
    if (r <= (1ull << m)) {
      out[0] = (uint32_t)t + 1;
      out[1] = 0;
    } else {
      out[0] = (uint32_t)t;
      out[1] = (uint32_t)t;
    }
    out[2] = (uint32_t)m;
  }
}

/* divu_pair (src/quantize.rs:139-153) */
int32_t orc_divu_pair(int32_t x, const uint32_t d[3]) {
  const uint64_t y = (uint64_t)(uint32_t)(x < 0 ? w_sub(0, x) : x);
  const int32_t q = (int32_t)(((((uint64_t)d[0] * y + d[1]) >> 32) >> d[2]));
  return x < 0 ? w_sub(0, q) : q;
}

/* QuantizationContext::update (src/quantize.rs:205-253) */
void orc_qctx_update(orc_qctx *c, int qindex, int tx_size, int is_intra, int bd,
                     int dc_delta_q, int ac_delta_q) {
  c->log_tx_scale = orc_get_log_tx_scale(tx_size);
  c->dc_quant = (uint32_t)orc_dc_q(qindex, dc_delta_q, bd);
  orc_divu_gen(c->dc_quant, c->dc_mul_add);
  c->ac_quant = (uint32_t)orc_ac_q(qindex, ac_delta_q, bd);
  orc_divu_gen(c->ac_quant, c->ac_mul_add);
  c->dc_offset = (int32_t)c->dc_quant * (is_intra ? 109 : 108) / 256;
  c->ac_offset0 = (int32_t)c->ac_quant * (is_intra ? 98 : 97) / 256;
  c->ac_offset1 = (int32_t)c->ac_quant * (is_intra ? 109 : 108) / 256;
  c->ac_offset_eob = (int32_t)c->ac_quant * (is_intra ? 88 : 44) / 256;
}

static int32_t signum(int32_t v) { return (v > 0) - (v < 0); }

/* QuantizationContext::quantize (src/quantize.rs:255-316).  coeffs: the
 * forward transform's output, indexed by scan position (< coded_tx_area);
 * qcoeffs: coded_tx_area entries.  Returns eob as the reference computes it
 * (1 + the index in scan[1..] of the last coefficient at or above the
 * deadzone, 1 if there is none). */
int orc_quantize(const orc_qctx *c, const int32_t *coeffs, int32_t *qcoeffs, int tx_size,
                 int tx_type) {
  const uint16_t *scan = ORC_SCANS + ORC_SCAN_OFF[tx_size * 16 + tx_type];
  const int n = orc_coded_tx_area(tx_size);
  const int s = c->log_tx_scale;
  const int32_t deadzone =
      (int32_t)(((size_t)(c->ac_quant - (uint32_t)c->ac_offset_eob) + (1u << s) - 1) >> s);
  int eob = 1;
  for (int i = n - 1; i >= 1; i--) {
    const int32_t v = coeffs[scan[i]];
    if ((v < 0 ? w_sub(0, v) : v) >= deadzone) {
      eob = i;  /* rposition in scan[1..] = i - 1, eob = that + 1 */
      break;
    }
  }
  int32_t dc = (int32_t)((uint32_t)coeffs[0] << s);
  dc = w_add(dc, w_mul(signum(dc), c->dc_offset));
  qcoeffs[0] = orc_divu_pair(dc, c->dc_mul_add);
  int level_mode = 1;
  for (int i = 1; i <= eob && i < n; i++) {
    const int pos = scan[i];
    const int32_t coeff = (int32_t)((uint32_t)coeffs[pos] << s);
    const int32_t level0 = orc_divu_pair(coeff, c->ac_mul_add);
    const int32_t offset = level0 > 1 - level_mode ? c->ac_offset1 : c->ac_offset0;
    const int32_t q = orc_divu_pair(w_add(coeff, w_mul(signum(coeff), offset)), c->ac_mul_add);
    qcoeffs[pos] = q;
    if (level_mode != 0 && q == 0)
      level_mode = 0;
    else if (q > 1)
      level_mode = 1;
  }
  for (int i = eob + 1; i < n; i++) qcoeffs[scan[i]] = 0;
  return eob;
}

/* dequantize (src/quantize.rs:319-333): coded_tx_area entries */
void orc_dequantize(int qindex, const int32_t *coeffs, int32_t *rcoeffs, int tx_size, int bd,
                    int dc_delta_q, int ac_delta_q) {
  const int s = orc_get_log_tx_scale(tx_size);
  const int32_t offset = (1 << s) - 1;
  const int32_t dcq = orc_dc_q(qindex, dc_delta_q, bd), acq = orc_ac_q(qindex, ac_delta_q, bd);
  const int n = orc_coded_tx_area(tx_size);
  for (int i = 0; i < n; i++) {
    const int32_t c = coeffs[i];
    rcoeffs[i] = w_add(w_mul(c, i == 0 ? dcq : acq), asr(c, 31) & offset) >> s;
  }
}

/* estimate_rate (src/rdo.rs:204-216): linear interpolation in the trained
 * RDO_RATE_TABLE between the two distortion bins around fast_distortion
 * (the tx-domain distortion of src/encoder.rs:1210-1224), i64 arithmetic. */
#include "orc_rate_table.h"
uint64_t orc_estimate_rate(int qindex, int tx_size, uint64_t fast_distortion) {
  const int q_bin = qindex / RV_RDO_QUANT_DIV;
  uint64_t down = fast_distortion / RV_RATE_EST_BIN_SIZE;
  if (down > RV_RDO_NUM_BINS - 2) down = RV_RDO_NUM_BINS - 2;
  uint64_t up = down + 1;
  if (up > RV_RDO_NUM_BINS - 1) up = RV_RDO_NUM_BINS - 1;
  const int64_t x0 = (int64_t)(down * RV_RATE_EST_BIN_SIZE);
  const int64_t x1 = (int64_t)(up * RV_RATE_EST_BIN_SIZE);
  const uint32_t *row = RV_RDO_RATE_TABLE + ((size_t)q_bin * 19 + tx_size) * RV_RDO_NUM_BINS;
  const int64_t y0 = row[down], y1 = row[up];
  const int64_t slope = (int64_t)((uint64_t)(y1 - y0) << 8) / (x1 - x0); /* truncates */
  const int64_t d = (int64_t)fast_distortion - x0;
  const int64_t r = y0 + ((int64_t)((uint64_t)d * (uint64_t)slope) >> 8); /* wrapping mul */
  return r > 0 ? (uint64_t)r : 0;
}
