/*
 * orc_ec.c -- CPU restatement of rav1e's range coder and coefficient coder.
 *
 * TEST INFRASTRUCTURE ONLY (see rav1e_oracle.h).  It is the checker of the
 * product's device tokenizer + host range coder (rav1e_amd/csrc/rv_ec.hip).
 *
 *   - WriterBase<WriterEncoder> (src/ec.rs:100-600): store / lr_compute /
 *     symbol / symbol_with_update / bool / bit / literal / write_golomb /
 *     done, and native::update_cdf (src/ec.rs:891-905);
 *   - the Reader of ec.rs's own test module (src/ec.rs:914-1010), restated as
 *     a decoder for round-trip checks;
 *   - ContextWriter::write_coeffs_lv_map (src/context.rs:3965-4220) with
 *     BlockContext's coefficient contexts: get_txb_ctx (:1776-1868),
 *     set_coeff_context / set_dc_sign (:1586-1609), reset_skip_context
 *     (:1651-1679), reset_left_contexts (:1681-1688), txb_init_levels,
 *     get_eob_pos_token, get_nz_mag / get_nz_map_ctx_from_stats /
 *     get_nz_map_contexts, get_br_ctx (:3755-3930), write_tx_type (:3419-3460,
 *     inter sets).  Square transform sizes only (the ones the replay codes).
 *
 * Pinned by vectors made by evaluating the reference's own text
 * (tools/refeval/gen_golden_ref.py gen_ec -> tests/golden/ref_ec.npz) and by
 * ec.rs's own tests run through the same evaluator (tools/refeval/gen_kat.py).
 * Integer types follow the reference: ec_window = u32, cnt i16, rng u16.
 */
#include <stdlib.h>
#include <string.h>

#include "orc_common.h"
#include "orc_ec_tables.h"
#include "orc_quant_tables.h"

_Static_assert(ORC_EC_TOTAL == ORC_EC_CDF_TOTAL, "CDF table layout");

#define EC_PROB_SHIFT 6
#define EC_MIN_PROB 4

/* ------------------------------------------------------------ writer */
void orc_ecw_init(orc_ecw *w) {
  memset(w, 0, sizeof(*w));
  w->rng = 0x8000;  /* WriterBase::new (src/ec.rs:320-337) */
  w->cnt = -9;
}

void orc_ecw_free(orc_ecw *w) {
  free(w->pre);
  w->pre = NULL;
  w->n = w->cap = 0;
}

static void push_pre(orc_ecw *w, uint16_t v) {
  if (w->n == w->cap) {
    w->cap = w->cap ? 2 * w->cap : 256;
    w->pre = (uint16_t *)realloc(w->pre, w->cap * sizeof(uint16_t));
  }
  w->pre[w->n++] = v;
}

static int ilog16(uint32_t r) { /* ILog for u16 (src/util/mod.rs:227-229) */
  int b = 0;
  while (r) {
    b++;
    r >>= 1;
  }
  return b;
}

/* lr_compute + StorageBackend::store for WriterEncoder (src/ec.rs:270-295, 339-364) */
int32_t *orc_ec_slog = NULL;  /* debugging aid: (fl, fh, nms) of every store */
int orc_ec_slog_n = 0;

static void ecw_store(orc_ecw *w, uint16_t fl, uint16_t fh, uint16_t nms) {
  if (orc_ec_slog) {
    orc_ec_slog[3 * orc_ec_slog_n] = fl;
    orc_ec_slog[3 * orc_ec_slog_n + 1] = fh;
    orc_ec_slog[3 * orc_ec_slog_n + 2] = nms;
    orc_ec_slog_n++;
  }
  uint32_t r = w->rng, l, rr;
  if (fl < 32768) {
    uint32_t u = (((r >> 8) * ((uint32_t)fl >> EC_PROB_SHIFT)) >> (7 - EC_PROB_SHIFT)) +
                 EC_MIN_PROB * (uint32_t)nms;
    uint32_t v = (((r >> 8) * ((uint32_t)fh >> EC_PROB_SHIFT)) >> (7 - EC_PROB_SHIFT)) +
                 EC_MIN_PROB * (uint32_t)(uint16_t)(nms - 1);
    l = r - u;
    rr = (uint16_t)(u - v);
  } else {
    r -= (((r >> 8) * ((uint32_t)fh >> EC_PROB_SHIFT)) >> (7 - EC_PROB_SHIFT)) +
         EC_MIN_PROB * (uint32_t)(uint16_t)(nms - 1);
    l = 0;
    rr = (uint16_t)r;
  }
  uint32_t low = l + w->low;
  int16_t c = w->cnt;
  const int d = 16 - ilog16(rr & 0xFFFF);
  int16_t s = (int16_t)(c + d);
  if (s >= 0) {
    c = (int16_t)(c + 16);
    uint32_t m = (1u << c) - 1;
    if (s >= 8) {
      push_pre(w, (uint16_t)(low >> c));
      low &= m;
      c = (int16_t)(c - 8);
      m >>= 8;
    }
    push_pre(w, (uint16_t)(low >> c));
    s = (int16_t)(c + d - 24);
    low &= m;
  }
  w->low = low << d;
  w->rng = (uint16_t)(rr << d);
  w->cnt = s;
}

/* Writer::symbol (src/ec.rs:523-531): cdf holds n entries, cdf[n-1] == 0 */
void orc_ecw_symbol(orc_ecw *w, uint32_t s, const uint16_t *cdf, int n) {
  const uint16_t nms = (uint16_t)(n - (int)s);
  const uint16_t fl = s > 0 ? cdf[s - 1] : 32768;
  const uint16_t fh = cdf[s];
  ecw_store(w, fl, fh, nms);
}

/* native::update_cdf (src/ec.rs:891-905): len = nsymbs + 1 (the counter last) */
void orc_update_cdf(uint16_t *cdf, int len, uint32_t val) {
  const int nsymbs = len - 1;
  const int rate = 3 + (nsymbs >> 1 < 2 ? nsymbs >> 1 : 2) + (cdf[nsymbs] >> 4);
  cdf[nsymbs] = (uint16_t)(cdf[nsymbs] + 1 - (cdf[nsymbs] >> 5));
  for (int i = 0; i < nsymbs - 1; i++) {
    if ((uint32_t)i >= val)
      cdf[i] = (uint16_t)(cdf[i] - (cdf[i] >> rate));
    else
      cdf[i] = (uint16_t)(cdf[i] + ((32768 - cdf[i]) >> rate));
  }
}

/* debugging aid: when set, every coded symbol is appended as (s, len, cdf[0]) */
int32_t *orc_ec_log = NULL;
int orc_ec_log_n = 0;

/* Writer::symbol_with_update (src/ec.rs:540-557): len = nsymbs + 1 */
void orc_ecw_symbol_update(orc_ecw *w, uint32_t s, uint16_t *cdf, int len) {
  if (orc_ec_log) {
    orc_ec_log[3 * orc_ec_log_n] = (int32_t)s;
    orc_ec_log[3 * orc_ec_log_n + 1] = len;
    orc_ec_log[3 * orc_ec_log_n + 2] = cdf[0];
    orc_ec_log_n++;
  }
  orc_ecw_symbol(w, s, cdf, len - 1);
  orc_update_cdf(cdf, len, s);
}

/* Writer::bool / bit / literal / write_golomb (src/ec.rs:493-521, 595-613) */
void orc_ecw_bool(orc_ecw *w, int val, uint16_t f) {
  const uint16_t cdf[2] = {f, 0};
  orc_ecw_symbol(w, val ? 1 : 0, cdf, 2);
}
void orc_ecw_bit(orc_ecw *w, int bit) {
  if (orc_ec_log) {
    orc_ec_log[3 * orc_ec_log_n] = bit;
    orc_ec_log[3 * orc_ec_log_n + 1] = -1;
    orc_ec_log[3 * orc_ec_log_n + 2] = 0;
    orc_ec_log_n++;
  }
  orc_ecw_bool(w, bit == 1, 16384);
}
void orc_ecw_literal(orc_ecw *w, int bits, uint32_t s) {
  for (int b = bits - 1; b >= 0; b--) orc_ecw_bit(w, (int)(1 & (s >> b)));
}
void orc_ecw_golomb(orc_ecw *w, uint16_t level) {
  const uint16_t x = (uint16_t)(level + 1);
  uint16_t i = x;
  int length = 0;
  while (i != 0) {
    i >>= 1;
    length++;
  }
  for (int k = 0; k < length - 1; k++) orc_ecw_bit(w, 0);
  for (int k = length - 1; k >= 0; k--) orc_ecw_bit(w, (x >> k) & 1);
}

/* WriterBase<WriterEncoder>::done (src/ec.rs:444-486), in two parts: the
 * flush into the pre-carry buffer (returns the byte count) and the carry
 * propagation into bytes. */
size_t orc_ecw_finish(orc_ecw *w) {
  const uint32_t l = w->low;
  int16_t c = w->cnt;
  int16_t s = 10;
  const uint32_t m = 0x3FFF;
  uint32_t e = ((l + m) & ~m) | (m + 1);
  s = (int16_t)(s + c);
  if (s > 0) {
    uint32_t n = (1u << (c + 16)) - 1;
    for (;;) {
      push_pre(w, (uint16_t)(e >> (c + 16)));
      e &= n;
      s = (int16_t)(s - 8);
      c = (int16_t)(c - 8);
      n >>= 8;
      if (s <= 0) break;
    }
  }
  return w->n;
}

void orc_ecw_bytes(const orc_ecw *w, uint8_t *out) {
  size_t offs = w->n;
  uint16_t cc = 0;
  while (offs > 0) {
    offs--;
    cc = (uint16_t)(cc + w->pre[offs]);
    out[offs] = (uint8_t)cc;
    cc >>= 8;
  }
}

size_t orc_ecw_done(orc_ecw *w, uint8_t *out, size_t cap) {
  const size_t n = orc_ecw_finish(w);
  if (out && n <= cap) orc_ecw_bytes(w, out);
  return n;
}

/* ------------------------------------------------------------ reader */
/* The Reader of ec.rs's test module (src/ec.rs:914-1010). */
#define WINDOW_SIZE 32
#define LOTS_OF_BITS 0x4000

static void ecr_refill(orc_ecr *r) {
  int s = WINDOW_SIZE - 9 - (r->cnt + 15);
  while (s >= 0 && r->bptr < r->len) {
    r->dif ^= (uint32_t)r->buf[r->bptr] << s;
    r->cnt = (int16_t)(r->cnt + 8);
    s -= 8;
    r->bptr++;
  }
  if (r->bptr >= r->len) r->cnt = LOTS_OF_BITS;
}

void orc_ecr_init(orc_ecr *r, const uint8_t *buf, size_t len) {
  r->buf = buf;
  r->len = len;
  r->bptr = 0;
  r->dif = (1u << (WINDOW_SIZE - 1)) - 1;
  r->rng = 0x8000;
  r->cnt = -15;
  ecr_refill(r);
}

static void ecr_normalize(orc_ecr *r, uint32_t dif, uint32_t rng) {
  const int d = __builtin_clz(rng) - 16;
  r->cnt = (int16_t)(r->cnt - d);
  r->dif = ((dif + 1) << d) - 1;
  r->rng = (uint16_t)(rng << d);
  if (r->cnt < 0) ecr_refill(r);
}

int orc_ecr_bool(orc_ecr *r, uint32_t f) {
  const uint32_t rr = r->rng;
  const uint32_t v = (((rr >> 8) * (f >> EC_PROB_SHIFT)) >> (7 - EC_PROB_SHIFT)) + EC_MIN_PROB;
  const uint32_t vw = v << (WINDOW_SIZE - 16);
  if (r->dif >= vw) {
    ecr_normalize(r, r->dif - vw, rr - v);
    return 0;
  }
  ecr_normalize(r, r->dif, v);
  return 1;
}

/* Reader::symbol: icdf holds n entries (the last 0) */
int orc_ecr_symbol(orc_ecr *r, const uint16_t *icdf, int n_entries) {
  const uint32_t rr = r->rng;
  const uint32_t n = (uint32_t)n_entries - 1;
  const uint32_t c = r->dif >> (WINDOW_SIZE - 16);
  uint32_t u, v = r->rng;
  int ret = 0;
  u = v;
  v = ((rr >> 8) * ((uint32_t)icdf[ret] >> EC_PROB_SHIFT)) >> (7 - EC_PROB_SHIFT);
  v += EC_MIN_PROB * (n - (uint32_t)ret);
  while (c < v) {
    u = v;
    ret++;
    v = ((rr >> 8) * ((uint32_t)icdf[ret] >> EC_PROB_SHIFT)) >> (7 - EC_PROB_SHIFT);
    v += EC_MIN_PROB * (n - (uint32_t)ret);
  }
  ecr_normalize(r, r->dif - (v << (WINDOW_SIZE - 16)), u - v);
  return ret;
}

/* ------------------------------------------------- coefficient contexts */
#define TX_PAD_HOR 4
#define TX_PAD_TOP 2
#define TX_PAD_2D ((64 + TX_PAD_HOR) * (64 + 6) + 16)
#define COEFF_CONTEXT_BITS 6
#define COEFF_CONTEXT_MASK 63
#define NUM_BASE_LEVELS 2
#define COEFF_BASE_RANGE 12
#define BR_CDF_SIZE 4

void orc_ec_ctx_init(orc_ec_ctx *c, int qctx) {
  memcpy(c->cdf, ORC_EC_DEFAULT_CDF[qctx], sizeof(c->cdf));
  memset(c->above, 0, sizeof(c->above));
  memset(c->left, 0, sizeof(c->left));
}

/* CDFContext::reset_counts (src/context.rs:851-): every adaptation counter 0 */
void orc_ec_reset_counts(uint16_t *cdf) {
  static const int fam[][3] = {  /* offset, count, entries */
      {ORC_EC_TXB_SKIP, 65, 3},   {ORC_EC_EOB16, 4, 6},      {ORC_EC_EOB32, 4, 7},
      {ORC_EC_EOB64, 4, 8},       {ORC_EC_EOB128, 4, 9},     {ORC_EC_EOB256, 4, 10},
      {ORC_EC_EOB512, 4, 11},     {ORC_EC_EOB1024, 4, 12},   {ORC_EC_EOB_EXTRA, 90, 3},
      {ORC_EC_BASE_EOB, 40, 4},   {ORC_EC_BASE, 420, 5},     {ORC_EC_BR, 210, 5},
      {ORC_EC_DC_SIGN, 6, 3},     {ORC_EC_INTER_TX, 16, 17}};
  for (size_t f = 0; f < sizeof(fam) / sizeof(fam[0]); f++)
    for (int i = 0; i < fam[f][1]; i++) cdf[fam[f][0] + i * fam[f][2] + fam[f][2] - 1] = 0;
}

static int txs_ctx_of(int tx) { return tx; } /* (sqr + sqr_up + 1) >> 1, square sizes */

/* get_txb_ctx (src/context.rs:1776-1868); plane_lg = log2 pixels of the
 * plane block (num_pels_log2_lookup), tx square log2 width = tx + 2 */
static void get_txb_ctx(const orc_ec_ctx *c, int plane, int plane_lg, int tx, int bx, int by,
                        int xdec, int ydec, int *skip_ctx, int *dc_ctx) {
  static const int8_t signs[3] = {0, -1, 1};
  const int n4 = 1 << tx;  /* width_mi = height_mi */
  const uint8_t *ab = c->above[plane] + (bx >> xdec);
  const uint8_t *lf = c->left[plane] + ((by & 15) >> ydec);
  int dc_sign = 0;
  for (int i = 0; i < n4; i++) dc_sign += signs[ab[i] >> COEFF_CONTEXT_BITS];
  for (int i = 0; i < n4; i++) dc_sign += signs[lf[i] >> COEFF_CONTEXT_BITS];
  /* dc_sign_contexts: 1 below 0, 0 at 0, 2 above (src/context.rs:1782-1786) */
  *dc_ctx = dc_sign < 0 ? 1 : dc_sign > 0 ? 2 : 0;
  const int tx_lg = 2 * (tx + 2);
  if (plane == 0) {
    if (plane_lg == tx_lg) {
      *skip_ctx = 0;
    } else {
      static const uint8_t skip_contexts[5][5] = {
          {1, 2, 2, 2, 3}, {1, 4, 4, 4, 5}, {1, 4, 4, 4, 5}, {1, 4, 4, 4, 5}, {1, 4, 4, 4, 6}};
      uint8_t top = 0, left = 0;
      for (int i = 0; i < n4; i++) top |= ab[i];
      for (int i = 0; i < n4; i++) left |= lf[i];
      top &= COEFF_CONTEXT_MASK;
      left &= COEFF_CONTEXT_MASK;
      int mx = top | left;
      mx = mx < 4 ? mx : 4;
      int mn = top < left ? top : left;
      mn = mn < 4 ? mn : 4;
      *skip_ctx = skip_contexts[mn][mx];
    }
  } else {
    uint8_t top = 0, left = 0;
    for (int i = 0; i < n4; i++) top |= ab[i];
    for (int i = 0; i < n4; i++) left |= lf[i];
    *skip_ctx = (top != 0) + (left != 0) + (plane_lg > tx_lg ? 10 : 7);
  }
}

static void set_coeff_context(orc_ec_ctx *c, int plane, int tx, int bx, int by, int xdec,
                              int ydec, uint8_t v) {
  const int n4 = 1 << tx;
  for (int i = 0; i < n4; i++) c->above[plane][(bx >> xdec) + i] = v;
  for (int i = 0; i < n4; i++) c->left[plane][((by & 15) >> ydec) + i] = v;
}

/* reset_skip_context (src/context.rs:1651-1679) for a block of log2 size
 * bw_lg x bh_lg pixels (bsize >= 8x8: all three planes) */
void orc_ec_reset_skip(orc_ec_ctx *c, int bx, int by, int bw_lg, int bh_lg, int xdec, int ydec) {
  for (int p = 0; p < 3; p++) {
    const int xd = p ? xdec : 0, yd = p ? ydec : 0;
    const int bw = 1 << (bw_lg - xd - 2), bh = 1 << (bh_lg - yd - 2);
    for (int i = 0; i < bw; i++) c->above[p][(bx >> xd) + i] = 0;
    for (int i = 0; i < bh; i++) c->left[p][((by & 15) >> yd) + i] = 0;
  }
}

void orc_ec_reset_left(orc_ec_ctx *c) { memset(c->left, 0, sizeof(c->left)); }

static uint8_t clip_max3(uint8_t x) { return x > 3 ? 3 : x; }

/* get_nz_map_ctx (TX_CLASS_2D, src/context.rs:3791-3878) */
static int nz_map_ctx(const uint8_t *levels, int pos, int bwl, int height, int scan_idx,
                      int is_eob, int tx) {
  if (is_eob) {
    if (scan_idx == 0) return 0;
    if (scan_idx <= (height << bwl) / 8) return 1;
    if (scan_idx <= (height << bwl) / 4) return 2;
    return 3;
  }
  const uint8_t *l = levels + pos + ((pos >> bwl) << 2);
  int mag = clip_max3(l[1]) + clip_max3(l[(1 << bwl) + TX_PAD_HOR]);
  mag += clip_max3(l[(1 << bwl) + TX_PAD_HOR + 1]) + clip_max3(l[2]);
  mag += clip_max3(l[(2 << bwl) + (2 << 2)]);
  if (pos == 0) return 0;  /* (tx_class | coeff_idx) == 0 */
  const int row = pos >> bwl, col = pos - (row << bwl);
  int ctx = (mag + 1) >> 1;
  ctx = ctx < 4 ? ctx : 4;
  return ctx + ORC_av1_nz_map_ctx_offset[tx * 25 + (row < 4 ? row : 4) * 5 + (col < 4 ? col : 4)];
}

/* get_br_ctx (TX_CLASS_2D, src/context.rs:3901-3948) */
static int br_ctx(const uint8_t *levels, int c, int bwl) {
  const int row = c >> bwl, col = c - (row << bwl);
  const int stride = (1 << bwl) + TX_PAD_HOR;
  const int pos = row * stride + col;
  int mag = levels[pos + 1] + levels[pos + stride] + levels[pos + stride + 1];
  mag = (mag + 1) >> 1;
  mag = mag < 6 ? mag : 6;
  if (c == 0) return mag;
  if (row < 2 && col < 2) return mag + 7;
  return mag + 14;
}

/* get_eob_pos_token (src/context.rs:3778-3789) */
static int eob_pos_token(int eob, uint32_t *extra) {
  int t;
  if (eob < 33) {
    t = ORC_eob_to_pos_small[eob];
  } else {
    int e = (eob - 1) >> 5;
    e = e < 16 ? e : 16;
    t = ORC_eob_to_pos_large[e];
  }
  *extra = (uint32_t)(eob - ORC_k_eob_group_start[t]);
  return t;
}

/* ContextWriter::write_coeffs_lv_map (src/context.rs:3965-4220) for a square
 * transform (tx 0..4 = TX_4X4 .. TX_64X64, 2-D class) at TileBlockOffset
 * (bx, by).  coeffs_in: the quantised coefficients, raster of the coded size.
 * Returns has_coeff; *cul_out gets the context value it stores. */
int orc_ec_write_coeffs(orc_ecw *w, orc_ec_ctx *cx, int plane, int bx, int by,
                        const int32_t *coeffs_in, int is_inter, int tx, int tx_type,
                        int plane_lg, int xdec, int ydec, int reduced, uint8_t *cul_out) {
  /* the transform-type sets restated: every square inter size below 64 in
   * the reduced set (speed >= 5, src/api/config.rs:370-372) is
   * TX_SET_DCT_IDTX; intra at 32 and 64 is TX_SET_DCTONLY (no symbol).
   * Other sets are not restated. */
  if (tx < 4 && (is_inter ? !reduced && tx < 3 : tx < 3)) return -1;
  const uint16_t *scan = ORC_SCANS + ORC_SCAN_OFF[tx * 16 + tx_type];
  const int cw = tx == 4 ? 32 : 4 << tx;  /* av1_get_coded_tx_size */
  const int area = cw * cw;
  int32_t coeffs[1024];
  uint32_t cul = 0;
  for (int i = 0; i < area; i++) {
    coeffs[i] = coeffs_in[scan[i]];
    cul += (uint32_t)(coeffs[i] < 0 ? -(int64_t)coeffs[i] : coeffs[i]);
  }
  int eob = 0;
  if (cul != 0)
    for (int i = area - 1; i >= 0; i--)
      if (coeffs[i] != 0) {
        eob = i + 1;
        break;
      }
  const int txs = txs_ctx_of(tx);
  int skip_ctx, dc_ctx;
  get_txb_ctx(cx, plane, plane_lg, tx, bx, by, xdec, ydec, &skip_ctx, &dc_ctx);
  orc_ecw_symbol_update(w, eob == 0, cx->cdf + ORC_EC_TXB_SKIP + (txs * 13 + skip_ctx) * 3, 3);
  if (eob == 0) {
    set_coeff_context(cx, plane, tx, bx, by, xdec, ydec, 0);
    if (cul_out) *cul_out = 0;
    return 0;
  }
  uint8_t levels_buf[TX_PAD_2D];
  memset(levels_buf, 0, sizeof(levels_buf));
  {  /* txb_init_levels */
    int off = TX_PAD_TOP * (cw + TX_PAD_HOR);
    for (int y = 0; y < cw; y++) {
      for (int x = 0; x < cw; x++) {
        int32_t a = coeffs_in[y * cw + x];
        int64_t v = a < 0 ? -(int64_t)a : a;
        levels_buf[off + x] = (uint8_t)(v > 127 ? 127 : v);
      }
      off += cw + TX_PAD_HOR;
    }
  }
  const int ptype = plane ? 1 : 0;
  if (plane == 0 && tx < 4 && is_inter) {
    /* write_tx_type: get_tx_set -> TX_SET_DCT_IDTX for every inter square
     * size below 64 (reduced, or sqr_up 32x32); inter_tx_cdf[set index][sqr][..=2] */
    const int set = 1;
    const int ntx = ORC_num_tx_set[set];
    const int idx = ORC_tx_set_index_inter[set];
    orc_ecw_symbol_update(w, ORC_av1_tx_ind[set * 16 + tx_type],
                          cx->cdf + ORC_EC_INTER_TX + (idx * 4 + tx) * 17, ntx + 1);
  }
  uint32_t eob_extra = 0;
  const int eob_pt = eob_pos_token(eob, &eob_extra);
  const int area_lg = 2 * (tx + 2);
  const int ems = area_lg - 4;
  static const int eob_off[7] = {ORC_EC_EOB16, ORC_EC_EOB32, ORC_EC_EOB64, ORC_EC_EOB128,
                                 ORC_EC_EOB256, ORC_EC_EOB512, ORC_EC_EOB1024};
  const int em = ems < 6 ? ems : 6;
  const int elen = 6 + em;
  orc_ecw_symbol_update(w, (uint32_t)(eob_pt - 1), cx->cdf + eob_off[em] + (ptype * 2 + 0) * elen,
                        elen);
  const int eob_bits = ORC_k_eob_offset_bits[eob_pt];
  if (eob_bits > 0) {
    int sh = eob_bits - 1;
    uint32_t bit = (eob_extra & (1u << sh)) ? 1 : 0;
    orc_ecw_symbol_update(w, bit,
                          cx->cdf + ORC_EC_EOB_EXTRA + ((txs * 2 + ptype) * 9 + (eob_pt - 3)) * 3,
                          3);
    for (int i = 1; i < eob_bits; i++) {
      sh = eob_bits - 1 - i;
      orc_ecw_bit(w, (eob_extra & (1u << sh)) ? 1 : 0);
    }
  }
  const uint8_t *levels = levels_buf + TX_PAD_TOP * (cw + TX_PAD_HOR);
  const int bwl = tx == 4 ? 5 : tx + 2;
  int8_t coeff_ctx[1024];
  for (int i = 0; i < eob; i++)
    coeff_ctx[scan[i]] = (int8_t)nz_map_ctx(levels, scan[i], bwl, cw, i, i == eob - 1, tx);
  for (int c = eob - 1; c >= 0; c--) {
    const int pos = scan[c];
    const int ctx = coeff_ctx[pos];
    const int32_t v = coeffs_in[pos];
    const uint32_t level = (uint32_t)(v < 0 ? -(int64_t)v : v);
    if (c == eob - 1) {
      orc_ecw_symbol_update(w, (level < 3 ? level : 3) - 1,
                            cx->cdf + ORC_EC_BASE_EOB + ((txs * 2 + ptype) * 4 + ctx) * 4, 4);
    } else {
      orc_ecw_symbol_update(w, level < 3 ? level : 3,
                            cx->cdf + ORC_EC_BASE + ((txs * 2 + ptype) * 42 + ctx) * 5, 5);
    }
    if (level > NUM_BASE_LEVELS) {
      const uint16_t l16 = (uint16_t)level;
      const uint16_t base_range = (uint16_t)(l16 - 1 - NUM_BASE_LEVELS);
      const int bctx = br_ctx(levels, pos, bwl);
      const int btx = txs < 3 ? txs : 3;
      for (int idx = 0; idx < COEFF_BASE_RANGE; idx += BR_CDF_SIZE - 1) {
        int k = base_range - idx;
        k = k < BR_CDF_SIZE - 1 ? k : BR_CDF_SIZE - 1;
        orc_ecw_symbol_update(w, (uint32_t)k,
                              cx->cdf + ORC_EC_BR + ((btx * 2 + ptype) * 21 + bctx) * 5, 5);
        if (k < BR_CDF_SIZE - 1) break;
      }
    }
  }
  for (int c = 0; c < eob; c++) {
    const int32_t v = coeffs_in[scan[c]];
    const uint32_t level = (uint32_t)(v < 0 ? -(int64_t)v : v);
    if (level == 0) continue;
    const int sign = v < 0;
    if (c == 0)
      orc_ecw_symbol_update(w, (uint32_t)sign, cx->cdf + ORC_EC_DC_SIGN + (ptype * 3 + dc_ctx) * 3,
                            3);
    else
      orc_ecw_bit(w, sign);
    if (level > COEFF_BASE_RANGE + NUM_BASE_LEVELS)
      orc_ecw_golomb(w, (uint16_t)(level - COEFF_BASE_RANGE - 1 - NUM_BASE_LEVELS));
  }
  cul = cul < COEFF_CONTEXT_MASK ? cul : COEFF_CONTEXT_MASK;
  if (coeffs[0] < 0)
    cul |= 1u << COEFF_CONTEXT_BITS;
  else if (coeffs[0] > 0)
    cul += 2u << COEFF_CONTEXT_BITS;
  set_coeff_context(cx, plane, tx, bx, by, xdec, ydec, (uint8_t)cul);
  if (cul_out) *cul_out = (uint8_t)cul;
  return 1;
}

/* A job sequence (the shape the reference vectors and the replay's tiles
 * take): kind 0 = write_coeffs_lv_map of one transform block, 1 =
 * reset_skip_context of a skip leaf, 2 = reset_left_contexts (a superblock
 * row starts), 3 = a new tile (fresh BlockContext + the initial CDFs).
 * Bytes of every tile go to out back to back; tile_bytes[t] their counts;
 * ret[j] = (has_coeff | cul << 1) of each tx job.  Returns total bytes, or
 * -1 if cap is exceeded.  The final CDFs of the last tile go to cdf_out. */
long orc_ec_code_jobs(const orc_ec_job *jobs, int n, const int32_t *coeffs, const uint16_t *cdf_init,
                      int xdec, int ydec, uint8_t *out, long cap, int32_t *tile_bytes,
                      uint16_t *ret, uint16_t *cdf_out) {
  orc_ec_ctx *cx = (orc_ec_ctx *)malloc(sizeof(orc_ec_ctx));
  orc_ecw w;
  orc_ecw_init(&w);
  memcpy(cx->cdf, cdf_init, sizeof(cx->cdf));
  memset(cx->above, 0, sizeof(cx->above));
  memset(cx->left, 0, sizeof(cx->left));
  long total = 0;
  int tile = 0, open = 0;
  for (int j = 0; j <= n; j++) {
    if (j == n || jobs[j].kind == 3) {
      if (open || j == n) {
        const size_t nb = orc_ecw_finish(&w);
        if (total + (long)nb > cap) {
          total = -1;
          break;
        }
        orc_ecw_bytes(&w, out + total);
        if (tile_bytes) tile_bytes[tile] = (int32_t)nb;
        total += (long)nb;
        tile++;
      }
      if (j == n) break;
      orc_ecw_free(&w);
      orc_ecw_init(&w);
      memcpy(cx->cdf, cdf_init, sizeof(cx->cdf));
      memset(cx->above, 0, sizeof(cx->above));
      memset(cx->left, 0, sizeof(cx->left));
      open = 1;
      if (ret) ret[j] = 0;
      continue;
    }
    open = 1;
    const orc_ec_job *jb = jobs + j;
    uint16_t r = 0;
    if (jb->kind == 0) {
      uint8_t cul = 0;
      const int has = orc_ec_write_coeffs(&w, cx, jb->plane, jb->bx, jb->by, coeffs + jb->coeff_off,
                                          jb->is_inter, jb->tx_size, jb->tx_type,
                                          jb->bw_lg + jb->bh_lg, jb->plane ? xdec : 0,
                                          jb->plane ? ydec : 0, 1, &cul);
      if (has < 0) {
        total = -2;
        break;
      }
      r = (uint16_t)(has | cul << 1);
    } else if (jb->kind == 1) {
      orc_ec_reset_skip(cx, jb->bx, jb->by, jb->bw_lg, jb->bh_lg, xdec, ydec);
    } else if (jb->kind == 2) {
      orc_ec_reset_left(cx);
    }
    if (ret) ret[j] = r;
  }
  if (cdf_out && total >= 0) memcpy(cdf_out, cx->cdf, sizeof(cx->cdf));
  orc_ecw_free(&w);
  free(cx);
  return total;
}

const uint16_t *orc_ec_default_cdf(int qctx) { return ORC_EC_DEFAULT_CDF[qctx]; }
