/* Inverse transform restatement (test infrastructure only).
 *
 * The reference's 1-D inverse kernels (src/transform/inverse.rs:35-1544,
 * av1_idct4..64 / av1_iadst4..16 / av1_iidentity4..32) are the AV1
 * normative inverse transforms written out stage by stage.  They are
 * restated here as the AV1 specification's generic butterfly programs
 * (section 7.13.2: B = rotation with Round2(.,12), H = add/sub), with the
 * reference's one deviation from the spec made explicit: every add/sub
 * result is clamped to `range` bits (clamp_value, src/transform/mod.rs:490).
 * Bit-exactness against the reference's own kernels is checked on golden
 * vectors produced from the reference source (tools/refeval).
 *
 * 2-D driver: NativeInvTxfm2D::inv_txfm2d / inv_txfm2d_add
 * (inverse.rs:1939-2114).
 */
#include <string.h>

#include "orc_common.h"

typedef int32_t T;

/* COSPI_INV, inverse.rs:22-29 (= round(4096 * cos(k*pi/128)), k = 0..63) */
static const int32_t COSPI[64] = {
    4096, 4095, 4091, 4085, 4076, 4065, 4052, 4036, 4017, 3996, 3973,
    3948, 3920, 3889, 3857, 3822, 3784, 3745, 3703, 3659, 3612, 3564,
    3513, 3461, 3406, 3349, 3290, 3229, 3166, 3102, 3035, 2967, 2896,
    2824, 2751, 2675, 2598, 2520, 2440, 2359, 2276, 2191, 2106, 2019,
    1931, 1842, 1751, 1660, 1567, 1474, 1380, 1285, 1189, 1092, 995,
    897,  799,  700,  601,  501,  401,  301,  201,  101};
/* SINPI_INV, inverse.rs:31 */
static const int32_t SINPI[5] = {0, 1321, 2482, 3344, 3803};

/* cos128 / sin128 of the spec: COSPI extended with cos(pi/2) = 0 at 64 */
static inline int32_t cospi_ext(int k) { return k == 64 ? 0 : COSPI[k]; }
static int32_t cos128(int angle) {
  int a = angle & 255;
  if (a <= 64) return cospi_ext(a);
  if (a <= 128) return -cospi_ext(128 - a);
  if (a <= 192) return -cospi_ext(a - 128);
  return cospi_ext(256 - a);
}
static int32_t sin128(int angle) { return cos128(angle - 64); }

static inline T clampv(T v, int bit) {
  int64_t hi = ((int64_t)1 << (bit - 1)) - 1, lo = -((int64_t)1 << (bit - 1));
  return v < lo ? (T)lo : (v > hi ? (T)hi : v);
}

/* half_btf, src/transform/mod.rs:476-488 */
static inline T half_btf(T w0, T in0, T w1, T in1) {
  T r = w_add(w_mul(w0, in0), w_mul(w1, in1));
  return asr(w_add(r, 1 << 11), 12);
}

/* B(a, b, angle, flip) */
static void B(T *t, int a, int b, int angle, int flip) {
  T c = cos128(angle), s = sin128(angle);
  T x = half_btf(c, t[a], -s, t[b]);
  T y = half_btf(s, t[a], c, t[b]);
  if (flip) {
    t[a] = y;
    t[b] = x;
  } else {
    t[a] = x;
    t[b] = y;
  }
}
/* H(a, b, flip) with the reference's clamp on both outputs */
static void H(T *t, int a, int b, int flip, int r) {
  if (flip) {
    int tmp = a;
    a = b;
    b = tmp;
  }
  T x = t[a], y = t[b];
  t[a] = clampv(w_add(x, y), r);
  t[b] = clampv(w_sub(x, y), r);
}

static inline int brev(int bits, int x) {
  int v = 0;
  for (int i = 0; i < bits; i++) v |= ((x >> i) & 1) << (bits - 1 - i);
  return v;
}

/* Inverse DCT process (AV1 spec 7.13.2.3) for n = log2(size) in 2..6. */
static void idct(T *t, int n, int r) {
  T c[64];
  int n0 = 1 << n;
  memcpy(c, t, (size_t)n0 * sizeof(T));
  for (int i = 0; i < n0; i++) t[i] = c[brev(n, i)];
  if (n == 6)
    for (int i = 0; i < 16; i++) B(t, 32 + i, 63 - i, 63 - 4 * brev(4, i), 0);
  if (n >= 5)
    for (int i = 0; i < 8; i++) B(t, 16 + i, 31 - i, 6 + (brev(3, 7 - i) << 3), 0);
  if (n == 6)
    for (int i = 0; i < 16; i++) H(t, 32 + i * 2, 33 + i * 2, i & 1, r);
  if (n >= 4)
    for (int i = 0; i < 4; i++) B(t, 8 + i, 15 - i, 12 + (brev(2, 3 - i) << 4), 0);
  if (n >= 5)
    for (int i = 0; i < 8; i++) H(t, 16 + 2 * i, 17 + 2 * i, i & 1, r);
  if (n == 6)
    for (int i = 0; i < 4; i++)
      for (int j = 0; j < 2; j++)
        B(t, 62 - i * 4 - j, 33 + i * 4 + j, 60 - 16 * brev(2, i) + 64 * j, 1);
  if (n >= 3)
    for (int i = 0; i < 2; i++) B(t, 4 + i, 7 - i, 56 - 32 * i, 0);
  if (n >= 4)
    for (int i = 0; i < 4; i++) H(t, 8 + 2 * i, 9 + 2 * i, i & 1, r);
  if (n >= 5)
    for (int i = 0; i < 2; i++)
      for (int j = 0; j < 2; j++)
        B(t, 30 - 4 * i - j, 17 + 4 * i + j, 24 + (j << 6) + ((1 - i) << 5), 1);
  if (n == 6)
    for (int i = 0; i < 8; i++)
      for (int j = 0; j < 2; j++) H(t, 32 + i * 4 + j, 35 + i * 4 - j, i & 1, r);
  for (int i = 0; i < 2; i++) B(t, 2 * i, 2 * i + 1, 32 + 16 * i, 1 - i);
  if (n >= 3)
    for (int i = 0; i < 2; i++) H(t, 4 + 2 * i, 5 + 2 * i, i, r);
  if (n >= 4)
    for (int i = 0; i < 2; i++) B(t, 14 - i, 9 + i, 48 + 64 * i, 1);
  if (n >= 5)
    for (int i = 0; i < 4; i++)
      for (int j = 0; j < 2; j++) H(t, 16 + 4 * i + j, 19 + 4 * i - j, i & 1, r);
  if (n == 6)
    for (int i = 0; i < 2; i++)
      for (int j = 0; j < 4; j++)
        B(t, 61 - i * 8 - j, 34 + i * 8 + j, 56 - i * 32 + (j >> 1) * 64, 1);
  for (int i = 0; i < 2; i++) H(t, i, 3 - i, 0, r);
  if (n >= 3) B(t, 6, 5, 32, 1);
  if (n >= 4)
    for (int i = 0; i < 2; i++)
      for (int j = 0; j < 2; j++) H(t, 8 + 4 * i + j, 11 + 4 * i - j, i, r);
  if (n >= 5)
    for (int i = 0; i < 4; i++) B(t, 29 - i, 18 + i, 48 + (i >> 1) * 64, 1);
  if (n == 6)
    for (int i = 0; i < 4; i++)
      for (int j = 0; j < 4; j++) H(t, 32 + 8 * i + j, 39 + 8 * i - j, i & 1, r);
  if (n >= 3)
    for (int i = 0; i < 4; i++) H(t, i, 7 - i, 0, r);
  if (n >= 4)
    for (int i = 0; i < 2; i++) B(t, 13 - i, 10 + i, 32, 1);
  if (n >= 5)
    for (int i = 0; i < 2; i++)
      for (int j = 0; j < 4; j++) H(t, 16 + i * 8 + j, 23 + i * 8 - j, i, r);
  if (n == 6)
    for (int i = 0; i < 8; i++) B(t, 59 - i, 36 + i, i < 4 ? 48 : 112, 1);
  if (n >= 4)
    for (int i = 0; i < 8; i++) H(t, i, 15 - i, 0, r);
  if (n >= 5)
    for (int i = 0; i < 4; i++) B(t, 27 - i, 20 + i, 32, 1);
  if (n == 6) {
    for (int i = 0; i < 8; i++) H(t, 32 + i, 47 - i, 0, r);
    for (int i = 0; i < 8; i++) H(t, 48 + i, 63 - i, 1, r);
  }
  if (n >= 5)
    for (int i = 0; i < 16; i++) H(t, i, 31 - i, 0, r);
  if (n == 6)
    for (int i = 0; i < 8; i++) B(t, 55 - i, 40 + i, 32, 1);
  if (n == 6)
    for (int i = 0; i < 32; i++) H(t, i, 63 - i, 0, r);
}

/* Inverse ADST4 (av1_iadst4, inverse.rs:63-109): no clamps, range unused */
static void iadst4(T *t) {
  T x0 = t[0], x1 = t[1], x2 = t[2], x3 = t[3];
  T s0 = w_mul(SINPI[1], x0), s1 = w_mul(SINPI[2], x0);
  T s2 = w_mul(SINPI[3], x1), s3 = w_mul(SINPI[4], x2);
  T s4 = w_mul(SINPI[1], x2), s5 = w_mul(SINPI[2], x3);
  T s6 = w_mul(SINPI[4], x3);
  T s7 = w_add(w_sub(x0, x2), x3);
  s0 = w_add(s0, s3);
  s1 = w_sub(s1, s4);
  s3 = s2;
  s2 = w_mul(SINPI[3], s7);
  s0 = w_add(s0, s5);
  s1 = w_sub(s1, s6);
  T y0 = w_add(s0, s3), y1 = w_add(s1, s3), y2 = s2;
  T y3 = w_sub(w_add(s0, s1), s3);
  t[0] = round_shift(y0, 12);
  t[1] = round_shift(y1, 12);
  t[2] = round_shift(y2, 12);
  t[3] = round_shift(y3, 12);
}

/* ADST input / output permutations (spec 7.13.2.7 / 7.13.2.8) */
static void adst_in_perm(T *t, int n) {
  T c[16];
  int n0 = 1 << n;
  memcpy(c, t, (size_t)n0 * sizeof(T));
  for (int i = 0; i < n0; i++) t[i] = c[(i & 1) ? (i - 1) : (n0 - i - 1)];
}
static void adst_out_perm(T *t, int n) {
  T c[16];
  int n0 = 1 << n;
  memcpy(c, t, (size_t)n0 * sizeof(T));
  for (int i = 0; i < n0; i++) {
    int a = (i >> 3) & 1;
    int b = ((i >> 2) & 1) ^ ((i >> 3) & 1);
    int cc = ((i >> 1) & 1) ^ ((i >> 2) & 1);
    int d = (i & 1) ^ ((i >> 1) & 1);
    int idx = ((d << 3) | (cc << 2) | (b << 1) | a) >> (4 - n);
    t[i] = (i & 1) ? w_sub(0, c[idx]) : c[idx];
  }
}

/* Inverse ADST8 (av1_iadst8, inverse.rs:173-252) */
static void iadst8(T *t, int r) {
  adst_in_perm(t, 3);
  for (int i = 0; i < 4; i++) B(t, 2 * i, 1 + 2 * i, 60 - 16 * i, 1);
  for (int i = 0; i < 4; i++) H(t, i, 4 + i, 0, r);
  for (int i = 0; i < 2; i++) B(t, 4 + 3 * i, 5 + i, 48 - 32 * i, 1);
  for (int i = 0; i < 2; i++)
    for (int j = 0; j < 2; j++) H(t, 4 * j + i, 2 + 4 * j + i, 0, r);
  for (int i = 0; i < 2; i++) B(t, 2 + 4 * i, 3 + 4 * i, 32, 1);
  adst_out_perm(t, 3);
}

/* Inverse ADST16 (av1_iadst16, inverse.rs:364-532) */
static void iadst16(T *t, int r) {
  adst_in_perm(t, 4);
  for (int i = 0; i < 8; i++) B(t, 2 * i, 1 + 2 * i, 62 - 8 * i, 1);
  for (int i = 0; i < 8; i++) H(t, i, 8 + i, 0, r);
  for (int i = 0; i < 2; i++) {
    B(t, 8 + 2 * i, 9 + 2 * i, 56 - 32 * i, 1);
    B(t, 13 + 2 * i, 12 + 2 * i, 8 + 32 * i, 1);
  }
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 2; j++) H(t, 8 * j + i, 4 + 8 * j + i, 0, r);
  for (int i = 0; i < 2; i++)
    for (int j = 0; j < 2; j++) B(t, 4 + 8 * j + 3 * i, 5 + 8 * j + i, 48 - 32 * i, 1);
  for (int i = 0; i < 2; i++)
    for (int j = 0; j < 4; j++) H(t, 4 * j + i, 2 + 4 * j + i, 0, r);
  for (int i = 0; i < 4; i++) B(t, 2 + 4 * i, 3 + 4 * i, 32, 1);
  adst_out_perm(t, 4);
}

/* txfm_types::Detail::inverse + INV_TXFM_FNS (inverse.rs:1580-1623). */
int orc_inv_txfm1d(int kind, int n, const int32_t *in, int32_t *out,
                   int range) {
  int lg = n == 4 ? 2 : n == 8 ? 3 : n == 16 ? 4 : n == 32 ? 5 : n == 64 ? 6 : 0;
  if (!lg) return -1;
  T t[64];
  memcpy(t, in, (size_t)n * sizeof(T));
  switch (kind) {
  case 0: /* av1_iidentity4/8/16/32 (inverse.rs:111, 254, 534, 841) */
    if (n == 64) return -1;
    for (int i = 0; i < n; i++) {
      if (n == 4) out[i] = round_shift(w_mul(5793, t[i]), 12);
      else if (n == 8) out[i] = w_mul(2, t[i]);
      else if (n == 16) out[i] = round_shift(w_mul(5793 * 2, t[i]), 12);
      else out[i] = w_mul(4, t[i]);
    }
    return 0;
  case 1:
    idct(t, lg, range);
    break;
  case 2:
  case 3:
    if (n == 4) iadst4(t);
    else if (n == 8) iadst8(t, range);
    else if (n == 16) iadst16(t, range);
    else return -1;
    if (kind == 3) { /* av1_iflipadst*: reversed output */
      for (int i = 0; i < n / 2; i++) {
        T x = t[i];
        t[i] = t[n - 1 - i];
        t[n - 1 - i] = x;
      }
    }
    break;
  default:
    return -1;
  }
  memcpy(out, t, (size_t)n * sizeof(T));
  return 0;
}

/* InvBlock::INTERMEDIATE_SHIFT (inverse.rs:1643-1666), by TxSize. */
static const uint8_t INV_SHIFT[19] = {0, 1, 2, 2, 2, 0, 0, 1, 1, 1,
                                      1, 1, 1, 1, 1, 2, 2, 2, 2};

/* NativeInvTxfm2D::inv_txfm2d_add (inverse.rs:1939-2114).  The native 2-D
 * path only supports the (kind, size) pairs its txfm_types table
 * implements (no FlipAdst, no Adst32/64, no Id64): others return -1. */
int orc_inv_txfm2d_add(const int32_t *coeffs, void *dst, ptrdiff_t dst_stride,
                       int tx_size, int tx_type, int bit_depth, int hbd) {
  if (tx_size < 0 || tx_size > 18 || tx_type < 0 || tx_type > 15) return -1;
  int w = 1 << ORC_TX_W_LOG2[tx_size], h = 1 << ORC_TX_H_LOG2[tx_size];
  int ck = ORC_TX_COL[tx_type], rk = ORC_TX_ROW[tx_type];
  if (ck == 3 || rk == 3) return -1;
  static const T zero[64];
  T probe[64];
  if (orc_inv_txfm1d(ck, h, zero, probe, 16) ||
      orc_inv_txfm1d(rk, w, zero, probe, 16))
    return -1;
  int wl = ORC_TX_W_LOG2[tx_size], hl = ORC_TX_H_LOG2[tx_size];
  int rect = wl - hl;
  int cw = w < 32 ? w : 32, ch = h < 32 ? h : 32;
  T buf[64 * 64];
  memset(buf, 0, sizeof(buf));
  /* rows: only the first min(H,32) rows of min(W,32) coefficients */
  int range = bit_depth + 8;
  for (int r = 0; r < ch; r++) {
    T tin[64] = {0};
    for (int c = 0; c < cw; c++) {
      T raw = coeffs[r * cw + c];
      T v = (rect == 1 || rect == -1) ? round_shift(w_mul(raw, 2896), 12) : raw;
      tin[c] = clampv(v, range);
    }
    orc_inv_txfm1d(rk, w, tin, buf + r * w, range);
  }
  /* columns */
  int crange = bit_depth + 6 > 16 ? bit_depth + 6 : 16;
  int32_t maxv = (1 << bit_depth) - 1;
  for (int c = 0; c < w; c++) {
    T tin[64], tout[64];
    for (int r = 0; r < h; r++)
      tin[r] = clampv(round_shift(buf[r * w + c], INV_SHIFT[tx_size]), crange);
    orc_inv_txfm1d(ck, h, tin, tout, crange);
    for (int r = 0; r < h; r++) {
      T v = round_shift(tout[r], 4);
      ptrdiff_t idx = r * dst_stride + c;
      orc_px_store(dst, hbd, idx,
                   clamp_i32(w_add(orc_px(dst, hbd, idx), v), 0, maxv));
    }
  }
  return 0;
}
