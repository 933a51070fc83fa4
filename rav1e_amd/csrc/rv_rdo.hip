// rv_rdo.hip -- fused RDO inter-candidate evaluation (replay stage F4).
//
// One wavefront per (candidate, transform block) runs the whole per-
// candidate chain of luma_chroma_mode_rdo -> encode_block_post_cdef ->
// encode_tx_block (src/rdo.rs:649-700, src/encoder.rs:1077-1237) for the
// pixel-domain distortion of the default tune (src/rdo.rs:338-411):
//
//   predict_inter's put_8tap (src/mc.rs:213-307, REGULAR, via
//   src/predict.rs:255-338)            -> prediction in LDS
//   skip variant: compute_distortion of the prediction (cdef_dist_wxh x
//   compute_distortion_bias for luma, sse_wxh x bias for chroma,
//   src/rdo.rs:219-335, 476-508)       -> one u64
//   diff (src/encoder.rs:1044-1058) + FwdTxfm2D::fht DCT_DCT
//   (src/transform/forward.rs:1804-1899) -> coefficients in LDS
//   quantize (src/quantize.rs:255-316, QuantizationContext at the
//   replay's qindex) on the first coded_tx_area entries of the W-stride
//   raster, the slice encode_tx_block hands it; the tx-domain distortion
//   of that slice against its dequantized values -> estimate_rate
//   (src/encoder.rs:1214-1231, src/rdo.rs:204-216)
//   dequantize (src/quantize.rs:319-333)      -> the inverse's input in LDS
//   inv_txfm2d_add (src/transform/inverse.rs:1939-2114)
//                                      -> reconstruction in LDS
//   non-skip variant: compute_distortion of the reconstruction -> one u64
//
// Score launch (F4): every candidate; HBM receives three u64 per candidate
// transform block [skip distortion, non-skip distortion, rate].  Commit
// launch (F6): the winner of every superblock runs the same chain (levels
// forced to zero for a skip winner, which makes the reconstruction the
// prediction) and stores its levels (the entropy coder's input) and its
// reconstruction into the frame.  Every intermediate stays in the
// wavefront's LDS slab.  The
// standalone batched kernels (rv_put_8tap_batch, rv_diff_fwd_txfm_batch,
// rv_inv_txfm_add_batch, rv_cdef_moments_batch, rv_sse_batch) compute the
// same values one stage per launch; the replay parity test pins the fused
// kernel to the CPU replay, which chains the oracle's restatements of them.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "rv_intra.h"
#include "rv_rdo.h"
#include "rv_tx.h"

namespace rv {


// SUBPEL_FILTERS REGULAR (src/mc.rs:70-179): [0] 8-tap, [1] 4-tap (get_filter
// for length <= 4, src/mc.rs:201-210).  Frac 0 is never filtered.
__constant__ int8_t kRdoReg[2][16][8] = {
    {{0, 0, 0, 127, 0, 0, 0, 0}, {0, 2, -6, 126, 8, -2, 0, 0},
     {0, 2, -10, 122, 18, -4, 0, 0}, {0, 2, -12, 116, 28, -8, 2, 0},
     {0, 2, -14, 110, 38, -10, 2, 0}, {0, 2, -14, 102, 48, -12, 2, 0},
     {0, 2, -16, 94, 58, -12, 2, 0}, {0, 2, -14, 84, 66, -12, 2, 0},
     {0, 2, -14, 76, 76, -14, 2, 0}, {0, 2, -12, 66, 84, -14, 2, 0},
     {0, 2, -12, 58, 94, -16, 2, 0}, {0, 2, -12, 48, 102, -14, 2, 0},
     {0, 2, -10, 38, 110, -14, 2, 0}, {0, 2, -8, 28, 116, -12, 2, 0},
     {0, 0, -4, 18, 122, -10, 2, 0}, {0, 0, -2, 8, 126, -6, 2, 0}},
    {{0, 0, 0, 127, 0, 0, 0, 0}, {0, 0, -4, 126, 8, -2, 0, 0},
     {0, 0, -8, 122, 18, -4, 0, 0}, {0, 0, -10, 116, 28, -6, 0, 0},
     {0, 0, -12, 110, 38, -8, 0, 0}, {0, 0, -12, 102, 48, -10, 0, 0},
     {0, 0, -14, 94, 58, -10, 0, 0}, {0, 0, -12, 84, 66, -10, 0, 0},
     {0, 0, -12, 76, 76, -12, 0, 0}, {0, 0, -10, 66, 84, -12, 0, 0},
     {0, 0, -10, 58, 94, -14, 0, 0}, {0, 0, -10, 48, 102, -12, 0, 0},
     {0, 0, -8, 38, 110, -12, 0, 0}, {0, 0, -6, 28, 116, -10, 0, 0},
     {0, 0, -4, 18, 122, -8, 0, 0}, {0, 0, -2, 8, 126, -4, 0, 0}}};

// FWD_SHIFT_{4X4, 8X8, 16X16, 32X32, 64X64} (forward.rs:22-26) by shift_idx
template <int N>
__device__ __forceinline__ void fwd_shifts(int idx, int &s0, int &s1, int &s2) {
  constexpr int8_t k4[3][3] = {{3, 0, 0}, {2, 0, 1}, {0, 0, 3}};
  constexpr int8_t k8[3][3] = {{4, -1, 0}, {2, 0, 1}, {0, 0, 3}};
  constexpr int8_t k32[3][3] = {{4, -2, 0}, {2, 0, 0}, {0, 0, 2}};
  constexpr int8_t k64[3][3] = {{4, -1, -2}, {2, 0, -1}, {0, 0, 1}};
  const int8_t *k = N == 64 ? k64[idx] : N == 32 ? k32[idx] : N == 4 ? k4[idx] : k8[idx];
  s0 = k[0];
  s1 = k[1];
  s2 = k[2];
}
// InvBlock::INTERMEDIATE_SHIFT (inverse.rs:1643-1666): 0 for 4x4, 1 for
// 8x8, 2 from 16x16 up
template <int N>
constexpr int inv_mid_shift() {
  return N == 4 ? 0 : N == 8 ? 1 : 2;
}

// round_shift_array (src/transform/mod.rs:499-521)
__device__ __forceinline__ int32_t rdo_rsa(int32_t v, int bit) {
  if (bit > 0) return round_shift(v, bit);
  if (bit < 0) return (int32_t)((uint32_t)v << -bit);
  return v;
}

// The per-task job: candidate (score) or superblock winner (commit) ->
// prediction block, transform block inside it, MC source and fracs.
struct RdoJob {
  int bx, by;        // prediction block origin in the plane
  int ox, oy;        // transform block offset inside the prediction block
  int src_x, src_y;  // predict_inter's clamped integer source position
  int cf, rf;        // 1/16-pel fracs
  int ref;           // reference index
  bool comp;         // compound: prep_8tap of references 0 and 1, mc_avg
  int src2_x, src2_y, cf2, rf2;  // compound: reference 1's source and fracs
  bool zero;         // commit of a skip winner: every level is zero
  int oi;            // output slot: candidate (or superblock) * ntx_per_cand + block
  int imode, ivar;   // intra (MODE 3): PredictionMode, PredictionVariant
  const void *iedge; // intra: this plane's get_intra_edges (kIntraEdge pixels)
};

// An intra task (MODE 3, RdoArgs::iedges): the superblock of list entry
// `slot`, its mode for this plane, the output slot (score: per superblock 3
// luma / 6 chroma chains; commit: the superblock).  plane: 0 Y, 1 U, 2 V.
template <typename Px, int N>
__device__ __forceinline__ RdoJob rdo_job_intra(const RdoArgs &a, int plane, int t) {
  RdoJob j;
  int sb, mode;
  if (a.commit) {
    sb = a.list[t];
    mode = a.iwin[sb * 2 + (plane ? 1 : 0)];
    j.oi = sb;
  } else if (plane == 0) {
    const int slot = t / 3, k = t - 3 * slot;
    sb = a.list[slot];
    mode = a.imodes[sb * 4 + 1 + k];
    j.oi = sb * 3 + k;
  } else {
    const int slot = t / 6, kc = t - 6 * slot;
    sb = a.list[slot];
    mode = (kc & 1) ? 0 : a.imodes[sb * 4 + 1 + (kc >> 1)];  // [m_k, DC_PRED]
    j.oi = sb * 6 + kc;
  }
  const int sx = sb % a.g.tw, sy = sb / a.g.tw;
  const int fx = a.g.tx0 + sx, fy = a.g.ty0 + sy;
  const int tsx = fx % a.g.tws, tsy = fy % a.g.ths;  // the superblock in its tile
  j.ivar = tsx == 0 && tsy == 0 ? 0 : tsy == 0 ? 1 : tsx == 0 ? 2 : 3;  // PredictionVariant::new
  j.imode = mode;
  j.iedge = (const uint8_t *)a.iedges + ((size_t)sb * 3 + plane) * kIntraEdge * sizeof(Px);
  j.bx = (fx * a.bsize) >> a.xdec;
  j.by = (fy * a.bsize) >> a.ydec;
  j.ox = j.oy = 0;
  j.src_x = j.src_y = j.cf = j.rf = j.ref = 0;
  j.src2_x = j.src2_y = j.cf2 = j.rf2 = 0;
  j.comp = false;
  j.zero = false;
  return j;
}

// The intra prediction of a job into pred (N x N, row-major) by the G lanes
// of a group: edges staged in e (i32, kIntraEdge), then pred_* per pixel.
template <typename Px, int N, int G>
__device__ __forceinline__ void intra_fill(const RdoJob &jb, int32_t *e, Px *pred, int bd, int lane) {
  const Px *eg = (const Px *)jb.iedge;
  for (int i = lane; i < kIntraEdge; i += G) e[i] = eg[i];
  wave_sync();
  IntraSetup st = intra_setup(jb.imode, jb.ivar);
  if (st.mode == 0) st.dcv = intra_dc<G>(e, jb.ivar, N, N, bd, lane);
  const int maxv = (1 << bd) - 1;
  for (int i = lane; i < N * N; i += G) {
    const int r = i / N, c = i - r * N;
    pred[i] = (Px)intra_px(st, e, N, N, r, c, maxv);
  }
  wave_sync();
}

// Transform blocks of this launch: n_tx, or count * ntx_per_cand for a
// compacted candidate list.
__device__ __forceinline__ int rdo_ntx(const RdoArgs &a) {
  return a.count ? __builtin_amdgcn_readfirstlane(*a.count) * a.ntx_per_cand : a.n_tx;
}

template <int N>
__device__ __forceinline__ RdoJob rdo_job(const RdoArgs &a, const RdoPlane &pl, int t) {
  const int ci = t / a.ntx_per_cand, sub = t - ci * a.ntx_per_cand;
  const int cand = a.list ? a.list[ci] : a.cand_base + ci;
  int sb, c;
  RdoJob j;
  j.zero = false;
  j.oi = cand * a.ntx_per_cand + sub;
  if (a.commit) {
    sb = cand;
    c = a.win[sb].c;
    j.zero = a.win[sb].skip != 0;
  } else {
    c = cand / a.g.nsb;
    sb = cand - c * a.g.nsb;
  }
  rv_mv mv, mv1{0, 0};
  j.comp = c >= a.g.R * a.g.M;
  if (j.comp) {
    comp_mvs(a.g, a.sub, sb, c - a.g.R * a.g.M, &mv, &mv1);
    j.ref = 0;
  } else {
    (void)cand_mv(a.g, a.sub, sb, c, &mv);
    j.ref = c / a.g.M;
  }
  const int sx = sb % a.g.tw, sy = sb / a.g.tw;
  j.bx = ((a.g.tx0 + sx) * a.bsize) >> a.xdec;
  j.by = ((a.g.ty0 + sy) * a.bsize) >> a.ydec;
  const int txc = a.mb_w / N;
  j.ox = (sub % txc) * N;
  j.oy = (sub / txc) * N;
  const rv_mc_job m = mc_job_for(pl.ref[j.ref], j.bx, j.by, mv, 0, 0);
  j.src_x = m.src_x;
  j.src_y = m.src_y;
  j.cf = m.col_frac;
  j.rf = m.row_frac;
  j.src2_x = j.src2_y = j.cf2 = j.rf2 = 0;
  if (j.comp) {
    const rv_mc_job m1 = mc_job_for(pl.ref[1], j.bx, j.by, mv1, 0, 0);
    j.src2_x = m1.src_x;
    j.src2_y = m1.src_y;
    j.cf2 = m1.col_frac;
    j.rf2 = m1.row_frac;
  }
  return j;
}

// ---- compound prediction: prep_8tap x 2 + mc_avg (src/predict.rs:300-338,
// src/mc.rs:310-408) ----------------------------------------------------------
// REGULAR filter setup of one reference: packed horizontal taps (u8: all 8
// as i8 for two v_dot4; u16: taps 1..6 as i16 pairs), vertical taps.
struct McF {
  uint32_t xp[3];
  int xsum;
  int yt[8];
  int cf, rf;
};
template <typename Px>
__device__ __forceinline__ McF mc_setup(int cf, int rf, int w, int h) {
  McF f;
  f.cf = cf;
  f.rf = rf;
  const int8_t *xf = kRdoReg[w <= 4][cf];
  const int8_t *yf = kRdoReg[h <= 4][rf];
#pragma unroll
  for (int k = 0; k < 8; k++) f.yt[k] = yf[k];
  f.xsum = 0;
  if constexpr (sizeof(Px) == 1) {
#pragma unroll
    for (int q = 0; q < 2; q++)
      f.xp[q] = (uint32_t)(uint8_t)xf[4 * q] | ((uint32_t)(uint8_t)xf[4 * q + 1] << 8) |
                ((uint32_t)(uint8_t)xf[4 * q + 2] << 16) | ((uint32_t)(uint8_t)xf[4 * q + 3] << 24);
#pragma unroll
    for (int k = 0; k < 8; k++) f.xsum += xf[k];
    f.xp[2] = 0;
  } else {
#pragma unroll
    for (int q = 0; q < 3; q++)
      f.xp[q] = (uint32_t)(uint16_t)(int16_t)xf[2 * q + 1] |
                ((uint32_t)(uint16_t)(int16_t)xf[2 * q + 2] << 16);
  }
  return f;
}
// The horizontal pass of window row `row` (staged like the single-reference
// MC: u8 as i8 = px - 128) at column col: i16 round_shift(sum, 7 - ib), or
// the pixel when the column frac is 0.
template <typename Px>
__device__ __forceinline__ int32_t mc_h(const McF &f, const uint32_t *row, int col, int ib) {
  if constexpr (sizeof(Px) == 1) {
    const int d0 = col >> 2, sh = col & 3;
    const uint32_t w0 = row[d0], w1 = row[d0 + 1], w2 = row[d0 + 2];
    const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh);
    const uint32_t hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
    if (!f.cf) return (int32_t)((lo >> 24) ^ 0x80u);
    int32_t s = dot4_i8(lo, f.xp[0], 128 * f.xsum);
    s = dot4_i8(hi, f.xp[1], s);
    return (int32_t)(int16_t)round_shift(s, 7 - ib);
  } else {
    const int c1 = col + 1, d0 = c1 >> 1, sh = (c1 & 1) * 2;  // pixels col+1 .. col+6
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; k++) w[k] = row[d0 + k];
    uint32_t pp[3];
#pragma unroll
    for (int k = 0; k < 3; k++) pp[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
    if (!f.cf) return (int32_t)(pp[1] & 0xffffu);  // pixel col + 3
    int32_t s = 0;
#pragma unroll
    for (int k = 0; k < 3; k++) s = dot2_i16(pp[k], f.xp[k], s);
    return (int32_t)(int16_t)round_shift(s, 7 - ib);
  }
}
// prep_8tap's output for ring position u (ring[j & 7] = h-pass of window
// row j): (0,0) px << ib; (x,0) the h-pass; (0,y) round_shift(sum, 7 - ib);
// (x,y) round_shift(sum, 7) -- REGULAR taps 0 and 7 are zero.
__device__ __forceinline__ int32_t mc_prep_v(const McF &f, const int32_t *ring, int u, int ib) {
  if (f.rf) {
    int32_t s = 0;
#pragma unroll
    for (int k = 1; k < 7; k++) s += __mul24(f.yt[k], ring[(u + k) & 7]);
    return round_shift(s, f.cf ? 7 : 7 - ib);
  }
  return f.cf ? ring[(u + 3) & 7] : ring[(u + 3) & 7] << ib;
}

// Compound prediction of an N x N block (lane = column) into pred, in bands
// of RB rows whose two windows (references 0 and 1) are staged in `win`;
// mc_avg = clamp(round_shift(t0 + t1, ib + 1)).  Ends with a wave sync.
template <typename Px, int N, int RB>
__device__ __forceinline__ void mc_compound(const RdoArgs &a, const RdoPlane &pl, const RdoJob &jb,
                                            uint32_t *win, Px *pred) {
  constexpr int B = (int)sizeof(Px);
  constexpr int P = B == 1 ? ((N + 8 + 15) / 16) * 16 : ((2 * (N + 8) + 15) / 16) * 16;
  constexpr int kRowDw = ((N + 7) * B + 3) / 4, kTot = (RB + 7) * kRowDw;
  static_assert((RB % 8 == 0 || RB < 8) && N % RB == 0, "bands of whole 8-row groups");
  constexpr int U = RB < 8 ? RB : 8;
  const int col = rv_tid() & (N - 1);
  const int ib = a.bd == 12 ? 2 : 4, maxv = (1 << a.bd) - 1;
  const McF f0 = mc_setup<Px>(jb.cf, jb.rf, a.mb_w, a.mb_h);
  const McF f1 = mc_setup<Px>(jb.cf2, jb.rf2, a.mb_w, a.mb_h);
  uint32_t *w0 = win, *w1 = win + (RB + 7) * (P / 4);
  const uint8_t *sp0 = (const uint8_t *)plane_ptr<Px>(pl.ref[0], jb.src_x + jb.ox - 3, jb.src_y + jb.oy - 3);
  const uint8_t *sp1 =
      (const uint8_t *)plane_ptr<Px>(pl.ref[1], jb.src2_x + jb.ox - 3, jb.src2_y + jb.oy - 3);
  const int64_t rs0 = (int64_t)pl.ref[0].stride * B, rs1 = (int64_t)pl.ref[1].stride * B;
#pragma unroll 1
  for (int band = 0; band < N / RB; band++) {
    if (band) wave_sync();  // the previous band's window reads are done
#pragma unroll 2
    for (int i = col; i < kTot; i += N) {
      const int r = i / kRowDw, d = i - r * kRowDw;
      uint32_t v0, v1;
      __builtin_memcpy(&v0, sp0 + (band * RB + r) * rs0 + 4 * d, 4);
      __builtin_memcpy(&v1, sp1 + (band * RB + r) * rs1 + 4 * d, 4);
      w0[r * (P / 4) + d] = B == 1 ? v0 ^ 0x80808080u : v0;
      w1[r * (P / 4) + d] = B == 1 ? v1 ^ 0x80808080u : v1;
    }
    wave_sync();
    int32_t g0[8], g1[8];
#pragma unroll
    for (int k = 1; k < 6; k++) {
      g0[k] = mc_h<Px>(f0, w0 + k * (P / 4), col, ib);
      g1[k] = mc_h<Px>(f1, w1 + k * (P / 4), col, ib);
    }
    g0[0] = g0[6] = g0[7] = g1[0] = g1[6] = g1[7] = 0;
#pragma unroll 1
    for (int r0 = 0; r0 < RB; r0 += U) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int r = r0 + u;
        g0[(u + 6) & 7] = mc_h<Px>(f0, w0 + (r + 6) * (P / 4), col, ib);
        g1[(u + 6) & 7] = mc_h<Px>(f1, w1 + (r + 6) * (P / 4), col, ib);
        const int32_t t = mc_prep_v(f0, g0, u, ib) + mc_prep_v(f1, g1, u, ib);
        pred[(band * RB + r) * N + col] = (Px)clamp_med3(round_shift(t, ib + 1), 0, maxv);
      }
    }
  }
  wave_sync();  // window reads done, prediction visible
}

// compute_distortion_bias (src/rdo.rs:476-508) of the importance area of
// m x m 4x4 blocks (BLOCK_8X8: m = 2; a chroma plane narrower than 8
// pixels biases BLOCK_4X4 areas, m = 1) at 4x4-block (mi_x, mi_y) of the
// frame: compute_mean_importance sums the f32 importances of the in-frame
// 4x4 blocks in y-then-x order and divides by the full area; the bias is
// (mean / 3) as f64 + 0.65.
__device__ __forceinline__ double rdo_bias(const RdoArgs &a, int mi_x, int mi_y, int m = 2) {
  if (!a.imp) return 0.65;  // (0f32 / 3) as f64 + 0.65
  const int x2 = mi_x + m < a.w_in_b ? mi_x + m : a.w_in_b;
  const int y2 = mi_y + m < a.h_in_b ? mi_y + m : a.h_in_b;
  float tot = 0.f;
  for (int y = mi_y; y < y2; y++)
    for (int x = mi_x; x < x2; x++) tot = __fadd_rn(tot, a.imp[(y >> 1) * a.w_imp + (x >> 1)]);
  return (double)__fdiv_rn(__fdiv_rn(tot, (float)(m * m)), 3.0f) + 0.65;
}
// RawDistortion * bias (src/rdo.rs:539-544): `(value as f64 * bias) as u64`
__device__ __forceinline__ uint64_t rdo_biased(uint64_t v, double bias) {
  return (uint64_t)((double)v * bias);
}

// cdef_dist_wxh_8x8 (src/rdo.rs:219-261) of the 8x8 block at o (plane) vs
// d (LDS, row pitch dp): i32 / i64 moments (64 products of 12-bit pixels
// stay below 2^30: u32 sums, one v_mad_u32_u24 per product), then the f64
// ssim boost; `(sse * ssim_boost + 0.5) as u64`.
__device__ __forceinline__ uint64_t rdo_cdef_finish(int32_t ss, int32_t sd, uint32_t ss2,
                                                    uint32_t sd2, uint32_t ssd, int bd);
template <typename Px>
__device__ __forceinline__ uint64_t rdo_cdef_8x8(const Px *o, int64_t os, const Px *d, int dp,
                                                 int bd) {
  int32_t ss = 0, sd = 0;
  uint32_t ss2 = 0, sd2 = 0, ssd = 0;
#pragma unroll
  for (int j = 0; j < 8; j++)
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int32_t s = o[(int64_t)j * os + i];
      const int32_t e = d[j * dp + i];
      ss += s;
      sd += e;
      ss2 += (uint32_t)wmul24(s, s);
      sd2 += (uint32_t)wmul24(e, e);
      ssd += (uint32_t)wmul24(s, e);
    }
  return rdo_cdef_finish(ss, sd, ss2, sd2, ssd, bd);
}
__device__ __forceinline__ uint64_t rdo_cdef_finish(int32_t ss, int32_t sd, uint32_t ss2,
                                                    uint32_t sd2, uint32_t ssd, int bd) {
  const int cs = bd - 8;
  const int64_t s2 = (int64_t)ss2, d2 = (int64_t)sd2, sdv = (int64_t)ssd;
  const double svar = (double)(s2 - (((int64_t)ss * ss + 32) >> 6));
  const double dvar = (double)(d2 - (((int64_t)sd * sd + 32) >> 6));
  const double sse = (double)(d2 + s2 - 2 * sdv);
  const double boost = (4033.0 / 16384.0) * (svar + dvar + (double)(16384ll << (2 * cs))) /
                       sqrt((double)(16265089ull << (4 * cs)) + svar * dvar);
  const double v = sse * boost + 0.5;
  return v > 0.0 ? (uint64_t)v : 0;
}

// sse_wxh (src/rdo.rs:286-335) over the transform block's sub-blocks (bw x
// bh chroma pixels = an 8x8 importance block), each biased; lanes of a
// group of LPB stride over the sub-blocks.  Returns the lane's partial sum.
template <typename Px, int N, int LPB>
__device__ __forceinline__ uint64_t rdo_sse_biased(const RdoArgs &a, const RdoJob &j, const Px *o,
                                                   int64_t os, const Px *d) {
  const int bw = a.sub_w, bh = a.sub_h, nbx = N / bw, nby = N / bh;
  const int lane = rv_tid() & (LPB - 1);
  uint64_t acc = 0;
  for (int k = lane; k < nbx * nby; k += LPB) {
    const int by = k / nbx, bx = k - by * nbx;
    uint64_t value = 0;
    for (int jj = 0; jj < bh; jj++) {
      uint32_t row = 0;
      for (int i = 0; i < bw; i++) {
        const int32_t c = (int32_t)(int16_t)o[(int64_t)(by * bh + jj) * os + bx * bw + i] -
                          (int32_t)(int16_t)d[(by * bh + jj) * N + bx * bw + i];
        row += (uint32_t)wmul24(c, c);
      }
      value += row;
    }
    const int px = j.bx + j.ox + bx * bw, py = j.by + j.oy + by * bh;
    acc += rdo_biased(value, rdo_bias(a, (px << a.xdec) >> 2, (py << a.ydec) >> 2, (N < 8 ? N : 8) / 4));
  }
  return acc;
}

// compute_distortion of one transform block (the lane's partial): luma
// cdef_dist_wxh_8x8 x bias per 8x8 (src/rdo.rs:263-283), chroma sse_wxh.
template <typename Px, int N, int LPB, bool LUMA>
__device__ __forceinline__ uint64_t rdo_dist_biased(const RdoArgs &a, const RdoJob &j, const Px *o,
                                                    int64_t os, const Px *d) {
  if constexpr (LUMA) {
    // one row of an 8x8 block per lane: row moments, a reduction over the
    // block's 8 lanes (aligned groups of 8), the f64 tail on its first lane
    constexpr int NB = N / 8, ROWS = NB * NB * 8;
    static_assert(LPB % 8 == 0 && ROWS % LPB == 0, "rows of 8x8 blocks over the lanes");
    const int lane = rv_tid() & (LPB - 1);
    uint64_t acc = 0;
#pragma unroll
    for (int k0 = 0; k0 < ROWS; k0 += LPB) {
      const int k = k0 + lane, blk = k >> 3, row = k & 7;
      const int by = blk / NB, bx = blk - by * NB;
      const Px *op = o + (int64_t)(by * 8 + row) * os + bx * 8;
      const Px *dp = d + (by * 8 + row) * N + bx * 8;
      int32_t ss = 0, sd = 0;
      uint32_t ss2 = 0, sd2 = 0, ssd = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const int32_t sv = op[i], e = dp[i];
        ss += sv;
        sd += e;
        ss2 += (uint32_t)wmul24(sv, sv);
        sd2 += (uint32_t)wmul24(e, e);
        ssd += (uint32_t)wmul24(sv, e);
      }
#pragma unroll
      for (int m = 1; m < 8; m <<= 1) {
        ss += __shfl_xor(ss, m, 64);
        sd += __shfl_xor(sd, m, 64);
        ss2 += __shfl_xor(ss2, m, 64);
        sd2 += __shfl_xor(sd2, m, 64);
        ssd += __shfl_xor(ssd, m, 64);
      }
      if (row == 0) {
        const uint64_t v = rdo_cdef_finish(ss, sd, ss2, sd2, ssd, a.bd);
        const int px = j.bx + j.ox + bx * 8, py = j.by + j.oy + by * 8;
        acc += rdo_biased(v, rdo_bias(a, px >> 2, py >> 2));
      }
    }
    return acc;
  } else {
    return rdo_sse_biased<Px, N, LPB>(a, j, o, os, d);
  }
}

// LPB = lanes per transform block: 64 (luma, N = 64) or 32 (chroma, N = 32:
// a wavefront carries two chroma blocks, one per half, so every phase keeps
// all 64 lanes busy).  `valid` = false for a second half without a block:
// it recomputes its partner's block and stores nothing.
// Bytes of a transform block's LDS slab: the i32 coefficient block, the MC
// window, or the two compound windows, whichever is largest.
template <typename Px, int N>
__host__ __device__ constexpr int rdo_slab_bytes() {
  constexpr int B = (int)sizeof(Px);
  constexpr int P = B == 1 ? ((N + 8 + 15) / 16) * 16 : ((2 * (N + 8) + 15) / 16) * 16;
  constexpr int RB = N < 16 ? N : 16;
  constexpr int a = N * (N + 1) * 4, b = (N + 7) * P, c = 2 * (RB + 7) * P;
  return ((a > b ? a : b) > c ? (a > b ? a : b) : c);
}

// MODE: 0 single-reference candidates, 1 compound candidates, 2 either
// (by the job: the commit launch).  LUMA: the distortion is cdef_dist_wxh
// per 8x8 (N >= 8), else sse_wxh per importance sub-block.  `buf` holds
// rdo_slab_bytes<Px, N>().
template <typename Px, int N, int LPB, int MODE, bool LUMA = false>
__device__ __forceinline__ void rdo_cand_body(const RdoArgs &a, const RdoPlane &pl, int t,
                                              bool valid, int32_t *buf, Px *pred,
                                              const uint16_t *scan) {
  constexpr int B = (int)sizeof(Px);
  constexpr int S = N + 1;                       // padded LDS row (i32)
  constexpr int G = LPB / N, RG = N / G;         // MC lane groups
  constexpr int U = RG < 8 ? RG : 8;             // MC rows per ring step
  constexpr int P = B == 1 ? ((N + 8 + 15) / 16) * 16 : ((2 * (N + 8) + 15) / 16) * 16;
  constexpr int C32 = N < 32 ? N : 32;           // coded coefficient extent
  static_assert(!LUMA || N >= 8, "cdef distortion runs on 8x8 blocks");
  const int lane = rv_tid() & (LPB - 1);
  RdoJob jb;
  if constexpr (MODE == 3)
    jb = rdo_job_intra<Px, N>(a, &pl == &a.p[1] ? 2 : 1, t);
  else
    jb = rdo_job<N>(a, pl, t);
  const rv_plane &ref = pl.ref[jb.ref];
  const int ox = jb.ox, oy = jb.oy;  // in the MC block
  const int bd = a.bd, ib = bd == 12 ? 2 : 4, maxv = (1 << bd) - 1;
  const int sx0 = jb.bx + ox, sy0 = jb.by + oy;  // the transform block in the plane
  auto wave_sync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };

  // ---- A. put_8tap into LDS (compound: prep_8tap x 2 + mc_avg; intra:
  // predict_intra from the block's edges) -----------------------------------
  if constexpr (MODE == 3) {
    intra_fill<Px, N, LPB>(jb, buf, pred, a.bd, lane);
  } else if (MODE == 1 || (MODE == 2 && jb.comp)) {
    static_assert(2 * (16 + 7) * (sizeof(Px) == 1 ? 48 : 80) <= N * (N + 1) * 4 || N != 32,
                  "compound windows must fit the coefficient slab");
    mc_compound<Px, N, (N < 16 ? N : 16)>(a, pl, jb, reinterpret_cast<uint32_t *>(buf), pred);
  } else
  {
    uint32_t *win = reinterpret_cast<uint32_t *>(buf);
    const uint8_t *sp = (const uint8_t *)plane_ptr<Px>(ref, jb.src_x + ox - 3, jb.src_y + oy - 3);
    const int64_t rs = (int64_t)ref.stride * B;
    constexpr int kRowDw = ((N + 7) * B + 3) / 4;
    constexpr int kTot = (N + 7) * kRowDw;
#pragma unroll 4
    for (int i = lane; i < kTot; i += LPB) {
      const int r = i / kRowDw, d = i - r * kRowDw;
      uint32_t v;
      __builtin_memcpy(&v, sp + r * rs + 4 * d, 4);
      win[r * (P / 4) + d] = B == 1 ? v ^ 0x80808080u : v;  // u8: stored as i8 = px - 128
    }
    wave_sync();
    const int cf = jb.cf, rf = jb.rf;
    const int8_t *xf = kRdoReg[a.mb_w <= 4][cf];
    const int8_t *yf = kRdoReg[a.mb_h <= 4][rf];
    int yt[8];
#pragma unroll
    for (int k = 0; k < 8; k++) yt[k] = yf[k];
    uint32_t xp[4];
    int xsum = 0;
    if constexpr (B == 1) {
#pragma unroll
      for (int h = 0; h < 2; h++)
        xp[h] = (uint32_t)(uint8_t)xf[4 * h] | ((uint32_t)(uint8_t)xf[4 * h + 1] << 8) |
                ((uint32_t)(uint8_t)xf[4 * h + 2] << 16) | ((uint32_t)(uint8_t)xf[4 * h + 3] << 24);
#pragma unroll
      for (int k = 0; k < 8; k++) xsum += xf[k];
      xp[2] = xp[3] = 0;
    } else {
#pragma unroll
      for (int h = 0; h < 3; h++)  // taps 1..6 (REGULAR taps 0 and 7 are zero)
        xp[h] = (uint32_t)(uint16_t)(int16_t)xf[2 * h + 1] |
                ((uint32_t)(uint16_t)(int16_t)xf[2 * h + 2] << 16);
      xp[3] = 0;
    }
    const int col = lane % N, grp = lane / N;
    auto hval = [&](int tr) -> int32_t {
      const uint32_t *row = win + (grp * RG + tr) * (P / 4);
      if constexpr (B == 1) {
        const int d0 = col >> 2, sh = col & 3;
        const uint32_t w0 = row[d0], w1 = row[d0 + 1], w2 = row[d0 + 2];
        const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh);
        const uint32_t hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
        if (!cf) return (int32_t)((lo >> 24) ^ 0x80u);
        int32_t s = dot4_i8(lo, xp[0], 128 * xsum);
        s = dot4_i8(hi, xp[1], s);
        return (int32_t)(int16_t)round_shift(s, 7 - ib);
      } else {
        const int c1 = col + 1, d0 = c1 >> 1, sh = (c1 & 1) * 2;  // pixels col+1 .. col+6
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; k++) w[k] = row[d0 + k];
        uint32_t pp[3];
#pragma unroll
        for (int k = 0; k < 3; k++) pp[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
        if (!cf) return (int32_t)(pp[1] & 0xffffu);  // pixel col + 3
        int32_t s = 0;
#pragma unroll
        for (int k = 0; k < 3; k++)
          s = dot2_i16(pp[k], xp[k], s);
        return (int32_t)(int16_t)round_shift(s, 7 - ib);
      }
    };
    const int vshift = cf ? 7 + ib : 7;
    int32_t ring[8];  // ring[j & 7] = intermediate of window row j
#pragma unroll
    for (int k = 1; k < 6; k++) ring[k] = hval(k);
    ring[0] = ring[6] = ring[7] = 0;
    static_assert(RG % 8 == 0 || RG < 8, "MC rows run in groups of 8 (static ring indices)");
#pragma unroll 1
    for (int r0 = 0; r0 < RG; r0 += U) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        const int r = r0 + u;
        ring[(u + 6) & 7] = hval(r + 6);
        int32_t v;
        if (rf) {  // taps 1..6: REGULAR taps 0 and 7 are zero (src/mc.rs:71-88)
          int32_t s = 0;
#pragma unroll
          for (int k = 1; k < 7; k++) s += __mul24(yt[k], ring[(u + k) & 7]);
          v = round_shift(s, vshift);
        } else {
          v = cf ? round_shift(ring[(u + 3) & 7], ib) : ring[(u + 3) & 7];
        }
        pred[(grp * RG + r) * N + col] = (Px)clamp_med3(v, 0, maxv);
      }
    }
    wave_sync();  // window reads done (buf is reused), prediction visible
  }
  const Px *o = plane_ptr<Px>(pl.org, sx0, sy0);
  const int64_t ost = pl.org.stride;
  // ---- skip variant: sse_wxh of the prediction ------------------------------
  if (!a.commit) {
    const uint64_t d = group_sum<LPB>(rdo_dist_biased<Px, N, LPB, LUMA>(a, jb, o, ost, pred));
    if (valid && lane == 0) pl.out[(int64_t)jb.oi * 3 + 0] = d;
  }

  int s0, s1, s2;
  fwd_shifts<N>((bd - 8) / 2, s0, s1, s2);
  // ---- B. residual = org - pred, << -shift[0] ------------------------------
  {
    constexpr int PPD = 4 / B;                 // pixels per dword
    constexpr int DPR = N / PPD;               // dwords per row
    const uint8_t *op = (const uint8_t *)o;
    const int64_t os = (int64_t)pl.org.stride * B;
#pragma unroll 8
    for (int i = lane; i < N * DPR; i += LPB) {
      const int r = i / DPR, c = (i - r * DPR) * PPD;
      uint32_t ov, pv;
      __builtin_memcpy(&ov, op + r * os + c * B, 4);
      __builtin_memcpy(&pv, pred + r * N + c, 4);
#pragma unroll
      for (int k = 0; k < PPD; k++) {
        const int sh = 8 * B * k, m = B == 1 ? 0xff : 0xffff;
        const int16_t d = (int16_t)((int16_t)((ov >> sh) & m) - (int16_t)((pv >> sh) & m));
        buf[r * S + c + k] = rdo_rsa((int32_t)d, -s0);
      }
    }
    wave_sync();
  }
  // ---- C. forward DCT_DCT: column pass, then the coded rows ---------------
  if (lane < N) {
    int32_t v[N];
#pragma unroll
    for (int r = 0; r < N; r++) v[r] = buf[r * S + lane];
    tx::fwd1d<1, N>(v, v);
#pragma unroll
    for (int r = 0; r < N; r++) buf[r * S + lane] = rdo_rsa(v[r], -s1);
  }
  wave_sync();
  // quantize reads the first coded_tx_area = C32 * C32 entries of the
  // W-stride raster (src/encoder.rs:1152-1170): for 64x64 that is raster
  // rows 0..15, so only those rows need the row pass.
  constexpr int CA = C32 * C32, RR = CA / N;  // coded area, raster rows it spans
  if (lane < RR) {
    int32_t v[N];
#pragma unroll
    for (int c = 0; c < N; c++) v[c] = buf[lane * S + c];
    tx::fwd1d<1, N>(v, v);
#pragma unroll
    for (int c = 0; c < N; c++) buf[lane * S + c] = rdo_rsa(v[c], -s2);
  }
  wave_sync();
  // quantize (levels -> HBM, the entropy coder's input) + dequantize in
  // place (the inverse transform's input, raster entry i = packed entry i)
  // Levels go back in place (scattered LDS writes); then one coalesced
  // pass stores them to HBM and dequantizes them in place.
  // the tx-domain distortion of the coded slice against its dequantized
  // values (src/encoder.rs:1214-1224): wrapping i32 square, sign-extended
  uint64_t txd = 0;
  quantize_block<CA, LPB>(
      pl.q, scan, [&](int pos) { return buf[(pos / N) * S + (pos % N)]; },
      [&](int pos, int32_t q, int32_t r) {
        int32_t *e = buf + (pos / N) * S + (pos % N);
        const int32_t dd = wsub(*e, r);
        txd += (uint64_t)(int64_t)wmul(dd, dd);
        *e = jb.zero ? 0 : q;
      });
  wave_sync();
  if (!a.commit) {
    txd = group_sum<LPB>(txd);
    const int bits = 2 * (3 - pl.q.log_tx_scale);
    if (valid && lane == 0)
      pl.out[(int64_t)jb.oi * 3 + 2] =
          q_estimate_rate(a.qindex, a.tx_size, (txd + (1ull << (bits - 1))) >> bits);
  }
  {
    int32_t *pk = pl.levels + (int64_t)jb.oi * CA;
#pragma unroll 4
    for (int i = lane; i < CA; i += LPB) {
      int32_t *e = buf + (i / N) * S + (i % N);
      const int32_t q = *e;
      if (valid && a.commit) pk[i] = q;
      *e = q_dequant(pl.q, q, i);
    }
  }
  wave_sync();
  // ---- D. inverse: rows of the coded coefficients, then columns + add ------
  // input row rr of the C32 x C32 block = packed[rr * C32 ..] = raster
  // entries rr * C32 ..; all reads precede the in-place row writes
  const int range = bd + 8;
  {
    int32_t v[N];
    if (lane < C32) {
#pragma unroll
      for (int c = 0; c < N; c++) {
        const int i = lane * C32 + c;
        v[c] = c < C32 ? tx::clampv(buf[(i / N) * S + (i % N)], range) : 0;
      }
    }
    wave_sync();
    if (lane < C32) {
      tx::inv1d<1, N>(v, range);
#pragma unroll
      for (int c = 0; c < N; c++) buf[lane * S + c] = v[c];
    }
  }
  wave_sync();
  if (lane < N) {
    const int crange = bd + 6 > 16 ? bd + 6 : 16;
    int32_t v[N];
#pragma unroll
    for (int r = 0; r < N; r++)
      v[r] = r < C32 ? tx::clampv(round_shift(buf[r * S + lane], inv_mid_shift<N>()), crange) : 0;
    tx::inv1d<1, N>(v, crange);
#pragma unroll
    for (int r = 0; r < N; r++) {
      Px *q = pred + r * N + lane;
      *q = (Px)clamp_med3(wadd((int32_t)*q, round_shift(v[r], 4)), 0, maxv);
    }
  }
  wave_sync();
  if (a.commit) {  // reconstruction -> the frame, coalesced dwords
    constexpr int PPD = 4 / B, DPR = N / PPD;
    uint8_t *dp = (uint8_t *)plane_ptr_mut<Px>(pl.dst, sx0, sy0);
    const int64_t ds = (int64_t)pl.dst.stride * B;
#pragma unroll 8
    for (int i = lane; i < N * DPR; i += LPB) {
      const int r = i / DPR, c = (i - r * DPR) * PPD;
      uint32_t v;
      __builtin_memcpy(&v, pred + r * N + c, 4);
      if (valid) __builtin_memcpy(dp + r * ds + c * B, &v, 4);
    }
    return;
  }
  // ---- non-skip variant: sse_wxh of the reconstruction ----------------------
  const uint64_t d = group_sum<LPB>(rdo_dist_biased<Px, N, LPB, LUMA>(a, jb, o, ost, pred));
  if (valid && lane == 0) pl.out[(int64_t)jb.oi * 3 + 1] = d;
}

// ---- luma candidates: 64x64 --------------------------------------------------
// The chain of rdo_cand_body<Px, 64, true, 64> without the 64x64 i32 slab:
//  * put_8tap in NPART bands of 64 / NPART output rows, their window rows
//    staged in turn;
//  * the residual is formed per column straight from the source plane and
//    the LDS prediction, and only column-DCT outputs 0..15 are kept: the
//    quantizer reads raster rows 0..15 of the 64x64 fht output
//    (src/encoder.rs:1152-1156), and row r of that raster is the row DCT of
//    column-pass row r, so the compiler drops the other 48 outputs;
//  * the inverse row pass stores round_shift(., INTERMEDIATE_SHIFT) clamped
//    to the column range max(bd + 6, 16) (inverse.rs:2075-2098): i16 up to
//    10 bits (Mid), i32 for 12.
// Phases: luma_front (MC, residual, column DCT -> fmid), luma_fwd_row (row
// DCT of one raster row, one lane per row), luma_quantize, luma_inv_row_load /
// _tx (one lane per coded row), luma_back (inverse columns, reconstruction,
// cdef moments).
__host__ __device__ constexpr int cmax(int a, int b) { return a > b ? a : b; }

template <typename Px, typename Mid, int NPART>
struct LumaLds {
  static constexpr int kWinP = sizeof(Px) == 1 ? 80 : 144;  // window row pitch, bytes
  static constexpr int kWinRows = 64 / NPART + 7;
  static constexpr int kCompRows = sizeof(Px) == 1 ? 16 : 8;  // compound MC band
  static constexpr int kScr =  // bytes of the phase-shared scratch
      cmax(cmax(cmax(kWinRows * kWinP, 16 * 65 * 4), 32 * 66 * (int)sizeof(Mid)),
           2 * (kCompRows + 7) * kWinP);
  static constexpr int kSlot = (kScr + 64 * 64 * (int)sizeof(Px) + 15) / 16 * 16;  // + pred
};


// MC into pred, then residual + column DCT: fmid = scr as i32 [16][65].  No
// trailing synchronisation (the caller's).
// The lane's 8x8 block (lane = 8 * row + column) of the 64x64 luma block:
// cdef_dist_wxh_8x8 x compute_distortion_bias, summed over the wavefront
// (cdef_dist_wxh, src/rdo.rs:263-283) -- the luma compute_distortion.
template <typename Px>
__device__ __forceinline__ uint64_t luma_dist(const RdoArgs &a, const RdoJob &j, const Px *o,
                                              int64_t os, const Px *pred) {
  const int lane = rv_tid() & 63, by = lane >> 3, bx = lane & 7;
  const uint64_t v =
      rdo_cdef_8x8<Px>(o + (int64_t)(by * 8) * os + bx * 8, os, pred + by * 8 * 64 + bx * 8, 64, a.bd);
  const int px = j.bx + bx * 8, py = j.by + by * 8;
  return group_sum<64>(rdo_biased(v, rdo_bias(a, px >> 2, py >> 2)));
}

template <typename Px, int NPART, int MODE>
__device__ __forceinline__ void luma_front(const RdoArgs &a, const RdoPlane &pl, int t,
                                           const RdoJob &jb, bool valid, uint8_t *scr, Px *pred,
                                           bool skip_dist = true) {
  constexpr int N = 64, B = (int)sizeof(Px);
  constexpr int P = LumaLds<Px, int16_t, NPART>::kWinP;
  constexpr int RP = N / NPART;  // output rows per band
  static_assert(RP % 8 == 0, "MC rows run in groups of 8");
  const int lane = rv_tid() & 63;
  const rv_plane &ref = pl.ref[jb.ref];
  const int ox = 0, oy = 0;
  const int bd = a.bd, ib = bd == 12 ? 2 : 4, maxv = (1 << bd) - 1;

  // ---- A. put_8tap (src/mc.rs:213-307) into pred, NPART bands; compound:
  // prep_8tap x 2 + mc_avg in bands of kCompRows; intra: predict_intra
  if constexpr (MODE == 3) {
    intra_fill<Px, 64, 64>(jb, reinterpret_cast<int32_t *>(scr), pred, bd, lane);
  } else if (MODE == 1 || (MODE == 2 && jb.comp)) {
    mc_compound<Px, 64, LumaLds<Px, int16_t, NPART>::kCompRows>(
        a, pl, jb, reinterpret_cast<uint32_t *>(scr), pred);
  } else
  {
    uint32_t *win = reinterpret_cast<uint32_t *>(scr);
    const int cf = jb.cf, rf = jb.rf;
    const int8_t *xf = kRdoReg[a.mb_w <= 4][cf];
    const int8_t *yf = kRdoReg[a.mb_h <= 4][rf];
    int yt[8];
#pragma unroll
    for (int k = 0; k < 8; k++) yt[k] = yf[k];
    uint32_t xp[4];
    int xsum = 0;
    if constexpr (B == 1) {
#pragma unroll
      for (int h = 0; h < 2; h++)
        xp[h] = (uint32_t)(uint8_t)xf[4 * h] | ((uint32_t)(uint8_t)xf[4 * h + 1] << 8) |
                ((uint32_t)(uint8_t)xf[4 * h + 2] << 16) | ((uint32_t)(uint8_t)xf[4 * h + 3] << 24);
#pragma unroll
      for (int k = 0; k < 8; k++) xsum += xf[k];
      xp[2] = xp[3] = 0;
    } else {
#pragma unroll
      for (int h = 0; h < 3; h++)  // taps 1..6 (REGULAR taps 0 and 7 are zero)
        xp[h] = (uint32_t)(uint16_t)(int16_t)xf[2 * h + 1] |
                ((uint32_t)(uint16_t)(int16_t)xf[2 * h + 2] << 16);
      xp[3] = 0;
    }
    const int col = lane;
    auto hval = [&](int tr) __attribute__((always_inline)) -> int32_t {
      const uint32_t *row = win + tr * (P / 4);
      if constexpr (B == 1) {
        const int d0 = col >> 2, sh = col & 3;
        const uint32_t w0 = row[d0], w1 = row[d0 + 1], w2 = row[d0 + 2];
        const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh);
        const uint32_t hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
        if (!cf) return (int32_t)((lo >> 24) ^ 0x80u);
        int32_t s = dot4_i8(lo, xp[0], 128 * xsum);
        s = dot4_i8(hi, xp[1], s);
        return (int32_t)(int16_t)round_shift(s, 7 - ib);
      } else {
        const int c1 = col + 1, d0 = c1 >> 1, sh = (c1 & 1) * 2;  // pixels col+1 .. col+6
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; k++) w[k] = row[d0 + k];
        uint32_t pp[3];
#pragma unroll
        for (int k = 0; k < 3; k++) pp[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
        if (!cf) return (int32_t)(pp[1] & 0xffffu);  // pixel col + 3
        int32_t s = 0;
#pragma unroll
        for (int k = 0; k < 3; k++)
          s = dot2_i16(pp[k], xp[k], s);
        return (int32_t)(int16_t)round_shift(s, 7 - ib);
      }
    };
    const int vshift = cf ? 7 + ib : 7;
    constexpr int kRowDw = ((N + 7) * B + 3) / 4;
    constexpr int kTot = (RP + 7) * kRowDw;
    const int64_t rs = (int64_t)ref.stride * B;
#pragma unroll 1
    for (int half = 0; half < NPART; half++) {
      const uint8_t *sp =
          (const uint8_t *)plane_ptr<Px>(ref, jb.src_x + ox - 3, jb.src_y + oy - 3 + RP * half);
      if (half) wave_sync();  // the previous band's window reads are done
#pragma unroll 4
      for (int i = lane; i < kTot; i += 64) {
        const int r = i / kRowDw, d = i - r * kRowDw;
        uint32_t v;
        __builtin_memcpy(&v, sp + r * rs + 4 * d, 4);
        win[r * (P / 4) + d] = B == 1 ? v ^ 0x80808080u : v;  // u8: stored as i8 = px - 128
      }
      wave_sync();
      int32_t ring[8];  // ring[j & 7] = intermediate of window row j
#pragma unroll
      for (int k = 1; k < 6; k++) ring[k] = hval(k);
      ring[0] = ring[6] = ring[7] = 0;
#pragma unroll 1
      for (int r0 = 0; r0 < RP; r0 += 8) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
          const int r = r0 + u;
          ring[(u + 6) & 7] = hval(r + 6);
          int32_t v;
          if (rf) {  // taps 1..6 (REGULAR taps 0 and 7 are zero)
            int32_t s = 0;
#pragma unroll
            for (int k = 1; k < 7; k++) s += __mul24(yt[k], ring[(u + k) & 7]);
            v = round_shift(s, vshift);
          } else {
            v = cf ? round_shift(ring[(u + 3) & 7], ib) : ring[(u + 3) & 7];
          }
          pred[(RP * half + r) * N + col] = (Px)clamp_med3(v, 0, maxv);
        }
      }
    }
    wave_sync();  // window reads done (scr is reused), prediction visible
  }

  const Px *o = plane_ptr<Px>(pl.org, jb.bx, jb.by);
  // ---- skip variant: compute_distortion of the prediction (or later, in a
  // narrow phase of the quad kernel: skip_dist = false) ----------------------
  if (!a.commit && skip_dist) {
    const uint64_t d = luma_dist<Px>(a, jb, o, pl.org.stride, pred);
    if (valid && lane == 0) pl.out[(int64_t)jb.oi * 3 + 0] = d;
  }
  int s0, s1, s2;
  fwd_shifts<N>((bd - 8) / 2, s0, s1, s2);
  int32_t *fmid = reinterpret_cast<int32_t *>(scr);  // [16][65]: column-DCT rows 0..15
  // ---- B + C. residual (src/encoder.rs:1044-1058) and the column DCT -------
  {
    int32_t v[N];
#pragma unroll
    for (int r = 0; r < N; r++) {
      const int16_t d = (int16_t)((int16_t)o[(int64_t)r * pl.org.stride + lane] -
                                  (int16_t)pred[r * N + lane]);
      v[r] = rdo_rsa((int32_t)d, -s0);
    }
    tx::fwd1d<1, N>(v, v);
#pragma unroll
    for (int r = 0; r < 16; r++) fmid[r * 65 + lane] = rdo_rsa(v[r], -s1);
  }
}

// Row DCT of one fmid row (raster row r of the 64x64 fht output), in place.
__device__ __forceinline__ void luma_fwd_row(int32_t *row, int bd) {
  int s0, s1, s2;
  fwd_shifts<64>((bd - 8) / 2, s0, s1, s2);
  int32_t v[64];
#pragma unroll
  for (int c = 0; c < 64; c++) v[c] = row[c];
  tx::fwd1d<1, 64>(v, v);
#pragma unroll
  for (int c = 0; c < 64; c++) row[c] = rdo_rsa(v[c], -s2);
}

// quantize + dequantize of the candidate's coded 32x32 area (raster entries
// 0..1023 of the 64x64 fht output = fmid rows 0..15, src/encoder.rs:1170,
// 1192), dequantized values in place (the inverse transform's input).
// Score: the tx-domain distortion of the slice -> estimate_rate -> out[2].
// Commit: levels -> pl.levels (the entropy coder's input), zero for a skip
// winner.
__device__ __forceinline__ void luma_quantize(const RdoArgs &a, const RdoPlane &pl, int t,
                                              const RdoJob &jb, bool valid, int32_t *fmid,
                                              const uint16_t *scan) {
  uint64_t txd = 0;
  quantize_block<1024, 64>(
      pl.q, scan, [&](int pos) { return fmid[(pos >> 6) * 65 + (pos & 63)]; },
      [&](int pos, int32_t q, int32_t r) {
        int32_t *e = fmid + (pos >> 6) * 65 + (pos & 63);
        const int32_t dd = wsub(*e, r);
        txd += (uint64_t)(int64_t)wmul(dd, dd);
        *e = jb.zero ? 0 : q;
      });
  const int lane = rv_tid() & 63;
  if (!a.commit) {
    txd = group_sum<64>(txd);
    const int bits = 2 * (3 - pl.q.log_tx_scale);
    if (valid && lane == 0)
      pl.out[(int64_t)jb.oi * 3 + 2] =
          q_estimate_rate(a.qindex, a.tx_size, (txd + (1ull << (bits - 1))) >> bits);
  }
  wave_sync();
  int32_t *pk = pl.levels + (int64_t)jb.oi * 1024;
#pragma unroll 4
  for (int i = lane; i < 1024; i += 64) {
    int32_t *e = fmid + (i >> 6) * 65 + (i & 63);
    const int32_t q = *e;
    if (a.commit) pk[i] = q;
    *e = q_dequant(pl.q, q, i);
  }
}

// Inverse row rr (0..31) of the coded 32x32 block: packed[rr * 32 ..] =
// raster entries of fmid row rr >> 1 from column (rr & 1) * 32.  pk (may be
// null) receives the 32 raw coefficients (the packed output).
__device__ __forceinline__ void luma_inv_row_load(const int32_t *fmid, int rr, int32_t *v,
                                                  int range, int32_t *pk) {
  const int32_t *src = fmid + (rr >> 1) * 65 + (rr & 1) * 32;
#pragma unroll
  for (int c = 0; c < 32; c++) {
    const int32_t x = src[c];
    if (pk) pk[c] = x;
    v[c] = tx::clampv(x, range);
  }
#pragma unroll
  for (int c = 32; c < 64; c++) v[c] = 0;
}
template <typename Mid>
__device__ __forceinline__ void luma_inv_row_tx(int32_t *v, Mid *dst, int range, int crange) {
  tx::inv1d<1, 64>(v, range);
#pragma unroll
  for (int c = 0; c < 64; c++) dst[c] = (Mid)tx::clampv(round_shift(v[c], 2), crange);
}

// Inverse columns + add into pred; commit: the reconstruction -> the
// frame; score: the non-skip compute_distortion -> out[1].  imid = [32][66]
// row-pass output.
template <typename Px, typename Mid>
__device__ __forceinline__ void luma_back(const RdoArgs &a, const RdoPlane &pl, int t,
                                          const RdoJob &jb, bool valid, const Mid *imid,
                                          Px *pred) {
  constexpr int N = 64, B = (int)sizeof(Px);
  const int lane = rv_tid() & 63;
  const int bd = a.bd, maxv = (1 << bd) - 1;
  const int crange = bd + 6 > 16 ? bd + 6 : 16;
  // ---- D'. inverse columns + add into pred ---------------------------------
  {
    int32_t v[N];
#pragma unroll
    for (int r = 0; r < N; r++) v[r] = r < 32 ? (int32_t)imid[r * 66 + lane] : 0;
    tx::inv1d<1, N>(v, crange);
#pragma unroll
    for (int r = 0; r < N; r++) {
      Px *q = pred + r * N + lane;
      *q = (Px)clamp_med3(wadd((int32_t)*q, round_shift(v[r], 4)), 0, maxv);
    }
  }
  wave_sync();
  if (a.commit) {  // reconstruction -> the frame, coalesced dwords
    constexpr int PPD = 4 / B, DPR = N / PPD;
    uint8_t *dp = (uint8_t *)plane_ptr_mut<Px>(pl.dst, jb.bx, jb.by);
    const int64_t ds = (int64_t)pl.dst.stride * B;
#pragma unroll 8
    for (int i = lane; i < N * DPR; i += 64) {
      const int r = i / DPR, c = (i - r * DPR) * PPD;
      uint32_t v;
      __builtin_memcpy(&v, pred + r * N + c, 4);
      if (valid) __builtin_memcpy(dp + r * ds + c * B, &v, 4);
    }
    return;
  }
  // ---- E. non-skip variant: compute_distortion of the reconstruction -------
  const uint64_t d = luma_dist<Px>(a, jb, plane_ptr<Px>(pl.org, jb.bx, jb.by), pl.org.stride, pred);
  if (valid && lane == 0) pl.out[(int64_t)jb.oi * 3 + 1] = d;
}

// One luma candidate per wavefront (12-bit).
template <typename Px, typename Mid, int NPART, int MODE>
__device__ __forceinline__ void rdo_luma_body(const RdoArgs &a, const RdoPlane &pl, int t,
                                              uint8_t *scr, Px *pred, const uint16_t *scan) {
  const int lane = rv_tid() & 63;
  RdoJob jb;
  if constexpr (MODE == 3)
    jb = rdo_job_intra<Px, 64>(a, 0, t);
  else
    jb = rdo_job<64>(a, pl, t);
  luma_front<Px, NPART, MODE>(a, pl, t, jb, true, scr, pred);
  wave_sync();
  int32_t *fmid = reinterpret_cast<int32_t *>(scr);
  if (lane < 16) luma_fwd_row(fmid + lane * 65, a.bd);
  wave_sync();
  luma_quantize(a, pl, t, jb, true, fmid, scan);
  wave_sync();
  const int range = a.bd + 8, crange = a.bd + 6 > 16 ? a.bd + 6 : 16;
  Mid *imid = reinterpret_cast<Mid *>(scr);  // [32][66]
  {
    int32_t v[64];
    if (lane < 32) luma_inv_row_load(fmid, lane, v, range, nullptr);
    wave_sync();  // every read of fmid precedes the imid writes (same bytes)
    if (lane < 32) luma_inv_row_tx(v, imid + lane * 66, range, crange);
  }
  wave_sync();
  luma_back<Px, Mid>(a, pl, t, jb, true, imid, pred);
}

// Chroma transform blocks, two per wavefront (one per half), plane U then
// V: pair b of the launch.
// pairs: per plane (default: the grid's size, from n_tx; list-driven
// launches pass the count's).
template <typename Px, int MODE>
__device__ __forceinline__ void rdo_chroma_pair(const RdoArgs &chroma, int b, int32_t *buf,
                                                Px *pred, const uint16_t *scan, int pairs = -1) {
  if (pairs < 0) pairs = (chroma.n_tx + 1) / 2;
  const int plane = b / pairs;
  const int half = (rv_tid() & 63) >> 5;
  const int n = rdo_ntx(chroma);
  int i = 2 * (b - plane * pairs) + half;
  if (i - half >= n) return;  // past the compacted list: the whole pair
  const bool valid = i < n;
  if (!valid) i -= 1;
  rdo_cand_body<Px, 32, 32, MODE>(chroma, chroma.p[plane], i, valid, buf + half * 32 * 33,
                            pred + half * 32 * 32, scan);
}

// The quantizer's scan (coded area <= 1024) staged in LDS for the
// workgroup; ends with a barrier.
__device__ __forceinline__ void stage_scan(uint16_t *dst, int tx_index) {
  const uint16_t *src = RV_SCANS + RV_SCAN_OFF[tx_index];
  for (int i = rv_tid(); i < 1024; i += blockDim.x) dst[i] = src[i];
  __syncthreads();
}

// One luma candidate or one chroma pair per 64-thread workgroup: the
// 12-bit path (its row-pass intermediate needs i32) and the split-stream
// option.  LDS: the larger of the luma slot and the chroma pair.
template <typename Px>
using SingleLds = LumaLds<Px, typename std::conditional<sizeof(Px) == 1, int16_t, int32_t>::type, 2>;
constexpr int kChromaPair(int pxb) { return 2 * 32 * 33 * 4 + 2 * 32 * 32 * pxb; }

// MODE 0 / 1: score single-reference / compound candidates; 2: commit
template <typename Px, int MODE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void rdo_frame_kernel(
    RdoArgs luma, RdoArgs chroma) {
  using L = SingleLds<Px>;
  using Mid = typename std::conditional<sizeof(Px) == 1, int16_t, int32_t>::type;
  __shared__ __align__(16) uint8_t lds[cmax(L::kSlot, kChromaPair(sizeof(Px)))];
  __shared__ uint16_t scan[1024];
  const int b = blockIdx.x;
  stage_scan(scan, b < luma.n_tx ? luma.q_tx_index : chroma.q_tx_index);
  if (b < luma.n_tx && b >= rdo_ntx(luma)) return;  // past the compacted list
  if (b < luma.n_tx)
    rdo_luma_body<Px, Mid, 2, MODE>(luma, luma.p[0], b, lds,
                              reinterpret_cast<Px *>(lds + L::kScr), scan);
  else
    rdo_chroma_pair<Px, MODE>(chroma, b - luma.n_tx, reinterpret_cast<int32_t *>(lds),
                        reinterpret_cast<Px *>(lds + 2 * 32 * 33 * 4), scan);
}

// 8- and 10-bit: 256-thread workgroups.  Blocks [0, nquads) carry four luma
// candidates, one per wavefront, that share the two narrow phases -- the row
// DCT (16 raster rows per candidate: wavefront 0 runs all 64 rows) and the
// inverse rows (32 per candidate: wavefronts 0 and 1 run all 128) -- so
// those phases issue a quarter / half of the instructions of the
// single-candidate body.  The rest carry chroma pairs, three per workgroup
// (wavefront 3 leaves at once), inside the same LDS.
template <typename Px>
struct QuadLds {
  using L = LumaLds<Px, int16_t, sizeof(Px) == 1 ? 2 : 4>;
  static constexpr int kBytes = cmax(4 * L::kSlot, 3 * kChromaPair(sizeof(Px)));
};

// RAV1E_HIP_RDO_PHASES=1 (diagnostic, var bit 4 on the list launches with a
// pool hint, i.e. the MV-stack rounds): thread 0 of each workgroup adds its
// item's phase spans (wall_clock64 ticks) into g_rdo_ph[set][k]: luma quads
// k = 0 front (scan staging, MC, skip distortion, column DCT), 1 row DCT,
// 2 quantize, 3 inverse rows, 4 inverse columns + reconstruction +
// distortion, 5 items; chroma triples (set 2) k = 0 whole item, 5 items
// Compiled in with -DRV_RDO_PHASES=1 only (a diagnostic build: the
// timestamps cost scratch in the product kernels).
#ifndef RV_RDO_PHASES
#define RV_RDO_PHASES 0
#endif
__device__ unsigned long long g_rdo_ph[3][8];
struct QuadPh {
  unsigned long long t[5];
};

// var (RAV1E_HIP_RDO_VARIANT, A/B): bit 0 moves the skip distortion of the
// scoring launches into the narrow phases (waves 1..3 during the row DCT,
// wave 2 for wave 0's candidate during the inverse rows); bit 1 raises the
// priority of the waves running a narrow phase (s_setprio).
// The workgroup's four luma candidates t0 = 4 b .. 4 b + 3 (n: the tasks)
template <typename Px, int MODE>
__device__ __forceinline__ void rdo_quad_luma(const RdoArgs &luma, int b, int n, int var,
                                              uint8_t *lds, const uint16_t *scan,
                                              QuadPh *ph = nullptr) {
  using L = typename QuadLds<Px>::L;
  constexpr int NPART = sizeof(Px) == 1 ? 2 : 4;
  const int wave = __builtin_amdgcn_readfirstlane(rv_tid() >> 6), lane = rv_tid() & 63;
  auto slot = [&](int q) __attribute__((always_inline)) { return lds + q * L::kSlot; };
  auto fmid = [&](int q) __attribute__((always_inline)) {
    return reinterpret_cast<int32_t *>(slot(q));
  };
  auto imid = [&](int q) __attribute__((always_inline)) {
    return reinterpret_cast<int16_t *>(slot(q));
  };
  auto pred = [&](int q) __attribute__((always_inline)) {
    return reinterpret_cast<Px *>(slot(q) + L::kScr);
  };
  const int t0 = 4 * b, t = t0 + wave;
  if (t0 >= n) return;  // past the compacted list (uniform over the workgroup)
  const bool valid = t < n;
  RdoJob jb;
  if constexpr (MODE == 3)
    jb = rdo_job_intra<Px, 64>(luma, 0, valid ? t : n - 1);
  else
    jb = rdo_job<64>(luma, luma.p[0], valid ? t : n - 1);
  const bool late_dist = (var & 1) && !luma.commit;
  const bool prio = (var & 2) != 0;
  if (valid)
    luma_front<Px, NPART, MODE>(luma, luma.p[0], t, jb, true, slot(wave), pred(wave), !late_dist);
  __syncthreads();
  if (RV_RDO_PHASES && ph) ph->t[1] = wall_clock64();
  if (wave == 0) {  // row DCT: lane = 16 * candidate + raster row
    if (prio) __builtin_amdgcn_s_setprio(2);
    const int q = lane >> 4;
    if (t0 + q < n) luma_fwd_row(fmid(q) + (lane & 15) * 65, luma.bd);
    if (prio) __builtin_amdgcn_s_setprio(0);
  } else if (late_dist && valid) {  // the skip variant's distortion of this wave's candidate
    const uint64_t d = luma_dist<Px>(luma, jb, plane_ptr<Px>(luma.p[0].org, jb.bx, jb.by),
                                     luma.p[0].org.stride, pred(wave));
    if (lane == 0) luma.p[0].out[(int64_t)jb.oi * 3 + 0] = d;
  }
  __syncthreads();
  if (RV_RDO_PHASES && ph) ph->t[2] = wall_clock64();
  if (valid) luma_quantize(luma, luma.p[0], t, jb, true, fmid(wave), scan);
  __syncthreads();
  if (RV_RDO_PHASES && ph) ph->t[3] = wall_clock64();
  if (wave < 2) {  // inverse rows: lane = 32 * (candidate & 1) + coded row
    if (prio) __builtin_amdgcn_s_setprio(2);
    const int q = 2 * wave + (lane >> 5), rr = lane & 31;
    const bool vq = t0 + q < n;
    const int range = luma.bd + 8, crange = luma.bd + 6 > 16 ? luma.bd + 6 : 16;
    int32_t v[64];
    if (vq) luma_inv_row_load(fmid(q), rr, v, range, nullptr);
    wave_sync();  // the wavefront's fmid reads precede its imid writes (same bytes)
    if (vq) luma_inv_row_tx(v, imid(q) + rr * 66, range, crange);
    if (prio) __builtin_amdgcn_s_setprio(0);
  } else if (wave == 2 && late_dist) {  // wave 0's candidate (its prediction is intact)
    RdoJob j0;
    if constexpr (MODE == 3)
      j0 = rdo_job_intra<Px, 64>(luma, 0, t0);
    else
      j0 = rdo_job<64>(luma, luma.p[0], t0);
    const uint64_t d = luma_dist<Px>(luma, j0, plane_ptr<Px>(luma.p[0].org, j0.bx, j0.by),
                                     luma.p[0].org.stride, pred(0));
    if (lane == 0) luma.p[0].out[(int64_t)j0.oi * 3 + 0] = d;
  }
  __syncthreads();
  if (RV_RDO_PHASES && ph) ph->t[4] = wall_clock64();
  if (valid) luma_back<Px, int16_t>(luma, luma.p[0], t, jb, true, imid(wave), pred(wave));
}

// Chroma pairs 3 c .. 3 c + 2 of the launch, one per wavefront (wave 3
// idles): wave-local, no workgroup barriers.  pairs: per plane.
template <typename Px, int MODE>
__device__ __forceinline__ void rdo_quad_chroma(const RdoArgs &chroma, int c, int pairs,
                                                uint8_t *lds, const uint16_t *scan) {
  const int wave = __builtin_amdgcn_readfirstlane(rv_tid() >> 6);
  const int pair = 3 * c + wave;
  if (wave == 3 || pair >= 2 * pairs) return;
  uint8_t *w = lds + wave * kChromaPair(sizeof(Px));
  rdo_chroma_pair<Px, MODE>(chroma, pair, reinterpret_cast<int32_t *>(w),
                            reinterpret_cast<Px *>(w + 2 * 32 * 33 * 4), scan, pairs);
}

// The MV-stack rounds' chroma (var bit 5): blocks 4 c .. 4 c + 3 of the
// launch (plane U's n, then V's), one per wavefront on all 64 lanes (two
// lanes per column in MC, twice the lanes in the residual, quantizer and
// distortion loops).  A round launch costs its slowest item, and a
// wavefront holding two blocks (one per half) was it: 61 us per triple
// against 55 us per single-reference luma quad (profiles/r06_phases.txt).
template <typename Px, int MODE>
__device__ __forceinline__ void rdo_quad_chroma4(const RdoArgs &chroma, int c, int n, uint8_t *lds,
                                                 const uint16_t *scan) {
  constexpr int kSlab = rdo_slab_bytes<Px, 32>();
  static_assert(4 * (kSlab + 32 * 32 * (int)sizeof(Px)) <= QuadLds<Px>::kBytes, "4 chroma slabs");
  const int wave = __builtin_amdgcn_readfirstlane(rv_tid() >> 6);
  const int k = 4 * c + wave;
  if (k >= 2 * n) return;
  const int plane = k >= n ? 1 : 0, i = k - plane * n;
  uint8_t *w = lds + wave * (kSlab + 32 * 32 * (int)sizeof(Px));
  rdo_cand_body<Px, 32, 64, MODE>(chroma, chroma.p[plane], i, true, reinterpret_cast<int32_t *>(w),
                                  reinterpret_cast<Px *>(w + kSlab), scan);
}

// One workgroup b of the quad launch: four luma candidates, or three
// chroma pairs past nquads.  The arguments come by value: bound by
// reference to the kernel's arguments they were copied to scratch memory
// (1.5 KB per lane; by value the kernels keep the 16-20 B they had)
template <typename Px, int MODE>
__device__ __forceinline__ void rdo_quad_wg(RdoArgs luma, RdoArgs chroma, int nquads,
                                            int var, int b, uint8_t *lds, uint16_t *scan) {
  // a workgroup past the compacted lists leaves before staging the scan:
  // the MV-stack rounds launch the full grid for a few dozen superblocks'
  // candidates (the device holds the count), so most workgroups exit here
  if (b >= nquads) {
    const int pairs = (chroma.n_tx + 1) / 2, nc = rdo_ntx(chroma);
    bool any = false;
    for (int w = 0; w < 3; w++) {
      const int p = 3 * (b - nquads) + w;
      if (p < 2 * pairs) any |= 2 * (p - (p / pairs) * pairs) < nc;
    }
    if (!any) return;
  } else if (4 * b >= rdo_ntx(luma)) {
    return;
  }
  stage_scan(scan, b >= nquads ? chroma.q_tx_index : luma.q_tx_index);
  if (b >= nquads)  // chroma pairs
    rdo_quad_chroma<Px, MODE>(chroma, b - nquads, (chroma.n_tx + 1) / 2, lds, scan);
  else
    rdo_quad_luma<Px, MODE>(luma, b, rdo_ntx(luma), var, lds, scan);
}

template <typename Px, int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void rdo_quad_kernel(
    RdoArgs luma, RdoArgs chroma, int nquads, int var) {
  __shared__ __align__(16) uint8_t lds[QuadLds<Px>::kBytes];
  __shared__ uint16_t scan[1024];
  rdo_quad_wg<Px, MODE>(luma, chroma, nquads, var, blockIdx.x, lds, scan);
}

// The single-reference (MODE 0) and the compound (MODE 1) candidates of a
// frame in one launch: workgroups below g0 run the single ones, the rest the
// compound ones.  They are independent, and in the MV-stack rounds each
// launch holds a few dozen superblocks' candidates, so two launches in a row
// cost two candidate latencies where one costs one.
template <typename Px>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void rdo_quad_pair_kernel(
    RdoArgs l0, RdoArgs c0, int nq0, int g0, RdoArgs l1, RdoArgs c1, int nq1, int var) {
  __shared__ __align__(16) uint8_t lds[QuadLds<Px>::kBytes];
  __shared__ uint16_t scan[1024];
  if ((int)blockIdx.x < g0)
    rdo_quad_wg<Px, 0>(l0, c0, nq0, var, blockIdx.x, lds, scan);
  else
    rdo_quad_wg<Px, 1>(l1, c1, nq1, var, blockIdx.x - g0, lds, scan);
}

// List-driven score launches (the compacted candidate lists of round 0 and of
// every MV-stack round): a pool of workgroups walks the live work only.  The
// device counts give the live luma quads and chroma triples of set A (MODE
// MA) and, when nsets == 2, of set B (MODE MB), laid out back to back:
//   [A luma quads | A chroma triples | B luma quads | B chroma triples]
// so a round of a few dozen superblocks launches a pool, not the frame's full
// grid of early exits (66 k waves per launch at 2160p: the ~60 us dispatch
// floor of the round-5 trace).  Chroma pairs are indexed by the live count
// (pairs per plane = ceil(count / 2)), which keeps them contiguous.
//
// The arguments [la, ca, lb, cb] come from device memory (rdo_args_store_kernel,
// once per frame): by value or bound to the kernel's parameters, a loop over
// the inlined bodies copies them to scratch.  The bodies read the work-item
// id through rv_tid(), so the loop does not hoist (and spill) their lane
// addresses either: 52 B of scratch per lane instead of ~2 KB.
template <typename Px, int MA, int MB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void rdo_quad_list_kernel(
    const RdoArgs *__restrict__ A, int nsets, int var, uint32_t *kp_cnt, unsigned long long *kp_t) {
  __shared__ __align__(16) uint8_t lds[QuadLds<Px>::kBytes];
  __shared__ uint16_t scan[1024];
  if (kp_t && threadIdx.x == 0) atomicMin(kp_t, (unsigned long long)wall_clock64());
  const RdoArgs &la = A[0], &ca = A[1], &lb = A[2], &cb = A[3];
  const int na = rdo_ntx(la), ma = rdo_ntx(ca);
  const int nb = nsets > 1 ? rdo_ntx(lb) : 0, mb = nsets > 1 ? rdo_ntx(cb) : 0;
  if (kp_cnt && blockIdx.x == 0 && threadIdx.x == 0) {  // the launch's units, once
    atomicAdd(kp_cnt + (MA ? 1 : 0), (uint32_t)na);
    atomicAdd(kp_cnt + (MA ? 3 : 2), (uint32_t)ma);
    if (nsets > 1) {
      atomicAdd(kp_cnt + (MB ? 1 : 0), (uint32_t)nb);
      atomicAdd(kp_cnt + (MB ? 3 : 2), (uint32_t)mb);
    }
  }
  const int pa = (ma + 1) / 2, pb = (mb + 1) / 2;
  const bool c4 = (var & 32) != 0;  // chroma: a block per wavefront (rounds)
  const int e0 = (na + 3) / 4, e1 = e0 + (c4 ? (2 * ma + 3) / 4 : (2 * pa + 2) / 3);
  const int e2 = e1 + (nb + 3) / 4, e3 = e2 + (c4 ? (2 * mb + 3) / 4 : (2 * pb + 2) / 3);
  const bool phd = RV_RDO_PHASES && (var & 16) && rv_tid() == 0;
  for (int b = blockIdx.x; b < e3; b += gridDim.x) {
    QuadPh ph;
    ph.t[0] = phd ? wall_clock64() : 0;
    QuadPh *pp = phd ? &ph : nullptr;
    int set = 2;
    if (b < e0) {
      stage_scan(scan, la.q_tx_index);
      rdo_quad_luma<Px, MA>(la, b, na, var, lds, scan, pp);
      set = MA;
    } else if (b < e1) {
      stage_scan(scan, ca.q_tx_index);
      if (c4)
        rdo_quad_chroma4<Px, MA>(ca, b - e0, ma, lds, scan);
      else
        rdo_quad_chroma<Px, MA>(ca, b - e0, pa, lds, scan);
    } else if (b < e2) {
      stage_scan(scan, lb.q_tx_index);
      rdo_quad_luma<Px, MB>(lb, b - e1, nb, var, lds, scan, pp);
      set = MB;
    } else {
      stage_scan(scan, cb.q_tx_index);
      if (c4)
        rdo_quad_chroma4<Px, MB>(cb, b - e2, mb, lds, scan);
      else
        rdo_quad_chroma<Px, MB>(cb, b - e2, pb, lds, scan);
    }
    __syncthreads();  // the slots and the scan are reused by the next item
    if (phd) {
      const unsigned long long te = wall_clock64();
      if (set < 2) {
        for (int k = 0; k < 4; k++) atomicAdd(&g_rdo_ph[set][k], ph.t[k + 1] - ph.t[k]);
        atomicAdd(&g_rdo_ph[set][4], te - ph.t[4]);
      } else {
        atomicAdd(&g_rdo_ph[2][0], te - ph.t[0]);
      }
      atomicAdd(&g_rdo_ph[set][5], 1ull);
    }
  }
  if (kp_t && threadIdx.x == 0) atomicMax(kp_t + 1, (unsigned long long)wall_clock64());
}

// Kernel arguments -> device memory (they are captured at launch, so the
// host's copies need not outlive the call).
__global__ __launch_bounds__(256) void rdo_args_store_kernel(RdoArgs a0, RdoArgs a1, RdoArgs a2,
                                                              RdoArgs a3, int n, RdoArgs *out) {
  static_assert(sizeof(RdoArgs) % 4 == 0, "word copy");
  constexpr int W = (int)(sizeof(RdoArgs) / 4);
  for (int i = threadIdx.x; i < n * W; i += blockDim.x) {
    const int k = i / W, w = i - k * W;
    const RdoArgs *s = k == 0 ? &a0 : k == 1 ? &a1 : k == 2 ? &a2 : &a3;
    uint32_t v;
    __builtin_memcpy(&v, reinterpret_cast<const uint8_t *>(s) + 4 * w, 4);
    __builtin_memcpy(reinterpret_cast<uint8_t *>(out + k) + 4 * w, &v, 4);
  }
}

// The pool of a list-driven launch: RAV1E_HIP_F4_POOL workgroups (default
// 1024, four per CU: the LDS of QuadLds allows four), never more than the
// full grid.
static int rdo_f4_pool() {
  static const int pool = [] {
    const char *e = getenv("RAV1E_HIP_F4_POOL");
    const int v = e ? atoi(e) : 1024;
    return v > 0 ? v : 1024;
  }();
  return pool;
}

}  // namespace rv

using namespace rv;

// Blocks below 64x64 (the speed-6 partition search): N x N transform
// blocks, N lanes each (64 / N per wavefront, four wavefronts per
// workgroup); the launch's tasks cover plane p[0] then p[1] (chroma).
template <typename Px, int N, int MODE, bool LUMA>
__global__ __launch_bounds__(256) void rdo_small_kernel(RdoArgs a, int nplanes) {
  constexpr int TPW = 64 / N;
  constexpr int SLAB = rdo_slab_bytes<Px, N>();
  constexpr int PER = (SLAB + N * N * (int)sizeof(Px) + 15) / 16 * 16;
  __shared__ __align__(16) uint8_t lds[4 * TPW * PER];
  __shared__ uint16_t scan[1024];
  stage_scan(scan, a.q_tx_index);
  const int wave = rv_tid() >> 6, g = (rv_tid() & 63) / N;
  const int n = rdo_ntx(a), total = n * nplanes;
  const int w0 = (blockIdx.x * 4 + wave) * TPW;
  if (w0 >= total) return;  // the whole wavefront is past the tasks
  const int i = w0 + g;
  const bool valid = i < total;
  const int ii = valid ? i : total - 1;  // recomputed, nothing stored
  const int plane = ii / n, t = ii - plane * n;
  uint8_t *mine = lds + (wave * TPW + g) * PER;
  rdo_cand_body<Px, N, N, MODE, LUMA>(a, a.p[plane], t, valid, reinterpret_cast<int32_t *>(mine),
                                       reinterpret_cast<Px *>(mine + SLAB), scan);
}

// One launch for a level's luma blocks (NL, plane p[0]) and both chroma
// planes' blocks (NC): workgroups below lgrid run the luma tasks, the rest
// the chroma ones (the partition levels' chain is launch-latency bound).
template <typename Px, int N, int MODE, bool LUMA>
__device__ __forceinline__ void rdo_small_part(const RdoArgs &a, int nplanes, int blk,
                                               uint8_t *lds, uint16_t *scan) {
  constexpr int TPW = 64 / N;
  constexpr int SLAB = rdo_slab_bytes<Px, N>();
  constexpr int PER = (SLAB + N * N * (int)sizeof(Px) + 15) / 16 * 16;
  stage_scan(scan, a.q_tx_index);
  const int wave = rv_tid() >> 6, g = (rv_tid() & 63) / N;
  const int n = rdo_ntx(a), total = n * nplanes;
  const int w0 = (blk * 4 + wave) * TPW;
  if (w0 >= total) return;
  const int i = w0 + g;
  const bool valid = i < total;
  const int ii = valid ? i : total - 1;
  const int plane = ii / n, t = ii - plane * n;
  uint8_t *mine = lds + (wave * TPW + g) * PER;
  rdo_cand_body<Px, N, N, MODE, LUMA>(a, a.p[plane], t, valid, reinterpret_cast<int32_t *>(mine),
                                       reinterpret_cast<Px *>(mine + SLAB), scan);
}

template <typename Px, int N>
constexpr int rdo_small_lds() {
  return 4 * (64 / N) * ((rdo_slab_bytes<Px, N>() + N * N * (int)sizeof(Px) + 15) / 16 * 16);
}

template <typename Px, int NL, int NC, int MODE>
__global__ __launch_bounds__(256) void rdo_small2_kernel(RdoArgs l, RdoArgs c, int lgrid) {
  constexpr int BL = rdo_small_lds<Px, NL>(), BC = rdo_small_lds<Px, NC>();
  __shared__ __align__(16) uint8_t lds[BL > BC ? BL : BC];
  __shared__ uint16_t scan[1024];
  if ((int)blockIdx.x < lgrid)
    rdo_small_part<Px, NL, MODE, true>(l, 1, blockIdx.x, lds, scan);
  else
    rdo_small_part<Px, NC, MODE, false>(c, 2, blockIdx.x - lgrid, lds, scan);
}

template <int NL, int NC>
static void rdo_small2_launch(const RdoArgs &l, const RdoArgs &c, int hbd, hipStream_t s,
                              int mode) {
  const int lg = (l.n_tx + 4 * (64 / NL) - 1) / (4 * (64 / NL));
  const int cg = (c.n_tx * 2 + 4 * (64 / NC) - 1) / (4 * (64 / NC));
  const unsigned grid = (unsigned)(lg + cg);
  if (grid == 0) return;
#define RV_SMALL2(PX, M) rdo_small2_kernel<PX, NL, NC, M><<<grid, 256, 0, s>>>(l, c, lg)
  if (hbd) {
    if (mode == 0) RV_SMALL2(uint16_t, 0); else if (mode == 1) RV_SMALL2(uint16_t, 1); else RV_SMALL2(uint16_t, 2);
  } else {
    if (mode == 0) RV_SMALL2(uint8_t, 0); else if (mode == 1) RV_SMALL2(uint8_t, 1); else RV_SMALL2(uint8_t, 2);
  }
#undef RV_SMALL2
}

template <int N, bool LUMA>
static void rdo_small_launch(const RdoArgs &a, int nplanes, int hbd, hipStream_t s, int mode) {
  constexpr int TPW = 64 / N;
  const unsigned grid = (unsigned)((a.n_tx * nplanes + 4 * TPW - 1) / (4 * TPW));
  if (grid == 0) return;
#define RV_SMALL(PX, M) rdo_small_kernel<PX, N, M, LUMA><<<grid, 256, 0, s>>>(a, nplanes)
  if (hbd) {
    if (mode == 0) RV_SMALL(uint16_t, 0); else if (mode == 1) RV_SMALL(uint16_t, 1); else RV_SMALL(uint16_t, 2);
  } else {
    if (mode == 0) RV_SMALL(uint8_t, 0); else if (mode == 1) RV_SMALL(uint8_t, 1); else RV_SMALL(uint8_t, 2);
  }
#undef RV_SMALL
}

template <int MODE>
static void rdo_launch(const RdoArgs &luma, const RdoArgs &chroma, int hbd, hipStream_t s,
                       bool single, unsigned cpairs) {
  // default 3: both (measured at 2160p: 880 vs 850 frames/s, r03g)
  static const int var = [] {
    const char *e = getenv("RAV1E_HIP_RDO_VARIANT");
    return e ? atoi(e) : 3;
  }();
  if (luma.bd == 12 || single) {  // 12-bit: i32 row-pass intermediate
    const unsigned grid = (unsigned)luma.n_tx + cpairs;
    if (grid == 0) return;
    if (hbd)
      rdo_frame_kernel<uint16_t, MODE><<<grid, 64, 0, s>>>(luma, chroma);
    else
      rdo_frame_kernel<uint8_t, MODE><<<grid, 64, 0, s>>>(luma, chroma);
    return;
  }
  const int nquads = (luma.n_tx + 3) / 4;
  const unsigned grid = (unsigned)nquads + (cpairs + 2) / 3;
  if (grid == 0) return;
  if (hbd)
    rdo_quad_kernel<uint16_t, MODE><<<grid, 256, 0, s>>>(luma, chroma, nquads, var);
  else
    rdo_quad_kernel<uint8_t, MODE><<<grid, 256, 0, s>>>(luma, chroma, nquads, var);
}

// Replay-internal entry (rv_replay.hip): luma (N = 64, cdef distortion)
// and both chroma planes (N = 32, SSE) of every task, one launch on `s`.
// compound: the tasks are compound candidates (score launches only).
int rv_rdo_candidates(const RdoArgs &luma, const RdoArgs &chroma, int hbd, hipStream_t s,
                      bool compound) {
  const unsigned cpairs = (unsigned)(2 * ((chroma.n_tx + 1) / 2));
  // RAV1E_HIP_RDO_SINGLE=1: one candidate per workgroup at every bit depth
  static const bool single = [] {
    const char *e = getenv("RAV1E_HIP_RDO_SINGLE");
    return e && e[0] == '1';
  }();
  if (luma.commit)
    rdo_launch<2>(luma, chroma, hbd, s, single, cpairs);
  else if (compound)
    rdo_launch<1>(luma, chroma, hbd, s, single, cpairs);
  else
    rdo_launch<0>(luma, chroma, hbd, s, single, cpairs);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

// The single-reference and the compound candidates in one launch
// (rdo_quad_pair_kernel); the 12-bit and RAV1E_HIP_RDO_SINGLE paths launch
// them one after the other.
int rv_rdo_candidates_pair(const RdoArgs &l0, const RdoArgs &c0, const RdoArgs &l1,
                           const RdoArgs &c1, int hbd, hipStream_t s) {
  static const bool single = [] {
    const char *e = getenv("RAV1E_HIP_RDO_SINGLE");
    return e && e[0] == '1';
  }();
  if (l0.bd == 12 || single || l0.commit) {
    const int rc = rv_rdo_candidates(l0, c0, hbd, s, false);
    return rc != RV_OK ? rc : rv_rdo_candidates(l1, c1, hbd, s, true);
  }
  static const int var = [] {
    const char *e = getenv("RAV1E_HIP_RDO_VARIANT");
    return e ? atoi(e) : 3;
  }();
  const unsigned cp0 = (unsigned)(2 * ((c0.n_tx + 1) / 2)), cp1 = (unsigned)(2 * ((c1.n_tx + 1) / 2));
  const int nq0 = (l0.n_tx + 3) / 4, nq1 = (l1.n_tx + 3) / 4;
  const unsigned g0 = (unsigned)nq0 + (cp0 + 2) / 3, g1 = (unsigned)nq1 + (cp1 + 2) / 3;
  if (g0 + g1 == 0) return RV_OK;
  if (hbd)
    rdo_quad_pair_kernel<uint16_t><<<g0 + g1, 256, 0, s>>>(l0, c0, nq0, (int)g0, l1, c1, nq1, var);
  else
    rdo_quad_pair_kernel<uint8_t><<<g0 + g1, 256, 0, s>>>(l0, c0, nq0, (int)g0, l1, c1, nq1, var);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

int rv_rdo_args_put(const RdoArgs *h, int n, RdoArgs *dev, hipStream_t s) {
  if (!h || !dev || n < 1 || n > 4) return rv_set_error(RV_EINVAL, "rv_rdo_args_put: bad arguments");
  rdo_args_store_kernel<<<1, 256, 0, s>>>(h[0], h[n > 1 ? 1 : 0], h[n > 2 ? 2 : 0], h[n > 3 ? 3 : 0],
                                          n, dev);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

int rv_rdo_candidates_list(const RdoArgs *h, const RdoArgs *dev, int nsets, int mode_a, int hbd,
                           hipStream_t s, int max_grid, uint32_t *kp_cnt, unsigned long long *kp_t) {
  if (!h || !dev || nsets < 1 || nsets > 2 || mode_a < 0 || mode_a > 1 || (nsets == 2 && mode_a) ||
      h[0].commit || h[0].bd == 12)
    return rv_set_error(RV_EINVAL, "rv_rdo_candidates_list: bad arguments");
  for (int k = 0; k < 2 * nsets; k++)
    if (!h[k].list || !h[k].count)
      return rv_set_error(RV_EINVAL, "rv_rdo_candidates_list: the sets must be list-driven");
  static const int var0 = [] {
    const char *e = getenv("RAV1E_HIP_RDO_VARIANT");
    return e ? atoi(e) : 3;
  }();
  static const bool phases = getenv("RAV1E_HIP_RDO_PHASES") && getenv("RAV1E_HIP_RDO_PHASES")[0] == '1';
  // RAV1E_HIP_F4_CHROMA4=0: the rounds' chroma two blocks per wavefront (A/B)
  static const bool chroma4 = !(getenv("RAV1E_HIP_F4_CHROMA4") && getenv("RAV1E_HIP_F4_CHROMA4")[0] == '0');
  const int var = var0 | (phases && max_grid > 0 ? 16 : 0) | (chroma4 && max_grid > 0 ? 32 : 0);
  // the full grid (every listed slot live) bounds the pool
  unsigned full = 0;
  for (int k = 0; k < nsets; k++)
    full += (unsigned)((h[2 * k].n_tx + 3) / 4) +
            ((var & 32) ? (unsigned)(2 * h[2 * k + 1].n_tx + 3) / 4
                        : (unsigned)(2 * ((h[2 * k + 1].n_tx + 1) / 2) + 2) / 3);
  unsigned grid = std::min(full, (unsigned)rdo_f4_pool());
  if (max_grid > 0) grid = std::min(grid, (unsigned)max_grid);
  if (grid == 0) return RV_OK;
#define RV_LIST(PX, MA, MB) \
  rdo_quad_list_kernel<PX, MA, MB><<<grid, 256, 0, s>>>(dev, nsets, var, kp_cnt, kp_t)
  if (hbd) {
    if (nsets == 2) RV_LIST(uint16_t, 0, 1); else if (mode_a) RV_LIST(uint16_t, 1, 1); else RV_LIST(uint16_t, 0, 0);
  } else {
    if (nsets == 2) RV_LIST(uint8_t, 0, 1); else if (mode_a) RV_LIST(uint8_t, 1, 1); else RV_LIST(uint8_t, 0, 0);
  }
#undef RV_LIST
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

int rv_rdo_intra(const RdoArgs &luma, const RdoArgs &chroma, int hbd, hipStream_t s) {
  const unsigned cpairs = (unsigned)(2 * ((chroma.n_tx + 1) / 2));
  rdo_launch<3>(luma, chroma, hbd, s, false, cpairs);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

// The speed-6 levels: luma N x N (N = 32, 16, 8; cdef distortion) or the
// chroma planes' transform blocks (N = 16, 8, 4 in 4:2:0; SSE) of every task.
int rv_rdo_blocks2(const RdoArgs &l, const RdoArgs &c, int nl, int nc, int hbd, hipStream_t s,
                   int mode) {
  if (nl == 32 && nc == 16) rdo_small2_launch<32, 16>(l, c, hbd, s, mode);
  else if (nl == 16 && nc == 8) rdo_small2_launch<16, 8>(l, c, hbd, s, mode);
  else if (nl == 8 && nc == 4) rdo_small2_launch<8, 4>(l, c, hbd, s, mode);
  else if (nl == 32 && nc == 32) rdo_small2_launch<32, 32>(l, c, hbd, s, mode);
  else if (nl == 16 && nc == 16) rdo_small2_launch<16, 16>(l, c, hbd, s, mode);
  else if (nl == 8 && nc == 8) rdo_small2_launch<8, 8>(l, c, hbd, s, mode);
  else return rv_set_error(RV_EINVAL, "rv_rdo_blocks2: sizes");
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

int rv_rdo_blocks(const RdoArgs &a, bool luma, int nplanes, int n_tx_size, int hbd,
                  hipStream_t s, int mode) {
  if (luma) {
    if (n_tx_size == 32) rdo_small_launch<32, true>(a, nplanes, hbd, s, mode);
    else if (n_tx_size == 16) rdo_small_launch<16, true>(a, nplanes, hbd, s, mode);
    else if (n_tx_size == 8) rdo_small_launch<8, true>(a, nplanes, hbd, s, mode);
    else return rv_set_error(RV_EINVAL, "rv_rdo_blocks: luma size");
  } else {
    if (n_tx_size == 32) rdo_small_launch<32, false>(a, nplanes, hbd, s, mode);
    else if (n_tx_size == 16) rdo_small_launch<16, false>(a, nplanes, hbd, s, mode);
    else if (n_tx_size == 8) rdo_small_launch<8, false>(a, nplanes, hbd, s, mode);
    else if (n_tx_size == 4) rdo_small_launch<4, false>(a, nplanes, hbd, s, mode);
    else return rv_set_error(RV_EINVAL, "rv_rdo_blocks: chroma size");
  }
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

// RAV1E_HIP_RDO_PHASES=1: print the MV-stack rounds' F4 item phases
// (g_rdo_ph, microseconds per item) to stderr and clear them
extern "C" int rv_rdo_phase_dump(void) {
  unsigned long long h[3][8];
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpyFromSymbol(h, HIP_SYMBOL(g_rdo_ph), sizeof(h)) != hipSuccess)
    return rv_set_error(RV_EHIP, "rv_rdo_phase_dump");
  const double us = 0.01;  // wall_clock64: 100 MHz
  static const char *kName[2] = {"single", "compound"};
  for (int m = 0; m < 2; m++) {
    const double n = h[m][5] ? (double)h[m][5] : 1.0;
    fprintf(stderr,
            "[f4 phases] %s luma quads %llu: front %.2f, row DCT %.2f, quantize %.2f, inverse rows %.2f, "
            "back %.2f us per quad\n",
            kName[m], h[m][5], h[m][0] * us / n, h[m][1] * us / n, h[m][2] * us / n, h[m][3] * us / n,
            h[m][4] * us / n);
  }
  fprintf(stderr, "[f4 phases] chroma triples %llu: %.2f us each\n", h[2][5],
          h[2][0] * us / (h[2][5] ? (double)h[2][5] : 1.0));
  memset(h, 0, sizeof(h));
  return hipMemcpyToSymbol(HIP_SYMBOL(g_rdo_ph), h, sizeof(h)) == hipSuccess ? RV_OK
                                                                           : rv_set_error(RV_EHIP, "rv_rdo_phase_dump");
}
