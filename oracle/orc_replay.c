/* CPU replay of the hot-path schedule (test infrastructure + the
 * bench's cpu_baseline leg only; see DESIGN.md "Replay driver").
 *
 * Runs the same per-frame schedule as rav1e_amd/csrc/rv_replay.hip with the
 * oracle's restatements of the reference functions, one superblock per
 * task on a pthread pool (rav1e runs tiles on rayon, src/encoder.rs:
 * 2772-2781; within one tile the replay's superblocks are independent):
 *   F0 downsample_from (src/frame/plane.rs:399-423)
 *   F1 full_search at 1/4 res (estimate_motion_ss4, src/me.rs:1023-1075)
 *   F2 diamond at 1/2 res (me_ss2, src/me.rs:470-519)
 *   F3 diamond full-pel + sub-pel at full res (src/me.rs:193-285)
 *   F4 put_8tap, diff + fht, quantize + dequantize, inverse + add,
 *      cdef moments / sse (src/encoder.rs:1077-1237, src/rdo.rs:219-411)
 *   F5 8x8 SATD importance (src/api/internal.rs:823-1010) + lookahead
 *      intra cost of the same blocks (:680-765, orc_lookahead_intra_costs)
 * It must produce the same result words as the GPU driver.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "orc_common.h"

#define SB 64
#define QIDX 100 /* kReplayQindex of rv_replay.hip */

typedef struct {
  uint8_t *mem; /* allocation, element 0 */
  int stride, alloc_h, w, h, xo, yo, xdec, ydec;
} oplane;

typedef struct {
  oplane y, u, v, hres, qres;
} oslot;

typedef struct orc_replay {
  int W, H, xdec, ydec, bd, hbd, R, C;
  int w_in_b, h_in_b, tx0, ty0, tw, th, mi_w, mi_h, nsb, cw, ch, vis_w, vis_h;
  double me_lambda;
  orc_qctx q_luma, q_chroma; /* TX_64X64 / TX_32X32, inter, qindex QIDX */
  oslot *slots;
  int threads;
  /* per frame */
  int scale;
  uint64_t *words;
  uint64_t tail[4];
  pthread_mutex_t mu;
  int next_sb;
} orc_replay;

static size_t px_of(const orc_replay *r) { return r->hbd ? 2 : 1; }

static int plane_init(oplane *p, int w, int h, int xdec, int ydec, int pad,
                      int hbd) {
  int out[4];
  orc_plane_geometry(w, h, pad >> xdec, pad >> ydec, hbd, out);
  p->stride = out[0];
  p->alloc_h = out[1];
  p->xo = out[2];
  p->yo = out[3];
  p->w = w;
  p->h = h;
  p->xdec = xdec;
  p->ydec = ydec;
  p->mem = calloc((size_t)p->stride * p->alloc_h, hbd ? 2 : 1);
  return p->mem ? 0 : -1;
}
/* data origin (visible (0,0)) */
static void *org_of(const oplane *p, int hbd) {
  return p->mem + ((size_t)p->yo * p->stride + p->xo) * (hbd ? 2 : 1);
}
static void *at(const oplane *p, int hbd, int x, int y) {
  return (uint8_t *)org_of(p, hbd) +
         ((ptrdiff_t)y * p->stride + x) * (ptrdiff_t)(hbd ? 2 : 1);
}

static void mv_range(const orc_replay *r, int bx, int by, int bw, int bh,
                     int m[4]) {
  int border_w = 128 + bw * 8, border_h = 128 + bh * 8;
  m[0] = -bx * 32 - border_w;
  m[1] = (r->w_in_b - bx - bw / 4) * 32 + border_w;
  m[2] = -by * 32 - border_h;
  m[3] = (r->h_in_b - by - bh / 4) * 32 + border_h;
}
static void adjust_bo(const orc_replay *r, int *bx, int *by, int bw, int bh) {
  int x = *bx < r->mi_w - bw / 4 ? *bx : r->mi_w - bw / 4;
  int y = *by < r->mi_h - bh / 4 ? *by : r->mi_h - bh / 4;
  *bx = x > 0 ? x : 0;
  *by = y > 0 ? y : 0;
}
static uint64_t pack_mv(orc_mv m) {
  return ((uint64_t)(uint16_t)m.row << 16) | (uint16_t)m.col;
}
static orc_mv qfull(orc_mv m) {
  orc_mv q = {(int16_t)((m.row / 8) * 8), (int16_t)((m.col / 8) * 8)};
  return q;
}

orc_replay *orc_replay_create(int W, int H, int xdec, int ydec, int bd,
                              int tile_x0, int tile_y0, int tile_w,
                              int tile_h, int n_refs, int threads) {
  if ((W & 7) || (H & 7) || (bd != 8 && bd != 10 && bd != 12) || n_refs < 1 || n_refs > 7)
    return NULL;
  orc_replay *r = calloc(1, sizeof(*r));
  r->W = W;
  r->H = H;
  r->xdec = xdec;
  r->ydec = ydec;
  r->bd = bd;
  r->hbd = bd > 8;
  r->R = n_refs;
  r->C = 2 * n_refs;
  r->w_in_b = 2 * ((W + 7) >> 3);
  r->h_in_b = 2 * ((H + 7) >> 3);
  int sbc = (W + SB - 1) / SB, sbr = (H + SB - 1) / SB;
  r->tx0 = tile_x0;
  r->ty0 = tile_y0;
  r->tw = tile_w > 0 ? tile_w : sbc - tile_x0;
  r->th = tile_h > 0 ? tile_h : sbr - tile_y0;
  r->vis_w = W - r->tx0 * SB < r->tw * SB ? W - r->tx0 * SB : r->tw * SB;
  r->vis_h = H - r->ty0 * SB < r->th * SB ? H - r->ty0 * SB : r->th * SB;
  r->mi_w = r->vis_w >> 2;
  r->mi_h = r->vis_h >> 2;
  r->nsb = r->tw * r->th;
  r->cw = SB >> xdec;
  r->ch = SB >> ydec;
  r->me_lambda = 24.0 * (double)(1 << (bd - 8));
  orc_qctx_update(&r->q_luma, QIDX, 4, 0, bd, 0, 0);
  orc_qctx_update(&r->q_chroma, QIDX, 3, 0, bd, 0, 0);
  r->threads = threads > 0 ? threads : 1;
  r->slots = calloc(n_refs + 1, sizeof(oslot));
  int cw = (W + xdec) >> xdec, ch = (H + ydec) >> ydec;
  for (int s = 0; s <= n_refs; s++) {
    oslot *o = &r->slots[s];
    if (plane_init(&o->y, W, H, 0, 0, 88, r->hbd) ||
        plane_init(&o->u, cw, ch, xdec, ydec, 88, r->hbd) ||
        plane_init(&o->v, cw, ch, xdec, ydec, 88, r->hbd) ||
        plane_init(&o->hres, W / 2, H / 2, 0, 0, 44, r->hbd) ||
        plane_init(&o->qres, W / 4, H / 4, 0, 0, 22, r->hbd))
      return NULL;
  }
  r->words = calloc((size_t)r->nsb * (8 * r->R + 2), 8);
  pthread_mutex_init(&r->mu, NULL);
  return r;
}

void orc_replay_destroy(orc_replay *r) {
  if (!r) return;
  for (int s = 0; s <= r->R; s++) {
    oslot *o = &r->slots[s];
    free(o->y.mem);
    free(o->u.mem);
    free(o->v.mem);
    free(o->hres.mem);
    free(o->qres.mem);
  }
  free(r->slots);
  free(r->words);
  pthread_mutex_destroy(&r->mu);
  free(r);
}

static void pad(const orc_replay *r, oplane *p) {
  orc_plane_pad(p->mem, p->stride, p->alloc_h, p->xo, p->yo, 0, 0, p->w, p->h,
                r->hbd);
}
static void downsample(const orc_replay *r, oplane *dst, const oplane *src) {
  orc_downsample(org_of(dst, r->hbd), dst->stride, dst->w, dst->h,
                 org_of(src, r->hbd), src->stride, r->hbd);
  pad(r, dst);
}

int orc_replay_set_frame(orc_replay *r, int slot, const void *yuv) {
  if (slot < 0 || slot > r->R) return -1;
  oslot *o = &r->slots[slot];
  size_t px = px_of(r);
  const uint8_t *p = yuv;
  oplane *pl[3] = {&o->y, &o->u, &o->v};
  for (int k = 0; k < 3; k++) {
    for (int y = 0; y < pl[k]->h; y++)
      memcpy(at(pl[k], r->hbd, 0, y), p + (size_t)y * pl[k]->w * px,
             (size_t)pl[k]->w * px);
    p += (size_t)pl[k]->w * pl[k]->h * px;
    pad(r, pl[k]);
  }
  downsample(r, &o->hres, &o->y);
  downsample(r, &o->qres, &o->hres);
  return 0;
}

/* predict_inter / get_params (src/predict.rs:267-283) + put_8tap */
static void predict(const orc_replay *r, const oplane *ref, int po_x, int po_y,
                    orc_mv mv, int w, int h, void *dst, int dst_stride) {
  int ys = 3 + ref->ydec, xs = 3 + ref->xdec;
  int roff = (int)mv.row >> ys, coff = (int)mv.col >> xs;
  int rf = ((int)mv.row - (roff << ys)) << (4 - ys);
  int cf = ((int)mv.col - (coff << xs)) << (4 - xs);
  int qx = clamp_i32(po_x + coff - 3, -ref->xo, ref->w) + 3;
  int qy = clamp_i32(po_y + roff - 3, -ref->yo, ref->h) + 3;
  orc_put_8tap(dst, dst_stride, at(ref, r->hbd, qx, qy), ref->stride, w, h, cf,
               rf, 0, 0, r->bd, r->hbd, 0);
}

static void ds_ctx(const orc_replay *r, orc_ds_ctx *c, const oplane *org,
                   const oplane *ref, int po_x, int po_y, int w, int h,
                   const int m[4], uint32_t lambda, int subpel) {
  memset(c, 0, sizeof(*c));
  c->org = org_of(org, r->hbd);
  c->org_stride = org->stride;
  c->ref = org_of(ref, r->hbd);
  c->ref_stride = ref->stride;
  c->ref_width = ref->w;
  c->ref_height = ref->h;
  c->ref_xorigin = ref->xo;
  c->ref_yorigin = ref->yo;
  c->ref_xdec = ref->xdec;
  c->ref_ydec = ref->ydec;
  c->hbd = r->hbd;
  c->bit_depth = r->bd;
  c->po_x = po_x;
  c->po_y = po_y;
  c->w = w;
  c->h = h;
  c->mvx_min = m[0];
  c->mvx_max = m[1];
  c->mvy_min = m[2];
  c->mvy_max = m[3];
  c->lambda = lambda;
  c->subpel = subpel;
}

/* One superblock through F1..F5; returns its tail contributions. */
static void run_sb(orc_replay *r, int sb, uint64_t tail[3]) {
  const oslot *cur = &r->slots[0];
  const int R = r->R, hbd = r->hbd;
  const int sx = sb % r->tw, sy = sb / r->tw;
  uint64_t *w = r->words + (size_t)sb * (8 * R + 2);
  orc_mv cmv[8], hmv, fmv, smv[8];
  uint64_t cost;
  /* F1 */
  int bx = sx * 16, by = sy * 16;
  adjust_bo(r, &bx, &by, 64, 64);
  int fbx = bx + r->tx0 * 16, fby = by + r->ty0 * 16;
  int m[4];
  mv_range(r, fbx, fby, 64, 64, m);
  uint32_t lambda4 = (uint32_t)(r->me_lambda * 256.0 / 16.0 * 0.125);
  uint32_t lambda2 = (uint32_t)(r->me_lambda * 256.0 / 4.0 * 0.125);
  uint32_t lambda1 = (uint32_t)(r->me_lambda * 256.0 * 0.5);
  int rx = 192 * r->scale, ry = 64 * r->scale;
  int x_lo = fbx + ((m[0] / 8 > -rx ? m[0] / 8 : -rx) >> 2);
  int x_hi = fbx + ((m[1] / 8 < rx ? m[1] / 8 : rx) >> 2);
  int y_lo = fby + ((m[2] / 8 > -ry ? m[2] / 8 : -ry) >> 2);
  int y_hi = fby + ((m[3] / 8 < ry ? m[3] / 8 : ry) >> 2);
  orc_mv zero = {0, 0};
  for (int k = 0; k < R; k++) {
    const oslot *ref = &r->slots[1 + k];
    orc_mv best = {0, 0};
    cost = UINT64_MAX;
    orc_full_search(org_of(&cur->qres, hbd), cur->qres.stride,
                    org_of(&ref->qres, hbd), ref->qres.stride, hbd, fbx, fby,
                    x_lo, x_hi, y_lo, y_hi, 16, 16, 1, lambda4, zero, zero, 0,
                    &best, &cost);
    cmv[k] = best;
    w[8 * k + 0] = pack_mv(best);
    w[8 * k + 1] = cost;
  }
  /* F2 */
  orc_mv preds[8];
  preds[0] = zero;
  for (int k = 0; k < R; k++) {
    orc_mv c4 = {(int16_t)(cmv[k].row * 4), (int16_t)(cmv[k].col * 4)};
    orc_mv q = qfull(c4);
    preds[1 + k].row = (int16_t)(q.row >> 1);
    preds[1 + k].col = (int16_t)(q.col >> 1);
  }
  int m2[4] = {m[0] >> 1, m[1] >> 1, m[2] >> 1, m[3] >> 1};
  int fbx0 = (sx + r->tx0) * 16, fby0 = (sy + r->ty0) * 16;
  int mf[4];
  mv_range(r, fbx0, fby0, 64, 64, mf);
  for (int k = 0; k < R; k++) {
    const oslot *ref = &r->slots[1 + k];
    orc_ds_ctx c;
    ds_ctx(r, &c, &cur->hres, &ref->hres, fbx * 2, fby * 2, 32, 32, m2, lambda2,
           0);
    orc_diamond_search(&c, preds, 1 + R, &hmv, &cost);
    w[8 * k + 2] = pack_mv(hmv);
    w[8 * k + 3] = cost;
    /* F3 */
    orc_mv fp[2] = {zero, qfull((orc_mv){(int16_t)(hmv.row * 2),
                                         (int16_t)(hmv.col * 2)})};
    ds_ctx(r, &c, &cur->y, &ref->y, fbx0 * 4, fby0 * 4, 64, 64, mf, lambda1, 0);
    orc_diamond_search(&c, fp, 2, &fmv, &cost);
    w[8 * k + 4] = pack_mv(fmv);
    w[8 * k + 5] = cost;
    c.subpel = 1;
    orc_diamond_search(&c, &fmv, 1, &smv[k], &cost);
    w[8 * k + 6] = pack_mv(smv[k]);
    w[8 * k + 7] = cost;
  }
  /* F4 */
  const int px = (sx + r->tx0) * SB, py = (sy + r->ty0) * SB;
  const int cwid = r->cw, chei = r->ch;
  const int cpx = px >> r->xdec, cpy = py >> r->ydec;
  uint64_t best_s = UINT64_MAX;
  int best_c = 0;
  uint16_t ly[SB * SB], lu[SB * SB], lv[SB * SB];
  int16_t res[SB * SB];
  int32_t co[SB * SB], qc[32 * 32], pk[32 * 32];
  for (int c = 0; c < r->C; c++) {
    const oslot *ref = &r->slots[1 + (c >> 1)];
    orc_mv mv = (c & 1) ? zero : smv[c >> 1];
    predict(r, &ref->y, px, py, mv, SB, SB, ly, SB);
    predict(r, &ref->u, cpx, cpy, mv, cwid, chei, lu, cwid);
    predict(r, &ref->v, cpx, cpy, mv, cwid, chei, lv, cwid);
    /* luma TX_64X64 DCT_DCT */
    orc_diff(res, at(&cur->y, hbd, px, py), cur->y.stride, ly, SB, SB, SB, hbd);
    orc_fwd_txfm2d(res, co, 4, 0, r->bd);
    /* quantize reads the first coded_tx_area (1024) entries of the
     * W-stride raster (src/encoder.rs:1152-1170; SURVEY.md §0.6 fork
     * quirk); dequantize feeds the inverse (:1192-1208) */
    orc_quantize(&r->q_luma, co, qc, 4, 0);
    for (int i = 0; i < 32 * 32; i++)
      tail[0] += (uint64_t)(int64_t)qc[i] * (uint64_t)(i + 1);
    orc_dequantize(QIDX, qc, pk, 4, r->bd, 0, 0);
    orc_inv_txfm2d_add(pk, ly, SB, 4, 0, r->bd, hbd);
    /* chroma TX_32X32 DCT_DCT blocks */
    uint16_t *cp[2] = {lu, lv};
    const oplane *cs[2] = {&cur->u, &cur->v};
    for (int pl = 0; pl < 2; pl++)
      for (int ty = 0; ty < chei; ty += 32)
        for (int tx = 0; tx < cwid; tx += 32) {
          uint8_t *pb = (uint8_t *)cp[pl] + ((size_t)ty * cwid + tx) * px_of(r);
          orc_diff(res, at(cs[pl], hbd, cpx + tx, cpy + ty), cs[pl]->stride, pb,
                   cwid, 32, 32, hbd);
          orc_fwd_txfm2d(res, co, 3, 0, r->bd);
          orc_quantize(&r->q_chroma, co, qc, 3, 0);
          for (int i = 0; i < 32 * 32; i++)
            tail[0] += (uint64_t)(int64_t)qc[i] * (uint64_t)(i + 1);
          orc_dequantize(QIDX, qc, pk, 3, r->bd, 0, 0);
          orc_inv_txfm2d_add(pk, pb, cwid, 3, 0, r->bd, hbd);
        }
    /* distortion: luma cdef moments (SSE part), chroma sse_wxh */
    uint64_t s = 0;
    for (int j = 0; j < SB; j += 8)
      for (int i = 0; i < SB; i += 8) {
        int64_t mo[5];
        orc_cdef_moments_8x8(at(&cur->y, hbd, px + i, py + j), cur->y.stride,
                             (uint8_t *)ly + ((size_t)j * SB + i) * px_of(r), SB,
                             hbd, mo);
        s += (uint64_t)(mo[3] + mo[2] - 2 * mo[4]);
      }
    uint64_t parts[SB * SB];
    for (int pl = 0; pl < 2; pl++) {
      int n = orc_sse_wxh(at(cs[pl], hbd, cpx, cpy), cs[pl]->stride, cp[pl], cwid,
                          cwid, chei, r->xdec, r->ydec, hbd, parts);
      for (int i = 0; i < n; i++) s += parts[i];
    }
    if (s < best_s) {
      best_s = s;
      best_c = c;
    }
    /* recon checksum over the candidate's blocks */
    for (int i = 0; i < SB * SB; i++) tail[1] += hbd ? ly[i] : ((uint8_t *)ly)[i];
    for (int i = 0; i < cwid * chei; i++)
      tail[1] += hbd ? (uint64_t)lu[i] + lv[i]
                     : (uint64_t)((uint8_t *)lu)[i] + ((uint8_t *)lv)[i];
  }
  w[8 * R] = (uint64_t)best_c;
  w[8 * R + 1] = best_s;
  /* F5: the 8x8 blocks of this superblock inside the tile's visible area */
  for (int j = 0; j < 8; j++)
    for (int i = 0; i < 8; i++) {
      int bxx = sx * 8 + i, byy = sy * 8 + j;
      if (bxx >= r->vis_w / 8 || byy >= r->vis_h / 8) continue;
      int x = r->tx0 * SB + bxx * 8, y = r->ty0 * SB + byy * 8;
      tail[2] += orc_get_satd(at(&cur->y, hbd, x, y), cur->y.stride,
                              at(&r->slots[1].y, hbd, x + ((int)smv[0].col >> 3),
                                 y + ((int)smv[0].row >> 3)),
                              r->slots[1].y.stride, 8, 8, hbd, 0);
      uint32_t ic;
      orc_lookahead_intra_costs(at(&cur->y, hbd, x, y), cur->y.stride, 8, 8, hbd, r->bd, &ic);
      tail[2] += ic;
    }
}

static void *worker(void *arg) {
  orc_replay *r = arg;
  uint64_t tail[3] = {0, 0, 0};
  for (;;) {
    pthread_mutex_lock(&r->mu);
    int sb = r->next_sb++;
    pthread_mutex_unlock(&r->mu);
    if (sb >= r->nsb) break;
    run_sb(r, sb, tail);
  }
  pthread_mutex_lock(&r->mu);
  for (int i = 0; i < 3; i++) r->tail[i] += tail[i];
  pthread_mutex_unlock(&r->mu);
  return NULL;
}

/* One frame; sb_limit > 0 runs only the first sb_limit superblocks (a
 * bounded sample for timing). */
int orc_replay_frame(orc_replay *r, int me_range_scale, int sb_limit) {
  if (me_range_scale != 1 && me_range_scale != 2 && me_range_scale != 4)
    return -1;
  oslot *cur = &r->slots[0];
  downsample(r, &cur->hres, &cur->y);
  downsample(r, &cur->qres, &cur->hres);
  r->scale = me_range_scale;
  memset(r->tail, 0, sizeof(r->tail));
  r->next_sb = 0;
  int nsb = r->nsb;
  if (sb_limit > 0 && sb_limit < nsb) r->nsb = sb_limit;
  pthread_t th[256];
  int nt = r->threads < 256 ? r->threads : 256;
  for (int i = 0; i < nt; i++) pthread_create(&th[i], NULL, worker, r);
  for (int i = 0; i < nt; i++) pthread_join(th[i], NULL);
  r->nsb = nsb;
  r->tail[3] = (uint64_t)(r->vis_w / 8) * (r->vis_h / 8);
  return 0;
}

int orc_replay_results(orc_replay *r, uint64_t *out, int cap) {
  int nw = r->nsb * (8 * r->R + 2);
  if (cap < nw + 4) return -1;
  memcpy(out, r->words, (size_t)nw * 8);
  memcpy(out + nw, r->tail, 4 * 8);
  return nw + 4;
}
