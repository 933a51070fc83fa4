/* CPU replay of the hot-path schedule (test infrastructure + the
 * bench's cpu_baseline leg only; see DESIGN.md "Replay driver").
 *
 * Runs the same stream schedule as rav1e_amd/csrc/rv_replay.hip with the
 * oracle's restatements of the reference functions, on a pthread pool over
 * superblocks (rav1e runs tiles on rayon, src/encoder.rs:2772-2781):
 *   key frame: its input is its reconstruction
 *   F0 downsample_from (src/frame/plane.rs:399-423) of the input
 *   pass A, per superblock:
 *     F1 full_search at 1/4 res (estimate_motion_ss4, src/me.rs:1023-1075)
 *     F2 diamond at 1/2 res (me_ss2, src/me.rs:470-519)
 *     F3 diamond full-pel + sub-pel at full res (src/me.rs:193-285)
 *   pass B, per superblock (needs the neighbours' NEWMVs):
 *     F4 every inter candidate of rdo_mode_decision (src/rdo.rs:825-1006),
 *        skip and non-skip (:649-700): put_8tap, compute_distortion,
 *        diff + fht, quantize, tx-domain distortion + estimate_rate,
 *        dequantize, inverse + add (src/encoder.rs:1077-1237,
 *        src/rdo.rs:204-569); compute_rd_cost and the argmin
 *     F6 the winner's levels and reconstruction into the frame
 *     F5 8x8 SATD importance (src/api/internal.rs:823-1010) + lookahead
 *        intra cost of the same blocks (:680-765)
 *   F7 pad the reconstruction (or export / import the tile group's region)
 * It must produce the same result words as the GPU driver.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "orc_common.h"

#define SB 64
#define NSLOT 12
#define NMODE 4
/* result words per superblock and reference: coarse (mv, cost), the four
 * half-res quadrants (the encode's build_half_res_pmvs), full-pel, sub-pel,
 * the 16 lookahead 16x16 blocks, the lookahead's four half-res quadrants */
#define WPR (2 + 8 + 2 + 2 + 32 + 8)

typedef struct {
  uint8_t *mem; /* allocation, element 0 */
  int stride, alloc_h, w, h, xo, yo, xdec, ydec;
} oplane;

typedef struct {
  oplane y, u, v;
  /* the coded frame's motion field (FrameState::frame_mvs, saved with the
   * reference, src/encoder.rs:3411-3429): [R][h_in_b][w_in_b] 4x4 units */
  orc_mv *fmv;
} oslot;

typedef struct {
  oplane y, u, v;
  /* input_hres / input_qres of the input (FrameState, src/encoder.rs:362-
   * 377; downsample_from + pad): the searches' half / quarter resolution
   * planes of this frame and of every frame that references it */
  oplane hres, qres;
  int pyr; /* the pyramid is current */
} oinput;


typedef struct {
  int display, me_range_scale, level, is_key, ref_display[2], compound;
} orc_frame_info; /* = rv_replay_frame_info */

/* The lookahead of one coded frame (compute_lookahead_motion_vectors +
 * compute_lookahead_intra_costs, src/api/internal.rs:514-765): its F1 /
 * F2L / FL results, and what compute_block_importances reads of it. */
/* The lookahead's references of a coded frame: rav1e's distinct DPB slots
 * of fi.ref_frames (compute_block_importances' unique_indices,
 * src/api/internal.rs:875-882), one search each in
 * compute_lookahead_motion_vectors (build_coarse_pmvs / build_half_res_pmvs /
 * build_full_res_pmvs loop over ALL_INTER_REFS and search each slot once,
 * src/encoder.rs:2732-2738, 3037-3040).  k < R are the encode's references
 * (k = 0 LAST / the backward reference, k = 1 LAST2 on level 0, ALTREF (the
 * forward reference) above); with R = 2 a level > 0 frame adds k = 2,
 * LAST3 = its own slot, i.e. the previous frame of its level (or the key
 * frame, which fills every slot), src/encoder.rs:772-828.  order: the
 * propagation's reference order (mv index order: LAST, LAST2 / LAST3,
 * ALTREF). */
typedef struct {
  int n, disp[3], order[3];
} orc_la_refs;

typedef struct {
  long coded; /* -1: empty */
  orc_frame_info fi;
  orc_la_refs lr;
  orc_mv *coarse, *half_l, *look; /* [RA][nsb] (x4, x16) */
  uint64_t *cc, *hlc, *lc;
  uint32_t *intra; /* lookahead_intra_costs [h_imp][w_imp] */
  orc_mv *mv8;     /* [RA][h_imp][w_imp]: lookahead_mvs[k][2y][2x] */
  uint32_t *inter; /* [RA][h_imp][w_imp]: get_satd against the reference block at mv8 */
  float *imp;      /* block_importances, per output frame */
} ola;

typedef struct orc_replay {
  int W, H, xdec, ydec, bd, hbd, R, C;
  /* RA: the lookahead arrays' references (R = 2: 3, orc_la_refs); la_mode:
   * the lookahead is running (its references are lar.disp[0 .. lar.n)) */
  int RA, la_mode;
  orc_la_refs lar;
  int w_in_b, h_in_b, w_imp, tx0, ty0, tw, th, tws, ths, nsb, cw, ch, vis_w, vis_h, ntx_c;
  /* per pyramid level: quantizers (TX_64X64 luma, TX_32X32 chroma, inter)
   * and lambdas (rv_replay_set_level_params) */
  struct {
    int set, qidx, dc[3], ac[3];
    orc_qctx q[3];
    orc_qctx qi[3]; /* the intra blocks' (is_intra: other rounding offsets) */
    double lambda, me_lambda, ds[3];
  } lv[3];
  oslot slots[NSLOT];
  oinput *inputs;
  int n_inputs;
  /* rdo_lookahead_frames (orc_replay_set_imp_window; 0: the importances are
   * an input, orc_replay_set_importances): the lookahead runs that many
   * coded frames ahead (ring la[W + 1]) and every frame's block importances
   * come from compute_block_importances over the window */
  int imp_window, h_imp;
  /* la_ext: a tile group's window -- the importances need the whole frame's
   * lookahead, so each group computes its own blocks' part
   * (orc_replay_la_group) and the caller exchanges the parts
   * (orc_replay_la_import) before coding; frame() does not run it */
  int la_ext;
  ola *la;
  long la_next;  /* the next coded frame whose lookahead runs */
  long la_limit; /* coded frames in the stream (0: unbounded) */
  float *imp_own; /* the propagated importances of the frame being coded */
  float *imp; /* block_importances, NULL = zero */
  int threads;
  long coded;
  orc_frame_info fi;
  /* per frame */
  orc_mv *coarse, *half, *full, *sub; /* [R][nsb] (half: [R][nsb][4]) */
  orc_mv *look;                        /* lookahead: [R][nsb][16] */
  orc_mv *half_l;                      /* the lookahead's half-res quadrants [R][nsb][4] */
  uint64_t *cc, *hc, *fc, *sc, *lc, *hlc;
  /* the tile motion fields (TileMotionVectors, ts.mvs) of the encode and of
   * the lookahead: [R][th * 16][tw * 16] over the group, 4x4 units */
  orc_mv *tmv_e, *tmv_l;
  uint64_t *words;
  int32_t *lev; /* committed levels: per SB luma 1024 + 2 * ntx_c * 1024 */
  uint64_t tail[5];
  /* the 32x32, 16x16 and 8x8 levels: speed 6 (orc_replay_set_speed) over
   * the whole group; speed 10 over the bounding rectangle of the group's
   * frame-edge superblocks (must_split), in group superblocks (ex0, ey0) +
   * (ew, eh) */
  int s6, lvl, ex0, ey0, ew, eh;
  /* per level: leaves exist (mode decision, commit) / the motion search runs
   * (16x16 and 8x8 seed from the 32x32 searches) */
  int lv_used[4], lv_me[4];
  struct olevel {
    int B, n, gw, gh, bc, bch, txl, txc, tx0, ty0, tws, ths;
    orc_mv *full, *sub; /* [R][n] */
    uint64_t *fc, *sc;
    double *cost;       /* the winners' rd cost */
    int32_t *lev;       /* per block: luma B * B, then U, V bc * bch */
    uint8_t *leaf;      /* committed by the partition decision */
    size_t woff;
  } pl[4];
  orc_qctx qs[3][4][3];
  uint8_t *leaf0;
  size_t nwords, wpart;
  /* speed 10: the superblocks' MV stacks are rav1e's (find_mvrefs over the
   * tile's coded blocks, orc_mvref.c); the block grid of the group (4x4
   * units, pitch tw * 16) and each superblock's stacks (first two entries;
   * n = min(len, 2); the compound stack always holds two) */
  int exact;
  orc_blk *bgrid;
  struct ostk {
    int n[2];
    orc_mv s[2][2];
    orc_mv c[2][2];
  } *stk;
  /* RV_REPLAY_DEBLOCK (orc_replay_set_deblock): the block map, fast levels */
  int deblock, mi_cols, mi_rows;
  uint8_t db_levels[4]; /* the last deblocked frame's levels */
  uint8_t *mi_lg, *mi_skip;
  /* RV_REPLAY_CDEF (orc_replay_set_cdef): (y, uv) strengths per level */
  int cdef;
  uint8_t cdef_str[3][2];
  /* RV_REPLAY_LRF (orc_replay_set_lrf): loop restoration, the frame's unit
   * geometry and each unit's filter (set -1: None) */
  int lrf;
  orc_lrf_plane_cfg lrf_cfg[3];
  orc_lrf_unit *lrf_units[3];
  int lrf_n[3];
  /* intra-mode screening + intra RDO of the non-skip superblocks
   * (orc_replay_set_intra; speed 10, 4:2:0): screened / intra winners this
   * frame */
  int intra;
  uint64_t istat[2];
  /* coefficient entropy coding of every coded frame (orc_replay_set_entropy):
   * the CDFs each pyramid level's next frame starts from (NULL: the key
   * frame's, stood in for by CDFContext::new), the last frame's stats */
  int entropy;
  uint16_t *ec_chain[3];
  uint64_t ec_stat[4];
  pthread_mutex_t mu;
  int next_sb, pass, sb_limit;
} orc_replay;

static size_t px_of(const orc_replay *r) { return r->hbd ? 2 : 1; }

static int plane_init(oplane *p, int w, int h, int xdec, int ydec, int pad, int hbd) {
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
static size_t plane_size(const oplane *p, int hbd) {
  return (size_t)p->stride * p->alloc_h * (hbd ? 2 : 1);
}
/* data origin (visible (0,0)) */
static void *org_of(const oplane *p, int hbd) {
  return p->mem + ((size_t)p->yo * p->stride + p->xo) * (hbd ? 2 : 1);
}
static void *at(const oplane *p, int hbd, int x, int y) {
  return (uint8_t *)org_of(p, hbd) + ((ptrdiff_t)y * p->stride + x) * (ptrdiff_t)(hbd ? 2 : 1);
}

static void mv_range(const orc_replay *r, int bx, int by, int bw, int bh, int m[4]) {
  int border_w = 128 + bw * 8, border_h = 128 + bh * 8;
  m[0] = -bx * 32 - border_w;
  m[1] = (r->w_in_b - bx - bw / 4) * 32 + border_w;
  m[2] = -by * 32 - border_h;
  m[3] = (r->h_in_b - by - bh / 4) * 32 + border_h;
}
/* the tile of group superblock (sx, sy): origin (SBs), visible 4x4 size */
static void sb_tile(const orc_replay *r, int sx, int sy, int *t0x, int *t0y, int *mi_w,
                    int *mi_h) {
  int fx = r->tx0 + sx, fy = r->ty0 + sy;
  *t0x = fx - fx % r->tws;
  *t0y = fy - fy % r->ths;
  int vw = r->W - *t0x * SB < r->tws * SB ? r->W - *t0x * SB : r->tws * SB;
  int vh = r->H - *t0y * SB < r->ths * SB ? r->H - *t0y * SB : r->ths * SB;
  *mi_w = vw >> 2;
  *mi_h = vh >> 2;
}
static void adjust_bo(int mi_w, int mi_h, int *bx, int *by, int bw, int bh) {
  int x = *bx < mi_w - bw / 4 ? *bx : mi_w - bw / 4;
  int y = *by < mi_h - bh / 4 ? *by : mi_h - bh / 4;
  *bx = x > 0 ? x : 0;
  *by = y > 0 ? y : 0;
}
/* a superblock of the group past the frame's right or bottom edge */
static int edge_sb(const orc_replay *r, int sb) {
  return (r->tx0 + sb % r->tw + 1) * SB > r->W || (r->ty0 + sb / r->tw + 1) * SB > r->H;
}
/* superblock sb inside the level rectangle: its (x, y) there, else 0 */
static int in_rect(const orc_replay *r, int sb, int *x, int *y) {
  const int sx = sb % r->tw - r->ex0, sy = sb / r->tw - r->ey0;
  if (!r->lvl || sx < 0 || sy < 0 || sx >= r->ew || sy >= r->eh) return 0;
  *x = sx;
  *y = sy;
  return 1;
}
static uint64_t pack_mv(orc_mv m) { return ((uint64_t)(uint16_t)m.row << 16) | (uint16_t)m.col; }
static orc_mv qfull(orc_mv m) {
  orc_mv q = {(int16_t)((m.row / 8) * 8), (int16_t)((m.col / 8) * 8)};
  return q;
}
static int mv_eq(orc_mv a, orc_mv b) { return a.row == b.row && a.col == b.col; }

/* A block grid (superblocks, or one speed-6 level): rv_chain.h CandGeo */
typedef struct {
  int nsb, tw, tx0, ty0, tws, ths;
  const orc_mv *sub; /* [R][nsb] sub-pel winners (NEWMV) */
} cgeo;

/* The MV stack and candidate MVs of rv_chain.h cand_stack / cand_mv: the
 * row above, then the column to the left (merged if equal), inside the
 * tile; NEARESTMV, NEAR0MV, GLOBALMV, NEWMV per reference
 * (src/rdo.rs:880-905). */
static int cand_mv_g(const cgeo *g, int sb, int c, orc_mv *mv) {
  int k = c / NMODE, m = c % NMODE;
  int sx = sb % g->tw, sy = sb / g->tw, fx = g->tx0 + sx, fy = g->ty0 + sy;
  const orc_mv *s = g->sub + (size_t)k * g->nsb;
  orc_mv st[2], zero = {0, 0};
  int n = 0;
  if (sy > 0 && fy % g->ths) st[n++] = s[sb - g->tw];
  if (sx > 0 && fx % g->tws) {
    orc_mv v = s[sb - 1];
    if (n == 0 || !mv_eq(v, st[0])) st[n++] = v;
  }
  switch (m) {
    case 0:
      *mv = n >= 1 ? st[0] : zero;
      return 1;
    case 1:
      *mv = n >= 2 ? st[1] : zero;
      return n >= 1;
    case 2:
      *mv = zero;
      return n >= 2;
    default: {
      orc_mv me = s[sb];
      *mv = me;
      return !(n >= 1 && mv_eq(st[0], me)) && !(n >= 2 && mv_eq(st[1], me)) &&
             (me.row != 0 || me.col != 0);
    }
  }
}

/* rv_chain.h comp_mvs: RAV1E_INTER_COMPOUND_MODES (src/predict.rs:51-58)
 * GLOBAL_GLOBALMV, NEAREST_NEARESTMV, NEW_NEWMV, NEAREST_NEWMV,
 * NEW_NEARESTMV, NEAR_NEARMV over the (ref 0, ref 1) stack of the above /
 * left neighbours' NEWMV pairs, merged if equal (src/rdo.rs:952-992) */
static void comp_mvs_g(const cgeo *g, int sb, int m, orc_mv *mv0, orc_mv *mv1) {
  int sx = sb % g->tw, sy = sb / g->tw, fx = g->tx0 + sx, fy = g->ty0 + sy;
  const orc_mv *s0 = g->sub, *s1 = g->sub + g->nsb;
  orc_mv zero = {0, 0}, e[2][2] = {{zero, zero}, {zero, zero}};
  int n = 0;
  if (sy > 0 && fy % g->ths) {
    e[0][0] = s0[sb - g->tw];
    e[0][1] = s1[sb - g->tw];
    n = 1;
  }
  if (sx > 0 && fx % g->tws) {
    orc_mv l0 = s0[sb - 1], l1 = s1[sb - 1];
    if (n == 0 || !mv_eq(l0, e[0][0]) || !mv_eq(l1, e[0][1])) {
      e[n][0] = l0;
      e[n][1] = l1;
      n++;
    }
  }
  orc_mv me0 = s0[sb], me1 = s1[sb];
  switch (m) {
    case 0: *mv0 = zero; *mv1 = zero; break;
    case 1: *mv0 = e[0][0]; *mv1 = e[0][1]; break;
    case 2: *mv0 = me0; *mv1 = me1; break;
    case 3: *mv0 = e[0][0]; *mv1 = me1; break;
    case 4: *mv0 = me0; *mv1 = e[0][1]; break;
    default:
      *mv0 = n >= 2 ? e[1][0] : zero;
      *mv1 = n >= 2 ? e[1][1] : zero;
      break;
  }
}

static cgeo sb_geo(const orc_replay *r) {
  cgeo g = {r->nsb, r->tw, r->tx0, r->ty0, r->tws, r->ths, r->sub};
  return g;
}
static cgeo level_geo(const orc_replay *r, int l) {
  const struct olevel *P = &r->pl[l];
  cgeo g = {P->n, P->gw, P->tx0, P->ty0, P->tws, P->ths, P->sub};
  return g;
}
/* The superblocks' candidates: speed 10 from rav1e's stacks (r->stk), speed
 * 6 from the neighbour-NEWMV stand-in above.  rdo_mode_decision
 * (src/rdo.rs:880-905, 949-986): NEARESTMV = stack[0] (zero if empty),
 * NEAR0MV = stack[1] if len > 1, pushed if the stack is non-empty, GLOBALMV
 * (zero) if len >= 2, NEWMV if the search MV is non-zero and not among the
 * first two entries. */
static int cand_mv(const orc_replay *r, int sb, int c, orc_mv *mv) {
  if (!r->exact) {
    cgeo g = sb_geo(r);
    return cand_mv_g(&g, sb, c, mv);
  }
  const int k = c / NMODE, m = c % NMODE;
  const struct ostk *s = &r->stk[sb];
  const int n = s->n[k];
  const orc_mv zero = {0, 0};
  switch (m) {
    case 0:
      *mv = n >= 1 ? s->s[k][0] : zero;
      return 1;
    case 1:
      *mv = n >= 2 ? s->s[k][1] : zero;
      return n >= 1;
    case 2:
      *mv = zero;
      return n >= 2;
    default: {
      const orc_mv me = r->sub[(size_t)k * r->nsb + sb];
      *mv = me;
      return !(n >= 1 && mv_eq(s->s[k][0], me)) && !(n >= 2 && mv_eq(s->s[k][1], me)) &&
             (me.row != 0 || me.col != 0);
    }
  }
}
/* RAV1E_INTER_COMPOUND_MODES over the (ref 0, ref 1) stack, which the extra
 * search always fills to two entries (src/context.rs:2858-2906) */
static void comp_mvs(const orc_replay *r, int sb, int m, orc_mv *mv0, orc_mv *mv1) {
  if (!r->exact) {
    cgeo g = sb_geo(r);
    comp_mvs_g(&g, sb, m, mv0, mv1);
    return;
  }
  const struct ostk *s = &r->stk[sb];
  const orc_mv zero = {0, 0}, me0 = r->sub[sb], me1 = r->sub[r->nsb + sb];
  switch (m) {
    case 0: *mv0 = zero; *mv1 = zero; break;               /* GLOBAL_GLOBALMV */
    case 1: *mv0 = s->c[0][0]; *mv1 = s->c[0][1]; break;   /* NEAREST_NEARESTMV */
    case 2: *mv0 = me0; *mv1 = me1; break;                 /* NEW_NEWMV */
    case 3: *mv0 = s->c[0][0]; *mv1 = me1; break;          /* NEAREST_NEWMV */
    case 4: *mv0 = me0; *mv1 = s->c[0][1]; break;          /* NEW_NEARESTMV */
    default: *mv0 = s->c[1][0]; *mv1 = s->c[1][1]; break;  /* NEAR_NEARMV */
  }
}

static int edge_levels(orc_replay *r);

orc_replay *orc_replay_create(int W, int H, int xdec, int ydec, int bd, int tile_x0, int tile_y0,
                              int tile_w, int tile_h, int tile_w_sb, int tile_h_sb, int n_refs,
                              int n_inputs, int threads) {
  if ((W & 7) || (H & 7) || (bd != 8 && bd != 10 && bd != 12) || n_refs < 1 || n_refs > 2 ||
      n_inputs < 1)
    return NULL;
  orc_replay *r = calloc(1, sizeof(*r));
  r->W = W;
  r->H = H;
  r->xdec = xdec;
  r->ydec = ydec;
  r->bd = bd;
  r->hbd = bd > 8;
  r->R = n_refs;
  r->RA = n_refs == 2 ? 3 : n_refs;
  r->C = NMODE * n_refs;
  r->w_in_b = 2 * ((W + 7) >> 3);
  r->h_in_b = 2 * ((H + 7) >> 3);
  r->w_imp = r->w_in_b / 2;
  int sbc = (W + SB - 1) / SB, sbr = (H + SB - 1) / SB;
  r->tx0 = tile_x0;
  r->ty0 = tile_y0;
  r->tw = tile_w > 0 ? tile_w : sbc - tile_x0;
  r->th = tile_h > 0 ? tile_h : sbr - tile_y0;
  r->tws = tile_w_sb > 0 ? tile_w_sb : sbc;
  r->ths = tile_h_sb > 0 ? tile_h_sb : sbr;
  r->vis_w = W - r->tx0 * SB < r->tw * SB ? W - r->tx0 * SB : r->tw * SB;
  r->vis_h = H - r->ty0 * SB < r->th * SB ? H - r->ty0 * SB : r->th * SB;
  r->nsb = r->tw * r->th;
  r->cw = SB >> xdec;
  r->ch = SB >> ydec;
  r->ntx_c = (r->cw / 32) * (r->ch / 32);
  r->threads = threads > 0 ? threads : 1;
  int cw = (W + xdec) >> xdec, ch = (H + ydec) >> ydec;
  for (int s = 0; s < NSLOT; s++) {
    oslot *o = &r->slots[s];
    if (plane_init(&o->y, W, H, 0, 0, 88, r->hbd) || plane_init(&o->u, cw, ch, xdec, ydec, 88, r->hbd) ||
        plane_init(&o->v, cw, ch, xdec, ydec, 88, r->hbd))
      return NULL;
    o->fmv = calloc((size_t)n_refs * r->w_in_b * r->h_in_b, sizeof(orc_mv));
    if (!o->fmv) return NULL;
  }
  r->n_inputs = n_inputs;
  r->inputs = calloc(n_inputs, sizeof(oinput));
  for (int i = 0; i < n_inputs; i++) {
    oinput *o = &r->inputs[i];
    if (plane_init(&o->y, W, H, 0, 0, 88, r->hbd) || plane_init(&o->u, cw, ch, xdec, ydec, 88, r->hbd) ||
        plane_init(&o->v, cw, ch, xdec, ydec, 88, r->hbd) ||
        plane_init(&o->hres, W / 2, H / 2, 0, 0, 44, r->hbd) ||
        plane_init(&o->qres, W / 4, H / 4, 0, 0, 22, r->hbd))
      return NULL;
  }
  r->h_imp = r->h_in_b / 2;
  r->la_next = 1;
  size_t nr = (size_t)r->R * r->nsb, na = (size_t)r->RA * r->nsb;
  r->coarse = calloc(na, sizeof(orc_mv));
  r->half = calloc(nr * 4, sizeof(orc_mv));
  r->half_l = calloc(na * 4, sizeof(orc_mv));
  r->hlc = calloc(na * 4, 8);
  r->tmv_e = calloc((size_t)r->R * r->tw * 16 * r->th * 16, sizeof(orc_mv));
  r->tmv_l = calloc((size_t)r->RA * r->tw * 16 * r->th * 16, sizeof(orc_mv));
  r->look = calloc(na * 16, sizeof(orc_mv));
  r->lc = calloc(na * 16, 8);
  r->full = calloc(nr, sizeof(orc_mv));
  r->sub = calloc(nr, sizeof(orc_mv));
  r->cc = calloc(na, 8);
  r->hc = calloc(nr * 4, 8);
  r->fc = calloc(nr, 8);
  r->sc = calloc(nr, 8);
  r->nwords = (size_t)r->nsb * (WPR * r->R + 4);
  r->words = calloc(r->nwords, 8);
  r->lev = calloc((size_t)r->nsb * (1024 + 2 * r->ntx_c * 1024), 4);
  r->exact = 1;
  r->bgrid = malloc((size_t)r->tw * 16 * r->th * 16 * sizeof(orc_blk));
  r->stk = calloc(r->nsb, sizeof(*r->stk));
  if (!r->bgrid || !r->stk) return NULL;
  pthread_mutex_init(&r->mu, NULL);
  if (edge_levels(r)) return NULL;
  return r;
}

static void free_levels(orc_replay *r);
static void free_la(orc_replay *r);

void orc_replay_destroy(orc_replay *r) {
  if (!r) return;
  for (int s = 0; s < NSLOT; s++) {
    oslot *o = &r->slots[s];
    free(o->y.mem);
    free(o->u.mem);
    free(o->v.mem);
    free(o->fmv);
  }
  free_la(r);
  free(r->imp_own);
  for (int i = 0; i < r->n_inputs; i++) {
    free(r->inputs[i].y.mem);
    free(r->inputs[i].u.mem);
    free(r->inputs[i].v.mem);
    free(r->inputs[i].hres.mem);
    free(r->inputs[i].qres.mem);
  }
  free(r->inputs);
  free(r->imp);
  free(r->coarse);
  free(r->half);
  free(r->half_l);
  free(r->hlc);
  free(r->tmv_e);
  free(r->tmv_l);
  free(r->look);
  free(r->lc);
  free(r->full);
  free(r->sub);
  free(r->cc);
  free(r->hc);
  free(r->fc);
  free(r->sc);
  free(r->words);
  free(r->lev);
  free(r->bgrid);
  free(r->stk);
  free_levels(r);
  free(r->mi_lg);
  free(r->mi_skip);
  for (int p = 0; p < 3; p++) free(r->lrf_units[p]);
  for (int l = 0; l < 3; l++) free(r->ec_chain[l]);
  pthread_mutex_destroy(&r->mu);
  free(r);
}

static void free_levels(orc_replay *r) {
  for (int l = 1; l < 4; l++) {
    struct olevel *P = &r->pl[l];
    free(P->full);
    free(P->sub);
    free(P->fc);
    free(P->sc);
    free(P->cost);
    free(P->lev);
    free(P->leaf);
    memset(P, 0, sizeof(*P));
  }
  free(r->leaf0);
  r->leaf0 = NULL;
  r->lvl = 0;
}

/* The level grids over group superblocks (x0, y0) + (w, h) and the result
 * words: per superblock, then per level block, then one partition mask per
 * superblock. */
static int alloc_levels(orc_replay *r, int x0, int y0, int w, int h) {
  free_levels(r);
  r->lvl = 1;
  r->ex0 = x0;
  r->ey0 = y0;
  r->ew = w;
  r->eh = h;
  r->nwords = (size_t)r->nsb * (WPR * r->R + 4);
  for (int l = 1; l < 4; l++) {
    struct olevel *P = &r->pl[l];
    int k = 1 << l;
    P->B = SB >> l;
    P->gw = w * k;
    P->gh = h * k;
    P->n = P->gw * P->gh;
    P->bc = P->B >> r->xdec;
    P->bch = P->B >> r->ydec;
    P->txl = 4 - l;
    P->txc = P->bc == 32 ? 3 : P->bc == 16 ? 2 : P->bc == 8 ? 1 : 0;
    P->tx0 = (r->tx0 + x0) * k;
    P->ty0 = (r->ty0 + y0) * k;
    P->tws = r->tws * k;
    P->ths = r->ths * k;
    size_t nr = (size_t)r->R * P->n;
    P->full = calloc(nr, sizeof(orc_mv));
    P->sub = calloc(nr, sizeof(orc_mv));
    P->fc = calloc(nr, 8);
    P->sc = calloc(nr, 8);
    P->cost = calloc(P->n, sizeof(double));
    P->lev = calloc((size_t)P->n * (P->B * P->B + 2 * P->bc * P->bch), 4);
    P->leaf = calloc(P->n, 1);
    if (!P->full || !P->sub || !P->fc || !P->sc || !P->cost || !P->lev || !P->leaf) return -1;
    P->woff = r->nwords;
    r->nwords += (size_t)P->n * (4 * r->R + 4);
  }
  r->wpart = r->nwords;
  r->nwords += (size_t)r->nsb;
  r->leaf0 = calloc(r->nsb, 1);
  /* the levels holding leaves: every one at speed 6; at speed 10 those of the
   * must_split walk of the edge superblocks (inside, parent not inside) */
  for (int l = 1; l < 4; l++) r->lv_used[l] = r->s6;
  for (int sb = 0; !r->s6 && sb < r->nsb; sb++) {
    if (!edge_sb(r, sb)) continue;
    const int X = (r->tx0 + sb % r->tw) * SB, Y = (r->ty0 + sb / r->tw) * SB;
    for (int l = 1; l < 4; l++) {
      const int B = SB >> l;
      for (int y = Y; y < Y + SB; y += B)
        for (int x = X; x < X + SB; x += B) {
          const int in = x + B <= r->W && y + B <= r->H;
          const int pin = (x & ~(2 * B - 1)) + 2 * B <= r->W && (y & ~(2 * B - 1)) + 2 * B <= r->H;
          if (in && !pin) r->lv_used[l] = 1;
        }
    }
  }
  r->lv_me[1] = r->lv_used[1] || r->lv_used[2] || r->lv_used[3];
  r->lv_me[2] = r->lv_used[2];
  r->lv_me[3] = r->lv_used[3];
  free(r->words);
  r->words = calloc(r->nwords, 8);
  return r->words && r->leaf0 ? 0 : -1;
}

/* Speed 10: encode_partition_topdown's must_split (src/encoder.rs:2407-
 * 2445) at the frame edges: the levels over the bounding rectangle of the
 * group's superblocks past the right / bottom edge (4:2:0 and 4:4:4). */
static int edge_levels(orc_replay *r) {
  int x0 = r->tw, y0 = r->th, x1 = -1, y1 = -1;
  for (int sb = 0; sb < r->nsb; sb++) {
    if (!edge_sb(r, sb)) continue;
    const int x = sb % r->tw, y = sb / r->tw;
    x0 = x < x0 ? x : x0;
    y0 = y < y0 ? y : y0;
    x1 = x > x1 ? x : x1;
    y1 = y > y1 ? y : y1;
  }
  if (x1 < 0 || r->xdec != r->ydec) return 0;
  return alloc_levels(r, x0, y0, x1 - x0 + 1, y1 - y0 + 1);
}

/* The speed-6 schedule (RV_REPLAY_SPEED6); call before the level params.
 * speed 10 is the default. */
int orc_replay_set_speed(orc_replay *r, int speed) {
  if (speed != 6 && speed != 10) return -1;
  if (speed == 10 || r->s6) return 0;
  if (r->xdec != r->ydec) return -1;
  r->s6 = 1;
  r->exact = 0; /* speed 6: the neighbour-NEWMV stand-in */
  return alloc_levels(r, 0, 0, r->tw, r->th);
}

/* Speed 10: the neighbour-NEWMV stand-in stacks instead of rav1e's (the
 * replay's RV_REPLAY_MVREF_STANDIN A/B). */
int orc_replay_set_mvref_standin(orc_replay *r, int on) {
  if (r->s6) return 0; /* speed 6 always takes the stand-in */
  r->exact = !on;
  return 0;
}

/* Deblock every coded frame before it becomes a reference (one tile group:
 * the replay's RV_REPLAY_DEBLOCK). */
int orc_replay_set_deblock(orc_replay *r, int on) {
  r->deblock = on != 0;
  if (!r->deblock) return 0;
  r->mi_cols = (r->W + 3) / 4;
  r->mi_rows = (r->H + 3) / 4;
  free(r->mi_lg);
  free(r->mi_skip);
  r->mi_lg = malloc((size_t)r->mi_cols * r->mi_rows);
  r->mi_skip = calloc((size_t)r->mi_cols * r->mi_rows, 1);
  if (r->mi_lg) memset(r->mi_lg, 4, (size_t)r->mi_cols * r->mi_rows);  /* as the device's */
  return r->mi_lg && r->mi_skip ? 0 : -1;
}

/* CDEF every coded frame after deblocking (the replay's RV_REPLAY_CDEF):
 * cdef_filter_frame with cdef_bits 0 and level l's strengths (y, uv) at
 * cdef_index 0.  Needs the deblocking block map (orc_replay_set_deblock). */
int orc_replay_set_cdef(orc_replay *r, int level, int y_strength, int uv_strength) {
  if (!r->deblock || level < 0 || level > 2 || y_strength < 0 || y_strength > 63 ||
      uv_strength < 0 || uv_strength > 63 || (r->W & 7) || (r->H & 7))
    return -1;
  r->cdef = 1;
  r->cdef_str[level][0] = (uint8_t)y_strength;
  r->cdef_str[level][1] = (uint8_t)uv_strength;
  return 0;
}

/* the block map of block (bx, by) of the level-l grid */
static void map_block(orc_replay *r, int l, int gx, int gy, int skip) {
  const int n4 = 16 >> l;
  for (int y = gy * n4; y < (gy + 1) * n4 && y < r->mi_rows; y++)
    for (int x = gx * n4; x < (gx + 1) * n4 && x < r->mi_cols; x++) {
      r->mi_lg[(size_t)y * r->mi_cols + x] = (uint8_t)(4 - l);
      r->mi_skip[(size_t)y * r->mi_cols + x] = (uint8_t)skip;
    }
}

/* the block map of this group's committed blocks */
static void map_own(orc_replay *r) {
  const int R = r->R;
  for (int sb = 0; sb < r->nsb; sb++) {
    const int sx = sb % r->tw, sy = sb / r->tw;
    if (!r->lvl || r->leaf0[sb])
      map_block(r, 0, r->tx0 + sx, r->ty0 + sy,
                (int)r->words[(size_t)sb * (WPR * R + 4) + WPR * R + 1]);
  }
  for (int l = 1; r->lvl && l < 4; l++) {
    const struct olevel *P = &r->pl[l];
    for (int b = 0; b < P->n; b++)
      if (P->leaf[b])
        map_block(r, l, P->tx0 + b % P->gw, P->ty0 + b / P->gw,
                  (int)r->words[P->woff + (size_t)b * (4 * R + 4) + 4 * R + 1]);
  }
}

/* deblock_filter_optimize + deblock_filter_frame (src/encoder.rs:2789-2793)
 * of the frame just coded (the whole frame: its block map must be
 * complete): speed 6 searches the levels (sse_optimize, src/deblock.rs:
 * 1418-1475, against the frame's source), speed 10 takes the fast ones;
 * nothing is filtered unless a luma level is non-zero. */
static void deblock_planes(orc_replay *r) {
  oslot *S = &r->slots[r->fi.display % NSLOT];
  oplane *pl[3] = {&S->y, &S->u, &S->v};
  uint8_t lv4[4];
  if (r->s6) {
    const oinput *cur = &r->inputs[r->fi.display % r->n_inputs];
    const oplane *src[3] = {&cur->y, &cur->u, &cur->v};
    int64_t v[3][65], h[3][65];
    for (int p = 0; p < 3; p++)
      orc_deblock_sse_plane(org_of(pl[p], r->hbd), pl[p]->stride, org_of(src[p], r->hbd),
                            src[p]->stride, r->hbd, r->bd, r->W, r->H, p ? r->xdec : 0,
                            p ? r->ydec : 0, p, r->mi_lg, r->mi_skip, r->mi_cols, v[p], h[p]);
    orc_deblock_sse_levels((const int64_t(*)[65])v, (const int64_t(*)[65])h, lv4);
  } else {
    const int qidx = r->lv[r->fi.level].qidx;
    const uint8_t lv = (uint8_t)orc_deblock_fast_level(orc_ac_q(qidx, 0, r->bd), r->bd, 0);
    for (int k = 0; k < 4; k++) lv4[k] = lv;
  }
  memcpy(r->db_levels, lv4, 4);
  if (!lv4[0] && !lv4[1]) return;
  for (int p = 0; p < 3; p++)
    orc_deblock_plane(org_of(pl[p], r->hbd), pl[p]->stride, r->hbd, r->bd, r->W, r->H,
                      p ? r->xdec : 0, p ? r->ydec : 0, p, r->mi_lg, r->mi_skip, r->mi_cols, lv4);
}

/* Loop restoration of every coded frame (the replay's RV_REPLAY_LRF):
 * rdo_loop_decision's restoration choice per unit while the frame is coded
 * (src/encoder.rs:3236-3320, src/rdo.rs:1726-2120), lrf_filter_frame after
 * CDEF (src/encoder.rs:2803-2806).  Needs the deblocking block map; one
 * tile group. */
int orc_replay_set_lrf(orc_replay *r, int on) {
  if (on && !r->deblock) return -1;
  r->lrf = on != 0;
  return 0;
}
/* the last frame's unit filters of plane p: (set, xqd0, xqd1) per
 * superblock in raster order (a superblock without a unit of its own --
 * stretched into its neighbour's -- reads None) */
void orc_replay_lrf_units(const orc_replay *r, int plane, int8_t *out, int cap) {
  const int sbc = (r->W + SB - 1) / SB, sbr = (r->H + SB - 1) / SB;
  const orc_lrf_plane_cfg *c = &r->lrf_cfg[plane];
  for (int y = 0; y < sbr; y++)
    for (int x = 0; x < sbc; x++) {
      const int i = y * sbc + x;
      if (3 * i + 2 >= cap) return;
      orc_lrf_unit u = {-1, {0, 0}};
      if (x < c->cols && y < c->rows && r->lrf_units[plane]) u = r->lrf_units[plane][y * c->cols + x];
      out[3 * i] = u.set;
      out[3 * i + 1] = u.xqd[0];
      out[3 * i + 2] = u.xqd[1];
    }
}

/* the levels deblock_filter_optimize chose for the last deblocked frame */
void orc_replay_deblock_levels(const orc_replay *r, uint8_t out[4]) {
  memcpy(out, r->db_levels, 4);
}

/* cdef_filter_frame (src/encoder.rs:2795-2802) of the frame just coded,
 * from a copy of its deblocked planes back into them */
static void cdef_planes(orc_replay *r) {
  oslot *S = &r->slots[r->fi.display % NSLOT];
  oplane *pl[3] = {&S->y, &S->u, &S->v};
  const void *in[3];
  void *out[3];
  ptrdiff_t ist[3], ost[3];
  for (int p = 0; p < 3; p++) {
    const size_t rowb = (size_t)pl[p]->w * px_of(r);
    uint8_t *c = malloc(rowb * pl[p]->h);
    const uint8_t *o = org_of(pl[p], r->hbd);
    for (int y = 0; y < pl[p]->h; y++)
      memcpy(c + y * rowb, o + (size_t)y * pl[p]->stride * px_of(r), rowb);
    in[p] = c;
    ist[p] = pl[p]->w;
    out[p] = org_of(pl[p], r->hbd);
    ost[p] = pl[p]->stride;
  }
  uint8_t ys[8] = {0}, us[8] = {0};
  ys[0] = r->cdef_str[r->fi.level][0];
  us[0] = r->cdef_str[r->fi.level][1];
  uint8_t *idx = calloc((size_t)((r->W + 63) / 64) * ((r->H + 63) / 64), 1);
  orc_cdef_filter_frame(in, ist, out, ost, r->hbd, r->bd, r->W, r->H, r->xdec, r->ydec,
                        r->mi_skip, r->mi_cols, idx, ys, us, 3, NULL, NULL);
  free(idx);
  for (int p = 0; p < 3; p++) free((void *)in[p]);
}

static double dist_bias(const orc_replay *r, int mi_x, int mi_y, int m);
static uint64_t biased(uint64_t v, double bias);
/* rdo_loop_plane_error (src/rdo.rs:1675-1720) of the superblock at tile
 * superblock (sx, sy) of the tile at superblock (t0x, t0y), plane p: test
 * holds the superblock's plane-p block at pitch tp; luma cdef_dist_wxh_8x8,
 * chroma sse_wxh of the 8x8's (8 >> xdec) x (8 >> ydec) part, each biased
 * with its 8x8's compute_distortion_bias, the sum scaled by dist_scale[p] */
static uint64_t lrf_plane_error(const orc_replay *r, const oplane *src, int p, int t0x, int t0y,
                                int sx, int sy, int mi_cols, int mi_rows, const void *test, int tp) {
  const int xd = p ? r->xdec : 0, yd = p ? r->ydec : 0, hbd = r->hbd;
  uint64_t err = 0;
  for (int by = 0; by < 8; by++)
    for (int bx = 0; bx < 8; bx++) {
      const int bo_x = sx * 16 + 2 * bx, bo_y = sy * 16 + 2 * by;  /* tile 4x4 units */
      if (bo_x >= mi_cols || bo_y >= mi_rows) continue;
      const int fx = t0x * 16 + bo_x, fy = t0y * 16 + bo_y;      /* frame 4x4 units */
      const double bias = dist_bias(r, fx, fy, 2);
      const int px = (fx * 4) >> xd, py = (fy * 4) >> yd;
      const int qx = (bx * 8) >> xd, qy = (by * 8) >> yd;
      const uint8_t *t = (const uint8_t *)test + ((size_t)qy * tp + qx) * px_of(r);
      if (p == 0) {
        int64_t mo[5];
        orc_cdef_moments_8x8(at(src, hbd, px, py), src->stride, t, tp, hbd, mo);
        err += biased(orc_cdef_dist_from_moments(mo, r->bd), bias);
      } else {
        uint64_t parts[4];
        const int n = orc_sse_wxh(at(src, hbd, px, py), src->stride, t, tp, 8 >> xd, 8 >> yd, xd, yd,
                                  hbd, parts);
        for (int k = 0; k < n; k++) err += biased(parts[k], bias);
      }
    }
  return (uint64_t)((double)err * r->lv[r->fi.level].ds[p]);
}

/* Loop restoration's choice of every unit of the frame just coded, as
 * rdo_loop_decision makes it while the tile is coded (src/encoder.rs:
 * 3236-3320: a unit's decision follows its last superblock; src/rdo.rs:
 * 1726-2120): units of one superblock in every plane (RestorationState::new
 * at base_q_idx <= 160, the replay's levels).  Per superblock in tile raster
 * order: the padded CDEF input of cdef_sb_padded_frame_copy (src/cdef.rs:
 * 345-406) -- the tile's reconstruction so far, 128 where a superblock is
 * not coded yet (Plane::new's fill), CDEF_VERY_LARGE outside the tile --
 * filtered with cdef index 0 into the unit's input; then per plane None and
 * the 16 sets (sgrproj_solve + sgrproj_stripe_filter), each priced with
 * count_lrf_switchable and compute_rd_cost (src/rdo.rs:563-568); the
 * cheapest (first minimum) is the unit's filter; write_lrf then updates
 * the tile's restoration CDF and the plane's sgrproj_ref.  Two quirks kept:
 * sgrproj_solve's source and the unit size read the whole frame at the
 * unit's tile-relative offset (ts.input with loop_tile_po, :2028-2033). */
static int lrf_decide(orc_replay *r) {
  const int lvl = r->fi.level, hbd = r->hbd, B = (int)px_of(r), cs = r->bd - 8;
  const int sbc = (r->W + SB - 1) / SB, sbr = (r->H + SB - 1) / SB;
  const int tiled = (sbc + r->tws - 1) / r->tws > 1 || (sbr + r->ths - 1) / r->ths > 1;
  orc_lrf_config(r->W, r->H, r->xdec, r->ydec, r->lv[lvl].qidx, tiled, r->tws, r->ths, r->lrf_cfg);
  for (int p = 0; p < 3; p++) {
    if (r->lrf_cfg[p].sb_h_shift || r->lrf_cfg[p].sb_v_shift) return -1;
    const int n = r->lrf_cfg[p].cols * r->lrf_cfg[p].rows;
    if (n != r->lrf_n[p]) {
      free(r->lrf_units[p]);
      r->lrf_units[p] = malloc(sizeof(orc_lrf_unit) * (size_t)n);
      if (!r->lrf_units[p]) return -1;
      r->lrf_n[p] = n;
    }
    for (int i = 0; i < n; i++) r->lrf_units[p][i] = (orc_lrf_unit){-1, {0, 0}};
  }
  const oinput *cur = &r->inputs[r->fi.display % r->n_inputs];
  const oslot *S = &r->slots[r->fi.display % NSLOT];
  const oplane *rec[3] = {&S->y, &S->u, &S->v}, *src[3] = {&cur->y, &cur->u, &cur->v};
  const double lambda = r->lv[lvl].lambda;
  enum { IIS = 264 };
  uint16_t *pad16[3];
  uint8_t *lin[3], *lout[3];
  uint32_t *ii = malloc(sizeof(uint32_t) * IIS * 72), *sq = malloc(sizeof(uint32_t) * IIS * 72);
  for (int p = 0; p < 3; p++) {
    pad16[p] = malloc(sizeof(uint16_t) * 68 * 68);
    lin[p] = malloc((size_t)64 * 64 * B);
    lout[p] = malloc((size_t)64 * 64 * B);
  }
  const uint8_t ys = r->cdef_str[lvl][0], us = r->cdef_str[lvl][1];
  const int pri_y = ys / 4, pri_uv = us / 4;
  int sec_y = ys % 4, sec_uv = us % 4;
  if (sec_y == 3) sec_y++;
  if (sec_uv == 3) sec_uv++;
  for (int t0y = 0; t0y < sbr; t0y += r->ths)
    for (int t0x = 0; t0x < sbc; t0x += r->tws) {
      const int tw_px = r->W - t0x * SB < r->tws * SB ? r->W - t0x * SB : r->tws * SB;
      const int th_px = r->H - t0y * SB < r->ths * SB ? r->H - t0y * SB : r->ths * SB;
      const int tsw = (tw_px + SB - 1) / SB, tsh = (th_px + SB - 1) / SB;
      const int mi_cols = tw_px >> 2, mi_rows = th_px >> 2;
      uint16_t cdf[4];
      int8_t ref[3][2];
      orc_lrf_tile_init(cdf, ref);
      int ucols[3], urows[3];
      for (int p = 0; p < 3; p++) {  /* TileRestorationState's unit view */
        const int c = r->lrf_cfg[p].cols, rw = r->lrf_cfg[p].rows;
        ucols[p] = t0x >= c ? 0 : (tsw < c - t0x ? tsw : c - t0x);
        urows[p] = t0y >= rw ? 0 : (tsh < rw - t0y ? tsh : rw - t0y);
      }
      for (int sy = 0; sy < tsh; sy++)
        for (int sx = 0; sx < tsw; sx++) {
          /* the unit's input: the superblock's reconstruction, CDEF'd */
          for (int p = 0; p < 3; p++) {
            const int xd = p ? r->xdec : 0, yd = p ? r->ydec : 0;
            const int bw = SB >> xd, bh = SB >> yd, pw_t = (tw_px + xd) >> xd, ph_t = (th_px + yd) >> yd;
            const int ox = (sx * SB) >> xd, oy = (sy * SB) >> yd;
            const int fx0 = (t0x * SB) >> xd, fy0 = (t0y * SB) >> yd;
            for (int y = -2; y < bh + 2; y++)
              for (int x = -2; x < bw + 2; x++) {
                const int tx = ox + x, ty = oy + y;
                uint16_t v = 0x8000;  /* CDEF_VERY_LARGE */
                if (tx >= 0 && tx < pw_t && ty >= 0 && ty < ph_t) {
                  const int csx = (tx << xd) / SB, csy = (ty << yd) / SB;
                  v = (csy < sy || (csy == sy && csx <= sx))
                          ? (uint16_t)orc_px(org_of(rec[p], hbd), hbd,
                                             (ptrdiff_t)(fy0 + ty) * rec[p]->stride + fx0 + tx)
                          : 128;
                }
                pad16[p][(y + 2) * (bw + 4) + x + 2] = v;
              }
            const int w = bw < pw_t - ox ? bw : pw_t - ox, h = bh < ph_t - oy ? bh : ph_t - oy;
            for (int y = 0; y < bh; y++)  /* copy + Plane::pad (replicate) */
              for (int x = 0; x < bw; x++) {
                const int cx = x < w ? x : w - 1, cy = y < h ? y : h - 1;
                orc_px_store(lin[p], hbd, y * bw + x,
                             orc_px(org_of(rec[p], hbd), hbd,
                                    (ptrdiff_t)(fy0 + oy + cy) * rec[p]->stride + fx0 + ox + cx));
              }
          }
          if (r->cdef)
            for (int by = 0; by < 8; by++)
              for (int bx = 0; bx < 8; bx++) {
                const int gx = sx * 16 + 2 * bx, gy = sy * 16 + 2 * by;
                if (gx >= mi_cols || gy >= mi_rows) continue;
                const int fx = t0x * 16 + gx, fy = t0y * 16 + gy;
                const uint8_t *sk = r->mi_skip + (size_t)fy * r->mi_cols + fx;
                const int skip = sk[0] & sk[1] & sk[r->mi_cols] & sk[r->mi_cols + 1];
                int dir = 0;
                int32_t var = 0;
                if (!skip) dir = orc_cdef_find_dir(pad16[0] + (8 * by + 2) * 68 + 8 * bx + 2, 68, &var, cs);
                for (int p = 0; p < 3; p++) {
                  const int xd = p ? r->xdec : 0, yd = p ? r->ydec : 0, bw = SB >> xd;
                  const int xs = 8 >> xd, ysz = 8 >> yd, x0 = (8 * bx) >> xd, y0 = (8 * by) >> yd;
                  const uint16_t *in = pad16[p] + (y0 + 2) * (bw + 4) + x0 + 2;
                  uint8_t *o = lin[p] + ((size_t)y0 * bw + x0) * B;
                  if (!skip) {
                    int pri, sec, dmp = 3 + cs, d;
                    if (p == 0) {
                      pri = orc_cdef_adjust_strength(pri_y << cs, var);
                      sec = sec_y << cs;
                      d = pri_y ? dir : 0;
                    } else {
                      pri = pri_uv << cs;
                      sec = sec_uv << cs;
                      dmp -= 1;
                      d = pri_uv ? dir : 0;
                    }
                    orc_cdef_filter_block(o, bw, hbd, in, bw + 4, pri, sec, d, dmp, r->bd, xd, yd);
                  } else {
                    for (int i = 0; i < ysz; i++)
                      for (int j = 0; j < xs; j++) orc_px_store(o, hbd, i * bw + j, in[i * (bw + 4) + j]);
                  }
                }
              }
          /* rdo_loop_decision's restoration pass (src/rdo.rs:2003-2116) */
          orc_lrf_unit pick[3];
          int has[3];
          for (int p = 0; p < 3; p++) {
            has[p] = sx < ucols[p] && sy < urows[p];
            if (!has[p]) continue;
            const int xd = p ? r->xdec : 0, yd = p ? r->ydec : 0, bw = SB >> xd;
            const int pw = p ? (r->W + xd) >> xd : r->W, ph = p ? (r->H + yd) >> yd : r->H;
            const int rx = (sx * SB) >> xd, ry = (sy * SB) >> yd;  /* tile-relative (quirk) */
            const int us_ = r->lrf_cfg[p].unit_size;
            const int uw = us_ < pw - rx ? us_ : pw - rx, uh = us_ < ph - ry ? us_ : ph - ry;
            orc_lrf_unit best = {-1, {0, 0}};
            const int8_t z[2] = {0, 0};
            uint64_t err = lrf_plane_error(r, src[p], p, t0x, t0y, sx, sy, mi_cols, mi_rows, lin[p], bw);
            double best_cost = (double)err + lambda * ((double)orc_lrf_rate(cdf, ref[p], -1, z) / 8.0);
            orc_lrf_integral(lin[p], bw, lin[p], bw, hbd, 0, 0, uw, uh, uw, uh, ii, sq, IIS);
            for (int k = 0; k < 64 * 64; k++) orc_px_store(lout[p], hbd, k, 128);
            for (int set = 0; set < 16; set++) {
              int8_t xqd[2];
              orc_sgr_solve(set, r->bd, ii, sq, IIS, at(src[p], hbd, rx, ry), src[p]->stride, lin[p], bw,
                            hbd, uw, uh, xqd);
              orc_sgr_stripe_filter(set, xqd, r->bd, ii, sq, IIS, uw, uh, lin[p], bw, lout[p], bw, hbd);
              err = lrf_plane_error(r, src[p], p, t0x, t0y, sx, sy, mi_cols, mi_rows, lout[p], bw);
              const double cost =
                  (double)err + lambda * ((double)orc_lrf_rate(cdf, ref[p], set, xqd) / 8.0);
              if (cost < best_cost) {
                best_cost = cost;
                best = (orc_lrf_unit){(int8_t)set, {xqd[0], xqd[1]}};
              }
            }
            pick[p] = best;
            r->lrf_units[p][(t0y + sy) * r->lrf_cfg[p].cols + t0x + sx] = best;
          }
          for (int p = 0; p < 3; p++)  /* write_lrf, planes in order */
            if (has[p]) orc_lrf_commit(cdf, ref[p], pick[p].set, pick[p].xqd);
        }
    }
  for (int p = 0; p < 3; p++) {
    free(pad16[p]);
    free(lin[p]);
    free(lout[p]);
  }
  free(ii);
  free(sq);
  return 0;
}

/* the loop filters in rav1e's order (src/encoder.rs:2789-2806) */
static void loop_filter_planes(orc_replay *r) {
  deblock_planes(r);
  if (!r->lrf) {
    if (r->cdef) cdef_planes(r);
    return;
  }
  /* pre_cdef_frame (:2795): the deblocked planes, for the stripes' edges */
  oslot *S = &r->slots[r->fi.display % NSLOT];
  oplane *pl[3] = {&S->y, &S->u, &S->v};
  void *pre[3], *out[3];
  ptrdiff_t st[3];
  for (int p = 0; p < 3; p++) {
    const size_t rowb = (size_t)pl[p]->w * px_of(r);
    uint8_t *c = malloc(rowb * pl[p]->h);
    for (int y = 0; y < pl[p]->h; y++)
      memcpy(c + y * rowb, (const uint8_t *)org_of(pl[p], r->hbd) + (size_t)y * pl[p]->stride * px_of(r),
             rowb);
    pre[p] = c;
    out[p] = org_of(pl[p], r->hbd);
    st[p] = pl[p]->stride;
  }
  if (r->cdef) cdef_planes(r);
  /* the deblocked copy's pitch is the plane width, the output's the stride:
   * lrf_filter_frame takes one stride, so the copy goes back to it */
  for (int p = 0; p < 3; p++) {
    const size_t rowb = (size_t)pl[p]->w * px_of(r);
    uint8_t *w = malloc((size_t)st[p] * pl[p]->h * px_of(r));
    for (int y = 0; y < pl[p]->h; y++)
      memcpy(w + (size_t)y * st[p] * px_of(r), (const uint8_t *)pre[p] + y * rowb, rowb);
    free(pre[p]);
    pre[p] = w;
  }
  const orc_lrf_unit *u[3] = {r->lrf_units[0], r->lrf_units[1], r->lrf_units[2]};
  orc_lrf_filter_frame(out, (const void *const *)pre, st, r->hbd, r->bd, r->W, r->H, r->xdec, r->ydec,
                       r->lrf_cfg, u, r->cdef);
  for (int p = 0; p < 3; p++) free(pre[p]);
}

static void pad(const orc_replay *r, oplane *p) {
  orc_plane_pad(p->mem, p->stride, p->alloc_h, p->xo, p->yo, 0, 0, p->w, p->h, r->hbd);
}
static void downsample(const orc_replay *r, oplane *dst, const oplane *src) {
  orc_downsample(org_of(dst, r->hbd), dst->stride, dst->w, dst->h, org_of(src, r->hbd),
                 src->stride, r->hbd);
  pad(r, dst);
}

static void copy_planes(orc_replay *r, oplane **pl, void *host, int to_plane) {
  size_t px = px_of(r);
  uint8_t *p = host;
  for (int k = 0; k < 3; k++) {
    for (int y = 0; y < pl[k]->h; y++) {
      if (to_plane)
        memcpy(at(pl[k], r->hbd, 0, y), p + (size_t)y * pl[k]->w * px, (size_t)pl[k]->w * px);
      else
        memcpy(p + (size_t)y * pl[k]->w * px, at(pl[k], r->hbd, 0, y), (size_t)pl[k]->w * px);
    }
    p += (size_t)pl[k]->w * pl[k]->h * px;
    if (to_plane) pad(r, pl[k]);
  }
}

int orc_replay_set_level_params(orc_replay *r, int level, int base_q_idx, const int32_t dc[3],
                                const int32_t ac[3], double lambda, double me_lambda,
                                const double ds[3]) {
  if (level < 0 || level > 2 || base_q_idx < 1 || base_q_idx > 255) return -1;
  r->lv[level].qidx = base_q_idx;
  for (int p = 0; p < 3; p++) {
    r->lv[level].dc[p] = dc[p];
    r->lv[level].ac[p] = ac[p];
    r->lv[level].ds[p] = ds[p];
    orc_qctx_update(&r->lv[level].q[p], base_q_idx, p ? 3 : 4, 0, r->bd, dc[p], ac[p]);
    orc_qctx_update(&r->lv[level].qi[p], base_q_idx, p ? 3 : 4, 1, r->bd, dc[p], ac[p]);
    for (int l = 1; r->lvl && l < 4; l++)
      orc_qctx_update(&r->qs[level][l][p], base_q_idx, p ? r->pl[l].txc : r->pl[l].txl, 0, r->bd,
                      dc[p], ac[p]);
  }
  r->lv[level].lambda = lambda;
  r->lv[level].me_lambda = me_lambda;
  r->lv[level].set = 1;
  return 0;
}

int orc_replay_set_input(orc_replay *r, int idx, const void *yuv) {
  if (idx < 0 || idx >= r->n_inputs) return -1;
  oinput *o = &r->inputs[idx];
  oplane *pl[3] = {&o->y, &o->u, &o->v};
  copy_planes(r, pl, (void *)yuv, 1);
  o->pyr = 0;
  return 0;
}

/* the input of display d with its pyramid */
static oinput *input_pyr(orc_replay *r, int d) {
  oinput *o = &r->inputs[d % r->n_inputs];
  if (!o->pyr) {
    downsample(r, &o->hres, &o->y);
    downsample(r, &o->qres, &o->hres);
    o->pyr = 1;
  }
  return o;
}

int orc_replay_get_recon(orc_replay *r, int display, void *yuv) {
  if (display < 0) return -1;
  oslot *o = &r->slots[display % NSLOT];
  oplane *pl[3] = {&o->y, &o->u, &o->v};
  copy_planes(r, pl, yuv, 0);
  return 0;
}

int orc_replay_set_importances(orc_replay *r, const float *imp, int n) {
  free(r->imp);
  r->imp = NULL;
  if (!imp) return 0;
  if (n != r->w_imp * (r->h_in_b / 2)) return -1;
  r->imp = malloc((size_t)n * 4);
  memcpy(r->imp, imp, (size_t)n * 4);
  return 0;
}

/* predict_inter / get_params (src/predict.rs:267-283) + put_8tap */
static void predict(const orc_replay *r, const oplane *ref, int po_x, int po_y, orc_mv mv, int w,
                    int h, void *dst, int dst_stride) {
  int ys = 3 + ref->ydec, xs = 3 + ref->xdec;
  int roff = (int)mv.row >> ys, coff = (int)mv.col >> xs;
  int rf = ((int)mv.row - roff * (1 << ys)) << (4 - ys);
  int cf = ((int)mv.col - coff * (1 << xs)) << (4 - xs);
  int qx = clamp_i32(po_x + coff - 3, -ref->xo, ref->w) + 3;
  int qy = clamp_i32(po_y + roff - 3, -ref->yo, ref->h) + 3;
  orc_put_8tap(dst, dst_stride, at(ref, r->hbd, qx, qy), ref->stride, w, h, cf, rf, 0, 0, r->bd,
               r->hbd, 0);
}

/* compound predict_inter (src/predict.rs:300-338): prep_8tap of both
 * references, mc_avg */
static void predict_comp(const orc_replay *r, const oplane *ref0, const oplane *ref1, int po_x,
                         int po_y, orc_mv mv0, orc_mv mv1, int w, int h, void *dst,
                         int dst_stride) {
  int16_t tmp[2][SB * SB];
  const oplane *rf[2] = {ref0, ref1};
  orc_mv mv[2] = {mv0, mv1};
  for (int i = 0; i < 2; i++) {
    const oplane *ref = rf[i];
    int ys = 3 + ref->ydec, xs = 3 + ref->xdec;
    int roff = (int)mv[i].row >> ys, coff = (int)mv[i].col >> xs;
    int rfr = ((int)mv[i].row - roff * (1 << ys)) << (4 - ys);
    int cfr = ((int)mv[i].col - coff * (1 << xs)) << (4 - xs);
    int qx = clamp_i32(po_x + coff - 3, -ref->xo, ref->w) + 3;
    int qy = clamp_i32(po_y + roff - 3, -ref->yo, ref->h) + 3;
    orc_prep_8tap(tmp[i], at(ref, r->hbd, qx, qy), ref->stride, w, h, cfr, rfr, 0, 0, r->bd,
                  r->hbd);
  }
  orc_mc_avg(dst, dst_stride, tmp[0], tmp[1], w, h, r->bd, r->hbd, 0);
}

static void ds_ctx(const orc_replay *r, orc_ds_ctx *c, const oplane *org, const oplane *ref,
                   int po_x, int po_y, int w, int h, const int m[4], uint32_t lambda, int subpel) {
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

/* compute_distortion_bias (src/rdo.rs:476-508) of the importance area of
 * m x m 4x4 blocks (BLOCK_8X8: m = 2; BLOCK_4X4 for chroma planes narrower
 * than 8: m = 1) at 4x4 block (mi_x, mi_y) */
static double dist_bias(const orc_replay *r, int mi_x, int mi_y, int m) {
  const float *imp = r->imp_window ? r->imp_own : r->imp;
  if (!imp) return 0.65;
  int x2 = mi_x + m < r->w_in_b ? mi_x + m : r->w_in_b;
  int y2 = mi_y + m < r->h_in_b ? mi_y + m : r->h_in_b;
  float tot = 0.f;
  for (int y = mi_y; y < y2; y++)
    for (int x = mi_x; x < x2; x++) tot += imp[(y >> 1) * r->w_imp + (x >> 1)];
  float mean = tot / (float)(m * m);
  return (double)(mean / 3.0f) + 0.65;
}
static uint64_t biased(uint64_t v, double bias) { return (uint64_t)((double)v * bias); }

/* compute_distortion (src/rdo.rs:338-411) of a B x B block at luma (px,
 * py) with bc x bch chroma blocks (predictions / reconstructions at pitch B
 * and bc): luma cdef_dist_wxh, chroma sse_wxh, each 8x8 / importance
 * sub-block biased */
static uint64_t blk_distortion(const orc_replay *r, const oinput *cur, int px, int py, int B,
                               int bc, int bch, const void *ly, const void *lu, const void *lv) {
  const int hbd = r->hbd;
  const double *ds = r->lv[r->fi.level].ds;
  uint64_t d = 0;
  for (int j = 0; j < B; j += 8)
    for (int i = 0; i < B; i += 8) {
      int64_t mo[5];
      orc_cdef_moments_8x8(at(&cur->y, hbd, px + i, py + j), cur->y.stride,
                           (const uint8_t *)ly + ((size_t)j * B + i) * px_of(r), B, hbd, mo);
      d += biased(orc_cdef_dist_from_moments(mo, r->bd),
                  dist_bias(r, (px + i) >> 2, (py + j) >> 2, 2));
    }
  /* Distortion * dist_scale[p] -> ScaledDistortion (src/rdo.rs:375, 406) */
  d = (uint64_t)((double)d * ds[0]);
  const int cpx = px >> r->xdec, cpy = py >> r->ydec;
  const int iw = bc < 8 ? bc : 8, ih = bch < 8 ? bch : 8;
  const int bw = iw >> r->xdec, bh = ih >> r->ydec, nbx = bc / bw, m = iw / 4;
  uint64_t parts[SB * SB];
  const oplane *cs[2] = {&cur->u, &cur->v};
  const void *cp[2] = {lu, lv};
  for (int pl = 0; pl < 2; pl++) {
    int n = orc_sse_wxh(at(cs[pl], hbd, cpx, cpy), cs[pl]->stride, cp[pl], bc, bc, bch, r->xdec,
                        r->ydec, hbd, parts);
    uint64_t dp = 0;
    for (int k = 0; k < n; k++) {
      int bx = k % nbx, by = k / nbx;
      int x = cpx + bx * bw, y = cpy + by * bh;
      dp += biased(parts[k], dist_bias(r, (x << r->xdec) >> 2, (y << r->ydec) >> 2, m));
    }
    d += (uint64_t)((double)dp * ds[1 + pl]);
  }
  return d;
}
static uint64_t sb_distortion(const orc_replay *r, const oinput *cur, int px, int py,
                              const void *ly, const void *lu, const void *lv) {
  return blk_distortion(r, cur, px, py, SB, r->cw, r->ch, ly, lu, lv);
}

/* encode_tx_block (src/encoder.rs:1077-1237) of one transform block:
 * diff + fht + quantize, tx-domain distortion -> estimate_rate,
 * dequantize, inverse + add into `rec` (stride rs).  Returns the rate. */
static uint64_t tx_block_q(const orc_replay *r, const oplane *src, int sx, int sy, void *rec,
                           int rs, int tx_size, int plane, int32_t *levels_out,
                           const orc_qctx *q) {
  const int lvl = r->fi.level, qidx = r->lv[lvl].qidx;
  const int n = 1 << ORC_TX_W_LOG2[tx_size];
  int16_t res[SB * SB];
  int32_t co[SB * SB], qc[32 * 32], rc[32 * 32];
  orc_diff(res, at(src, r->hbd, sx, sy), src->stride, rec, rs, n, n, r->hbd);
  orc_fwd_txfm2d(res, co, tx_size, 0, r->bd);
  orc_quantize(q, co, qc, tx_size, 0);
  orc_dequantize(qidx, qc, rc, tx_size, r->bd, r->lv[lvl].dc[plane], r->lv[lvl].ac[plane]);
  const int ca = orc_coded_tx_area(tx_size);
  uint64_t rate = orc_estimate_rate(qidx, tx_size, orc_tx_dist(co, rc, ca, n, n));
  orc_inv_txfm2d_add(rc, rec, rs, tx_size, 0, r->bd, r->hbd);
  if (levels_out) memcpy(levels_out, qc, (size_t)ca * 4);
  return rate;
}
static uint64_t tx_block(const orc_replay *r, const oplane *src, int sx, int sy, void *rec, int rs,
                         int tx_size, int plane, int32_t *levels_out) {
  return tx_block_q(r, src, sx, sy, rec, rs, tx_size, plane, levels_out,
                    &r->lv[r->fi.level].q[plane]);
}

/* Static search geometry of superblock sb: its tile's origin, visible
 * 4x4 size, the superblock's place in the tile and the tile's size in
 * superblocks. */
typedef struct {
  int t0x, t0y, mi_w, mi_h, tsx, tsy, tsw, tsh;
} sbgeo;
static sbgeo sb_geo_of(const orc_replay *r, int sb) {
  sbgeo g;
  const int sx = sb % r->tw, sy = sb / r->tw;
  sb_tile(r, sx, sy, &g.t0x, &g.t0y, &g.mi_w, &g.mi_h);
  g.tsx = r->tx0 + sx - g.t0x;
  g.tsy = r->ty0 + sy - g.t0y;
  g.tsw = (g.mi_w + 15) / 16;
  g.tsh = (g.mi_h + 15) / 16;
  return g;
}
/* A diamond search context at tile-relative 4x4 offset (bx, by) of size
 * bw (adjust_bo'd if adj), on the 1 >> shift resolution planes. */
static void ds_at(const orc_replay *r, orc_ds_ctx *c, const sbgeo *g, const oplane *org,
                  const oplane *ref, int bx, int by, int bw, int adj, int shift, uint32_t lambda) {
  if (adj) adjust_bo(g->mi_w, g->mi_h, &bx, &by, bw, bw);
  const int fbx = bx + g->t0x * 16, fby = by + g->t0y * 16;
  int m[4];
  mv_range(r, fbx, fby, bw, bw, m);
  int ms[4] = {m[0] >> shift, m[1] >> shift, m[2] >> shift, m[3] >> shift};
  ds_ctx(r, c, org, ref, (fbx * 4) >> shift, (fby * 4) >> shift, bw >> shift, bw >> shift, ms,
         lambda, 0);
}
/* coarse / half-res MVs in 1/8 pel of full resolution, quantize_to_fullpel */
static orc_mv coarse_fp(const orc_replay *r, int k, int sb) {
  orc_mv c = r->coarse[(size_t)k * r->nsb + sb];
  return qfull((orc_mv){(int16_t)(c.row * 4), (int16_t)(c.col * 4)});
}
static orc_mv half_fp(const orc_replay *r, int k, int sb, int q) {
  orc_mv h = r->half_l[((size_t)k * r->nsb + sb) * 4 + q];
  return qfull((orc_mv){(int16_t)(h.row * 2), (int16_t)(h.col * 2)});
}

/* the references the current search pass runs over: the lookahead's (la_mode)
 * or the encode's */
static int nrefs(const orc_replay *r) { return r->la_mode ? r->lar.n : r->R; }
static int rdisp(const orc_replay *r, int k) {
  return r->la_mode ? r->lar.disp[k] : r->fi.ref_display[k];
}

/* Pass A1: F1 estimate_motion_ss4 (build_coarse_pmvs) of one superblock. */
static void run_coarse(orc_replay *r, int sb) {
  const oinput *S = &r->inputs[r->fi.display % r->n_inputs];
  const int hbd = r->hbd;
  const sbgeo g = sb_geo_of(r, sb);
  int bx = g.tsx * 16, by = g.tsy * 16;
  adjust_bo(g.mi_w, g.mi_h, &bx, &by, 64, 64);
  int fbx = bx + g.t0x * 16, fby = by + g.t0y * 16;
  int m[4];
  mv_range(r, fbx, fby, 64, 64, m);
  const double me_lambda = r->lv[r->fi.level].me_lambda;
  uint32_t lambda4 = (uint32_t)(me_lambda * 256.0 / 16.0 * 0.125);
  int scale = r->fi.me_range_scale;
  int rx = 192 * scale, ry = 64 * scale;
  int x_lo = fbx + ((m[0] / 8 > -rx ? m[0] / 8 : -rx) >> 2);
  int x_hi = fbx + ((m[1] / 8 < rx ? m[1] / 8 : rx) >> 2);
  int y_lo = fby + ((m[2] / 8 > -ry ? m[2] / 8 : -ry) >> 2);
  int y_hi = fby + ((m[3] / 8 < ry ? m[3] / 8 : ry) >> 2);
  orc_mv zero = {0, 0};
  for (int k = 0; k < nrefs(r); k++) {
    const oinput *ref = &r->inputs[rdisp(r, k) % r->n_inputs];
    orc_mv best = {0, 0};
    uint64_t cost = UINT64_MAX;
    orc_full_search(org_of(&S->qres, hbd), S->qres.stride, org_of(&ref->qres, hbd),
                    ref->qres.stride, hbd, fbx, fby, x_lo, x_hi, y_lo, y_hi, 16, 16, 1, lambda4,
                    zero, zero, 0, &best, &cost);
    r->coarse[k * r->nsb + sb] = best;
    r->cc[k * r->nsb + sb] = cost;
  }
}

/* ---- EPZS: the tile motion fields ------------------------------------------
 * get_subset_predictors (src/me.rs:82-174) reads the tile's field ts.mvs
 * (save_block_motion, src/encoder.rs:1432-1444): FrameState starts it at
 * zero for every frame; build_half_res_pmvs saves the four quadrant MVs of
 * each superblock, the lookahead's build_full_res_pmvs its 16x16 MVs, and
 * the encode every coded inter block's MV (its first reference's index,
 * src/encoder.rs:2607-2613).  The encode's field becomes the frame's
 * frame_mvs, which later frames read through their LAST reference (subset
 * C); the lookahead's reference frames carry none. */

/* reference k's field of a group grid, at the tile of g (pitch tw * 16) */
static orc_mv *tile_field(const orc_replay *r, orc_mv *grid, int k, const sbgeo *g) {
  const size_t gp = (size_t)r->tw * 16;
  return grid + (size_t)k * gp * r->th * 16 + (size_t)(g->t0y - r->ty0) * 16 * gp +
         (size_t)(g->t0x - r->tx0) * 16;
}
/* save_block_motion: mv over the w4 x h4 block at tile offset (bx, by),
 * clipped to the tile */
static void save_motion(const orc_replay *r, orc_mv *tile, const sbgeo *g, int bx, int by, int w4,
                        int h4, orc_mv mv) {
  const size_t gp = (size_t)r->tw * 16;
  const int xe = bx + w4 < g->mi_w ? bx + w4 : g->mi_w, ye = by + h4 < g->mi_h ? by + h4 : g->mi_h;
  for (int y = by; y < ye; y++)
    for (int x = bx; x < xe; x++) tile[(size_t)y * gp + x] = mv;
}
/* estimate_motion_ss4's result (the coarse MV * 4) */
static orc_mv coarse4(const orc_replay *r, int k, int sb) {
  const orc_mv c = r->coarse[(size_t)k * r->nsb + sb];
  return (orc_mv){(int16_t)(c.row * 4), (int16_t)(c.col * 4)};
}

/* estimate_motion_ss2 (src/me.rs:280-327) of quadrant q of superblock sb
 * against reference k: me_ss2 (:465-519) from get_subset_predictors at the
 * adjust_bo'd 32x32 -- cmvs: the coarse MVs of the superblock and of its
 * horizontal and vertical neighbour in the tile (build_half_res_pmvs,
 * src/encoder.rs:2864-3019) -- over the tile field of `grid` and the
 * reference frame's field `prev` (NULL: none), every predictor halved. */
static void half_quadrant(orc_replay *r, int sb, int k, int q, orc_mv *grid, const orc_mv *prev,
                          orc_mv *mv, uint64_t *cost) {
  const oinput *S = &r->inputs[r->fi.display % r->n_inputs];
  const oinput *ref = &r->inputs[rdisp(r, k) % r->n_inputs];
  const sbgeo g = sb_geo_of(r, sb);
  const double me_lambda = r->lv[r->fi.level].me_lambda;
  const uint32_t lambda2 = (uint32_t)(me_lambda * 256.0 / 4.0 * 0.125);
  const int hw = g.tsx > 0, he = g.tsx < g.tsw - 1, hn = g.tsy > 0, hs = g.tsy < g.tsh - 1;
  orc_mv cm[3];
  int nc = 0;
  cm[nc++] = coarse4(r, k, sb);
  if ((q & 1) ? he : hw) cm[nc++] = coarse4(r, k, (q & 1) ? sb + 1 : sb - 1);
  if ((q >> 1) ? hs : hn) cm[nc++] = coarse4(r, k, (q >> 1) ? sb + r->tw : sb - r->tw);
  int bx = g.tsx * 16 + (q & 1) * 8, by = g.tsy * 16 + (q >> 1) * 8;
  adjust_bo(g.mi_w, g.mi_h, &bx, &by, 32, 32);
  orc_mv p[ORC_MAX_PRED];
  const int n = orc_subset_predictors(bx, by, cm, nc, tile_field(r, grid, k, &g), r->tw * 16,
                                      g.mi_w, prev, r->w_in_b, r->w_in_b, r->h_in_b,
                                      g.t0x * 16 + bx, g.t0y * 16 + by, p);
  for (int i = 0; i < n; i++) {
    p[i].row = (int16_t)(p[i].row >> 1);
    p[i].col = (int16_t)(p[i].col >> 1);
  }
  orc_ds_ctx c;
  ds_at(r, &c, &g, &S->hres, &ref->hres, bx, by, 32, 1, 1, lambda2);
  orc_diamond_search(&c, p, n, mv, cost);
}
/* build_half_res_pmvs of superblock sb over `grid`: the four quadrants per
 * reference, then their MVs (estimate_motion_ss2 returns the half-res MV *
 * 2) saved into the field at the quadrants' own offsets (no adjust_bo). */
static void half_sb(orc_replay *r, int sb, orc_mv *grid, orc_mv *mvs, uint64_t *costs, int encode) {
  const sbgeo g = sb_geo_of(r, sb);
  for (int k = 0; k < nrefs(r); k++) {
    /* subset C: the LAST reference's frame_mvs (fi.rec_buffer.frames[
     * fi.ref_frames[0]], src/me.rs:399-402, 479-481) */
    const orc_mv *prev = encode ? r->slots[r->fi.ref_display[0] % NSLOT].fmv +
                                      (size_t)k * r->w_in_b * r->h_in_b
                                : NULL;
    const size_t o = ((size_t)k * r->nsb + sb) * 4;
    for (int q = 0; q < 4; q++) half_quadrant(r, sb, k, q, grid, prev, &mvs[o + q], &costs[o + q]);
    orc_mv *tile = tile_field(r, grid, k, &g);
    for (int q = 0; q < 4; q++) {
      const orc_mv m = {(int16_t)(mvs[o + q].row * 2), (int16_t)(mvs[o + q].col * 2)};
      save_motion(r, tile, &g, g.tsx * 16 + (q & 1) * 8, g.tsy * 16 + (q >> 1) * 8, 8, 8, m);
    }
  }
}

/* F3 motion_estimation of the 64x64 (src/me.rs:193-278): the full-pel
 * diamond from zero and the coarse MV, then sub-pel; the rate predictors
 * pmv are the first two entries of the reference's MV stack
 * (rdo_mode_decision, src/rdo.rs:858-870; zero without the exact stacks). */
static void me64_sb(orc_replay *r, int sb) {
  const oinput *cur = &r->inputs[r->fi.display % r->n_inputs];
  const sbgeo g = sb_geo_of(r, sb);
  const double me_lambda = r->lv[r->fi.level].me_lambda;
  uint32_t lambda1 = (uint32_t)(me_lambda * 256.0 * 0.5);
  const orc_mv zero = {0, 0};
  for (int k = 0; k < r->R; k++) {
    const oslot *ref = &r->slots[r->fi.ref_display[k] % NSLOT];
    orc_ds_ctx c;
    orc_mv fmv, smv;
    uint64_t cost;
    orc_mv fp[ORC_MAX_PRED] = {zero, coarse_fp(r, k, sb)};
    int np = 2;
    ds_at(r, &c, &g, &cur->y, &ref->y, g.tsx * 16, g.tsy * 16, 64, 0, 0, lambda1);
    if (r->exact) {
      const struct ostk *s = &r->stk[sb];
      c.pmv[0] = s->n[k] >= 1 ? s->s[k][0] : zero;
      c.pmv[1] = s->n[k] >= 2 ? s->s[k][1] : zero;
      /* full_pixel_me (src/me.rs:390-431): get_subset_predictors at the
       * block, cmvs = [pmvs[0], the coarse MV], the encode's tile field,
       * the LAST reference's frame field */
      const orc_mv cm = coarse4(r, k, sb);
      np = orc_subset_predictors(g.tsx * 16, g.tsy * 16, &cm, 1, tile_field(r, r->tmv_e, k, &g),
                                 r->tw * 16, g.mi_w,
                                 r->slots[r->fi.ref_display[0] % NSLOT].fmv +
                                     (size_t)k * r->w_in_b * r->h_in_b,
                                 r->w_in_b, r->w_in_b, r->h_in_b, g.t0x * 16 + g.tsx * 16,
                                 g.t0y * 16 + g.tsy * 16, fp);
    }
    orc_diamond_search(&c, fp, np, &fmv, &cost);
    r->full[k * r->nsb + sb] = fmv;
    r->fc[k * r->nsb + sb] = cost;
    c.subpel = 1;
    c.satd = r->s6; /* use_satd_subpel (speed <= 9) */
    orc_diamond_search(&c, &fmv, 1, &smv, &cost);
    r->sub[k * r->nsb + sb] = smv;
    r->sc[k * r->nsb + sb] = cost;
  }
}

/* The lookahead's build_full_res_pmvs of superblock sb (src/encoder.rs:
 * 3021-3166; compute_lookahead_motion_vectors, src/api/internal.rs:514-622):
 * per reference the 16 16x16 blocks in raster order, each estimate_motion
 * (src/me.rs:337-390: full-pel, adjust_bo'd) against the reference's
 * original frame from get_subset_predictors over the lookahead's field --
 * cmvs: the coarse MV, the covering quadrant, two vertical and two
 * horizontal candidates of this and the adjacent superblocks -- its MV
 * saved at the block (the reference frames carry no field: no subset C). */
static void full_res_sb(orc_replay *r, int sb) {
  const oinput *cur = &r->inputs[r->fi.display % r->n_inputs];
  const sbgeo g = sb_geo_of(r, sb);
  const double me_lambda = r->lv[r->fi.level].me_lambda;
  uint32_t lambda1 = (uint32_t)(me_lambda * 256.0 * 0.5);
  const int hw = g.tsx > 0, he = g.tsx < g.tsw - 1, hn = g.tsy > 0, hs = g.tsy < g.tsh - 1;
  for (int k = 0; k < nrefs(r); k++) {
    const oplane *orig = &r->inputs[rdisp(r, k) % r->n_inputs].y;
    orc_mv *tile = tile_field(r, r->tmv_l, k, &g);
    /* pmvs_X[e] of superblock sb + (dx, dy): e = 0 coarse, 1..4 quadrants */
#define PM(dx, dy, e)                                                              \
  do {                                                                             \
    const int ok_ = (dx) < 0 ? hw : (dx) > 0 ? he : (dy) < 0 ? hn : (dy) > 0 ? hs : 1; \
    if (ok_) {                                                                     \
      const int s2_ = sb + (dx) + (dy) * r->tw;                                    \
      cand[nc++] = (e) == 0 ? coarse_fp(r, k, s2_) : half_fp(r, k, s2_, (e) - 1);  \
    }                                                                              \
  } while (0)
    for (int y = 0; y < 4; y++)
      for (int x = 0; x < 4; x++) {
        orc_mv cand[6];
        int nc = 0;
        const int L = x <= 1, T = y <= 1;
        PM(0, 0, 0);
        PM(0, 0, T ? (L ? 1 : 2) : (L ? 3 : 4));
        switch (y) {
          case 0: PM(0, -1, 0); PM(0, -1, L ? 3 : 4); break;
          case 1: PM(0, -1, L ? 3 : 4); PM(0, 0, L ? 3 : 4); break;
          case 2: PM(0, 1, L ? 1 : 2); PM(0, 0, L ? 1 : 2); break;
          default: PM(0, 1, 0); PM(0, 1, L ? 1 : 2); break;
        }
        switch (x) {
          case 0: PM(-1, 0, 0); PM(-1, 0, T ? 2 : 4); break;
          case 1: PM(-1, 0, T ? 2 : 4); PM(0, 0, T ? 2 : 4); break;
          case 2: PM(1, 0, T ? 1 : 3); PM(0, 0, T ? 1 : 3); break;
          default: PM(1, 0, 0); PM(1, 0, T ? 2 : 4); break;
        }
        int bx = g.tsx * 16 + x * 4, by = g.tsy * 16 + y * 4;
        adjust_bo(g.mi_w, g.mi_h, &bx, &by, 16, 16);
        orc_mv p[ORC_MAX_PRED];
        const int np = orc_subset_predictors(bx, by, cand, nc, tile, r->tw * 16, g.mi_w, NULL, 0,
                                             0, 0, 0, 0, p);
        orc_ds_ctx c;
        ds_at(r, &c, &g, &cur->y, orig, bx, by, 16, 1, 0, lambda1);
        orc_mv mv;
        uint64_t cost;
        orc_diamond_search(&c, p, np, &mv, &cost);
        r->look[((size_t)k * r->nsb + sb) * 16 + y * 4 + x] = mv;
        r->lc[((size_t)k * r->nsb + sb) * 16 + y * 4 + x] = cost;
        save_motion(r, tile, &g, g.tsx * 16 + x * 4, g.tsy * 16 + y * 4, 4, 4, mv);
      }
#undef PM
  }
}

/* The lookahead of one tile (index t of the group's tiles) in rav1e's
 * order: build_half_res_pmvs of every superblock, then build_full_res_pmvs
 * of every superblock, raster order (src/api/internal.rs:604-620). */
static void lookahead_tile(orc_replay *r, int t) {
  const int gtx = (r->tw + r->tws - 1) / r->tws;
  const int tx0 = (t % gtx) * r->tws, ty0 = (t / gtx) * r->ths;
  for (int pass = 0; pass < 2; pass++)
    for (int y = ty0; y < ty0 + r->ths && y < r->th; y++)
      for (int x = tx0; x < tx0 + r->tws && x < r->tw; x++) {
        const int sb = y * r->tw + x;
        if (r->sb_limit > 0 && sb >= r->sb_limit) continue; /* a bounded timing sample */
        if (pass == 0)
          half_sb(r, sb, r->tmv_l, r->half_l, r->hlc, 0);
        else
          full_res_sb(r, sb);
      }
}

/* Pass A3: F3 motion_estimation of the 64x64 (src/me.rs:193-278: zero + the
 * coarse MV, then sub-pel) outside coding order, and the levels' blocks. */
static void run_me(orc_replay *r, int sb) {
  const oinput *cur = &r->inputs[r->fi.display % r->n_inputs];
  const int R = r->R;
  uint64_t cost;
  const double me_lambda = r->lv[r->fi.level].me_lambda;
  uint32_t lambda1 = (uint32_t)(me_lambda * 256.0 * 0.5);
  orc_mv zero = {0, 0};
  const oslot *ref[2];
  for (int k = 0; k < R; k++) ref[k] = &r->slots[r->fi.ref_display[k] % NSLOT];
  /* speed 10: the 64x64 search needs the superblock's MV stack (its pmv),
   * so it runs in coding order (chain_tile) */
  if (!r->exact) me64_sb(r, sb);
  /* the levels (speed 6: every superblock; speed 10: the frame-edge
   * rectangle): motion_estimation of every 32x32, then 16x16 and 8x8 block
   * of the superblock at its own position (src/me.rs:193-278), seeded with
   * the pmvs entry: a 32x32 its half-res quadrant search, a 16x16 / 8x8 its
   * 32x32's sub-pel winner; sub-pel by SATD at speed 6, SAD at speed 10 */
  int ex, ey;
  if (!in_rect(r, sb, &ex, &ey)) return;
  for (int l = 1; l < 4; l++) {
    if (!r->lv_me[l]) continue;
    struct olevel *P = &r->pl[l];
    const int k2 = 1 << l, B = P->B;
    const struct olevel *U = &r->pl[1];
    for (int j = 0; j < k2; j++)
      for (int i = 0; i < k2; i++) {
        const int bx = ex * k2 + i, by = ey * k2 + j, b = by * P->gw + bx;
        const int X = (P->tx0 + bx) * B, Y = (P->ty0 + by) * B;
        int mb[4];
        mv_range(r, X >> 2, Y >> 2, B, B, mb);
        for (int k = 0; k < R; k++) {
          orc_mv par = l == 1 ? half_fp(r, k, sb, j * 2 + i)
                              : qfull(U->sub[(size_t)k * U->n + (by >> (l - 1)) * U->gw +
                                             (bx >> (l - 1))]);
          orc_mv fp[2] = {zero, par}, fmv, smv;
          orc_ds_ctx c;
          ds_ctx(r, &c, &cur->y, &ref[k]->y, X, Y, B, B, mb, lambda1, 0);
          orc_diamond_search(&c, fp, 2, &fmv, &cost);
          P->full[(size_t)k * P->n + b] = fmv;
          P->fc[(size_t)k * P->n + b] = cost;
          c.subpel = 1;
          c.satd = r->s6;
          orc_diamond_search(&c, &fmv, 1, &smv, &cost);
          P->sub[(size_t)k * P->n + b] = smv;
          P->sc[(size_t)k * P->n + b] = cost;
        }
      }
  }
}

/* Speed 6: rdo_mode_decision of block b of level l (B x B luma with one
 * TX_BxB, bc x bch chroma blocks with one transform each): the winner's
 * words, levels and rd cost; its reconstruction into oy / ou / ov (pitch
 * SB and r->cw). */
static void rdo_level_block(orc_replay *r, int l, int b, const oinput *cur, const oslot **ref,
                            uint8_t *oy, uint8_t *ou, uint8_t *ov) {
  struct olevel *P = &r->pl[l];
  const int R = r->R, B = P->B, bc = P->bc, bch = P->bch;
  const size_t px = px_of(r);
  const int X = (P->tx0 + b % P->gw) * B, Y = (P->ty0 + b / P->gw) * B;
  const int cpx = X >> r->xdec, cpy = Y >> r->ydec;
  const cgeo g = level_geo(r, l);
  const int lvl = r->fi.level;
  const double lambda = r->lv[lvl].lambda;
  const int per = B * B + 2 * bc * bch;
  int32_t *blev = P->lev + (size_t)b * per;
  int32_t clev[32 * 32 * 3];
  uint16_t ly[32 * 32], lu[32 * 32], lv[32 * 32], by_[32 * 32], bu_[32 * 32], bv_[32 * 32];
  double best = 1.7976931348623157e308;
  int best_c = 0, best_skip = 0;
  uint64_t best_d = 0;
  const int ncand = r->C + (r->fi.compound ? 6 : 0);
  for (int c = 0; c < ncand; c++) {
    if (c < r->C) {
      orc_mv mv;
      if (!cand_mv_g(&g, b, c, &mv)) continue;
      const oslot *rf = ref[c / NMODE];
      predict(r, &rf->y, X, Y, mv, B, B, ly, B);
      predict(r, &rf->u, cpx, cpy, mv, bc, bch, lu, bc);
      predict(r, &rf->v, cpx, cpy, mv, bc, bch, lv, bc);
    } else {
      orc_mv m0, m1;
      comp_mvs_g(&g, b, c - r->C, &m0, &m1);
      predict_comp(r, &ref[0]->y, &ref[1]->y, X, Y, m0, m1, B, B, ly, B);
      predict_comp(r, &ref[0]->u, &ref[1]->u, cpx, cpy, m0, m1, bc, bch, lu, bc);
      predict_comp(r, &ref[0]->v, &ref[1]->v, cpx, cpy, m0, m1, bc, bch, lv, bc);
    }
    uint64_t ds = blk_distortion(r, cur, X, Y, B, bc, bch, ly, lu, lv);
    int zero_dist = 0;
    double rs = (double)ds + lambda * (0.0 / 8.0);
    if (rs < best) {
      best = rs;
      best_c = c;
      best_skip = 1;
      best_d = ds;
      zero_dist = ds == 0;
      memcpy(by_, ly, (size_t)B * B * px);
      memcpy(bu_, lu, (size_t)bc * bch * px);
      memcpy(bv_, lv, (size_t)bc * bch * px);
    }
    if (zero_dist) continue;
    uint32_t rate = (uint32_t)tx_block_q(r, &cur->y, X, Y, ly, B, P->txl, 0, clev,
                                          &r->qs[lvl][l][0]);
    rate += (uint32_t)tx_block_q(r, &cur->u, cpx, cpy, lu, bc, P->txc, 1, clev + B * B,
                                 &r->qs[lvl][l][1]);
    rate += (uint32_t)tx_block_q(r, &cur->v, cpx, cpy, lv, bc, P->txc, 2,
                                 clev + B * B + bc * bch, &r->qs[lvl][l][2]);
    uint64_t dn = blk_distortion(r, cur, X, Y, B, bc, bch, ly, lu, lv);
    double rn = (double)dn + lambda * ((double)rate / 8.0);
    if (rn < best) {
      best = rn;
      best_c = c;
      best_skip = 0;
      best_d = dn;
      memcpy(by_, ly, (size_t)B * B * px);
      memcpy(bu_, lu, (size_t)bc * bch * px);
      memcpy(bv_, lv, (size_t)bc * bch * px);
      memcpy(blev, clev, (size_t)per * 4);
    }
  }
  if (best_skip) memset(blev, 0, (size_t)per * 4);
  P->cost[b] = best;
  uint64_t *w = r->words + P->woff + (size_t)b * (4 * R + 4);
  for (int k = 0; k < R; k++) {
    size_t o = (size_t)k * P->n + b;
    w[4 * k + 0] = pack_mv(P->full[o]);
    w[4 * k + 1] = P->fc[o];
    w[4 * k + 2] = pack_mv(P->sub[o]);
    w[4 * k + 3] = P->sc[o];
  }
  uint64_t cb;
  memcpy(&cb, &best, 8);
  w[4 * R + 0] = (uint64_t)best_c;
  w[4 * R + 1] = (uint64_t)best_skip;
  w[4 * R + 2] = cb;
  w[4 * R + 3] = best_d;
  for (int y = 0; y < B; y++) memcpy(oy + (size_t)y * SB * px, (uint8_t *)by_ + (size_t)y * B * px, B * px);
  for (int y = 0; y < bch; y++) {
    memcpy(ou + (size_t)y * r->cw * px, (uint8_t *)bu_ + (size_t)y * bc * px, bc * px);
    memcpy(ov + (size_t)y * r->cw * px, (uint8_t *)bv_ + (size_t)y * bc * px, bc * px);
  }
}

/* encode_partition_topdown (src/encoder.rs:2392-2470) of superblock sb
 * (rv_replay.hip partition_kernel): a block past the frame edge must split;
 * a block that fits compares its mode decision's rd cost with the sum of its
 * four children's (rdo_partition_decision, src/rdo.rs:1500-1668; strict
 * `<`); 8x8 blocks are leaves.  The leaves' reconstructions (rec[l], the
 * superblock at pitch SB / cw) go into the frame. */
static double level_cost(const orc_replay *r, double c0, int l, int x, int y) {
  if (l == 0) return c0;
  const struct olevel *P = &r->pl[l];
  return P->cost[((y / P->B) - P->ty0) * P->gw + (x / P->B) - P->tx0];
}
static int split_at(const orc_replay *r, double c0, int l, int x, int y) {
  const int B = SB >> l;
  if (x + B > r->W || y + B > r->H) return 1;
  if (l == 3 || !r->s6) return 0; /* speed 10: the minimum block is 64x64 */
  const int h = B / 2;
  double s = 0.0;
  s += level_cost(r, c0, l + 1, x, y);
  s += level_cost(r, c0, l + 1, x + h, y);
  s += level_cost(r, c0, l + 1, x, y + h);
  s += level_cost(r, c0, l + 1, x + h, y + h);
  return 0.0 + s < level_cost(r, c0, l, x, y);
}
static void commit_leaf(orc_replay *r, int l, int x, int y, int X, int Y, oslot *S,
                        uint16_t (*ry)[SB * SB], uint16_t (*ru)[SB * SB],
                        uint16_t (*rv)[SB * SB]) {
  const int B = SB >> l, hbd = r->hbd, cw = r->cw;
  const size_t px = px_of(r);
  const int bc = B >> r->xdec, bch = B >> r->ydec;
  const int ox = x - X, oy = y - Y, cox = ox >> r->xdec, coy = oy >> r->ydec;
  for (int j = 0; j < B; j++)
    memcpy(at(&S->y, hbd, x, y + j), (uint8_t *)ry[l] + ((size_t)(oy + j) * SB + ox) * px, B * px);
  for (int j = 0; j < bch; j++) {
    memcpy(at(&S->u, hbd, x >> r->xdec, (y >> r->ydec) + j),
           (uint8_t *)ru[l] + ((size_t)(coy + j) * cw + cox) * px, bc * px);
    memcpy(at(&S->v, hbd, x >> r->xdec, (y >> r->ydec) + j),
           (uint8_t *)rv[l] + ((size_t)(coy + j) * cw + cox) * px, bc * px);
  }
  if (l == 0)
    r->leaf0[((Y / SB) - r->ty0) * r->tw + (X / SB) - r->tx0] = 1;
  else {
    struct olevel *P = &r->pl[l];
    P->leaf[((y / B) - P->ty0) * P->gw + (x / B) - P->tx0] = 1;
  }
}
static void partition_sb(orc_replay *r, int sb, double c0, oslot *S, uint16_t (*ry)[SB * SB],
                         uint16_t (*ru)[SB * SB], uint16_t (*rv)[SB * SB]) {
  const int X = (r->tx0 + sb % r->tw) * SB, Y = (r->ty0 + sb / r->tw) * SB;
  uint64_t mask = 0;
  /* clear this superblock's leaf flags */
  r->leaf0[sb] = 0;
  int ex = 0, ey = 0;
  (void)in_rect(r, sb, &ex, &ey); /* the caller's superblock is in the rectangle */
  for (int l = 1; l < 4; l++) {
    struct olevel *P = &r->pl[l];
    const int k2 = 1 << l, bx0 = ex * k2, by0 = ey * k2;
    for (int j = 0; j < k2; j++) memset(P->leaf + (size_t)(by0 + j) * P->gw + bx0, 0, k2);
  }
  if (!split_at(r, c0, 0, X, Y)) {
    commit_leaf(r, 0, X, Y, X, Y, S, ry, ru, rv);
  } else {
    mask |= 1;
    for (int q = 0; q < 4; q++) {
      const int x1 = X + (q & 1) * 32, y1 = Y + (q >> 1) * 32;
      if (x1 >= r->W || y1 >= r->H) continue;
      if (!split_at(r, c0, 1, x1, y1)) {
        commit_leaf(r, 1, x1, y1, X, Y, S, ry, ru, rv);
        continue;
      }
      mask |= 2u << q;
      for (int t = 0; t < 4; t++) {
        const int x2 = x1 + (t & 1) * 16, y2 = y1 + (t >> 1) * 16;
        if (x2 >= r->W || y2 >= r->H) continue;
        if (!split_at(r, c0, 2, x2, y2)) {
          commit_leaf(r, 2, x2, y2, X, Y, S, ry, ru, rv);
          continue;
        }
        mask |= 1u << (5 + ((y2 - Y) / 16) * 4 + (x2 - X) / 16);
        for (int u = 0; u < 4; u++) {
          const int x3 = x2 + (u & 1) * 8, y3 = y2 + (u >> 1) * 8;
          if (x3 < r->W && y3 < r->H) commit_leaf(r, 3, x3, y3, X, Y, S, ry, ru, rv);
        }
      }
    }
  }
  r->words[r->wpart + sb] = mask;
}

/* Pass B: F4 + F6 + F5 for one superblock. */
static void run_rdo(orc_replay *r, int sb, uint64_t tail[3]) {
  const oinput *cur = &r->inputs[r->fi.display % r->n_inputs];
  oslot *S = &r->slots[r->fi.display % NSLOT];
  const int R = r->R, hbd = r->hbd;
  const size_t px = px_of(r);
  const int sx = sb % r->tw, sy = sb / r->tw;
  const oslot *ref[2];
  for (int k = 0; k < R; k++) ref[k] = &r->slots[r->fi.ref_display[k] % NSLOT];
  uint64_t *w = r->words + (size_t)sb * (WPR * R + 4);
  for (int k = 0; k < R; k++) {
    size_t o = (size_t)k * r->nsb + sb;
    uint64_t *wk = w + WPR * k;
    wk[0] = pack_mv(r->coarse[o]);
    wk[1] = r->cc[o];
    for (int q = 0; q < 4; q++) {
      wk[2 + 2 * q] = pack_mv(r->half[o * 4 + q]);
      wk[3 + 2 * q] = r->hc[o * 4 + q];
    }
    wk[10] = pack_mv(r->full[o]);
    wk[11] = r->fc[o];
    wk[12] = pack_mv(r->sub[o]);
    wk[13] = r->sc[o];
    for (int q = 0; q < 16; q++) {
      wk[14 + 2 * q] = pack_mv(r->look[o * 16 + q]);
      wk[15 + 2 * q] = r->lc[o * 16 + q];
    }
    for (int q = 0; q < 4; q++) {
      wk[46 + 2 * q] = pack_mv(r->half_l[o * 4 + q]);
      wk[47 + 2 * q] = r->hlc[o * 4 + q];
    }
  }
  const int ppx = (sx + r->tx0) * SB, ppy = (sy + r->ty0) * SB;
  const int cwid = r->cw, chei = r->ch, cpx = ppx >> r->xdec, cpy = ppy >> r->ydec;
  const int ntx_c = r->ntx_c;
  /* the best so far: reconstruction and levels */
  uint16_t by_[SB * SB], bu_[SB * SB], bv_[SB * SB];
  int32_t *blev = r->lev + (size_t)sb * (1024 + 2 * ntx_c * 1024);
  int32_t clev[1024 + 2 * 4 * 1024];
  uint16_t ly[SB * SB], lu[SB * SB], lv[SB * SB];
  double best = 1.7976931348623157e308;
  int best_c = 0, best_skip = 0;
  uint64_t best_d = 0;
  const int ncand = r->C + (r->fi.compound ? 6 : 0);
  for (int c = 0; c < ncand; c++) {
    orc_mv mv;
    if (c < r->C) {
      if (!cand_mv(r, sb, c, &mv)) continue;
      const oslot *rf = ref[c / NMODE];
      predict(r, &rf->y, ppx, ppy, mv, SB, SB, ly, SB);
      predict(r, &rf->u, cpx, cpy, mv, cwid, chei, lu, cwid);
      predict(r, &rf->v, cpx, cpy, mv, cwid, chei, lv, cwid);
    } else {
      orc_mv m0, m1;
      comp_mvs(r, sb, c - r->C, &m0, &m1);
      predict_comp(r, &ref[0]->y, &ref[1]->y, ppx, ppy, m0, m1, SB, SB, ly, SB);
      predict_comp(r, &ref[0]->u, &ref[1]->u, cpx, cpy, m0, m1, cwid, chei, lu, cwid);
      predict_comp(r, &ref[0]->v, &ref[1]->v, cpx, cpy, m0, m1, cwid, chei, lv, cwid);
    }
    /* skip: the prediction is the reconstruction */
    uint64_t ds = sb_distortion(r, cur, ppx, ppy, ly, lu, lv);
    int zero_dist = 0;
    const double lambda = r->lv[r->fi.level].lambda;
    double rs = (double)ds + lambda * (0.0 / 8.0);
    if (rs < best) {
      best = rs;
      best_c = c;
      best_skip = 1;
      best_d = ds;
      zero_dist = ds == 0;
      memcpy(by_, ly, SB * SB * px);
      memcpy(bu_, lu, (size_t)cwid * chei * px);
      memcpy(bv_, lv, (size_t)cwid * chei * px);
    }
    if (zero_dist) continue;
    /* non-skip: luma TX_64X64, chroma TX_32X32 blocks */
    uint32_t rate = (uint32_t)tx_block(r, &cur->y, ppx, ppy, ly, SB, 4, 0, clev);
    uint16_t *cp[2] = {lu, lv};
    const oplane *cs[2] = {&cur->u, &cur->v};
    for (int pl = 0; pl < 2; pl++)
      for (int t = 0; t < ntx_c; t++) {
        int tx = (t % (cwid / 32)) * 32, ty = (t / (cwid / 32)) * 32;
        uint8_t *pb = (uint8_t *)cp[pl] + ((size_t)ty * cwid + tx) * px;
        rate += (uint32_t)tx_block(r, cs[pl], cpx + tx, cpy + ty, pb, cwid, 3, 1 + pl,
                                   clev + 1024 + (pl * ntx_c + t) * 1024);
      }
    uint64_t dn = sb_distortion(r, cur, ppx, ppy, ly, lu, lv);
    double rn = (double)dn + lambda * ((double)rate / 8.0);
    if (rn < best) {
      best = rn;
      best_c = c;
      best_skip = 0;
      best_d = dn;
      memcpy(by_, ly, SB * SB * px);
      memcpy(bu_, lu, (size_t)cwid * chei * px);
      memcpy(bv_, lv, (size_t)cwid * chei * px);
      memcpy(blev, clev, (size_t)(1024 + 2 * ntx_c * 1024) * 4);
    }
  }
  if (best_skip) memset(blev, 0, (size_t)(1024 + 2 * ntx_c * 1024) * 4);
  uint64_t cb;
  memcpy(&cb, &best, 8);
  w[WPR * R + 0] = (uint64_t)best_c;
  w[WPR * R + 1] = (uint64_t)best_skip;
  w[WPR * R + 2] = cb;
  w[WPR * R + 3] = best_d;
  int ex, ey;
  const int lv_sb = in_rect(r, sb, &ex, &ey);
  if (!lv_sb) {
    /* F6: the winner into the frame (whole superblock) */
    if (r->lvl) {
      r->leaf0[sb] = 1;
      r->words[r->wpart + sb] = 0;
    }
    for (int y = 0; y < SB; y++) memcpy(at(&S->y, hbd, ppx, ppy + y), (uint8_t *)by_ + y * SB * px, SB * px);
    for (int y = 0; y < chei; y++) {
      memcpy(at(&S->u, hbd, cpx, cpy + y), (uint8_t *)bu_ + (size_t)y * cwid * px, cwid * px);
      memcpy(at(&S->v, hbd, cpx, cpy + y), (uint8_t *)bv_ + (size_t)y * cwid * px, cwid * px);
    }
  } else {
    /* every 32x32, 16x16 and 8x8 block of the superblock, the partition
     * decision (speed 10: must_split only), the leaves into the frame */
    static _Thread_local uint16_t ry[4][SB * SB], ru[4][SB * SB], rv[4][SB * SB];
    memcpy(ry[0], by_, SB * SB * px);
    memcpy(ru[0], bu_, (size_t)cwid * chei * px);
    memcpy(rv[0], bv_, (size_t)cwid * chei * px);
    for (int l = 1; l < 4; l++) {
      if (!r->lv_used[l]) continue;
      const struct olevel *P = &r->pl[l];
      const int k2 = 1 << l;
      for (int j = 0; j < k2; j++)
        for (int i = 0; i < k2; i++) {
          const int b = (ey * k2 + j) * P->gw + ex * k2 + i;
          rdo_level_block(r, l, b, cur, ref, (uint8_t *)ry[l] + ((size_t)j * P->B * SB + i * P->B) * px,
                          (uint8_t *)ru[l] + ((size_t)j * P->bch * cwid + i * P->bc) * px,
                          (uint8_t *)rv[l] + ((size_t)j * P->bch * cwid + i * P->bc) * px);
        }
    }
    partition_sb(r, sb, best, S, ry, ru, rv);
  }
  /* F5: the 8x8 blocks of this superblock inside the group's visible area,
   * against reference 0's original frame at the lookahead MV of their 16x16 */
  const oplane *o0 = &r->inputs[r->fi.ref_display[0] % r->n_inputs].y;
  for (int j = 0; j < 8; j++)
    for (int i = 0; i < 8; i++) {
      int bxx = sx * 8 + i, byy = sy * 8 + j;
      if (bxx >= r->vis_w / 8 || byy >= r->vis_h / 8) continue;
      int x = r->tx0 * SB + bxx * 8, y = r->ty0 * SB + byy * 8;
      const orc_mv mv0 = r->look[(size_t)sb * 16 + (j / 2) * 4 + i / 2];
      tail[2] += orc_get_satd(at(&cur->y, hbd, x, y), cur->y.stride,
                              at(o0, hbd, x + ((int)mv0.col >> 3), y + ((int)mv0.row >> 3)),
                              o0->stride, 8, 8, hbd, 0);
      uint32_t ic;
      orc_lookahead_intra_costs(at(&cur->y, hbd, x, y), cur->y.stride, 8, 8, hbd, r->bd, &ic);
      tail[2] += ic;
    }
}

/* ---- intra-mode screening and intra RDO (rdo_mode_decision,
 * src/rdo.rs:1008-1152), speed 10, 4:2:0 ------------------------------------
 * After every superblock's inter decision and commit: the superblocks of
 * each tile in raster order.  A non-skip winner (`!best.skip`) fully inside
 * the frame gets get_intra_edges (None) of the current reconstruction, the 13
 * RAV1E_INTRA_MODES predicted at TX_64X64 and their get_satd, a stable sort,
 * the modes to try = [the most probable mode under the intra y-mode CDF:
 * DC_PRED in default_if_y_mode_cdf (src/entropymode.rs:166-184), which is
 * not adapted here] + the three lowest SATDs not already in, take 3; each
 * runs luma_chroma_mode_rdo with chroma modes [mode, DC_PRED] (DC_PRED only
 * once): intra prediction, encode_tx_block with the intra quantizer, no
 * skip variant; strict `<` against the inter winner's cost.  A winner's
 * reconstruction and levels replace the inter winner's. */
#define INTRA_C 1000 /* result word of an intra winner: 1000 + 16 * luma + chroma mode */

/* get_intra_edges of plane p (0 luma) for superblock (ppx, ppy) of tile
 * geometry g; n = the transform size in that plane */
static void sb_edges(const orc_replay *r, const oplane *pl, const sbgeo *g, int ppx, int ppy,
                     int dec_x, int dec_y, int n, void *edge) {
  const int tx = (g->t0x * SB) >> dec_x, ty = (g->t0y * SB) >> dec_y;
  const int tw = (g->mi_w * 4) >> dec_x, th = (g->mi_h * 4) >> dec_y;
  const int x = (ppx >> dec_x) - tx, y = (ppy >> dec_y) - ty;
  orc_intra_edges_sb(at(pl, r->hbd, tx, ty), pl->stride, r->hbd, r->bd, tw, th, x, y, n,
                     g->tsy > 0, g->tsx > 0, edge);
}
static int variant_of(int x, int y) { return x == 0 && y == 0 ? 0 : y == 0 ? 1 : x == 0 ? 2 : 3; }

static void intra_sb(orc_replay *r, int sb) {
  const int R = r->R, hbd = r->hbd;
  const size_t px = px_of(r);
  uint64_t *w = r->words + (size_t)sb * (WPR * R + 4) + WPR * R;
  if (w[1]) return; /* the inter winner is skip: no screening */
  if (r->sb_limit > 0 && sb >= r->sb_limit) return; /* a bounded timing sample */
  const int sx = sb % r->tw, sy = sb / r->tw;
  const int ppx = (sx + r->tx0) * SB, ppy = (sy + r->ty0) * SB;
  if (ppx + SB > r->W || ppy + SB > r->H) return; /* rav1e splits it (must_split) */
  const sbgeo g = sb_geo_of(r, sb);
  const oinput *cur = &r->inputs[r->fi.display % r->n_inputs];
  oslot *S = &r->slots[r->fi.display % NSLOT];
  const int lvl = r->fi.level;
  const double lambda = r->lv[lvl].lambda;
  const int cpx = ppx >> r->xdec, cpy = ppy >> r->ydec, cn = SB >> r->xdec;
  uint16_t ey[4 * 64 + 1], eu[4 * 64 + 1], ev[4 * 64 + 1];
  sb_edges(r, &S->y, &g, ppx, ppy, 0, 0, SB, ey);
  sb_edges(r, &S->u, &g, ppx, ppy, r->xdec, r->ydec, cn, eu);
  sb_edges(r, &S->v, &g, ppx, ppy, r->xdec, r->ydec, cn, ev);
  const int lx = ppx - g.t0x * SB, ly_ = ppy - g.t0y * SB;
  const int var = variant_of(lx, ly_), cvar = variant_of(lx >> r->xdec, ly_ >> r->ydec);
  /* screening: RAV1E_INTRA_MODES order (src/predict.rs:32-46) */
  static const int kModes[13] = {0, 2, 1, 9, 11, 10, 12, 3, 4, 5, 6, 7, 8};
  uint32_t satd[13];
  uint16_t pb[SB * SB];
  for (int k = 0; k < 13; k++) {
    orc_predict_intra(kModes[k], var, pb, SB, SB, SB, r->bd, hbd, ey);
    satd[k] = orc_get_satd(at(&cur->y, hbd, ppx, ppy), cur->y.stride, pb, SB, SB, SB, hbd, 0);
  }
  int order[13];
  for (int k = 0; k < 13; k++) order[k] = k;
  for (int i = 1; i < 13; i++) /* stable insertion sort by satd (sort_by_key) */
    for (int j = i; j > 0 && satd[order[j]] < satd[order[j - 1]]; j--) {
      int t = order[j];
      order[j] = order[j - 1];
      order[j - 1] = t;
    }
  int modes[4], nm = 0;
  modes[nm++] = 0; /* DC_PRED: the most probable mode */
  for (int i = 0; i < 3; i++) {
    int m = kModes[order[i]], seen = 0;
    for (int j = 0; j < nm; j++) seen |= modes[j] == m;
    if (!seen) modes[nm++] = m;
  }
  if (nm > 3) nm = 3;
  /* RDO of each (luma mode, chroma mode) */
  uint64_t cb = w[2];
  double best;
  memcpy(&best, &cb, 8);
  int won = 0, bl = 0, bc = 0;
  uint64_t bd_ = 0;
  uint16_t by_[SB * SB], bu_[SB * SB], bv_[SB * SB];
  int32_t blev[1024 + 2 * 1024];
  uint16_t ly[SB * SB], lu[SB * SB], lv[SB * SB];
  int32_t lev[1024 + 2 * 1024];
  const orc_qctx *qi = r->lv[lvl].qi;
  for (int i = 0; i < nm; i++) {
    const int m = modes[i];
    orc_predict_intra(m, var, ly, SB, SB, SB, r->bd, hbd, ey);
    const uint32_t lrate = (uint32_t)tx_block_q(r, &cur->y, ppx, ppy, ly, SB, 4, 0, lev, &qi[0]);
    const int cm[2] = {m, 0};
    for (int j = 0; j < (m ? 2 : 1); j++) {
      orc_predict_intra(cm[j], cvar, lu, cn, cn, cn, r->bd, hbd, eu);
      orc_predict_intra(cm[j], cvar, lv, cn, cn, cn, r->bd, hbd, ev);
      uint32_t rate = lrate;
      rate += (uint32_t)tx_block_q(r, &cur->u, cpx, cpy, lu, cn, 3, 1, lev + 1024, &qi[1]);
      rate += (uint32_t)tx_block_q(r, &cur->v, cpx, cpy, lv, cn, 3, 2, lev + 2048, &qi[2]);
      const uint64_t d = sb_distortion(r, cur, ppx, ppy, ly, lu, lv);
      const double rd = (double)d + lambda * ((double)rate / 8.0);
      if (rd < best) {
        best = rd;
        won = 1;
        bl = m;
        bc = cm[j];
        bd_ = d;
        memcpy(by_, ly, SB * SB * px);
        memcpy(bu_, lu, (size_t)cn * cn * px);
        memcpy(bv_, lv, (size_t)cn * cn * px);
        memcpy(blev, lev, sizeof(blev));
      }
    }
  }
  __atomic_fetch_add(&r->istat[0], 1, __ATOMIC_RELAXED);
  if (!won) return;
  __atomic_fetch_add(&r->istat[1], 1, __ATOMIC_RELAXED);
  for (int y = 0; y < SB; y++)
    memcpy(at(&S->y, hbd, ppx, ppy + y), (uint8_t *)by_ + y * SB * px, SB * px);
  for (int y = 0; y < cn; y++) {
    memcpy(at(&S->u, hbd, cpx, cpy + y), (uint8_t *)bu_ + (size_t)y * cn * px, cn * px);
    memcpy(at(&S->v, hbd, cpx, cpy + y), (uint8_t *)bv_ + (size_t)y * cn * px, cn * px);
  }
  memcpy(r->lev + (size_t)sb * (1024 + 2 * r->ntx_c * 1024), blev, sizeof(blev));
  memcpy(&cb, &best, 8);
  w[0] = INTRA_C + 16 * bl + bc;
  w[1] = 0;
  w[2] = cb;
  w[3] = bd_;
}

/* The intra pass over one tile (index t of the group's tiles), raster order. */
static void intra_tile(orc_replay *r, int t) {
  const int gtx = (r->tw + r->tws - 1) / r->tws;  /* tiles across the group */
  const int tx0 = (t % gtx) * r->tws, ty0 = (t / gtx) * r->ths;
  for (int y = ty0; y < ty0 + r->ths && y < r->th; y++)
    for (int x = tx0; x < tx0 + r->tws && x < r->tw; x++) intra_sb(r, y * r->tw + x);
}

/* ---- speed 10 in coding order: rav1e's MV stacks -------------------------
 * encode_tile codes a tile's superblocks in raster order
 * (src/encoder.rs:3190-3235); rdo_mode_decision's find_mvrefs reads the
 * blocks coded before (above, left, top-right, top-left), and the 64x64
 * search's rate predictors are that stack's first two entries.  So per
 * superblock: the stacks, F3, the inter candidates (run_rdo), the intra
 * screening, and its blocks into the grid for the ones after it. */

/* the Block fields of the group grid (FrameBlocks::new: Block::default,
 * src/context.rs:1425-1442: intra, 64x64) */
static void grid_reset(orc_replay *r) {
  const size_t n = (size_t)r->tw * 16 * r->th * 16;
  const orc_blk d = {{ORC_INTRA_FRAME, ORC_INTRA_FRAME}, 16, 16, 0, {0, 0, 0}, {{0, 0}, {0, 0}}};
  for (size_t i = 0; i < n; i++) r->bgrid[i] = d;
}
/* a coded block (group 4x4 units x, y, size w4 x h4) into the grid:
 * candidate c (single: reference c / NMODE; compound: c >= C), intra if
 * c >= INTRA_C */
static void grid_set(orc_replay *r, int x, int y, int w4, int h4, int c, orc_mv m0, orc_mv m1) {
  orc_blk b;
  memset(&b, 0, sizeof(b));
  b.n4_w = (uint8_t)w4;
  b.n4_h = (uint8_t)h4;
  if (c >= INTRA_C) {
    b.ref[0] = ORC_INTRA_FRAME;
    b.ref[1] = ORC_NONE_FRAME;
  } else if (c < r->C) {
    b.ref[0] = (int8_t)(1 + c / NMODE);
    b.ref[1] = ORC_NONE_FRAME;
    b.mv[0] = m0;
    b.newmv = c % NMODE == 3; /* NEWMV (pushed only for a non-zero MV) */
  } else {
    const int m = c - r->C;
    b.ref[0] = 1;
    b.ref[1] = 2;
    b.mv[0] = m0;
    b.mv[1] = m1;
    b.newmv = m >= 2 && m <= 4; /* NEW_NEWMV, NEAREST_NEWMV, NEW_NEARESTMV */
  }
  const int gs = r->tw * 16, gh = r->th * 16;
  for (int j = y; j < y + h4 && j < gh; j++)
    for (int i = x; i < x + w4 && i < gs; i++) r->bgrid[(size_t)j * gs + i] = b;
}
/* the coded blocks of superblock sb: its 64x64 winner, or the leaves the
 * partition committed (their candidates come from the levels' stand-in) */
/* an inter block's first MV into the encode's field, under its first
 * reference (save_block_motion after the partition decision,
 * src/encoder.rs:2607-2613) */
static void save_decision(orc_replay *r, const sbgeo *g, int bx, int by, int n4, int c, orc_mv m0) {
  if (c >= INTRA_C) return;
  const int k = c < r->C ? c / NMODE : 0;
  save_motion(r, tile_field(r, r->tmv_e, k, g), g, bx, by, n4, n4, m0);
}
static void record_sb(orc_replay *r, int sb) {
  const int sx = sb % r->tw, sy = sb / r->tw;
  const sbgeo g = sb_geo_of(r, sb);
  const uint64_t *w = r->words + (size_t)sb * (WPR * r->R + 4) + WPR * r->R;
  if (!r->lvl || r->leaf0[sb]) {
    const int c = (int)w[0];
    orc_mv m0 = {0, 0}, m1 = {0, 0};
    if (c < r->C)
      (void)cand_mv(r, sb, c, &m0);
    else if (c < INTRA_C)
      comp_mvs(r, sb, c - r->C, &m0, &m1);
    grid_set(r, sx * 16, sy * 16, 16, 16, c, m0, m1);
    save_decision(r, &g, g.tsx * 16, g.tsy * 16, 16, c, m0);
    return;
  }
  int ex, ey;
  if (!in_rect(r, sb, &ex, &ey)) return;
  const sbgeo sg = g;
  for (int l = 1; l < 4; l++) {
    const struct olevel *P = &r->pl[l];
    const int k2 = 1 << l, n4 = 16 >> l;
    const cgeo g = level_geo(r, l);
    for (int j = 0; j < k2; j++)
      for (int i = 0; i < k2; i++) {
        const int b = (ey * k2 + j) * P->gw + ex * k2 + i;
        if (!P->leaf[b]) continue;
        const int c = (int)r->words[P->woff + (size_t)b * (4 * r->R + 4) + 4 * r->R];
        orc_mv m0 = {0, 0}, m1 = {0, 0};
        if (c < r->C)
          (void)cand_mv_g(&g, b, c, &m0);
        else
          comp_mvs_g(&g, b, c - r->C, &m0, &m1);
        grid_set(r, sx * 16 + i * n4, sy * 16 + j * n4, n4, n4, c, m0, m1);
        save_decision(r, &sg, sg.tsx * 16 + i * n4, sg.tsy * 16 + j * n4, n4, c, m0);
      }
  }
}
/* find_mvrefs of the 64x64 of superblock sb for every reference and, on
 * compound frames, the (ref 0, ref 1) pair (src/rdo.rs:847-943);
 * ref_frame_sign_bias: the backward references (src/encoder.rs:842-855) */
static void stacks_sb(orc_replay *r, int sb) {
  const sbgeo g = sb_geo_of(r, sb);
  const int gs = r->tw * 16;
  const orc_blk *tile = r->bgrid + (size_t)(g.t0y - r->ty0) * 16 * gs + (size_t)(g.t0x - r->tx0) * 16;
  uint8_t sbias[2] = {0, 0};
  for (int k = 0; k < r->R; k++) sbias[k] = r->fi.ref_display[k] > r->fi.display;
  struct ostk *s = &r->stk[sb];
  memset(s, 0, sizeof(*s));
  /* a superblock past the frame edge is split (must_split): its 64x64 is
   * evaluated but never coded, with empty stacks */
  if (r->lvl && edge_sb(r, sb)) return;
  orc_mv_cand st[9];
  int n;
  for (int k = 0; k < r->R; k++) {
    const int rf[2] = {1 + k, ORC_NONE_FRAME};
    orc_find_mvrefs(tile, gs, g.mi_w, g.mi_h, g.t0x * 16, g.t0y * 16, r->w_in_b, r->h_in_b,
                    g.tsx * 16, g.tsy * 16, 16, 16, rf, sbias, st, &n);
    s->n[k] = n < 2 ? n : 2;
    if (n >= 1) s->s[k][0] = st[0].this_mv;
    if (n >= 2) s->s[k][1] = st[1].this_mv;
  }
  if (r->fi.compound) {
    const int rf[2] = {1, 2};
    orc_find_mvrefs(tile, gs, g.mi_w, g.mi_h, g.t0x * 16, g.t0y * 16, r->w_in_b, r->h_in_b,
                    g.tsx * 16, g.tsy * 16, 16, 16, rf, sbias, st, &n);
    for (int i = 0; i < 2; i++) {
      s->c[i][0] = st[i].this_mv;
      s->c[i][1] = st[i].comp_mv;
    }
  }
}
/* one tile (index t of the group's tiles) in raster order */
static void chain_tile(orc_replay *r, int t, uint64_t tail[3]) {
  const int gtx = (r->tw + r->tws - 1) / r->tws;
  const int tx0 = (t % gtx) * r->tws, ty0 = (t / gtx) * r->ths;
  for (int y = ty0; y < ty0 + r->ths && y < r->th; y++)
    for (int x = tx0; x < tx0 + r->tws && x < r->tw; x++) {
      const int sb = y * r->tw + x;
      if (r->sb_limit > 0 && sb >= r->sb_limit) continue; /* a bounded timing sample */
      half_sb(r, sb, r->tmv_e, r->half, r->hc, 1);  /* build_half_res_pmvs (encode) */
      stacks_sb(r, sb);
      me64_sb(r, sb);
      run_rdo(r, sb, tail);
      if (r->intra) intra_sb(r, sb);
      record_sb(r, sb);
    }
}

void orc_replay_intra_stats(const orc_replay *r, uint64_t out[2]) {
  out[0] = r->istat[0];
  out[1] = r->istat[1];
}

int orc_replay_set_intra(orc_replay *r, int on) {
  r->intra = on != 0 && !r->s6 && r->xdec == 1 && r->ydec == 1;
  return r->intra == (on != 0) ? 0 : -1;
}

/* ---- coefficient entropy coding of the committed frame ------------------
 * encode_tile's superblock loop (src/encoder.rs:3160-3340) down to the
 * transform blocks (write_tx_tree for inter leaves, :1907-2030;
 * write_tx_blocks for the intra superblocks, :1757-1906), coefficient
 * syntax only: per tile, a fresh BlockContext and range coder from the
 * frame's initial CDFs; reset_left_contexts at every superblock row; per
 * superblock the committed partition's leaves in z-order
 * (encode_partition_topdown, :2392-2470); a skip leaf resets its coefficient
 * contexts (encode_block_post_cdef, :1499-1501), a coded leaf writes its
 * luma block, then U, then V (write_coeffs_lv_map, src/context.rs:3965).
 * The frame's CDFs: get_initial_cdfcontext (:2750-2761) -- the primary
 * reference LAST3 is the previous frame of the same pyramid level
 * (:776-830) -- and the biggest tile's CDFs with reset_counts
 * (:2824-2833; Iterator::max_by_key keeps the last maximum). */
typedef struct {
  orc_ec_job *j;
  int32_t *c;
  size_t nj, cj, nc, cc;
} ec_list;

static void ec_push(ec_list *L, orc_ec_job jb, const int32_t *co, int n) {
  if (L->nj == L->cj) {
    L->cj = L->cj ? 2 * L->cj : 1024;
    L->j = realloc(L->j, L->cj * sizeof(orc_ec_job));
  }
  if (co) {
    if (L->nc + (size_t)n > L->cc) {
      while (L->nc + (size_t)n > L->cc) L->cc = L->cc ? 2 * L->cc : 65536;
      L->c = realloc(L->c, L->cc * 4);
    }
    jb.coeff_off = (int32_t)L->nc;
    memcpy(L->c + L->nc, co, (size_t)n * 4);
    L->nc += (size_t)n;
  }
  L->j[L->nj++] = jb;
}

/* the committed levels of a leaf of log2 size lg at luma 4x4 (x4, y4) of the
 * frame: plane p's coefficients of chroma transform t */
static const int32_t *ec_coeffs(const orc_replay *r, int lg, int x4, int y4, int p, int t) {
  const int l = 6 - lg;
  if (l == 0) {
    const int sb = (y4 / 16 - r->ty0) * r->tw + (x4 / 16 - r->tx0);
    const int32_t *b = r->lev + (size_t)sb * (1024 + 2 * r->ntx_c * 1024);
    return p == 0 ? b : b + 1024 + ((size_t)(p - 1) * r->ntx_c + t) * 1024;
  }
  const struct olevel *P = &r->pl[l];
  const int n4 = 16 >> l;
  const int bi = (y4 / n4 - P->ty0) * P->gw + (x4 / n4 - P->tx0);
  const size_t per = (size_t)P->B * P->B + 2 * (size_t)P->bc * P->bch;
  const int32_t *b = P->lev + (size_t)bi * per;
  return p == 0 ? b : b + (size_t)P->B * P->B + (size_t)(p - 1) * P->bc * P->bch;
}

static void ec_walk(const orc_replay *r, ec_list *L, int x4, int y4, int lg, int t0x4, int t0y4) {
  if (x4 >= r->mi_cols || y4 >= r->mi_rows) return;
  const int code = r->mi_lg[(size_t)y4 * r->mi_cols + x4];
  if (code != lg - 2 && lg > 3) {  /* 8x8 is the smallest partition */
    const int h = 1 << (lg - 3);
    ec_walk(r, L, x4, y4, lg - 1, t0x4, t0y4);
    ec_walk(r, L, x4 + h, y4, lg - 1, t0x4, t0y4);
    ec_walk(r, L, x4, y4 + h, lg - 1, t0x4, t0y4);
    ec_walk(r, L, x4 + h, y4 + h, lg - 1, t0x4, t0y4);
    return;
  }
  const int bx = x4 - t0x4, by = y4 - t0y4;
  if (r->mi_skip[(size_t)y4 * r->mi_cols + x4]) {
    orc_ec_job jb = {1, 0, bx, by, 0, 0, 0, lg, lg, 0};
    ec_push(L, jb, NULL, 0);
    return;
  }
  int inter = 1;
  if (lg == 6) {
    const int sb = (y4 / 16 - r->ty0) * r->tw + (x4 / 16 - r->tx0);
    inter = r->words[(size_t)sb * (WPR * r->R + 4) + WPR * r->R] < INTRA_C;
  }
  const int ltx = lg - 2 < 4 ? lg - 2 : 4, lcw = ltx == 4 ? 32 : 4 << ltx;
  orc_ec_job jl = {0, 0, bx, by, ltx, 0, inter, lg, lg, 0};
  ec_push(L, jl, ec_coeffs(r, lg, x4, y4, 0, 0), lcw * lcw);
  const int plg = lg - r->xdec;  /* xdec == ydec */
  const int n_tx = plg == 6 ? 4 : 1;
  const int ctx_ = plg == 6 ? 3 : plg - 2, ccw = ctx_ == 4 ? 32 : 4 << ctx_;
  for (int p = 1; p < 3; p++)
    for (int t = 0; t < n_tx; t++) {
      orc_ec_job jc = {0, p, bx + (n_tx == 4 ? (t % 2) * 8 : 0), by + (n_tx == 4 ? (t / 2) * 8 : 0),
                       ctx_, 0, inter, plg, plg, 0};
      ec_push(L, jc, ec_coeffs(r, lg, x4, y4, p, t), ccw * ccw);
    }
}

static int ec_qctx(int q) { return q <= 20 ? 0 : q <= 60 ? 1 : q <= 120 ? 2 : 3; }

static void entropy_frame(orc_replay *r) {
  const int lv = r->fi.level;
  uint16_t init[ORC_EC_CDF_TOTAL];
  if (r->ec_chain[lv])
    memcpy(init, r->ec_chain[lv], sizeof(init));
  else
    memcpy(init, orc_ec_default_cdf(ec_qctx(r->lv[lv].qidx)), sizeof(init));
  const int ntx = (r->tw + r->tws - 1) / r->tws, nty = (r->th + r->ths - 1) / r->ths;
  uint64_t total = 0, h = 1469598103934665603ull;
  long best = -1;
  uint16_t *best_cdf = malloc(sizeof(init)), *cdf = malloc(sizeof(init));
  for (int ty = 0; ty < nty; ty++)
    for (int tx = 0; tx < ntx; tx++) {
      ec_list L = {0};
      const int sx0 = r->tx0 + tx * r->tws, sy0 = r->ty0 + ty * r->ths;
      const int sx1 = sx0 + r->tws < r->tx0 + r->tw ? sx0 + r->tws : r->tx0 + r->tw;
      const int sy1 = sy0 + r->ths < r->ty0 + r->th ? sy0 + r->ths : r->ty0 + r->th;
      orc_ec_job j3 = {3, 0, 0, 0, 0, 0, 0, 0, 0, 0}, j2 = {2, 0, 0, 0, 0, 0, 0, 0, 0, 0};
      ec_push(&L, j3, NULL, 0);
      for (int sy = sy0; sy < sy1; sy++) {
        ec_push(&L, j2, NULL, 0);
        for (int sx = sx0; sx < sx1; sx++) ec_walk(r, &L, sx * 16, sy * 16, 6, sx0 * 16, sy0 * 16);
      }
      const long cap = (long)(L.nc * 4 + L.nj * 16 + 4096);
      uint8_t *out = malloc((size_t)cap);
      int32_t tb[2] = {0, 0};
      const long nb = orc_ec_code_jobs(L.j, (int)L.nj, L.c, init, r->xdec, r->ydec, out, cap, tb,
                                       NULL, cdf);
      for (long i = 0; i < nb; i++) h = (h ^ out[i]) * 1099511628211ull;
      total += (uint64_t)(nb > 0 ? nb : 0);
      if (nb >= best) {
        best = nb;
        memcpy(best_cdf, cdf, sizeof(init));
      }
      free(out);
      free(L.j);
      free(L.c);
    }
  orc_ec_reset_counts(best_cdf);
  free(r->ec_chain[lv]);
  r->ec_chain[lv] = best_cdf;
  free(cdf);
  r->ec_stat[0] = total;
  r->ec_stat[1] = (uint64_t)(ntx * nty);
  r->ec_stat[2] = h;
  r->ec_stat[3]++;
}

/* Coefficient entropy coding of every coded frame; xdec == ydec.  With
 * several tile groups each codes its own tiles and keeps its own biggest
 * tile's CDFs (rav1e: the frame's; exact with one group). */
int orc_replay_set_entropy(orc_replay *r, int on) {
  if (on && r->xdec != r->ydec) return -1;
  r->entropy = on != 0;
  if (r->entropy && !r->mi_lg) {
    r->mi_cols = (r->W + 3) / 4;
    r->mi_rows = (r->H + 3) / 4;
    r->mi_lg = malloc((size_t)r->mi_cols * r->mi_rows);
    r->mi_skip = calloc((size_t)r->mi_cols * r->mi_rows, 1);
    if (!r->mi_lg || !r->mi_skip) return -1;
    memset(r->mi_lg, 4, (size_t)r->mi_cols * r->mi_rows);  /* 64x64 until written */
  }
  return 0;
}

/* [bytes, tiles, FNV-1a 64 of the tiles' bytes in order, frames coded] of
 * the last frame */
void orc_replay_entropy_stats(const orc_replay *r, uint64_t out[4]) {
  memcpy(out, r->ec_stat, sizeof(r->ec_stat));
}

static void *worker(void *arg) {
  orc_replay *r = arg;
  uint64_t tail[3] = {0, 0, 0};
  int lim = r->sb_limit > 0 && r->sb_limit < r->nsb ? r->sb_limit : r->nsb;
  if (r->pass >= 4) /* the group's tiles (passes 4, 5, 6) */
    lim = ((r->tw + r->tws - 1) / r->tws) * ((r->th + r->ths - 1) / r->ths);
  for (;;) {
    pthread_mutex_lock(&r->mu);
    int sb = r->next_sb++;
    pthread_mutex_unlock(&r->mu);
    if (sb >= lim) break;
    if (r->pass == 0)
      run_coarse(r, sb);
    else if (r->pass == 2)
      run_me(r, sb);
    else if (r->pass == 3)
      run_rdo(r, sb, tail);
    else if (r->pass == 4)
      intra_tile(r, sb); /* passes 4, 5, 6: `sb` counts tiles */
    else if (r->pass == 5)
      chain_tile(r, sb, tail);
    else
      lookahead_tile(r, sb);
  }
  pthread_mutex_lock(&r->mu);
  for (int i = 0; i < 3; i++) r->tail[i] += tail[i];
  pthread_mutex_unlock(&r->mu);
  return NULL;
}

static void free_la(orc_replay *r) {
  if (!r->la) return;
  for (int i = 0; i <= r->imp_window; i++) {
    ola *e = &r->la[i];
    free(e->coarse);
    free(e->half_l);
    free(e->look);
    free(e->cc);
    free(e->hlc);
    free(e->lc);
    free(e->intra);
    free(e->mv8);
    free(e->inter);
    free(e->imp);
  }
  free(r->la);
  r->la = NULL;
}

static void run_pass(orc_replay *r, int pass) {
  r->pass = pass;
  r->next_sb = 0;
  pthread_t th[256];
  int nt = r->threads < 256 ? r->threads : 256;
  for (int i = 0; i < nt; i++) pthread_create(&th[i], NULL, worker, r);
  for (int i = 0; i < nt; i++) pthread_join(th[i], NULL);
}

/* Coding order of the reorder pyramid (rv_replay.hip frame_info). */
static void frame_info(long n, int R, orc_frame_info *f) {
  memset(f, 0, sizeof(*f));
  if (n == 0) {
    f->is_key = 1;
    return;
  }
  long g = (n - 1) / 4, j = (n - 1) % 4;
  static const int off[4] = {4, 2, 1, 3}, scale[4] = {4, 2, 1, 1};
  static const int rf[4][2] = {{0, -4}, {0, 4}, {0, 2}, {2, 4}};
  f->display = (int)(4 * g + off[j]);
  f->me_range_scale = scale[j];
  f->level = j == 0 ? 0 : j == 1 ? 1 : 2;
  for (int k = 0; k < R; k++) {
    long d = 4 * g + rf[j][k];
    f->ref_display[k] = (int)(d < 0 ? 0 : d);
  }
  /* reference_mode SELECT with a forward and a backward reference
   * (src/encoder.rs:832-836, src/rdo.rs:914-941) */
  f->compound = R == 2 && (j == 1 || j == 3);
}

/* ---- block importances over the lookahead window (rdo_lookahead_frames) --
 * compute_lookahead_data (src/api/internal.rs:767-820) runs the lookahead of
 * every frame as it arrives, far ahead of its encode; compute_block_importances
 * (:823-1081) then propagates over the window [n, n + W] of coded frames.
 * Here frame m's lookahead (F1, F2L, FL -- it reads only the inputs) runs
 * once, W frames before m is coded, into ring entry m % (W + 1), with what
 * the propagation reads of it: lookahead_intra_costs, the 8x8 blocks'
 * lookahead MVs ([2y][2x] of the field: the FL MV of the 16x16 holding the
 * block) and their get_satd against each reference's original frame. */

/* the coded index of display d (inverse of frame_info) */
static long coded_of_display(long d) {
  if (d == 0) return 0;
  static const int jof[4] = {0, 2, 1, 3}, off[4] = {4, 2, 1, 3};
  const int j = jof[d % 4];
  return 4 * ((d - off[j]) / 4) + j + 1;
}

static ola *la_of(orc_replay *r, long m) { return &r->la[m % (r->imp_window + 1)]; }

/* this group's 8x8 importance blocks [x0, x1) x [y0, y1) */
static void group_blocks(const orc_replay *r, int *x0, int *y0, int *x1, int *y1) {
  *x0 = r->tx0 * 8;
  *y0 = r->ty0 * 8;
  *x1 = (r->tx0 + r->tw) * 8 < r->w_imp ? (r->tx0 + r->tw) * 8 : r->w_imp;
  *y1 = (r->ty0 + r->th) * 8 < r->h_imp ? (r->ty0 + r->th) * 8 : r->h_imp;
}

/* orc_la_refs of coded frame m >= 1 (frame_info's group g, position j) */
static orc_la_refs la_refs_of(long m, int R) {
  orc_la_refs l;
  memset(&l, 0, sizeof(l));
  orc_frame_info f;
  frame_info(m, R, &f);
  for (int k = 0; k < R; k++) {
    l.disp[k] = f.ref_display[k];
    l.order[k] = k;
  }
  l.n = R;
  const long g = (m - 1) / 4, j = (m - 1) % 4;
  if (R == 2 && j > 0) {
    /* LAST3: the previous frame of this level (4g+2: 4g-2; 4g+1: 4g-1, the
     * last level-2 frame of group g-1; 4g+3: 4g+1), the key frame before */
    const long d3 = j == 1 ? 4 * g - 2 : j == 2 ? 4 * g - 1 : 4 * g + 1;
    l.disp[2] = (int)(d3 < 0 ? 0 : d3);
    l.n = 3;
    l.order[0] = 0;  /* LAST (the backward reference) */
    l.order[1] = 2;  /* LAST3 */
    l.order[2] = 1;  /* ALTREF (the forward reference) */
  }
  return l;
}

static void la_compute(orc_replay *r, long m) {
  const orc_frame_info save = r->fi;
  const int save_lim = r->sb_limit;
  frame_info(m, r->R, &r->fi);
  r->sb_limit = 0;
  r->lar = la_refs_of(m, r->R);
  r->la_mode = 1;
  const int RL = r->lar.n;
  const size_t nr = (size_t)RL * r->nsb;
  input_pyr(r, r->fi.display);
  for (int k = 0; k < RL; k++) input_pyr(r, r->lar.disp[k]);
  memset(r->tmv_l, 0, (size_t)RL * r->tw * 16 * r->th * 16 * sizeof(orc_mv));
  run_pass(r, 0);
  run_pass(r, 6);
  r->la_mode = 0;
  ola *e = la_of(r, m);
  e->coded = m;
  e->fi = r->fi;
  e->lr = r->lar;
  memcpy(e->coarse, r->coarse, nr * sizeof(orc_mv));
  memcpy(e->cc, r->cc, nr * 8);
  memcpy(e->half_l, r->half_l, nr * 4 * sizeof(orc_mv));
  memcpy(e->hlc, r->hlc, nr * 4 * 8);
  memcpy(e->look, r->look, nr * 16 * sizeof(orc_mv));
  memcpy(e->lc, r->lc, nr * 16 * 8);
  const int w = r->w_imp, h = r->h_imp, hbd = r->hbd;
  const size_t ni = (size_t)w * h;
  const oinput *cur = &r->inputs[r->fi.display % r->n_inputs];
  /* the group's 8x8 blocks (the whole frame with one group) */
  int bx0, by0, bx1, by1;
  group_blocks(r, &bx0, &by0, &bx1, &by1);
  for (int y = by0; y < by1; y++)
    for (int x = bx0; x < bx1; x++) {
      orc_lookahead_intra_costs(at(&cur->y, hbd, x * 8, y * 8), cur->y.stride, 8, 8, hbd, r->bd,
                                &e->intra[(size_t)y * w + x]);
      const int sb = (y / 8 - r->ty0) * r->tw + x / 8 - r->tx0, b = ((y % 8) / 2) * 4 + (x % 8) / 2;
      for (int k = 0; k < RL; k++) {
        const orc_mv mv = r->look[((size_t)k * r->nsb + sb) * 16 + b];
        e->mv8[k * ni + (size_t)y * w + x] = mv;
        /* get_satd against the reference block at the MV (:902-931; the
         * region at (x * 64 + mv.col) / 8, isize `/`), as
         * orc_importance_inter_costs does for a whole frame */
        const oplane *ref = &r->inputs[r->lar.disp[k] % r->n_inputs].y;
        const int64_t px_x = ((int64_t)x * 64 + mv.col) / 8, px_y = ((int64_t)y * 64 + mv.row) / 8;
        e->inter[k * ni + (size_t)y * w + x] =
            orc_get_satd(at(&cur->y, hbd, x * 8, y * 8), cur->y.stride,
                         at(ref, hbd, (int)px_x, (int)px_y), ref->stride, 8, 8, hbd, 0);
      }
    }
  r->fi = save;
  r->sb_limit = save_lim;
}

/* the last coded frame whose lookahead frame n = r->coded needs: n + W,
 * or the stream's last frame */
static long la_last(const orc_replay *r) {
  long last = r->coded + r->imp_window;
  if (r->la_limit > 0 && last > r->la_limit - 1) last = r->la_limit - 1;
  return last;
}

/* the lookahead of every frame up to n + W (n: the frame being coded) */
static void la_fill(orc_replay *r) {
  const long last = la_last(r);
  for (; r->la_next <= last; r->la_next++) la_compute(r, r->la_next);
}

/* ---- a tile group's window (la_ext) ------------------------------------------
 * Each group computes the lookahead of its own superblocks (the searches
 * are tile-local) and the importance data of its own 8x8 blocks; the
 * caller all-gathers the groups' parts (the importance propagation reads
 * the whole frame) and imports them; then frame() propagates over the
 * whole frame, exactly as a one-group replay does.  A part: per block of
 * the group's rectangle in raster order, the intra cost, then per
 * reference slot k < 3 the lookahead MV and the inter cost (28 bytes). */
#define LA_PART_B 28
static size_t la_part_bytes(int bw, int bh) { return (size_t)bw * bh * LA_PART_B; }

/* the 8x8 importance blocks [x0, x1) x [y0, y1) of a superblock rectangle */
static void sb_rect_blocks(const orc_replay *r, int tx0, int ty0, int tw, int th, int *x0, int *y0,
                           int *x1, int *y1) {
  *x0 = tx0 * 8;
  *y0 = ty0 * 8;
  *x1 = (tx0 + tw) * 8 < r->w_imp ? (tx0 + tw) * 8 : r->w_imp;
  *y1 = (ty0 + th) * 8 < r->h_imp ? (ty0 + th) * 8 : r->h_imp;
}

/* (next, last): the next coded frame whose group part is due and the last
 * one frame() of the next frame needs; out[2] = the part's bytes */
int orc_replay_la_due(orc_replay *r, long *out) {
  if (!r->imp_window || !r->la_ext) return -1;
  int x0, y0, x1, y1;
  sb_rect_blocks(r, r->tx0, r->ty0, r->tw, r->th, &x0, &y0, &x1, &y1);
  out[0] = r->la_next;
  out[1] = la_last(r);
  out[2] = (long)la_part_bytes(x1 - x0, y1 - y0);
  return 0;
}

static void la_pack(const orc_replay *r, const ola *e, int x0, int y0, int x1, int y1,
                    uint8_t *buf, int unpack, ola *dst) {
  const size_t ni = (size_t)r->w_imp * r->h_imp;
  for (int y = y0; y < y1; y++)
    for (int x = x0; x < x1; x++) {
      uint8_t *p = buf + ((size_t)(y - y0) * (x1 - x0) + (x - x0)) * LA_PART_B;
      const size_t i = (size_t)y * r->w_imp + x;
      if (!unpack) {
        memset(p, 0, LA_PART_B);
        memcpy(p, &e->intra[i], 4);
        for (int k = 0; k < e->lr.n; k++) {
          memcpy(p + 4 + 8 * k, &e->mv8[k * ni + i], 4);
          memcpy(p + 8 + 8 * k, &e->inter[k * ni + i], 4);
        }
      } else {
        memcpy(&dst->intra[i], p, 4);
        for (int k = 0; k < dst->lr.n; k++) {
          memcpy(&dst->mv8[k * ni + i], p + 4 + 8 * k, 4);
          memcpy(&dst->inter[k * ni + i], p + 8 + 8 * k, 4);
        }
      }
    }
}

/* coded frame m's group part (m = the next due): its lookahead, then the
 * part of this group's blocks into buf (la_due's bytes) */
int orc_replay_la_group(orc_replay *r, long m, uint8_t *buf) {
  if (!r->imp_window || !r->la_ext || m != r->la_next) return -1;
  la_compute(r, m);
  r->la_next++;
  int x0, y0, x1, y1;
  sb_rect_blocks(r, r->tx0, r->ty0, r->tw, r->th, &x0, &y0, &x1, &y1);
  la_pack(r, la_of(r, m), x0, y0, x1, y1, buf, 0, NULL);
  return 0;
}

/* another group's part of coded frame m (its superblock rectangle) */
int orc_replay_la_import(orc_replay *r, long m, int tx0, int ty0, int tw, int th,
                         const uint8_t *buf) {
  if (!r->imp_window || !r->la_ext || m >= r->la_next) return -1;
  ola *e = la_of(r, m);
  if (e->coded != m) return -1;
  int x0, y0, x1, y1;
  sb_rect_blocks(r, tx0, ty0, tw, th, &x0, &y0, &x1, &y1);
  la_pack(r, e, x0, y0, x1, y1, (uint8_t *)buf, 1, e);
  return 0;
}

/* compute_block_importances for frame n = r->coded: zero the window's
 * importances, propagate from its last frame down to n + 1 (each frame's
 * distinct reference slots in mv index order, orc_la_refs, the split by
 * their count -- two slots may hold one frame, e.g. the key frame; targets
 * before n are outside the window and gone, :944-948), then log2(1 +
 * importance / intra cost) for frame n (:1052-1070). */
static void importance_frame(orc_replay *r) {
  const long n = r->coded, last = r->la_next - 1;
  const int w = r->w_imp, h = r->h_imp;
  const size_t ni = (size_t)w * h;
  for (long m = n; m <= last; m++) memset(la_of(r, m)->imp, 0, ni * sizeof(float));
  for (long m = last; m > n; m--) {
    const ola *e = la_of(r, m);
    if (e->fi.is_key) continue;
    const int nu = e->lr.n;
    for (int j = 0; j < nu; j++) {
      const int k = e->lr.order[j];
      const long mref = coded_of_display(e->lr.disp[k]);
      if (mref < n) continue;
      orc_propagate_importances_costs(w, h, e->mv8 + k * ni, e->inter + k * ni, e->intra, e->imp,
                                      nu, la_of(r, mref)->imp);
    }
  }
  const ola *c = la_of(r, n);
  for (size_t i = 0; i < ni; i++) {
    const float intra = (float)c->intra[i];
    r->imp_own[i] = intra > 0.f ? orc_log2f(1.f + c->imp[i] / intra) : 0.f;
  }
}

/* The window W (rdo_lookahead_frames; 0: the importances are an input,
 * orc_replay_set_importances) and the stream's length in coded frames
 * (limit; 0: unbounded -- the inputs of frame n + W must be set before
 * frame n is coded).  Only before the first frame, and only for a replay of
 * the whole frame (a group's importances would need the other groups'). */
int orc_replay_set_imp_window(orc_replay *r, int window, long limit) {
  if (window < 0 || r->coded > 0) return -1;
  /* a tile group's window needs the other groups' parts (la_ext) */
  r->la_ext = r->tx0 || r->ty0 || r->vis_w != r->W || r->vis_h != r->H;
  free_la(r);
  free(r->imp_own);
  r->imp_own = NULL;
  r->imp_window = 0;
  r->la_limit = limit;
  r->la_next = 1;
  if (!window) return 0;
  const size_t nr = (size_t)r->RA * r->nsb, ni = (size_t)r->w_imp * r->h_imp;
  r->la = calloc((size_t)window + 1, sizeof(ola));
  r->imp_own = calloc(ni, sizeof(float));
  if (!r->la || !r->imp_own) return -1;
  r->imp_window = window;
  for (int i = 0; i <= window; i++) {
    ola *e = &r->la[i];
    e->coded = -1;
    e->coarse = calloc(nr, sizeof(orc_mv));
    e->cc = calloc(nr, 8);
    e->half_l = calloc(nr * 4, sizeof(orc_mv));
    e->hlc = calloc(nr * 4, 8);
    e->look = calloc(nr * 16, sizeof(orc_mv));
    e->lc = calloc(nr * 16, 8);
    e->intra = calloc(ni, 4);
    e->mv8 = calloc(ni * r->RA, sizeof(orc_mv));
    e->inter = calloc(ni * r->RA, 4);
    e->imp = calloc(ni, 4);
    if (!e->coarse || !e->cc || !e->half_l || !e->hlc || !e->look || !e->lc || !e->intra ||
        !e->mv8 || !e->inter || !e->imp)
      return -1;
  }
  return 0;
}

/* ring entry of coded frame m (tests): its intra costs [h_imp][w_imp], 8x8
 * lookahead MVs and inter costs [n][h_imp][w_imp] of its lookahead
 * references, and refs[0] = n, refs[1..3] their displays (k order),
 * refs[4..6] the propagation order; -1: absent */
int orc_replay_la_data(orc_replay *r, long m, uint32_t *intra, orc_mv *mv8, uint32_t *inter,
                       int32_t *refs) {
  if (!r->imp_window || m < 1) return -1;
  const ola *e = la_of(r, m);
  if (e->coded != m) return -1;
  const size_t ni = (size_t)r->w_imp * r->h_imp;
  memcpy(intra, e->intra, ni * 4);
  memcpy(mv8, e->mv8, ni * e->lr.n * sizeof(orc_mv));
  memcpy(inter, e->inter, ni * e->lr.n * 4);
  refs[0] = e->lr.n;
  for (int k = 0; k < 3; k++) {
    refs[1 + k] = k < e->lr.n ? e->lr.disp[k] : -1;
    refs[4 + k] = k < e->lr.n ? e->lr.order[k] : -1;
  }
  return 0;
}

/* the orc_la_refs of coded frame m >= 1 (tests): out[0] = n, out[1..3] the
 * displays in k order, out[4..6] the propagation order (-1: unused) */
int orc_replay_la_refs(long m, int R, int32_t *out) {
  if (m < 1 || R < 1 || R > 2) return -1;
  const orc_la_refs l = la_refs_of(m, R);
  out[0] = l.n;
  for (int k = 0; k < 3; k++) {
    out[1 + k] = k < l.n ? l.disp[k] : -1;
    out[4 + k] = k < l.n ? l.order[k] : -1;
  }
  return 0;
}

/* frame n's importances (the window's, or the input's) for a caller */
int orc_replay_get_importances(orc_replay *r, float *out, int n) {
  if (n != r->w_imp * r->h_imp) return -1;
  const float *imp = r->imp_window ? r->imp_own : r->imp;
  if (imp)
    memcpy(out, imp, (size_t)n * 4);
  else
    memset(out, 0, (size_t)n * 4);
  return 0;
}

/* Code the next frame.  sb_limit > 0 runs only the first sb_limit
 * superblocks of both passes (a bounded sample for timing).  pad_recon = 0
 * leaves the padding to orc_replay_import (tile groups). */
int orc_replay_frame(orc_replay *r, orc_frame_info *info, int sb_limit, int pad_recon) {
  frame_info(r->coded, r->R, &r->fi);
  if (info) *info = r->fi;
  if (r->fi.is_key) {
    oinput *in = &r->inputs[0];
    oslot *s = &r->slots[0];
    memcpy(s->y.mem, in->y.mem, plane_size(&in->y, r->hbd));
    memcpy(s->u.mem, in->u.mem, plane_size(&in->u, r->hbd));
    memcpy(s->v.mem, in->v.mem, plane_size(&in->v, r->hbd));
    /* an intra frame saves no motion: its field stays zero */
    memset(s->fmv, 0, (size_t)r->R * r->w_in_b * r->h_in_b * sizeof(orc_mv));
    r->coded++;
    return 0;
  }
  if (!r->lv[0].set || !r->lv[1].set || !r->lv[2].set) return -1;
  oslot *S = &r->slots[r->fi.display % NSLOT];
  input_pyr(r, r->fi.display);
  for (int k = 0; k < r->R; k++) input_pyr(r, r->fi.ref_display[k]);
  memset(r->tail, 0, sizeof(r->tail));
  r->sb_limit = sb_limit;
  r->istat[0] = r->istat[1] = 0;
  /* the tile fields start at zero (FrameState::new_with_frame) */
  const size_t nf = (size_t)r->R * r->tw * 16 * r->th * 16;
  memset(r->tmv_e, 0, nf * sizeof(orc_mv));
  memset(r->tmv_l, 0, nf * sizeof(orc_mv));
  /* F1; the lookahead (its F2 and 16x16 searches, tile by tile) -- with
   * an importance window, run W frames ahead and kept in the ring */
  if (r->imp_window) {
    if (!r->la_ext)
      la_fill(r);
    else if (r->la_next <= la_last(r))
      return -1; /* a group's parts are due first (orc_replay_la_due) */
    const ola *e = la_of(r, r->coded);
    if (e->coded != r->coded) return -1; /* the stream ended before this frame */
    const size_t nr = (size_t)r->R * r->nsb;
    memcpy(r->coarse, e->coarse, nr * sizeof(orc_mv));
    memcpy(r->cc, e->cc, nr * 8);
    memcpy(r->half_l, e->half_l, nr * 4 * sizeof(orc_mv));
    memcpy(r->hlc, e->hlc, nr * 4 * 8);
    memcpy(r->look, e->look, nr * 16 * sizeof(orc_mv));
    memcpy(r->lc, e->lc, nr * 16 * 8);
    importance_frame(r);
  } else {
    run_pass(r, 0);
    run_pass(r, 6);
  }
  if (r->exact) {
    /* speed 10: the levels' searches, then each tile in coding order (F2,
     * F3, F4, F6, F6b per superblock) */
    run_pass(r, 2);
    grid_reset(r);
    run_pass(r, 5);
    /* the encode's field becomes the frame's frame_mvs (the group's part) */
    for (int k = 0; k < r->R; k++)
      for (int y = 0; y < r->th * 16 && r->ty0 * 16 + y < r->h_in_b; y++)
        for (int x = 0; x < r->tw * 16 && r->tx0 * 16 + x < r->w_in_b; x++)
          S->fmv[((size_t)k * r->h_in_b + r->ty0 * 16 + y) * r->w_in_b + r->tx0 * 16 + x] =
              r->tmv_e[((size_t)k * r->th * 16 + y) * r->tw * 16 + x];
  } else {
    /* speed 6 / the MV-stack stand-in: the encode's half-res quadrants are
     * the lookahead's (no coding-order field) */
    memcpy(r->half, r->half_l, (size_t)r->R * r->nsb * 4 * sizeof(orc_mv));
    memcpy(r->hc, r->hlc, (size_t)r->R * r->nsb * 4 * 8);
    for (int pass = 2; pass < 4; pass++) run_pass(r, pass);
    if (r->intra) run_pass(r, 4);
  }
  if (r->deblock || r->entropy) map_own(r);
  if (r->lrf && lrf_decide(r) != 0) return -1;
  if (r->entropy) entropy_frame(r);
  if (r->deblock && pad_recon) loop_filter_planes(r);  /* tile groups: after the imports */
  r->tail[3] = (uint64_t)(r->vis_w / 8) * (r->vis_h / 8);
  if (pad_recon) {
    pad(r, &S->y);
    pad(r, &S->u);
    pad(r, &S->v);
  }
  r->coded++;
  return 0;
}

/* The group's visible rectangle of plane p (x0, y0, w, h). */
static void group_rect(const orc_replay *r, int p, const int32_t *gr, int out[4]) {
  int xd = p ? r->xdec : 0, yd = p ? r->ydec : 0;
  int pw = p ? (r->W + r->xdec) >> r->xdec : r->W, ph = p ? (r->H + r->ydec) >> r->ydec : r->H;
  int x0 = (gr[0] * SB) >> xd, y0 = (gr[1] * SB) >> yd;
  int x1 = ((gr[0] + gr[2]) * SB) >> xd, y1 = ((gr[1] + gr[3]) * SB) >> yd;
  out[0] = x0;
  out[1] = y0;
  out[2] = (x1 < pw ? x1 : pw) - x0;
  out[3] = (y1 < ph ? y1 : ph) - y0;
}

/* Pack (to_buf = 1) or unpack group `gr`'s region of the last coded frame
 * (Y, U, V rows, tightly packed); returns the bytes. */
int64_t orc_replay_xcopy(orc_replay *r, const int32_t *gr, void *buf, int to_buf) {
  oslot *s = &r->slots[r->fi.display % NSLOT];
  oplane *pl[3] = {&s->y, &s->u, &s->v};
  size_t px = px_of(r);
  uint8_t *b = buf;
  int64_t off = 0;
  for (int p = 0; p < 3; p++) {
    int rc[4];
    group_rect(r, p, gr, rc);
    for (int y = 0; y < rc[3]; y++) {
      uint8_t *q = at(pl[p], r->hbd, rc[0], rc[1] + y);
      if (b) {
        if (to_buf)
          memcpy(b + off, q, (size_t)rc[2] * px);
        else
          memcpy(q, b + off, (size_t)rc[2] * px);
      }
      off += (int64_t)rc[2] * px;
    }
  }
  if (r->exact) { /* the group's part of the frame's motion field, per reference */
    const int x0 = gr[0] * 16, y0 = gr[1] * 16;
    const int x1 = (gr[0] + gr[2]) * 16 < r->w_in_b ? (gr[0] + gr[2]) * 16 : r->w_in_b;
    const int y1 = (gr[1] + gr[3]) * 16 < r->h_in_b ? (gr[1] + gr[3]) * 16 : r->h_in_b;
    for (int k = 0; k < r->R; k++)
      for (int y = y0; y < y1; y++) {
        orc_mv *q = s->fmv + ((size_t)k * r->h_in_b + y) * r->w_in_b + x0;
        const size_t nb = (size_t)(x1 - x0) * sizeof(orc_mv);
        if (b) {
          if (to_buf)
            memcpy(b + off, q, nb);
          else
            memcpy(q, b + off, nb);
        }
        off += (int64_t)nb;
      }
  }
  if (r->deblock) { /* the group's rows of the block map: log2 sizes, skip flags */
    const int x0 = gr[0] * 16, y0 = gr[1] * 16;
    const int x1 = (gr[0] + gr[2]) * 16 < r->mi_cols ? (gr[0] + gr[2]) * 16 : r->mi_cols;
    const int y1 = (gr[1] + gr[3]) * 16 < r->mi_rows ? (gr[1] + gr[3]) * 16 : r->mi_rows;
    uint8_t *maps[2] = {r->mi_lg, r->mi_skip};
    for (int m = 0; m < 2; m++)
      for (int y = y0; y < y1; y++) {
        uint8_t *q = maps[m] + (size_t)y * r->mi_cols + x0;
        if (b) {
          if (to_buf)
            memcpy(b + off, q, (size_t)(x1 - x0));
          else
            memcpy(q, b + off, (size_t)(x1 - x0));
        }
        off += x1 - x0;
      }
  }
  return off;
}

/* Pad the last coded frame (after every group's region is in). */
void orc_replay_pad_recon(orc_replay *r) {
  oslot *s = &r->slots[r->fi.display % NSLOT];
  if (r->deblock && !r->fi.is_key) loop_filter_planes(r);
  pad(r, &s->y);
  pad(r, &s->u);
  pad(r, &s->v);
}

int orc_replay_results(orc_replay *r, uint64_t *out, int cap) {
  int nw = (int)r->nwords;
  if (cap < nw + 5) return -1;
  memcpy(out, r->words, (size_t)nw * 8);
  /* levels checksum (speed 6: of the committed blocks), recon sums of the
   * group and of the frame */
  uint64_t lc = 0;
  size_t per = 1024 + 2 * (size_t)r->ntx_c * 1024;
  for (int sb = 0; sb < r->nsb; sb++) {
    if (r->lvl && !r->leaf0[sb]) continue;
    for (size_t i = 0; i < per; i++)
      lc += (uint64_t)(int64_t)r->lev[sb * per + i] * (uint64_t)(i % 1024 + 1);
  }
  for (int l = 1; r->lvl && l < 4; l++) {
    const struct olevel *P = &r->pl[l];
    const size_t pl_ = (size_t)P->B * P->B, pc = (size_t)P->bc * P->bch, pb = pl_ + 2 * pc;
    for (int b = 0; b < P->n; b++) {
      if (!P->leaf[b]) continue;
      const int32_t *v = P->lev + (size_t)b * pb;
      for (size_t i = 0; i < pl_; i++) lc += (uint64_t)(int64_t)v[i] * (uint64_t)(i + 1);
      for (size_t i = 0; i < 2 * pc; i++)
        lc += (uint64_t)(int64_t)v[pl_ + i] * (uint64_t)(i % pc + 1);
    }
  }
  oslot *s = &r->slots[r->fi.display % NSLOT];
  oplane *pl[3] = {&s->y, &s->u, &s->v};
  int32_t gr[4] = {r->tx0, r->ty0, r->tw, r->th};
  uint64_t gs = 0, fs = 0;
  for (int p = 0; p < 3; p++) {
    int rc[4];
    group_rect(r, p, gr, rc);
    for (int y = 0; y < rc[3]; y++)
      for (int x = 0; x < rc[2]; x++) gs += (uint64_t)orc_px(at(pl[p], r->hbd, rc[0] + x, rc[1] + y), r->hbd, 0);
    for (int y = 0; y < pl[p]->h; y++)
      for (int x = 0; x < pl[p]->w; x++) fs += (uint64_t)orc_px(at(pl[p], r->hbd, x, y), r->hbd, 0);
  }
  out[nw + 0] = lc;
  out[nw + 1] = gs;
  out[nw + 2] = r->tail[2];
  out[nw + 3] = (uint64_t)(r->vis_w / 8) * (r->vis_h / 8);
  out[nw + 4] = fs;
  return nw + 5;
}
