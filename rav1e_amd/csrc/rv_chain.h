// rv_chain.h -- device-side job chaining between the replay's dependent
// search stages.
//
// motion_estimation feeds every stage's winner into the next stage's
// predictor list (full-pel diamond -> sub-pel diamond -> the RDO
// candidates, src/me.rs:193-278; src/rdo.rs:949-1006).  The workgroup that
// finishes a full-pel search writes its result straight into the sub-pel
// job record (whose static fields -- positions, MV ranges, lambdas -- are
// built once when the replay is created); the RDO kernels derive their
// candidates from the sub-pel results in-kernel.  One writer per
// destination field, and the consumer runs in a later launch on the same
// stream, so no synchronisation beyond stream order is needed.
#pragma once

#include "rv_device.h"

namespace rv {

// quantize_to_fullpel (src/me.rs): Rust `/` truncates toward zero
__host__ __device__ inline rv_mv qfull(rv_mv m) {
  return rv_mv{(int16_t)((m.row / 8) * 8), (int16_t)((m.col / 8) * 8)};
}

// predict_inter / get_params (src/predict.rs:267-283) for plane geometry p:
// integer source origin (PlaneSlice::clamp of the -3 origin,
// src/frame/plane.rs:521-533) and 1/16-pel fracs.
__host__ __device__ inline rv_mc_job mc_job_for(const rv_plane &p, int po_x, int po_y, rv_mv mv,
                                       int dst_x, int dst_y) {
  const int ys = 3 + p.ydec, xs = 3 + p.xdec;
  const int roff = (int)mv.row >> ys, coff = (int)mv.col >> xs;
  rv_mc_job m;
  m.row_frac = ((int)mv.row - (roff << ys)) << (4 - ys);
  m.col_frac = ((int)mv.col - (coff << xs)) << (4 - xs);
  m.src_x = clampi(po_x + coff - 3, -p.xorigin, p.width) + 3;
  m.src_y = clampi(po_y + roff - 3, -p.yorigin, p.height) + 3;
  m.dst_x = dst_x;
  m.dst_y = dst_y;
  return m;
}

enum ChainMode {
  kChainNone = 0,
  kChainFullToSub = 3,  // full-pel -> sub-pel diamond of the same job: pred[0]
};

struct ChainNext {
  int mode;
  rv_ds_job *jobs;
};

// Called by one thread of the workgroup that finished job `job` with its
// best MV.  (The coarse and half-res results feed several later jobs each;
// fill_preds_kernel in rv_replay.hip gathers those.)
__device__ inline void chain_emit(const ChainNext &c, int job, int n_per_ref, int n_refs,
                                  rv_mv best) {
  (void)n_per_ref;
  (void)n_refs;
  if (c.mode == kChainFullToSub) c.jobs[job].pred[0] = best;
}

// ---- RDO inter candidates (rdo_mode_decision, src/rdo.rs:825-1006) ---------
// Superblock grid of a replay instance: a rectangle of whole AV1 tiles
// (uniform tile size tws x ths superblocks, TilingInfo, src/tiling/tiler.rs:
// 49-126) at superblock (tx0, ty0) of the frame, tw x th superblocks.
// rav1e's MV stacks of a superblock (find_mvrefs, src/context.rs:2650-2965,
// built by mvref_kernel in coding-order rounds, rv_mvref.hip): per
// reference k the first two entries and n = min(len, 2); the compound
// (ref 0, ref 1) stack's first two (this, comp) pairs -- its extra search
// always leaves two (:2858-2906).
struct MvStack {
  int32_t n[2];
  rv_mv s[2][2];
  rv_mv c[2][2];
};

struct CandGeo {
  int nsb, tw, th, tx0, ty0, tws, ths;
  int R;     // references searched
  int M;     // inter modes per reference (kCandModes)
  int comp;  // compound candidates after the R * M single ones (0 or kCompModes)
  // rav1e's stacks (speed 10 superblocks); null: the neighbour-NEWMV
  // stand-in below (the speed-6 / frame-edge levels)
  const MvStack *stk;
};

// Per reference, rav1e pushes (src/rdo.rs:880-905, speed 10: no near MVs
// beyond NEAR0): NEARESTMV, NEAR0MV if the MV stack is non-empty, GLOBALMV
// if it holds >= 2 entries, NEWMV if the motion-search MV is non-zero and
// not among the first two stack entries; every mode runs skip, then
// non-skip unless skip had zero distortion (luma_chroma_mode_rdo, :649-700).
// GLOBALMV is the zero MV (no global motion).
enum CandMode { kNearestMv = 0, kNear0Mv = 1, kGlobalMv = 2, kNewMv = 3, kCandModes = 4 };
// RAV1E_INTER_COMPOUND_MODES (src/predict.rs:51-58), pushed for the
// (forward, backward) reference pair when the frame's reference_mode is
// SELECT (src/rdo.rs:914-941, src/encoder.rs:832-836)
enum CompMode {
  kGlobalGlobal = 0, kNearestNearest = 1, kNewNew = 2, kNearestNew = 3, kNewNearest = 4,
  kNearNear = 5, kCompModes = 6
};

__host__ __device__ inline bool mv_eq(rv_mv a, rv_mv b) { return a.row == b.row && a.col == b.col; }

// The MV stack of superblock sb for reference k: find_mvrefs scans the row
// above before the column to the left and merges equal MVs
// (src/mvref / context.rs add_ref_mv_candidate); neighbours never cross a
// tile edge.  The replay takes the neighbours' motion-search MVs (their
// NEWMV) instead of the MVs their RDO chose, so every superblock of a frame
// stays independent: one batched launch per stage.  Returns the entry
// count (0..2); s0 / s1 the entries (scalars: no scratch on the device).
__host__ __device__ inline int cand_stack(const CandGeo &g, const rv_fs_result *sub, int sb,
                                          int k, rv_mv &s0, rv_mv &s1) {
  if (g.stk) {
    const MvStack &m = g.stk[sb];
    s0 = m.s[k][0];
    s1 = m.s[k][1];
    return m.n[k];
  }
  const int sx = sb % g.tw, sy = sb / g.tw;
  const int fx = g.tx0 + sx, fy = g.ty0 + sy;
  // neighbours inside the grid and the tile (a level grid over the frame-edge
  // rectangle starts below / right of blocks it does not hold)
  const bool up = sy > 0 && fy % g.ths != 0, left = sx > 0 && fx % g.tws != 0;
  const rv_mv zero{0, 0};
  const rv_mv a = up ? sub[k * g.nsb + sb - g.tw].best_mv : zero;
  const rv_mv l = left ? sub[k * g.nsb + sb - 1].best_mv : zero;
  if (up) {
    s0 = a;
    s1 = l;
    return left && !mv_eq(l, a) ? 2 : 1;
  }
  s0 = l;
  s1 = zero;
  return left ? 1 : 0;
}

// The compound MV stack of (reference 0, reference 1): the above and left
// neighbours' (NEWMV 0, NEWMV 1) pairs, merged if equal (the same
// neighbour-NEWMV stand-in as cand_stack).  Entries in scalars (no
// scratch on the device); returns the count.
__host__ __device__ inline int comp_stack(const CandGeo &g, const rv_fs_result *sub, int sb,
                                          rv_mv &e00, rv_mv &e01, rv_mv &e10, rv_mv &e11) {
  if (g.stk) {
    const MvStack &m = g.stk[sb];
    e00 = m.c[0][0];
    e01 = m.c[0][1];
    e10 = m.c[1][0];
    e11 = m.c[1][1];
    return 2;
  }
  const int sx = sb % g.tw, sy = sb / g.tw;
  const int fx = g.tx0 + sx, fy = g.ty0 + sy;
  // neighbours inside the grid and the tile (a level grid over the frame-edge
  // rectangle starts below / right of blocks it does not hold)
  const bool up = sy > 0 && fy % g.ths != 0, left = sx > 0 && fx % g.tws != 0;
  const rv_mv zero{0, 0};
  const rv_mv a0 = up ? sub[sb - g.tw].best_mv : zero, a1 = up ? sub[g.nsb + sb - g.tw].best_mv : zero;
  const rv_mv l0 = left ? sub[sb - 1].best_mv : zero, l1 = left ? sub[g.nsb + sb - 1].best_mv : zero;
  e10 = e11 = zero;
  if (up) {
    e00 = a0;
    e01 = a1;
    if (left && (!mv_eq(l0, a0) || !mv_eq(l1, a1))) {
      e10 = l0;
      e11 = l1;
      return 2;
    }
    return 1;
  }
  e00 = l0;
  e01 = l1;
  return left ? 1 : 0;
}

// The two MVs of compound candidate m of superblock sb (rdo_mode_decision's
// mvs for the compound modes, src/rdo.rs:952-992; an empty stack reads as
// zero MVs).  Always pushed.
__host__ __device__ inline void comp_mvs(const CandGeo &g, const rv_fs_result *sub, int sb, int m,
                                         rv_mv *mv0, rv_mv *mv1) {
  rv_mv e00, e01, e10, e11;
  const int n = comp_stack(g, sub, sb, e00, e01, e10, e11);
  const rv_mv zero{0, 0};
  const rv_mv me0 = sub[sb].best_mv, me1 = sub[g.nsb + sb].best_mv;
  const rv_mv n00 = n >= 1 ? e00 : zero, n01 = n >= 1 ? e01 : zero;
  switch (m) {
    case kGlobalGlobal:
      *mv0 = *mv1 = zero;
      break;
    case kNearestNearest:
      *mv0 = n00;
      *mv1 = n01;
      break;
    case kNewNew:
      *mv0 = me0;
      *mv1 = me1;
      break;
    case kNearestNew:
      *mv0 = n00;
      *mv1 = me1;
      break;
    case kNewNearest:
      *mv0 = me0;
      *mv1 = n01;
      break;
    default:  // kNearNear
      *mv0 = n >= 2 ? e10 : zero;
      *mv1 = n >= 2 ? e11 : zero;
      break;
  }
}

// MV of candidate c = k * M + m of superblock sb; false if rav1e would not
// push that mode (rdo_mode_decision's inter_mode_set).  Compound
// candidates (c >= R * M) are handled by comp_mvs.
__host__ __device__ inline bool cand_mv(const CandGeo &g, const rv_fs_result *sub, int sb, int c,
                                        rv_mv *mv) {
  const int k = c / g.M, m = c - k * g.M;
  rv_mv s0, s1;
  const int n = cand_stack(g, sub, sb, k, s0, s1);
  const rv_mv zero{0, 0};
  switch (m) {
    case kNearestMv:
      *mv = n >= 1 ? s0 : zero;
      return true;
    case kNear0Mv:
      *mv = n >= 2 ? s1 : zero;
      return n >= 1;
    case kGlobalMv:
      *mv = zero;
      return n >= 2;
    default: {  // kNewMv
      const rv_mv me = sub[k * g.nsb + sb].best_mv;
      *mv = me;
      return !(n >= 1 && mv_eq(s0, me)) && !(n >= 2 && mv_eq(s1, me)) &&
             (me.row != 0 || me.col != 0);
    }
  }
}

// A candidate whose reference and MV (compound: MV pair) repeat an earlier
// pushed one of the same block predicts, distorts and costs exactly the
// same, so it can never win the strict-`<` argmin after that one (skip or
// non-skip): it is evaluated once, as the first.  cand_live / comp_live:
// pushed and not such a repeat.
__host__ __device__ inline bool cand_live(const CandGeo &g, const rv_fs_result *sub, int sb, int c,
                                          rv_mv *mv) {
  if (!cand_mv(g, sub, sb, c, mv)) return false;
  for (int c2 = (c / g.M) * g.M; c2 < c; c2++) {
    rv_mv m2;
    if (cand_mv(g, sub, sb, c2, &m2) && mv_eq(m2, *mv)) return false;
  }
  return true;
}
__host__ __device__ inline bool comp_live(const CandGeo &g, const rv_fs_result *sub, int sb, int m) {
  rv_mv a0, a1;
  comp_mvs(g, sub, sb, m, &a0, &a1);
  for (int m2 = 0; m2 < m; m2++) {
    rv_mv b0, b1;
    comp_mvs(g, sub, sb, m2, &b0, &b1);
    if (mv_eq(a0, b0) && mv_eq(a1, b1)) return false;
  }
  return true;
}

}  // namespace rv
