// rv_chain.h -- device-side job chaining between the replay's dependent
// search stages.
//
// motion_estimation feeds every stage's winner into the next stage's
// predictor list (estimate_motion_ss4 -> me_ss2 -> full-pel diamond ->
// sub-pel diamond -> the RDO candidates, src/me.rs:193-519, 1023-1075;
// src/rdo.rs:949-1006).  Instead of a job-building launch between stages,
// the workgroup that finishes a search writes its result straight into the
// next stage's job records (whose static fields -- positions, MV ranges,
// lambdas -- are built once when the replay is created).  One writer per
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
  kChainCoarseToHalf = 1,  // F1 -> F2: pred[1 + r] of every reference's job
  kChainHalfToFull = 2,    // F2 -> F3 full-pel: pred[1]
  kChainFullToSub = 3,     // F3 full-pel -> F3 sub-pel: pred[0]
  kChainSubToMc = 4,       // F3 sub-pel -> F4: the sub-pel MV candidate's MC jobs
};

struct ChainNext {
  int mode;
  rv_ds_job *jobs;  // modes 1-3
  // mode 4: candidate c = 2 * ref (sub-pel MV) of superblock sb predicts
  // into the tall scratch planes at (sx * cw, (c * th + sy) * ch)
  rv_mc_job *l_mc, *c_mc;
  rv_plane luma, chroma;
  int tw, th, tx0, ty0, cw, ch;
};

// Called by one thread of the workgroup that finished job `job` (= r *
// n_per_ref + sb, reference-major) with its best MV.
__device__ inline void chain_emit(const ChainNext &c, int job, int n_per_ref, int n_refs,
                                  rv_mv best) {
  const int r = job / n_per_ref, sb = job - r * n_per_ref;
  switch (c.mode) {
    case kChainCoarseToHalf: {  // me_ss2 predictors (src/me.rs:470-519)
      const rv_mv q = qfull(rv_mv{(int16_t)(best.row * 4), (int16_t)(best.col * 4)});
      const rv_mv p{(int16_t)(q.row >> 1), (int16_t)(q.col >> 1)};
      for (int k = 0; k < n_refs; k++) c.jobs[k * n_per_ref + sb].pred[1 + r] = p;
      break;
    }
    case kChainHalfToFull:
      c.jobs[job].pred[1] = qfull(rv_mv{(int16_t)(best.row * 2), (int16_t)(best.col * 2)});
      break;
    case kChainFullToSub:
      c.jobs[job].pred[0] = best;
      break;
    case kChainSubToMc: {
      const int sx = sb % c.tw, sy = sb / c.tw;
      const int px = (sx + c.tx0) * 64, py = (sy + c.ty0) * 64;
      const int cand = 2 * r;  // k = 0: the sub-pel MV
      const int o = cand * n_per_ref + sb;
      c.l_mc[o] = mc_job_for(c.luma, px, py, best, sx * 64, (cand * c.th + sy) * 64);
      c.c_mc[o] = mc_job_for(c.chroma, px >> c.chroma.xdec, py >> c.chroma.ydec, best,
                             sx * c.cw, (cand * c.th + sy) * c.ch);
      break;
    }
    default:
      break;
  }
}

}  // namespace rv
