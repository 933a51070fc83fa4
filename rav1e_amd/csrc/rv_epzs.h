// rv_epzs.h -- rav1e's EPZS predictor sets (get_subset_predictors,
// src/me.rs:82-174) for the replay's searches, device side.
//
// Every full-pel search of rav1e starts from zero, its coarse MVs
// (quantize_to_fullpel) and the MVs around the block: subsets A and B from
// the tile's motion field ts.mvs (the left, top and top-right 4x4 units, and
// their mean), subset C from the LAST reference frame's saved field
// (left, top, right, bottom, co-located).  The tile field fills in coding
// order (save_block_motion, src/encoder.rs:1432-1444), so a search depends
// on the searches and decisions before it in the tile; the replay reaches
// that order by the rounds of rv_replay_frame: every check
// recomputes each job's set from the current state and re-runs the jobs
// whose set changed.
#pragma once

#include "rv_chain.h"

namespace rv {

// The group's superblock grid and the frame (4x4 units: w_in_b x h_in_b)
struct EpzsGeo {
  int tx0, ty0, tw, th, tws, ths, W, H, w_in_b, h_in_b;
};

// The tile of frame superblock (fx, fy): its origin (superblocks) and
// visible size in 4x4 units (TileStateMut mi_width / mi_height)
__device__ inline void epzs_tile(const EpzsGeo &g, int fx, int fy, int &t0x, int &t0y, int &mi_w,
                                 int &mi_h) {
  t0x = fx - fx % g.tws;
  t0y = fy - fy % g.ths;
  const int vw = g.W - t0x * 64 < g.tws * 64 ? g.W - t0x * 64 : g.tws * 64;
  const int vh = g.H - t0y * 64 < g.ths * 64 ? g.H - t0y * 64 : g.ths * 64;
  mi_w = vw >> 2;
  mi_h = vh >> 2;
}

// adjust_bo (src/me.rs:993-1004) on tile-relative 4x4 offsets
__device__ inline void epzs_adjust_bo(int mi_w, int mi_h, int &bx, int &by, int bw, int bh) {
  const int x = bx < mi_w - bw / 4 ? bx : mi_w - bw / 4;
  const int y = by < mi_h - bh / 4 ? by : mi_h - bh / 4;
  bx = x > 0 ? x : 0;
  by = y > 0 ? y : 0;
}

__device__ inline rv_mv epzs_qfull(rv_mv m) {
  return rv_mv{(int16_t)((m.row / 8) * 8), (int16_t)((m.col / 8) * 8)};
}
__device__ inline bool epzs_zero(rv_mv m) { return m.row == 0 && m.col == 0; }

// get_subset_predictors of the block at tile offset (bx, by) of the tile at
// frame 4x4 (tx4, ty4), mi_w columns: zero, the ncm (<= NCM) coarse MVs cm,
// subsets A / B through rd(X4, Y4) (the tile field at frame 4x4 (X4, Y4)),
// subset C from prev (the reference frame's field at 8x8 granularity --
// every value of rav1e's field is constant over 8x8 cells at speed 10;
// null: none) (cell (x, y) of prev at prev[((y * w_in_b / 2) + x) * pr]),
// stored into job j (shr: every predictor >> 1, me_ss2) unless it already
// holds that set; returns whether it changed.  The set's entries sit in 17
// fixed slots (zero, 7 coarse, left, top, top-right, the mean, 5 of subset
// C), each with a validity bit, so no local array is indexed at run time
// (no scratch); the job's list is their compaction.  Every field value is
// read once.
template <int NCM, typename Rd>
__device__ inline bool epzs_update(rv_ds_job *j, int shr, const EpzsGeo &g, int tx4, int ty4,
                                   int mi_w, int bx, int by, const rv_mv (&cm)[NCM], int ncm,
                                   Rd rd, const rv_mv *prev, int pr) {
  static_assert(NCM >= 1 && 1 + NCM + 4 + 5 <= RV_DS_MAX_PRED, "slots");
  constexpr int NS = 1 + NCM + 4 + 5;
  const bool hl = bx > 0, ht = by > 0, htr = ht && bx < mi_w - 1;
  const rv_mv z{0, 0};
  const rv_mv l = hl ? rd(tx4 + bx - 1, ty4 + by) : z;
  const rv_mv t = ht ? rd(tx4 + bx, ty4 + by - 1) : z;
  const rv_mv tr = htr ? rd(tx4 + bx + 1, ty4 + by - 1) : z;
  rv_mv c[NS];
  uint32_t valid = 1;
  c[0] = z;
#pragma unroll
  for (int i = 0; i < NCM; i++) {
    c[1 + i] = epzs_qfull(cm[i]);
    valid |= (uint32_t)(i < ncm) << (1 + i);
  }
  c[NCM + 1] = l;
  c[NCM + 2] = t;
  c[NCM + 3] = tr;
  valid |= (uint32_t)(hl && !epzs_zero(l)) << (NCM + 1);
  valid |= (uint32_t)(ht && !epzs_zero(t)) << (NCM + 2);
  valid |= (uint32_t)(htr && !epzs_zero(tr)) << (NCM + 3);
  const int nm = (int)hl + (int)ht + (int)htr;
  {  // the mean: MotionVector Add / Div<i16> (truncating)
    const int16_t sr = (int16_t)((int16_t)(l.row + t.row) + tr.row);
    const int16_t sc = (int16_t)((int16_t)(l.col + t.col) + tr.col);
    const int d = nm ? nm : 1;
    c[NCM + 4] = epzs_qfull(rv_mv{(int16_t)(sr / d), (int16_t)(sc / d)});
    valid |= (uint32_t)(nm && !epzs_zero(c[NCM + 4])) << (NCM + 4);
  }
  if (prev) {
    const int fx = tx4 + bx, fy = ty4 + by, w8 = g.w_in_b >> 1;
    auto pv = [&](int x, int y) { return prev[((y >> 1) * w8 + (x >> 1)) * pr]; };
    c[NCM + 5] = fx > 0 ? pv(fx - 1, fy) : z;
    c[NCM + 6] = fy > 0 ? pv(fx, fy - 1) : z;
    c[NCM + 7] = fx < g.w_in_b - 1 ? pv(fx + 1, fy) : z;
    c[NCM + 8] = fy < g.h_in_b - 1 ? pv(fx, fy + 1) : z;
    c[NCM + 9] = pv(fx, fy);
#pragma unroll
    for (int i = NCM + 5; i < NS; i++) valid |= (uint32_t)!epzs_zero(c[i]) << i;
  } else {
#pragma unroll
    for (int i = NCM + 5; i < NS; i++) c[i] = z;
  }
  auto tf = [&](rv_mv m) { return shr ? rv_mv{(int16_t)(m.row >> 1), (int16_t)(m.col >> 1)} : m; };
  // the set by list position: slot i goes to position popcount(valid below
  // i) -- a selection over static indices (a list indexed by a running
  // count would live in scratch memory)
  rv_mv nw[NS];
#pragma unroll
  for (int p = 0; p < NS; p++) nw[p] = z;
#pragma unroll
  for (int i = 0; i < NS; i++) {
    const bool v = (valid >> i) & 1;
    const int pos = __popc(valid & ((1u << i) - 1));
    const rv_mv ti = tf(c[i]);
#pragma unroll
    for (int p = 0; p <= i; p++)
      if (v && pos == p) nw[p] = ti;
  }
  const int n = __popc(valid);
  // compare with the job's list: every entry read unconditionally, so the
  // loads are in flight together (a compare that stops at the first
  // difference issues them one after another)
  rv_mv old[NS];
#pragma unroll
  for (int p = 0; p < NS; p++) old[p] = j->pred[p];
  const int old_n = j->n_pred;
  bool same = old_n == n;
#pragma unroll
  for (int p = 0; p < NS; p++) same &= (p >= n) | mv_eq(old[p], nw[p]);
  if (same) return false;
#pragma unroll
  for (int p = 0; p < NS; p++)
    if (p < n) j->pred[p] = nw[p];
  j->n_pred = n;
  return true;
}

// The round checks' counts: check q counts into cnt[0..1] (slot q of the
// ring), the last workgroup to finish reads them, zeroes the next check's
// slot and the ticket, and stores (seq << 32 | cnt[0] + cnt[1]) into
// host-mapped memory (the host spins on it, no stream synchronisation).
// Every workgroup's counted appends returned before its ticket.
struct RoundPub {
  int32_t *cnt, *next;
  uint32_t *ticket;
  unsigned long long *host;  // null: nothing published
  uint32_t seq;
};
__device__ inline void round_publish(const RoundPub &p) {
  if (!p.host) return;
  __syncthreads();
  if (threadIdx.x != 0) return;
  __threadfence();
  const uint32_t t = atomicAdd(p.ticket, 1u);
  if (t != gridDim.x - 1) return;
  __threadfence();
  const int c = atomicAdd(p.cnt, 0) + atomicAdd(p.cnt + 1, 0);
  p.next[0] = p.next[1] = 0;
  *p.ticket = 0;
  __threadfence();
  __hip_atomic_store(p.host, ((unsigned long long)p.seq << 32) | (uint32_t)c, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace rv
