// rv_mvref.hip -- rav1e's MV reference stacks for the replay's 64x64
// superblocks (ContextWriter::find_mvrefs / setup_mvref_list,
// src/context.rs:2308-2965), one thread per superblock.
//
// rav1e codes a tile's superblocks in raster order, and a superblock's
// stacks read the blocks coded before it: the one above (scan_row_mbmi of
// row -1), to the left (scan_col_mbmi of column -1), the top-right and the
// top-left one (scan_blk_mbmi).  For a 64x64 block every outer row / column
// scan (-3, -5) is already covered (processed_rows = 6 after row -1), so
// those four blocks are the whole input.  Their candidates enter with
// weights 16 * 6 = 96 (above, left) and 4 (top-right), then REF_CAT_LEVEL
// (640) is added, then the top-left's 4; a stable sort by weight; when
// fewer than two entries were found the extra search (7.10.2.12) takes the
// above and the left block's other references (sign-flipped across the
// frame's direction); the compound stack is then filled to two entries;
// finally the MVs are clamped to the block's border.
//
// The replay runs it in rounds (rv_replay_frame): every superblock is
// evaluated with the stacks of the decisions it has so far, and a round
// re-evaluates exactly those whose stacks changed, until none does -- the
// fixed point of the raster-order dependency chain, which is the
// sequential result.
#include <algorithm>

#include "rv_mvref.h"

using namespace rv;

namespace {

struct Cand {
  rv_mv t, c;  // this_mv, comp_mv
  uint32_t w;
};

__device__ inline bool inter_of(const BlkDec &b) { return b.ref[0] != kIntraFrame; }

// The stack in registers: at most kSlots entries reach it for a 64x64
// block (one per neighbour from the scans -- a single-reference stack takes
// one MV of a block, a compound one one pair -- and at most two from the
// extra search), so MAX_REF_MV_STACK_SIZE (8) never binds.  Every access
// uses a compile-time slot index (unrolled loops), so nothing goes to
// scratch memory.
constexpr int kSlots = 6;
struct Stk {
  Cand e[kSlots];
  int n;
};

// find_matching_mv(_and_update_weight) / push
__device__ __forceinline__ void push_or_add(Stk &k, rv_mv t, rv_mv c, uint32_t w, bool comp,
                                            bool add_weight) {
  bool found = false;
#pragma unroll
  for (int i = 0; i < kSlots; i++)
    if (i < k.n && !found && mv_eq(k.e[i].t, t) && (!comp || mv_eq(k.e[i].c, c))) {
      if (add_weight) k.e[i].w += w;
      found = true;
    }
  if (found) return;
#pragma unroll
  for (int i = 0; i < kSlots; i++)
    if (i == k.n) k.e[i] = Cand{t, c, w};
  k.n++;
}

// add_ref_mv_candidate (src/context.rs:2366-2435)
__device__ __forceinline__ void add_ref(Stk &k, const BlkDec &b, uint32_t w, int rf0, int rf1,
                                        bool compound) {
  if (!inter_of(b)) return;
  if (compound) {
    if (b.ref[0] == rf0 && b.ref[1] == rf1) push_or_add(k, b.mv[0], b.mv[1], w, true, true);
    return;
  }
  if (b.ref[0] == rf0) push_or_add(k, b.mv[0], rv_mv{0, 0}, w, false, true);
  if (b.ref[1] == rf0) push_or_add(k, b.mv[1], rv_mv{0, 0}, w, false, true);
}

__device__ inline rv_mv neg(rv_mv m) { return rv_mv{(int16_t)-m.row, (int16_t)-m.col}; }

struct Nb {
  bool up, left, tr, tl;
  BlkDec a, l, r, d;  // above, left, top-right, top-left
};

// setup_mvref_list of a 64x64 block for ref_frames (rf0, rf1; rf1 = NONE:
// single): the first two entries (clamped) into s0 / s1, the length returned
__device__ inline int stack64(const Nb &nb, int rf0, int rf1, uint32_t sbias, int fx, int fy,
                              int fcols, int frows, Cand &s0, Cand &s1) {
  const bool compound = rf1 != kNoneFrame;
  Stk k;
  k.n = 0;
#pragma unroll
  for (int i = 0; i < kSlots; i++) k.e[i] = Cand{rv_mv{0, 0}, rv_mv{0, 0}, 0};
  if (nb.up) add_ref(k, nb.a, 16 * 6, rf0, rf1, compound);
  if (nb.left) add_ref(k, nb.l, 16 * 6, rf0, rf1, compound);
  if (nb.tr) add_ref(k, nb.r, 4, rf0, rf1, compound);
#pragma unroll
  for (int i = 0; i < kSlots; i++)
    if (i < k.n) k.e[i].w += 640;  // add_offset, REF_CAT_LEVEL
  if (nb.tl) add_ref(k, nb.d, 4, rf0, rf1, compound);
  // 7.10.2.11: stable sort, descending weight (an insertion sort over the
  // slots; empty slots carry weight 0 and stay behind)
#pragma unroll
  for (int i = 1; i < kSlots; i++)
#pragma unroll
    for (int j = i; j > 0; j--)
      if (j < k.n && k.e[j].w > k.e[j - 1].w) {
        const Cand t = k.e[j];
        k.e[j] = k.e[j - 1];
        k.e[j - 1] = t;
      }
  if (k.n < 2) {
    // 7.10.2.12: the above block (pass 0), then the left one (pass 1); each
    // 64x64 pass reads one block (idx += n4_w = 16)
    int idc0 = 0, idc1 = 0, dfc0 = 0, dfc1 = 0;
    rv_mv id0[2] = {rv_mv{0, 0}, rv_mv{0, 0}}, id1[2] = {rv_mv{0, 0}, rv_mv{0, 0}};
    rv_mv df0[2] = {rv_mv{0, 0}, rv_mv{0, 0}}, df1[2] = {rv_mv{0, 0}, rv_mv{0, 0}};
#pragma unroll
    for (int p = 0; p < 2; p++) {
      if (p == 0 ? !nb.up : !nb.left) continue;
      if (k.n >= 2) break;
      const BlkDec &b = p == 0 ? nb.a : nb.l;
#pragma unroll
      for (int cl = 0; cl < 2; cl++) {
        const int cr = b.ref[cl];
        if (cr == kIntraFrame || cr == kNoneFrame) continue;
        const rv_mv m = b.mv[cl];
        if (compound) {
          // list 0 (rf0), then list 1 (rf1)
          if (cr == rf0 && idc0 < 2) {
            if (idc0 == 0) id0[0] = m; else id0[1] = m;
            idc0++;
          } else if (dfc0 < 2) {
            const rv_mv v = ((sbias >> (cr - 1)) & 1) != ((sbias >> (rf0 - 1)) & 1) ? neg(m) : m;
            if (dfc0 == 0) df0[0] = v; else df0[1] = v;
            dfc0++;
          }
          if (cr == rf1 && idc1 < 2) {
            if (idc1 == 0) id1[0] = m; else id1[1] = m;
            idc1++;
          } else if (dfc1 < 2) {
            const rv_mv v = ((sbias >> (cr - 1)) & 1) != ((sbias >> (rf1 - 1)) & 1) ? neg(m) : m;
            if (dfc1 == 0) df1[0] = v; else df1[1] = v;
            dfc1++;
          }
        } else {
          const rv_mv v = ((sbias >> (cr - 1)) & 1) != ((sbias >> (rf0 - 1)) & 1) ? neg(m) : m;
          push_or_add(k, v, rv_mv{0, 0}, 2, false, false);
        }
      }
    }
    if (compound) {
      // combined_mvs[i][list]: the same-reference MVs, then the others
      rv_mv c00 = rv_mv{0, 0}, c10 = rv_mv{0, 0}, c01 = rv_mv{0, 0}, c11 = rv_mv{0, 0};
      {
        int cc = 0;
        if (idc0 > 0) { c00 = id0[0]; cc++; }
        if (idc0 > 1) { c10 = id0[1]; cc++; }
#pragma unroll
        for (int i = 0; i < 2; i++)  // (static indices: no scratch)
          if (i < dfc0 && cc < 2) {
            if (cc == 0) c00 = df0[i]; else c10 = df0[i];
            cc++;
          }
      }
      {
        int cc = 0;
        if (idc1 > 0) { c01 = id1[0]; cc++; }
        if (idc1 > 1) { c11 = id1[1]; cc++; }
#pragma unroll
        for (int i = 0; i < 2; i++)
          if (i < dfc1 && cc < 2) {
            if (cc == 0) c01 = df1[i]; else c11 = df1[i];
            cc++;
          }
      }
      if (k.n == 1) {
        const bool same = mv_eq(c00, k.e[0].t) && mv_eq(c01, k.e[0].c);
        k.e[1] = same ? Cand{c10, c11, 2} : Cand{c00, c01, 2};
        k.n = 2;
      } else {
        k.e[0] = Cand{c00, c01, 2};
        k.e[1] = Cand{c10, c11, 2};
        k.n = 2;
      }
    }
  }
  // clamp (src/context.rs:2911-2941), 64x64: border 128 + 512
  const int xmin = -fx * 32 - 640, xmax = (fcols - fx - 16) * 32 + 640;
  const int ymin = -fy * 32 - 640, ymax = (frows - fy - 16) * 32 + 640;
  auto cl = [&](rv_mv m) {
    return rv_mv{(int16_t)clampi(m.row, ymin, ymax), (int16_t)clampi(m.col, xmin, xmax)};
  };
  s0 = Cand{cl(k.e[0].t), cl(k.e[0].c), k.e[0].w};
  s1 = Cand{cl(k.e[1].t), cl(k.e[1].c), k.e[1].w};
  return k.n;
}

// The coded block at frame pixel (X, Y) inside superblock nsb: its 64x64
// winner, or (a superblock past the frame's right / bottom edge, speed 10)
// the must_split leaf holding it -- the largest block inside the frame.
__device__ inline BlkDec coded_at(const MvrefArgs &a, int nsb, int X, int Y) {
  const int SX = X & ~63, SY = Y & ~63;
  if ((SX + 64 <= a.W && SY + 64 <= a.H) || !a.lvl) {
    BlkDec d = a.dec[nsb];
    if (a.iwas && a.iwas[nsb]) d.ref[0] = kIntraFrame, d.ref[1] = kNoneFrame;
    return d;
  }
  int l = 1;
  for (; l < 3; l++) {
    const int B = 64 >> l, bx = X & ~(B - 1), by = Y & ~(B - 1);
    if (bx + B <= a.W && by + B <= a.H) break;
  }
  // constant indices into the argument arrays (a runtime index would copy
  // the arguments into scratch memory)
  auto leaf = [&](const CandGeo &g, const rv_fs_result *sub, const RdoWinner *win, int B) {
    const int b = (Y / B - g.ty0) * g.tw + (X / B - g.tx0);
    return blk_dec_of(g, sub, b, win[b].c);
  };
  if (l == 1) return leaf(a.lcg[1], a.lsub[1], a.lwin[1], 32);
  if (l == 2) return leaf(a.lcg[2], a.lsub[2], a.lwin[2], 16);
  return leaf(a.lcg[3], a.lsub[3], a.lwin[3], 8);
}

// The superblock's stacks: every reference's and, on compound frames, the
// (ref 0, ref 1) pair's (empty for a must_split superblock)
__device__ inline MvStack stacks_of(const MvrefArgs &a, const Nb &nb, bool split, int fsx,
                                    int fsy) {
  MvStack s;
  for (int k = 0; k < 2; k++) {
    s.n[k] = 0;
    s.s[k][0] = s.s[k][1] = rv_mv{0, 0};
  }
  Cand e0, e1;
  // (every loop over the references runs to the stack's two slots with a
  // compile-time index: a runtime one kept the MvStack in scratch memory)
#pragma unroll
  for (int k = 0; k < 2; k++) {
    if (k >= a.R || split) continue;
    const int n = stack64(nb, 1 + k, kNoneFrame, a.sign_bias, fsx * 16, fsy * 16, a.w_in_b,
                          a.h_in_b, e0, e1);
    s.n[k] = n < 2 ? n : 2;
    if (n >= 1) s.s[k][0] = e0.t;
    if (n >= 2) s.s[k][1] = e1.t;
  }
  s.c[0][0] = s.c[0][1] = s.c[1][0] = s.c[1][1] = rv_mv{0, 0};
  if (a.comp && !split) {
    (void)stack64(nb, 1, 2, a.sign_bias, fsx * 16, fsy * 16, a.w_in_b, a.h_in_b, e0, e1);
    s.c[0][0] = e0.t;
    s.c[0][1] = e0.c;
    s.c[1][0] = e1.t;
    s.c[1][1] = e1.c;
  }
  return s;
}
// the stacks a superblock was evaluated with still hold (never on the first round)
__device__ inline bool same_stacks(const MvrefArgs &a, const MvStack &o, const MvStack &s) {
  bool same = !a.init;
#pragma unroll
  for (int k = 0; k < 2; k++)
    if (k < a.R)
      same = same && o.n[k] == s.n[k] && mv_eq(o.s[k][0], s.s[k][0]) && mv_eq(o.s[k][1], s.s[k][1]);
  if (a.comp && same)
    same = mv_eq(o.c[0][0], s.c[0][0]) && mv_eq(o.c[0][1], s.c[0][1]) &&
           mv_eq(o.c[1][0], s.c[1][0]) && mv_eq(o.c[1][1], s.c[1][1]);
  return same;
}
// a marked superblock's new stacks and motion_estimation's rate predictors
// (src/rdo.rs:858-870)
__device__ inline void set_stacks(const MvrefArgs &a, int sb, const MvStack &s) {
  a.stk[sb] = s;
#pragma unroll
  for (int k = 0; k < 2; k++) {
    if (k >= a.R) continue;
    const int j = k * a.nsb + sb;
    a.jf[j].pmv[0] = a.js[j].pmv[0] = s.s[k][0];
    a.jf[j].pmv[1] = a.js[j].pmv[1] = s.s[k][1];
  }
}

// The encode's tile field of reference k at frame 4x4 (X4, Y4), as the
// superblock at frame (fsx, fsy) would read it in coding order
__device__ inline rv_mv enc_field(const MvrefArgs &a, int k, int X4, int Y4, int fsx, int fsy) {
  const int SX = X4 >> 4, SY = Y4 >> 4;
  if (SX == fsx && SY == fsy) return rv_mv{0, 0};  // its own quadrants are saved after its F2
  const int gsb = (SY - a.ty0) * a.tw + (SX - a.tx0);
  const bool edge = a.lvl && ((SX + 1) * 64 > a.W || (SY + 1) * 64 > a.H);
  // the quadrant's MV is read before the decision, not after it: the two
  // loads are then in flight together
  const rv_mv h = a.hq[((size_t)k * a.nsb + gsb) * 4 + ((Y4 >> 3) & 1) * 2 + ((X4 >> 3) & 1)].best_mv;
  BlkDec d;
  d.ref[0] = kIntraFrame;
  if ((!edge || a.edge_ok) && !(a.init && a.field_guess_la)) d = coded_at(a, gsb, X4 * 4, Y4 * 4);
  if (d.ref[0] != kIntraFrame && d.ref[0] - 1 == k) return d.mv[0];
  return rv_mv{(int16_t)(h.row * 2), (int16_t)(h.col * 2)};
}

// estimate_motion_ss4's result: the coarse MV * 4
__device__ inline rv_mv coarse4(const MvrefArgs &a, int k, int sb) {
  const rv_mv c = a.coarse[(size_t)k * a.nsb + sb].best_mv;
  return rv_mv{(int16_t)(c.row * 4), (int16_t)(c.col * 4)};
}

// EPZS job j of the superblock (j < R: F3 of reference j; then F2 quadrant
// q of reference k at j = R + 4 k + q): its predictor set from the current
// state into the job; returns whether it changed.
template <typename Fld>
__device__ inline bool epzs_job_f(const MvrefArgs &a, int sb, int fsx, int fsy, int j, Fld fld) {
  int t0x, t0y, mi_w, mi_h;
  epzs_tile(a.eg, fsx, fsy, t0x, t0y, mi_w, mi_h);
  const int tsx = fsx - t0x, tsy = fsy - t0y;
  const int k = j < a.R ? j : (j - a.R) >> 2;
  auto rd = [&](int X4, int Y4) { return fld(k, X4, Y4); };
  const rv_mv *prev = a.prev ? a.prev + k : nullptr;
  if (j < a.R) {  // F3: full_pixel_me of the 64x64 (src/me.rs:390-431), cmvs = [pmvs[0]]
    const rv_mv cm[1] = {coarse4(a, k, sb)};
    return epzs_update(a.jf + (size_t)k * a.nsb + sb, 0, a.eg, t0x * 16, t0y * 16, mi_w, tsx * 16,
                       tsy * 16, cm, 1, rd, prev, a.R);
  }
  // F2: me_ss2 of quadrant q (src/me.rs:465-519), adjust_bo'd, cmvs = the
  // coarse MVs of the superblock and its neighbour on each side
  const int q = (j - a.R) & 3;
  const int tsw = (mi_w + 15) / 16, tsh = (mi_h + 15) / 16;
  // [own, horizontal neighbour if any, vertical neighbour if any] in static slots
  const bool hh = (q & 1) ? tsx < tsw - 1 : tsx > 0, hv = (q >> 1) ? tsy < tsh - 1 : tsy > 0;
  // the neighbours' loads from a valid index either way, then a select of
  // the values (a select of the loads became a flat load through a pointer
  // to a zero in scratch memory)
  const rv_mv ch0 = coarse4(a, k, hh ? ((q & 1) ? sb + 1 : sb - 1) : sb);
  const rv_mv cv0 = coarse4(a, k, hv ? ((q >> 1) ? sb + a.tw : sb - a.tw) : sb);
  const rv_mv ch = hh ? ch0 : rv_mv{0, 0};
  const rv_mv cv = hv ? cv0 : rv_mv{0, 0};
  const rv_mv cm[3] = {coarse4(a, k, sb), hh ? ch : cv, cv};
  const int nc = 1 + (int)hh + (int)hv;
  int bx = tsx * 16 + (q & 1) * 8, by = tsy * 16 + (q >> 1) * 8;
  epzs_adjust_bo(mi_w, mi_h, bx, by, 32, 32);
  return epzs_update(a.jh + ((size_t)k * a.nsb + sb) * 4 + q, 1, a.eg, t0x * 16, t0y * 16, mi_w, bx,
                     by, cm, nc, rd, prev, a.R);
}

__device__ inline bool epzs_job(const MvrefArgs &a, int sb, int fsx, int fsy, int j) {
  return epzs_job_f(a, sb, fsx, fsy, j,
                    [&](int k, int X4, int Y4) { return enc_field(a, k, X4, Y4, fsx, fsy); });
}

// The coded frame's field: one thread per 8x8 cell of the group (inside the
// frame), every reference
__global__ __launch_bounds__(256) void mvref_field_kernel(MvrefArgs a, rv_mv *field) {
  const int w8 = a.w_in_b >> 1, h8 = a.h_in_b >> 1;
  const int x0 = a.tx0 * 8, y0 = a.ty0 * 8;
  const int x1 = min((a.tx0 + a.tw) * 8, w8), y1 = min((a.ty0 + a.th) * 8, h8);
  const int gw = x1 - x0;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= gw * (y1 - y0)) return;
  const int x8 = x0 + i % gw, y8 = y0 + i / gw;
  for (int k = 0; k < a.R; k++)
    field[((size_t)y8 * w8 + x8) * a.R + k] = enc_field(a, k, 2 * x8, 2 * y8, -1, -1);
}

// One check: 16 lanes per superblock -- lane 0 its stacks, lanes 1 .. 5 R
// its EPZS jobs (F3 per reference, F2 per quadrant and reference) -- so a
// superblock's eleven sets are built side by side.
constexpr int kCheckLanes = 16;
__global__ __launch_bounds__(256) void mvref_kernel(MvrefArgs a) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int sb = t / kCheckLanes, j = t % kCheckLanes;
  const int lane = threadIdx.x & 63;
  bool changed = false;
  uint32_t pmask = 0;  // lane 0: the references whose rate predictors changed
  const bool live = sb < a.nsb;
  if (live) {
    const int sx = sb % a.tw, sy = sb / a.tw;
    const int fsx = a.tx0 + sx, fsy = a.ty0 + sy;  // frame superblock
    if (j == 0) {
      // the tile: its origin in superblocks and its size in 4x4 units
      // (TileBlocks cols / rows, src/tiling/tiler.rs:194-202)
      const int t0x = fsx - fsx % a.tws, t0y = fsy - fsy % a.ths;
      const int cols = min(a.tws * 16, a.w_in_b - t0x * 16);
      const int bx = (fsx - t0x) * 16, by = (fsy - t0y) * 16;  // tile-relative 4x4 offset
      const int X = fsx * 64, Y = fsy * 64;
      // a superblock past the frame edge is split (must_split): its 64x64 is
      // evaluated but never coded, with empty stacks (and it reads no
      // neighbour: the edge levels' winners may still be in flight)
      const bool split = a.lvl && (X + 64 > a.W || Y + 64 > a.H);
      Nb nb;
      nb.up = !split && by > 0;
      nb.left = !split && bx > 0;
      nb.tr = !split && by > 0 && bx + 16 < cols;  // has_tr(64x64) && scan_blk_mbmi's bound
      nb.tl = !split && bx > 0 && by > 0;
      if (nb.up) nb.a = coded_at(a, sb - a.tw, X, Y - 4);
      if (nb.left) nb.l = coded_at(a, sb - 1, X - 4, Y);
      if (nb.tr) nb.r = coded_at(a, sb - a.tw + 1, X + 64, Y - 4);
      if (nb.tl) nb.d = coded_at(a, sb - a.tw - 1, X - 4, Y - 4);
      const MvStack s = stacks_of(a, nb, split, fsx, fsy);
      changed = !same_stacks(a, a.stk[sb], s);
#pragma unroll
      for (int k = 0; k < 2; k++)
        if (k < a.R && (a.init || !mv_eq(a.stk[sb].s[k][0], s.s[k][0]) ||
                        !mv_eq(a.stk[sb].s[k][1], s.s[k][1])))
          pmask |= 1u << k;
      if (changed) set_stacks(a, sb, s);  // (its pmv: the F3 jobs' rate predictors)
    } else if (a.epzs && j <= 5 * a.R) {
      changed = epzs_job(a, sb, fsx, fsy, j - 1);
    }
  }
  // the superblock's lanes: any change marks it (lane 0 records and lists it)
  const uint64_t cm = __ballot(changed);
  const int g0 = lane & ~(kCheckLanes - 1);
  const uint32_t pm = (uint32_t)__shfl((int)pmask, g0, 64);
  if (a.f3dirty && live && j >= 1 && j <= a.R)  // F3 job j - 1: its set or its pmv
    a.f3dirty[(size_t)(j - 1) * a.nsb + sb] = (changed || ((pm >> (j - 1)) & 1)) ? 1 : 0;
  if (a.f2dirty && live && j > a.R && j <= 5 * a.R) {  // F2 quadrant job (me_ss2's rate
    const int e = j - 1 - a.R, k = e >> 2;             // predictor is the global MV: its set
    a.f2dirty[((size_t)k * a.nsb + sb) * 4 + (e & 3)] = (changed || a.init) ? 1 : 0;  // alone)
  }
  const bool mark = live && ((cm >> g0) & ((1ull << kCheckLanes) - 1)) != 0;
  const bool lead = live && j == 0;
  if (lead) a.active[sb] = mark;
  // wave-aggregated append to the list (the returned base orders the
  // workgroup's adds before its ticket below)
  const uint64_t m = __ballot(lead && mark);
  int base = 0;
  if (lane == 0 && m) base = atomicAdd(a.count, (int)__popcll(m));
  base = __shfl(base, 0, 64);
  if (lead && mark) a.list[base + __popcll(m & ((1ull << lane) - 1))] = sb;
  round_publish(a.pub);
}

// The same check with one role per wavefront: a workgroup holds 64
// superblocks, wavefront 0 their stacks and wavefront r (1 .. 5 R) their
// EPZS job r - 1, so no wavefront runs two roles' code one after the other
// (the 16-lane layout above executes the stack path and the EPZS path of
// its lanes in turn, with their loads' latencies in series).  A
// superblock's roles meet in LDS.
constexpr int kSplitSb = 64;
// One role of superblock sb's check: role 0 its stacks (pmask: the
// references whose rate predictors changed), role r its EPZS job r - 1.
// Returns whether what the role checked changed.
__device__ __forceinline__ bool check_role(const MvrefArgs &a, int sb, int role, uint32_t *pmask) {
  const int sx = sb % a.tw, sy = sb / a.tw;
  const int fsx = a.tx0 + sx, fsy = a.ty0 + sy;
  if (role == 0) {  // the stacks (as in mvref_kernel's lane 0)
    const int t0x = fsx - fsx % a.tws, t0y = fsy - fsy % a.ths;
    const int cols = min(a.tws * 16, a.w_in_b - t0x * 16);
    const int bx = (fsx - t0x) * 16, by = (fsy - t0y) * 16;
    const int X = fsx * 64, Y = fsy * 64;
    const bool split = a.lvl && (X + 64 > a.W || Y + 64 > a.H);
    Nb nb;
    nb.up = !split && by > 0;
    nb.left = !split && bx > 0;
    nb.tr = !split && by > 0 && bx + 16 < cols;
    nb.tl = !split && bx > 0 && by > 0;
    if (nb.up) nb.a = coded_at(a, sb - a.tw, X, Y - 4);
    if (nb.left) nb.l = coded_at(a, sb - 1, X - 4, Y);
    if (nb.tr) nb.r = coded_at(a, sb - a.tw + 1, X + 64, Y - 4);
    if (nb.tl) nb.d = coded_at(a, sb - a.tw - 1, X - 4, Y - 4);
    const MvStack st = stacks_of(a, nb, split, fsx, fsy);
    const bool changed = !same_stacks(a, a.stk[sb], st);
    uint32_t pm = 0;
#pragma unroll
    for (int k = 0; k < 2; k++)
      if (k < a.R && (a.init || !mv_eq(a.stk[sb].s[k][0], st.s[k][0]) ||
                      !mv_eq(a.stk[sb].s[k][1], st.s[k][1])))
        pm |= 1u << k;
    *pmask = pm;
    if (changed) set_stacks(a, sb, st);
    return changed;
  }
  return epzs_job(a, sb, fsx, fsy, role - 1);
}

// The end of a check of superblock sb (role's thread): its F3 / F2 dirty
// flags from the roles' changes cm (bit r: role r) and the rate predictors'
// pm; role 0 marks it and appends it, wave-aggregated (sbl = its lane).
__device__ __forceinline__ void check_finish(const MvrefArgs &a, int sb, int role, int sbl, bool live,
                                    uint32_t cm, uint32_t pm) {
  if (a.f3dirty && live && role >= 1 && role <= a.R)  // F3 job role - 1: its set or its pmv
    a.f3dirty[(size_t)(role - 1) * a.nsb + sb] = (((cm >> role) & 1) || ((pm >> (role - 1)) & 1)) ? 1 : 0;
  if (a.f2dirty && live && role > a.R) {  // F2 quadrant job: its set alone
    const int e = role - 1 - a.R, k = e >> 2;
    a.f2dirty[((size_t)k * a.nsb + sb) * 4 + (e & 3)] = (((cm >> role) & 1) || a.init) ? 1 : 0;
  }
  if (role == 0) {
    const bool mark = live && cm != 0;
    if (live) a.active[sb] = mark;
    const uint64_t m = __ballot(mark);
    int base = 0;
    if (sbl == 0 && m) base = atomicAdd(a.count, (int)__popcll(m));
    base = __shfl(base, 0, 64);
    if (mark) a.list[base + __popcll(m & ((1ull << sbl) - 1))] = sb;
  }
}

__global__ __launch_bounds__(1024) void mvref_split_kernel(MvrefArgs a) {
  __shared__ uint32_t chg[kSplitSb];  // per superblock: bit r = role r changed
  __shared__ uint32_t pmk[kSplitSb];  // role 0: the references whose rate predictors changed
  const int role = (int)(threadIdx.x >> 6), sbl = (int)(threadIdx.x & 63);
  const int sb = (int)blockIdx.x * kSplitSb + sbl;
  const bool live = sb < a.nsb;
  if (threadIdx.x < kSplitSb) chg[threadIdx.x] = pmk[threadIdx.x] = 0;
  __syncthreads();
  if (live) {
    uint32_t pm = 0;
    const bool changed = check_role(a, sb, role, &pm);
    if (role == 0) pmk[sbl] = pm;
    if (changed) atomicOr(&chg[sbl], 1u << role);
  }
  __syncthreads();
  check_finish(a, sb, role, sbl, live, chg[sbl], pmk[sbl]);
  round_publish(a.pub);
}

// The incremental check (a.plist): the same roles over the dependents of
// the previous check's list, 64 candidates per workgroup pass; a candidate
// is claimed once per check through epoch (the first claimant checks it).
__global__ __launch_bounds__(1024) void mvref_inc_kernel(MvrefArgs a) {
  __shared__ int32_t sbs[kSplitSb];
  __shared__ uint32_t chg[kSplitSb];
  __shared__ uint32_t pmk[kSplitSb];
  const int role = (int)(rv_tid() >> 6), sbl = (int)(rv_tid() & 63);
  const int items = 4 * __builtin_amdgcn_readfirstlane(*a.pcount);
  for (int base = (int)blockIdx.x * kSplitSb; base < items; base += (int)gridDim.x * kSplitSb) {
    if (role == 0) {
      int s = -1;
      const int it = base + sbl;
      if (it < items) {
        const int e = a.plist[it >> 2], d = it & 3;  // right, below-left, below, below-right
        const int nx = e % a.tw + (d == 0 ? 1 : d - 2), ny = e / a.tw + (d == 0 ? 0 : 1);
        if (nx >= 0 && nx < a.tw && ny < a.th) {
          const int c = ny * a.tw + nx;
          if (atomicMax(&a.epoch[c], a.tag) < a.tag) s = c;
        }
      }
      sbs[sbl] = s;
      chg[sbl] = pmk[sbl] = 0;
    }
    __syncthreads();
    const int sb = sbs[sbl];
    const bool live = sb >= 0;
    if (live) {
      uint32_t pm = 0;
      const bool changed = check_role(a, sb, role, &pm);
      if (role == 0) pmk[sbl] = pm;
      if (changed) atomicOr(&chg[sbl], 1u << role);
    }
    __syncthreads();
    check_finish(a, live ? sb : 0, role, sbl, live, chg[sbl], pmk[sbl]);
    __syncthreads();  // the slot tables are rewritten by the next pass
  }
  round_publish(a.pub);
}

// A decision predicted under a new stack: the same candidate, its MVs taken
// from the new stack (NEWMV keeps the last search's MV).  Only a guess that
// lets a change run down a dependency chain in one round; the fixed point
// does not depend on it.
__device__ inline BlkDec predict(BlkDec d, const MvStack &s, int M, int R) {
  if (d.cand == 255 || d.ref[0] == kIntraFrame) return d;
  const int c = d.cand, ns = R * M;
  if (c < ns) {
    const int k = c / M, m = c - k * M;
    if (m == kNearestMv) d.mv[0] = s.n[k] >= 1 ? s.s[k][0] : rv_mv{0, 0};
    if (m == kNear0Mv && s.n[k] >= 1) d.mv[0] = s.n[k] >= 2 ? s.s[k][1] : rv_mv{0, 0};
    return d;
  }
  switch (c - ns) {
    case kNearestNearest: d.mv[0] = s.c[0][0]; d.mv[1] = s.c[0][1]; break;
    case kNearNear: d.mv[0] = s.c[1][0]; d.mv[1] = s.c[1][1]; break;
    case kNearestNew: d.mv[0] = s.c[0][0]; break;
    case kNewNearest: d.mv[1] = s.c[0][1]; break;
    default: break;
  }
  return d;
}

// The tail rounds (few superblocks still changing, mostly along dependency
// chains): one workgroup per tile scans its superblocks in anti-diagonal
// wavefronts (x + 2 y = d: the left, above, top-right and top-left
// neighbours lie on earlier ones).  A superblock whose stack and EPZS sets
// held keeps its evaluated decision; one whose stack changed is marked and,
// for the superblocks after it, predicted (the same candidate under the new
// stack), so a chain of changes is evaluated in one round when the
// predictions hold.  The EPZS sets read the field of those (predicted)
// decisions, or the quadrant results.  The tile's decisions live in LDS.
// Per wavefront: (A) one thread per superblock, its stacks; (B) one thread
// per (superblock, EPZS job); (C) one thread per superblock, the mark.
constexpr int kScanThreads = 256, kScanMaxDiag = 64;
__global__ __launch_bounds__(kScanThreads) void mvref_scan_kernel(MvrefArgs a) {
  extern __shared__ BlkDec pd[];
  __shared__ uint8_t smark[kScanMaxDiag], sch[kScanMaxDiag];
  __shared__ uint32_t spm[kScanMaxDiag];
  const int gtx = (a.tw + a.tws - 1) / a.tws;
  const int lx0 = (int)(blockIdx.x % gtx) * a.tws, ly0 = (int)(blockIdx.x / gtx) * a.ths;
  const int twd = min(a.tws, a.tw - lx0), tht = min(a.ths, a.th - ly0);
  const int ndiag = (twd - 1) + 2 * (tht - 1) + 1;
  const int t0x = a.tx0 + lx0, t0y = a.ty0 + ly0;
  const int cols = min(a.tws * 16, a.w_in_b - t0x * 16);
  const int nj = a.epzs ? 5 * a.R : 0;  // EPZS jobs per superblock
  auto is_split = [&](int SX, int SY) { return a.lvl && ((SX + 1) * 64 > a.W || (SY + 1) * 64 > a.H); };
  __syncthreads();
  for (int d = 0; d < ndiag; d++) {
    const int ylo = max(0, (d - twd + 2) / 2), yhi = min(tht - 1, d / 2);
    const int nd = yhi - ylo + 1;  // superblocks on this wavefront (<= kScanMaxDiag)
    // (A) stacks
    for (int i = (int)threadIdx.x; i < nd; i += kScanThreads) {
      const int y = ylo + i, x = d - 2 * y;
      const int sb = (ly0 + y) * a.tw + lx0 + x;
      const int fsx = t0x + x, fsy = t0y + y;
      const int X = fsx * 64, Y = fsy * 64, bx = x * 16, by = y * 16;
      const bool split = is_split(fsx, fsy);
      // a neighbour: LDS (this tile), or a must_split leaf
      auto nbr = [&](int nx, int ny, int PX, int PY) -> BlkDec {
        if (is_split(t0x + nx, t0y + ny)) return coded_at(a, 0, PX, PY);
        BlkDec v = pd[ny * twd + nx];
        if (a.iwas && a.iwas[(ly0 + ny) * a.tw + lx0 + nx]) v.ref[0] = kIntraFrame, v.ref[1] = kNoneFrame;
        return v;
      };
      Nb nb;
      nb.up = !split && by > 0;
      nb.left = !split && bx > 0;
      nb.tr = !split && by > 0 && bx + 16 < cols;
      nb.tl = !split && bx > 0 && by > 0;
      if (nb.up) nb.a = nbr(x, y - 1, X, Y - 4);
      if (nb.left) nb.l = nbr(x - 1, y, X - 4, Y);
      if (nb.tr) nb.r = nbr(x + 1, y - 1, X + 64, Y - 4);
      if (nb.tl) nb.d = nbr(x - 1, y - 1, X - 4, Y - 4);
      const MvStack st = stacks_of(a, nb, split, fsx, fsy);
      const bool mark = !same_stacks(a, a.stk[sb], st);
      uint32_t pm = 0;
#pragma unroll
      for (int k = 0; k < 2; k++)
        if (k < a.R && (!mv_eq(a.stk[sb].s[k][0], st.s[k][0]) ||
                        !mv_eq(a.stk[sb].s[k][1], st.s[k][1])))
          pm |= 1u << k;
      const BlkDec cur = a.dec[sb];
      if (mark) set_stacks(a, sb, st);
      pd[y * twd + x] = mark ? predict(cur, st, kCandModes, a.R) : cur;
      smark[i] = mark;
      sch[i] = 0;
      spm[i] = pm;
    }
    __syncthreads();
    // (B) the EPZS sets, the field from the tile's (predicted) decisions
    for (int t = (int)threadIdx.x; t < nd * nj; t += kScanThreads) {
      const int i = t / nj, j = t - i * nj;
      const int y = ylo + i, x = d - 2 * y;
      const int sb = (ly0 + y) * a.tw + lx0 + x;
      const int fsx = t0x + x, fsy = t0y + y;
      auto fld = [&](int k, int X4, int Y4) -> rv_mv {
        const int SX = X4 >> 4, SY = Y4 >> 4;
        if (SX == fsx && SY == fsy) return rv_mv{0, 0};  // its own quadrants: after its F2
        const int gsb = (SY - a.ty0) * a.tw + (SX - a.tx0);
        const int lx = SX - t0x, ly = SY - t0y;
        BlkDec dd;
        dd.ref[0] = kIntraFrame;
        if (is_split(SX, SY)) {
          if (a.edge_ok) dd = coded_at(a, gsb, X4 * 4, Y4 * 4);
        } else if (lx >= 0 && lx < twd && ly >= 0 && ly < tht) {
          dd = pd[ly * twd + lx];
          if (a.iwas && a.iwas[gsb]) dd.ref[0] = kIntraFrame;
        } else {
          dd = coded_at(a, gsb, X4 * 4, Y4 * 4);
        }
        if (dd.ref[0] != kIntraFrame && dd.ref[0] - 1 == k) return dd.mv[0];
        const rv_mv h = a.hq[((size_t)k * a.nsb + gsb) * 4 + ((Y4 >> 3) & 1) * 2 + ((X4 >> 3) & 1)].best_mv;
        return rv_mv{(int16_t)(h.row * 2), (int16_t)(h.col * 2)};
      };
      const bool ch = epzs_job_f(a, sb, fsx, fsy, j, fld);
      if (ch) sch[i] = 1;  // (any writer)
      if (j < a.R) {
        if (a.f3dirty) a.f3dirty[(size_t)j * a.nsb + sb] = (ch || ((spm[i] >> j) & 1)) ? 1 : 0;
      } else if (a.f2dirty) {
        const int e = j - a.R;
        a.f2dirty[((size_t)(e >> 2) * a.nsb + sb) * 4 + (e & 3)] = ch ? 1 : 0;
      }
    }
    __syncthreads();
    // (C) the mark (a superblock marked by its sets alone keeps its decision)
    for (int i = (int)threadIdx.x; i < nd; i += kScanThreads) {
      const int y = ylo + i, x = d - 2 * y;
      const int sb = (ly0 + y) * a.tw + lx0 + x;
      const bool mark = smark[i] || sch[i];
      a.active[sb] = mark;
      if (!a.epzs && a.f3dirty)
        for (int k = 0; k < a.R; k++) a.f3dirty[(size_t)k * a.nsb + sb] = (spm[i] >> k) & 1;
      if (mark) a.list[atomicAdd(a.count, 1)] = sb;  // the returned index orders it before the ticket
    }
    __syncthreads();  // the wavefront's decisions before the next one reads them
  }
  round_publish(a.pub);
}
}  // namespace

int rv_mvref_round(const MvrefArgs &a, hipStream_t s, bool scan) {
  if (a.nsb <= 0) return RV_OK;
  // RAV1E_HIP_CHECK_SPLIT=0: the 16-lane check (A/B)
  static const bool check_split = !(getenv("RAV1E_HIP_CHECK_SPLIT") && getenv("RAV1E_HIP_CHECK_SPLIT")[0] == '0');
  // the scan: a tile's decisions in LDS, at most kScanMaxDiag superblocks
  // per wavefront; otherwise the Jacobi check
  const bool scan_ok = a.tws * a.ths <= kMvrefScanMaxSb && (a.ths < a.tws ? a.ths : a.tws) <= kScanMaxDiag;
  if (scan && !a.init && scan_ok) {
    const int ntiles = ((a.tw + a.tws - 1) / a.tws) * ((a.th + a.ths - 1) / a.ths);
    mvref_scan_kernel<<<ntiles, kScanThreads, (size_t)a.tws * a.ths * sizeof(BlkDec), s>>>(a);
  } else if (check_split && a.plist && a.epoch) {
    const int nr = 1 + (a.epzs ? 5 * a.R : 0);
    const int full = (a.nsb + kSplitSb - 1) / kSplitSb;
    const int grid = a.inc_grid > 0 ? std::min(a.inc_grid, full) : full;
    mvref_inc_kernel<<<grid, kSplitSb * nr, 0, s>>>(a);
  } else if (check_split) {
    const int nr = 1 + (a.epzs ? 5 * a.R : 0);
    mvref_split_kernel<<<(a.nsb + kSplitSb - 1) / kSplitSb, kSplitSb * nr, 0, s>>>(a);
  } else {
    mvref_kernel<<<(a.nsb * kCheckLanes + 255) / 256, 256, 0, s>>>(a);
  }
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

int rv_mvref_field(const MvrefArgs &a, rv_mv *field, hipStream_t s) {
  const int w8 = a.w_in_b >> 1, h8 = a.h_in_b >> 1;
  const int gw = std::min((a.tx0 + a.tw) * 8, w8) - a.tx0 * 8;
  const int gh = std::min((a.ty0 + a.th) * 8, h8) - a.ty0 * 8;
  if (gw <= 0 || gh <= 0) return RV_OK;
  mvref_field_kernel<<<(gw * gh + 255) / 256, 256, 0, s>>>(a, field);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}
