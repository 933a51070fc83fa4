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
#include "rv_mvref.h"

using namespace rv;

namespace {

struct Cand {
  rv_mv t, c;  // this_mv, comp_mv
  uint32_t w;
};

__device__ inline bool inter_of(const BlkDec &b) { return b.ref[0] != kIntraFrame; }

// add_ref_mv_candidate (src/context.rs:2366-2435), MAX_REF_MV_STACK_SIZE 8
__device__ inline void add_ref(Cand *st, int &n, const BlkDec &b, uint32_t w, int rf0, int rf1,
                               bool compound) {
  if (!inter_of(b)) return;
  if (compound) {
    if (b.ref[0] != rf0 || b.ref[1] != rf1) return;
    for (int i = 0; i < n; i++)
      if (mv_eq(st[i].t, b.mv[0]) && mv_eq(st[i].c, b.mv[1])) {
        st[i].w += w;
        return;
      }
    if (n < 8) st[n++] = Cand{b.mv[0], b.mv[1], w};
    return;
  }
  for (int i = 0; i < 2; i++) {
    if (b.ref[i] != rf0) continue;
    bool found = false;
    for (int j = 0; j < n && !found; j++)
      if (mv_eq(st[j].t, b.mv[i])) {
        st[j].w += w;
        found = true;
      }
    if (!found && n < 8) st[n++] = Cand{b.mv[i], rv_mv{0, 0}, w};
  }
}

__device__ inline rv_mv neg(rv_mv m) { return rv_mv{(int16_t)-m.row, (int16_t)-m.col}; }

struct Nb {
  bool up, left, tr, tl;
  BlkDec a, l, r, d;  // above, left, top-right, top-left
};

// setup_mvref_list of a 64x64 block for ref_frames (rf0, rf1; rf1 = NONE:
// single); n out, entries into st (clamped)
__device__ inline int stack64(const Nb &nb, int rf0, int rf1, const uint8_t *sbias, int fx, int fy,
                              int fcols, int frows, Cand *st) {
  const bool compound = rf1 != kNoneFrame;
  int n = 0;
  if (nb.up) add_ref(st, n, nb.a, 16 * 6, rf0, rf1, compound);
  if (nb.left) add_ref(st, n, nb.l, 16 * 6, rf0, rf1, compound);
  if (nb.tr) add_ref(st, n, nb.r, 4, rf0, rf1, compound);
  for (int i = 0; i < n; i++) st[i].w += 640;  // add_offset, REF_CAT_LEVEL
  if (nb.tl) add_ref(st, n, nb.d, 4, rf0, rf1, compound);
  // 7.10.2.11: stable sort, descending weight
  for (int i = 1; i < n; i++)
    for (int j = i; j > 0 && st[j].w > st[j - 1].w; j--) {
      const Cand t = st[j];
      st[j] = st[j - 1];
      st[j - 1] = t;
    }
  if (n < 2) {
    // 7.10.2.12: the above block (pass 0), then the left one (pass 1); each
    // 64x64 pass reads one block (idx += n4_w = 16)
    int idc[2] = {0, 0}, dfc[2] = {0, 0};
    rv_mv idm[2][2], dfm[2][2];
    for (int p = nb.up ? 0 : 1; p < (nb.left ? 2 : 1); p++) {
      if (n >= 2) break;
      const BlkDec &b = p == 0 ? nb.a : nb.l;
      for (int cl = 0; cl < 2; cl++) {
        const int cr = b.ref[cl];
        if (cr == kIntraFrame || cr == kNoneFrame) continue;
        if (compound) {
          for (int list = 0; list < 2; list++) {
            const int rl = list ? rf1 : rf0;
            if (cr == rl && idc[list] < 2) {
              idm[list][idc[list]++] = b.mv[cl];
            } else if (dfc[list] < 2) {
              dfm[list][dfc[list]++] = sbias[cr - 1] != sbias[rl - 1] ? neg(b.mv[cl]) : b.mv[cl];
            }
          }
        } else {
          const rv_mv m = sbias[cr - 1] != sbias[rf0 - 1] ? neg(b.mv[cl]) : b.mv[cl];
          bool found = false;
          for (int j = 0; j < n; j++) found |= mv_eq(st[j].t, m);
          if (!found) st[n++] = Cand{m, rv_mv{0, 0}, 2};
        }
      }
    }
    if (compound) {
      rv_mv cm[2][2] = {{rv_mv{0, 0}, rv_mv{0, 0}}, {rv_mv{0, 0}, rv_mv{0, 0}}};
      for (int list = 0; list < 2; list++) {
        int cc = 0;
        for (int i = 0; i < idc[list]; i++) cm[cc++][list] = idm[list][i];
        for (int i = 0; i < dfc[list] && cc < 2; i++) cm[cc++][list] = dfm[list][i];
      }
      if (n == 1) {
        const int pick = mv_eq(cm[0][0], st[0].t) && mv_eq(cm[0][1], st[0].c) ? 1 : 0;
        st[n++] = Cand{cm[pick][0], cm[pick][1], 2};
      } else {
        st[n++] = Cand{cm[0][0], cm[0][1], 2};
        st[n++] = Cand{cm[1][0], cm[1][1], 2};
      }
    }
  }
  // clamp (src/context.rs:2911-2941), 64x64: border 128 + 512
  const int xmin = -fx * 32 - 640, xmax = (fcols - fx - 16) * 32 + 640;
  const int ymin = -fy * 32 - 640, ymax = (frows - fy - 16) * 32 + 640;
  for (int i = 0; i < n && i < 2; i++) {
    st[i].t = rv_mv{(int16_t)clampi(st[i].t.row, ymin, ymax), (int16_t)clampi(st[i].t.col, xmin, xmax)};
    st[i].c = rv_mv{(int16_t)clampi(st[i].c.row, ymin, ymax), (int16_t)clampi(st[i].c.col, xmin, xmax)};
  }
  return n;
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
  const int B = 64 >> l;
  const CandGeo &g = a.lcg[l];
  const int b = (Y / B - g.ty0) * g.tw + (X / B - g.tx0);
  return blk_dec_of(g, a.lsub[l], b, a.lwin[l][b].c);
}

__global__ __launch_bounds__(256) void mvref_kernel(MvrefArgs a) {
  const int sb = blockIdx.x * 256 + threadIdx.x;
  bool mark = false;
  if (sb < a.nsb) {
    const int sx = sb % a.tw, sy = sb / a.tw;
    const int fsx = a.tx0 + sx, fsy = a.ty0 + sy;  // frame superblock
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
    MvStack s;
    Cand st[10];
    for (int k = 0; k < 2; k++) {
      s.n[k] = 0;
      s.s[k][0] = s.s[k][1] = rv_mv{0, 0};
    }
    for (int k = 0; k < a.R && !split; k++) {
      const int n = stack64(nb, 1 + k, kNoneFrame, a.sign_bias, fsx * 16, fsy * 16, a.w_in_b,
                            a.h_in_b, st);
      s.n[k] = n < 2 ? n : 2;
      if (n >= 1) s.s[k][0] = st[0].t;
      if (n >= 2) s.s[k][1] = st[1].t;
    }
    s.c[0][0] = s.c[0][1] = s.c[1][0] = s.c[1][1] = rv_mv{0, 0};
    if (a.comp && !split) {
      (void)stack64(nb, 1, 2, a.sign_bias, fsx * 16, fsy * 16, a.w_in_b, a.h_in_b, st);
      s.c[0][0] = st[0].t;
      s.c[0][1] = st[0].c;
      s.c[1][0] = st[1].t;
      s.c[1][1] = st[1].c;
    }
    const MvStack &o = a.stk[sb];
    bool same = !a.init;
    for (int k = 0; k < a.R && same; k++)
      same = o.n[k] == s.n[k] && mv_eq(o.s[k][0], s.s[k][0]) && mv_eq(o.s[k][1], s.s[k][1]);
    if (a.comp && same)
      same = mv_eq(o.c[0][0], s.c[0][0]) && mv_eq(o.c[0][1], s.c[0][1]) &&
             mv_eq(o.c[1][0], s.c[1][0]) && mv_eq(o.c[1][1], s.c[1][1]);
    mark = !same;
    a.active[sb] = mark;
    if (mark) {
      a.stk[sb] = s;
      // motion_estimation's rate predictors (src/rdo.rs:858-870)
      for (int k = 0; k < a.R; k++) {
        const int j = k * a.nsb + sb;
        a.jf[j].pmv[0] = a.js[j].pmv[0] = s.s[k][0];
        a.jf[j].pmv[1] = a.js[j].pmv[1] = s.s[k][1];
      }
    }
  }
  const uint64_t m = __ballot(mark);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd(a.count, (int)__popcll(m));
}

}  // namespace

int rv_mvref_round(const MvrefArgs &a, hipStream_t s) {
  if (a.nsb <= 0) return RV_OK;
  mvref_kernel<<<(a.nsb + 255) / 256, 256, 0, s>>>(a);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}
