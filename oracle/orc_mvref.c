/* Oracle restatement of rav1e's MV reference stack (test infrastructure:
 * only tests/, smoke() and bench.py's cpu_baseline leg load it, through
 * orc_replay.c).
 *
 * ContextWriter::find_mvrefs / setup_mvref_list (src/context.rs:2650-2965)
 * over a tile's block grid: the row above, the column to the left, the
 * top-right block, REF_CAT_LEVEL, the top-left block and the outer rows /
 * columns, the weight sort, the extra search (7.10.2.12) and the MV clamp.
 * Block records carry what the scans read: ref_frames, mv, mode (for the
 * NEWMV count) and the block size in 4x4 units.
 */
#include <string.h>

#include "orc_common.h"

#define MAX_REF_MV_STACK_SIZE 8 /* src/context.rs:89 */
#define REF_CAT_LEVEL 640       /* src/context.rs:90 */
#define MVREF_ROW_COLS 3        /* src/partition.rs:98 */

static int mvq(orc_mv a, orc_mv b) { return a.row == b.row && a.col == b.col; }
static int iabs(int v) { return v < 0 ? -v : v; }
static int imin(int a, int b) { return a < b ? a : b; }
static int imax(int a, int b) { return a > b ? a : b; }

typedef struct {
  const orc_blk *g;
  int stride, cols, rows; /* the tile: grid pitch, bc.blocks.cols() / rows() */
} tgrid;

static const orc_blk *blk_at(const tgrid *t, int x, int y) { return &t->g[(size_t)y * t->stride + x]; }

/* Block::is_inter (src/context.rs:1417): mode >= NEARESTMV */
static int is_inter(const orc_blk *b) { return b->ref[0] != ORC_INTRA_FRAME; }

/* find_matching_mv / find_matching_comp_mv_and_update_weight
 * (src/context.rs:2326-2364) */
static int match_weight(orc_mv_cand *st, int n, orc_mv m, uint32_t w) {
  for (int i = 0; i < n; i++)
    if (mvq(st[i].this_mv, m)) {
      st[i].weight += w;
      return 1;
    }
  return 0;
}
static int match_comp_weight(orc_mv_cand *st, int n, orc_mv m0, orc_mv m1, uint32_t w) {
  for (int i = 0; i < n; i++)
    if (mvq(st[i].this_mv, m0) && mvq(st[i].comp_mv, m1)) {
      st[i].weight += w;
      return 1;
    }
  return 0;
}

/* add_ref_mv_candidate (src/context.rs:2366-2435) */
static int add_ref_mv_candidate(const int rf[2], const orc_blk *b, orc_mv_cand *st, int *n,
                                uint32_t weight, int *newmv_count, int compound) {
  if (!is_inter(b)) return 0;
  if (compound) {
    if (b->ref[0] != rf[0] || b->ref[1] != rf[1]) return 0;
    if (!match_comp_weight(st, *n, b->mv[0], b->mv[1], weight) && *n < MAX_REF_MV_STACK_SIZE) {
      st[*n].this_mv = b->mv[0];
      st[*n].comp_mv = b->mv[1];
      st[*n].weight = weight;
      (*n)++;
    }
    if (b->newmv) (*newmv_count)++;
    return 1;
  }
  int found = 0;
  for (int i = 0; i < 2; i++) {
    if (b->ref[i] != rf[0]) continue;
    if (!match_weight(st, *n, b->mv[i], weight) && *n < MAX_REF_MV_STACK_SIZE) {
      st[*n].this_mv = b->mv[i];
      st[*n].comp_mv = (orc_mv){0, 0};
      st[*n].weight = weight;
      (*n)++;
    }
    if (b->newmv) (*newmv_count)++;
    found = 1;
  }
  return found;
}

/* scan_row_mbmi (src/context.rs:2491-2555) */
static int scan_row(const tgrid *t, int bx, int by, int row_offset, int max_row_offs,
                    int *processed_rows, const int rf[2], orc_mv_cand *st, int *n, int *newmv,
                    int bw4, int compound) {
  const int target_n4_w = bw4;
  const int end_mi = imin(imin(target_n4_w, t->cols - bx), 16);
  const int n4_w_8 = 2, n4_w_16 = 4;
  int col_offset = 0;
  if (iabs(row_offset) > 1) {
    col_offset = 1;
    if ((bx & 1) && target_n4_w < n4_w_8) col_offset -= 1;
  }
  const int use_step_16 = target_n4_w >= 16;
  int found = 0;
  for (int i = 0; i < end_mi;) {
    const orc_blk *c = blk_at(t, bx + col_offset + i, by + row_offset);
    const int n4_w = c->n4_w;
    int len = imin(target_n4_w, n4_w);
    if (use_step_16)
      len = imax(n4_w_16, len);
    else if (iabs(row_offset) > 1)
      len = imax(len, n4_w_8);
    uint32_t weight = 2;
    if (target_n4_w >= n4_w_8 && target_n4_w <= n4_w) {
      const int inc = imin(-max_row_offs + row_offset + 1, c->n4_h);
      weight = imax((int)weight, inc);
      *processed_rows = inc - row_offset - 1;
    }
    if (add_ref_mv_candidate(rf, c, st, n, (uint32_t)len * weight, newmv, compound)) found = 1;
    i += len;
  }
  return found;
}

/* scan_col_mbmi (src/context.rs:2557-2621) */
static int scan_col(const tgrid *t, int bx, int by, int col_offset, int max_col_offs,
                    int *processed_cols, const int rf[2], orc_mv_cand *st, int *n, int *newmv,
                    int bh4, int compound) {
  const int target_n4_h = bh4;
  const int end_mi = imin(imin(target_n4_h, t->rows - by), 16);
  const int n4_h_8 = 2, n4_h_16 = 4;
  int row_offset = 0;
  if (iabs(col_offset) > 1) {
    row_offset = 1;
    if ((by & 1) && target_n4_h < n4_h_8) row_offset -= 1;
  }
  const int use_step_16 = target_n4_h >= 16;
  int found = 0;
  for (int i = 0; i < end_mi;) {
    const orc_blk *c = blk_at(t, bx + col_offset, by + row_offset + i);
    const int n4_h = c->n4_h;
    int len = imin(target_n4_h, n4_h);
    if (use_step_16)
      len = imax(n4_h_16, len);
    else if (iabs(col_offset) > 1)
      len = imax(len, n4_h_8);
    uint32_t weight = 2;
    if (target_n4_h >= n4_h_8 && target_n4_h <= n4_h) {
      const int inc = imin(-max_col_offs + col_offset + 1, c->n4_w);
      weight = imax((int)weight, inc);
      *processed_cols = inc - col_offset - 1;
    }
    if (add_ref_mv_candidate(rf, c, st, n, (uint32_t)len * weight, newmv, compound)) found = 1;
    i += len;
  }
  return found;
}

/* scan_blk_mbmi (src/context.rs:2623-2642) */
static int scan_blk(const tgrid *t, int x, int y, const int rf[2], orc_mv_cand *st, int *n,
                    int *newmv, int compound) {
  if (x >= t->cols || y >= t->rows) return 0;
  return add_ref_mv_candidate(rf, blk_at(t, x, y), st, n, 2 * 2, newmv, compound);
}

/* has_tr (src/partition.rs:695-750), 64x64 superblocks */
static int has_tr(int bx, int by, int bw4, int bh4) {
  const int sb_mi = 16, mask_row = by & 15, mask_col = bx & 15;
  int bs = imax(bw4, bh4);
  if (bs > 16) return 0;
  int tr = !((mask_row & bs) && (mask_col & bs));
  while (bs < sb_mi) {
    if (mask_col & bs) {
      if ((mask_col & (2 * bs)) && (mask_row & (2 * bs))) {
        tr = 0;
        break;
      }
    } else {
      break;
    }
    bs <<= 1;
  }
  if (bw4 < bh4 && (bx & bw4) == 0) tr = 1;
  if (bw4 > bh4 && (by & bh4) != 0) tr = 0;
  return tr;
}

/* find_valid_row_offs / find_valid_col_offs (src/context.rs:2308-2324) */
static int valid_offs(int off, int mi, int n) { return imin(imax(off, -mi), n - mi - 1); }

/* add_extra_mv_candidate (src/context.rs:2437-2489) */
static void add_extra(const orc_blk *b, const int rf[2], orc_mv_cand *st, int *n,
                      const uint8_t *sign_bias, int compound, int id_cnt[2], orc_mv id_mvs[2][2],
                      int diff_cnt[2], orc_mv diff_mvs[2][2]) {
  for (int cl = 0; cl < 2; cl++) {
    const int cr = b->ref[cl];
    if (cr == ORC_INTRA_FRAME || cr == ORC_NONE_FRAME) continue;
    if (compound) {
      for (int list = 0; list < 2; list++) {
        orc_mv m = b->mv[cl];
        if (cr == rf[list] && id_cnt[list] < 2) {
          id_mvs[list][id_cnt[list]++] = m;
        } else if (diff_cnt[list] < 2) {
          if (sign_bias[cr - 1] != sign_bias[rf[list] - 1]) {
            m.row = (int16_t)-m.row;
            m.col = (int16_t)-m.col;
          }
          diff_mvs[list][diff_cnt[list]++] = m;
        }
      }
    } else {
      orc_mv m = b->mv[cl];
      if (sign_bias[cr - 1] != sign_bias[rf[0] - 1]) {
        m.row = (int16_t)-m.row;
        m.col = (int16_t)-m.col;
      }
      int found = 0;
      for (int i = 0; i < *n; i++) found |= mvq(st[i].this_mv, m);
      if (!found) {
        st[*n].this_mv = m;
        st[*n].comp_mv = (orc_mv){0, 0};
        st[*n].weight = 2;
        (*n)++;
      }
    }
  }
}

int orc_find_mvrefs(const orc_blk *grid, int stride, int cols, int rows, int tile_mi_x,
                    int tile_mi_y, int frame_cols, int frame_rows, int bx, int by, int bw4,
                    int bh4, const int ref_frames[2], const uint8_t *sign_bias,
                    orc_mv_cand stack[9], int *n_out) {
  const tgrid t = {grid, stride, cols, rows};
  const int compound = ref_frames[1] != ORC_NONE_FRAME;
  int n = 0;
  *n_out = 0;
  if (ref_frames[0] == ORC_INTRA_FRAME) return 0; /* find_mvrefs, :2957-2962 */
  const int target_n4_h = bh4, target_n4_w = bw4;
  int max_row_offs = 0, max_col_offs = 0;
  const int row_adj = target_n4_h < 2 && (by & 1);
  const int col_adj = target_n4_w < 2 && (bx & 1);
  int processed_rows = 0, processed_cols = 0;
  const int up_avail = by > 0, left_avail = bx > 0;
  if (up_avail) {
    max_row_offs = -2 * MVREF_ROW_COLS + row_adj;
    if (target_n4_h < 2) max_row_offs = -2 * 2 + row_adj;
    max_row_offs = valid_offs(max_row_offs, by, rows);
  }
  if (left_avail) {
    max_col_offs = -2 * MVREF_ROW_COLS + col_adj;
    if (target_n4_w < 2) max_col_offs = -2 * 2 + col_adj;
    max_col_offs = valid_offs(max_col_offs, bx, cols);
  }
  int row_match = 0, col_match = 0, newmv_count = 0;
  if (iabs(max_row_offs) >= 1)
    row_match |= scan_row(&t, bx, by, -1, max_row_offs, &processed_rows, ref_frames, stack, &n,
                          &newmv_count, bw4, compound);
  if (iabs(max_col_offs) >= 1)
    col_match |= scan_col(&t, bx, by, -1, max_col_offs, &processed_cols, ref_frames, stack, &n,
                          &newmv_count, bh4, compound);
  if (has_tr(bx, by, bw4, bh4) && by > 0)
    row_match |= scan_blk(&t, bx + target_n4_w, by - 1, ref_frames, stack, &n, &newmv_count,
                          compound);
  const int nearest_match = row_match + col_match;
  for (int i = 0; i < n; i++) stack[i].weight += REF_CAT_LEVEL; /* add_offset */
  int far_newmv = 0;
  if (bx > 0 && by > 0)
    row_match |= scan_blk(&t, bx - 1, by - 1, ref_frames, stack, &n, &far_newmv, compound);
  for (int idx = 2; idx <= MVREF_ROW_COLS; idx++) {
    const int row_offset = -2 * idx + 1 + row_adj, col_offset = -2 * idx + 1 + col_adj;
    if (iabs(row_offset) <= iabs(max_row_offs) && iabs(row_offset) > processed_rows)
      row_match |= scan_row(&t, bx, by, row_offset, max_row_offs, &processed_rows, ref_frames,
                            stack, &n, &far_newmv, bw4, compound);
    if (iabs(col_offset) <= iabs(max_col_offs) && iabs(col_offset) > processed_cols)
      col_match |= scan_col(&t, bx, by, col_offset, max_col_offs, &processed_cols, ref_frames,
                            stack, &n, &far_newmv, bh4, compound);
  }
  const int total_match = row_match + col_match;
  int mode_context;
  if (nearest_match == 0)
    mode_context = imin(total_match, 1) + (total_match << 4);
  else if (nearest_match == 1)
    mode_context = 3 - imin(newmv_count, 1) + ((2 + total_match) << 4);
  else
    mode_context = 5 - imin(newmv_count, 1) + (5 << 4);
  /* 7.10.2.11: sort by weight, descending (slice::sort_by is stable) */
  for (int i = 1; i < n; i++)
    for (int j = i; j > 0 && stack[j].weight > stack[j - 1].weight; j--) {
      orc_mv_cand tmp = stack[j];
      stack[j] = stack[j - 1];
      stack[j - 1] = tmp;
    }
  if (n < 2) {
    /* 7.10.2.12 extra search */
    const int w4 = imin(imin(bw4, 16), cols - bx), h4 = imin(imin(bh4, 16), rows - by);
    const int num4x4 = imin(w4, h4);
    int id_cnt[2] = {0, 0}, diff_cnt[2] = {0, 0};
    orc_mv id_mvs[2][2], diff_mvs[2][2];
    memset(id_mvs, 0, sizeof(id_mvs));
    memset(diff_mvs, 0, sizeof(diff_mvs));
    for (int pass = up_avail ? 0 : 1; pass < (left_avail ? 2 : 1); pass++) {
      for (int idx = 0; idx < num4x4 && n < 2;) {
        const orc_blk *b = pass == 0 ? blk_at(&t, bx + idx, by - 1) : blk_at(&t, bx - 1, by + idx);
        add_extra(b, ref_frames, stack, &n, sign_bias, compound, id_cnt, id_mvs, diff_cnt,
                  diff_mvs);
        idx += pass == 0 ? b->n4_w : b->n4_h;
      }
    }
    if (compound) {
      orc_mv comb[2][2];
      memset(comb, 0, sizeof(comb));
      for (int list = 0; list < 2; list++) {
        int cc = 0;
        for (int i = 0; i < id_cnt[list]; i++) comb[cc++][list] = id_mvs[list][i];
        for (int i = 0; i < diff_cnt[list] && cc < 2; i++) comb[cc++][list] = diff_mvs[list][i];
      }
      if (n == 1) {
        const int same = mvq(comb[0][0], stack[0].this_mv) && mvq(comb[0][1], stack[0].comp_mv);
        stack[1].this_mv = comb[same ? 1 : 0][0];
        stack[1].comp_mv = comb[same ? 1 : 0][1];
        stack[1].weight = 2;
        n = 2;
      } else {
        for (int i = 0; i < 2; i++) {
          stack[n].this_mv = comb[i][0];
          stack[n].comp_mv = comb[i][1];
          stack[n].weight = 2;
          n++;
        }
      }
    }
  }
  /* clamp (src/context.rs:2911-2941) */
  const int fx = tile_mi_x + bx, fy = tile_mi_y + by;
  const int border_w = 128 + bw4 * 4 * 8, border_h = 128 + bh4 * 4 * 8;
  const int xmin = -fx * 32 - border_w, xmax = (frame_cols - fx - bw4) * 32 + border_w;
  const int ymin = -fy * 32 - border_h, ymax = (frame_rows - fy - bh4) * 32 + border_h;
  for (int i = 0; i < n; i++) {
    orc_mv *m[2] = {&stack[i].this_mv, &stack[i].comp_mv};
    for (int j = 0; j < 2; j++) {
      m[j]->row = (int16_t)imin(imax(m[j]->row, ymin), ymax);
      m[j]->col = (int16_t)imin(imax(m[j]->col, xmin), xmax);
    }
  }
  *n_out = n;
  return mode_context;
}
