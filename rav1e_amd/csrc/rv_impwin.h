// rv_impwin.h -- block importances over the lookahead window
// (compute_block_importances, src/api/internal.rs:823-1081) for the replay's
// lookahead engine (rv_replay.hip, RvLaEngine).
//
// The reference propagates, for every frame of the window from the last one
// down to the second, each 8x8 block's share of (intra cost + its own
// importance) into the four blocks of each reference its MV-displaced area
// overlaps, with f32 `+=` in source raster order.  Where a source's
// contributions land depends only on its lookahead MV, so the device
// computes that once per frame (impwin_frame_data): a stable sort by target
// turns the frame's 4 x n_imp (target, source) pairs into per-target lists
// in source order (CSR, a counting sort: rv_csr.h).  A window pass (impwin_pass) is then one thread
// per target that adds its list's contributions onto its current value in
// that order -- the reference's sum, rounding for rounding, with no atomics.
#pragma once

#include "rv_device.h"

namespace rv {

// references whose lookahead a frame's importances propagate into: rav1e's
// distinct DPB slots of fi.ref_frames, at most 3 (src/api/internal.rs:875-882)
constexpr int kImpMaxRefs = 3;

// The importance data of one coded frame (a lookahead ring entry); every
// array over the frame's 8x8 blocks [h_imp][w_imp] (n = w_imp * h_imp).
struct ImpFrame {
  uint32_t *intra = nullptr;  // lookahead_intra_costs [n]
  rv_mv *mv8 = nullptr;       // [R][n]: lookahead_mvs[k][2y][2x] (the FL MV of the 16x16)
  float *frac = nullptr;      // [R][n]: max(1 - inter / intra, 0) (inter: get_satd at mv8)
  int32_t *off = nullptr;     // [R][n + 1]: target t's sources at src[off[t] .. off[t + 1])
  int32_t *src = nullptr;     // [R][4 n]: 4 * source + corner, by target, in source order
  float *imp = nullptr;       // [n]: block_importances while a window propagates
  float *fin = nullptr;       // [n]: the frame's final importances (log2(1 + imp / intra))
};

size_t impwin_frame_bytes(int n, int R);        // one ImpFrame's arrays
void impwin_frame_carve(ImpFrame &f, void *base, int n, int R);
size_t impwin_scratch_bytes(int n);             // impwin_lists' scratch

// A tile group's (tx0, ty0, tw, th superblocks) 8x8 importance blocks:
// [bx0, bx0 + bw) x [by0, by0 + bh) of the frame's w_imp x h_imp
inline void impwin_group_blocks(int tx0, int ty0, int tw, int th, int w_imp, int h_imp, int &bx0,
                                int &by0, int &bw, int &bh) {
  bx0 = tx0 * 8;
  by0 = ty0 * 8;
  bw = ((tx0 + tw) * 8 < w_imp ? (tx0 + tw) * 8 : w_imp) - bx0;
  bh = ((ty0 + th) * 8 < h_imp ? (ty0 + th) * 8 : h_imp) - by0;
}

// Frame data of the group's blocks of the coded frame whose luma input is
// `cur`: intra costs, the 8x8 blocks' lookahead MVs from `look` ([R][nsb][16]
// over the group's tw x th superblocks), their fractions against each
// reference's original frame refs[k].
int impwin_group_data(const rv_plane &cur, const rv_plane *refs, int R, int bit_depth,
                      const rv_fs_result *look, int tx0, int ty0, int tw, int th, int w_imp,
                      int h_imp, const ImpFrame &f, hipStream_t st);

// A group's part for the exchange (kImpPartBytes per block of its
// rectangle) out of the frame data, or (unpack) back into it.
constexpr int kImpPartBytes = 4 + 8 * kImpMaxRefs;
int impwin_part(const ImpFrame &f, int R, int tx0, int ty0, int tw, int th, int w_imp, int h_imp,
                void *buf, bool unpack, hipStream_t st);

// Once every block's data is in: per reference the target lists of the
// whole frame.
int impwin_lists(const ImpFrame &f, int R, int w_imp, int h_imp, void *scratch,
                 size_t scratch_bytes, hipStream_t st);

// The (frame, reference ks[i]) passes, i < np <= kImpMaxRefs, in one
// launch: the source frame's contributions (split over its nu reference
// slots) added onto ref_imp[i] (distinct frames).
int impwin_pass(const ImpFrame &src, const int *ks, float *const *ref_imp, int np, int nu,
                int w_imp, int h_imp, hipStream_t st);

// imp[0 .. count) (n floats each) to zero.
int impwin_zero(float *const *imp, int count, int n, hipStream_t st);

// The frame's final importances from its propagated ones.
int impwin_final(const ImpFrame &f, int w_imp, int h_imp, hipStream_t st);

}  // namespace rv
