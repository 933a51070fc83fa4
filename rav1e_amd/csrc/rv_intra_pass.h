// rv_intra_pass.h -- the replay's intra-mode screening / intra RDO pass
// (rv_intra_pass.hip), driven by rv_replay_frame.
#pragma once

#include "rv_rdo.h"

namespace rv {

// result word `c` of an intra winner: kIntraWord + 16 * luma mode + chroma mode
constexpr int kIntraWord = 1000;

// The group's superblock grid and tiles (a subset of rv_replay's Geo).
struct IntraGeo {
  int W, H, bd;
  int nsb, tw, tx0, ty0, tws, ths;
};

struct IntraScreenArgs {
  IntraGeo g;
  rv_plane rec[3];      // the frame being coded (Y, U, V)
  rv_plane org;         // its input luma
  const int32_t *list;  // superblocks to evaluate
  const int32_t *count;
  void *edges;          // out: 3 x kIntraEdge pixels per superblock
  uint8_t *modes;       // out: [n, m0, m1, m2] per superblock
};

struct IntraDecideArgs {
  IntraGeo g;
  const RdoWinner *win;       // the inter winners
  const uint8_t *modes;
  const uint64_t *lout, *uout, *vout;  // rv_rdo_intra's score outputs
  double lambda, ds_u, ds_v;
  const int32_t *list, *count;
  uint8_t *iwin;              // [luma, chroma] mode of an intra winner
  uint8_t *iwas;              // 1: the superblock's reconstruction is intra
  const uint8_t *elig;
  int32_t *mark;              // round stamp: already in the next list
  int round;
  uint64_t *words;            // result words (the winner's four at win_off)
  int words_per_sb, win_off;
  int32_t *commit_list, *commit_count, *revert_list, *revert_count;
  int32_t *next_list, *next_count;
};

}  // namespace rv

int rv_intra_elig(const rv::IntraGeo &g, const rv::RdoWinner *win, uint8_t *elig, uint8_t *iwas,
                  int32_t *mark, int32_t *list, int32_t *count, hipStream_t s);
int rv_intra_screen(const rv::IntraScreenArgs &a, int n, int hbd, hipStream_t s);
int rv_intra_decide(const rv::IntraDecideArgs &a, hipStream_t s);
int rv_intra_stats(int nsb, const uint8_t *elig, const uint8_t *iwas, uint32_t *out, hipStream_t s);
