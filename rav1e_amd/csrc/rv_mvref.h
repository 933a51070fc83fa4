// rv_mvref.h -- rav1e's MV reference stacks of the replay's 64x64
// superblocks (rv_mvref.hip), driven by rv_replay_frame's coding-order
// rounds (DESIGN.md §3 "MV stacks in coding order").
#pragma once

#include "rv_chain.h"
#include "rv_epzs.h"
#include "rv_rdo.h"

namespace rv {

// RefType codes of a coded block (src/partition.rs RefType): INTRA_FRAME 0,
// the replay's reference k is 1 + k, NONE_FRAME 8
constexpr int kIntraFrame = 0, kNoneFrame = 8;

// The fields of a coded block (Block, src/context.rs:1395-1440) that
// find_mvrefs reads: ref_frames and mv.
struct BlkDec {
  int8_t ref[2];
  int8_t newmv;
  uint8_t cand;  // the replay's candidate index of the winner (255: intra / none)
  rv_mv mv[2];
};

struct MvrefArgs {
  // the group's superblock grid, its tiles and the frame (4x4 units)
  int nsb, tw, th, tx0, ty0, tws, ths, W, H, w_in_b, h_in_b;
  int R, comp;             // references; compound stack on this frame
  uint32_t sign_bias;      // bit k: ref_frame_sign_bias of reference k (a bit mask: no
                           // runtime index into the arguments)
  const BlkDec *dec;       // the superblocks' coded blocks
  const uint8_t *iwas;     // null, or 1: the superblock is an intra winner
  MvStack *stk;            // in / out: the stacks the superblocks were evaluated with
  uint8_t *active;         // out: 1 = (re-)evaluate this round
  int32_t *count;          // out: += superblocks marked (= pub.cnt)
  int32_t *list;           // out: the marked superblocks (any order), count of them
  RoundPub pub;            // the count's publication (pub.host null: none)
  rv_ds_job *jf, *js;      // the F3 jobs [R][nsb]: pmv = the stack's first two
  int init;                // 1: mark every superblock (the frame's first round)
  // speed 10 frame-edge leaves (a top-right neighbour past the right edge):
  // lvl = the edge superblocks are split; per level 1..3 (those holding
  // leaves) the winners, sub-pel MVs and candidate geometry
  int lvl;
  const RdoWinner *lwin[4];
  const rv_fs_result *lsub[4];
  CandGeo lcg[4];
  // EPZS (get_subset_predictors, src/me.rs:82-174): a superblock is also
  // marked when the predictor set of one of its F2 (build_half_res_pmvs
  // quadrant) or F3 (64x64 full-pel) searches changed, the new set stored
  // into the job.  The encode's tile field at a 4x4 unit: the coded block's
  // first MV under its first reference, else the superblock's F2 quadrant
  // MV (hq; the first check: the lookahead's, a guess), zero inside the
  // superblock searching.
  int epzs;
  EpzsGeo eg;
  rv_ds_job *jh;                // F2 jobs [R][nsb][4]
  const rv_fs_result *coarse;   // F1 [R][nsb]
  const rv_fs_result *hq;       // quadrant MVs (half-res) [R][nsb][4]
  const rv_mv *prev;            // the LAST reference's field, [h_in_b/2][w_in_b/2][R]; null: none
  int edge_ok;                  // the frame-edge leaves are final (lwin / lsub readable)
  // out (null: none): per F3 job [R][nsb], 1 = its predictor set or rate
  // predictors (pmv) changed, so its full-pel and sub-pel searches must
  // re-run; a listed superblock's other jobs keep their results
  uint8_t *f3dirty;
  uint8_t *f2dirty;  // out (null: none): per F2 job [R][nsb][4], 1 = its set changed
  int field_guess_la;  // the first check: the EPZS field from the quadrants alone (A/B)
  // An incremental check (plist non-null): only the superblocks whose inputs
  // the previous round can have changed -- the right, below-left, below and
  // below-right neighbours of every superblock the previous check listed
  // (its list plist, *pcount entries): a superblock's stacks and EPZS sets
  // read only its left, top-left, top and top-right neighbours (DESIGN.md
  // §3).  epoch[sb] holds the tag of the last check that claimed sb (each
  // candidate is checked once per check); tag > every earlier check's.
  const int32_t *plist;
  const int32_t *pcount;
  uint32_t *epoch;
  uint32_t tag;
  int inc_grid;  // workgroups of the incremental check (0: the full check's)
};

// The decision record of superblock sb's winner (candidate c of the
// superblock grid cg, or an intra word)
__device__ inline BlkDec blk_dec_of(const CandGeo &cg, const rv_fs_result *sub, int sb, int c) {
  BlkDec d;
  d.ref[1] = kNoneFrame;
  d.newmv = 0;
  d.cand = 255;
  d.mv[0] = d.mv[1] = rv_mv{0, 0};
  const int ns = cg.R * cg.M;
  if (c >= 1000 || c < 0 || c >= ns + kCompModes) {  // kIntraWord (the range guards the reads)
    d.ref[0] = kIntraFrame;
  } else if (c < ns) {
    d.cand = (uint8_t)c;
    d.ref[0] = (int8_t)(1 + c / cg.M);
    (void)cand_mv(cg, sub, sb, c, &d.mv[0]);
    d.newmv = (c % cg.M) == kNewMv;
  } else {
    d.cand = (uint8_t)c;
    d.ref[0] = 1;
    d.ref[1] = 2;
    comp_mvs(cg, sub, sb, c - ns, &d.mv[0], &d.mv[1]);
    d.newmv = (c - ns) >= kNewNew && (c - ns) <= kNewNearest;
  }
  return d;
}

}  // namespace rv

// One round over the group's superblocks (the first marks every one); scan:
// the tail rounds' predictive per-tile wavefront scan (its tile must fit
// the 64 KiB of LDS a workgroup may take: RV_EINVAL otherwise).
int rv_mvref_round(const rv::MvrefArgs &a, hipStream_t s, bool scan = false);
// The coded frame's field (the frame_mvs subset C of later frames reads) of
// the group's part, into field ([h_in_b/2][w_in_b/2][R] rv_mv).
int rv_mvref_field(const rv::MvrefArgs &a, rv_mv *field, hipStream_t s);
// The largest tile (superblocks) the scan takes.
constexpr int kMvrefScanMaxSb = (65536 - 1024) / (int)sizeof(rv::BlkDec);  // + the scan's static LDS
