// rv_rdo.h -- the fused RDO inter-candidate launches (rv_rdo.hip) of the
// replay driver: stage F4 (score every candidate) and F6 (commit the
// winner of every superblock into the reconstruction).
#pragma once

#include "rv_chain.h"
#include "rv_device.h"
#include "rv_quant.h"

namespace rv {

struct RdoPlane {
  rv_plane org;                  // source plane
  rv_plane ref[2];               // reference planes of this plane type (the replay's R <= 2)
  rv_plane dst;                  // commit: the reconstruction plane (frame slot)
  int32_t *levels;               // commit: CA i32 levels per transform block
  uint64_t *out;                 // score: [dist skip, dist non-skip, rate] per transform block
  QCtx q;                        // QuantizationContext of this plane's transform
};

// The winner of a superblock (score_candidates -> commit).
struct RdoWinner {
  int32_t c;     // candidate index (ref * M + mode)
  int32_t skip;  // 1: the skip variant (no residual)
  double cost;   // compute_rd_cost
  uint64_t dist; // its ScaledDistortion
};

struct RdoArgs {
  RdoPlane p[2];       // chroma: U, V (the launch's blocks cover both)
  CandGeo g;           // superblock grid + candidate MVs (rv_chain.h)
  const rv_fs_result *sub;  // NEWMV of every (reference, superblock)
  const RdoWinner *win;     // commit: per superblock
  const float *imp;         // block_importances (w_imp per row), may be null
  int w_in_b, h_in_b, w_imp;
  int n_tx;            // transform blocks per plane in this launch (the grid's size)
  int cand_base;       // score without a list: candidate = cand_base + task / ntx_per_cand
  const int32_t *list;  // score: the valid candidates (c * nsb + sb), compacted on
  const int32_t *count; //   the device; the launch covers count * ntx_per_cand blocks
  int commit;          // 0: score every candidate, 1: commit the winners
  int ntx_per_cand;    // transform blocks per candidate
  int bd;
  int bsize;           // luma block size of this launch's superblock grid (64 .. 8)
  int mb_w, mb_h;      // prediction block (filter choice)
  int sub_w, sub_h;    // SSE distortion sub-block (chroma)
  int xdec, ydec;      // this plane type's subsampling
  int q_tx_index;      // tx_size * 16 + tx_type: av1_scan_orders entry
  int tx_size, qindex; // estimate_rate
  // intra chains (MODE 3, rv_rdo_intra): per superblock the get_intra_edges
  // of Y, U, V (3 x kIntraEdge pixels), the modes to try [n, m0, m1, m2]
  // (score; luma task = slot * 3 + k, chroma task = slot * 6 + 2 k + (0:
  // chroma mode m_k, 1: DC_PRED)) and the winner's [luma, chroma] mode
  // (commit; task = list entry)
  const void *iedges;
  const uint8_t *imodes;
  const uint8_t *iwin;
};

}  // namespace rv

// QuantizationContext::update (src/quantize.rs:205-253) evaluated on the
// device (the lookups live there), for the replay's launch arguments.
int rv_quant_ctx(int qindex, int tx_area, int is_intra, int bit_depth, int dc_delta_q,
                 int ac_delta_q, rv::QCtx *out);

// Luma candidates (64x64 transform, cdef distortion) and the chroma
// transform blocks of planes U and V (32x32, SSE) in one launch.
int rv_rdo_candidates(const rv::RdoArgs &luma, const rv::RdoArgs &chroma, int hbd,
                      hipStream_t s, bool compound = false);
// The single-reference (l0, c0) and the compound (l1, c1) candidates in one
// launch.
int rv_rdo_candidates_pair(const rv::RdoArgs &l0, const rv::RdoArgs &c0, const rv::RdoArgs &l1,
                           const rv::RdoArgs &c1, int hbd, hipStream_t s);

// Blocks below 64x64 (speed 6): one launch over the tasks of a (luma or
// the two chroma planes) for transform size n_tx_size; mode 0 single,
// 1 compound (score), 2 commit.
// a level's luma blocks (nl) and both chroma planes' (nc) in one launch
int rv_rdo_blocks2(const rv::RdoArgs &l, const rv::RdoArgs &c, int nl, int nc, int hbd,
                   hipStream_t s, int mode);
int rv_rdo_blocks(const rv::RdoArgs &a, bool luma, int nplanes, int n_tx_size, int hbd,
                  hipStream_t s, int mode);

// The list-driven score launches on a pool of workgroups (rdo_quad_list_kernel):
// the sets' arguments in device memory (rv_rdo_args_put, up to four: [luma,
// chroma] of set A, then set B), nsets 1 (set A, MODE mode_a) or 2 (A single-
// reference, B compound); h: the same arguments on the host (grid bound);
// max_grid > 0 caps the pool (a round's expected work).
int rv_rdo_args_put(const rv::RdoArgs *h, int n, rv::RdoArgs *dev, hipStream_t s);
// kp_cnt / kp_t (the replay's kernel probe, may be null): the launch adds
// its single / compound luma candidates and single / compound chroma
// transform blocks into kp_cnt[0..3], and min / max's its workgroups'
// device-clock start / end into kp_t[0] / kp_t[1].
int rv_rdo_candidates_list(const rv::RdoArgs *h, const rv::RdoArgs *dev, int nsets, int mode_a,
                           int hbd, hipStream_t s, int max_grid = 0, uint32_t *kp_cnt = nullptr,
                           unsigned long long *kp_t = nullptr);

// Intra chains of the 64x64 superblocks listed in luma.list (count): luma
// TX_64X64 + chroma TX_32X32 (4:2:0), intra prediction from the edges in
// RdoArgs::iedges, the intra quantizers; score (3 luma modes, 6 chroma
// chains per plane) or commit (the winner's modes).
int rv_rdo_intra(const rv::RdoArgs &luma, const rv::RdoArgs &chroma, int hbd, hipStream_t s);
