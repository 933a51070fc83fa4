// rv_replay.hip -- hot-path replay driver: the per-frame call structure of a
// speed-10 encode of a stream, for the stages this library accelerates, with
// every frame resident in HBM.  Per coded frame:
//
//   F0  hres / qres of the input (encode_frame, src/encoder.rs:3382-3385)
//   F1  coarse ME: full_search at 1/4 res, 16x16 per 64x64 superblock and
//       reference (estimate_motion_ss4, src/me.rs:1023-1075)
//   F2  half-res diamond, 32x32 (me_ss2, src/me.rs:287-519)
//   F3  full-res full-pel diamond then sub-pel diamond, 64x64
//       (motion_estimation, src/me.rs:193-285)
//   F4  RDO: every inter candidate of rdo_mode_decision (src/rdo.rs:825-1006:
//       NEARESTMV / NEAR0MV / GLOBALMV / NEWMV per reference), skip and
//       non-skip (luma_chroma_mode_rdo, :649-700): put_8tap, diff + fht,
//       quantize + dequantize, estimate_rate, inverse + add,
//       compute_distortion (rv_rdo.hip); then compute_rd_cost and the
//       per-superblock argmin in rav1e's candidate order
//   F6  commit: the winner of every superblock re-runs its chain and writes
//       its levels and its reconstruction into the frame
//   F5  8x8 importance SATD against reference 0 (compute_block_importances,
//       src/api/internal.rs:823-1010) + lookahead intra cost (:680-765)
//   F7  the reconstruction becomes a reference: pad (single tile group), or
//       pack the group's region, all-gather it over RCCL, unpack every other
//       group's region and pad (tile-parallel multi-GPU, src/encoder.rs:
//       2772-2781, 3411-3429)
//
// Frames run in the coding order of rav1e's reorder pyramid (src/api/
// internal.rs:40-95; group_input_len 4): display 4g+4, 4g+2, 4g+1, 4g+3 at
// me_range_scale 4, 2, 1, 1 (src/encoder.rs:838), each referencing the
// reconstructions its pyramid level sees.  Display frame 0 is the key frame:
// intra coding is out of scope, its input is taken as its reconstruction.
// The CPU replay (oracle/orc_replay.c) runs the same schedule and must
// produce the same result words.
#include <string.h>

#include <chrono>
#include <condition_variable>
#include <algorithm>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "rv_chain.h"
#include "rv_device.h"
#include "rv_ec.h"
#include "rv_intra.h"
#include "rv_intra_pass.h"
#include "rv_mvref.h"
#include "rv_impwin.h"
#include "rv_lrf.h"
#include "rv_rdo.h"
#include <string>

#if __has_include(<rccl/rccl.h>)
#include <rccl/rccl.h>
#define RV_HAVE_RCCL 1
#else
#define RV_HAVE_RCCL 0
#endif

// rv_me.hip / rv_me_diamond.hip: every reference in one launch, per-job
// evaluation counts, winners chained into the next stage's jobs
int rv_full_search_multi(const rv_plane *org, const rv_plane *refs, int n_refs,
                         const rv_fs_job *d_jobs, int n_per_ref, int blk_w, int blk_h,
                         int step, int allow_hp, rv_fs_result *d_out, const rv::ChainNext *next,
                         const uint32_t *const *box, void *stream);
int rv_diamond_search_multi(const rv_plane *org, const rv_plane *refs, int n_refs,
                            const rv_ds_job *d_jobs, int n_per_ref, int blk_w, int blk_h,
                            int subpixel, int use_satd, int allow_hp, int bit_depth,
                            rv_fs_result *d_out, uint32_t *d_evals, const rv::ChainNext *next,
                            void *stream, const uint8_t *active = nullptr,
                            const int32_t *alist = nullptr, const int32_t *acount = nullptr,
                            int lper = 1, const uint8_t *dirty = nullptr, int list_grid = 0,
                            uint32_t *eval_acc = nullptr, unsigned long long *t01 = nullptr);
int rv_diamond_f2_f3(const rv_plane *org_h, const rv_plane *refs_h, const rv_ds_job *jobs_h,
                     rv_fs_result *out_h, const uint8_t *dirty_h, const rv_plane *org,
                     const rv_plane *refs, const rv_ds_job *jobs, rv_fs_result *out,
                     const uint8_t *dirty, const rv::ChainNext *next, int n_refs, int n_per_ref,
                     int bit_depth, const int32_t *alist, const int32_t *acount, int list_grid,
                     void *stream, const rv_ds_job *jobs_sub = nullptr,
                     rv_fs_result *out_sub = nullptr, uint32_t *eval_acc = nullptr,
                     unsigned long long *t01 = nullptr);
// rv_deblock.hip
int rv_deblock_plane_dev(const rv_plane *p, int pli, int width, int height, const uint8_t *d_lg,
                         const uint8_t *d_skip, int mi_stride, const uint8_t levels[4],
                         int bit_depth, hipStream_t s);
extern "C" int rv_deblock_fast_level(int ac_q, int bit_depth, int is_key);
int rv_deblock_sse_dev(const rv_plane rec[3], const rv_plane src[3], int width, int height,
                       const uint8_t *d_lg, const uint8_t *d_skip, int mi_stride,
                       int64_t *d_tally, uint8_t *d_levels, int bit_depth, hipStream_t s);
int rv_deblock_frame_dev(const rv_plane planes[3], int width, int height, const uint8_t *d_lg,
                         const uint8_t *d_skip, int mi_stride, const uint8_t *d_levels,
                         int bit_depth, hipStream_t s, const uint8_t *levels);
extern "C" int rv_q_lookup(int ac, int qindex, int bit_depth);
#define RV_R(expr)                  \
  do {                              \
    int e_ = (expr);                \
    if (e_ != RV_OK) return e_;     \
  } while (0)
#define RV_H(expr)                                            \
  do {                                                        \
    hipError_t e_ = (expr);                                   \
    if (e_ != hipSuccess) return rv_set_hip_error(e_, #expr); \
  } while (0)

// rv_frame.hip
int rv_frame_pad_dev(const rv_plane dst[3], const rv_plane *src, hipStream_t s);
// rv_cdef.hip
int rv_cdef_filter_frame_dev(const rv_plane src[3], const rv_plane dst[3], int width, int height,
                             const uint8_t *d_skip, int mi_stride, const uint8_t *d_dir,
                             const int32_t *d_var, const uint8_t *d_cdef_index,
                             const uint8_t *y_strengths, const uint8_t *uv_strengths, int damping,
                             int bit_depth, hipStream_t s);
int rv_plane_pyramid(const rv_plane *y, const rv_plane *h, const rv_plane *q, void *stream);
int rv_synth_frame(const rv_plane *y, const rv_plane *u, const rv_plane *v, int t, int bit_depth,
                   void *stream);

namespace rv {

constexpr int kSb = 64;
// DPB slots, keyed by display index % kSlots.  24 (round 6; 12 before): the
// reuse of a slot orders a level-0 frame after the level-2 frames that read
// the slot's previous occupant, and with 12 slots that closed a cycle of
// two groups (level 0 of g -> level 1 -> level 2 -> level 0 of g + 2) that
// bounded the three pipelined instances; with 24 it spans five groups.
constexpr int kSlots = 24;
// result words per superblock and reference: coarse (mv, cost), the four
// half-res quadrants, full-pel, sub-pel, the 16 lookahead 16x16 blocks
constexpr int kWordsPerRef = 2 + 8 + 2 + 2 + 32 + 8;
// Workgroups of the list-driven launches of the MV-stack rounds after the
// first (a fixed pool that loops over the device counts)
constexpr int kRoundGrid = 256;
constexpr int kMaxGroups = 8;

struct Geo {
  int W, H, xdec, ydec, bd, hbd;
  int w_in_b, h_in_b;       // MiCols / MiRows (src/encoder.rs:580-581)
  int tx0, ty0, tw, th;     // this instance's tile group, in superblocks
  int tws, ths;             // uniform tile size in superblocks (TilingInfo)
  int nsb, R, M, C;         // superblocks, references, modes per ref, candidates
  int cw, ch;               // chroma block of a superblock
  int w_imp, h_imp;         // importance grid (src/encoder.rs:624-625)
  int vis_w, vis_h;         // the group's visible size (pixels)
};

__host__ __device__ inline int div_trunc8(int v) { return v / 8; }

// get_mv_range (src/me.rs:64-80); bo in 4x4 units (frame).  Rust usize
// arithmetic wraps and is cast back to isize, i.e. signed here.
__host__ __device__ inline void mv_range(const Geo &g, int bx, int by, int bw, int bh, int r[4]) {
  const int border_w = 128 + bw * 8, border_h = 128 + bh * 8;
  r[0] = -bx * 32 - border_w;
  r[1] = (g.w_in_b - bx - bw / 4) * 32 + border_w;
  r[2] = -by * 32 - border_h;
  r[3] = (g.h_in_b - by - bh / 4) * 32 + border_h;
}
// The tile of superblock (sx, sy) of the group: its origin (superblocks)
// and visible size in 4x4 units (TileStateMut mi_width / mi_height,
// src/tiling/tile_state.rs:93).
__host__ __device__ inline void sb_tile(const Geo &g, int sx, int sy, int &t0x, int &t0y,
                                        int &mi_w, int &mi_h) {
  const int fx = g.tx0 + sx, fy = g.ty0 + sy;
  t0x = fx - fx % g.tws;
  t0y = fy - fy % g.ths;
  const int vw = g.W - t0x * kSb < g.tws * kSb ? g.W - t0x * kSb : g.tws * kSb;
  const int vh = g.H - t0y * kSb < g.ths * kSb ? g.H - t0y * kSb : g.ths * kSb;
  mi_w = vw >> 2;
  mi_h = vh >> 2;
}
// adjust_bo (src/me.rs:993-1004) on tile-relative 4x4 offsets
__host__ __device__ inline void adjust_bo(int mi_w, int mi_h, int &bx, int &by, int bw, int bh) {
  int x = bx < mi_w - bw / 4 ? bx : mi_w - bw / 4;
  int y = by < mi_h - bh / 4 ? by : mi_h - bh / 4;
  bx = x > 0 ? x : 0;
  by = y > 0 ? y : 0;
}
__host__ __device__ inline uint32_t pack_mv(rv_mv m) {
  return ((uint32_t)(uint16_t)m.row << 16) | (uint16_t)m.col;
}
// Block-level reduction helper: one atomic per workgroup (never one per
// wavefront: same-address atomics serialise, MI355X_MICROARCH.md).
__device__ inline void block_atomic_add(uint64_t s, unsigned long long *out) {
  __shared__ uint64_t red[4];
  s = group_sum<64>(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); i++) t += red[i];
    if (t) atomicAdd(out, (unsigned long long)t);
  }
}

// Verification checksum of the committed levels (results time, not per
// frame): sum of q * (position in block + 1), wrapping u64.
__global__ void coeff_checksum(const int32_t *packed, int64_t total, int per_block,
                               unsigned long long *out) {
  uint64_t s = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x)
    s += (uint64_t)(int64_t)packed[i] * (uint64_t)(i % per_block + 1);
  block_atomic_add(s, out);
}

// compute_rd_cost + the per-superblock argmin (rdo_mode_decision): the
// candidates in rav1e's order (reference-major: NEARESTMV, NEAR0MV,
// GLOBALMV, NEWMV), each skip first, then non-skip unless the skip variant
// became the best with zero distortion (luma_chroma_mode_rdo,
// src/rdo.rs:690-700); strict `<`.  ScaledDistortion = luma + U + V
// (dist_scale 1.0); rate = the estimate_rate bits of every transform block
// (the rate model of RDOType::TxDistEstRate, src/encoder.rs:1226-1231; the
// entropy coder's mode and MV bits are out of scope); rd = dist as f64 +
// lambda * rate / 8 (src/rdo.rs:563-569).  One thread per superblock, which
// also writes the superblock's result words.
// One candidate's rd costs: skip (rs, distortion ds) and non-skip (rn, dn);
// live = rav1e pushes it and it repeats no earlier candidate's MVs.
struct CandCost {
  double rs, rn;
  uint64_t ds, dn;
  int live;
};
__device__ inline CandCost cand_cost(const CandGeo &cg, double lambda, double ds_u, double ds_v,
                                     const rv_fs_result *sub, const uint64_t *lout,
                                     const uint64_t *uout, const uint64_t *vout, int ntx_c, int sb,
                                     int c) {
  CandCost k{0.0, 0.0, 0, 0, 0};
  const int ns = cg.R * cg.M;  // single-reference candidates; compound ones follow
  rv_mv mv;
  if (c < ns ? !cand_live(cg, sub, sb, c, &mv) : !comp_live(cg, sub, sb, c - ns)) return k;
  k.live = 1;
  const int64_t o = (int64_t)c * cg.nsb + sb;
  uint64_t su = 0, sv = 0, nu = 0, nv = 0;
  uint32_t rate = (uint32_t)lout[o * 3 + 2];
  for (int j = 0; j < ntx_c; j++) {
    const int64_t t = (o * ntx_c + j) * 3;
    su += uout[t];
    sv += vout[t];
    nu += uout[t + 1];
    nv += vout[t + 1];
    rate += (uint32_t)uout[t + 2] + (uint32_t)vout[t + 2];
  }
  // Distortion * dist_scale[p] -> ScaledDistortion, summed over planes
  k.ds = (uint64_t)((double)lout[o * 3 + 0] * 1.0) + (uint64_t)((double)su * ds_u) +
         (uint64_t)((double)sv * ds_v);
  k.dn = (uint64_t)((double)lout[o * 3 + 1] * 1.0) + (uint64_t)((double)nu * ds_u) +
         (uint64_t)((double)nv * ds_v);
  k.rs = (double)k.ds + lambda * (0.0 / 8.0);
  k.rn = (double)k.dn + lambda * ((double)rate / 8.0);
  return k;
}
// The argmin step of candidate k after the ones before it (strict <; skip
// first, non-skip unless the skip variant became the best at zero distortion)
__device__ inline void argmin_step(RdoWinner &w, const CandCost &k, int c) {
  if (!k.live) return;
  bool zero_dist = false;
  if (k.rs < w.cost) {
    w = RdoWinner{c, 1, k.rs, k.ds};
    zero_dist = k.ds == 0;
  }
  if (!zero_dist && k.rn < w.cost) w = RdoWinner{c, 0, k.rn, k.dn};
}

// compute_rd_cost + the per-superblock argmin (rdo_mode_decision): the
// candidates in rav1e's order (reference-major: NEARESTMV, NEAR0MV,
// GLOBALMV, NEWMV, then the compound modes), each skip first, then non-skip
// unless the skip variant became the best with zero distortion
// (luma_chroma_mode_rdo, src/rdo.rs:690-700); strict `<`.  ScaledDistortion
// = luma + U + V (dist_scale 1.0); rate = the estimate_rate bits of every
// transform block (the rate model of RDOType::TxDistEstRate,
// src/encoder.rs:1226-1231; the entropy coder's mode and MV bits are out of
// scope); rd = dist as f64 + lambda * rate / 8 (src/rdo.rs:563-569).
__device__ inline RdoWinner block_argmin(const CandGeo &cg, double lambda, double ds_u,
                                         double ds_v, const rv_fs_result *sub,
                                         const uint64_t *lout, const uint64_t *uout,
                                         const uint64_t *vout, int ntx_c, int sb) {
  RdoWinner w{0, 0, 1.7976931348623157e308, 0};  // f64::MAX
  for (int c = 0; c < cg.R * cg.M + cg.comp; c++)
    argmin_step(w, cand_cost(cg, lambda, ds_u, ds_v, sub, lout, uout, vout, ntx_c, sb, c), c);
  return w;
}

// The scoring of the superblocks a round evaluated, one wavefront per
// superblock: lane c costs candidate c (the loads of every candidate in
// flight at once), lane 0 walks the argmin in rav1e's order over the
// wavefront's LDS copy, then the wavefront writes the superblock's winner,
// decision record and result words.  The superblocks: every one (alist
// null, round 0) or the list the round's check wrote (alist[0 .. *acount)).
// A fixed pool of workgroups loops over them.  Block 0 also resets the
// candidate lists' counts (consumed) and, on round 0, the frame's counters.
constexpr int kScoreMaxCands = 2 * kCandModes + kCompModes;
__global__ __launch_bounds__(256) void score_wave_kernel(
    Geo g, CandGeo cg, double lambda, double ds_u, double ds_v, const rv_fs_result *sub,
    const uint64_t *lout, const uint64_t *uout, const uint64_t *vout, int ntx_c, RdoWinner *win,
    const rv_fs_result *coarse, const rv_fs_result *half, const rv_fs_result *full,
    const rv_fs_result *look, const rv_fs_result *half_l, uint64_t *words, int32_t *cand_count,
    unsigned long long *imp_sum, uint32_t *evals, int32_t *leaf_count, const int32_t *alist,
    const int32_t *acount, BlkDec *dec, int round) {
  __shared__ CandCost kc[4][kScoreMaxCands];
  __shared__ RdoWinner ws[4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n = alist ? __builtin_amdgcn_readfirstlane(*acount) : g.nsb;
  const int nc = cg.R * cg.M + cg.comp;
  const int per = kWordsPerRef * g.R + 4;
  for (int i = blockIdx.x * 4 + wave; i < n; i += gridDim.x * 4) {
    const int sb = alist ? __builtin_amdgcn_readfirstlane(alist[i]) : i;
    if (lane < nc)
      kc[wave][lane] = cand_cost(cg, lambda, ds_u, ds_v, sub, lout, uout, vout, ntx_c, sb, lane);
    wave_sync();
    if (lane == 0) {
      RdoWinner w{0, 0, 1.7976931348623157e308, 0};  // f64::MAX
      for (int c = 0; c < nc; c++) argmin_step(w, kc[wave][c], c);
      ws[wave] = w;
      win[sb] = w;
      if (dec) dec[sb] = blk_dec_of(cg, sub, sb, w.c);
    }
    wave_sync();
    const RdoWinner w = ws[wave];
    uint64_t *base = words + (int64_t)sb * per;
    for (int wi = lane; wi < per; wi += 64) {
      uint64_t v;
      if (wi < kWordsPerRef * g.R) {
        const int r = wi / kWordsPerRef, k = wi - r * kWordsPerRef, e = k >> 1;
        const int64_t o = (int64_t)r * g.nsb + sb;
        // [coarse, 4 half-res quadrants, full-pel, sub-pel, 16 lookahead, the
        // lookahead's 4 half-res quadrants]
        const rv_fs_result &f = e == 0 ? coarse[o] : e < 5 ? half[o * 4 + e - 1] : e == 5 ? full[o]
                                : e == 6 ? sub[o] : e < 23 ? look[o * 16 + e - 7]
                                : half_l[o * 4 + e - 23];
        v = (k & 1) ? f.cost : pack_mv(f.best_mv);
      } else {
        const int j = wi - kWordsPerRef * g.R;
        if (j == 0) {
          v = (uint64_t)w.c;
        } else if (j == 1) {
          v = (uint64_t)w.skip;
        } else if (j == 2) {
          __builtin_memcpy(&v, &w.cost, 8);
        } else {
          v = w.dist;
        }
      }
      base[wi] = v;
    }
    wave_sync();  // kc / ws of this superblock are read before the next one's writes
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    // F4's lists are consumed: ready for the next round / frame.  Round 0:
    // the single-reference and compound candidates of the frame's first F4
    // launch (the one the roofline times; later rounds are counted by
    // rv_replay_counters' [15]); F5 sums next; the partition decision
    // appends next (the rounds the intra pass triggers may run after it)
    if (!round) {
      evals[0] = (uint32_t)cand_count[0];
      evals[1] = (uint32_t)cand_count[1];
      if (imp_sum) *imp_sum = 0;  // null: F5 ran on the side stream (it zeroed its sum)
      if (leaf_count)
        for (int l = 0; l < 4; l++) leaf_count[l] = 0;
    }
    cand_count[0] = cand_count[1] = 0;
  }
}

// The searches' predictor lists (get_subset_predictors, src/me.rs:82-96:
// zero, then the coarse MVs quantize_to_fullpel'd): slot p >= 1 of job i
// takes source src[8 i + p] (-1: none) = 2 * index + kind, kind 0 a coarse
// result (estimate_motion_ss4's MV * 4), 1 a half-res result
// (estimate_motion_ss2's MV * 2); `shr`: me_ss2 halves every predictor.
__global__ void fill_preds_kernel(rv_ds_job *jobs, const int32_t *src, int n,
                                  const rv_fs_result *coarse, const rv_fs_result *half, int shr) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  for (int p = 1; p < 8; p++) {  // src: 8 entries per job, [0] unused
    const int v = src[8 * i + p];
    if (v < 0) break;
    const rv_mv m = (v & 1) ? half[v >> 1].best_mv : coarse[v >> 1].best_mv;
    const int sc = (v & 1) ? 2 : 4;
    rv_mv q = qfull(rv_mv{(int16_t)(m.row * sc), (int16_t)(m.col * sc)});
    if (shr) q = rv_mv{(int16_t)(q.row >> 1), (int16_t)(q.col >> 1)};
    jobs[i].pred[p] = q;
  }
}

// ---- the lookahead's EPZS rounds ---------------------------------------------
// compute_lookahead_motion_vectors (src/api/internal.rs:514-622) searches a
// tile's superblocks in raster order, first every build_half_res_pmvs
// (F2L: four 32x32 quadrants at half resolution), then every
// build_full_res_pmvs (FL: sixteen 16x16 blocks), each from
// get_subset_predictors over the lookahead's own tile field, which starts
// at zero and takes the quadrants' and then the 16x16 blocks' MVs as they
// are found (save_block_motion); its references carry no field (no subset
// C).  A check recomputes every job's set from the current results and
// lists the jobs whose set changed; a round re-runs them.
struct LaArgs {
  Geo g;
  EpzsGeo eg;
  rv_ds_job *jh, *jl;            // F2L jobs [R][nsb][4], FL jobs [R][nsb][16]
  const int32_t *sl;             // FL's cmv sources (8 per job, fill_preds_kernel's code)
  const rv_fs_result *coarse, *half_l, *look;
  int32_t *list_h, *list_l;      // out: the marked F2L / FL jobs
  int init;                      // 1: store the sets, mark nothing
  int what;                      // bit 0: the F2L jobs, bit 1: the FL jobs
  int nref;                      // the lookahead's references (LaRefs::n)
  RoundPub pub;                  // pub.cnt: [F2L marked, FL marked]
};

__device__ inline rv_mv la_coarse4(const LaArgs &a, int k, int sb) {
  const rv_mv c = a.coarse[(size_t)k * a.g.nsb + sb].best_mv;
  return rv_mv{(int16_t)(c.row * 4), (int16_t)(c.col * 4)};
}

__global__ __launch_bounds__(256) void la_check_kernel(LaArgs a) {
  const Geo &g = a.g;
  const int nh = (a.what & 1) ? a.nref * g.nsb * 4 : 0, nl = (a.what & 2) ? a.nref * g.nsb * 16 : 0;
  const int i = blockIdx.x * 256 + threadIdx.x;
  bool mh = false, ml = false;
  int job = 0;
  if (i < nh) {  // F2L: me_ss2 of quadrant q (src/me.rs:465-519)
    job = i;
    const int k = i / (g.nsb * 4), sb = (i / 4) % g.nsb, q = i % 4;
    const int sx = sb % g.tw, sy = sb / g.tw;
    int t0x, t0y, mi_w, mi_h;
    sb_tile(g, sx, sy, t0x, t0y, mi_w, mi_h);
    const int fsx = g.tx0 + sx, fsy = g.ty0 + sy, tsx = fsx - t0x, tsy = fsy - t0y;
    const int tsw = (mi_w + 15) / 16, tsh = (mi_h + 15) / 16;
    const bool hh = (q & 1) ? tsx < tsw - 1 : tsx > 0, hv = (q >> 1) ? tsy < tsh - 1 : tsy > 0;
    const rv_mv ch = hh ? la_coarse4(a, k, (q & 1) ? sb + 1 : sb - 1) : rv_mv{0, 0};
    const rv_mv cv = hv ? la_coarse4(a, k, (q >> 1) ? sb + g.tw : sb - g.tw) : rv_mv{0, 0};
    const rv_mv cm[3] = {la_coarse4(a, k, sb), hh ? ch : cv, cv};  // static slots
    const int nc = 1 + (int)hh + (int)hv;
    int bx = tsx * 16 + (q & 1) * 8, by = tsy * 16 + (q >> 1) * 8;
    adjust_bo(mi_w, mi_h, bx, by, 32, 32);
    // the field: an earlier superblock's quadrant MV (estimate_motion_ss2's *
    // 2), zero inside this one (its quadrants are saved after all four)
    auto rd = [&](int X4, int Y4) {
      const int SX = X4 >> 4, SY = Y4 >> 4;
      if (SX == fsx && SY == fsy) return rv_mv{0, 0};
      const int gsb = (SY - g.ty0) * g.tw + (SX - g.tx0);
      const rv_mv h =
          a.half_l[((size_t)k * g.nsb + gsb) * 4 + ((Y4 >> 3) & 1) * 2 + ((X4 >> 3) & 1)].best_mv;
      return rv_mv{(int16_t)(h.row * 2), (int16_t)(h.col * 2)};
    };
    mh = epzs_update(a.jh + i, 1, a.eg, t0x * 16, t0y * 16, mi_w, bx, by, cm, nc, rd, nullptr, 1) &&
         !a.init;
  } else if (i - nh < nl) {  // FL: estimate_motion of 16x16 block b (src/me.rs:337-390)
    const int j = i - nh;
    job = j;
    const int k = j / (g.nsb * 16), sb = (j / 16) % g.nsb, b = j % 16;
    const int sx = sb % g.tw, sy = sb / g.tw;
    int t0x, t0y, mi_w, mi_h;
    sb_tile(g, sx, sy, t0x, t0y, mi_w, mi_h);
    const int tsx = g.tx0 + sx - t0x, tsy = g.ty0 + sy - t0y;
    rv_mv cm[6];
    int nc = 0;
    bool more = true;
#pragma unroll
    for (int p = 1; p < 7; p++) {  // the coarse MV, the covering quadrant, 4 neighbours' (a prefix)
      const int v = more ? a.sl[8 * j + p] : -1;
      more = more && v >= 0;
      const rv_mv m = !more ? rv_mv{0, 0}
                            : (v & 1) ? a.half_l[v >> 1].best_mv : a.coarse[v >> 1].best_mv;
      const int sc = (v & 1) ? 2 : 4;
      cm[p - 1] = rv_mv{(int16_t)(m.row * sc), (int16_t)(m.col * sc)};
      nc += more ? 1 : 0;
    }
    int bx = tsx * 16 + (b % 4) * 4, by = tsy * 16 + (b / 4) * 4;
    adjust_bo(mi_w, mi_h, bx, by, 16, 16);
    // the field: the 16x16 block holding the unit (every block read comes
    // before this one in raster order, so it holds its FL MV)
    auto rd = [&](int X4, int Y4) {
      const int gsb = ((Y4 >> 4) - g.ty0) * g.tw + ((X4 >> 4) - g.tx0);
      return a.look[((size_t)k * g.nsb + gsb) * 16 + ((Y4 & 15) >> 2) * 4 + ((X4 & 15) >> 2)]
          .best_mv;
    };
    ml = epzs_update(a.jl + j, 0, a.eg, t0x * 16, t0y * 16, mi_w, bx, by, cm, nc, rd, nullptr, 1) &&
         !a.init;
  }
  const int lane = threadIdx.x & 63;
  const uint64_t below = (1ull << lane) - 1;
  const uint64_t bh = __ballot(mh), bl = __ballot(ml);
  int b0 = 0, b1 = 0;
  if (lane == 0) {
    if (bh) b0 = atomicAdd(a.pub.cnt, (int)__popcll(bh));
    if (bl) b1 = atomicAdd(a.pub.cnt + 1, (int)__popcll(bl));
  }
  b0 = __shfl(b0, 0, 64);
  b1 = __shfl(b1, 0, 64);
  if (mh) a.list_h[b0 + __popcll(bh & below)] = job;
  if (ml) a.list_l[b1 + __popcll(bl & below)] = job;
  round_publish(a.pub);
}

// What a candidate slot's F4 outputs (l_out / c_out) were computed for: an
// F4 evaluation (rdo_quad: prediction, transform, quantisation, distortion,
// coefficient rate) is a function of the block, its reference(s) and
// MV(s) alone -- the stacks only enter the mode / MV rates, which the argmin
// adds (cand_cost) -- so a later round of the same frame whose candidate has
// the MV the slot was last evaluated with keeps the slot's outputs instead of
// re-running it.  tag: the frame (rv_replay::coded + 1; 0 = never).
struct CandKey {
  uint32_t tag, mv0, mv1;
};
struct CandKeys {
  CandKey *key;  // [nsingle + nsb * kCompModes]
  uint32_t tag;
  int reuse;     // 0: record only (round 0); 1: skip a slot whose key matches
};
__device__ inline uint32_t mv_bits(rv_mv m) {
  return (uint32_t)(uint16_t)m.row | ((uint32_t)(uint16_t)m.col << 16);
}
// v: the candidate is live; returns whether F4 must evaluate it
__device__ inline bool cand_key_step(const CandKeys &k, int slot, bool v, rv_mv m0, rv_mv m1) {
  if (!v || !k.key) return v;
  const CandKey n{k.tag, mv_bits(m0), mv_bits(m1)};
  const CandKey o = k.key[slot];
  if (k.reuse && o.tag == n.tag && o.mv0 == n.mv0 && o.mv1 == n.mv1) return false;
  k.key[slot] = n;
  return true;
}

// The valid candidates (cand_mv true) of every superblock, compacted for
// the F4 launch: rav1e evaluates only the modes it pushes (about half of
// the 4 per reference on smooth motion: NEWMV often repeats a neighbour's
// MV).  One thread per candidate c * nsb + sb; wave-aggregated appends
// (the order of the list does not matter: every output is indexed by the
// candidate).
__global__ __launch_bounds__(256) void cand_list_kernel(CandGeo cg, const rv_fs_result *sub,
                                                         int n, int32_t *list, int32_t *count,
                                                         const uint8_t *active = nullptr,
                                                         CandKeys keys = CandKeys{nullptr, 0, 0}) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  bool v = false;
  if (i < n) {
    rv_mv mv;
    const int c = i / cg.nsb, sb = i - c * cg.nsb;
    v = (!active || active[sb]) && cand_live(cg, sub, sb, c, &mv);
    v = cand_key_step(keys, i, v, mv, rv_mv{0, 0});
  }
  const uint64_t m = __ballot(v);
  const int lane = threadIdx.x & 63;
  int base = 0;
  if (lane == 0 && m) base = atomicAdd(count, (int)__popcll(m));
  base = __shfl(base, 0, 64);
  if (v) list[base + __popcll(m & ((1ull << lane) - 1))] = i;
}
// The compound candidates (all pushed on SELECT frames) without repeated
// MV pairs: entries are absolute candidate indices nsingle + m * nsb + sb.
__global__ __launch_bounds__(256) void comp_list_kernel(CandGeo cg, const rv_fs_result *sub,
                                                         int nsingle, int32_t *list, int32_t *count,
                                                         const uint8_t *active = nullptr,
                                                         CandKeys keys = CandKeys{nullptr, 0, 0}) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  bool v = false;
  if (i < cg.comp * cg.nsb) {
    const int mm = i / cg.nsb, sb = i - mm * cg.nsb;
    v = (!active || active[sb]) && comp_live(cg, sub, sb, mm);
    if (v && keys.key) {
      rv_mv a0, a1;
      comp_mvs(cg, sub, sb, mm, &a0, &a1);
      v = cand_key_step(keys, nsingle + i, v, a0, a1);
    }
  }
  const uint64_t m = __ballot(v);
  const int lane = threadIdx.x & 63;
  int base = 0;
  if (lane == 0 && m) base = atomicAdd(count, (int)__popcll(m));
  base = __shfl(base, 0, 64);
  if (v) list[base + __popcll(m & ((1ull << lane) - 1))] = nsingle + i;
}

// The rounds after the first: both candidate lists (single-reference, then
// compound from nsingle on) of the superblocks the round's check listed,
// over a fixed pool of workgroups; wave-aggregated appends as above.
__global__ __launch_bounds__(256) void round_lists_kernel(CandGeo cg, const rv_fs_result *sub,
                                                          int nsingle, int32_t *list,
                                                          int32_t *count, const int32_t *alist,
                                                          const int32_t *acount, CandKeys keys) {
  const int cnt = __builtin_amdgcn_readfirstlane(*acount);
  const int ns = cg.R * cg.M, total = cnt * (ns + cg.comp);
  const int lane = threadIdx.x & 63;
  for (int b0 = blockIdx.x * 256; b0 < total; b0 += gridDim.x * 256) {
    const int i = b0 + (int)threadIdx.x;
    bool v = false;
    int c = 0, sb = 0;
    if (i < total) {
      c = i / cnt;
      sb = alist[i - c * cnt];
      rv_mv mv, m1{0, 0};
      if (c < ns) {
        v = cand_live(cg, sub, sb, c, &mv);
      } else {
        v = comp_live(cg, sub, sb, c - ns);
        if (v) comp_mvs(cg, sub, sb, c - ns, &mv, &m1);
      }
      const int slot = c < ns ? c * cg.nsb + sb : nsingle + (c - ns) * cg.nsb + sb;
      v = cand_key_step(keys, slot, v, mv, m1);
    }
    const bool comp = c >= ns;  // uniform per wavefront only where the split falls between them
    const uint64_t ms = __ballot(v && !comp), mc = __ballot(v && comp);
    int bs = 0, bc = 0;
    if (lane == 0) {
      if (ms) bs = atomicAdd(count, (int)__popcll(ms));
      if (mc) bc = atomicAdd(count + 1, (int)__popcll(mc));
    }
    bs = __shfl(bs, 0, 64);
    bc = __shfl(bc, 0, 64);
    const uint64_t below = (1ull << lane) - 1;
    if (v && !comp) list[bs + __popcll(ms & below)] = c * cg.nsb + sb;
    if (v && comp) list[nsingle + bc + __popcll(mc & below)] = nsingle + (c - ns) * cg.nsb + sb;
  }
}

// F5: get_satd of every 8x8 luma block of the group inside the frame
// against reference 0's original frame at the full-pel part of its
// lookahead MV (the 16x16 block's, fi.lookahead_mvs[y * 2][x * 2];
// compute_block_importances, src/api/internal.rs:823-1010) plus its
// lookahead intra cost (get_satd against pred_dc_128,
// src/api/internal.rs:680-765), summed.  One lane per block; the source
// block is read once for both.
template <typename Px>
__global__ __launch_bounds__(256) void importance_kernel(Geo g, rv_plane org, rv_plane ref,
                                                          const rv_fs_result *look, int nbx,
                                                          int nby, unsigned long long *sum) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t v = 0;
  if (i < nbx * nby) {
    const int bx = i % nbx, by = i / nbx;
    const int sb = (by / 8) * g.tw + (bx / 8), q = ((by % 8) / 2) * 4 + (bx % 8) / 2;
    const rv_mv mv = look[sb * 16 + q].best_mv;  // reference 0
    const int x = g.tx0 * kSb + bx * 8, y = g.ty0 * kSb + by * 8;
    const Px *o = plane_ptr<Px>(org, x, y);
    const Px *r = plane_ptr<Px>(ref, x + ((int)mv.col >> 3), y + ((int)mv.row >> 3));
    const int32_t base = 128 << (g.bd - 8);
    int32_t d[64], e[64];
#pragma unroll
    for (int rr = 0; rr < 8; rr++)
#pragma unroll
      for (int cc = 0; cc < 8; cc++) {
        const int32_t ov = (int32_t)o[(int64_t)rr * org.stride + cc];
        d[rr * 8 + cc] = ov - (int32_t)r[(int64_t)rr * ref.stride + cc];
        e[rr * 8 + cc] = ov - base;
      }
    // (sum + (1 << ln >> 1)) >> ln, ln = 3
    v = ((satd_chunk<8>(d) + 4) >> 3) + ((satd_chunk<8>(e) + 4) >> 3);
  }
  block_atomic_add(v, sum);
}

// Sum of the visible pixels of a rectangle of a plane (results time).
template <typename Px>
__global__ void sum_rect(rv_plane p, int x0, int y0, int w, int h, unsigned long long *out) {
  uint64_t s = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)w * h;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int y = (int)(i / w), x = (int)(i - (int64_t)y * w);
    s += *plane_ptr<Px>(p, x0 + x, y0 + y);
  }
  block_atomic_add(s, out);
}

// F7 exchange: copy rectangles between planes and a packed buffer (row-major
// per rectangle, `off` bytes into it).  blockIdx.y = rectangle.
struct XRect {
  int64_t off;
  int plane, x0, y0, w, h;
};
struct XArgs {
  rv_plane pl[3];
  XRect rect[3 * kMaxGroups];  // pixel rectangles (or block-map ones, bytewise)
  int n;
  int to_plane;  // 1: buffer -> planes (unpack), 0: planes -> buffer (pack)
  uint8_t *buf;
};
template <typename Px>
__global__ __launch_bounds__(256) void xcopy_kernel(XArgs a) {
  const XRect &r = a.rect[blockIdx.y];
  const int64_t n = (int64_t)r.w * r.h;
  Px *b = reinterpret_cast<Px *>(a.buf + r.off);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int y = (int)(i / r.w), x = (int)(i - (int64_t)y * r.w);
    Px *p = plane_ptr_mut<Px>(a.pl[r.plane], r.x0 + x, r.y0 + y);
    if (a.to_plane)
      *p = b[i];
    else
      b[i] = *p;
  }
}

// ---- speed 6 (config D): the partition levels below 64x64 -----------------
constexpr int kLevels = 4;  // 64x64, 32x32, 16x16, 8x8

// The full-pel jobs of a level take their pmvs entry as the coarse
// predictor, quantize_to_fullpel'd (get_subset_predictors, src/me.rs:82-96):
// a 32x32 block the half-res search of its quadrant (build_half_res_pmvs),
// a 16x16 / 8x8 block the sub-pel winner of its 32x32 (rdo_mode_decision
// stores b_me into pmvs for 32x32 and 64x64 blocks, src/rdo.rs:866-876).
__global__ void seed_level_kernel(rv_ds_job *jobs, int n, int gw, int R,
                                  const rv_fs_result *parent, int pn, int pgw, int f, int ex0,
                                  int ey0, int tw) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n * R) return;
  const int k = i / n, b = i - k * n, bx = b % gw, by = b / gw;
  if (pgw == 0) {  // 32x32: the half-res search of its quadrant (pmvs[1..4], MV * 2)
    // the group superblock of the level grid's block (the grid starts at
    // group superblock (ex0, ey0))
    const int sb = (ey0 + (by >> 1)) * tw + ex0 + (bx >> 1), q = (by & 1) * 2 + (bx & 1);
    const rv_mv m = parent[((int64_t)k * pn + sb) * 4 + q].best_mv;
    jobs[i].pred[1] = qfull(rv_mv{(int16_t)(m.row * 2), (int16_t)(m.col * 2)});
    return;
  }
  jobs[i].pred[1] = qfull(parent[k * pn + (by / f) * pgw + bx / f].best_mv);
}

// rdo_mode_decision's winner of every block of a level + its result words
// (the level's full-pel / sub-pel searches, winner, skip, cost, distortion).
__global__ __launch_bounds__(64) void score_level(CandGeo cg, double lambda, double ds_u,
                                                  double ds_v, const rv_fs_result *full,
                                                  const rv_fs_result *sub, const uint64_t *lout,
                                                  const uint64_t *uout, const uint64_t *vout,
                                                  RdoWinner *win, uint64_t *words,
                                                  int32_t *cand_count, uint32_t *evals) {
  const int b = blockIdx.x * 64 + threadIdx.x;
  if (b == 0) {
    evals[0] = (uint32_t)cand_count[0];
    evals[1] = (uint32_t)cand_count[1];
    cand_count[0] = cand_count[1] = 0;
  }
  if (b >= cg.nsb) return;
  const RdoWinner w = block_argmin(cg, lambda, ds_u, ds_v, sub, lout, uout, vout, 1, b);
  win[b] = w;
  uint64_t *wd = words + (int64_t)b * (4 * cg.R + 4);
  for (int k = 0; k < cg.R; k++) {
    const rv_fs_result f = full[k * cg.nsb + b], s = sub[k * cg.nsb + b];
    wd[4 * k + 0] = pack_mv(f.best_mv);
    wd[4 * k + 1] = f.cost;
    wd[4 * k + 2] = pack_mv(s.best_mv);
    wd[4 * k + 3] = s.cost;
  }
  uint64_t cb;
  __builtin_memcpy(&cb, &w.cost, 8);
  wd[4 * cg.R + 0] = (uint64_t)w.c;
  wd[4 * cg.R + 1] = (uint64_t)w.skip;
  wd[4 * cg.R + 2] = cb;
  wd[4 * cg.R + 3] = w.dist;
}

struct PartArgs {
  const RdoWinner *win[kLevels];
  int gw[kLevels];          // level grid width (blocks)
  int x0[kLevels], y0[kLevels];  // level grid origin (frame pixels)
  int ex0, ey0, ew, eh;     // the group superblocks the level grids cover
  int forced;               // speed 10: must_split only (the minimum block is 64x64)
  int32_t *leaf[kLevels];   // the committed blocks of each level
  int32_t *leaf_count;      // [kLevels], zeroed by score_candidates
  uint64_t *words;          // one partition mask per superblock
};

// encode_partition_topdown (src/encoder.rs:2392-2470) over every superblock
// of the group: a block past the frame edge must split; a block that fits
// compares PARTITION_NONE (its mode decision's rd cost) with
// PARTITION_SPLIT (the sum of its four children's, rdo_partition_decision,
// src/rdo.rs:1500-1668; strict `<`; the partition symbol's rate is not
// modelled) and recurses into a split; 8x8 blocks are leaves.  One thread
// per superblock; the leaves go to per-level lists (wave-aggregated
// appends, order irrelevant: every output is indexed by block).
__global__ __launch_bounds__(64) void partition_kernel(Geo g, PartArgs p) {
  const int sb = blockIdx.x * 64 + threadIdx.x;
  const bool live = sb < g.nsb;
  const int gx0 = g.tx0 * kSb, gy0 = g.ty0 * kSb;  // the group (level 0 grid)
  const int X = gx0 + (live ? sb % g.tw : 0) * kSb, Y = gy0 + (live ? sb / g.tw : 0) * kSb;
  const int sx = live ? sb % g.tw - p.ex0 : -1, sy = live ? sb / g.tw - p.ey0 : -1;
  const bool in_rect = sx >= 0 && sy >= 0 && sx < p.ew && sy < p.eh;
  auto idx = [&](int l, int x, int y) {
    const int B = kSb >> l;
    return ((y - p.y0[l]) / B) * p.gw[l] + (x - p.x0[l]) / B;
  };
  auto cost = [&](int l, int x, int y) { return p.win[l][idx(l, x, y)].cost; };
  auto split = [&](int l, int x, int y) -> bool {
    const int B = kSb >> l;
    if (!in_rect) return false;  // no level grid here: the superblock is a leaf
    if (x + B > g.W || y + B > g.H) return true;  // must_split
    if (l == kLevels - 1 || p.forced) return false;
    const int h = B / 2;
    double s = 0.0;
    s += cost(l + 1, x, y);
    s += cost(l + 1, x + h, y);
    s += cost(l + 1, x, y + h);
    s += cost(l + 1, x + h, y + h);
    return 0.0 + s < cost(l, x, y);
  };
  uint32_t mask = 0;
  auto walk = [&](auto emit) {
    if (!live) return;
    if (!split(0, X, Y)) {
      emit(0, X, Y);
      return;
    }
    mask |= 1u;
    for (int q = 0; q < 4; q++) {
      const int x1 = X + (q & 1) * 32, y1 = Y + (q >> 1) * 32;
      if (x1 >= g.W || y1 >= g.H) continue;
      if (!split(1, x1, y1)) {
        emit(1, x1, y1);
        continue;
      }
      mask |= 2u << q;
      for (int r = 0; r < 4; r++) {
        const int x2 = x1 + (r & 1) * 16, y2 = y1 + (r >> 1) * 16;
        if (x2 >= g.W || y2 >= g.H) continue;
        if (!split(2, x2, y2)) {
          emit(2, x2, y2);
          continue;
        }
        mask |= 1u << (5 + ((y2 - Y) / 16) * 4 + (x2 - X) / 16);
        for (int t = 0; t < 4; t++) {
          const int x3 = x2 + (t & 1) * 8, y3 = y2 + (t >> 1) * 8;
          if (x3 < g.W && y3 < g.H) emit(3, x3, y3);
        }
      }
    }
  };
  int cnt[kLevels] = {0, 0, 0, 0};
  walk([&](int l, int, int) { cnt[l]++; });
  const int lane = threadIdx.x & 63;
  int base[kLevels];
  for (int l = 0; l < kLevels; l++) {
    int v = cnt[l];
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(v, o, 64);
      if (lane >= o) v += t;
    }
    const int total = __shfl(v, 63, 64);
    int b0 = 0;
    if (lane == 63 && total) b0 = atomicAdd(&p.leaf_count[l], total);
    b0 = __shfl(b0, 63, 64);
    base[l] = b0 + v - cnt[l];
  }
  walk([&](int l, int x, int y) { p.leaf[l][base[l]++] = idx(l, x, y); });
  if (live) p.words[sb] = mask;
}

// The deblocking filter's block map: every 4x4 of a committed block gets
// the block's log2 size (4x4 units) and skip flag.  One thread per 4x4 row
// of a block: block i = list ? list[i] : i of the level grid (gw wide,
// origin (x0, y0) in blocks), lg = 4 - level.
__global__ void block_map_kernel(const int32_t *list, const int32_t *count, int n, int gw, int x0,
                                 int y0, int level, const RdoWinner *win, uint8_t *lg,
                                 uint8_t *skip, int mi_stride, int mi_cols, int mi_rows) {
  const int n4 = 16 >> level;
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int nb = count ? *count : n;
  if (i >= nb * n4) return;
  const int j = i / n4, r = i - j * n4;
  const int b = list ? list[j] : j;
  const int mx = (x0 + b % gw) * n4, my = (y0 + b / gw) * n4 + r;
  if (my >= mi_rows) return;
  const uint8_t sk = (uint8_t)win[b].skip;
  for (int c = 0; c < n4 && mx + c < mi_cols; c++) {
    lg[(int64_t)my * mi_stride + mx + c] = (uint8_t)(4 - level);
    skip[(int64_t)my * mi_stride + mx + c] = sk;
  }
}

// Levels checksum over the committed blocks of a list: sum of q *
// (position in its transform block + 1), wrapping u64.
__global__ void coeff_checksum_list(const int32_t *packed, const int32_t *list,
                                    const int32_t *count, int per, int wmod,
                                    unsigned long long *out) {
  const int64_t total = (int64_t)*count * per;
  uint64_t s = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = i / per;
    const int e = (int)(i - j * per);
    s += (uint64_t)(int64_t)packed[(int64_t)list[j] * per + e] * (uint64_t)(e % wmod + 1);
  }
  block_atomic_add(s, out);
}

}  // namespace rv

using namespace rv;

struct RvSlot {  // one frame of the DPB: the reconstruction and its motion field
  rv_plane y, u, v;
  // the frame's motion field (frame_mvs: the encode's tile field when the
  // frame was coded; zero for the key frame), 8x8 cells [h_in_b/2][w_in_b/2][R]
  rv_mv *fmv = nullptr;
};
struct RvInput {
  rv_plane y, u, v;
  // input_hres / input_qres (FrameState, src/encoder.rs:362-377: downsample
  // + pad): the half / quarter resolution planes the searches of this frame
  // and of every frame referencing it read; F0 of the frame (or the
  // lookahead running ahead) writes them
  rv_plane hres, qres;
  uint32_t *qres_box = nullptr;  // rv_plane_box_sums of qres (the SEA coarse search)
};

// The host side of stage F8 (RV_REPLAY_ENTROPY): a thread that range-codes
// each frame's tile token streams once the device has written them into
// host-mapped memory (two ring slots), keeping the CDF chain per pyramid
// level (get_initial_cdfcontext / the biggest tile, src/encoder.rs:
// 2750-2761, 2824-2833).
struct EcHost {
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  struct Item {
    int slot, level, qctx;
  };
  std::deque<Item> q;
  bool stop = false;
  long queued = 0, done = 0;
  int ntiles = 1;
  uint32_t *tok_h[2] = {nullptr, nullptr}, *stat_h[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
  bool busy[2] = {false, false};
  std::vector<uint16_t> chain[3];
  uint64_t stat[5] = {0, 0, 0, 0, 0};
  int err = 0;

  void code(const Item &it) {
    const uint32_t *st = stat_h[it.slot];
    if (st[1]) {  // tokens past the buffer were dropped
      err = RV_EINVAL;
      return;
    }
    const int total = rv_ec_cdf_total();
    std::vector<uint16_t> init(total), cdf(total), best_cdf(total);
    if (chain[it.level].empty())
      rv_ec_default_cdf(it.qctx, init.data());
    else
      init = chain[it.level];
    uint64_t h = 1469598103934665603ull, bytes = 0;
    long best = -1;
    std::vector<uint8_t> out;
    for (int t = 0; t < ntiles; t++) {
      const uint32_t a = st[3 + t], b = st[3 + t + 1];
      cdf = init;
      out.resize(2 * (size_t)(b - a) + 64);
      const long nb = rv_ec_code_tokens(tok_h[it.slot] + a, b - a, cdf.data(), out.data(), out.size());
      if (nb < 0 || (size_t)nb > out.size()) {
        err = RV_EINVAL;
        return;
      }
      for (long i = 0; i < nb; i++) h = (h ^ out[i]) * 1099511628211ull;
      bytes += (uint64_t)nb;
      if (nb >= best) {  // Iterator::max_by_key keeps the last maximum
        best = nb;
        best_cdf = cdf;
      }
    }
    rv_ec_reset_counts(best_cdf.data());
    chain[it.level] = best_cdf;
    stat[0] = bytes;
    stat[1] = (uint64_t)ntiles;
    stat[2] = h;
    stat[3]++;
    stat[4] += bytes;
  }
  void run() {
    for (;;) {
      Item it;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return stop || !q.empty(); });
        if (q.empty()) return;
        it = q.front();
        q.pop_front();
      }
      (void)hipEventSynchronize(ev[it.slot]);
      code(it);
      std::lock_guard<std::mutex> lk(mu);
      busy[it.slot] = false;
      done++;
      cv.notify_all();
    }
  }
  void drain() {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return done == queued; });
  }
};

// The counts of one chain of round checks (the lookahead's EPZS rounds, the
// MV-stack rounds): check q counts into the device slot q % kCnt and
// publishes (q << 32 | count) into the host-mapped ring at q % kPub
// (round_publish), where the host reads it without a stream sync.  One
// ring per host thread that runs round loops.
struct RoundRing {
  static constexpr int kCnt = 64, kPub = 64;
  int32_t *cnt = nullptr;  // [kCnt][2], then the ticket
  uint32_t *ticket = nullptr;
  unsigned long long *h_pub = nullptr, *d_pub = nullptr;
  uint32_t seq = 0;
  int last_count = -1;  // the run's last count the host read (-1: none yet)
  int32_t *slot(uint32_t q) const { return cnt + 2 * (q % kCnt); }
  // check q's publication (publish = false: counted, not published)
  RoundPub pub(uint32_t q, bool publish = true) const {
    return RoundPub{slot(q), slot(q + 1), ticket, publish ? d_pub + q % kPub : nullptr, q};
  }
};

// A frame's lookahead references (la_refs_of below): the displays in k order
// and the propagation order
struct LaRefs {
  int n, disp[kImpMaxRefs], order[kImpMaxRefs];
};

// Where a frame's lookahead writes (compute_lookahead_motion_vectors):
// F1 [R][nsb], F2L [R][nsb][4], FL [R][nsb][16]
struct LaOut {
  rv_fs_result *coarse = nullptr, *half_l = nullptr, *look = nullptr;
};

// The lookahead engine of an importance window W (rdo_lookahead_frames,
// src/api/config.rs:158; rv_replay_set_imp_window).  rav1e computes every
// frame's lookahead as the frame arrives, far ahead of its encode
// (compute_lookahead_data, src/api/internal.rs:767-820), and before coding
// output frame n propagates block importances over the window [n, n + W]
// (compute_block_importances, :823-1081).  Here a host thread of its own
// runs, on its own stream and round ring, the lookahead of coded frame m
// (F0 pyramids, F1, F2L, FL with their EPZS rounds, then the importance
// data of rv_impwin.h) into ring entry m % RW, and as soon as frame n + W is
// in, the window propagation for frame n.  The encode of frame n waits for
// that (a host flag, then a stream event), takes its lookahead results and
// final importances from the entry, and marks the entry used when the frame
// is done; the engine reuses entry m % RW for frame m + RW only after that.
// RW = W + 1 + kLaSlack: the slack covers the frames a twin instance still
// has in flight behind the primary.
constexpr int kEngineWaitS = 60;  // la_engine_take's bound on one frame's wait

// An in-process exchange of the lookahead engines' frame parts between the
// tile groups of one process (rv_la_hub_create: the GPU tests and the
// bench's rank emulation; real ranks all-gather over RCCL).  Group k's
// engine packs coded frame m's part into its buffer m % kRing, records an
// event and posts m; once every group has posted m it waits on the others'
// events and unpacks their parts.  A buffer is rewritten kRing frames later,
// after every group's unpack of it (each group posts frame m + 1 only after
// issuing its unpack of m).
struct rv_la_hub {
  static constexpr int kRing = 4;
  int n = 0;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<long> posted;
  std::vector<uint8_t *> buf[kRing];
  std::vector<hipEvent_t> ev[kRing];
};

struct RvLaEngine {
  static constexpr int kLaSlack = 28;
  int W = 0, RW = 0, dev = 0;
  long limit = 0;  // coded frames in the stream (0: unbounded)
  hipStream_t las = nullptr;
  // the window passes' stream (split): frame m's searches on las overlap
  // window m - W's propagation (they share only the entries' lists, handed
  // over with ev_lists); null: everything on las (the default; RAV1E_HIP_LA_SPLIT=1)
  hipStream_t lap = nullptr;
  bool split = false;
  RoundRing rr;
  int32_t *la_list = nullptr;
  void *scratch = nullptr;
  size_t scratch_bytes = 0;
  struct Entry {
    LaOut o;
    ImpFrame f;
    long m = -1;       // the coded frame the entry holds
    long used_by = -1; // host: the frame whose encode recorded ev_used
    rv_replay_frame_info fi{};
    LaRefs lr{};
    hipEvent_t ev_imp = nullptr, ev_used = nullptr;
    hipEvent_t ev_data = nullptr, ev_xchg = nullptr;  // RCCL parts: data in / exchanged
    hipEvent_t ev_lists = nullptr;  // split: the frame's lists are built (las -> lap)
  };
  std::vector<Entry> ring;
  std::vector<long> pyr_display;  // per input: the display whose pyramid it holds
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  long requested = 0;  // the highest frame an encode has asked for (0: none yet)
  long inputs_ready = 0;  // the inputs of displays < this are in place (rv_replay_set_inputs_ready)
  long imp_ready = 0;  // the importances of frames <= imp_ready are recorded
  long imp_next = 1;
  bool stop = false;
  int err = 0;
  std::string msg;
  long la_round_sum = 0, la_reeval = 0, la_frames = 0;  // under mu
  // several tile groups (rv_replay_set_la_exchange): every group's part of
  // each frame's importance data reaches every group, over RCCL (comm, the
  // part buffers psend / precv, pbytes per group) or an in-process hub.
  // RCCL: the all-gathers run on the encode's stream with the reconstruction
  // all-gathers, one communicator and one stream per rank, so every rank
  // issues its collectives in the same order on one queue (la_encode_
  // exchange; two communicators on streams sharing hardware queues can
  // deadlock across ranks).  The engine posts a frame's data (data_ready,
  // ev_data) and waits for its exchange (xchg_done, ev_xchg).
  void *comm = nullptr;
  uint8_t *psend = nullptr, *precv = nullptr;
  size_t pbytes = 0;
  long data_ready = 0, xchg_done = 0, xchg_next = 1;
  rv_la_hub *hub = nullptr;
  int hub_k = -1;
  std::vector<hipEvent_t> hub_ev;  // this member's hub events (destroyed with the engine)
  Entry &at(long m) { return ring[(size_t)(m % RW)]; }
};

struct rv_replay {
  rv_replay_cfg cfg;
  Geo g;
  int RA = 1;  // the lookahead's references (LaRefs; R = 2: 3, LAST3 added)
  CandGeo cg;
  hipStream_t stream;
  // FL runs on a second stream, overlapping F3/F4 (it only needs F1/F2's
  // MVs; score_candidates and F5 join it).  RAV1E_HIP_REPLAY_SERIAL=1: one
  // stream (A/B).
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipEvent_t ev_ielig = nullptr;  // intra_begin's count is on the host
  bool overlap = false;
  bool own_stream;
  bool sea;  // successive-elimination coarse search (bit depth <= 10)
  // per pyramid level: the frame's quantizers (QuantizationContext of
  // TX_64X64 luma / TX_32X32 chroma, inter) and lambdas
  struct Level {
    bool set = false;
    int qidx;
    QCtx ql, qu, qv;
    QCtx qil, qiu, qiv;   // the same transforms, intra (is_intra rounding)
    QCtx qs[kLevels][3];  // speed 6: luma / U / V of the 32x32 .. 8x8 blocks
    double lambda, me_lambda, ds[3];
  } lv[3];
  // speed 6: the partition levels below 64x64 (index 0 = the superblocks,
  // whose arrays are the ones above)
  struct PLevel {
    int B, n, gw, gh, bc, bch, txl, txc;
    CandGeo cg;
    rv_ds_job *jobs_full[3] = {nullptr, nullptr, nullptr}, *jobs_sub[3] = {nullptr, nullptr, nullptr};
    rv_fs_result *full = nullptr, *sub = nullptr;
    uint64_t *l_out = nullptr, *c_out = nullptr;
    RdoWinner *win = nullptr;
    int32_t *cand_list = nullptr, *cand_count = nullptr;
    int32_t *l_lev = nullptr, *c_lev = nullptr;
    int32_t *leaf = nullptr;
    size_t woff = 0;  // result words offset
  } pl[kLevels];
  bool s6 = false;
  // the 32x32 .. 8x8 level grids: speed 6 over the group, speed 10 over the
  // bounding rectangle (group superblocks ex0, ey0 + ew x eh) of the
  // superblocks past the frame's right / bottom edge (must_split)
  bool lvl = false;
  int ex0 = 0, ey0 = 0, ew = 0, eh = 0;
  // per level: leaves exist (RDO, score, commit) / the motion search runs
  // (a 16x16 / 8x8 level seeds from the 32x32 searches)
  bool lv_used[kLevels] = {false, false, false, false};
  bool lv_me[kLevels] = {false, false, false, false};
  // speed 10: the edge levels run on their own stream beside the 64x64 stages
  hipStream_t edge[kLevels] = {nullptr, nullptr, nullptr, nullptr};  // [1..3]: one per level
  hipEvent_t ev_efork = nullptr, ev_l1me = nullptr, ev_epart = nullptr;
  hipEvent_t ev_ejoin[kLevels] = {nullptr, nullptr, nullptr, nullptr};
  hipEvent_t ev_ecommit[kLevels] = {nullptr, nullptr, nullptr, nullptr};
  bool deblock = false;           // RV_REPLAY_DEBLOCK
  uint8_t *mi_lg = nullptr, *mi_skip = nullptr;  // the deblocking block map
  int mi_stride = 0, mi_cols = 0, mi_rows = 0;
  uint8_t db_level[3] = {0, 0, 0};  // fast level per pyramid level
  // speed 6: sse_optimize's level search (rv_deblock_sse): tallies, levels
  int64_t *db_tally = nullptr;
  uint8_t *db_dlev = nullptr;
  bool cdef = false;                // RV_REPLAY_CDEF
  // RV_REPLAY_LRF: the units' distortions / solved xqd per (plane,
  // superblock), the units' filters, the restored frame before its padding
  bool lrf = false;
  uint64_t *lrf_err = nullptr;
  int8_t *lrf_xqd = nullptr, *lrf_units = nullptr;
  // the decision's side stream (RAV1E_LRF_SIDE=1; default: the replay stream)
  hipStream_t lrf_side = nullptr;
  hipEvent_t ev_lrf0 = nullptr, ev_lrf1 = nullptr;
  bool lrf_pending = false;
  int lrf_fix_passes = 1 << 30;  // the decision kernel (create: RAV1E_LRF_FIX[_PASSES])
  RvInput lrf_out;
  RvInput cdef_pre;                 // the deblocked, pre-CDEF frame (the padded copy's source)
  uint8_t *cdef_dir = nullptr, *cdef_idx = nullptr;  // per 8x8 block; per 64x64 (all 0)
  int32_t *cdef_var = nullptr;
  uint8_t cdef_str[3][2] = {};      // [level] = (y, uv) strengths at cdef_index 0
  int32_t *leaf_count = nullptr;  // [kLevels]
  // RV_REPLAY_ENTROPY: the coefficient-coding stage (F8)
  bool entropy = false;
  EcFrameBufs ecb{};
  EcHost *ech = nullptr;
  long ec_frames = 0;
  // F8 runs on its own stream after the frame's block map, beside F7 and the
  // next frame's F0..F4; the next commit (F6) waits for it
  hipStream_t ecs = nullptr;
  hipEvent_t ev_f8fork = nullptr, ev_f8done = nullptr;
  bool f8_pending = false;
  // intra-mode screening (rv_intra_pass.hip; speed 10, 4:2:0)
  bool intra = false;
  uint8_t *i_elig = nullptr, *i_was = nullptr, *i_win = nullptr, *i_modes = nullptr;
  int32_t *i_mark = nullptr, *i_list[2] = {nullptr, nullptr}, *i_commit = nullptr,
          *i_revert = nullptr;
  int32_t *i_cnt = nullptr;    // [list 0, list 1, commit, revert]
  int32_t *h_cnt = nullptr;    // pinned host copy of one count
  void *i_edges = nullptr;
  uint64_t *i_lout = nullptr, *i_cout = nullptr;
  uint32_t *i_stats = nullptr; // [kRing][3]: screened, intra winners, rounds
  // speed 10: rav1e's MV stacks (rv_mvref.hip) in coding-order rounds
  bool exact = false;
  MvStack *stk = nullptr;              // the stacks each superblock was evaluated with
  BlkDec *dec_lv[3] = {nullptr, nullptr, nullptr};  // decisions, per pyramid level
  uint8_t *mv_active = nullptr;        // re-evaluate this round
  // the round checks' counts (this instance's host thread)
  static constexpr int kRoundsAhead = 2;  // rounds queued beyond the last count read
  RoundRing rr;
  int32_t *mv_list = nullptr;          // [2][nsb]: check q lists into half q & 1
  uint32_t *mv_epoch = nullptr;        // [nsb]: the incremental checks' claims (MvrefArgs::epoch)
  bool edge_tr = false;                // a stack reads a frame-edge leaf (top-right)
  // RAV1E_HIP_MV_HP=1: the rounds after the first on a high-priority stream
  hipStream_t hp = nullptr;
  hipEvent_t ev_hp0 = nullptr, ev_hp1 = nullptr;
  // RAV1E_HIP_ROUND_FORK=1: a round's independent launches on a second
  // stream (F2 beside F3, the compound F4 beside the single-reference one).
  // Off: 2160p A/B 144-148 vs 164-165 fps (r04q) -- with the twin and the
  // lookahead engine the process already has more streams than hardware
  // queues, and the fork's events cost more than the overlap gains
  hipStream_t rs2 = nullptr;
  hipEvent_t ev_rfork = nullptr, ev_rlists = nullptr, ev_rjoin = nullptr;
  // evaluation rounds (round 0 included), re-evaluated superblocks and
  // round runs (1 + the MV / intra passes) per frame, summed
  long mv_round_sum = 0, mv_reeval = 0, mv_run_sum = 0;
  long mv_frames = 0;  // the frames this instance coded with the rounds (a twin codes some)
  size_t nwords = 0, wpart = 0;   // result words; offset of the partition masks
  bool jobs_built = false;
  std::mutex jobs_mu;  // ensure_jobs: the encode and the lookahead engine may both need them
  std::vector<RvSlot> slots;
  std::vector<RvInput> inputs;
  std::vector<void *> allocs;
  rv_fs_job *fs_jobs[3] = {nullptr, nullptr, nullptr};  // per level (scale 4, 2, 1)
  rv_fs_result *coarse, *half, *full, *sub;  // half: 4 quadrants per superblock
  rv_fs_result *look;                         // lookahead: 16 16x16 blocks per superblock
  rv_fs_result *half_l = nullptr;             // the lookahead's 4 quadrants per superblock
  rv_ds_job *jobs_half[3], *jobs_full[3], *jobs_sub[3], *jobs_look[3];  // per level
  rv_ds_job *jobs_half_l[3] = {nullptr, nullptr, nullptr};  // the lookahead's F2 (per level)
  int32_t *la_list = nullptr;  // the lookahead rounds' marked jobs: F2 [R nsb 4], then FL [R nsb 16]
  long la_round_sum = 0, la_reeval = 0;  // the lookahead rounds (round 0 included), re-evaluated jobs
  long la_frames = 0;                    // ... and their frames
  RvLaEngine *eng = nullptr;  // the importance window's lookahead engine (null: W = 0)
  bool eng_owned = false;     // the primary owns it; a twin borrows it
  const float *imp_last = nullptr;  // the importances the last coded frame used
  int32_t *src_half = nullptr, *src_full = nullptr, *src_look = nullptr;  // predictor sources
  uint64_t *l_out, *c_out;  // F4: [skip dist, non-skip dist, rate] per transform block
  RdoWinner *win;
  int32_t *cand_list, *cand_count;  // F4: the valid candidates
  RdoArgs *f4_args = nullptr;        // F4: the frame's list-launch arguments [la, ca, lc, cc]
  CandKey *cand_key = nullptr;       // F4: what each candidate slot was last evaluated with
  uint8_t *f3dirty = nullptr;        // rounds: the F3 jobs whose set / pmv changed [R][nsb]
  uint8_t *f2dirty = nullptr;        // rounds: the F2 jobs whose set changed [R][nsb][4]
  bool cand_reuse = true;            // a round keeps the F4 outputs of an unchanged candidate
  uint32_t *cand_evals;  // [kRing][2 * kLevels]: F4 candidates per frame and level (single, compound)
  int32_t *l_lev, *c_lev;   // F6: committed levels
  uint64_t *words;
  unsigned long long *tail;  // [levels csum, group recon sum, imp satd sum, -, frame recon sum]
  float *imp = nullptr;      // block_importances (null: all zero)
  int n_imp, imp_bx, imp_by, ntx_c;
  long coded = 0;            // frames coded so far (0 = the key frame next)
  rv_replay_frame_info last{};
  // tile-group exchange (F7)
  int n_groups = 1, my_group = 0;
  int32_t grects[4 * kMaxGroups];
  size_t xbytes = 0;         // packed bytes per group (the largest group)
  uint8_t *xsend = nullptr, *xrecv = nullptr;
  void *comm = nullptr;      // ncclComm_t (rv_comm)
  // Event ring: instrumented frame k records into set k % kRing, so per-
  // kernel times can be summed over a timed run without a host sync per
  // frame.  Every `timing_stride`-th block of frames is instrumented (each
  // record costs ~4.4 us of idle GPU between kernels on MI355X).
  static constexpr int kRing = 64;
  // e[0..13]: the stage boundaries on the main stream; e[14], e[15]: the
  // lookahead's start and end (on the side stream when it overlaps); e[16],
  // e[17]: the edge levels' span; e[18], e[19]: F8's (coefficient tokens)
  static constexpr int kEv = 20;
  static constexpr int kStageEv = 14;
  hipEvent_t evs[kRing][kEv];
  int timing_stride = 1, timing_block = 1;
  long timed = 0;
  // diamond candidate evaluations per job, per ring slot: [kRing][2][nsb*R]
  uint32_t *ds_evals;
  // Kernel probes (rv_replay_set_kernel_probe): on instrumented frames
  // every launch of a probed kernel -- probe 0: F3 sub-pel
  // (ds_fast_kernel<W = H = 64, sub-pel>), probe 1: the F4 candidate lists
  // (rdo_quad_list_kernel); round 0 and the MV-stack rounds -- is bracketed
  // by an event pair on its stream, and the launches add their units into
  // kp_cnt[p] (probe 0: candidate evaluations, jobs; probe 1: single /
  // compound luma candidates, single / compound chroma transform blocks).
  // Pair i of probe p uses kp_ev[p][2 (i % kKp)], harvested (elapsed time
  // summed) before reuse.
  static constexpr int kProbes = 2, kKpCnt = 4;
  bool kprobe = false;
  static constexpr int kKp = 512;
  std::vector<hipEvent_t> kp_ev[kProbes];
  long kp_n[kProbes] = {0, 0}, kp_done[kProbes] = {0, 0}, kp_base[kProbes] = {0, 0};
  // span slots [kp_n, kp_init) are initialised (start = max, end = 0): one
  // copy per kKpInit launches instead of one per launch (each a dependent
  // blit on the round's stream: the probe cost 2.5 % of the line, r06np)
  long kp_init[kProbes] = {0, 0};
  static constexpr int kKpInit = 256;
  double kp_ms[kProbes] = {0.0, 0.0}, kp_dev_ms[kProbes] = {0.0, 0.0};
  uint32_t *kp_cnt[kProbes] = {nullptr, nullptr};  // device [kKpCnt] each
  // ... and each launch's span on the device clock: [kKp][2] (first
  // workgroup's start, last one's end), harvested with the events
  unsigned long long *kp_ts[kProbes] = {nullptr, nullptr};
  double kp_tick_ms = 0.0;  // ms per wall_clock64 tick
};

namespace {

void *dalloc(rv_replay *r, size_t bytes) {
  void *p = nullptr;
  if (hipMalloc(&p, bytes ? bytes : 16) != hipSuccess) return nullptr;
  r->allocs.push_back(p);
  return p;
}

// kernel probe p's pairs [kp_done, upto): their elapsed times and device
// spans summed (the spans in at most two copies)
hipError_t kp_harvest(rv_replay *r, int p, long upto) {
  const long d0 = r->kp_done[p], n = upto - d0;
  if (n <= 0) return hipSuccess;
  constexpr long K = rv_replay::kKp;
  for (long k = d0; k < upto; k++) {
    const size_t i = 2 * (size_t)(k % K);
    hipError_t e = hipEventSynchronize(r->kp_ev[p][i + 1]);
    float ms = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, r->kp_ev[p][i], r->kp_ev[p][i + 1]);
    if (e != hipSuccess) return e;
    r->kp_ms[p] += ms;
  }
  std::vector<unsigned long long> t(2 * (size_t)n);
  const long s0 = d0 % K, first = std::min(n, K - s0);
  hipError_t e = hipMemcpy(t.data(), r->kp_ts[p] + 2 * s0, 2 * sizeof(unsigned long long) * first,
                           hipMemcpyDeviceToHost);
  if (e == hipSuccess && n > first)
    e = hipMemcpy(t.data() + 2 * first, r->kp_ts[p], 2 * sizeof(unsigned long long) * (n - first),
                  hipMemcpyDeviceToHost);
  if (e != hipSuccess) return e;
  for (long k = 0; k < n; k++)
    if (t[2 * k + 1] > t[2 * k]) r->kp_dev_ms[p] += (double)(t[2 * k + 1] - t[2 * k]) * r->kp_tick_ms;
  r->kp_done[p] = upto;
  return hipSuccess;
}

// Frame::new (src/frame/mod.rs:55-90): luma pad 64 + 24, chroma >> dec
size_t frame_planes(const Geo &g, rv_plane &y, rv_plane &u, rv_plane &v) {
  const int pad = 88;
  const int cw = (g.W + g.xdec) >> g.xdec, ch = (g.H + g.ydec) >> g.ydec;
  size_t b = rv_plane_geometry(&y, g.W, g.H, 0, 0, pad, pad, g.hbd);
  b += rv_plane_geometry(&u, cw, ch, g.xdec, g.ydec, pad >> g.xdec, pad >> g.ydec, g.hbd);
  rv_plane_geometry(&v, cw, ch, g.xdec, g.ydec, pad >> g.xdec, pad >> g.ydec, g.hbd);
  y.bit_depth = u.bit_depth = v.bit_depth = g.bd;
  return b;
}
size_t plane_bytes(const rv_plane &p) { return (size_t)p.stride * p.alloc_height * (p.hbd ? 2 : 1); }

bool alloc_input(rv_replay *r, RvInput &in, bool pyramid) {
  const Geo &g = r->g;
  frame_planes(g, in.y, in.u, in.v);
  const int pad = 88;
  rv_plane_geometry(&in.hres, g.W / 2, g.H / 2, 1, 1, pad / 2, pad / 2, g.hbd);
  rv_plane_geometry(&in.qres, g.W / 4, g.H / 4, 2, 2, pad / 4, pad / 4, g.hbd);
  in.hres.bit_depth = in.qres.bit_depth = g.bd;
  const size_t al = 256;
  auto up = [&](size_t v) { return (v + al - 1) / al * al; };
  const size_t by = plane_bytes(in.y), bu = plane_bytes(in.u);
  const size_t bh = pyramid ? plane_bytes(in.hres) : 0, bq = pyramid ? plane_bytes(in.qres) : 0;
  const size_t bs8 = pyramid ? (size_t)in.qres.stride * in.qres.alloc_height * 8 : 0;
  const size_t total = up(by) + 2 * up(bu) + up(bh) + up(bq) + up(bs8);
  uint8_t *m = (uint8_t *)dalloc(r, total);
  if (!m) return false;
  uint8_t *m0 = m;
  in.y.data = m;
  m += up(by);
  in.u.data = m;
  m += up(bu);
  in.v.data = m;
  m += up(bu);
  if (pyramid) {
    in.hres.data = m;
    m += up(bh);
    in.qres.data = m;
    m += up(bq);
    in.qres_box = (uint32_t *)m;
  }
  return hipMemsetAsync(m0, 0, total, r->stream) == hipSuccess;
}

bool alloc_slot(rv_replay *r, RvSlot &s) {
  const Geo &g = r->g;
  frame_planes(g, s.y, s.u, s.v);
  const size_t al = 256;
  auto up = [&](size_t v) { return (v + al - 1) / al * al; };
  const size_t by = plane_bytes(s.y), bu = plane_bytes(s.u);
  const size_t bf = (size_t)(g.w_in_b / 2) * (g.h_in_b / 2) * g.R * sizeof(rv_mv);
  const size_t total = up(by) + 2 * up(bu) + up(bf);
  uint8_t *m = (uint8_t *)dalloc(r, total);
  if (!m) return false;
  s.y.data = m;
  m += up(by);
  s.u.data = m;
  m += up(bu);
  s.v.data = m;
  m += up(bu);
  s.fmv = (rv_mv *)m;
  return hipMemsetAsync(s.y.data, 0, total, r->stream) == hipSuccess;
}

bool round_ring_alloc(rv_replay *r, RoundRing &q, hipStream_t st) {
  const size_t b = RoundRing::kCnt * 8 + 4;
  q.cnt = (int32_t *)dalloc(r, b);
  if (!q.cnt || hipMemsetAsync(q.cnt, 0, b, st) != hipSuccess) return false;
  q.ticket = (uint32_t *)(q.cnt + 2 * RoundRing::kCnt);
  if (hipHostMalloc((void **)&q.h_pub, RoundRing::kPub * 8,
                    hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
      hipHostGetDevicePointer((void **)&q.d_pub, q.h_pub, 0) != hipSuccess)
    return false;
  for (int i = 0; i < RoundRing::kPub; i++) q.h_pub[i] = ~0ull;
  return true;
}

int build_static_jobs(rv_replay *r) {
  const Geo &g = r->g;
  auto mx = [](int a, int b) { return a > b ? a : b; };
  auto mn = [](int a, int b) { return a < b ? a : b; };
  auto upload = [&](auto &vec, auto *&dst) -> int {
    if (!dst) dst = (std::remove_reference_t<decltype(dst)>)dalloc(r, vec.size() * sizeof(vec[0]));
    if (!dst) return RV_EHIP;
    return hipMemcpy(dst, vec.data(), vec.size() * sizeof(vec[0]), hipMemcpyHostToDevice) ==
                   hipSuccess
               ? RV_OK
               : RV_EHIP;
  };
  for (int lv = 0; lv < 3; lv++) {
    const double me_lambda = r->lv[lv].me_lambda;
    // F1 coarse jobs (estimate_motion_ss4) at this level's me_range_scale
    const int s = 4 >> lv;
    const uint32_t lambda4 = (uint32_t)(me_lambda * 256.0 / 16.0 * 0.125);
    // every job array holds the lookahead's references (RA >= R: the
    // encode's first, then LAST3, la_refs_of); the encode launches R
    std::vector<rv_fs_job> jobs(g.nsb * r->RA);
    for (int sb = 0; sb < g.nsb; sb++) {
      const int sx = sb % g.tw, sy = sb / g.tw;
      int t0x, t0y, mi_w, mi_h;
      sb_tile(g, sx, sy, t0x, t0y, mi_w, mi_h);
      int bx = (g.tx0 + sx - t0x) * 16, by = (g.ty0 + sy - t0y) * 16;
      adjust_bo(mi_w, mi_h, bx, by, 64, 64);
      const int fbx = bx + t0x * 16, fby = by + t0y * 16;
      const int range_x = 192 * s, range_y = 64 * s;
      int mr[4];
      mv_range(g, fbx, fby, 64, 64, mr);
      rv_fs_job j;
      memset(&j, 0, sizeof(j));
      j.po_x = fbx;  // (bo << 2) >> 2
      j.po_y = fby;
      j.x_lo = fbx + (mx(-range_x, div_trunc8(mr[0])) >> 2);
      j.x_hi = fbx + (mn(range_x, div_trunc8(mr[1])) >> 2);
      j.y_lo = fby + (mx(-range_y, div_trunc8(mr[2])) >> 2);
      j.y_hi = fby + (mn(range_y, div_trunc8(mr[3])) >> 2);
      j.lambda = lambda4;
      for (int k = 0; k < r->RA; k++) jobs[k * g.nsb + sb] = j;  // ref-major
    }
    int e;
    if ((e = upload(jobs, r->fs_jobs[lv]))) return e;
    // F2 / F3 / lookahead diamond jobs: static fields (positions, MV ranges,
    // lambdas, predictor counts); fill_preds_kernel writes the predictors
    // from the coarse / half-res results every frame
    const uint32_t lambda2 = (uint32_t)(me_lambda * 256.0 / 4.0 * 0.125);
    const uint32_t lambda1 = (uint32_t)(me_lambda * 256.0 * 0.5);
    const int nsb = g.nsb;
    std::vector<rv_ds_job> jh((size_t)nsb * r->RA * 4), jf(nsb * r->RA), js(nsb * r->RA),
        jl((size_t)nsb * r->RA * 16);
    std::vector<int32_t> sh(jh.size() * 8, -1), sf(jf.size() * 8, -1), sl(jl.size() * 8, -1);
    for (int k = 0; k < r->RA; k++)
      for (int sb = 0; sb < nsb; sb++) {
        const int i = k * nsb + sb;
        const int sx = sb % g.tw, sy = sb / g.tw;
        int t0x, t0y, mi_w, mi_h;
        sb_tile(g, sx, sy, t0x, t0y, mi_w, mi_h);
        // the superblock in its tile, and the tile's size in superblocks
        const int tsx = g.tx0 + sx - t0x, tsy = g.ty0 + sy - t0y;
        const int tsw = (mi_w + 15) / 16, tsh = (mi_h + 15) / 16;
        const bool hw = tsx > 0, he = tsx < tsw - 1, hn = tsy > 0, hs = tsy < tsh - 1;
        auto coarse_src = [&](int sb2) { return 2 * (k * nsb + sb2); };
        auto half_src = [&](int sb2, int q) { return 2 * ((k * nsb + sb2) * 4 + q) + 1; };
        // diamond job at tile-relative 4x4 offset (bx, by), size bw, adjust_bo'd
        auto make = [&](int bx, int by, int bw, bool adj, int shift, uint32_t lambda) {
          if (adj) adjust_bo(mi_w, mi_h, bx, by, bw, bw);
          const int fbx = bx + t0x * 16, fby = by + t0y * 16;
          int mr[4];
          mv_range(g, fbx, fby, bw, bw, mr);
          rv_ds_job j;
          memset(&j, 0, sizeof(j));
          j.po_x = (fbx * 4) >> shift;
          j.po_y = (fby * 4) >> shift;
          j.mvx_min = mr[0] >> shift;
          j.mvx_max = mr[1] >> shift;
          j.mvy_min = mr[2] >> shift;
          j.mvy_max = mr[3] >> shift;
          j.lambda = lambda;
          return j;
        };
        // F2: build_half_res_pmvs (src/encoder.rs:2864-3019): the four 32x32
        // quadrants at half resolution (estimate_motion_ss2 / me_ss2,
        // src/me.rs:280-327, 465-519) from [the superblock's coarse MV, the
        // horizontal, the vertical neighbour's] (inside the tile)
        for (int q = 0; q < 4; q++) {
          rv_ds_job j = make(tsx * 16 + (q & 1) * 8, tsy * 16 + (q >> 1) * 8, 32, true, 1, lambda2);
          int32_t *ps = &sh[((size_t)i * 4 + q) * 8];
          int n = 1;
          ps[n++] = coarse_src(sb);
          if ((q & 1) ? he : hw) ps[n++] = coarse_src((q & 1) ? sb + 1 : sb - 1);
          if ((q >> 1) ? hs : hn) ps[n++] = coarse_src((q >> 1) ? sb + g.tw : sb - g.tw);
          j.n_pred = n;
          jh[(size_t)i * 4 + q] = j;
        }
        // F3: motion_estimation of the 64x64 (src/me.rs:193-278) from zero and
        // pmvs[0], the coarse MV; sub-pel from the full-pel winner
        {
          rv_ds_job j = make(tsx * 16, tsy * 16, 64, false, 0, lambda1);
          sf[(size_t)i * 8 + 1] = coarse_src(sb);
          j.n_pred = 2;
          jf[i] = j;
          j.n_pred = 1;
          js[i] = j;
        }
        // lookahead: build_full_res_pmvs (src/encoder.rs:3021-3166), the 16
        // 16x16 blocks from [the coarse MV, the covering quadrant, two
        // vertical and two horizontal candidates of this and the adjacent
        // superblocks] (estimate_motion, src/me.rs:337-390, full-pel)
        for (int y = 0; y < 4; y++)
          for (int x = 0; x < 4; x++) {
            rv_ds_job j = make(tsx * 16 + x * 4, tsy * 16 + y * 4, 16, true, 0, lambda1);
            // pmvs_X[0] = coarse, [1..4] = quadrants of superblock X; -1 absent
            auto pm = [&](int dx, int dy, int e) -> int {
              const bool ok = dx < 0 ? hw : dx > 0 ? he : dy < 0 ? hn : dy > 0 ? hs : true;
              if (!ok) return -1;
              const int sb2 = sb + dx + dy * g.tw;
              return e == 0 ? coarse_src(sb2) : half_src(sb2, e - 1);
            };
            const int L = x <= 1, T = y <= 1;
            const int cover = pm(0, 0, T ? (L ? 1 : 2) : (L ? 3 : 4));
            int v1, v2, h1, h2;
            switch (y) {
              case 0: v1 = pm(0, -1, 0); v2 = pm(0, -1, L ? 3 : 4); break;
              case 1: v1 = pm(0, -1, L ? 3 : 4); v2 = pm(0, 0, L ? 3 : 4); break;
              case 2: v1 = pm(0, 1, L ? 1 : 2); v2 = pm(0, 0, L ? 1 : 2); break;
              default: v1 = pm(0, 1, 0); v2 = pm(0, 1, L ? 1 : 2); break;
            }
            switch (x) {
              case 0: h1 = pm(-1, 0, 0); h2 = pm(-1, 0, T ? 2 : 4); break;
              case 1: h1 = pm(-1, 0, T ? 2 : 4); h2 = pm(0, 0, T ? 2 : 4); break;
              case 2: h1 = pm(1, 0, T ? 1 : 3); h2 = pm(0, 0, T ? 1 : 3); break;
              default: h1 = pm(1, 0, 0); h2 = pm(1, 0, T ? 2 : 4); break;
            }
            const int cand[6] = {coarse_src(sb), cover, v1, v2, h1, h2};
            int32_t *ps = &sl[((size_t)i * 16 + y * 4 + x) * 8];
            int n = 1;
            for (int c = 0; c < 6; c++)
              if (cand[c] >= 0) ps[n++] = cand[c];
            j.n_pred = n;
            jl[(size_t)i * 16 + y * 4 + x] = j;
          }
      }
    if ((e = upload(jh, r->jobs_half[lv])) || (e = upload(jh, r->jobs_half_l[lv])) ||
        (e = upload(jf, r->jobs_full[lv])) || (e = upload(js, r->jobs_sub[lv])) ||
        (e = upload(jl, r->jobs_look[lv])))
      return e;
    if (lv == 0 && ((e = upload(sh, r->src_half)) || (e = upload(sf, r->src_full)) ||
                    (e = upload(sl, r->src_look))))
      return e;
    // speed 6: motion_estimation of every 32x32 / 16x16 / 8x8 block at its
    // own position (no adjust_bo, src/me.rs:193-278): zero + the seeded
    // coarse predictor, then the sub-pel search from the full-pel winner
    for (int l = 1; r->lvl && l < kLevels; l++) {
      rv_replay::PLevel &P = r->pl[l];
      std::vector<rv_ds_job> f6((size_t)P.n * g.R), s6((size_t)P.n * g.R);
      for (int k = 0; k < g.R; k++)
        for (int b = 0; b < P.n; b++) {
          const int X = (P.cg.tx0 + b % P.gw) * P.B, Y = (P.cg.ty0 + b / P.gw) * P.B;
          int mr[4];
          mv_range(g, X >> 2, Y >> 2, P.B, P.B, mr);
          rv_ds_job j;
          memset(&j, 0, sizeof(j));
          j.po_x = X;
          j.po_y = Y;
          j.mvx_min = mr[0];
          j.mvx_max = mr[1];
          j.mvy_min = mr[2];
          j.mvy_max = mr[3];
          j.lambda = lambda1;
          j.n_pred = 2;
          f6[(size_t)k * P.n + b] = j;
          j.n_pred = 1;
          s6[(size_t)k * P.n + b] = j;
        }
      if ((e = upload(f6, P.jobs_full[lv])) || (e = upload(s6, P.jobs_sub[lv]))) return e;
    }
  }
  r->jobs_built = true;
  return RV_OK;
}

// The static job records, built once: the first coded frame, or the
// lookahead engine when it starts before any frame (inputs declared ready).
int ensure_jobs(rv_replay *r) {
  std::lock_guard<std::mutex> lk(r->jobs_mu);
  if (r->jobs_built) return RV_OK;
  if (!r->lv[0].set || !r->lv[1].set || !r->lv[2].set)
    return rv_set_error(RV_EINVAL, "rv_replay: level params not set");
  return build_static_jobs(r);
}

// Packed rectangles of group k (its visible Y, U, V region; with
// deblocking also its rows of the block map, planes 3 = log2 size, 4 =
// skip), bytes into the group's slice of the exchange buffer.  Returns the
// bytes; *n = the rectangles.
int group_rects(const rv_replay *r, int k, XRect out[9], int *n) {
  const Geo &g = r->g;
  const int32_t *gr = r->grects + 4 * k;
  const int px = g.hbd ? 2 : 1;
  const int cw = (g.W + g.xdec) >> g.xdec, ch = (g.H + g.ydec) >> g.ydec;
  int64_t off = 0;
  for (int p = 0; p < 3; p++) {
    const int xd = p ? g.xdec : 0, yd = p ? g.ydec : 0;
    const int pw = p ? cw : g.W, ph = p ? ch : g.H;
    const int x0 = (gr[0] * kSb) >> xd, y0 = (gr[1] * kSb) >> yd;
    int x1 = ((gr[0] + gr[2]) * kSb) >> xd, y1 = ((gr[1] + gr[3]) * kSb) >> yd;
    x1 = x1 < pw ? x1 : pw;
    y1 = y1 < ph ? y1 : ph;
    out[p] = XRect{off, p, x0, y0, x1 - x0, y1 - y0};
    off += (int64_t)(x1 - x0) * (y1 - y0) * px;
  }
  *n = 3;
  if (r->deblock) {
    const int x0 = gr[0] * 16, y0 = gr[1] * 16;
    int x1 = (gr[0] + gr[2]) * 16, y1 = (gr[1] + gr[3]) * 16;
    x1 = x1 < r->mi_cols ? x1 : r->mi_cols;
    y1 = y1 < r->mi_rows ? y1 : r->mi_rows;
    for (int m = 0; m < 2; m++) {
      out[3 + m] = XRect{off, 3 + m, x0, y0, x1 - x0, y1 - y0};
      off += (int64_t)(x1 - x0) * (y1 - y0);
    }
    *n = 5;
  }
  if (r->exact) {  // the group's 8x8 cells of the frame's motion field (bytes)
    const int w8 = g.w_in_b / 2, h8 = g.h_in_b / 2, cb = g.R * (int)sizeof(rv_mv);
    const int x0 = gr[0] * 8, y0 = gr[1] * 8;
    int x1 = (gr[0] + gr[2]) * 8, y1 = (gr[1] + gr[3]) * 8;
    x1 = x1 < w8 ? x1 : w8;
    y1 = y1 < h8 ? y1 : h8;
    out[*n] = XRect{off, 5, x0 * cb, y0, (x1 - x0) * cb, y1 - y0};
    off += (int64_t)(x1 - x0) * cb * (y1 - y0);
    (*n)++;
  }
  if (r->lrf) {  // the group's loop-restoration units ((set, xqd0, xqd1) per superblock)
    const int sbc = (g.W + kSb - 1) / kSb, sbr = (g.H + kSb - 1) / kSb;
    const int x0 = gr[0], y0 = gr[1];
    int x1 = gr[0] + gr[2], y1 = gr[1] + gr[3];
    x1 = x1 < sbc ? x1 : sbc;
    y1 = y1 < sbr ? y1 : sbr;
    for (int p = 0; p < 3; p++) {
      out[*n] = XRect{off, 6 + p, 3 * x0, y0, 3 * (x1 - x0), y1 - y0};
      off += (int64_t)3 * (x1 - x0) * (y1 - y0);
      (*n)++;
    }
  }
  return (int)off;
}

template <typename Px>
static void xcopy_launch(hipStream_t st, const rv_plane *pl, const XRect *rects, int n,
                         int to_plane, uint8_t *buf) {
  if (n == 0) return;
  XArgs a;
  memset(&a, 0, sizeof(a));
  for (int p = 0; p < 3; p++) a.pl[p] = pl[p];
  int64_t most = 0;
  for (int i = 0; i < n; i++) {
    a.rect[i] = rects[i];
    const int64_t px = (int64_t)rects[i].w * rects[i].h;
    most = px > most ? px : most;
  }
  a.n = n;
  a.to_plane = to_plane;
  a.buf = buf;
  int64_t gx = (most + 255) / 256;
  gx = gx > 4096 ? 4096 : gx < 1 ? 1 : gx;
  xcopy_kernel<Px><<<dim3((unsigned)gx, (unsigned)n), 256, 0, st>>>(a);
}

// Copy rectangles between the slot's planes / the block map and a packed
// buffer (pixel rectangles at the pixel width, map rectangles bytewise).
int xcopy(rv_replay *r, const RvSlot &s, const XRect *rects, int n, int to_plane, uint8_t *buf) {
  XRect px[3 * kMaxGroups], mp[3 * kMaxGroups], un[3 * kMaxGroups];
  int npx = 0, nmp = 0, nun = 0;
  for (int i = 0; i < n; i++) {
    if (rects[i].plane < 3) {
      px[npx++] = rects[i];
    } else if (rects[i].plane < 6) {
      mp[nmp] = rects[i];
      mp[nmp++].plane -= 3;
    } else {
      un[nun] = rects[i];
      un[nun++].plane -= 6;
    }
  }
  const rv_plane pl[3] = {s.y, s.u, s.v};
  if (r->g.hbd)
    xcopy_launch<uint16_t>(r->stream, pl, px, npx, to_plane, buf);
  else
    xcopy_launch<uint8_t>(r->stream, pl, px, npx, to_plane, buf);
  if (nmp) {
    rv_plane m[3];
    memset(m, 0, sizeof(m));
    m[0].data = r->mi_lg;
    m[1].data = r->mi_skip;
    for (int i = 0; i < 2; i++) {
      m[i].stride = r->mi_stride;
      m[i].width = r->mi_cols;
      m[i].height = r->mi_rows;
    }
    // plane 5: the slot's motion field as bytes ([h8][w8][R] rv_mv)
    const int fb = r->g.w_in_b / 2 * r->g.R * (int)sizeof(rv_mv);
    m[2].data = s.fmv;
    m[2].stride = fb;
    m[2].width = fb;
    m[2].height = r->g.h_in_b / 2;
    xcopy_launch<uint8_t>(r->stream, m, mp, nmp, to_plane, buf);
  }
  if (nun) {  // planes 6-8: the loop-restoration units of Y, U, V ([sbr][sbc][3] bytes each)
    const int sbc = (r->g.W + kSb - 1) / kSb, sbr = (r->g.H + kSb - 1) / kSb;
    rv_plane u[3];
    memset(u, 0, sizeof(u));
    for (int p = 0; p < 3; p++) {
      u[p].data = r->lrf_units + (size_t)p * sbr * sbc * 3;
      u[p].stride = 3 * sbc;
      u[p].width = 3 * sbc;
      u[p].height = sbr;
    }
    xcopy_launch<uint8_t>(r->stream, u, un, nun, to_plane, buf);
  }
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

int pad_slot(rv_replay *r, const RvSlot &s) {
  const rv_plane pl3[3] = {s.y, s.u, s.v};
  return rv_frame_pad_dev(pl3, nullptr, r->stream);
}

// deblock_filter_optimize + deblock_filter_frame of a slot coded from input
// `in` (src/encoder.rs:2789-2793): speed 6 searches the levels on the
// device (sse_optimize) and the filter reads them there; speed 10 takes
// pyramid level lv's fast levels.  Nothing is filtered unless a luma level
// is non-zero.
int deblock_slot(rv_replay *r, const RvSlot &s, const RvInput &in, int lv) {
  const rv_plane pl3[3] = {s.y, s.u, s.v};
  if (r->s6) {
    const rv_plane src[3] = {in.y, in.u, in.v};
    const int e = rv_deblock_sse_dev(pl3, src, r->g.W, r->g.H, r->mi_lg, r->mi_skip,
                                     r->mi_stride, r->db_tally, r->db_dlev, r->g.bd, r->stream);
    if (e != RV_OK) return e;
    return rv_deblock_frame_dev(pl3, r->g.W, r->g.H, r->mi_lg, r->mi_skip, r->mi_stride,
                                r->db_dlev, r->g.bd, r->stream, nullptr);
  }
  const uint8_t l = r->db_level[lv];
  if (!l) return RV_OK;
  const uint8_t lv4[4] = {l, l, l, l};
  return rv_deblock_frame_dev(pl3, r->g.W, r->g.H, r->mi_lg, r->mi_skip, r->mi_stride, nullptr,
                              r->g.bd, r->stream, lv4);
}

// cdef_filter_frame of a deblocked slot (src/encoder.rs:2795-2802), then
// the slot's padding: the directions come from the slot's luma, every plane
// is filtered out of the slot into the scratch frame (one launch), and the
// scratch frame is copied back and padded in one pass (rv_frame_pad_dev) --
// three launches.  cdef_bits 0: every superblock uses entry 0 of the
// tables, the level's strengths.
int cdef_pad_slot(rv_replay *r, const RvSlot &s, int lv, const LrfGeo *lg) {
  const rv_plane rec[3] = {s.y, s.u, s.v};
  const rv_plane out[3] = {r->cdef_pre.y, r->cdef_pre.u, r->cdef_pre.v};
  uint8_t ys[8] = {}, us[8] = {};
  ys[0] = r->cdef_str[lv][0];
  us[0] = r->cdef_str[lv][1];
  RV_R(rv_cdef_find_dirs(&rec[0], r->g.W, r->g.H, r->mi_skip, r->mi_stride, r->cdef_dir,
                         r->cdef_var, r->g.bd, r->stream));
  // cdef_damping = 3 (src/encoder.rs:665)
  RV_R(rv_cdef_filter_frame_dev(rec, out, r->g.W, r->g.H, r->mi_skip, r->mi_stride, r->cdef_dir,
                                r->cdef_var, r->cdef_idx, ys, us, 3, r->g.bd, r->stream));
  if (!lg) return rv_frame_pad_dev(rec, out, r->stream);
  // lrf_filter_frame: the CDEF output restored, the deblocked slot for the
  // stripes' edges (pre_cdef_frame, src/encoder.rs:2795-2806)
  const rv_plane lo[3] = {r->lrf_out.y, r->lrf_out.u, r->lrf_out.v};
  if (r->lrf_pending) {  // the units of the side stream's decision
    RV_H(hipStreamWaitEvent(r->stream, r->ev_lrf1, 0));
    r->lrf_pending = false;
  }
  RV_R(lrf_filter_launch(out, rec, lo, *lg, r->lrf_units, 1, r->stream));
  return rv_frame_pad_dev(rec, lo, r->stream);
}

// rdo_loop_decision's restoration choices for the superblocks of group
// rect (in superblocks; null: the frame), from the reconstruction as the
// tile's coding leaves it (before the deblocking), into r->lrf_units.
static int lrf_decide_slot(rv_replay *r, const RvSlot &s, const RvInput &in, int lv, const LrfGeo &lg,
                           const int32_t *rect) {
  const Geo &g = r->g;
  const rv_plane rec[3] = {s.y, s.u, s.v}, src[3] = {in.y, in.u, in.v};
  // its CDEF's directions (cdef_pad_slot finds the deblocked frame's
  // afterwards, in the same buffers)
  if (r->cdef)
    RV_R(rv_cdef_find_dirs(&rec[0], g.W, g.H, r->mi_skip, r->mi_stride, r->cdef_dir, r->cdef_var, g.bd,
                           r->stream));
  RV_R(lrf_rdo_launch(rec, src, r->mi_skip, r->mi_stride, r->imp_last, g.w_imp, g.w_in_b, g.h_in_b, lg,
                      r->cdef, r->cdef_dir, r->cdef_var, r->cdef_str[lv], r->lv[lv].ds, r->lrf_err,
                      r->lrf_xqd, rect, r->stream));
  if (rect || !r->lrf_side)  // a group's units are packed right after: no overlap
    return lrf_decide_launch(lg, r->lrf_err, r->lrf_xqd, r->lv[lv].lambda, r->lrf_units, rect, r->lrf_fix_passes, r->stream);
  // the sequential decision (a few waves, latency only) on the side stream,
  // beside the deblocking and CDEF; lrf_filter_launch waits for it
  RV_H(hipEventRecord(r->ev_lrf0, r->stream));
  RV_H(hipStreamWaitEvent(r->lrf_side, r->ev_lrf0, 0));
  RV_R(lrf_decide_launch(lg, r->lrf_err, r->lrf_xqd, r->lv[lv].lambda, r->lrf_units, rect, r->lrf_fix_passes, r->lrf_side));
  RV_H(hipEventRecord(r->ev_lrf1, r->lrf_side));
  r->lrf_pending = true;
  return RV_OK;
}

// several tile groups (or a one-rank all-gather): each rank decides its own
// units before the exchange and imports the others'
static bool groups_active(const rv_replay *r) { return r->n_groups >= 2 || r->comm; }

// The loop filters of a coded slot and its padding: the frame is then a
// reference (src/encoder.rs:2789-2802, 3411-3429).
int filter_slot(rv_replay *r, const RvSlot &s, const RvInput &in, int lv) {
  LrfGeo lg;
  if (r->lrf) {
    const Geo &g = r->g;
    RV_R(lrf_geometry(g.W, g.H, g.xdec, g.ydec, g.bd, r->lv[lv].qidx, g.tws, g.ths, &lg));
    if (!groups_active(r)) RV_R(lrf_decide_slot(r, s, in, lv, lg, nullptr));
  }
  if (r->deblock) RV_R(deblock_slot(r, s, in, lv));
  return r->cdef ? cdef_pad_slot(r, s, lv, r->lrf ? &lg : nullptr) : pad_slot(r, s);
}

// Coding order of the reorder pyramid: coded frame n >= 1 (n = 0 is the
// key frame, display 0).
void frame_info(long n, int R, rv_replay_frame_info *f) {
  memset(f, 0, sizeof(*f));
  if (n == 0) {
    f->is_key = 1;
    return;
  }
  const long g = (n - 1) / 4, j = (n - 1) % 4;
  static const int kOff[4] = {4, 2, 1, 3}, kScale[4] = {4, 2, 1, 1};
  static const int kRef[4][2] = {{0, -4}, {0, 4}, {0, 2}, {2, 4}};
  f->display = (int)(4 * g + kOff[j]);
  f->me_range_scale = kScale[j];
  f->level = j == 0 ? 0 : j == 1 ? 1 : 2;
  for (int k = 0; k < R; k++) {
    long d = 4 * g + kRef[j][k];
    f->ref_display[k] = (int)(d < 0 ? 0 : d);
  }
  // reference_mode SELECT unless the frame is the first output of its group
  // (src/encoder.rs:832-836); compound needs a forward and a backward
  // reference (src/rdo.rs:914-941): display 4g+2 and 4g+3
  f->compound = R == 2 && (j == 1 || j == 3);
}

// The lookahead's references of coded frame m >= 1: rav1e's distinct DPB
// slots of fi.ref_frames (compute_block_importances' unique_indices,
// src/api/internal.rs:875-882); compute_lookahead_motion_vectors searches
// each slot once (build_coarse_pmvs / build_full_res_pmvs loop over
// ALL_INTER_REFS, src/encoder.rs:2732-2738, 3037-3040).  k < R are the
// encode's references (k = 0: LAST, the backward reference; k = 1: LAST2 at
// level 0, ALTREF -- the forward reference -- above); with R = 2 a frame
// above level 0 adds k = 2, LAST3: its own slot, which holds the previous
// frame of its level, or the key frame, which fills every slot
// (src/encoder.rs:658, 772-828).  order: the propagation's reference order
// (mv index order: LAST, LAST2 / LAST3, ALTREF).  oracle/orc_replay.c
// la_refs_of is the same table; tests/test_importance_window.py derives it
// from rav1e's slot logic.
LaRefs la_refs_of(long m, int R) {
  LaRefs l;
  memset(&l, 0, sizeof(l));
  rv_replay_frame_info f;
  frame_info(m, R, &f);
  for (int k = 0; k < R; k++) {
    l.disp[k] = f.ref_display[k];
    l.order[k] = k;
  }
  l.n = R;
  const long g = (m - 1) / 4, j = (m - 1) % 4;
  if (R == 2 && j > 0) {
    const long d3 = j == 1 ? 4 * g - 2 : j == 2 ? 4 * g - 1 : 4 * g + 1;
    l.disp[2] = (int)(d3 < 0 ? 0 : d3);
    l.n = 3;
    l.order[1] = 2;
    l.order[2] = 1;
  }
  return l;
}

}  // namespace

// F6b: rdo_mode_decision's intra-mode screening and intra RDO of every
// superblock whose inter winner is not skip (rv_intra_pass.hip), round by
// round until no decision changes.  la / ca: the F6 commit arguments.
// The eligible superblocks (they need only the inter winners): queued right
// after the argmin, so the host's read of their count completes while the
// commit (F6) runs instead of draining the stream.
static int intra_begin(rv_replay *r) {
  const Geo &g = r->g;
  hipStream_t st = r->stream;
  const IntraGeo ig{g.W, g.H, g.bd, g.nsb, g.tw, g.tx0, g.ty0, g.tws, g.ths};
  RV_H(hipMemsetAsync(r->i_cnt, 0, 4 * sizeof(int32_t), st));
  RV_R(rv_intra_elig(ig, r->win, r->i_elig, r->i_was, r->i_mark, r->i_list[0], r->i_cnt, st));
  RV_H(hipMemcpyAsync(r->h_cnt, r->i_cnt, 4, hipMemcpyDeviceToHost, st));
  RV_H(hipEventRecord(r->ev_ielig, st));
  return RV_OK;
}

static int intra_pass(rv_replay *r, const RdoArgs &la, const RdoArgs &ca, const RvInput &cur,
                      const RvSlot &S, const rv_replay::Level &L, int slot, int *nrounds) {
  const Geo &g = r->g;
  hipStream_t st = r->stream;
  const IntraGeo ig{g.W, g.H, g.bd, g.nsb, g.tw, g.tx0, g.ty0, g.tws, g.ths};
  uint32_t *stats = r->i_stats + (size_t)slot * 3;
  RV_H(hipEventSynchronize(r->ev_ielig));  // intra_begin's count
  int n = *r->h_cnt, round = 0;
  // the rounds are bounded by the longest dependency chain of a tile (its
  // anti-diagonals: right, below-left)
  const int max_rounds = g.tws + 2 * g.ths + 4;
  while (n > 0) {
    if (round >= max_rounds)
      return rv_set_error(RV_EHIP, "rv_replay_frame: the intra rounds did not converge");
    const int ci = round & 1;
    int32_t *list = r->i_list[ci], *cnt = r->i_cnt + ci;
    RV_H(hipMemsetAsync(r->i_cnt + (ci ^ 1), 0, sizeof(int32_t), st));
    RV_H(hipMemsetAsync(r->i_cnt + 2, 0, 2 * sizeof(int32_t), st));
    // screening: edges + the modes to try
    IntraScreenArgs sa;
    sa.g = ig;
    sa.rec[0] = S.y;
    sa.rec[1] = S.u;
    sa.rec[2] = S.v;
    sa.org = cur.y;
    sa.list = list;
    sa.count = cnt;
    sa.edges = r->i_edges;
    sa.modes = r->i_modes;
    RV_R(rv_intra_screen(sa, n, g.hbd, st));
    // the intra chains: 3 luma modes, 6 chroma chains per plane
    RdoArgs li = la, cl = ca;
    li.commit = cl.commit = 0;
    li.list = cl.list = list;
    li.count = cl.count = cnt;
    // grids sized by the round's count (the host read it): the lists hold
    // n superblocks, the commit / revert lists at most n
    li.ntx_per_cand = 3;
    li.n_tx = n * 3;
    cl.ntx_per_cand = 6;
    cl.n_tx = n * 6;
    li.iedges = cl.iedges = r->i_edges;
    li.imodes = cl.imodes = r->i_modes;
    li.iwin = cl.iwin = r->i_win;
    li.p[0].q = L.qil;
    li.p[0].out = r->i_lout;
    cl.p[0].q = L.qiu;
    cl.p[1].q = L.qiv;
    cl.p[0].out = r->i_cout;
    cl.p[1].out = r->i_cout + (size_t)g.nsb * 6 * 3;
    RV_R(rv_rdo_intra(li, cl, g.hbd, st));
    // the decisions, the commit / revert lists, the next round
    IntraDecideArgs da;
    da.g = ig;
    da.win = r->win;
    da.modes = r->i_modes;
    da.lout = r->i_lout;
    da.uout = r->i_cout;
    da.vout = r->i_cout + (size_t)g.nsb * 6 * 3;
    da.lambda = L.lambda;
    da.ds_u = L.ds[1];
    da.ds_v = L.ds[2];
    da.list = list;
    da.count = cnt;
    da.iwin = r->i_win;
    da.iwas = r->i_was;
    da.elig = r->i_elig;
    da.mark = r->i_mark;
    da.round = round;
    da.words = r->words;
    da.words_per_sb = kWordsPerRef * g.R + 4;
    da.win_off = kWordsPerRef * g.R;
    da.commit_list = r->i_commit;
    da.commit_count = r->i_cnt + 2;
    da.revert_list = r->i_revert;
    da.revert_count = r->i_cnt + 3;
    da.next_list = r->i_list[ci ^ 1];
    da.next_count = r->i_cnt + (ci ^ 1);
    RV_R(rv_intra_decide(da, st));
    // intra winners into the frame; superblocks back to inter: the F6 chain
    li.commit = cl.commit = 1;
    li.list = cl.list = r->i_commit;
    li.count = cl.count = r->i_cnt + 2;
    li.ntx_per_cand = cl.ntx_per_cand = 1;
    li.n_tx = cl.n_tx = n;
    li.p[0].out = cl.p[0].out = cl.p[1].out = nullptr;
    RV_R(rv_rdo_intra(li, cl, g.hbd, st));
    RdoArgs lr = la, cr = ca;
    lr.list = cr.list = r->i_revert;
    lr.count = cr.count = r->i_cnt + 3;
    lr.n_tx = n;
    cr.n_tx = n * cr.ntx_per_cand;
    RV_R(rv_rdo_candidates(lr, cr, g.hbd, st));
    RV_H(hipMemcpyAsync(r->h_cnt, r->i_cnt + (ci ^ 1), 4, hipMemcpyDeviceToHost, st));
    RV_H(hipStreamSynchronize(st));
    n = *r->h_cnt;
    round++;
  }
  RV_R(rv_intra_stats(g.nsb, r->i_elig, r->i_was, stats, st));
  RV_H(hipMemcpyAsync(stats + 2, &round, 4, hipMemcpyHostToDevice, st));
  if (nrounds) *nrounds = round;
  return RV_OK;
}

extern "C" {

static void la_engine_destroy(rv_replay *r);

void rv_replay_destroy(rv_replay *r) {
  if (!r) return;
  la_engine_destroy(r);  // its thread first: it launches on the replay's arrays
  // both streams drain before anything they may still read is freed (an
  // error return between the lookahead's fork and its join leaves the side
  // stream running)
  if (r->stream) (void)hipStreamSynchronize(r->stream);
  if (r->side) (void)hipStreamSynchronize(r->side);
  if (r->rs2) (void)hipStreamSynchronize(r->rs2);
  if (r->ecs) (void)hipStreamSynchronize(r->ecs);
  if (r->ech) {  // the host coder finishes the frames it holds, then stops
    {
      std::lock_guard<std::mutex> lk(r->ech->mu);
      r->ech->stop = true;
    }
    r->ech->cv.notify_all();
    if (r->ech->th.joinable()) r->ech->th.join();
    for (int k = 0; k < 2; k++) {
      if (r->ech->tok_h[k]) (void)hipHostFree(r->ech->tok_h[k]);
      if (r->ech->stat_h[k]) (void)hipHostFree(r->ech->stat_h[k]);
      if (r->ech->ev[k]) (void)hipEventDestroy(r->ech->ev[k]);
    }
    delete r->ech;
    r->ech = nullptr;
  }
  if (r->ev_f8fork) (void)hipEventDestroy(r->ev_f8fork);
  if (r->ev_f8done) (void)hipEventDestroy(r->ev_f8done);
  if (r->ecs) (void)hipStreamDestroy(r->ecs);
  for (hipStream_t es : r->edge)
    if (es) (void)hipStreamSynchronize(es);
  for (void *p : r->allocs) (void)hipFree(p);
  if (r->h_cnt) (void)hipHostFree(r->h_cnt);
  if (r->rr.h_pub) (void)hipHostFree(r->rr.h_pub);
  for (int f = 0; f < rv_replay::kRing; f++)
    for (int i = 0; i < rv_replay::kEv; i++)
      if (r->evs[f][i]) (void)hipEventDestroy(r->evs[f][i]);
  for (const auto &evs : r->kp_ev)
    for (hipEvent_t ev : evs)
    if (ev) (void)hipEventDestroy(ev);
  if (r->ev_fork) (void)hipEventDestroy(r->ev_fork);
  if (r->ev_join) (void)hipEventDestroy(r->ev_join);
  if (r->ev_ielig) (void)hipEventDestroy(r->ev_ielig);
  if (r->side) (void)hipStreamDestroy(r->side);
  if (r->rs2) (void)hipStreamDestroy(r->rs2);
  for (hipEvent_t ev : {r->ev_rfork, r->ev_rlists, r->ev_rjoin})
    if (ev) (void)hipEventDestroy(ev);
  if (r->hp) (void)hipStreamSynchronize(r->hp), (void)hipStreamDestroy(r->hp);
  if (r->lrf_side) (void)hipStreamSynchronize(r->lrf_side), (void)hipStreamDestroy(r->lrf_side);
  for (hipEvent_t ev : {r->ev_lrf0, r->ev_lrf1})
    if (ev) (void)hipEventDestroy(ev);
  if (r->ev_hp0) (void)hipEventDestroy(r->ev_hp0);
  if (r->ev_hp1) (void)hipEventDestroy(r->ev_hp1);
  for (hipEvent_t ev : {r->ev_efork, r->ev_l1me, r->ev_epart})
    if (ev) (void)hipEventDestroy(ev);
  for (int l = 0; l < kLevels; l++) {
    if (r->ev_ejoin[l]) (void)hipEventDestroy(r->ev_ejoin[l]);
    if (r->ev_ecommit[l]) (void)hipEventDestroy(r->ev_ecommit[l]);
    if (r->edge[l] && (l <= 1 || r->edge[l] != r->edge[1])) (void)hipStreamDestroy(r->edge[l]);
  }
  if (r->own_stream && r->stream) (void)hipStreamDestroy(r->stream);
  delete r;
}

// share: a primary instance whose DPB and inputs this one borrows
// (rv_replay_create_twin)
static rv_replay *create_impl(const rv_replay_cfg *cfg, void *stream, const rv_replay *share) {
  if (!cfg || cfg->width <= 0 || cfg->height <= 0 || (cfg->width & 7) || (cfg->height & 7) ||
      (cfg->bit_depth != 8 && cfg->bit_depth != 10 && cfg->bit_depth != 12) || cfg->xdec < 0 ||
      cfg->xdec > 1 || cfg->ydec < 0 || cfg->ydec > 1 || cfg->n_refs < 1 || cfg->n_refs > 2 ||
      cfg->n_inputs < 1 || cfg->tile_w_sb < 0 || cfg->tile_h_sb < 0) {
    rv_set_error(RV_EINVAL, "rv_replay_create: bad config");
    return nullptr;
  }
  rv_replay *r = new rv_replay();
  memset(r->evs, 0, sizeof(r->evs));
  r->cfg = *cfg;
  Geo &g = r->g;
  g.W = cfg->width;
  g.H = cfg->height;
  g.xdec = cfg->xdec;
  g.ydec = cfg->ydec;
  g.bd = cfg->bit_depth;
  g.hbd = cfg->bit_depth > 8;
  g.w_in_b = 2 * ((g.W + 7) >> 3);
  g.h_in_b = 2 * ((g.H + 7) >> 3);
  const int sbc = (g.W + kSb - 1) / kSb, sbr = (g.H + kSb - 1) / kSb;
  g.tx0 = cfg->tile_x0;
  g.ty0 = cfg->tile_y0;
  g.tw = cfg->tile_w > 0 ? cfg->tile_w : sbc - g.tx0;
  g.th = cfg->tile_h > 0 ? cfg->tile_h : sbr - g.ty0;
  g.tws = cfg->tile_w_sb > 0 ? cfg->tile_w_sb : sbc;
  g.ths = cfg->tile_h_sb > 0 ? cfg->tile_h_sb : sbr;
  // the group is a rectangle of whole tiles
  if (g.tx0 < 0 || g.ty0 < 0 || g.tw <= 0 || g.th <= 0 || g.tx0 + g.tw > sbc ||
      g.ty0 + g.th > sbr || g.tx0 % g.tws || g.ty0 % g.ths ||
      ((g.tx0 + g.tw) % g.tws && g.tx0 + g.tw != sbc) ||
      ((g.ty0 + g.th) % g.ths && g.ty0 + g.th != sbr)) {
    rv_set_error(RV_EINVAL, "rv_replay_create: the tile group is not a rectangle of whole tiles");
    delete r;
    return nullptr;
  }
  g.vis_w = (g.W - g.tx0 * kSb) < g.tw * kSb ? g.W - g.tx0 * kSb : g.tw * kSb;
  g.vis_h = (g.H - g.ty0 * kSb) < g.th * kSb ? g.H - g.ty0 * kSb : g.th * kSb;
  g.nsb = g.tw * g.th;
  g.R = cfg->n_refs;
  r->RA = g.R == 2 ? kImpMaxRefs : g.R;
  g.M = kCandModes;
  g.C = g.R * g.M + (g.R == 2 ? kCompModes : 0);  // the most a frame evaluates
  g.cw = kSb >> g.xdec;
  g.ch = kSb >> g.ydec;
  g.w_imp = g.w_in_b / 2;
  g.h_imp = g.h_in_b / 2;
  r->cg = CandGeo{g.nsb, g.tw, g.th, g.tx0, g.ty0, g.tws, g.ths, g.R, g.M, 0};
  // 8x8 sums of 10-bit pixels fit the u16 box-sum table; 12-bit searches
  // exhaustively
  r->sea = g.bd <= 10 && (cfg->flags & RV_REPLAY_EXHAUSTIVE_FS) == 0;
  if (stream) {
    r->stream = (hipStream_t)stream;
    r->own_stream = false;
  } else {
    r->own_stream = true;
    if (hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking) != hipSuccess) {
      rv_set_error(RV_EHIP, "rv_replay_create: stream");
      delete r;
      return nullptr;
    }
  }
  bool ok = true;
  if (share) {
    r->slots = share->slots;
    r->inputs = share->inputs;
  } else {
    r->slots.resize(kSlots);
    for (auto &s : r->slots) ok = ok && alloc_slot(r, s);
    r->inputs.resize(cfg->n_inputs);
    for (auto &in : r->inputs) ok = ok && alloc_input(r, in, true);
  }
  r->ntx_c = (g.cw / 32) * (g.ch / 32);
  const int nr = g.nsb * g.R;
  const int64_t nc = (int64_t)g.nsb * g.C;
  r->coarse = (rv_fs_result *)dalloc(r, nr * sizeof(rv_fs_result));
  r->half = (rv_fs_result *)dalloc(r, nr * 4 * sizeof(rv_fs_result));
  r->look = (rv_fs_result *)dalloc(r, nr * 16 * sizeof(rv_fs_result));
  r->half_l = (rv_fs_result *)dalloc(r, nr * 4 * sizeof(rv_fs_result));
  r->la_list = (int32_t *)dalloc(r, (size_t)nr * 20 * 4);
  if (r->half_l) (void)hipMemsetAsync(r->half_l, 0, nr * 4 * sizeof(rv_fs_result), r->stream);
  if (r->look) (void)hipMemsetAsync(r->look, 0, nr * 16 * sizeof(rv_fs_result), r->stream);
  r->full = (rv_fs_result *)dalloc(r, nr * sizeof(rv_fs_result));
  r->sub = (rv_fs_result *)dalloc(r, nr * sizeof(rv_fs_result));
  r->l_out = (uint64_t *)dalloc(r, (size_t)nc * 3 * 8);
  r->c_out = (uint64_t *)dalloc(r, (size_t)nc * r->ntx_c * 3 * 8 * 2);
  r->win = (RdoWinner *)dalloc(r, (size_t)g.nsb * sizeof(RdoWinner));
  r->cand_list = (int32_t *)dalloc(r, (size_t)nc * 4);
  {  // zeroed: tag 0 matches no frame
    const size_t kb = ((size_t)g.nsb * (g.R * g.M + kCompModes)) * sizeof(CandKey);
    r->cand_key = (CandKey *)dalloc(r, kb);
    ok = ok && r->cand_key && hipMemsetAsync(r->cand_key, 0, kb, r->stream) == hipSuccess;
    const char *e = getenv("RAV1E_HIP_F4_REUSE");  // =0: every round re-runs its F4 (A/B)
    r->cand_reuse = !(e && e[0] == '0');
    r->f3dirty = (uint8_t *)dalloc(r, (size_t)g.nsb * g.R);
    r->f2dirty = (uint8_t *)dalloc(r, (size_t)g.nsb * g.R * 4);
    ok = ok && r->f3dirty && r->f2dirty;
  }
  r->cand_count = (int32_t *)dalloc(r, 8);  // [single, compound]
  r->f4_args = (RdoArgs *)dalloc(r, 4 * sizeof(RdoArgs));
  r->cand_evals = (uint32_t *)dalloc(r, rv_replay::kRing * 2 * kLevels * 4);
  if (r->cand_evals)
    (void)hipMemsetAsync(r->cand_evals, 0, rv_replay::kRing * 2 * kLevels * 4, r->stream);
  if (r->cand_count) (void)hipMemsetAsync(r->cand_count, 0, 8, r->stream);
  r->l_lev = (int32_t *)dalloc(r, (size_t)g.nsb * 1024 * 4);
  r->c_lev = (int32_t *)dalloc(r, (size_t)g.nsb * r->ntx_c * 1024 * 4 * 2);
  r->nwords = (size_t)g.nsb * (kWordsPerRef * g.R + 4);
  if (cfg->flags & RV_REPLAY_SPEED6) {
    if (g.xdec != g.ydec) {
      rv_set_error(RV_EINVAL, "rv_replay_create: speed 6 needs 4:2:0 or 4:4:4");
      rv_replay_destroy(r);
      return nullptr;
    }
    r->s6 = true;
    r->lvl = true;
    r->ew = g.tw;
    r->eh = g.th;
  } else if (g.xdec == g.ydec) {
    // speed 10: encode_partition_topdown's must_split (src/encoder.rs:2407-
    // 2445) at the frame edges, over the bounding rectangle of the group's
    // superblocks past the right / bottom edge
    int x0 = g.tw, y0 = g.th, x1 = -1, y1 = -1;
    for (int sb = 0; sb < g.nsb; sb++) {
      const int x = sb % g.tw, y = sb / g.tw;
      if ((g.tx0 + x + 1) * kSb <= g.W && (g.ty0 + y + 1) * kSb <= g.H) continue;
      x0 = x < x0 ? x : x0;
      y0 = y < y0 ? y : y0;
      x1 = x > x1 ? x : x1;
      y1 = y > y1 ? y : y1;
    }
    if (x1 >= 0) {
      r->lvl = true;
      r->ex0 = x0;
      r->ey0 = y0;
      r->ew = x1 - x0 + 1;
      r->eh = y1 - y0 + 1;
    }
  }
  if (r->lvl) {
    // the levels holding leaves: every one at speed 6; at speed 10 those of
    // the must_split walk of the edge superblocks (largest blocks inside)
    for (int l = 1; l < kLevels; l++) r->lv_used[l] = r->s6;
    if (!r->s6) {
      for (int sb = 0; sb < g.nsb; sb++) {
        const int X = (g.tx0 + sb % g.tw) * kSb, Y = (g.ty0 + sb / g.tw) * kSb;
        if (X + kSb <= g.W && Y + kSb <= g.H) continue;
        for (int l = 1; l < kLevels; l++) {
          const int B = kSb >> l;
          for (int y = Y; y < Y + kSb; y += B)
            for (int x = X; x < X + kSb; x += B) {
              const int inside = x + B <= g.W && y + B <= g.H;
              const int pin = (x & ~(2 * B - 1)) + 2 * B <= g.W && (y & ~(2 * B - 1)) + 2 * B <= g.H;
              if (inside && !pin) r->lv_used[l] = true;  // a leaf: inside, its parent is not
            }
        }
      }
    }
    r->lv_me[1] = r->lv_used[1] || r->lv_used[2] || r->lv_used[3];
    r->lv_me[2] = r->lv_used[2];
    r->lv_me[3] = r->lv_used[3];
    rv_replay::PLevel &P0 = r->pl[0];
    P0.B = kSb;
    P0.n = g.nsb;
    P0.gw = g.tw;
    P0.gh = g.th;
    size_t nleaf = (size_t)g.nsb;
    for (int l = 1; l < kLevels; l++) {
      rv_replay::PLevel &P = r->pl[l];
      const int k = 1 << l;
      P.B = kSb >> l;
      P.gw = r->ew * k;
      P.gh = r->eh * k;
      P.n = P.gw * P.gh;
      P.bc = P.B >> g.xdec;
      P.bch = P.B >> g.ydec;
      P.txl = 4 - l;                                              // TX_32X32 .. TX_8X8
      P.txc = P.bc == 32 ? 3 : P.bc == 16 ? 2 : P.bc == 8 ? 1 : 0;  // .. TX_4X4
      P.cg = CandGeo{P.n, P.gw, P.gh, (g.tx0 + r->ex0) * k, (g.ty0 + r->ey0) * k, g.tws * k,
                     g.ths * k, g.R, g.M, 0};
      const int64_t nc = (int64_t)P.n * g.C;
      P.full = (rv_fs_result *)dalloc(r, (size_t)P.n * g.R * sizeof(rv_fs_result));
      P.sub = (rv_fs_result *)dalloc(r, (size_t)P.n * g.R * sizeof(rv_fs_result));
      P.l_out = (uint64_t *)dalloc(r, (size_t)nc * 3 * 8);
      P.c_out = (uint64_t *)dalloc(r, (size_t)nc * 3 * 8 * 2);
      P.win = (RdoWinner *)dalloc(r, (size_t)P.n * sizeof(RdoWinner));
      P.cand_list = (int32_t *)dalloc(r, (size_t)nc * 4);
      P.cand_count = (int32_t *)dalloc(r, 8);
      P.l_lev = (int32_t *)dalloc(r, (size_t)P.n * P.B * P.B * 4);
      P.c_lev = (int32_t *)dalloc(r, (size_t)P.n * P.bc * P.bch * 4 * 2);
      ok = ok && P.full && P.sub && P.l_out && P.c_out && P.win && P.cand_list && P.cand_count &&
           P.l_lev && P.c_lev;
      if (P.cand_count) (void)hipMemsetAsync(P.cand_count, 0, 8, r->stream);
      if (P.l_lev) (void)hipMemsetAsync(P.l_lev, 0, (size_t)P.n * P.B * P.B * 4, r->stream);
      if (P.c_lev) (void)hipMemsetAsync(P.c_lev, 0, (size_t)P.n * P.bc * P.bch * 8, r->stream);
      P.woff = r->nwords;
      r->nwords += (size_t)P.n * (4 * g.R + 4);
      nleaf += (size_t)P.n;
    }
    r->wpart = r->nwords;
    r->nwords += (size_t)g.nsb;
    int32_t *lf = (int32_t *)dalloc(r, nleaf * 4);
    r->leaf_count = (int32_t *)dalloc(r, kLevels * 4);
    ok = ok && lf && r->leaf_count;
    if (r->leaf_count) (void)hipMemsetAsync(r->leaf_count, 0, kLevels * 4, r->stream);
    for (int l = 0; l < kLevels && lf; l++) {
      r->pl[l].leaf = lf;
      lf += r->pl[l].n;
    }
  }
  r->words = (uint64_t *)dalloc(r, r->nwords * 8);
  // intra-mode screening: speed 10 4:2:0 unless RV_REPLAY_NO_INTRA
  r->intra = !r->s6 && !(cfg->flags & RV_REPLAY_NO_INTRA) && g.xdec == 1 && g.ydec == 1;
  r->i_stats = (uint32_t *)dalloc(r, (size_t)rv_replay::kRing * 3 * 4);
  ok = ok && r->i_stats && hipMemsetAsync(r->i_stats, 0, (size_t)rv_replay::kRing * 3 * 4,
                                          r->stream) == hipSuccess;
  if (r->intra) {
    const size_t n = (size_t)g.nsb;
    r->i_elig = (uint8_t *)dalloc(r, n);
    r->i_was = (uint8_t *)dalloc(r, n);
    r->i_win = (uint8_t *)dalloc(r, 2 * n);
    r->i_modes = (uint8_t *)dalloc(r, 4 * n);
    r->i_mark = (int32_t *)dalloc(r, 4 * n);
    r->i_list[0] = (int32_t *)dalloc(r, 4 * n);
    r->i_list[1] = (int32_t *)dalloc(r, 4 * n);
    r->i_commit = (int32_t *)dalloc(r, 4 * n);
    r->i_revert = (int32_t *)dalloc(r, 4 * n);
    r->i_cnt = (int32_t *)dalloc(r, 4 * sizeof(int32_t));
    r->i_edges = dalloc(r, n * 3 * kIntraEdge * (g.hbd ? 2 : 1));
    r->i_lout = (uint64_t *)dalloc(r, n * 3 * 3 * 8);
    r->i_cout = (uint64_t *)dalloc(r, n * 6 * 3 * 8 * 2);
    ok = ok && r->i_elig && r->i_was && r->i_win && r->i_modes && r->i_mark && r->i_list[0] &&
         r->i_list[1] && r->i_commit && r->i_revert && r->i_cnt && r->i_edges && r->i_lout &&
         r->i_cout && hipHostMalloc((void **)&r->h_cnt, 16, hipHostMallocDefault) == hipSuccess &&
         hipEventCreateWithFlags(&r->ev_ielig, hipEventDisableTiming) == hipSuccess;
    if (r->i_was) (void)hipMemsetAsync(r->i_was, 0, n, r->stream);
    if (r->i_win) (void)hipMemsetAsync(r->i_win, 0, 2 * n, r->stream);
  }
  // the rounds' counts (the lookahead's EPZS rounds at every speed, the MV-
  // stack rounds at speed 10): a device ring of count pairs + the ticket, the
  // host-mapped publication ring
  ok = ok && round_ring_alloc(r, r->rr, r->stream);
  // speed 10: rav1e's MV stacks in coding-order rounds
  r->exact = !r->s6 && !(cfg->flags & RV_REPLAY_MVREF_STANDIN);
  if (r->exact) {
    const size_t n = (size_t)g.nsb;
    r->stk = (MvStack *)dalloc(r, n * sizeof(MvStack));
    for (int l = 0; l < 3; l++) {
      r->dec_lv[l] = (BlkDec *)dalloc(r, n * sizeof(BlkDec));
      if (r->dec_lv[l]) (void)hipMemsetAsync(r->dec_lv[l], 0, n * sizeof(BlkDec), r->stream);
      ok = ok && r->dec_lv[l];
    }
    r->mv_active = (uint8_t *)dalloc(r, n);
    r->mv_list = (int32_t *)dalloc(r, 2 * n * 4);
    r->mv_epoch = (uint32_t *)dalloc(r, n * 4);
    ok = ok && r->stk && r->mv_active && r->mv_list && r->mv_epoch &&
         hipMemsetAsync(r->mv_epoch, 0, n * 4, r->stream) == hipSuccess;
    // RAV1E_HIP_MV_HP=1: the rounds after the first on a high-priority
    // stream (2160p A/B: 140 vs 177 fps -- the other instance's work loses
    // more than the rounds gain; off)
    const char *hpe = getenv("RAV1E_HIP_MV_HP");
    if (hpe && hpe[0] == '1') {
      int least = 0, greatest = 0;
      ok = ok && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess &&
           hipStreamCreateWithPriority(&r->hp, hipStreamNonBlocking, greatest) == hipSuccess &&
           hipEventCreateWithFlags(&r->ev_hp0, hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&r->ev_hp1, hipEventDisableTiming) == hipSuccess;
    }
    const char *rfe = getenv("RAV1E_HIP_ROUND_FORK");
    if (rfe && rfe[0] == '1')
      ok = ok && hipStreamCreateWithFlags(&r->rs2, hipStreamNonBlocking) == hipSuccess &&
           hipEventCreateWithFlags(&r->ev_rfork, hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&r->ev_rlists, hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&r->ev_rjoin, hipEventDisableTiming) == hipSuccess;
    // does a superblock's top-right neighbour (same tile) lie past the right
    // frame edge, i.e. is it a must_split leaf?
    for (int sb = 0; sb < g.nsb && r->lvl; sb++) {
      const int fsx = g.tx0 + sb % g.tw, fsy = g.ty0 + sb / g.tw;
      const int t0x = fsx - fsx % g.tws;
      const int cols = std::min(g.tws * 16, g.w_in_b - t0x * 16);
      if ((fsx + 1) * 64 <= g.W && (fsy + 1) * 64 <= g.H && fsy % g.ths != 0 &&
          (fsx - t0x) * 16 + 16 < cols && (fsx + 2) * 64 > g.W)
        r->edge_tr = true;
    }
  }
  if (cfg->flags & RV_REPLAY_CDEF) {
    if (!(cfg->flags & RV_REPLAY_DEBLOCK) || (g.W & 7) || (g.H & 7)) {
      rv_set_error(RV_EINVAL, "rv_replay_create: RV_REPLAY_CDEF needs RV_REPLAY_DEBLOCK and a "
                              "frame size that is a multiple of 8");
      rv_replay_destroy(r);
      return nullptr;
    }
    r->cdef = true;
    const size_t n8 = (size_t)(g.W / 8) * (g.H / 8), n64 = (size_t)((g.W + 63) / 64) * ((g.H + 63) / 64);
    r->cdef_dir = (uint8_t *)dalloc(r, n8);
    r->cdef_var = (int32_t *)dalloc(r, n8 * 4);
    r->cdef_idx = (uint8_t *)dalloc(r, n64);
    ok = ok && r->cdef_dir && r->cdef_var && r->cdef_idx && alloc_input(r, r->cdef_pre, false);
    if (r->cdef_idx) (void)hipMemsetAsync(r->cdef_idx, 0, n64, r->stream);
  }
  if (cfg->flags & RV_REPLAY_LRF) {
    LrfGeo lg;
    // (the unit size depends on the quantizer: rv_replay_set_level_params
    // checks every level's; 100 here is the replay's default level 0)
    if (!r->cdef || g.xdec != g.ydec ||
        lrf_geometry(g.W, g.H, g.xdec, g.ydec, g.bd, 100, g.tws, g.ths, &lg) != RV_OK) {
      rv_set_error(RV_EINVAL, "rv_replay_create: RV_REPLAY_LRF needs RV_REPLAY_CDEF, 4:2:0 or 4:4:4 "
                              "(rav1e's enable_restoration is off in 4:2:2) and units of one superblock");
      rv_replay_destroy(r);
      return nullptr;
    }
    r->lrf = true;
    r->lrf_err = (uint64_t *)dalloc(r, (size_t)3 * lg.nsb * 17 * 8);
    r->lrf_xqd = (int8_t *)dalloc(r, (size_t)3 * lg.nsb * 32);
    r->lrf_units = (int8_t *)dalloc(r, (size_t)3 * lg.nsb * 3);
    ok = ok && r->lrf_err && r->lrf_xqd && r->lrf_units && alloc_input(r, r->lrf_out, false);
    // RAV1E_LRF_SIDE=1: the decision on a side stream (2160p A/B, r05an:
    // 136-142 vs 152-154 fps without -- one more stream per instance than
    // the hardware queues serve well; off)
    // RAV1E_LRF_FIX=0 (A/B): the one-wave serial decision; RAV1E_LRF_FIX_PASSES
    // = 1 .. caps the fixed point's parallel passes (tests: the serial rest
    // after the cap).  Read here, once: the worker threads of a pipelined
    // replay must not call getenv per frame while the caller may setenv.
    {
      const char *fe = getenv("RAV1E_LRF_FIX"), *fp = getenv("RAV1E_LRF_FIX_PASSES");
      r->lrf_fix_passes = (fe && fe[0] == '0') ? 0 : fp ? std::max(atoi(fp), 1) : 1 << 30;
    }
    const char *se = getenv("RAV1E_LRF_SIDE");
    if (se && se[0] == '1')
      ok = ok && hipStreamCreateWithFlags(&r->lrf_side, hipStreamNonBlocking) == hipSuccess &&
           hipEventCreateWithFlags(&r->ev_lrf0, hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&r->ev_lrf1, hipEventDisableTiming) == hipSuccess;
  }
  r->entropy = (cfg->flags & RV_REPLAY_ENTROPY) != 0;
  if (r->entropy && g.xdec != g.ydec) {
    rv_set_error(RV_EINVAL, "rv_replay_create: RV_REPLAY_ENTROPY needs xdec == ydec");
    rv_replay_destroy(r);
    return nullptr;
  }
  if (cfg->flags & (RV_REPLAY_DEBLOCK | RV_REPLAY_ENTROPY)) {
    r->deblock = (cfg->flags & RV_REPLAY_DEBLOCK) != 0;
    r->mi_cols = (g.W + 3) / 4;
    r->mi_rows = (g.H + 3) / 4;
    r->mi_stride = (r->mi_cols + 15) / 16 * 16;
    const size_t mb = (size_t)r->mi_stride * (r->mi_rows + 16);
    r->mi_lg = (uint8_t *)dalloc(r, mb);
    r->mi_skip = (uint8_t *)dalloc(r, mb);
    ok = ok && r->mi_lg && r->mi_skip;
    if (r->mi_lg) (void)hipMemsetAsync(r->mi_lg, 4, mb, r->stream);
    if (r->mi_skip) (void)hipMemsetAsync(r->mi_skip, 0, mb, r->stream);
    if (r->s6 && r->deblock) {
      r->db_tally = (int64_t *)dalloc(r, 3 * 130 * 8);
      r->db_dlev = (uint8_t *)dalloc(r, 4);
      ok = ok && r->db_tally && r->db_dlev;
    }
  }
  if (r->entropy) {  // F8 buffers, the host-mapped token rings and the coder thread
    EcFrameBufs &b = r->ecb;
    b.ntiles = ((g.tw + g.tws - 1) / g.tws) * ((g.th + g.ths - 1) / g.ths);
    b.max_jobs = ec_max_jobs(g.nsb, b.ntiles);
    b.map_w4 = g.tws * 16;
    b.map_h4 = g.ths * 16;
    b.jobs = (rv_ec_job *)dalloc(r, (size_t)b.max_jobs * sizeof(rv_ec_job));
    b.sb_off = (uint32_t *)dalloc(r, ((size_t)g.nsb + 1) * 4);
    b.map = (uint8_t *)dalloc(r, (size_t)b.ntiles * 3 * b.map_w4 * b.map_h4);
    b.scratch = dalloc(r, rv_ec_scratch_bytes(b.max_jobs));
    b.offsets = (uint32_t *)dalloc(r, ((size_t)b.max_jobs + 1) * 4);
    b.dstat = (uint32_t *)dalloc(r, 16);
    // one token per coded coefficient plus 4 per job covers every block
    // whose levels stay below 3; more sets the overflow flag (an error)
    b.cap = (uint32_t)((size_t)g.nsb * (1024 + 2 * r->ntx_c * 1024) + (size_t)b.max_jobs * 4);
    ok = ok && b.jobs && b.sb_off && b.map && b.scratch && b.offsets && b.dstat;
    EcHost *eh = new EcHost();
    r->ech = eh;
    eh->ntiles = b.ntiles;
    for (int k = 0; k < 2 && ok; k++) {
      ok = hipHostMalloc((void **)&eh->tok_h[k], (size_t)b.cap * 4,
                         hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
           hipHostMalloc((void **)&eh->stat_h[k], ((size_t)b.ntiles + 8) * 4,
                         hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
           // blocking sync: the coder thread sleeps instead of spinning on the GPU
           hipEventCreateWithFlags(&eh->ev[k], hipEventBlockingSync | hipEventDisableTiming) ==
               hipSuccess;
    }
    if (getenv("RAV1E_HIP_F8_STREAM") && atoi(getenv("RAV1E_HIP_F8_STREAM")))
      ok = ok && hipStreamCreateWithFlags(&r->ecs, hipStreamNonBlocking) == hipSuccess &&
           hipEventCreateWithFlags(&r->ev_f8fork, hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&r->ev_f8done, hipEventDisableTiming) == hipSuccess;
    if (ok) eh->th = std::thread([eh] { eh->run(); });
  }
  r->imp_bx = g.vis_w / 8;
  r->imp_by = g.vis_h / 8;
  r->n_imp = r->imp_bx * r->imp_by;
  r->tail = (unsigned long long *)dalloc(r, 5 * 8);
  ok = ok && r->coarse && r->half && r->look && r->half_l && r->la_list && r->full && r->sub &&
       r->l_out && r->c_out && r->win &&
       r->cand_list && r->cand_count && r->f4_args && r->cand_evals &&
       r->l_lev && r->c_lev && r->words && r->tail;
  if (ok) {
    ok = hipMemsetAsync(r->words, 0, r->nwords * 8, r->stream) == hipSuccess &&
         hipMemsetAsync(r->tail, 0, 5 * 8, r->stream) == hipSuccess &&
         hipMemsetAsync(r->l_lev, 0, (size_t)g.nsb * 1024 * 4, r->stream) == hipSuccess &&
         hipMemsetAsync(r->c_lev, 0, (size_t)g.nsb * r->ntx_c * 1024 * 4 * 2, r->stream) ==
             hipSuccess;
  }
  for (int f = 0; f < rv_replay::kRing; f++)
    for (int i = 0; i < rv_replay::kEv; i++)
      ok = ok && hipEventCreateWithFlags(&r->evs[f][i], hipEventDisableSystemFence) == hipSuccess;
  {
    const char *e = getenv("RAV1E_HIP_REPLAY_SERIAL");
    r->overlap = !(e && e[0] == '1');
  }
  if (r->overlap && r->lvl && !r->s6) {
    ok = ok && hipEventCreateWithFlags(&r->ev_efork, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&r->ev_l1me, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&r->ev_epart, hipEventDisableTiming) == hipSuccess;
    // RAV1E_HIP_EDGE_STREAMS=3: one stream per level; default one stream for
    // all levels (in order) -- every stream beyond the hardware queues
    // (GPU_MAX_HW_QUEUES) is multiplexed onto them
    const char *es = getenv("RAV1E_HIP_EDGE_STREAMS");
    const bool per_level = es && es[0] == '3';
    for (int l = 1; l < kLevels; l++) {
      if (l == 1 || per_level)
        ok = ok && hipStreamCreateWithFlags(&r->edge[l], hipStreamNonBlocking) == hipSuccess;
      else
        r->edge[l] = r->edge[1];  // an alias (destroyed once)
      ok = ok && hipEventCreateWithFlags(&r->ev_ejoin[l], hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&r->ev_ecommit[l], hipEventDisableTiming) == hipSuccess;
    }
  }
  const size_t ev_bytes = (size_t)rv_replay::kRing * 2 * nr * 4;
  r->ds_evals = (uint32_t *)dalloc(r, ev_bytes);
  ok = ok && r->ds_evals && hipMemsetAsync(r->ds_evals, 0, ev_bytes, r->stream) == hipSuccess;
  r->grects[0] = g.tx0;
  r->grects[1] = g.ty0;
  r->grects[2] = g.tw;
  r->grects[3] = g.th;
  for (int lv = 0; lv < 3; lv++)
    r->jobs_half[lv] = r->jobs_full[lv] = r->jobs_sub[lv] = r->jobs_look[lv] = nullptr;
  if (!ok) {
    rv_set_error(RV_EHIP, "rv_replay_create: device allocation failed");
    rv_replay_destroy(r);
    return nullptr;
  }
  if (hipStreamSynchronize(r->stream) != hipSuccess) {
    rv_replay_destroy(r);
    return nullptr;
  }
  return r;
}

// The quantizers and lambdas of the frames of pyramid level `level`
// (FrameInvariants::set_quantizers, src/encoder.rs:865-880, from
// QuantizerParameters; the host computes them, rav1e_amd/rate.py).  Every
// level must be set before the first inter frame.
rv_replay *rv_replay_create(const rv_replay_cfg *cfg, void *stream) {
  return create_impl(cfg, stream, nullptr);
}

rv_replay *rv_replay_create_twin(rv_replay *primary, void *stream) {
  if (!primary || primary->n_groups > 1) {
    rv_set_error(RV_EINVAL, "rv_replay_create_twin: needs a one-group primary");
    return nullptr;
  }
  rv_replay *r = create_impl(&primary->cfg, stream, primary);
  if (!r) return nullptr;
  for (int l = 0; l < 3; l++) {
    r->lv[l] = primary->lv[l];
    r->db_level[l] = primary->db_level[l];
    r->cdef_str[l][0] = primary->cdef_str[l][0];
    r->cdef_str[l][1] = primary->cdef_str[l][1];
  }
  r->imp = primary->imp;  // owned by the primary
  r->eng = primary->eng;  // so is the importance window's engine
  r->coded = primary->coded;
  return r;
}

int rv_replay_seek(rv_replay *r, long n) {
  if (!r || n < 1) return rv_set_error(RV_EINVAL, "rv_replay_seek: n >= 1");
  r->coded = n;
  return RV_OK;
}

void *rv_replay_stream(rv_replay *r) { return r ? (void *)r->stream : nullptr; }

int rv_replay_set_level_params(rv_replay *r, int level, const rv_replay_level_params *p) {
  if (!r || !p || level < 0 || level > 2 || p->base_q_idx < 1 || p->base_q_idx > 255)
    return rv_set_error(RV_EINVAL, "rv_replay_set_level_params: bad arguments");
  rv_replay::Level &L = r->lv[level];
  const int bd = r->g.bd;
  // QuantizationContext::update of write_tx_tree's inter blocks
  // (src/encoder.rs:1925-1931, 1987-1994): per plane dc / ac deltas
  RV_R(rv_quant_ctx(p->base_q_idx, 64 * 64, 0, bd, p->dc_delta_q[0], p->ac_delta_q[0], &L.ql));
  RV_R(rv_quant_ctx(p->base_q_idx, 32 * 32, 0, bd, p->dc_delta_q[1], p->ac_delta_q[1], &L.qu));
  RV_R(rv_quant_ctx(p->base_q_idx, 32 * 32, 0, bd, p->dc_delta_q[2], p->ac_delta_q[2], &L.qv));
  RV_R(rv_quant_ctx(p->base_q_idx, 64 * 64, 1, bd, p->dc_delta_q[0], p->ac_delta_q[0], &L.qil));
  RV_R(rv_quant_ctx(p->base_q_idx, 32 * 32, 1, bd, p->dc_delta_q[1], p->ac_delta_q[1], &L.qiu));
  RV_R(rv_quant_ctx(p->base_q_idx, 32 * 32, 1, bd, p->dc_delta_q[2], p->ac_delta_q[2], &L.qiv));
  for (int l = 1; r->lvl && l < kLevels; l++) {  // the levels' smaller transforms
    const rv_replay::PLevel &P = r->pl[l];
    RV_R(rv_quant_ctx(p->base_q_idx, P.B * P.B, 0, bd, p->dc_delta_q[0], p->ac_delta_q[0], &L.qs[l][0]));
    for (int c = 1; c < 3; c++)
      RV_R(rv_quant_ctx(p->base_q_idx, P.bc * P.bch, 0, bd, p->dc_delta_q[c], p->ac_delta_q[c],
                        &L.qs[l][c]));
  }
  if (r->lrf) {  // the level's restoration units must be one superblock (checked before any frame)
    LrfGeo lg;
    RV_R(lrf_geometry(r->g.W, r->g.H, r->g.xdec, r->g.ydec, bd, p->base_q_idx, r->g.tws, r->g.ths, &lg));
  }
  L.qidx = p->base_q_idx;
  // deblock_filter_optimize's fast levels (inter frames at speed 10; speed 6
  // searches them on the device, deblock_slot)
  r->db_level[level] = (uint8_t)rv_deblock_fast_level(rv_q_lookup(1, p->base_q_idx, bd), bd, 0);
  r->cdef_str[level][0] = (uint8_t)(p->cdef_strengths & 0xff);
  r->cdef_str[level][1] = (uint8_t)((p->cdef_strengths >> 8) & 0xff);
  if (r->cdef_str[level][0] > 63 || r->cdef_str[level][1] > 63)
    return rv_set_error(RV_EINVAL, "rv_replay_set_level_params: cdef strength above 63");
  L.lambda = p->lambda;
  L.me_lambda = p->me_lambda;
  for (int i = 0; i < 3; i++) L.ds[i] = p->dist_scale[i];
  L.set = true;
  r->jobs_built = false;
  return RV_OK;
}

int rv_replay_synth_inputs(rv_replay *r, int t0) {
  if (!r) return rv_set_error(RV_EINVAL, "rv_replay_synth_inputs: null");
  for (size_t i = 0; i < r->inputs.size(); i++) {
    const RvInput &in = r->inputs[i];
    RV_R(rv_synth_frame(&in.y, &in.u, &in.v, t0 + (int)i, r->g.bd, r->stream));
  }
  RV_H(hipStreamSynchronize(r->stream));
  return RV_OK;
}

static int copy_plane(rv_replay *r, const rv_plane &p, uint8_t *host, bool to_device) {
  const int px = p.hbd ? 2 : 1;
  uint8_t *dev = (uint8_t *)p.data + ((size_t)p.yorigin * p.stride + p.xorigin) * px;
  if (to_device) {
    RV_H(hipMemcpy2DAsync(dev, (size_t)p.stride * px, host, (size_t)p.width * px,
                          (size_t)p.width * px, p.height, hipMemcpyHostToDevice, r->stream));
    return rv_plane_pad(&p, r->stream);
  }
  RV_H(hipMemcpy2DAsync(host, (size_t)p.width * px, dev, (size_t)p.stride * px,
                        (size_t)p.width * px, p.height, hipMemcpyDeviceToHost, r->stream));
  return RV_OK;
}

static int copy_frame(rv_replay *r, const rv_plane *pl, void *host, bool to_device) {
  const int px = r->g.hbd ? 2 : 1;
  uint8_t *p = (uint8_t *)host;
  for (int k = 0; k < 3; k++) {
    RV_R(copy_plane(r, pl[k], p, to_device));
    p += (size_t)pl[k].width * pl[k].height * px;
  }
  RV_H(hipStreamSynchronize(r->stream));
  return RV_OK;
}

int rv_replay_set_input(rv_replay *r, int idx, const void *host_yuv) {
  if (!r || !host_yuv || idx < 0 || idx >= (int)r->inputs.size())
    return rv_set_error(RV_EINVAL, "rv_replay_set_input: bad index");
  const RvInput &in = r->inputs[idx];
  const rv_plane pl[3] = {in.y, in.u, in.v};
  return copy_frame(r, pl, const_cast<void *>(host_yuv), true);
}

int rv_replay_get_input(rv_replay *r, int idx, void *host_yuv) {
  if (!r || !host_yuv || idx < 0 || idx >= (int)r->inputs.size())
    return rv_set_error(RV_EINVAL, "rv_replay_get_input: bad index");
  const RvInput &in = r->inputs[idx];
  const rv_plane pl[3] = {in.y, in.u, in.v};
  return copy_frame(r, pl, host_yuv, false);
}

// The reconstruction of display frame `display` (it must still be in the
// DPB: the last 12 displays).
int rv_replay_get_recon(rv_replay *r, int display, void *host_yuv) {
  if (!r || !host_yuv || display < 0) return rv_set_error(RV_EINVAL, "rv_replay_get_recon");
  const RvSlot &s = r->slots[display % kSlots];
  const rv_plane pl[3] = {s.y, s.u, s.v};
  return copy_frame(r, pl, host_yuv, false);
}

int rv_replay_set_importances(rv_replay *r, const float *host, int n) {
  if (!r) return rv_set_error(RV_EINVAL, "rv_replay_set_importances: null");
  const int need = r->g.w_imp * r->g.h_imp;
  if (!host) {
    r->imp = nullptr;
    return RV_OK;
  }
  if (n != need) return rv_set_error(RV_EINVAL, "rv_replay_set_importances: size != w_imp * h_imp");
  float *d = (float *)dalloc(r, (size_t)need * 4);
  if (!d) return rv_set_error(RV_EHIP, "rv_replay_set_importances: alloc");
  RV_H(hipMemcpy(d, host, (size_t)need * 4, hipMemcpyHostToDevice));
  r->imp = d;
  return RV_OK;
}

// Tile groups of all ranks (rects in superblocks, 4 per group), this
// instance's index among them, and the RCCL communicator (rv_comm_create)
// that all-gathers the reconstructions; comm may be null: then the caller
// moves the packed regions itself (rv_replay_exchange_buffers,
// rv_replay_import).
int rv_replay_set_groups(rv_replay *r, int n_groups, const int32_t *rects, int my_group,
                         void *comm) {
  if (!r || n_groups < 1 || n_groups > kMaxGroups || !rects || my_group < 0 ||
      my_group >= n_groups)
    return rv_set_error(RV_EINVAL, "rv_replay_set_groups: bad groups");
  const Geo &g = r->g;
  if (rects[4 * my_group] != g.tx0 || rects[4 * my_group + 1] != g.ty0 ||
      rects[4 * my_group + 2] != g.tw || rects[4 * my_group + 3] != g.th)
    return rv_set_error(RV_EINVAL, "rv_replay_set_groups: my group != the configured tile group");
  memcpy(r->grects, rects, (size_t)n_groups * 4 * sizeof(int32_t));
  r->n_groups = n_groups;
  r->my_group = my_group;
  size_t most = 0;
  for (int k = 0; k < n_groups; k++) {
    XRect xr[9];
    int nx;
    const size_t b = (size_t)group_rects(r, k, xr, &nx);
    most = b > most ? b : most;
  }
  r->xbytes = (most + 255) / 256 * 256;
  if (n_groups > 1 || comm) {  // one group + a communicator: a 1-rank all-gather
    r->xsend = (uint8_t *)dalloc(r, r->xbytes);
    r->xrecv = (uint8_t *)dalloc(r, r->xbytes * n_groups);
    if (!r->xsend || !r->xrecv) return rv_set_error(RV_EHIP, "rv_replay_set_groups: alloc");
  }
  r->comm = comm;
  return RV_OK;
}

int rv_replay_exchange_buffers(rv_replay *r, void **send, void **recv, size_t *bytes_per_group) {
  if (!r || !send || !recv || !bytes_per_group)
    return rv_set_error(RV_EINVAL, "rv_replay_exchange_buffers: null");
  *send = r->xsend;
  *recv = r->xrecv;
  *bytes_per_group = r->xbytes;
  return RV_OK;
}

// Unpack every other group's region of the last coded frame from the
// gathered buffer (group k at k * bytes_per_group) and pad: the frame is
// then a complete reference on this rank (src/encoder.rs:3411-3429).
int rv_replay_import(rv_replay *r) {
  if (!r) return rv_set_error(RV_EINVAL, "rv_replay_import: null");
  // one group without a communicator, or the key frame (every rank copied
  // its own input): nothing to move
  if ((r->n_groups < 2 && !r->comm) || r->last.is_key) return RV_OK;
  const RvSlot &s = r->slots[r->last.display % kSlots];
  XRect rects[9 * kMaxGroups];
  int n = 0;
  for (int k = 0; k < r->n_groups; k++) {
    if (k == r->my_group) continue;
    XRect xr[9];
    int nx;
    group_rects(r, k, xr, &nx);
    for (int p = 0; p < nx; p++) {
      xr[p].off += (int64_t)k * (int64_t)r->xbytes;
      rects[n++] = xr[p];
    }
  }
  RV_R(xcopy(r, s, rects, n, 1, r->xrecv));
  // the whole frame and its block map are in: deblock it (every rank the
  // same way), then pad
  return filter_slot(r, s, r->inputs[r->last.display % r->inputs.size()], r->last.level);
}

// The host side of a round loop: check(q) queues check q, which lists the
// jobs to re-run and publishes their count into the ring; eval(q) queues the
// round that re-runs check q's list.  The host keeps kRoundsAhead rounds
// queued beyond the last count it has read (it spins on the published
// counts, no stream synchronisation), so the GPU never waits on the host;
// the loop ends at the first check that lists nothing (the rounds queued
// after it find empty lists).  budget: the chain's depth bound (see the
// callers); a check still listing jobs after it is an internal error.
}  // extern "C"

template <typename Check, typename Eval>
static int run_rounds(RoundRing &rr, hipStream_t xs, int budget, Check &&check, Eval &&eval,
               long *nrounds, long *nre, bool *changed, const char *what, long frame, int level) {
  static const bool mv_trace = getenv("RAV1E_HIP_MV_TRACE") != nullptr;
  // RAV1E_HIP_ROUNDS_AHEAD=n: rounds queued beyond the last count read (A/B)
  static const int ahead = getenv("RAV1E_HIP_ROUNDS_AHEAD") ? atoi(getenv("RAV1E_HIP_ROUNDS_AHEAD"))
                                                            : rv_replay::kRoundsAhead;
  if (changed) *changed = false;
  rr.last_count = -1;
  const uint32_t first = rr.seq++;
  RV_R(check(first));
  int queued = 0;  // evaluation rounds queued (round j evaluates check j - 1's list)
  for (int seen = 0;; seen++) {
    while (queued < budget && queued < seen + (ahead > 0 ? ahead : 1)) {
      RV_R(eval(first + (uint32_t)queued));
      RV_R(check(rr.seq++));
      queued++;
    }
    const uint32_t q = first + (uint32_t)seen;
    volatile unsigned long long *pub = rr.h_pub + q % RoundRing::kPub;
    const auto t0 = std::chrono::steady_clock::now();
    unsigned long long v;
    for (long spin = 0;; spin++) {
      v = *pub;
      if ((uint32_t)(v >> 32) == q) break;
      if ((spin & 1023) == 1023) {
        const hipError_t he = hipStreamQuery(xs);
        if (he != hipSuccess && he != hipErrorNotReady)
          return rv_set_error(RV_EHIP, "rv_replay_frame: a round failed");
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30))
          return rv_set_error(RV_EHIP, "rv_replay_frame: a round's count never arrived");
        std::this_thread::yield();
      }
    }
    const int c = (int)(uint32_t)v;
    rr.last_count = c;
    if (mv_trace) fprintf(stderr, "%s frame %ld level %d check %d: %d\n", what, frame, level, seen, c);
    if (c == 0) return RV_OK;
    if (seen >= budget)
      return rv_set_error(RV_EHIP, "rv_replay_frame: rounds beyond the chain's dependency "
                                   "depth (internal error)");
    *nre += c;
    (*nrounds)++;
    if (changed) *changed = true;
  }
}

extern "C" {

// The lookahead of coded frame fi (compute_lookahead_motion_vectors,
// src/api/internal.rs:514-622) on stream xs: F0 the input's hres / qres
// (pyramid: false when they are already current), F1 build_coarse_pmvs,
// then F2L + FL (build_half_res_pmvs / build_full_res_pmvs) with their EPZS
// sets (la_check_kernel): round 0 stores every F2L set (the field guessed
// from o's previous contents) and runs every F2L search, then the same for
// FL; then the rounds.  Budget: a quadrant search reads the quadrants of
// the superblocks left of and above it, so it settles by round tws + ths - 1;
// a 16x16 search reads its coarse / quadrant predictors (settled by then)
// and the 16x16 blocks left of and above it, so it settles 4 tws + 4 ths - 2
// rounds later.  e: the frame's timing events (null: untimed).
static int lookahead_frame(rv_replay *r, RoundRing &rr, hipStream_t xs,
                           const rv_replay_frame_info &fi, const LaRefs &lr, long frame,
                           const LaOut &o, int32_t *la_list, bool pyramid, long *nrounds,
                           long *nre, hipEvent_t *e) {
  const Geo &g = r->g;
  const int lv = fi.level, nr = g.nsb, RL = lr.n;
  const RvInput &cur = r->inputs[fi.display % r->inputs.size()];
  rv_plane refs_h[kImpMaxRefs], refs_q[kImpMaxRefs], refs_o[kImpMaxRefs];
  const uint32_t *box[kImpMaxRefs];
  for (int k = 0; k < RL; k++) {
    const RvInput &ri = r->inputs[lr.disp[k] % r->inputs.size()];
    refs_h[k] = ri.hres;
    refs_q[k] = ri.qres;
    refs_o[k] = ri.y;  // the lookahead searches the references' original frames
    box[k] = ri.qres_box;
  }
  auto ev = [&](int i) -> int {
    if (e) RV_H(hipEventRecord(e[i], xs));
    return RV_OK;
  };
  if (pyramid) {  // F0 (encode_frame, src/encoder.rs:3382-3385)
    RV_R(rv_plane_pyramid(&cur.y, &cur.hres, &cur.qres, xs));
    if (r->sea) RV_R(rv_plane_box_sums(&cur.qres, cur.qres_box, xs));
  }
  RV_R(ev(1));
  // F1 coarse full search (build_coarse_pmvs), every reference in one launch
  RV_R(rv_full_search_multi(&cur.qres, refs_q, RL, r->fs_jobs[lv], nr, 16, 16, 1, 0, o.coarse,
                            nullptr, r->sea ? box : nullptr, xs));
  RV_R(ev(2));
  LaArgs la_a;
  memset(&la_a, 0, sizeof(la_a));
  la_a.g = g;
  la_a.eg = EpzsGeo{g.tx0, g.ty0, g.tw, g.th, g.tws, g.ths, g.W, g.H, g.w_in_b, g.h_in_b};
  la_a.jh = r->jobs_half_l[lv];
  la_a.jl = r->jobs_look[lv];
  la_a.sl = r->src_look;
  la_a.coarse = o.coarse;
  la_a.half_l = o.half_l;
  la_a.look = o.look;
  const int nh = nr * RL * 4, nl = nr * RL * 16;
  la_a.nref = RL;
  la_a.list_h = la_list;
  la_a.list_l = la_list + nh;
  auto la_launch = [&](int what, uint32_t q, bool init) -> int {
    la_a.what = what;
    la_a.init = init ? 1 : 0;
    la_a.pub = rr.pub(q, !init);
    const int n = ((what & 1) ? nh : 0) + ((what & 2) ? nl : 0);
    la_check_kernel<<<(n + 255) / 256, 256, 0, xs>>>(la_a);
    RV_H(hipGetLastError());
    return RV_OK;
  };
  auto f2l = [&](const int32_t *list, const int32_t *cnt) {
    return rv_diamond_search_multi(&cur.hres, refs_h, RL, r->jobs_half_l[lv], nr * 4, 16, 16, 0,
                                   0, 0, g.bd, o.half_l, nullptr, nullptr, xs, nullptr, list, cnt,
                                   0);
  };
  auto fl = [&](const int32_t *list, const int32_t *cnt) {
    return rv_diamond_search_multi(&cur.y, refs_o, RL, r->jobs_look[lv], nr * 16, 16, 16, 0, 0, 0,
                                   g.bd, o.look, nullptr, nullptr, xs, nullptr, list, cnt, 0);
  };
  RV_R(la_launch(1, 0, true));
  RV_R(f2l(nullptr, nullptr));
  RV_R(ev(3));
  RV_R(ev(rv_replay::kStageEv));
  RV_R(la_launch(2, 0, true));
  RV_R(fl(nullptr, nullptr));
  (*nrounds)++;
  RV_R(run_rounds(
      rr, xs, 5 * (g.tws + g.ths), [&](uint32_t q) { return la_launch(3, q, false); },
      [&](uint32_t q) -> int {
        RV_R(f2l(la_list, rr.slot(q)));
        return fl(la_list + nh, rr.slot(q) + 1);
      },
      nrounds, nre, nullptr, "lookahead", frame, lv));
  RV_R(ev(rv_replay::kStageEv + 1));
  return RV_OK;
}

// the coded index of display d (frame_info's inverse)
static long coded_of_display(long d) {
  if (d == 0) return 0;
  static const int jof[4] = {0, 2, 1, 3}, off[4] = {4, 2, 1, 3};
  const int j = jof[d % 4];
  return 4 * ((d - off[j]) / 4) + j + 1;
}

// Several tile groups: every group's part of frame m's importance data into
// every group's entry (the propagation reads the whole frame).  One group
// covering the frame: nothing to do.
static int la_exchange(rv_replay *r, long m, RvLaEngine::Entry &e, int R, hipStream_t xs) {
  RvLaEngine &E = *r->eng;
  const Geo &g = r->g;
  const int ng = r->n_groups;
  if (ng <= 1 && !E.comm) {
    if (g.tx0 || g.ty0 || g.vis_w != g.W || g.vis_h != g.H)
      return rv_set_error(RV_EINVAL, "rv_replay_frame: a tile group's window needs the other groups "
                                     "(rv_replay_set_groups + rv_replay_set_la_exchange)");
    return RV_OK;
  }
  auto rect = [&](int j) { return r->grects + 4 * j; };
  (void)R;
  if (E.comm) {  // the encode thread all-gathers (la_encode_exchange)
    RV_H(hipEventRecord(e.ev_data, xs));
    std::unique_lock<std::mutex> lk(E.mu);
    E.data_ready = m;
    E.cv.notify_all();
    if (!E.cv.wait_for(lk, std::chrono::seconds(kEngineWaitS),
                       [&] { return E.stop || E.xchg_done >= m; }))
      return rv_set_error(RV_EHIP, "la_exchange: the frame's parts were never all-gathered");
    if (E.stop) return rv_set_error(RV_EINVAL, "la_exchange: stopped");
    lk.unlock();
    RV_H(hipStreamWaitEvent(xs, e.ev_xchg, 0));
    return RV_OK;
  }
  rv_la_hub *h = E.hub;
  if (!h || h->n != ng)
    return rv_set_error(RV_EINVAL, "rv_replay_frame: a tile group's window needs an exchange "
                                   "(rv_replay_set_la_exchange)");
  const int k = E.hub_k, slot = (int)(m % rv_la_hub::kRing);
  const int32_t *me = rect(k);
  RV_R(impwin_part(e.f, R, me[0], me[1], me[2], me[3], g.w_imp, g.h_imp, h->buf[slot][k], false, xs));
  RV_H(hipEventRecord(h->ev[slot][k], xs));
  {
    std::unique_lock<std::mutex> lk(h->mu);
    h->posted[k] = m;
    h->cv.notify_all();
    if (!h->cv.wait_for(lk, std::chrono::seconds(kEngineWaitS), [&] {
          for (int j = 0; j < ng; j++)
            if (h->posted[j] < m) return false;
          return true;
        }))
      return rv_set_error(RV_EHIP, "la_exchange: a group's part never arrived");
  }
  for (int j = 0; j < ng; j++) {
    if (j == k) continue;
    RV_H(hipStreamWaitEvent(xs, h->ev[slot][j], 0));
    RV_R(impwin_part(e.f, R, rect(j)[0], rect(j)[1], rect(j)[2], rect(j)[3], g.w_imp, g.h_imp,
                     h->buf[slot][j], true, xs));
  }
  return RV_OK;
}

// One step of the engine: coded frame m's lookahead and importance data
// into its entry, then the window propagation of every frame whose window
// is now complete (n + W = m, or the stream's last frame).
static int la_step(rv_replay *r, long m) {
  RvLaEngine &E = *r->eng;
  const Geo &g = r->g;
  hipStream_t xs = E.las;
  RvLaEngine::Entry &e = E.at(m);
  if (m - E.RW >= 1) RV_H(hipStreamWaitEvent(xs, e.ev_used, 0));  // frame m - RW is done with it
  rv_replay_frame_info fi;
  frame_info(m, g.R, &fi);
  const LaRefs lr = la_refs_of(m, g.R);
  // the pyramids of the frame's and its lookahead references' inputs
  long ds[1 + kImpMaxRefs];
  int nd = 0;
  ds[nd++] = fi.display;
  for (int k = 0; k < lr.n; k++) ds[nd++] = lr.disp[k];
  for (int i = 0; i < nd; i++) {
    const size_t idx = (size_t)(ds[i] % (long)r->inputs.size());
    if (E.pyr_display[idx] == ds[i]) continue;
    const RvInput &in = r->inputs[idx];
    RV_R(rv_plane_pyramid(&in.y, &in.hres, &in.qres, xs));
    if (r->sea) RV_R(rv_plane_box_sums(&in.qres, in.qres_box, xs));
    E.pyr_display[idx] = ds[i];
  }
  const size_t nr = (size_t)g.nsb * lr.n;
  if (m > 1) {  // the field's first guess: the previous frame's lookahead
    const RvLaEngine::Entry &p = E.at(m - 1);
    RV_H(hipMemcpyAsync(e.o.half_l, p.o.half_l, nr * 4 * sizeof(rv_fs_result),
                        hipMemcpyDeviceToDevice, xs));
    RV_H(hipMemcpyAsync(e.o.look, p.o.look, nr * 16 * sizeof(rv_fs_result),
                        hipMemcpyDeviceToDevice, xs));
  }
  long la_rounds = 0, la_reeval = 0;
  RV_R(lookahead_frame(r, E.rr, xs, fi, lr, m - 1, e.o, E.la_list, false, &la_rounds, &la_reeval,
                       nullptr));
  {
    std::lock_guard<std::mutex> lk(E.mu);
    E.la_round_sum += la_rounds;
    E.la_reeval += la_reeval;
    E.la_frames++;
  }
  rv_plane refs_o[kImpMaxRefs];
  for (int k = 0; k < lr.n; k++) refs_o[k] = r->inputs[lr.disp[k] % r->inputs.size()].y;
  // the entry is frame m's from here on (the encode's part exchange reads it)
  e.m = m;
  e.fi = fi;
  e.lr = lr;
  RV_R(impwin_group_data(r->inputs[fi.display % r->inputs.size()].y, refs_o, lr.n, g.bd, e.o.look,
                         g.tx0, g.ty0, g.tw, g.th, g.w_imp, g.h_imp, e.f, xs));
  RV_R(la_exchange(r, m, e, lr.n, xs));
  RV_R(impwin_lists(e.f, lr.n, g.w_imp, g.h_imp, E.scratch, E.scratch_bytes, xs));
  const long last_frame = E.limit > 0 ? E.limit - 1 : -1;
  const size_t ni = (size_t)g.w_imp * g.h_imp;
  // split: the passes run on lap once frame m's lists are in.  Entry reuse
  // stays ordered: las waits ev_used of frame m - RW, recorded after that
  // frame's encode waited its ev_imp on lap -- behind every earlier
  // window's passes, the only other readers of the entry's lists.
  if (E.split && E.imp_next <= m && (E.imp_next + E.W <= m || m == last_frame)) {
    RV_H(hipEventRecord(e.ev_lists, xs));
    RV_H(hipStreamWaitEvent(E.lap, e.ev_lists, 0));
    xs = E.lap;
  }
  while (E.imp_next <= m && (E.imp_next + E.W <= m || m == last_frame)) {
    const long n = E.imp_next, last = n + E.W < m ? n + E.W : m;
    {
      std::vector<float *> zs;
      for (long t = n; t <= last; t++) zs.push_back(E.at(t).f.imp);
      RV_R(impwin_zero(zs.data(), (int)zs.size(), (int)ni, xs));
    }
    for (long s2 = last; s2 > n; s2--) {
      const RvLaEngine::Entry &es = E.at(s2);
      // the frame's passes into its reference slots in the window (mv index
      // order; the split is over every slot, :886-942), one launch: within
      // the window they land on distinct frames (only the key frame, before
      // every window, can fill two slots)
      const int nu = es.lr.n;
      int ks[kImpMaxRefs], np = 0;
      float *dst[kImpMaxRefs];
      for (int j = 0; j < nu; j++) {
        const int k = es.lr.order[j];
        const long t = coded_of_display(es.lr.disp[k]);
        if (t < n) continue;  // before the window: gone (:944-948)
        for (int i = 0; i < np; i++)
          if (dst[i] == E.at(t).f.imp)
            return rv_set_error(RV_EINVAL, "la_step: two passes into one frame");
        ks[np] = k;
        dst[np++] = E.at(t).f.imp;
      }
      if (np) RV_R(impwin_pass(es.f, ks, dst, np, nu, g.w_imp, g.h_imp, xs));
    }
    RV_R(impwin_final(E.at(n).f, g.w_imp, g.h_imp, xs));
    RV_H(hipEventRecord(E.at(n).ev_imp, xs));
    std::lock_guard<std::mutex> lk(E.mu);
    E.imp_ready = n;
    E.imp_next = n + 1;
    E.cv.notify_all();
  }
  return RV_OK;
}

// the engine's stream (RAV1E_HIP_LA_PRIORITY=1: the lowest priority, which
// HIP serves from a queue pool of its own)
static int la_stream_create(RvLaEngine *E) {
  const char *lpe = getenv("RAV1E_HIP_LA_PRIORITY");
  const bool low = lpe && lpe[0] == '1';
  int least = 0, greatest = 0;
  if (low) {
    RV_H(hipDeviceGetStreamPriorityRange(&least, &greatest));
    RV_H(hipStreamCreateWithPriority(&E->las, hipStreamNonBlocking, least));
    if (E->split) RV_H(hipStreamCreateWithPriority(&E->lap, hipStreamNonBlocking, least));
  } else {
    RV_H(hipStreamCreateWithFlags(&E->las, hipStreamNonBlocking));
    if (E->split) RV_H(hipStreamCreateWithFlags(&E->lap, hipStreamNonBlocking));
  }
  return RV_OK;
}

static void la_thread_main(rv_replay *r) {
  RvLaEngine &E = *r->eng;
  (void)hipSetDevice(E.dev);
  for (long m = 1;; m++) {
    {
      std::unique_lock<std::mutex> lk(E.mu);
      E.cv.wait(lk, [&] {
        if (E.stop) return true;
        // frame m reads the inputs of displays <= 4 ((m - 1) / 4) + 4
        // (frame_info): with them in place it may run before frame m - W
        // is asked for, as rav1e computes a frame's lookahead on arrival
        // not before the first frame is asked for -- or the inputs are declared
        // in place (tile groups coded one after another in one process need
        // every group's engine running: their parts meet in the hub)
        if (E.requested < 1 && E.inputs_ready == 0) return false;
        if (m > E.requested + E.W && 4 * ((m - 1) / 4) + 4 >= E.inputs_ready) return false;
        if (E.limit > 0 && m >= E.limit) return false;
        return m - E.RW < 1 || E.at(m).used_by == m - E.RW;
      });
      if (E.stop) return;
    }
    int rc = E.las ? RV_OK : la_stream_create(&E);
    if (rc == RV_OK) rc = ensure_jobs(r);  // (the engine may start before the first frame)
    if (rc == RV_OK) rc = la_step(r, m);
    if (rc != RV_OK) {
      std::lock_guard<std::mutex> lk(E.mu);
      E.err = rc;
      E.msg = rv_last_error();
      E.cv.notify_all();
      return;
    }
  }
}

static void la_engine_destroy(rv_replay *r) {
  RvLaEngine *E = r->eng;
  r->eng = nullptr;
  if (!E || !r->eng_owned) return;
  {
    std::lock_guard<std::mutex> lk(E->mu);
    E->stop = true;
    E->cv.notify_all();
  }
  if (E->th.joinable()) E->th.join();
  if (E->las) (void)hipStreamSynchronize(E->las);
  if (E->lap) (void)hipStreamSynchronize(E->lap);
  for (auto &en : E->ring)
    for (hipEvent_t ev : {en.ev_imp, en.ev_used, en.ev_data, en.ev_xchg, en.ev_lists})
      if (ev) (void)hipEventDestroy(ev);
  for (hipEvent_t ev : E->hub_ev)
    if (ev) (void)hipEventDestroy(ev);
  if (E->rr.h_pub) (void)hipHostFree(E->rr.h_pub);
  if (E->las) (void)hipStreamDestroy(E->las);
  if (E->lap) (void)hipStreamDestroy(E->lap);
  delete E;  // its device arrays are the replay's allocations (freed with it)
}

// Tile groups over RCCL: before frame n takes its importances, the encode
// thread all-gathers the lookahead parts of every frame up to n + W (the
// window's end) on its own stream, with the same communicator as the
// reconstruction all-gathers -- each rank issues the same collectives in
// the same order on one stream: [parts 1 .. W + 1], frame 1, recon 1,
// [part W + 2], frame 2, ...
static int la_encode_exchange(rv_replay *r, long n, hipStream_t st) {
  RvLaEngine &E = *r->eng;
  if (!E.comm) return RV_OK;
  if (!r->eng_owned)
    return rv_set_error(RV_EINVAL, "rv_replay_frame: RCCL lookahead parts on the primary only");
#if RV_HAVE_RCCL
  const Geo &g = r->g;
  long last = n + E.W;
  if (E.limit > 0 && last > E.limit - 1) last = E.limit - 1;
  {
    std::lock_guard<std::mutex> lk(E.mu);
    if (n > E.requested) E.requested = n;  // the engine runs up to n + W
    E.cv.notify_all();
  }
  for (long m = E.xchg_next; m <= last; m++) {
    {
      std::unique_lock<std::mutex> lk(E.mu);
      if (!E.cv.wait_for(lk, std::chrono::seconds(kEngineWaitS),
                         [&] { return E.err != 0 || E.data_ready >= m; }))
        return rv_set_error(RV_EHIP, "rv_replay_frame: the lookahead engine's part never came");
      if (E.err) return rv_set_error(E.err, E.msg.c_str());
    }
    RvLaEngine::Entry &e = E.at(m);
    if (e.m != m) return rv_set_error(RV_EINVAL, "rv_replay_frame: the lookahead ring lost a frame");
    const int R = e.lr.n;
    const int32_t *me = r->grects + 4 * r->my_group;
    RV_H(hipStreamWaitEvent(st, e.ev_data, 0));
    RV_R(impwin_part(e.f, R, me[0], me[1], me[2], me[3], g.w_imp, g.h_imp, E.psend, false, st));
    if (ncclAllGather(E.psend, E.precv, E.pbytes, ncclUint8, (ncclComm_t)E.comm, st) != ncclSuccess)
      return rv_set_error(RV_EHIP, "rv_replay_frame: ncclAllGather (lookahead parts)");
    for (int j = 0; j < r->n_groups; j++) {
      if (j == r->my_group) continue;
      const int32_t *q = r->grects + 4 * j;
      RV_R(impwin_part(e.f, R, q[0], q[1], q[2], q[3], g.w_imp, g.h_imp,
                       E.precv + (size_t)j * E.pbytes, true, st));
    }
    RV_H(hipEventRecord(e.ev_xchg, st));
    std::lock_guard<std::mutex> lk(E.mu);
    E.xchg_done = m;
    E.xchg_next = m + 1;
    E.cv.notify_all();
  }
  return RV_OK;
#else
  (void)n;
  (void)st;
  return rv_set_error(RV_EINVAL, "rv_replay_frame: built without RCCL");
#endif
}

// The encode side: wait for frame n's importances, take its lookahead.
// (rv_replay_set_inputs_ready below lets the engine run further ahead.)
static int la_engine_take(rv_replay *r, long n, hipStream_t st, const float **imp) {
  RvLaEngine &E = *r->eng;
  // the engine never computes a frame at or past the stream's limit
  if (E.limit > 0 && n >= E.limit)
    return rv_set_error(RV_EINVAL, "rv_replay_frame: past the stream's limit "
                                   "(rv_replay_set_imp_window)");
  {
    std::unique_lock<std::mutex> lk(E.mu);
    if (n > E.requested) E.requested = n;
    E.cv.notify_all();
    // Bounded: an engine frame takes milliseconds.  It never arrives when a
    // frame RW or more back was skipped (rv_replay_seek) and never coded:
    // the engine then waits for that frame's entry to be released.
    if (!E.cv.wait_for(lk, std::chrono::seconds(kEngineWaitS),
                       [&] { return E.err != 0 || E.imp_ready >= n; }))
      return rv_set_error(RV_EHIP, "rv_replay_frame: the lookahead engine did not deliver the "
                                   "frame's importances (a frame skipped and never coded?)");
    if (E.err) return rv_set_error(E.err, E.msg.c_str());
  }
  const RvLaEngine::Entry &e = E.at(n);
  if (e.m != n) return rv_set_error(RV_EINVAL, "rv_replay_frame: the lookahead ring lost a frame");
  RV_H(hipStreamWaitEvent(st, e.ev_imp, 0));
  const size_t nr = (size_t)r->g.nsb * r->g.R;
  RV_H(hipMemcpyAsync(r->coarse, e.o.coarse, nr * sizeof(rv_fs_result), hipMemcpyDeviceToDevice, st));
  RV_H(hipMemcpyAsync(r->half_l, e.o.half_l, nr * 4 * sizeof(rv_fs_result),
                      hipMemcpyDeviceToDevice, st));
  RV_H(hipMemcpyAsync(r->look, e.o.look, nr * 16 * sizeof(rv_fs_result), hipMemcpyDeviceToDevice,
                      st));
  *imp = e.f.fin;
  return RV_OK;
}

// ... and when the frame's last reader of the entry is queued
static int la_engine_release(rv_replay *r, long n, hipStream_t st) {
  RvLaEngine &E = *r->eng;
  RvLaEngine::Entry &e = E.at(n);
  RV_H(hipEventRecord(e.ev_used, st));
  std::lock_guard<std::mutex> lk(E.mu);
  e.used_by = n;
  E.cv.notify_all();
  return RV_OK;
}

}  // extern "C" (closed for the C++ helpers above)
extern "C" {

// The inputs of displays < `displays` are in place and stay until coded:
// the engine may run the lookahead of every frame they cover (up to its
// ring), not only up to W frames past the last frame asked for.
int rv_replay_set_inputs_ready(rv_replay *r, long displays) {
  if (!r || displays < 0) return rv_set_error(RV_EINVAL, "rv_replay_set_inputs_ready: bad arguments");
  if (displays > (long)r->inputs.size())
    return rv_set_error(RV_EINVAL, "rv_replay_set_inputs_ready: more displays than input slots");
  if (r->eng) {
    // the engine may start now, before any frame: its job records first
    RV_R(ensure_jobs(r));
    std::lock_guard<std::mutex> lk(r->eng->mu);
    r->eng->inputs_ready = displays;
    r->eng->cv.notify_all();
  }
  return RV_OK;
}

// The importance window W (rdo_lookahead_frames) and the stream's length in
// coded frames (limit; 0: unbounded).  W = 0: the importances are an input
// (rv_replay_set_importances).  Only before the first frame, on a primary
// instance replaying the whole frame as one group.
int rv_replay_set_imp_window(rv_replay *r, int window, long limit) {
  if (!r || window < 0 || window > 1024 || limit < 0)
    return rv_set_error(RV_EINVAL, "rv_replay_set_imp_window: bad arguments");
  if (r->coded > 0) return rv_set_error(RV_EINVAL, "rv_replay_set_imp_window: after the first frame");
  const Geo &g = r->g;
  (void)g;  // a tile group's window exchanges parts (rv_replay_set_la_exchange)
  if (r->eng && !r->eng_owned)
    return rv_set_error(RV_EINVAL, "rv_replay_set_imp_window: on the primary instance");
  la_engine_destroy(r);
  if (!window) return RV_OK;
  RvLaEngine *E = new RvLaEngine();
  E->W = window;
  E->RW = window + 1 + RvLaEngine::kLaSlack;
  E->limit = limit;
  // RAV1E_HIP_LA_PRIORITY=1: the engine's stream at the lowest priority.
  // HIP keeps a queue pool per priority, so it then gets a hardware queue of
  // its own instead of sharing one (GPU_MAX_HW_QUEUES: 4) with the twin's
  // stream.  Measured at 2160p (r04p1): 101-103 vs 118 fps -- the lookahead's
  // kernels then run beside the rounds' and slow them more than the shared
  // queue's ordering does; off.
  //
  // The stream is created on the engine's thread when the first frame is
  // asked for, after the twin instance's streams: HIP gives a new stream the
  // least-used hardware queue, so the engine's then shares one with a
  // frame-edge or entropy stream instead of with the twin's round kernels
  // (which the trace showed waiting 6-7 us behind the lookahead's).
  // RAV1E_HIP_LA_LAZY=0: created here (A/B).
  // RAV1E_HIP_LA_SPLIT=1: the window passes on a stream of their own.  Off:
  // the extra stream shares the 4 hardware queues with the encode's and
  // measured 4-10 % slower (profiles/r05i_*).
  const char *spe = getenv("RAV1E_HIP_LA_SPLIT");
  E->split = spe && spe[0] == '1';
  const char *lze = getenv("RAV1E_HIP_LA_LAZY");
  const bool lazy = !(lze && lze[0] == '0');
  bool ok = hipGetDevice(&E->dev) == hipSuccess &&
            (lazy || la_stream_create(E) == RV_OK) && round_ring_alloc(r, E->rr, r->stream);
  const int ni = g.w_imp * g.h_imp, nr = g.nsb * r->RA;  // the lookahead's references
  E->la_list = ok ? (int32_t *)dalloc(r, (size_t)nr * 20 * 4) : nullptr;
  E->scratch_bytes = impwin_scratch_bytes(ni);
  E->scratch = ok ? dalloc(r, E->scratch_bytes) : nullptr;
  ok = ok && E->la_list && E->scratch;
  E->ring.resize((size_t)E->RW);
  const size_t ob = ((size_t)nr * 21 * sizeof(rv_fs_result) + 255) / 256 * 256;
  for (auto &en : E->ring) {
    if (!ok) break;
    uint8_t *m = (uint8_t *)dalloc(r, ob + impwin_frame_bytes(ni, r->RA));
    ok = m && hipMemsetAsync(m, 0, ob, r->stream) == hipSuccess &&
         hipEventCreateWithFlags(&en.ev_imp, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&en.ev_used, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&en.ev_data, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&en.ev_xchg, hipEventDisableTiming) == hipSuccess &&
         hipEventCreateWithFlags(&en.ev_lists, hipEventDisableTiming) == hipSuccess;
    if (!ok) break;
    en.o.coarse = (rv_fs_result *)m;
    en.o.half_l = en.o.coarse + nr;
    en.o.look = en.o.half_l + (size_t)nr * 4;
    impwin_frame_carve(en.f, m + ob, ni, r->RA);
  }
  E->pyr_display.assign(r->inputs.size(), -1);
  r->eng = E;
  r->eng_owned = true;
  if (!ok || hipStreamSynchronize(r->stream) != hipSuccess) {
    la_engine_destroy(r);
    return rv_set_error(RV_EHIP, "rv_replay_set_imp_window: allocation failed");
  }
  E->th = std::thread(la_thread_main, r);
  return RV_OK;
}

// Tile groups with an importance window: how each frame's importance data
// of the other groups arrives (la_exchange).
rv_la_hub *rv_la_hub_create(int n_groups) {
  if (n_groups < 2 || n_groups > kMaxGroups) {
    rv_set_error(RV_EINVAL, "rv_la_hub_create: 2 .. kMaxGroups groups");
    return nullptr;
  }
  rv_la_hub *h = new rv_la_hub();
  h->n = n_groups;
  h->posted.assign((size_t)n_groups, 0);
  for (int s = 0; s < rv_la_hub::kRing; s++) {
    h->buf[s].assign((size_t)n_groups, nullptr);
    h->ev[s].assign((size_t)n_groups, nullptr);
  }
  return h;
}
void rv_la_hub_destroy(rv_la_hub *h) { delete h; }  // the members own the buffers / events

int rv_replay_set_la_exchange(rv_replay *r, void *comm, rv_la_hub *hub) {
  if (!r || (!comm == !hub)) return rv_set_error(RV_EINVAL, "rv_replay_set_la_exchange: comm xor hub");
  if (!r->eng || !r->eng_owned || r->coded > 0)
    return rv_set_error(RV_EINVAL, "rv_replay_set_la_exchange: a primary instance with a window, "
                                   "before the first frame");
  if (r->n_groups < 2 && !comm)
    return rv_set_error(RV_EINVAL, "rv_replay_set_la_exchange: rv_replay_set_groups first");
  RvLaEngine &E = *r->eng;
  const Geo &g = r->g;
  size_t most = 0;
  for (int j = 0; j < r->n_groups; j++) {
    int bx0, by0, bw, bh;
    impwin_group_blocks(r->grects[4 * j], r->grects[4 * j + 1], r->grects[4 * j + 2],
                        r->grects[4 * j + 3], g.w_imp, g.h_imp, bx0, by0, bw, bh);
    const size_t b = (size_t)bw * bh * kImpPartBytes;
    most = b > most ? b : most;
  }
  E.pbytes = (most + 255) / 256 * 256;
  if (comm) {
    E.psend = (uint8_t *)dalloc(r, E.pbytes);
    E.precv = (uint8_t *)dalloc(r, E.pbytes * (size_t)r->n_groups);
    if (!E.psend || !E.precv) return rv_set_error(RV_EHIP, "rv_replay_set_la_exchange: alloc");
    E.comm = comm;
    return RV_OK;
  }
  if (hub->n != r->n_groups)
    return rv_set_error(RV_EINVAL, "rv_replay_set_la_exchange: the hub's group count");
  const int k = r->my_group;
  std::lock_guard<std::mutex> lk(hub->mu);
  for (int s = 0; s < rv_la_hub::kRing; s++) {
    if (hub->buf[s][k]) return rv_set_error(RV_EINVAL, "rv_replay_set_la_exchange: group joined twice");
    hub->buf[s][k] = (uint8_t *)dalloc(r, E.pbytes);
    hipEvent_t ev = nullptr;
    RV_H(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    E.hub_ev.push_back(ev);
    hub->ev[s][k] = ev;
    if (!hub->buf[s][k]) return rv_set_error(RV_EHIP, "rv_replay_set_la_exchange: alloc");
  }
  E.hub = hub;
  E.hub_k = k;
  return RV_OK;
}

// The importances ([h_imp][w_imp] f32) the last coded frame's RDO used.
int rv_replay_get_importances(rv_replay *r, float *host, int n) {
  if (!r || !host || n != r->g.w_imp * r->g.h_imp)
    return rv_set_error(RV_EINVAL, "rv_replay_get_importances: bad arguments");
  RV_H(hipStreamSynchronize(r->stream));
  if (!r->imp_last) {
    memset(host, 0, (size_t)n * 4);
    return RV_OK;
  }
  RV_H(hipMemcpy(host, r->imp_last, (size_t)n * 4, hipMemcpyDeviceToHost));
  return RV_OK;
}

}  // extern "C"

extern "C" {

// Event layout per instrumented frame: e[0] start, e[1..13] after F0, F1,
// F2, FL (lookahead), F3 full-pel, F3 sub-pel, F4 single-reference
// candidates, F4 compound candidates, F4 argmin, F6 commit, F6b intra, F5,
// F7.
int rv_replay_frame(rv_replay *r, rv_replay_frame_info *info) {
  if (!r) return rv_set_error(RV_EINVAL, "rv_replay_frame: null");
  const Geo &g = r->g;
  hipStream_t st = r->stream;
  rv_replay_frame_info fi;
  frame_info(r->coded, g.R, &fi);
  if (fi.is_key) {
    // the key frame: its input is its reconstruction (intra coding is out
    // of scope); the pyramid of its input for the searches that reference it
    const RvInput &in = r->inputs[0];
    const RvSlot &s = r->slots[0];
    RV_H(hipMemcpyAsync(s.y.data, in.y.data, plane_bytes(in.y), hipMemcpyDeviceToDevice, st));
    RV_H(hipMemcpyAsync(s.u.data, in.u.data, plane_bytes(in.u), hipMemcpyDeviceToDevice, st));
    RV_H(hipMemcpyAsync(s.v.data, in.v.data, plane_bytes(in.v), hipMemcpyDeviceToDevice, st));
    if (!r->eng) {  // (the lookahead engine computes every pyramid itself)
      RV_R(rv_plane_pyramid(&in.y, &in.hres, &in.qres, st));
      if (r->sea) RV_R(rv_plane_box_sums(&in.qres, in.qres_box, st));
    }
    // an intra frame saves no motion: its frame_mvs stay zero
    RV_H(hipMemsetAsync(s.fmv, 0, (size_t)(g.w_in_b / 2) * (g.h_in_b / 2) * g.R * sizeof(rv_mv), st));
    r->coded++;
    r->last = fi;
    if (info) *info = fi;
    RV_H(hipGetLastError());
    return RV_OK;
  }
  if (!r->lv[0].set || !r->lv[1].set || !r->lv[2].set)
    return rv_set_error(RV_EINVAL, "rv_replay_frame: level params not set");
  // RAV1E_HIP_HOST_TRACE=1: the host's time per frame phase (stderr)
  static const bool host_trace = getenv("RAV1E_HIP_HOST_TRACE") != nullptr;
  using hclock = std::chrono::steady_clock;
  const auto h0 = hclock::now();
  auto h_take = h0, h_r0 = h0, h_mv = h0, h_intra = h0;
  auto us = [&](hclock::time_point a, hclock::time_point b) {
    return (long)std::chrono::duration_cast<std::chrono::microseconds>(b - a).count();
  };
  RV_R(ensure_jobs(r));
  const rv_replay::Level &L = r->lv[fi.level];
  const int lv = fi.level;
  CandGeo cg = r->cg;
  cg.comp = fi.compound ? kCompModes : 0;
  cg.stk = r->exact ? r->stk : nullptr;  // speed 10: rav1e's stacks (rv_mvref.hip)
  const RvInput &cur = r->inputs[fi.display % r->inputs.size()];
  const RvSlot &S = r->slots[fi.display % kSlots];
  const RvSlot *ref[2];
  rv_plane refs_y[RV_MAX_REFS], refs_h[RV_MAX_REFS], refs_q[RV_MAX_REFS];
  const uint32_t *box[RV_MAX_REFS];
  for (int k = 0; k < g.R; k++) {
    ref[k] = &r->slots[fi.ref_display[k] % kSlots];
    refs_y[k] = ref[k]->y;
    const RvInput &ri = r->inputs[fi.ref_display[k] % r->inputs.size()];
    refs_h[k] = ri.hres;
    refs_q[k] = ri.qres;
    box[k] = ri.qres_box;
  }
  const int nr = g.nsb;  // jobs per reference
  const long ncoded = r->coded - 1;  // non-key frames before this one
  const int slot = (int)(ncoded % rv_replay::kRing);
  uint32_t *ev_full = r->ds_evals + (size_t)slot * 2 * nr * g.R;
  uint32_t *ev_sub = ev_full + (size_t)nr * g.R;
  ChainNext to_sub{kChainFullToSub, r->jobs_sub[lv]};
  // the lookahead searches the references' original frames
  rv_plane refs_o[RV_MAX_REFS];
  for (int k = 0; k < g.R; k++) refs_o[k] = r->inputs[fi.ref_display[k] % r->inputs.size()].y;

  const bool tm = r->timing_stride > 0 && (ncoded / r->timing_block) % r->timing_stride == 0;
  hipEvent_t *e = r->evs[r->timed % rv_replay::kRing];
  if (tm) r->timed++;
#define RV_EV(i)                                   \
  do {                                             \
    if (tm) RV_H(hipEventRecord(e[i], st));        \
  } while (0)
  RV_EV(0);
  // the kernel probe's brackets around the F3 sub-pel launches (speed 10)
  const bool kp = tm && r->kprobe && !r->s6;
  uint32_t *kp_acc = kp ? r->kp_cnt[0] : nullptr;
  uint32_t *kp_f4 = kp ? r->kp_cnt[1] : nullptr;
  auto kp_open = [&](hipStream_t xs, int p = 0) -> int {
    if (!kp) return RV_OK;
    if (r->kp_n[p] >= r->kp_init[p]) {
      // the next kKpInit launches' device-clock span slots: start = max,
      // end = 0, in one or two copies; their previous pairs harvested first
      constexpr long K = rv_replay::kKp, C = rv_replay::kKpInit;
      static_assert(C <= K, "the initialised slots fit the ring");
      const long need = r->kp_n[p] + C - K;
      if (r->kp_done[p] < need) RV_H(kp_harvest(r, p, need));
      static const std::vector<unsigned long long> init = [] {
        std::vector<unsigned long long> v(2 * (size_t)C, 0ull);
        for (long i = 0; i < C; i++) v[2 * (size_t)i] = ~0ull;
        return v;
      }();
      const long s0 = r->kp_n[p] % K, first = std::min(C, K - s0);
      RV_H(hipMemcpyAsync(r->kp_ts[p] + 2 * s0, init.data(), 2 * sizeof(unsigned long long) * first,
                          hipMemcpyHostToDevice, xs));
      if (C > first)
        RV_H(hipMemcpyAsync(r->kp_ts[p], init.data(), 2 * sizeof(unsigned long long) * (C - first),
                            hipMemcpyHostToDevice, xs));
      r->kp_init[p] = r->kp_n[p] + C;
    }
    RV_H(hipEventRecord(r->kp_ev[p][2 * (size_t)(r->kp_n[p] % rv_replay::kKp)], xs));
    return RV_OK;
  };
  auto kp_ts = [&](int p = 0) -> unsigned long long * {
    return kp ? r->kp_ts[p] + 2 * (size_t)(r->kp_n[p] % rv_replay::kKp) : nullptr;
  };
  auto kp_close = [&](hipStream_t xs, int p = 0) -> int {
    if (!kp) return RV_OK;
    RV_H(hipEventRecord(r->kp_ev[p][2 * (size_t)(r->kp_n[p] % rv_replay::kKp) + 1], xs));
    r->kp_n[p]++;
    return RV_OK;
  };
  // F0 .. FL: the frame's lookahead (lookahead_frame), or with an importance
  // window the engine's, run W frames ahead, and the window's importances
  const float *imp = r->imp;
  if (r->eng) {
    RV_R(la_encode_exchange(r, r->coded, st));
    RV_R(la_engine_take(r, r->coded, st, &imp));
    if (tm)  // F0 .. FL ran on the engine: empty stages here
      for (int i : {1, 2, 3, rv_replay::kStageEv, rv_replay::kStageEv + 1})
        RV_H(hipEventRecord(e[i], st));
  } else {
    LaRefs er;  // without a window: the encode's references only
    memset(&er, 0, sizeof(er));
    er.n = g.R;
    for (int k = 0; k < g.R; k++) er.disp[k] = fi.ref_display[k], er.order[k] = k;
    RV_R(lookahead_frame(r, r->rr, st, fi, er, ncoded, LaOut{r->coarse, r->half_l, r->look}, r->la_list,
                         true, &r->la_round_sum, &r->la_reeval, tm ? e : nullptr));
    r->la_frames++;
  }
  r->imp_last = imp;
  h_take = hclock::now();
  auto rounds = [&](hipStream_t xs, int budget, auto &&check, auto &&eval, long *nrounds,
                    long *nre, bool *changed, const char *what) -> int {
    return run_rounds(r->rr, xs, budget, check, eval, nrounds, nre, changed, what, ncoded, lv);
  };
  auto slot_cnt = [&](uint32_t q) { return r->rr.slot(q); };
  // check q's list (two halves: an incremental check reads the previous one)
  auto mvl = [&](uint32_t q) { return r->mv_list + (size_t)(q & 1) * g.nsb; };
  const EpzsGeo eg{g.tx0, g.ty0, g.tw, g.th, g.tws, g.ths, g.W, g.H, g.w_in_b, g.h_in_b};
  // F5: the 8x8 importance SATD against reference 0's original frame at the
  // lookahead MVs (FL's output; after the frame's decisions)
  auto f5_importance = [&](hipStream_t fs) -> int {
    const unsigned nb = (unsigned)((r->n_imp + 255) / 256);
    if (g.hbd)
      importance_kernel<uint16_t><<<nb, 256, 0, fs>>>(g, cur.y, refs_o[0], r->look, r->imp_bx,
                                                      r->imp_by, r->tail + 2);
    else
      importance_kernel<uint8_t><<<nb, 256, 0, fs>>>(g, cur.y, refs_o[0], r->look, r->imp_bx,
                                                     r->imp_by, r->tail + 2);
    return RV_OK;
  };
  RV_EV(4);
  // An error return from here on must not leave the frame-edge levels (edge
  // streams) running: the next frame rewrites the MVs they read, and
  // rv_replay_destroy frees them.  Disarmed once the main stream has joined
  // them.
  struct SideJoin {
    rv_replay *r;
    bool armed;
    ~SideJoin() {
      for (int l = 1; l < kLevels; l++)
        if (armed && r->edge[l]) (void)hipStreamSynchronize(r->edge[l]);
    }
  } side_join{r, r->edge[1] != nullptr};
  // the candidates' RDO arguments: luma (N = 64, cdef distortion) and both
  // chroma planes (N = 32, SSE) of every candidate
  const int nsingle = g.nsb * g.R * g.M;
  RdoArgs la, ca;
  memset(&la, 0, sizeof(la));
  la.p[0].org = cur.y;
  for (int k = 0; k < g.R; k++) la.p[0].ref[k] = ref[k]->y;
  la.p[0].dst = S.y;
  la.p[0].levels = r->l_lev;
  la.p[0].out = r->l_out;
  la.g = cg;
  la.sub = r->sub;
  la.win = r->win;
  la.imp = imp;
  la.w_in_b = g.w_in_b;
  la.h_in_b = g.h_in_b;
  la.w_imp = g.w_imp;
  la.n_tx = nsingle;
  la.list = r->cand_list;
  la.count = r->cand_count;
  la.ntx_per_cand = 1;
  la.bd = g.bd;
  la.bsize = kSb;
  la.mb_w = la.mb_h = kSb;
  la.sub_w = la.sub_h = 8;
  la.p[0].q = L.ql;
  la.q_tx_index = 4 * 16 + 0;  // TX_64X64, DCT_DCT
  la.tx_size = 4;
  la.qindex = L.qidx;
  ca = la;
  const int ntx_c = r->ntx_c;
  const int64_t nct = (int64_t)g.nsb * g.C * ntx_c;  // output blocks per chroma plane
  const rv_plane cur_c[2] = {cur.u, cur.v}, s_c[2] = {S.u, S.v};
  for (int p = 0; p < 2; p++) {
    ca.p[p].org = cur_c[p];
    for (int k = 0; k < g.R; k++) ca.p[p].ref[k] = p ? ref[k]->v : ref[k]->u;
    ca.p[p].dst = s_c[p];
    ca.p[p].levels = r->c_lev + (size_t)p * g.nsb * ntx_c * 1024;
    ca.p[p].out = r->c_out + (size_t)p * nct * 3;
    ca.p[p].q = p ? L.qv : L.qu;
  }
  ca.n_tx = nsingle * ntx_c;
  ca.ntx_per_cand = ntx_c;
  ca.mb_w = g.cw;
  ca.mb_h = g.ch;
  ca.xdec = g.xdec;
  ca.ydec = g.ydec;
  ca.sub_w = (g.cw < 8 ? g.cw : 8) >> g.xdec;
  ca.sub_h = (g.ch < 8 ? g.ch : 8) >> g.ydec;
  ca.q_tx_index = 3 * 16 + 0;  // TX_32X32, DCT_DCT
  ca.tx_size = 3;

  // ---- the 32x32 .. 8x8 levels (speed 6: every block; speed 10: the frame-
  // edge rectangle), in pieces the schedule places: speed 6 interleaves them
  // with the 64x64 stages on the main stream, speed 10 runs them all on the
  // edge stream beside the 64x64 stages (levels with no leaf are skipped)
  RdoArgs ll[kLevels], lc6[kLevels];
  // motion_estimation of every block (sub-pel by SATD at speed 6,
  // use_satd_subpel, src/api/config.rs:429-431; SAD at speed 10), seeded with
  // the pmvs entry: a 32x32 its half-res quadrant search, a 16x16 / 8x8 its
  // 32x32's sub-pel winner
  auto lv_me = [&](hipStream_t es, int only = 0) -> int {
    for (int l = only ? only : 1; l < (only ? only + 1 : kLevels); l++) {
      if (!r->lv_me[l]) continue;
      rv_replay::PLevel &P = r->pl[l];
      if (l == 1)
        seed_level_kernel<<<(P.n * g.R + 255) / 256, 256, 0, es>>>(
            P.jobs_full[lv], P.n, P.gw, g.R, r->half_l, g.nsb, 0, 0, r->ex0, r->ey0, g.tw);
      else
        seed_level_kernel<<<(P.n * g.R + 255) / 256, 256, 0, es>>>(
            P.jobs_full[lv], P.n, P.gw, g.R, r->pl[1].sub, r->pl[1].n, r->pl[1].gw, 1 << (l - 1),
            0, 0, 0);
      ChainNext to_s{kChainFullToSub, P.jobs_sub[lv]};
      RV_R(rv_diamond_search_multi(&cur.y, refs_y, g.R, P.jobs_full[lv], P.n, P.B, P.B, 0, 0, 0,
                                   g.bd, P.full, nullptr, &to_s, es));
      RV_R(rv_diamond_search_multi(&cur.y, refs_y, g.R, P.jobs_sub[lv], P.n, P.B, P.B, 1,
                                   r->s6 ? 1 : 0, 0, g.bd, P.sub, nullptr, nullptr, es));
    }
    return RV_OK;
  };
  // the candidate lists of every used level (single, then compound)
  auto lv_lists = [&](hipStream_t es, bool comp, int only = 0) {
    for (int l = only ? only : 1; l < (only ? only + 1 : kLevels); l++) {
      if (!r->lv_used[l]) continue;
      rv_replay::PLevel &P = r->pl[l];
      const int ns = P.n * g.R * g.M;
      if (!comp) {
        cand_list_kernel<<<(ns + 255) / 256, 256, 0, es>>>(P.cg, P.sub, ns, P.cand_list,
                                                            P.cand_count);
      } else {
        CandGeo cgl = P.cg;
        cgl.comp = cg.comp;
        comp_list_kernel<<<(P.n * cg.comp + 255) / 256, 256, 0, es>>>(
            cgl, P.sub, ns, P.cand_list + ns, P.cand_count + 1);
      }
    }
  };
  // the single-reference candidates of every used level: luma (cdef
  // distortion) and chroma launches
  auto lv_rdo = [&](hipStream_t es, int only = 0) -> int {
    for (int l = only ? only : 1; l < (only ? only + 1 : kLevels); l++) {
      if (!r->lv_used[l]) continue;
      rv_replay::PLevel &P = r->pl[l];
      CandGeo cgl = P.cg;
      cgl.comp = cg.comp;
      const int ns = P.n * g.R * g.M;
      RdoArgs a = la;
      a.p[0].levels = P.l_lev;
      a.p[0].out = P.l_out;
      a.p[0].q = L.qs[l][0];
      a.g = cgl;
      a.sub = P.sub;
      a.win = P.win;
      a.n_tx = ns;
      a.list = P.cand_list;
      a.count = P.cand_count;
      a.ntx_per_cand = 1;
      a.bsize = P.B;
      a.mb_w = a.mb_h = P.B;
      a.q_tx_index = P.txl * 16;  // DCT_DCT
      a.tx_size = P.txl;
      RdoArgs c = ca;
      for (int q = 0; q < 2; q++) {
        c.p[q].levels = P.c_lev + (size_t)q * P.n * P.bc * P.bch;
        c.p[q].out = P.c_out + (size_t)q * P.n * g.C * 3;
        c.p[q].q = L.qs[l][1 + q];
      }
      c.g = cgl;
      c.sub = P.sub;
      c.win = P.win;
      c.n_tx = ns;
      c.list = P.cand_list;
      c.count = P.cand_count;
      c.ntx_per_cand = 1;
      c.bsize = P.B;
      c.mb_w = P.bc;
      c.mb_h = P.bch;
      c.sub_w = (P.bc < 8 ? P.bc : 8) >> g.xdec;   // sse_wxh's importance blocks
      c.sub_h = (P.bch < 8 ? P.bch : 8) >> g.ydec;
      c.q_tx_index = P.txc * 16;
      c.tx_size = P.txc;
      ll[l] = a;
      lc6[l] = c;
      RV_R(rv_rdo_blocks2(a, c, P.B, P.bc, g.hbd, es, 0));
    }
    return RV_OK;
  };
  // the compound candidates of every used level (all pushed)
  auto lv_rdo_comp = [&](hipStream_t es, int only = 0) -> int {
    for (int l = only ? only : 1; l < (only ? only + 1 : kLevels); l++) {
      if (!r->lv_used[l]) continue;
      const rv_replay::PLevel &P = r->pl[l];
      RdoArgs a = ll[l], c = lc6[l];
      a.list = c.list = P.cand_list + P.n * g.R * g.M;
      a.count = c.count = P.cand_count + 1;
      a.cand_base = c.cand_base = 0;
      a.n_tx = c.n_tx = P.n * cg.comp;
      RV_R(rv_rdo_blocks2(a, c, P.B, P.bc, g.hbd, es, 1));
    }
    return RV_OK;
  };
  // every used level's winners and result words
  auto lv_score = [&](hipStream_t es, int only = 0) {
    for (int l = only ? only : 1; l < (only ? only + 1 : kLevels); l++) {
      if (!r->lv_used[l]) continue;
      rv_replay::PLevel &P = r->pl[l];
      CandGeo cgl = P.cg;
      cgl.comp = cg.comp;
      score_level<<<(P.n + 63) / 64, 64, 0, es>>>(cgl, L.lambda, L.ds[1], L.ds[2], P.full, P.sub,
                                                  P.l_out, P.c_out, P.c_out + (size_t)P.n * g.C * 3,
                                                  P.win, r->words + P.woff, P.cand_count,
                                                  r->cand_evals + 2 * (slot * kLevels + l));
    }
  };
  // the leaves of every used level into the frame
  auto lv_commit = [&](hipStream_t es, int only = 0) -> int {
    for (int l = only ? only : 1; l < (only ? only + 1 : kLevels); l++) {
      if (!r->lv_used[l]) continue;
      const rv_replay::PLevel &P = r->pl[l];
      RdoArgs a = ll[l], c = lc6[l];
      a.commit = c.commit = 1;
      a.list = c.list = P.leaf;
      a.count = c.count = r->leaf_count + l;
      a.n_tx = c.n_tx = P.n;
      RV_R(rv_rdo_blocks2(a, c, P.B, P.bc, g.hbd, es, 2));
    }
    return RV_OK;
  };
  // speed 10: the edge levels on their own stream, forked after F2
  // one stream per level: the 32x32 searches first (the smaller levels seed
  // from them), then each level's candidates and scores beside the others'
  const bool edge = r->lvl && !r->s6 && r->edge[1];
  if (edge) {
    RV_H(hipEventRecord(r->ev_efork, st));
    for (int l = 1; l < kLevels; l++) RV_H(hipStreamWaitEvent(r->edge[l], r->ev_efork, 0));
    if (tm) RV_H(hipEventRecord(e[rv_replay::kStageEv + 2], r->edge[1]));
    RV_R(lv_me(r->edge[1], 1));
    RV_H(hipEventRecord(r->ev_l1me, r->edge[1]));
    for (int l = 1; l < kLevels; l++) {
      hipStream_t es = r->edge[l];
      if (l > 1 && r->lv_me[l]) {
        RV_H(hipStreamWaitEvent(es, r->ev_l1me, 0));
        RV_R(lv_me(es, l));
      }
      if (!r->lv_used[l]) continue;
      lv_lists(es, false, l);
      if (cg.comp) lv_lists(es, true, l);
      RV_R(lv_rdo(es, l));
      if (cg.comp) RV_R(lv_rdo_comp(es, l));
      lv_score(es, l);
      RV_H(hipEventRecord(r->ev_ejoin[l], es));
    }
    for (int l = 2; l < kLevels; l++)
      if (r->lv_used[l]) RV_H(hipStreamWaitEvent(r->edge[1], r->ev_ejoin[l], 0));
    if (tm) RV_H(hipEventRecord(e[rv_replay::kStageEv + 3], r->edge[1]));
  } else if (tm) {  // no edge stream: an empty span
    RV_H(hipEventRecord(e[rv_replay::kStageEv + 2], st));
    RV_H(hipEventRecord(e[rv_replay::kStageEv + 3], st));
  }

  // speed 10: the levels' work (edge rectangle) does not depend on the
  // superblocks' and, without edge streams, runs first: the stack rounds may
  // read their leaves (a top-right neighbour past the right frame edge)
  const bool lv_early = r->exact && r->lvl && !edge;
  if (lv_early) {
    RV_R(lv_me(st));
    lv_lists(st, false);
    if (cg.comp) lv_lists(st, true);
    RV_R(lv_rdo(st));
    if (cg.comp) RV_R(lv_rdo_comp(st));
    lv_score(st);
  }
  // speed 10: rav1e's MV stacks in coding-order rounds (rv_mvref.hip): round
  // 0 evaluates every superblock with the stacks of this level's previous
  // frame's decisions (a guess), each later round re-evaluates the
  // superblocks whose stacks changed, until none does
  MvrefArgs ma;
  memset(&ma, 0, sizeof(ma));
  if (r->exact) {
    ma.nsb = g.nsb;
    ma.tw = g.tw;
    ma.th = g.th;
    ma.tx0 = g.tx0;
    ma.ty0 = g.ty0;
    ma.tws = g.tws;
    ma.ths = g.ths;
    ma.W = g.W;
    ma.H = g.H;
    ma.w_in_b = g.w_in_b;
    ma.h_in_b = g.h_in_b;
    ma.R = g.R;
    ma.comp = cg.comp ? 1 : 0;
    for (int k = 0; k < g.R; k++) ma.sign_bias |= (uint32_t)(fi.ref_display[k] > fi.display) << k;
    ma.dec = r->dec_lv[lv];
    ma.stk = r->stk;
    ma.active = r->mv_active;
    ma.count = r->rr.cnt;
    ma.jf = r->jobs_full[lv];
    ma.js = r->jobs_sub[lv];
    ma.init = 1;
    ma.lvl = r->lvl ? 1 : 0;
    if (r->lvl)
      for (int l = 1; l < kLevels; l++)
        if (r->lv_used[l]) {
          ma.lwin[l] = r->pl[l].win;
          ma.lsub[l] = r->pl[l].sub;
          ma.lcg[l] = r->pl[l].cg;
        }
    if (edge && r->edge_tr)  // the leaves the stacks read
      for (int l = 1; l < kLevels; l++)
        if (r->lv_used[l]) RV_H(hipStreamWaitEvent(st, r->ev_ejoin[l], 0));
    // EPZS: the F2 / F3 sets from the coding-order field; the first check
    // guesses it from the previous decisions of this level and the
    // lookahead's quadrants, and never reads the frame-edge leaves (they may
    // be in flight)
    ma.epzs = 1;
    ma.eg = eg;
    ma.jh = r->jobs_half[lv];
    ma.coarse = r->coarse;
    ma.hq = r->half_l;
    ma.prev = r->slots[fi.ref_display[0] % kSlots].fmv;  // the LAST reference's frame_mvs
    ma.edge_ok = 0;
    ma.f3dirty = r->cand_reuse ? r->f3dirty : nullptr;
    static const bool gla = getenv("RAV1E_HIP_GUESS_LA") && getenv("RAV1E_HIP_GUESS_LA")[0] == '1';
    ma.field_guess_la = gla ? 1 : 0;
    static const bool f2d = !(getenv("RAV1E_HIP_F2_DIRTY") && getenv("RAV1E_HIP_F2_DIRTY")[0] == '0');
    ma.f2dirty = r->cand_reuse && f2d ? r->f2dirty : nullptr;
    // the first check marks every superblock (its count is not read)
    const uint32_t q = r->rr.seq++;
    ma.count = slot_cnt(q);
    ma.pub = r->rr.pub(q);
    ma.list = mvl(q);
    ma.plist = nullptr;
    RV_R(rv_mvref_round(ma, st));
  }
  // F2: build_half_res_pmvs of the encode (speed 10: the sets the check
  // stored; otherwise the lookahead's quadrants stand in) and the F3
  // full-pel predictors (otherwise zero + the coarse MV)
  if (r->exact) {
    RV_R(rv_diamond_search_multi(&cur.hres, refs_h, g.R, r->jobs_half[lv], nr * 4, 16, 16, 0, 0, 0,
                                 g.bd, r->half, nullptr, nullptr, st));
  } else {
    RV_H(hipMemcpyAsync(r->half, r->half_l, (size_t)nr * g.R * 4 * sizeof(rv_fs_result),
                        hipMemcpyDeviceToDevice, st));
    fill_preds_kernel<<<(nr * g.R + 255) / 256, 256, 0, st>>>(r->jobs_full[lv], r->src_full,
                                                              nr * g.R, r->coarse, r->half, 0);
  }
  const uint8_t *act = r->exact ? r->mv_active : nullptr;
  // F4's arguments (la / ca become F6's commit arguments below; the rounds
  // after the intra pass evaluate candidates again)
  const RdoArgs la4 = la, ca4 = ca;
  // the compound sets (all pushed; distinct MV pairs from the list) and the
  // list launches' arguments in device memory: [la4, ca4, lc4, cc4]
  RdoArgs lc4 = la4, cc4 = ca4;
  lc4.list = cc4.list = r->cand_list + nsingle;
  lc4.count = cc4.count = r->cand_count + 1;
  lc4.cand_base = cc4.cand_base = 0;
  lc4.n_tx = g.nsb * cg.comp;
  cc4.n_tx = g.nsb * cg.comp * ntx_c;
  const RdoArgs f4h[4] = {la4, ca4, lc4, cc4};
  // RAV1E_HIP_F4_LIST=0: the full-grid launches (A/B); 12-bit keeps them
  static const bool f4_list_env = !(getenv("RAV1E_HIP_F4_LIST") && getenv("RAV1E_HIP_F4_LIST")[0] == '0');
  const bool f4_list = f4_list_env && g.bd != 12;
  if (f4_list) RV_R(rv_rdo_args_put(f4h, cg.comp ? 4 : 2, r->f4_args, st));
  // F3 full-res full-pel diamond -> sub-pel predictor; sub-pel diamond
  // (speed 10: SAD, no hp) -> NEWMV of every superblock and reference;
  // the candidates; F4; the argmin.  Round 0: every superblock, full grids.
  auto f3_f4 = [&]() -> int {
    RV_R(rv_diamond_search_multi(&cur.y, refs_y, g.R, r->jobs_full[lv], nr, 64, 64, 0, 0, 0, g.bd,
                                 r->full, ev_full, &to_sub, st, act));
    RV_EV(5);
    RV_R(kp_open(st));
    RV_R(rv_diamond_search_multi(&cur.y, refs_y, g.R, r->jobs_sub[lv], nr, 64, 64, 1,
                                 r->s6 ? 1 : 0, 0, g.bd, r->sub, ev_sub, nullptr, st, act, nullptr,
                                 nullptr, 1, nullptr, 0, kp_acc, kp_ts()));
    RV_R(kp_close(st));
    if (r->lvl && !edge && !lv_early) RV_R(lv_me(st));
    // the valid candidates (a few microseconds; bracketed with F3 sub-pel;
    // the count was zeroed by the previous argmin or at creation)
    const CandKeys keys0{r->cand_key, (uint32_t)(r->coded + 1), 0};
    cand_list_kernel<<<(nsingle + 255) / 256, 256, 0, st>>>(cg, r->sub, nsingle, r->cand_list,
                                                            r->cand_count, act, keys0);
    if (r->lvl && !edge && !lv_early) lv_lists(st, false);
    if (cg.comp) {  // the compound lists (after the single ones in the same arrays)
      comp_list_kernel<<<(g.nsb * cg.comp + 255) / 256, 256, 0, st>>>(
          cg, r->sub, nsingle, r->cand_list + nsingle, r->cand_count + 1, act, keys0);
      if (r->lvl && !edge && !lv_early) lv_lists(st, true);
    }
    RV_EV(6);
    // F4 every valid candidate, luma + both chroma planes in one fused launch
    if (f4_list) {
      RV_R(kp_open(st, 1));
      RV_R(rv_rdo_candidates_list(f4h, r->f4_args, 1, 0, g.hbd, st, 0, kp_f4, kp_ts(1)));
      RV_R(kp_close(st, 1));
    } else
      RV_R(rv_rdo_candidates(la4, ca4, g.hbd, st));
    if (r->lvl && !edge && !lv_early) RV_R(lv_rdo(st));
    if (cg.comp) {  // the compound candidates (all pushed), distinct MV pairs from the list
      RV_EV(7);
      if (f4_list) {
        RV_R(kp_open(st, 1));
        RV_R(rv_rdo_candidates_list(f4h + 2, r->f4_args + 2, 1, 1, g.hbd, st, 0, kp_f4, kp_ts(1)));
        RV_R(kp_close(st, 1));
      } else
        RV_R(rv_rdo_candidates(lc4, cc4, g.hbd, st, true));
      if (r->lvl && !edge && !lv_early) RV_R(lv_rdo_comp(st));
    } else {
      RV_EV(7);
    }
    RV_EV(8);
    score_wave_kernel<<<(g.nsb + 3) / 4, 256, 0, st>>>(
        g, cg, L.lambda, L.ds[1], L.ds[2], r->sub, r->l_out, r->c_out, r->c_out + nct * 3, ntx_c,
        r->win, r->coarse, r->half, r->full, r->look, r->half_l, r->words, r->cand_count,
        r->tail + 2, r->cand_evals + 2 * slot * kLevels, r->leaf_count, nullptr, nullptr,
        r->exact ? r->dec_lv[lv] : nullptr, 0);
    return RV_OK;
  };
  // A later round: the same stages over the superblocks check q listed
  // (r->mv_list, its count in the ring), each launch a fixed pool of
  // workgroups that loops over the device count -- a round of a few dozen
  // superblocks costs their latency, not a full grid of early exits.
  // the first round of a run lists most superblocks (check 1 after round 0:
  // 70-80 % at 2160p): its searches take full grids, later ones the pool
  uint32_t q_first = 0;
  // RAV1E_HIP_F4_PAIR=0: the rounds' single and compound F4 in two launches (A/B)
  static const bool f4_pair = !(getenv("RAV1E_HIP_F4_PAIR") && getenv("RAV1E_HIP_F4_PAIR")[0] == '0');
  // RAV1E_HIP_F2_F3=0: the rounds' F2 and F3 full-pel searches in two launches (A/B)
  static const bool f2_f3 = !(getenv("RAV1E_HIP_F2_F3") && getenv("RAV1E_HIP_F2_F3")[0] == '0');
  // RAV1E_HIP_F3_FUSE=0: the rounds' F3 sub-pel searches in a launch of their
  // own after F2 || F3 full-pel (A/B); fused, each F3 workgroup runs its
  // job's sub-pel search right after the full-pel one
  static const bool f3_fuse = !(getenv("RAV1E_HIP_F3_FUSE") && getenv("RAV1E_HIP_F3_FUSE")[0] == '0');
  auto f3_f4_list = [&](hipStream_t xs, uint32_t q) -> int {
    const int32_t *acnt = slot_cnt(q);
    int lg = q == q_first ? nr * g.R : 0;
    // A later round's grids from the last count the host read (a check one
    // or two rounds back): twice that many superblocks, so the launches
    // carry the live work and few empty workgroups (a round's fixed pools
    // put ~12 k waves through the dispatcher for a few dozen superblocks).
    // A list longer than the hint loops over the grid, so the hint only
    // sizes, never decides.  RAV1E_HIP_ROUND_HINT=0: the fixed pools (A/B).
    static const bool round_hint = !(getenv("RAV1E_HIP_ROUND_HINT") && getenv("RAV1E_HIP_ROUND_HINT")[0] == '0');
    const int hint = q == q_first || !round_hint ? -1 : r->rr.last_count;
    const int hsb = hint >= 0 ? std::max(2 * hint, 16) : 0;
    int f4_grid = 0;
    if (hsb) {
      lg = std::min(hsb * g.R, 512);
      f4_grid = std::min(6 * hsb, 1024);
    }
    // the check's F2 / F3 sets came from the state before this round, so F2
    // and F3 are independent (F2's results feed the next check): F2 on the
    // second stream
    hipStream_t x2 = r->rs2 ? r->rs2 : xs;
    if (r->rs2) {
      RV_H(hipEventRecord(r->ev_rfork, xs));
      RV_H(hipStreamWaitEvent(x2, r->ev_rfork, 0));
    }
    const bool fused = f2_f3 && f3_fuse && !r->rs2 && !r->s6;
    if (f2_f3 && !r->rs2) {  // F2 and F3 full-pel (+ F3 sub-pel when fused) in one launch
      // fused: the probe brackets the launch (its sub-pel candidates, its span)
      if (fused) RV_R(kp_open(xs));
      RV_R(rv_diamond_f2_f3(&cur.hres, refs_h, r->jobs_half[lv], r->half, ma.f2dirty, &cur.y,
                            refs_y, r->jobs_full[lv], r->full, ma.f3dirty, &to_sub, g.R, nr, g.bd,
                            mvl(q), acnt, lg, xs, fused ? r->jobs_sub[lv] : nullptr,
                            fused ? r->sub : nullptr, fused ? kp_acc : nullptr,
                            fused ? kp_ts() : nullptr));
      if (fused) RV_R(kp_close(xs));
    } else {
      // F2 of the listed superblocks (their 4 quadrants per reference)
      RV_R(rv_diamond_search_multi(&cur.hres, refs_h, g.R, r->jobs_half[lv], nr * 4, 16, 16, 0, 0,
                                   0, g.bd, r->half, nullptr, nullptr, x2, nullptr, mvl(q),
                                   acnt, 4, ma.f2dirty, lg));
      // F3 of the listed superblocks: only the jobs whose set or pmv changed
      RV_R(rv_diamond_search_multi(&cur.y, refs_y, g.R, r->jobs_full[lv], nr, 64, 64, 0, 0, 0,
                                   g.bd, r->full, nullptr, &to_sub, xs, nullptr, mvl(q), acnt,
                                   1, ma.f3dirty, lg));
    }
    if (!fused) {
      RV_R(kp_open(xs));
      RV_R(rv_diamond_search_multi(&cur.y, refs_y, g.R, r->jobs_sub[lv], nr, 64, 64, 1, 0, 0, g.bd,
                                   r->sub, nullptr, nullptr, xs, nullptr, mvl(q), acnt, 1,
                                   ma.f3dirty, lg, kp_acc, kp_ts()));
      RV_R(kp_close(xs));
    }
    // the pools of the small per-round kernels: kRoundGrid for a run's first
    // round (most superblocks listed), RAV1E_HIP_ROUND_POOL (A/B) after it
    static const int round_pool = getenv("RAV1E_HIP_ROUND_POOL") ? std::max(1, atoi(getenv("RAV1E_HIP_ROUND_POOL")))
                                                                 : kRoundGrid;
    const int rg = q == q_first ? kRoundGrid
                   : hsb ? std::min(kRoundGrid, std::max((14 * hsb + 255) / 256, (hsb + 3) / 4))
                         : round_pool;
    round_lists_kernel<<<rg, 256, 0, xs>>>(
        cg, r->sub, nsingle, r->cand_list, r->cand_count, mvl(q), acnt,
        CandKeys{r->cand_key, (uint32_t)(r->coded + 1), r->cand_reuse ? 1 : 0});
    if (r->rs2) {  // the lists are out: the compound F4 runs beside the single one
      RV_H(hipEventRecord(r->ev_rlists, xs));
      RV_H(hipStreamWaitEvent(x2, r->ev_rlists, 0));
    }
    // F4: a pool of workgroups over the live list entries (rdo_quad_list_kernel;
    // RAV1E_HIP_F4_LIST=0: full grids whose workgroups past the device counts
    // exit at once); on a compound frame the single and compound candidates
    // in one launch
    if (cg.comp) {
      if (f4_list && f4_pair && !r->rs2) {  // the pool over both lists
        RV_R(kp_open(xs, 1));
        RV_R(rv_rdo_candidates_list(f4h, r->f4_args, 2, 0, g.hbd, xs, f4_grid, kp_f4, kp_ts(1)));
        RV_R(kp_close(xs, 1));
      } else if (f4_pair && !r->rs2) {
        RV_R(rv_rdo_candidates_pair(la4, ca4, lc4, cc4, g.hbd, xs));
      } else {
        RV_R(rv_rdo_candidates(la4, ca4, g.hbd, xs));
        RV_R(rv_rdo_candidates(lc4, cc4, g.hbd, x2, true));
      }
    } else if (f4_list) {
      RV_R(kp_open(xs, 1));
      RV_R(rv_rdo_candidates_list(f4h, r->f4_args, 1, 0, g.hbd, xs, f4_grid, kp_f4, kp_ts(1)));
      RV_R(kp_close(xs, 1));
    } else {
      RV_R(rv_rdo_candidates(la4, ca4, g.hbd, xs));
    }
    if (r->rs2) {  // F2 and the compound F4 join before the argmin
      RV_H(hipEventRecord(r->ev_rjoin, x2));
      RV_H(hipStreamWaitEvent(xs, r->ev_rjoin, 0));
    }
    score_wave_kernel<<<rg, 256, 0, xs>>>(
        g, cg, L.lambda, L.ds[1], L.ds[2], r->sub, r->l_out, r->c_out, r->c_out + nct * 3, ntx_c,
        r->win, r->coarse, r->half, r->full, r->look, r->half_l, r->words, r->cand_count, nullptr,
        nullptr, nullptr, mvl(q), acnt, r->dec_lv[lv], 1);
    return RV_OK;
  };
  RV_R(f3_f4());
  // The MV-stack rounds after the first (`rounds` above): a check
  // recomputes every superblock's stacks and F2 / F3 EPZS sets from the
  // decisions and results so far and lists the superblocks where one
  // changed; the round re-runs their F2, F3, candidates, F4 and argmin.
  //
  // Termination: within a tile a superblock's stacks read its
  // left, top-left, top and top-right neighbours, and its EPZS sets read
  // fields of its left and top neighbours, so its dependency depth is at
  // most x + 2 y <= (tws - 1) + 2 (ths - 1).  A superblock of depth d is
  // settled (evaluated with its final inputs) after evaluation round d + 1:
  // its predecessors are settled after round d, so check d + 1 gives its
  // final inputs.  Hence every run ends by evaluation round tws + 2 ths - 2
  // and the check after it lists nothing; that is the budget, per run.
  //
  // Returns with *changed = some round evaluated.
  const int budget = g.tws + 2 * g.ths - 2;
  int mv_runs = 0;
  auto mv_rounds_run = [&](const uint8_t *iwas, bool *changed) -> int {
    mv_runs++;
    hipStream_t xs = r->hp ? r->hp : st;
    // the rounds follow the main stream's work and it waits for them
    struct Join {
      rv_replay *r;
      hipStream_t st;
      ~Join() {
        if (r->hp && hipEventRecord(r->ev_hp1, r->hp) == hipSuccess)
          (void)hipStreamWaitEvent(st, r->ev_hp1, 0);
      }
    } join{r, st};
    if (r->hp) {
      RV_H(hipEventRecord(r->ev_hp0, st));
      RV_H(hipStreamWaitEvent(r->hp, r->ev_hp0, 0));
    }
    q_first = r->rr.seq;  // run_rounds' first check (its list: the first round)
    // Long chains (a change running down a tile's columns, one superblock
    // row per Jacobi round: compound frames reach ~70 rounds at 2160p): from
    // check kScanAfter on, up to kScanMax checks are the predictive scan
    // (mvref_scan_kernel), which lets a chain run down in one round when the
    // predicted decisions hold.  The Jacobi bound still holds after them, so
    // the run's budget grows by kScanMax.
    static const int scan_after = getenv("RAV1E_HIP_MV_SCAN_AFTER")
                                      ? atoi(getenv("RAV1E_HIP_MV_SCAN_AFTER")) : 0;
    constexpr int kScanMax = 8;
    const bool scans = scan_after > 0;
    return rounds(
        xs, budget + (scans ? kScanMax : 0),
        [&](uint32_t q) {
          ma.init = 0;
          ma.iwas = iwas;
          ma.count = slot_cnt(q);
          ma.pub = r->rr.pub(q);
          ma.list = mvl(q);
          // RAV1E_HIP_CHECK_INC=1 (A/B, off: DESIGN.md §8): from the run's
          // third check on, each check covers only the dependents of the
          // previous check's list.  The second check follows the run's
          // first round, which lists most superblocks: it stays full (their
          // dependents, 4 per listed superblock, would take the incremental
          // kernel several passes).  The incremental grid is the full
          // check's: a short list leaves most workgroups empty, which exit
          // at once, and a long one never loops.
          static const bool inc = getenv("RAV1E_HIP_CHECK_INC") && getenv("RAV1E_HIP_CHECK_INC")[0] == '1';
          if (inc && q > q_first + 1) {
            ma.plist = mvl(q - 1);
            ma.pcount = slot_cnt(q - 1);
            ma.epoch = r->mv_epoch;
            ma.tag = q + 1;
            ma.inc_grid = 0;
          } else {
            ma.plist = nullptr;
          }
          const uint32_t c = q - q_first;
          return rv_mvref_round(ma, xs, scans && c >= (uint32_t)scan_after &&
                                            c < (uint32_t)(scan_after + kScanMax));
        },
        [&](uint32_t q) { return f3_f4_list(xs, q); }, &r->mv_round_sum, &r->mv_reeval, changed,
        "mvref");
  };
  if (r->exact) {
    // from here on the checks read the frame-edge leaves (the EPZS field of
    // the edge superblocks) and the encode's own F2 results
    if (edge)
      for (int l = 1; l < kLevels; l++)
        if (r->lv_used[l]) RV_H(hipStreamWaitEvent(st, r->ev_ejoin[l], 0));
    ma.hq = r->half;
    ma.edge_ok = 1;
    h_r0 = hclock::now();
    RV_R(mv_rounds_run(nullptr, nullptr));
    h_mv = hclock::now();
  }
  if (r->lvl) {
    if (edge) {  // the levels' winners
      for (int l = 1; l < kLevels; l++)
        if (r->lv_used[l]) RV_H(hipStreamWaitEvent(st, r->ev_ejoin[l], 0));
    } else if (!lv_early) {
      lv_score(st);
    }
    PartArgs pa;
    memset(&pa, 0, sizeof(pa));
    for (int l = 0; l < kLevels; l++) {
      rv_replay::PLevel &P = r->pl[l];
      pa.win[l] = l ? P.win : r->win;
      pa.gw[l] = P.gw;
      pa.x0[l] = (g.tx0 + (l ? r->ex0 : 0)) * kSb;
      pa.y0[l] = (g.ty0 + (l ? r->ey0 : 0)) * kSb;
      pa.leaf[l] = P.leaf;
    }
    pa.ex0 = r->ex0;
    pa.ey0 = r->ey0;
    pa.ew = r->ew;
    pa.eh = r->eh;
    pa.forced = !r->s6;
    pa.leaf_count = r->leaf_count;
    pa.words = r->words + r->wpart;
    partition_kernel<<<(g.nsb + 63) / 64, 64, 0, st>>>(g, pa);
  }
  if (r->intra) RV_R(intra_begin(r));
  RV_EV(9);
  // the previous frame's F8 still reads the committed levels and the block map
  if (r->f8_pending) {
    RV_H(hipStreamWaitEvent(st, r->ev_f8done, 0));
    r->f8_pending = false;
  }
  // F6 commit the winners into the frame: the levels' leaves (speed 10: on
  // the edge stream, beside the superblocks' commit)
  if (edge) {
    RV_H(hipEventRecord(r->ev_epart, st));
    for (int l = 1; l < kLevels; l++) {
      if (!r->lv_used[l]) continue;
      RV_H(hipStreamWaitEvent(r->edge[l], r->ev_epart, 0));
      RV_R(lv_commit(r->edge[l], l));
      RV_H(hipEventRecord(r->ev_ecommit[l], r->edge[l]));
    }
  }
  la.commit = ca.commit = 1;
  la.list = ca.list = r->lvl ? r->pl[0].leaf : nullptr;  // with levels: the unsplit superblocks
  la.count = ca.count = r->lvl ? r->leaf_count : nullptr;
  la.n_tx = g.nsb;
  ca.n_tx = g.nsb * ntx_c;
  la.ntx_per_cand = 1;
  RV_R(rv_rdo_candidates(la, ca, g.hbd, st));
  if (r->lvl && !edge) RV_R(lv_commit(st));
  for (int l = 1; edge && l < kLevels; l++)
    if (r->lv_used[l]) RV_H(hipStreamWaitEvent(st, r->ev_ecommit[l], 0));
  side_join.armed = false;  // both side streams have joined the main one
  RV_EV(10);
  // F6b intra-mode screening + intra RDO of the non-skip superblocks
  int irounds = 0;
  if (r->intra) RV_R(intra_pass(r, la, ca, cur, S, L, slot, &irounds));
  h_intra = hclock::now();
  // an intra winner is no MV source (add_ref_mv_candidate skips intra
  // blocks): the superblocks whose stacks it changes are re-decided, the
  // frame re-committed and the intra pass re-run, until the stacks hold
  // (the joint fixed point of the tile's coding order)
  // Bound: each pass settles at least the next superblock of every tile's
  // raster order (its predecessors' decisions, intra flags and
  // reconstruction are final, so its stacks, inter winner and intra
  // decision are too), so tws * ths passes always suffice.
  for (int pass = 0; r->exact && r->intra; pass++) {
    if (pass > g.tws * g.ths)
      return rv_set_error(RV_EHIP, "rv_replay_frame: the MV / intra passes did not settle "
                                   "(internal error)");
    // no screened superblock (no intra round): no superblock is intra, the
    // stacks are the ones the MV rounds settled -- the check would list
    // nothing (only after the first pass: later ones follow a run whose
    // stacks saw intra blocks)
    if (pass == 0 && irounds == 0) break;
    bool changed = false;
    RV_R(mv_rounds_run(r->i_was, &changed));
    if (!changed) break;
    RV_R(rv_rdo_candidates(la, ca, g.hbd, st));  // F6 again: every inter winner
    RV_R(intra_begin(r));
    RV_R(intra_pass(r, la, ca, cur, S, L, slot, &irounds));
  }
  if (r->exact) {
    r->mv_round_sum++;  // round 0
    r->mv_run_sum += mv_runs;
    r->mv_frames++;
    // the encode's field becomes the frame's frame_mvs (the group's part;
    // the other groups' arrive with the exchange)
    ma.iwas = r->intra ? r->i_was : nullptr;
    RV_R(rv_mvref_field(ma, S.fmv, st));
  }
  RV_EV(11);
  // F5 importance SATD against reference 0 (the sum was zeroed by the argmin;
  // with the side stream F5 ran there, after the lookahead)
  RV_R(f5_importance(st));
  RV_EV(12);
  // F7 deblock_filter_frame (src/encoder.rs:2789-2793) when enabled: the
  // block map of the committed blocks, then (once every group's pixels and
  // map are in) Y, U, V in place; the reconstruction becomes a reference
  if (r->deblock || r->entropy) {
    if (!r->lvl) {
      block_map_kernel<<<(g.nsb * 16 + 255) / 256, 256, 0, st>>>(
          nullptr, nullptr, g.nsb, g.tw, g.tx0, g.ty0, 0, r->win, r->mi_lg, r->mi_skip,
          r->mi_stride, r->mi_cols, r->mi_rows);
    } else {
      for (int l = 0; l < kLevels; l++) {
        const rv_replay::PLevel &P = r->pl[l];
        const int n4 = 16 >> l;
        block_map_kernel<<<(P.n * n4 + 255) / 256, 256, 0, st>>>(
            P.leaf, r->leaf_count + l, P.n, P.gw, l ? P.cg.tx0 : g.tx0, l ? P.cg.ty0 : g.ty0, l,
            l ? P.win : r->win, r->mi_lg, r->mi_skip, r->mi_stride, r->mi_cols, r->mi_rows);
      }
    }
  }
  // F8 (RV_REPLAY_ENTROPY): the committed transform blocks' symbols, in
  // coding order, into a host-mapped ring slot; the host thread range-codes
  // them beside the next frames
  if (r->entropy) {
    EcHost *eh = r->ech;
    const int slot = (int)(r->ec_frames & 1);
    {
      std::unique_lock<std::mutex> lk(eh->mu);
      eh->cv.wait(lk, [&] { return !eh->busy[slot]; });
      eh->busy[slot] = true;
    }
    EcFrameArgs ea;
    ea.tx0 = g.tx0;
    ea.ty0 = g.ty0;
    ea.tw = g.tw;
    ea.th = g.th;
    ea.tws = g.tws;
    ea.ths = g.ths;
    ea.xdec = g.xdec;
    ea.ydec = g.ydec;
    ea.ntx_c = r->ntx_c;
    ea.nsb = g.nsb;
    ea.mi_lg = r->mi_lg;
    ea.mi_skip = r->mi_skip;
    ea.mi_stride = r->mi_stride;
    ea.mi_cols = r->mi_cols;
    ea.mi_rows = r->mi_rows;
    ea.lv[0].l_lev = r->l_lev;
    ea.lv[0].c_lev = r->c_lev;
    ea.lv[0].n = g.nsb;
    ea.lv[0].gw = g.tw;
    ea.lv[0].x0 = g.tx0;
    ea.lv[0].y0 = g.ty0;
    for (int l = 1; r->lvl && l < kLevels; l++) {
      const rv_replay::PLevel &P = r->pl[l];
      ea.lv[l].l_lev = P.l_lev;
      ea.lv[l].c_lev = P.c_lev;
      ea.lv[l].n = P.n;
      ea.lv[l].gw = P.gw;
      ea.lv[l].x0 = P.cg.tx0;
      ea.lv[l].y0 = P.cg.ty0;
      ea.lv[l].B = P.B;
      ea.lv[l].bc = P.bc;
    }
    ea.words = r->words;
    ea.words_per_sb = kWordsPerRef * g.R + 4;
    ea.win_off = kWordsPerRef * g.R;
    EcFrameBufs b = r->ecb;
    RV_H(hipHostGetDevicePointer((void **)&b.tokens, eh->tok_h[slot], 0));
    RV_H(hipHostGetDevicePointer((void **)&b.stat, eh->stat_h[slot], 0));
    // RAV1E_HIP_F8_STREAM=1: on its own stream (A/B; default: the main one)
    const bool own = r->ecs != nullptr;
    hipStream_t es = own ? r->ecs : st;
    if (own) {
      RV_H(hipEventRecord(r->ev_f8fork, st));
      RV_H(hipStreamWaitEvent(r->ecs, r->ev_f8fork, 0));
    }
    if (tm) RV_H(hipEventRecord(e[rv_replay::kStageEv + 4], es));
    RV_R(ec_frame_tokens(ea, b, es));
    if (tm) RV_H(hipEventRecord(e[rv_replay::kStageEv + 5], es));
    RV_H(hipEventRecord(eh->ev[slot], es));
    if (own) {
      RV_H(hipEventRecord(r->ev_f8done, r->ecs));
      r->f8_pending = true;
    }
    const int q = r->lv[lv].qidx;
    {
      std::lock_guard<std::mutex> lk(eh->mu);
      eh->q.push_back({slot, lv, q <= 20 ? 0 : q <= 60 ? 1 : q <= 120 ? 2 : 3});
      eh->queued++;
    }
    eh->cv.notify_all();
    r->ec_frames++;
  }
  if (host_trace) {
    static thread_local hclock::time_point prev_end = h0;
    const auto h1 = hclock::now();
    fprintf(stderr, "host frame %ld level %d: since-last-exit %ld take %ld r0 %ld mv %ld intra %ld tail %ld us\n",
            r->coded, lv, us(prev_end, h0), us(h0, h_take), us(h_take, h_r0), us(h_r0, h_mv),
            us(h_mv, h_intra), us(h_intra, h1));
    prev_end = h1;
  }
  r->coded++;
  r->last = fi;
  if (r->n_groups < 2 && !r->comm) {
    RV_R(filter_slot(r, S, cur, lv));
  } else {
    XRect xr[9];
    int nx;
    if (r->lrf) {  // this group's units travel with its reconstruction
      LrfGeo lg;
      RV_R(lrf_geometry(g.W, g.H, g.xdec, g.ydec, g.bd, r->lv[lv].qidx, g.tws, g.ths, &lg));
      RV_R(lrf_decide_slot(r, S, cur, lv, lg, r->grects + 4 * r->my_group));
    }
    group_rects(r, r->my_group, xr, &nx);
    RV_R(xcopy(r, S, xr, nx, 0, r->xsend));
    if (r->comm) {
#if RV_HAVE_RCCL
      if (ncclAllGather(r->xsend, r->xrecv, r->xbytes, ncclUint8, (ncclComm_t)r->comm, st) !=
          ncclSuccess)
        return rv_set_error(RV_EHIP, "rv_replay_frame: ncclAllGather");
      RV_R(rv_replay_import(r));
#else
      return rv_set_error(RV_EINVAL, "rv_replay_frame: built without RCCL");
#endif
    }
  }
  RV_EV(13);
#undef RV_EV
  if (r->eng) RV_R(la_engine_release(r, r->coded - 1, st));  // its lookahead entry is free
  if (info) *info = fi;
  RV_H(hipGetLastError());
  return RV_OK;
}

int rv_replay_results(rv_replay *r, uint64_t *host_out, int cap) {
  if (!r || !host_out) return rv_set_error(RV_EINVAL, "rv_replay_results: null");
  const Geo &g = r->g;
  const int nw = (int)r->nwords;
  const int total = nw + 5;
  if (cap < total) return rv_set_error(RV_EINVAL, "rv_replay_results: cap too small");
  // verification checksums of the last coded frame (outside the per-frame work)
  hipStream_t st = r->stream;
  const int64_t nl = (int64_t)g.nsb * 1024, nc = (int64_t)g.nsb * r->ntx_c * 1024;
  RV_H(hipMemsetAsync(r->tail, 0, 2 * 8, st));
  RV_H(hipMemsetAsync(r->tail + 3, 0, 2 * 8, st));
  if (!r->lvl) {
    coeff_checksum<<<1024, 256, 0, st>>>(r->l_lev, nl, 1024, r->tail);
    coeff_checksum<<<1024, 256, 0, st>>>(r->c_lev, 2 * nc, 1024, r->tail);
  } else {  // the committed blocks (leaves) of every level
    coeff_checksum_list<<<1024, 256, 0, st>>>(r->l_lev, r->pl[0].leaf, r->leaf_count, 1024, 1024,
                                              r->tail);
    for (int q = 0; q < 2; q++)
      coeff_checksum_list<<<1024, 256, 0, st>>>(r->c_lev + q * nc, r->pl[0].leaf, r->leaf_count,
                                                r->ntx_c * 1024, 1024, r->tail);
    for (int l = 1; l < kLevels; l++) {
      const rv_replay::PLevel &P = r->pl[l];
      const int pl_ = P.B * P.B, pc = P.bc * P.bch;
      coeff_checksum_list<<<1024, 256, 0, st>>>(P.l_lev, P.leaf, r->leaf_count + l, pl_, pl_,
                                                r->tail);
      for (int q = 0; q < 2; q++)
        coeff_checksum_list<<<1024, 256, 0, st>>>(P.c_lev + (size_t)q * P.n * pc, P.leaf,
                                                  r->leaf_count + l, pc, pc, r->tail);
    }
  }
  const RvSlot &s = r->slots[r->last.display % kSlots];
  const rv_plane *pl[3] = {&s.y, &s.u, &s.v};
  for (int i = 0; i < 3; i++) {
    const rv_plane &p = *pl[i];
    const int xd = i ? g.xdec : 0, yd = i ? g.ydec : 0;
    const int x0 = (g.tx0 * kSb) >> xd, y0 = (g.ty0 * kSb) >> yd;
    int x1 = ((g.tx0 + g.tw) * kSb) >> xd, y1 = ((g.ty0 + g.th) * kSb) >> yd;
    x1 = x1 < p.width ? x1 : p.width;
    y1 = y1 < p.height ? y1 : p.height;
    // the group's region, and (after the exchange) the whole frame
    if (g.hbd) {
      sum_rect<uint16_t><<<1024, 256, 0, st>>>(p, x0, y0, x1 - x0, y1 - y0, r->tail + 1);
      sum_rect<uint16_t><<<1024, 256, 0, st>>>(p, 0, 0, p.width, p.height, r->tail + 4);
    } else {
      sum_rect<uint8_t><<<1024, 256, 0, st>>>(p, x0, y0, x1 - x0, y1 - y0, r->tail + 1);
      sum_rect<uint8_t><<<1024, 256, 0, st>>>(p, 0, 0, p.width, p.height, r->tail + 4);
    }
  }
  RV_H(hipGetLastError());
  RV_H(hipMemcpyAsync(host_out, r->words, (size_t)nw * 8, hipMemcpyDeviceToHost, st));
  RV_H(hipMemcpyAsync(host_out + nw, r->tail, 5 * 8, hipMemcpyDeviceToHost, st));
  RV_H(hipStreamSynchronize(st));
  host_out[nw + 3] = (uint64_t)r->n_imp;
  return total;
}

static int stage_times(rv_replay *r, float *ms_out, int cap, int last) {
  if (!r || !ms_out) return rv_set_error(RV_EINVAL, "rv_replay_stage_times: null");
  if (r->timed == 0) return rv_set_error(RV_EINVAL, "rv_replay_stage_times: no timed frame");
  if (last < 1) last = 1;
  if (last > rv_replay::kRing) last = rv_replay::kRing;
  if (last > r->timed) last = (int)r->timed;
  constexpr int kS = rv_replay::kStageEv;
  for (int i = 0; i < cap && i < kS; i++) ms_out[i] = 0.f;
  int n = 0;
  for (int f = 0; f < last; f++) {
    hipEvent_t *e = r->evs[(r->timed - 1 - f) % rv_replay::kRing];
    RV_H(hipEventSynchronize(e[kS - 1]));
    RV_H(hipEventSynchronize(e[kS + 1]));
    n = 0;
    for (int i = 0; i < kS - 1 && n < cap; i++) {
      float ms = 0.f;
      RV_H(hipEventElapsedTime(&ms, e[i], e[i + 1]));
      ms_out[n++] += ms;
    }
    if (n < cap) {  // the lookahead's own span (overlapped with F3/F4 by default)
      float ms = 0.f;
      RV_H(hipEventElapsedTime(&ms, e[kS], e[kS + 1]));
      ms_out[n++] += ms;
    }
    if (n < cap) {  // the edge levels' own span (speed 10, beside F3..F4)
      float ms = 0.f;
      RV_H(hipEventSynchronize(e[kS + 3]));
      RV_H(hipEventElapsedTime(&ms, e[kS + 2], e[kS + 3]));
      ms_out[n++] += ms;
    }
    if (n < cap && r->entropy) {  // F8: the coefficient tokens
      float ms = 0.f;
      RV_H(hipEventSynchronize(e[kS + 5]));
      RV_H(hipEventElapsedTime(&ms, e[kS + 4], e[kS + 5]));
      ms_out[n++] += ms;
    }
  }
  return n;
}

int rv_replay_entropy_stats(rv_replay *r, uint64_t *out, int cap) {
  if (!r || !out || cap < 4) return rv_set_error(RV_EINVAL, "rv_replay_entropy_stats: null / cap");
  if (!r->ech) return rv_set_error(RV_EINVAL, "rv_replay_entropy_stats: RV_REPLAY_ENTROPY off");
  r->ech->drain();
  if (r->ech->err) return rv_set_error(r->ech->err, "rv_replay_entropy_stats: token buffer overflow");
  const int n = cap < 5 ? cap : 5;
  for (int i = 0; i < n; i++) out[i] = r->ech->stat[i];
  return n;
}

int rv_replay_set_timing(rv_replay *r, int stride, int block) {
  if (!r || stride < 0 || block < 1)
    return rv_set_error(RV_EINVAL, "rv_replay_set_timing: bad stride / block");
  r->timing_stride = stride;
  r->timing_block = block;
  return RV_OK;
}

int rv_replay_stage_times(rv_replay *r, float *ms_out, int cap) {
  return stage_times(r, ms_out, cap, 1);
}
int rv_replay_stage_times_sum(rv_replay *r, int last_frames, float *ms_out, int cap) {
  return stage_times(r, ms_out, cap, last_frames);
}

// The kernel probe: on (re)start, the sums so far are dropped (the pairs in
// flight are waited for); off stops recording.
int rv_replay_set_kernel_probe(rv_replay *r, int on) {
  if (!r) return rv_set_error(RV_EINVAL, "rv_replay_set_kernel_probe: null");
  constexpr int P = rv_replay::kProbes, C = rv_replay::kKpCnt;
  if (on && r->kp_ev[0].empty()) {
    for (int p = 0; p < P; p++) {
      r->kp_ev[p].assign(2 * rv_replay::kKp, nullptr);
      for (auto &ev : r->kp_ev[p]) RV_H(hipEventCreate(&ev));
      r->kp_cnt[p] = (uint32_t *)dalloc(r, C * sizeof(uint32_t));
      r->kp_ts[p] = (unsigned long long *)dalloc(r, 2 * sizeof(unsigned long long) * rv_replay::kKp);
      if (!r->kp_cnt[p] || !r->kp_ts[p])
        return rv_set_error(RV_EHIP, "rv_replay_set_kernel_probe: allocation failed");
    }
    int dev = 0, khz = 0;
    RV_H(hipGetDevice(&dev));
    RV_H(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
    r->kp_tick_ms = khz > 0 ? 1.0 / (double)khz : 0.0;
  }
  if (!r->kp_ev[0].empty()) {
    for (int p = 0; p < P; p++) RV_H(kp_harvest(r, p, r->kp_n[p]));
    RV_H(hipDeviceSynchronize());
    for (int p = 0; p < P; p++) RV_H(hipMemset(r->kp_cnt[p], 0, C * sizeof(uint32_t)));
    RV_H(hipDeviceSynchronize());
  }
  for (int p = 0; p < P; p++) {
    r->kp_ms[p] = 0.0;
    r->kp_dev_ms[p] = 0.0;
    r->kp_base[p] = r->kp_n[p];
  }
  r->kprobe = on != 0;
  return RV_OK;
}

// probe 0: out[0] launches, [1] their summed milliseconds (event pairs on
// their streams), [2] candidate evaluations, [3] jobs, [4] device-clock ms;
// probe 1 (cap >= 11): out[5] launches, [6] event ms, [7] device-clock ms,
// [8] single / [9] compound luma candidates, [10] single chroma transform
// blocks, [11] compound ones (cap >= 12)
int rv_replay_kernel_probe(rv_replay *r, double *out, int cap) {
  if (!r || !out || cap < 4) return rv_set_error(RV_EINVAL, "rv_replay_kernel_probe: null / cap");
  const int nout = cap >= 12 ? 12 : cap < 5 ? 4 : 5;
  for (int i = 0; i < nout; i++) out[i] = 0.0;
  if (r->kp_ev[0].empty()) return nout;
  for (int p = 0; p < rv_replay::kProbes; p++) RV_H(kp_harvest(r, p, r->kp_n[p]));
  uint32_t c[2][rv_replay::kKpCnt] = {{0}};
  RV_H(hipDeviceSynchronize());
  for (int p = 0; p < rv_replay::kProbes; p++)
    RV_H(hipMemcpy(c[p], r->kp_cnt[p], sizeof(c[p]), hipMemcpyDeviceToHost));
  out[0] = (double)(r->kp_n[0] - r->kp_base[0]);
  out[1] = r->kp_ms[0];
  out[2] = (double)c[0][0];
  out[3] = (double)c[0][1];
  if (nout > 4) out[4] = r->kp_dev_ms[0];
  if (nout >= 12) {
    out[5] = (double)(r->kp_n[1] - r->kp_base[1]);
    out[6] = r->kp_ms[1];
    out[7] = r->kp_dev_ms[1];
    for (int i = 0; i < 4; i++) out[8 + i] = (double)c[1][i];
  }
  return nout;
}
// Candidate evaluations summed over the last min(frames, 64) coded frames:
// out[0] F3 full-pel diamond, out[1] F3 sub-pel diamond (64x64 jobs), out[2]
// frames summed, (cap >= 5) out[3] / out[4] the F4 single-reference /
// compound RDO candidates of the 64x64 blocks, (cap >= 11, speed 6) out[5 +
// 2 (l - 1)] / out[6 + 2 (l - 1)] those of the 32x32, 16x16, 8x8 blocks.
int rv_replay_dpb_slots(void) { return kSlots; }

int rv_replay_counters(rv_replay *r, uint64_t *out, int cap) {
  if (!r || !out || cap < 3) return rv_set_error(RV_EINVAL, "rv_replay_counters");
  const Geo &g = r->g;
  const int nj = g.nsb * g.R;
  const long nonkey = r->coded > 0 ? r->coded - 1 : 0;
  const int nf = nonkey < rv_replay::kRing ? (int)nonkey : rv_replay::kRing;
  RV_H(hipStreamSynchronize(r->stream));
  std::vector<uint32_t> h((size_t)nf * 2 * nj);
  if (nf) RV_H(hipMemcpy(h.data(), r->ds_evals, h.size() * 4, hipMemcpyDeviceToHost));
  out[0] = out[1] = 0;
  for (int f = 0; f < nf; f++)
    for (int k = 0; k < 2; k++)
      for (int j = 0; j < nj; j++) out[k] += h[((size_t)f * 2 + k) * nj + j];
  out[2] = (uint64_t)nf;
  if (cap < 5) return 3;
  const int nl = cap >= 11 ? kLevels : 1;
  std::vector<uint32_t> ce((size_t)nf * 2 * kLevels);
  if (nf) RV_H(hipMemcpy(ce.data(), r->cand_evals, ce.size() * 4, hipMemcpyDeviceToHost));
  for (int l = 0; l < nl; l++) {
    uint64_t &a = out[l ? 5 + 2 * (l - 1) : 3], &b = out[l ? 6 + 2 * (l - 1) : 4];
    a = b = 0;
    for (int f = 0; f < nf; f++) {
      a += ce[(size_t)(f * kLevels + l) * 2];
      b += ce[(size_t)(f * kLevels + l) * 2 + 1];
    }
  }
  if (cap < 14) return nl == 1 ? 5 : 11;
  std::vector<uint32_t> is((size_t)nf * 3);
  if (nf) RV_H(hipMemcpy(is.data(), r->i_stats, is.size() * 4, hipMemcpyDeviceToHost));
  out[11] = out[12] = out[13] = 0;
  for (int f = 0; f < nf; f++)
    for (int k = 0; k < 3; k++) out[11 + k] += is[(size_t)f * 3 + k];
  if (cap < 17) return 14;
  // speed 10 MV-stack rounds since creation: rounds (F3 + F4 launches),
  // superblock re-evaluations after the first round, frames
  out[14] = (uint64_t)r->mv_round_sum;
  out[15] = (uint64_t)r->mv_reeval;
  out[16] = (uint64_t)r->mv_frames;
  if (cap < 18) return 17;
  // round runs: 1 + the MV / intra passes (the joint fixed point's outer
  // iterations), summed over frames
  out[17] = (uint64_t)r->mv_run_sum;
  if (cap < 20) return 18;
  // the lookahead's EPZS rounds and re-run jobs (the engine's on its owner)
  const bool own_eng = r->eng && r->eng_owned;
  long er = 0, ere = 0, ef = 0;
  if (own_eng) {
    std::lock_guard<std::mutex> lk(r->eng->mu);
    er = r->eng->la_round_sum;
    ere = r->eng->la_reeval;
    ef = r->eng->la_frames;
  }
  out[18] = (uint64_t)(r->la_round_sum + er);
  out[19] = (uint64_t)(r->la_reeval + ere);
  if (cap < 21) return 20;
  // the frames those lookahead rounds belong to (the engine runs ahead of
  // the encode: up to W frames past the last coded one)
  out[20] = (uint64_t)(r->la_frames + ef);
  return 21;
}

// Host-only test hook: the slots RoundRing gives check q -- out[0] the
// device count slot it counts into, out[1] the slot it zeroes for check
// q + 1, out[2] its host publication slot -- and out[3] kRoundsAhead,
// out[4] kCnt, out[5] kPub (cap >= 6).  Returns 6.
int rv_round_ring_slots(uint32_t q, int32_t *out, int cap) {
  if (!out || cap < 6) return rv_set_error(RV_EINVAL, "rv_round_ring_slots: cap");
  static int32_t cnt[2 * RoundRing::kCnt + 1];
  static unsigned long long pub[RoundRing::kPub];
  RoundRing rr;
  rr.cnt = cnt;
  rr.d_pub = pub;
  const RoundPub p = rr.pub(q);
  out[0] = (int32_t)((p.cnt - cnt) / 2);
  out[1] = (int32_t)((p.next - cnt) / 2);
  out[2] = (int32_t)(p.host - pub);
  out[3] = rv_replay::kRoundsAhead;
  out[4] = RoundRing::kCnt;
  out[5] = RoundRing::kPub;
  return 6;
}

// Host-only test hook: the lookahead references of coded frame m >= 1
// (la_refs_of): out[0] = n, out[1..3] their displays in k order, out[4..6]
// the propagation order (-1: unused).  Returns 0.
// RV_REPLAY_LRF: the last coded frame's loop-restoration units of plane p,
// (set, xqd0, xqd1) per unit in raster order (set -1: None); synchronous
int rv_replay_lrf_units(rv_replay *r, int plane, int8_t *out, int cap) {
  if (!r || !out || plane < 0 || plane > 2) return rv_set_error(RV_EINVAL, "rv_replay_lrf_units: bad arguments");
  if (!r->lrf) return rv_set_error(RV_EINVAL, "rv_replay_lrf_units: RV_REPLAY_LRF is off");
  const Geo &g = r->g;
  const int nsb = ((g.W + 63) / 64) * ((g.H + 63) / 64);
  if (cap < 3 * nsb) return rv_set_error(RV_EINVAL, "rv_replay_lrf_units: cap < 3 * superblocks");
  RV_H(hipStreamSynchronize(r->stream));
  RV_H(hipMemcpy(out, r->lrf_units + (size_t)plane * nsb * 3, (size_t)nsb * 3, hipMemcpyDeviceToHost));
  return RV_OK;
}

int rv_replay_la_refs(long m, int R, int32_t *out) {
  if (!out || m < 1 || R < 1 || R > 2) return rv_set_error(RV_EINVAL, "rv_replay_la_refs");
  const LaRefs l = la_refs_of(m, R);
  out[0] = l.n;
  for (int k = 0; k < 3; k++) {
    out[1 + k] = k < l.n ? l.disp[k] : -1;
    out[4 + k] = k < l.n ? l.order[k] : -1;
  }
  return RV_OK;
}

// ---- RCCL communicator for the tile-group exchange ---------------------------
int rv_comm_unique_id(uint8_t *out, int cap) {
#if RV_HAVE_RCCL
  if (!out || cap < (int)sizeof(ncclUniqueId)) return rv_set_error(RV_EINVAL, "rv_comm_unique_id");
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return rv_set_error(RV_EHIP, "ncclGetUniqueId");
  memcpy(out, &id, sizeof(id));
  return (int)sizeof(id);
#else
  (void)out;
  (void)cap;
  return rv_set_error(RV_EINVAL, "rv_comm_unique_id: built without RCCL");
#endif
}

void *rv_comm_create(const uint8_t *id, int nranks, int rank) {
#if RV_HAVE_RCCL
  if (!id || nranks < 1 || rank < 0 || rank >= nranks) {
    rv_set_error(RV_EINVAL, "rv_comm_create");
    return nullptr;
  }
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclComm_t c = nullptr;
  if (ncclCommInitRank(&c, nranks, u, rank) != ncclSuccess) {
    rv_set_error(RV_EHIP, "ncclCommInitRank");
    return nullptr;
  }
  return c;
#else
  (void)id;
  (void)nranks;
  (void)rank;
  rv_set_error(RV_EINVAL, "rv_comm_create: built without RCCL");
  return nullptr;
#endif
}

void rv_comm_destroy(void *comm) {
#if RV_HAVE_RCCL
  if (comm) (void)ncclCommDestroy((ncclComm_t)comm);
#else
  (void)comm;
#endif
}

}  // extern "C"
