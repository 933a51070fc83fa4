// rv_replay.hip -- hot-path replay driver: the per-frame call structure of
// a speed-10 encode of one tile, for the stages this library accelerates,
// with every frame resident in HBM.  Schedule (DESIGN.md "Replay driver"):
//
//   F0  hres / qres of the input (encode_frame, src/encoder.rs:3382-3385)
//   F1  coarse ME: full_search at 1/4 res, 16x16 per 64x64 superblock and
//       reference (estimate_motion_ss4, src/me.rs:1023-1075)
//   F2  half-res diamond, 32x32 (estimate_motion_ss2 / me_ss2,
//       src/me.rs:287-519)
//   F3  full-res full-pel diamond then sub-pel diamond, 64x64
//       (motion_estimation, src/me.rs:193-285)
//   F4  RDO candidates per superblock: {sub-pel MV, zero MV} x reference:
//       put_8tap luma + chroma, diff + forward DCT (TX_64X64 luma,
//       TX_32X32 chroma), quantize + dequantize at qindex kReplayQindex,
//       inverse transform + add, cdef-moment luma / SSE chroma distortion,
//       argmin (encode_tx_block src/encoder.rs:1077-1237,
//       compute_distortion src/rdo.rs:338-411)
//   F5  8x8 importance SATD against reference 1 (compute_block_importances,
//       src/api/internal.rs:823-1010) and the lookahead intra cost of the
//       same blocks (compute_lookahead_intra_costs, :680-765: SATD against
//       pred_dc_128, rv_dist.hip)
//
// Every stage is one batched launch over all superblocks of the tile.  The
// glue between dependent stages is chained on the device (rv_chain.h): the
// workgroup finishing a search writes its winner into the next stage's job
// records, whose static fields are built once at creation.  A frame is 8
// launches on one stream with no host round trip.  The CPU baseline
// (oracle/orc_replay.c) runs the same schedule and must produce the same
// result words.
#include <string.h>

#include <vector>

#include "rv_chain.h"
#include "rv_device.h"
#include "rv_rdo.h"

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
                            void *stream);
// rv_frame.hip: hres + qres (+ padding) in one launch
int rv_plane_pyramid(const rv_plane *y, const rv_plane *h, const rv_plane *q, void *stream);

namespace rv {

constexpr int kSb = 64;
// base_q_idx of the replay's frames: rav1e's default --quantizer (100) used
// directly as the qindex; the rate controller that would vary it per frame
// type is out of scope.  oracle/orc_replay.c uses the same value.
constexpr int kReplayQindex = 100;

struct Geo {
  int W, H, xdec, ydec, bd, hbd;
  int w_in_b, h_in_b;       // MiCols / MiRows (src/encoder.rs:580-581)
  int tx0, ty0, tw, th;     // tile rect in superblocks
  int mi_w, mi_h;           // tile size in 4x4 units (tile_state.rs:93)
  int nsb, R, C, nctx;      // superblocks, references, candidates, nsb * C
  int cw, ch;               // chroma block of a superblock
};

__host__ __device__ inline int div_trunc8(int v) { return v / 8; }

// get_mv_range (src/me.rs:64-80); bo in 4x4 units (frame).  Rust usize
// arithmetic wraps and is cast back to isize, i.e. signed here.
__host__ __device__ inline void mv_range(const Geo &g, int bx, int by, int bw,
                                         int bh, int r[4]) {
  const int border_w = 128 + bw * 8, border_h = 128 + bh * 8;
  r[0] = -bx * 32 - border_w;
  r[1] = (g.w_in_b - bx - bw / 4) * 32 + border_w;
  r[2] = -by * 32 - border_h;
  r[3] = (g.h_in_b - by - bh / 4) * 32 + border_h;
}
// adjust_bo (src/me.rs:993-1004) on tile-relative 4x4 offsets
__host__ __device__ inline void adjust_bo(const Geo &g, int &bx, int &by,
                                          int bw, int bh) {
  int x = bx < g.mi_w - bw / 4 ? bx : g.mi_w - bw / 4;
  int y = by < g.mi_h - bh / 4 ? by : g.mi_h - bh / 4;
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

// Verification checksum of packed coefficients (results time, not per
// frame): sum of q * (position in block + 1), wrapping u64.
__global__ void coeff_checksum(const int32_t *packed, int64_t total, int per_block,
                               unsigned long long *out) {
  uint64_t s = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x)
    s += (uint64_t)(int64_t)packed[i] * (uint64_t)(i % per_block + 1);
  block_atomic_add(s, out);
}

// Candidate score = luma SSE (from the cdef moments) + chroma SSE, then the
// per-superblock argmin (first minimum) and result words.  One wavefront
// per superblock: lanes stride over the sub-blocks of a candidate.
__global__ __launch_bounds__(64) void score_candidates(
    Geo g, const int64_t *lmom, const uint64_t *usse, const uint64_t *vsse, int lsub, int csub,
    const rv_fs_result *coarse, const rv_fs_result *half, const rv_fs_result *full,
    const rv_fs_result *sub, uint64_t *words, unsigned long long *imp_sum) {
  const int sb = blockIdx.x;
  const int lane = threadIdx.x;
  if (sb == 0 && lane == 0) *imp_sum = 0;  // F5 accumulates after this launch
  uint64_t best = ~0ull;
  int best_c = 0;
  for (int c = 0; c < g.C; c++) {
    const int64_t o = (int64_t)c * g.nsb + sb;  // candidate-major, like the MC jobs
    uint64_t s = 0;
    for (int k = lane; k < lsub; k += 64) {
      const int64_t *m = lmom + (o * lsub + k) * 5;
      s += (uint64_t)(m[3] + m[2] - 2 * m[4]);
    }
    for (int k = lane; k < csub; k += 64) s += usse[o * csub + k] + vsse[o * csub + k];
    s = group_sum<64>(s);
    if (s < best) {
      best = s;
      best_c = c;
    }
  }
  uint64_t *w = words + (int64_t)sb * (8 * g.R + 2);
  for (int i = lane; i < 8 * g.R; i += 64) {
    const int r = i >> 3, f = i & 7;
    const rv_fs_result *src = (f >> 1) == 0 ? coarse : (f >> 1) == 1 ? half : (f >> 1) == 2 ? full : sub;
    const rv_fs_result v = src[r * g.nsb + sb];
    w[i] = (f & 1) ? v.cost : pack_mv(v.best_mv);
  }
  if (lane == 0) {
    w[8 * g.R] = (uint64_t)best_c;
    w[8 * g.R + 1] = best;
  }
}

// F5: get_satd of every 8x8 luma block of the tile inside the frame against
// reference 1 at the full-pel part of its superblock's sub-pel MV
// (compute_block_importances, src/api/internal.rs:823-1010) plus its
// lookahead intra cost (get_satd against pred_dc_128,
// src/api/internal.rs:680-765), summed.  One lane per block; the job is
// computed in place, the source block read once for both.
template <typename Px>
__global__ __launch_bounds__(256) void importance_kernel(Geo g, rv_plane org, rv_plane ref,
                                                          const rv_fs_result *sub, int nbx,
                                                          int nby, unsigned long long *sum) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t v = 0;
  if (i < nbx * nby) {
    const int bx = i % nbx, by = i / nbx;
    const rv_mv mv = sub[(by / 8) * g.tw + (bx / 8)].best_mv;  // reference 1
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

// Sum of the reconstructed pixels of a plane (all candidates; results time).
template <typename Px>
__global__ void sum_plane(rv_plane p, int w, int h, unsigned long long *out) {
  uint64_t s = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (int64_t)w * h;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int y = (int)(i / w), x = (int)(i - (int64_t)y * w);
    s += *plane_ptr<Px>(p, x, y);
  }
  block_atomic_add(s, out);
}

}  // namespace rv

using namespace rv;

struct RvFrameSlot {
  rv_plane y, u, v, hres, qres;
  uint32_t *qres_box = nullptr;  // rv_plane_box_sums of qres (the SEA coarse search)
  void *mem = nullptr;
};

struct rv_replay {
  rv_replay_cfg cfg;
  Geo g;
  hipStream_t stream;
  hipStream_t side;  // zero-MV RDO candidates, concurrent with the searches
  bool own_stream;
  bool sea;  // successive-elimination coarse search (bit depth <= 10)
  double me_lambda;
  QCtx q_luma, q_chroma;  // QuantizationContext, TX_64X64 / TX_32X32 inter
  std::vector<RvFrameSlot> slots;  // 0 = input, 1..R = references
  // scratch
  rv_plane tall_y, tall_u, tall_v;
  void *tall_mem = nullptr;
  std::vector<void *> allocs;
  rv_fs_job *fs_jobs[3] = {nullptr, nullptr, nullptr};  // per scale 1, 2, 4
  rv_fs_result *coarse, *half, *full, *sub;
  // chained search jobs (static fields built at creation, predictors
  // written by the previous stage, rv_chain.h)
  rv_ds_job *jobs_half, *jobs_full, *jobs_sub;
  rv_mc_job *l_mc, *c_mc;
  rv_tx_job *l_tx, *c_tx;
  int32_t *l_packed, *c_packed;
  int64_t *l_mom;
  uint64_t *u_sse, *v_sse, *words;
  unsigned long long *tail;  // [coeff csum, recon csum, imp satd sum]
  int n_imp, imp_bx, imp_by, lsub, csub;
  // Event ring: frame f records into set f % kRing (stage bounds and
  // kernel brackets, see rv_replay_frame), so per-kernel times can be
  // summed over a whole timed run without a host sync per frame.
  static constexpr int kRing = 64;
  static constexpr int kEv = 11;  // + [9,10]: side-stream RDO bracket
  hipEvent_t evs[kRing][kEv];
  hipEvent_t fork[kRing], join[kRing], fork2[kRing], join2[kRing];  // cross-stream ordering
  hipEvent_t *ev;
  long frames = 0;
  // Every `timing_stride`-th frame records the timing events (each record
  // costs ~4.4 us of idle GPU between kernels on MI355X); `timed` counts
  // the instrumented frames, which own the event ring slots.
  int timing_stride = 1, timing_block = 1;
  long timed = 0;
  bool ev_side[kRing];
  // diamond candidate evaluations per job, per ring slot: [kRing][2][nsb*R]
  // (F3 full-pel, F3 sub-pel)
  uint32_t *ds_evals;
};

namespace {

void *dalloc(rv_replay *r, size_t bytes) {
  void *p = nullptr;
  if (hipMalloc(&p, bytes ? bytes : 16) != hipSuccess) return nullptr;
  r->allocs.push_back(p);
  return p;
}

bool alloc_slot(rv_replay *r, RvFrameSlot &s) {
  const Geo &g = r->g;
  // Frame::new (src/frame/mod.rs:55-90): luma pad 64 + 24, chroma >> dec
  const int pad = 88;
  const int cw = (g.W + g.xdec) >> g.xdec, ch = (g.H + g.ydec) >> g.ydec;
  size_t by = rv_plane_geometry(&s.y, g.W, g.H, 0, 0, pad, pad, g.hbd);
  size_t bu = rv_plane_geometry(&s.u, cw, ch, g.xdec, g.ydec, pad >> g.xdec, pad >> g.ydec, g.hbd);
  size_t bv = rv_plane_geometry(&s.v, cw, ch, g.xdec, g.ydec, pad >> g.xdec, pad >> g.ydec, g.hbd);
  // input_hres / input_qres (src/encoder.rs:362-377)
  size_t bh = rv_plane_geometry(&s.hres, g.W / 2, g.H / 2, 1, 1, pad / 2, pad / 2, g.hbd);
  size_t bq = rv_plane_geometry(&s.qres, g.W / 4, g.H / 4, 2, 2, pad / 4, pad / 4, g.hbd);
  s.y.bit_depth = s.u.bit_depth = s.v.bit_depth = s.hres.bit_depth = s.qres.bit_depth = g.bd;
  const size_t al = 256;
  auto up = [&](size_t v) { return (v + al - 1) / al * al; };
  const size_t bs8 = (size_t)s.qres.stride * s.qres.alloc_height * 8;
  size_t total = up(by) + up(bu) + up(bv) + up(bh) + up(bq) + up(bs8);
  uint8_t *m = (uint8_t *)dalloc(r, total);
  if (!m) return false;
  s.mem = m;
  s.y.data = m;
  m += up(by);
  s.u.data = m;
  m += up(bu);
  s.v.data = m;
  m += up(bv);
  s.hres.data = m;
  m += up(bh);
  s.qres.data = m;
  m += up(bq);
  s.qres_box = (uint32_t *)m;
  return hipMemsetAsync(s.mem, 0, total, r->stream) == hipSuccess;
}

int build_static_jobs(rv_replay *r) {
  const Geo &g = r->g;
  // F1 coarse jobs for me_range_scale 1, 2, 4 (estimate_motion_ss4)
  const uint32_t lambda4 = (uint32_t)(r->me_lambda * 256.0 / 16.0 * 0.125);
  for (int si = 0; si < 3; si++) {
    const int s = 1 << si;
    std::vector<rv_fs_job> jobs(g.nsb * g.R);
    for (int sb = 0; sb < g.nsb; sb++) {
      int bx = (sb % g.tw) * 16, by = (sb / g.tw) * 16;
      adjust_bo(g, bx, by, 64, 64);
      const int fbx = bx + g.tx0 * 16, fby = by + g.ty0 * 16;
      const int pox = fbx, poy = fby;  // (bo << 2) >> 2
      const int range_x = 192 * s, range_y = 64 * s;
      int mr[4];
      mv_range(g, fbx, fby, 64, 64, mr);
      auto mx = [](int a, int b) { return a > b ? a : b; };
      auto mn = [](int a, int b) { return a < b ? a : b; };
      rv_fs_job j;
      memset(&j, 0, sizeof(j));
      j.po_x = pox;
      j.po_y = poy;
      j.x_lo = pox + (mx(-range_x, div_trunc8(mr[0])) >> 2);
      j.x_hi = pox + (mn(range_x, div_trunc8(mr[1])) >> 2);
      j.y_lo = poy + (mx(-range_y, div_trunc8(mr[2])) >> 2);
      j.y_hi = poy + (mn(range_y, div_trunc8(mr[3])) >> 2);
      j.lambda = lambda4;
      for (int k = 0; k < g.R; k++) jobs[k * g.nsb + sb] = j;  // ref-major
    }
    r->fs_jobs[si] = (rv_fs_job *)dalloc(r, jobs.size() * sizeof(rv_fs_job));
    if (!r->fs_jobs[si]) return RV_EHIP;
    if (hipMemcpy(r->fs_jobs[si], jobs.data(), jobs.size() * sizeof(rv_fs_job),
                  hipMemcpyHostToDevice) != hipSuccess)
      return RV_EHIP;
  }
  // F2 / F3 diamond jobs: static fields (positions, MV ranges, lambdas);
  // the predictors are chained in by the previous stage each frame
  const uint32_t lambda2 = (uint32_t)(r->me_lambda * 256.0 / 4.0 * 0.125);
  const uint32_t lambda1 = (uint32_t)(r->me_lambda * 256.0 * 0.5);
  std::vector<rv_ds_job> jh(g.nsb * g.R), jf(g.nsb * g.R), js(g.nsb * g.R);
  for (int k = 0; k < g.R; k++)
    for (int sb = 0; sb < g.nsb; sb++) {
      const int i = k * g.nsb + sb;
      // me_ss2 (src/me.rs:470-519): adjusted 64x64 origin at 1/2 res
      int bx = (sb % g.tw) * 16, by = (sb / g.tw) * 16;
      adjust_bo(g, bx, by, 64, 64);
      int fbx = bx + g.tx0 * 16, fby = by + g.ty0 * 16;
      int mr[4];
      mv_range(g, fbx, fby, 64, 64, mr);
      rv_ds_job j;
      memset(&j, 0, sizeof(j));
      j.po_x = fbx * 2;  // (bo << BLOCK_TO_PLANE_SHIFT) >> 1
      j.po_y = fby * 2;
      j.mvx_min = mr[0] >> 1;
      j.mvx_max = mr[1] >> 1;
      j.mvy_min = mr[2] >> 1;
      j.mvy_max = mr[3] >> 1;
      j.lambda = lambda2;
      j.n_pred = 1 + g.R;  // zero + the coarse MV of every reference
      jh[i] = j;
      // full resolution (motion_estimation, src/me.rs:193-285)
      fbx = (sb % g.tw + g.tx0) * 16;
      fby = (sb / g.tw + g.ty0) * 16;
      mv_range(g, fbx, fby, 64, 64, mr);
      memset(&j, 0, sizeof(j));
      j.po_x = fbx * 4;
      j.po_y = fby * 4;
      j.mvx_min = mr[0];
      j.mvx_max = mr[1];
      j.mvy_min = mr[2];
      j.mvy_max = mr[3];
      j.lambda = lambda1;
      j.n_pred = 2;  // zero + the half-res winner
      jf[i] = j;
      j.n_pred = 1;  // the full-pel winner
      js[i] = j;
    }
  // F4 MC jobs of the zero-MV candidates (k = 1); the sub-pel MV ones
  // (k = 0) are chained in by the sub-pel search
  RvFrameSlot &cur = r->slots[0];
  std::vector<rv_mc_job> lmc(g.nctx), cmc(g.nctx);
  for (int c = 0; c < g.C; c++)
    for (int sb = 0; sb < g.nsb; sb++) {
      const int o = c * g.nsb + sb;
      const int sx = sb % g.tw, sy = sb / g.tw;
      const int px = (sx + g.tx0) * kSb, py = (sy + g.ty0) * kSb;
      lmc[o] = mc_job_for(cur.y, px, py, rv_mv{0, 0}, sx * kSb, (c * g.th + sy) * kSb);
      cmc[o] = mc_job_for(cur.u, px >> g.xdec, py >> g.ydec, rv_mv{0, 0}, sx * g.cw,
                          (c * g.th + sy) * g.ch);
    }
  // F4 transform jobs (static: positions only)
  const int ntx_c = (g.cw / 32) * (g.ch / 32);  // 32x32 chroma tx per plane
  std::vector<rv_tx_job> ltx(g.nctx), ctx_(g.nctx * ntx_c);
  for (int c = 0; c < g.C; c++)
    for (int sb = 0; sb < g.nsb; sb++) {
      const int o = c * g.nsb + sb;
      const int sx = sb % g.tw, sy = sb / g.tw;
      const int px = (sx + g.tx0) * kSb, py = (sy + g.ty0) * kSb;
      const int tx = sx * kSb, ty = (c * g.th + sy) * kSb;
      ltx[o] = rv_tx_job{px, py, tx, ty};
      const int cpx = px >> g.xdec, cpy = py >> g.ydec;
      const int ctx0 = sx * g.cw, cty0 = (c * g.th + sy) * g.ch;
      for (int t = 0; t < ntx_c; t++) {
        const int ox = (t % (g.cw / 32)) * 32, oy = (t / (g.cw / 32)) * 32;
        ctx_[o * ntx_c + t] = rv_tx_job{cpx + ox, cpy + oy, ctx0 + ox, cty0 + oy};
      }
    }
  auto upload = [&](auto &vec, auto *&dst) -> int {
    dst = (std::remove_reference_t<decltype(dst)>)dalloc(r, vec.size() * sizeof(vec[0]));
    if (!dst) return RV_EHIP;
    return hipMemcpy(dst, vec.data(), vec.size() * sizeof(vec[0]), hipMemcpyHostToDevice) ==
                   hipSuccess
               ? RV_OK
               : RV_EHIP;
  };
  int e;
  if ((e = upload(ltx, r->l_tx)) || (e = upload(ctx_, r->c_tx)) || (e = upload(jh, r->jobs_half)) ||
      (e = upload(jf, r->jobs_full)) || (e = upload(js, r->jobs_sub)) || (e = upload(lmc, r->l_mc)) ||
      (e = upload(cmc, r->c_mc)))
    return e;
  return RV_OK;
}

}  // namespace

#define RV_R(expr)                                        \
  do {                                                    \
    int e_ = (expr);                                      \
    if (e_ != RV_OK) return e_;                           \
  } while (0)
#define RV_H(expr)                                                   \
  do {                                                               \
    hipError_t e_ = (expr);                                          \
    if (e_ != hipSuccess) return rv_set_hip_error(e_, #expr);        \
  } while (0)

extern "C" {

void rv_replay_destroy(rv_replay *r) {
  if (!r) return;
  for (void *p : r->allocs) (void)hipFree(p);
  for (int f = 0; f < rv_replay::kRing; f++) {
    for (int i = 0; i < rv_replay::kEv; i++)
      if (r->evs[f][i]) (void)hipEventDestroy(r->evs[f][i]);
    if (r->fork[f]) (void)hipEventDestroy(r->fork[f]);
    if (r->join[f]) (void)hipEventDestroy(r->join[f]);
    if (r->fork2[f]) (void)hipEventDestroy(r->fork2[f]);
    if (r->join2[f]) (void)hipEventDestroy(r->join2[f]);
  }
  if (r->side) (void)hipStreamDestroy(r->side);
  if (r->own_stream && r->stream) (void)hipStreamDestroy(r->stream);
  delete r;
}

rv_replay *rv_replay_create(const rv_replay_cfg *cfg, void *stream) {
  if (!cfg || cfg->width <= 0 || cfg->height <= 0 || (cfg->width & 7) ||
      (cfg->height & 7) || (cfg->bit_depth != 8 && cfg->bit_depth != 10 && cfg->bit_depth != 12) ||
      cfg->xdec < 0 || cfg->xdec > 1 || cfg->ydec < 0 || cfg->ydec > 1 ||
      cfg->n_refs < 1 || cfg->n_refs > RV_DS_MAX_PRED - 1) {
    rv_set_error(RV_EINVAL, "rv_replay_create: bad config");
    return nullptr;
  }
  rv_replay *r = new rv_replay();
  memset(r->evs, 0, sizeof(r->evs));
  memset(r->fork, 0, sizeof(r->fork));
  memset(r->join, 0, sizeof(r->join));
  memset(r->fork2, 0, sizeof(r->fork2));
  memset(r->join2, 0, sizeof(r->join2));
  r->side = nullptr;
  r->ev = r->evs[0];
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
  if (g.tx0 < 0 || g.ty0 < 0 || g.tw <= 0 || g.th <= 0 || g.tx0 + g.tw > sbc ||
      g.ty0 + g.th > sbr) {
    rv_set_error(RV_EINVAL, "rv_replay_create: bad tile");
    delete r;
    return nullptr;
  }
  const int vis_w = (g.W - g.tx0 * kSb) < g.tw * kSb ? g.W - g.tx0 * kSb : g.tw * kSb;
  const int vis_h = (g.H - g.ty0 * kSb) < g.th * kSb ? g.H - g.ty0 * kSb : g.th * kSb;
  g.mi_w = vis_w >> 2;
  g.mi_h = vis_h >> 2;
  g.nsb = g.tw * g.th;
  g.R = cfg->n_refs;
  g.C = 2 * g.R;
  g.nctx = g.nsb * g.C;
  g.cw = kSb >> g.xdec;
  g.ch = kSb >> g.ydec;
  // me_lambda = sqrt(lambda), lambda scaled by 1 << 2 (bd - 8)
  // (src/encoder.rs:876-878); the replay fixes the 8-bit value.
  r->me_lambda = 24.0 * (double)(1 << (g.bd - 8));
  // quantizer of every RDO candidate: base_q_idx kReplayQindex with no
  // per-plane deltas, inter (QuantizationContext::update calls of
  // write_tx_tree, src/encoder.rs:1925-1931, 1987-1994)
  if (rv_quant_ctx(kReplayQindex, 64 * 64, 0, g.bd, 0, 0, &r->q_luma) != RV_OK ||
      rv_quant_ctx(kReplayQindex, 32 * 32, 0, g.bd, 0, 0, &r->q_chroma) != RV_OK) {
    delete r;
    return nullptr;
  }
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
  r->slots.resize(g.R + 1);
  for (auto &s : r->slots) ok = ok && alloc_slot(r, s);
  // tall scratch planes: candidate c of superblock (sx, sy) at
  // (sx * bw, (c * th + sy) * bh)
  size_t by = rv_plane_geometry(&r->tall_y, g.tw * kSb, g.C * g.th * kSb, 0, 0, 0, 0, g.hbd);
  size_t bu = rv_plane_geometry(&r->tall_u, g.tw * g.cw, g.C * g.th * g.ch, g.xdec, g.ydec, 0, 0,
                                g.hbd);
  r->tall_v = r->tall_u;
  r->tall_y.data = dalloc(r, by);
  r->tall_u.data = dalloc(r, bu);
  r->tall_v.data = dalloc(r, bu);
  const int ntx_c = (g.cw / 32) * (g.ch / 32);
  const int nr = g.nsb * g.R;
  r->coarse = (rv_fs_result *)dalloc(r, nr * sizeof(rv_fs_result));
  r->half = (rv_fs_result *)dalloc(r, nr * sizeof(rv_fs_result));
  r->full = (rv_fs_result *)dalloc(r, nr * sizeof(rv_fs_result));
  r->sub = (rv_fs_result *)dalloc(r, nr * sizeof(rv_fs_result));
  r->l_packed = (int32_t *)dalloc(r, (size_t)g.nctx * 1024 * 4);
  r->c_packed = (int32_t *)dalloc(r, (size_t)g.nctx * ntx_c * 1024 * 4 * 2);
  r->lsub = (kSb / 8) * (kSb / 8);
  {
    const int bw = (g.cw < 8 ? g.cw : 8) >> g.xdec, bh = (g.ch < 8 ? g.ch : 8) >> g.ydec;
    r->csub = (g.cw / bw) * (g.ch / bh);
  }
  r->l_mom = (int64_t *)dalloc(r, (size_t)g.nctx * r->lsub * 5 * 8);
  r->u_sse = (uint64_t *)dalloc(r, (size_t)g.nctx * r->csub * 8);
  r->v_sse = (uint64_t *)dalloc(r, (size_t)g.nctx * r->csub * 8);
  r->words = (uint64_t *)dalloc(r, (size_t)g.nsb * (8 * g.R + 2) * 8);
  r->imp_bx = vis_w / 8;
  r->imp_by = vis_h / 8;
  r->n_imp = r->imp_bx * r->imp_by;
  r->tail = (unsigned long long *)dalloc(r, 4 * 8);
  for (int f = 0; f < rv_replay::kRing; f++) {
    for (int i = 0; i < rv_replay::kEv; i++)
      ok = ok && hipEventCreateWithFlags(&r->evs[f][i], hipEventDisableSystemFence) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&r->fork[f], hipEventDisableTiming) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&r->join[f], hipEventDisableTiming) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&r->fork2[f], hipEventDisableTiming) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&r->join2[f], hipEventDisableTiming) == hipSuccess;
  }
  ok = ok && hipStreamCreateWithFlags(&r->side, hipStreamNonBlocking) == hipSuccess;
  const size_t ev_bytes = (size_t)rv_replay::kRing * 2 * nr * 4;
  r->ds_evals = (uint32_t *)dalloc(r, ev_bytes);
  ok = ok && r->ds_evals && hipMemsetAsync(r->ds_evals, 0, ev_bytes, r->stream) == hipSuccess;
  ok = ok && r->tall_y.data && r->tall_u.data && r->tall_v.data && r->tail;
  if (!ok || build_static_jobs(r) != RV_OK) {
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

static int upload_plane(rv_replay *r, const rv_plane &p, const uint8_t *src) {
  const int px = p.hbd ? 2 : 1;
  uint8_t *dst = (uint8_t *)p.data + ((size_t)p.yorigin * p.stride + p.xorigin) * px;
  RV_H(hipMemcpy2DAsync(dst, (size_t)p.stride * px, src, (size_t)p.width * px,
                        (size_t)p.width * px, p.height, hipMemcpyHostToDevice, r->stream));
  return rv_plane_pad(&p, r->stream);
}

int rv_replay_set_frame(rv_replay *r, int slot, const void *host_yuv) {
  if (!r || !host_yuv || slot < 0 || slot > r->g.R)
    return rv_set_error(RV_EINVAL, "rv_replay_set_frame: bad slot");
  RvFrameSlot &s = r->slots[slot];
  const int px = r->g.hbd ? 2 : 1;
  const uint8_t *p = (const uint8_t *)host_yuv;
  RV_R(upload_plane(r, s.y, p));
  p += (size_t)s.y.width * s.y.height * px;
  RV_R(upload_plane(r, s.u, p));
  p += (size_t)s.u.width * s.u.height * px;
  RV_R(upload_plane(r, s.v, p));
  RV_R(rv_plane_pyramid(&s.y, &s.hres, &s.qres, r->stream));
  if (r->sea) RV_R(rv_plane_box_sums(&s.qres, s.qres_box, r->stream));
  RV_H(hipStreamSynchronize(r->stream));
  return RV_OK;
}

// Event layout per frame (ring slot): e[0..6] = stage bounds F0..F5 end;
// e[7] splits F3 between the full-pel and the sub-pel diamond launch, e[8]
// splits F4 between the fused candidate launch and the scoring launch.
// Every stage is one launch except those two, so the stage bounds are also
// the kernel brackets.  The events are created without the system-scope
// fence (they only time).
int rv_replay_frame(rv_replay *r, int me_range_scale) {
  if (!r || (me_range_scale != 1 && me_range_scale != 2 && me_range_scale != 4))
    return rv_set_error(RV_EINVAL, "rv_replay_frame: bad me_range_scale");
  const Geo &g = r->g;
  hipStream_t st = r->stream;
  RvFrameSlot &cur = r->slots[0];
  const int nr = g.nsb;  // jobs per reference
  const int si = me_range_scale == 1 ? 0 : me_range_scale == 2 ? 1 : 2;
  rv_plane refs_y[RV_DS_MAX_PRED], refs_h[RV_DS_MAX_PRED], refs_q[RV_DS_MAX_PRED];
  for (int k = 0; k < g.R; k++) {
    refs_y[k] = r->slots[1 + k].y;
    refs_h[k] = r->slots[1 + k].hres;
    refs_q[k] = r->slots[1 + k].qres;
  }
  const int slot = (int)(r->frames % rv_replay::kRing);
  uint32_t *ev_full = r->ds_evals + (size_t)slot * 2 * nr * g.R;
  uint32_t *ev_sub = ev_full + (size_t)nr * g.R;
  ChainNext to_half{}, to_full{}, to_sub{}, to_mc{};
  to_half.mode = kChainCoarseToHalf;
  to_half.jobs = r->jobs_half;
  to_full.mode = kChainHalfToFull;
  to_full.jobs = r->jobs_full;
  to_sub.mode = kChainFullToSub;
  to_sub.jobs = r->jobs_sub;
  to_mc.mode = kChainSubToMc;
  to_mc.l_mc = r->l_mc;
  to_mc.c_mc = r->c_mc;
  to_mc.luma = cur.y;
  to_mc.chroma = cur.u;
  to_mc.tw = g.tw;
  to_mc.th = g.th;
  to_mc.tx0 = g.tx0;
  to_mc.ty0 = g.ty0;
  to_mc.cw = g.cw;
  to_mc.ch = g.ch;

  const bool tm = r->timing_stride > 0 && (r->frames / r->timing_block) % r->timing_stride == 0;
  const int tslot = (int)(r->timed % rv_replay::kRing);
  hipEvent_t *e = r->evs[tslot];
  r->ev = e;
  r->frames++;
  if (tm) r->timed++;
#define RV_EV(i, stream)                                 \
  do {                                                   \
    if (tm) RV_H(hipEventRecord(e[i], (stream)));        \
  } while (0)
  RV_EV(0, st);
  // F4 zero-MV candidates need no motion search: they run on the side
  // stream concurrently with F0-F3 (rav1e evaluates them in the same RDO
  // loop, src/rdo.rs:949-1006; only the order of independent work changes)
  const int ntx_c = (g.cw / 32) * (g.ch / 32);
  const int nct = g.nctx * ntx_c;
  RdoArgs la, ca;
  {
    memset(&la, 0, sizeof(la));
    la.p[0].org = cur.y;
    for (int k = 0; k < g.R; k++) la.p[0].ref[k] = r->slots[1 + k].y;
    la.p[0].dst = r->tall_y;
    la.p[0].mc = r->l_mc;
    la.p[0].tx = r->l_tx;
    la.p[0].packed = r->l_packed;
    la.p[0].dist = r->l_mom;
    la.n_tx = g.nctx / 2;  // one candidate kind per launch
    la.ntx_per_cand = 1;
    la.cands_per_ref = 2 * nr;
    la.nsb = nr;
    la.bd = g.bd;
    la.mb_w = la.mb_h = kSb;
    la.sub_w = la.sub_h = 8;
    la.q = r->q_luma;
    la.q_tx_index = 4 * 16 + 0;  // TX_64X64, DCT_DCT
    ca = la;
    ca.q = r->q_chroma;
    ca.q_tx_index = 3 * 16 + 0;  // TX_32X32, DCT_DCT
    const rv_plane *cp[2] = {&cur.u, &cur.v};
    const rv_plane *tp[2] = {&r->tall_u, &r->tall_v};
    uint64_t *cs[2] = {r->u_sse, r->v_sse};
    for (int p = 0; p < 2; p++) {
      ca.p[p].org = *cp[p];
      for (int k = 0; k < g.R; k++) ca.p[p].ref[k] = p ? r->slots[1 + k].v : r->slots[1 + k].u;
      ca.p[p].dst = *tp[p];
      ca.p[p].mc = r->c_mc;
      ca.p[p].tx = r->c_tx;
      ca.p[p].packed = r->c_packed + (size_t)p * nct * 1024;
      ca.p[p].dist = cs[p];
    }
    ca.n_tx = nct / 2;
    ca.ntx_per_cand = ntx_c;
    ca.mb_w = g.cw;
    ca.mb_h = g.ch;
    ca.sub_w = (g.cw < 8 ? g.cw : 8) >> g.xdec;
    ca.sub_h = (g.ch < 8 ? g.ch : 8) >> g.ydec;
  }
  const bool serial = (r->cfg.flags & RV_REPLAY_SIDE_RDO) == 0;
  if (!serial) {
    RV_H(hipEventRecord(r->fork[slot], st));
    RV_H(hipStreamWaitEvent(r->side, r->fork[slot], 0));
    la.k_sel = ca.k_sel = 1;
    RV_EV(9, r->side);
    RV_R(rv_rdo_candidates(la, ca, g.hbd, r->side));
    RV_EV(10, r->side);
    RV_H(hipEventRecord(r->join[slot], r->side));
  }
  // F0 hres + qres of the input (encode_frame, src/encoder.rs:3382-3385)
  RV_R(rv_plane_pyramid(&cur.y, &cur.hres, &cur.qres, st));
  // box sums of the input's qres: the table this frame's coarse search
  // needs once it is a reference (one per frame in a real encode; the
  // replay's references are fixed, so it is computed and not consumed)
  if (r->sea) RV_R(rv_plane_box_sums(&cur.qres, cur.qres_box, st));
  RV_EV(1, st);
  // F1 coarse full search, every reference in one launch -> F2 predictors
  const uint32_t *box[RV_DS_MAX_PRED];
  for (int k = 0; k < g.R; k++) box[k] = r->slots[1 + k].qres_box;
  RV_R(rv_full_search_multi(&cur.qres, refs_q, g.R, r->fs_jobs[si], nr, 16, 16, 1, 0, r->coarse,
                            &to_half, r->sea ? box : nullptr, st));
  RV_EV(2, st);
  // F2 half-res diamond -> F3 full-pel predictors
  RV_R(rv_diamond_search_multi(&cur.hres, refs_h, g.R, r->jobs_half, nr, 32, 32, 0, 0, 0, g.bd,
                               r->half, nullptr, &to_full, st));
  RV_EV(3, st);
  // F3 full-res full-pel diamond -> sub-pel predictor; sub-pel diamond
  // (speed 10: SAD, no hp) -> the F4 MC jobs of the sub-pel candidates
  RV_R(rv_diamond_search_multi(&cur.y, refs_y, g.R, r->jobs_full, nr, 64, 64, 0, 0, 0, g.bd,
                               r->full, ev_full, &to_sub, st));
  RV_EV(7, st);
  RV_R(rv_diamond_search_multi(&cur.y, refs_y, g.R, r->jobs_sub, nr, 64, 64, 1, 0, 0, g.bd,
                               r->sub, ev_sub, &to_mc, st));
  RV_EV(4, st);
  // F4 sub-pel MV candidates (all candidates when serial): luma + both
  // chroma planes in one fused launch
  if (serial) {
    la.k_sel = ca.k_sel = -1;
    la.n_tx *= 2;
    ca.n_tx *= 2;
  } else {
    la.k_sel = ca.k_sel = 0;
  }
  const bool split = serial && (r->cfg.flags & RV_REPLAY_SPLIT_RDO) != 0;
  if (split) {  // luma here, chroma pairs concurrently on the side stream
    RV_H(hipEventRecord(r->fork2[slot], st));
    RV_H(hipStreamWaitEvent(r->side, r->fork2[slot], 0));
    RV_R(rv_rdo_candidates(la, ca, g.hbd, st, r->side));
    RV_H(hipEventRecord(r->join2[slot], r->side));
    RV_H(hipStreamWaitEvent(st, r->join2[slot], 0));
  } else {
    RV_R(rv_rdo_candidates(la, ca, g.hbd, st));
  }
  RV_EV(8, st);
  if (tm) r->ev_side[tslot] = !serial;
  if (serial) {
  } else {
    RV_H(hipStreamWaitEvent(st, r->join[slot], 0));
  }
  score_candidates<<<g.nsb, 64, 0, st>>>(g, r->l_mom, r->u_sse, r->v_sse, r->lsub, r->csub,
                                         r->coarse, r->half, r->full, r->sub, r->words,
                                         r->tail + 2);
  RV_EV(5, st);
  // F5 importance SATD against reference 1
  {
    const unsigned nb = (unsigned)((r->n_imp + 255) / 256);
    if (g.hbd)
      importance_kernel<uint16_t><<<nb, 256, 0, st>>>(g, cur.y, r->slots[1].y, r->sub, r->imp_bx,
                                                      r->imp_by, r->tail + 2);
    else
      importance_kernel<uint8_t><<<nb, 256, 0, st>>>(g, cur.y, r->slots[1].y, r->sub, r->imp_bx,
                                                     r->imp_by, r->tail + 2);
  }
  RV_EV(6, st);
#undef RV_EV
  RV_H(hipGetLastError());
  return RV_OK;
}

int rv_replay_results(rv_replay *r, uint64_t *host_out, int cap) {
  if (!r || !host_out) return rv_set_error(RV_EINVAL, "rv_replay_results: null");
  const Geo &g = r->g;
  const int nw = g.nsb * (8 * g.R + 2);
  const int total = nw + 4;
  if (cap < total) return rv_set_error(RV_EINVAL, "rv_replay_results: cap too small");
  // verification checksums of the last frame (outside the per-frame work)
  hipStream_t st = r->stream;
  const int ntx_c = (g.cw / 32) * (g.ch / 32);
  const int64_t nl = (int64_t)g.nctx * 1024, nc = (int64_t)g.nctx * ntx_c * 1024;
  RV_H(hipMemsetAsync(r->tail, 0, 2 * 8, st));
  coeff_checksum<<<1024, 256, 0, st>>>(r->l_packed, nl, 1024, r->tail);
  coeff_checksum<<<1024, 256, 0, st>>>(r->c_packed, 2 * nc, 1024, r->tail);
  const rv_plane *tp[3] = {&r->tall_y, &r->tall_u, &r->tall_v};
  for (int i = 0; i < 3; i++) {
    if (g.hbd)
      sum_plane<uint16_t><<<1024, 256, 0, st>>>(*tp[i], tp[i]->width, tp[i]->height, r->tail + 1);
    else
      sum_plane<uint8_t><<<1024, 256, 0, st>>>(*tp[i], tp[i]->width, tp[i]->height, r->tail + 1);
  }
  RV_H(hipGetLastError());
  RV_H(hipMemcpyAsync(host_out, r->words, (size_t)nw * 8, hipMemcpyDeviceToHost, r->stream));
  RV_H(hipMemcpyAsync(host_out + nw, r->tail, 3 * 8, hipMemcpyDeviceToHost, r->stream));
  RV_H(hipStreamSynchronize(r->stream));
  host_out[nw + 3] = (uint64_t)r->n_imp;
  return total;
}

static int stage_times(rv_replay *r, float *ms_out, int cap, int last) {
  if (!r || !ms_out) return rv_set_error(RV_EINVAL, "rv_replay_stage_times: null");
  if (r->timed == 0) return rv_set_error(RV_EINVAL, "rv_replay_stage_times: no timed frame");
  if (last < 1) last = 1;
  if (last > rv_replay::kRing) last = rv_replay::kRing;
  if (last > r->timed) last = (int)r->timed;
  for (int i = 0; i < cap && i < 10; i++) ms_out[i] = 0.f;
  int n = 0;
  for (int f = 0; f < last; f++) {
    const int ts = (int)((r->timed - 1 - f) % rv_replay::kRing);
    hipEvent_t *e = r->evs[ts];
    RV_H(hipEventSynchronize(e[6]));
    n = 0;
    for (int i = 0; i < 6 && n < cap; i++) {  // stages F0..F5
      float ms = 0.f;
      RV_H(hipEventElapsedTime(&ms, e[i], e[i + 1]));
      ms_out[n++] += ms;
    }
    // kernel brackets: F3 full-pel diamond, F3 sub-pel diamond, F4 fused
    // sub-pel MV candidates (main stream), F4 fused zero-MV candidates
    // (side stream, concurrent with F0-F3)
    const int br[4][2] = {{3, 7}, {7, 4}, {4, 8}, {9, 10}};
    for (int i = 0; i < 4 && n < cap; i++) {
      float ms = 0.f;
      if (i < 3 || r->ev_side[ts]) RV_H(hipEventElapsedTime(&ms, e[br[i][0]], e[br[i][1]]));
      ms_out[n++] += ms;
    }
  }
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
// Diamond-search candidate evaluations summed over the last min(frames, 64)
// frames: out[0] F3 full-pel, out[1] F3 sub-pel, out[2] frames summed.
int rv_replay_counters(rv_replay *r, uint64_t *out, int cap) {
  if (!r || !out || cap < 3) return rv_set_error(RV_EINVAL, "rv_replay_counters");
  const Geo &g = r->g;
  const int nj = g.nsb * g.R;
  const int nf = r->frames < rv_replay::kRing ? (int)r->frames : rv_replay::kRing;
  RV_H(hipStreamSynchronize(r->stream));
  std::vector<uint32_t> h((size_t)nf * 2 * nj);
  if (nf) RV_H(hipMemcpy(h.data(), r->ds_evals, h.size() * 4, hipMemcpyDeviceToHost));
  out[0] = out[1] = 0;
  for (int f = 0; f < nf; f++)
    for (int k = 0; k < 2; k++)
      for (int j = 0; j < nj; j++) out[k] += h[((size_t)f * 2 + k) * nj + j];
  out[2] = (uint64_t)nf;
  return 3;
}

}  // extern "C"
