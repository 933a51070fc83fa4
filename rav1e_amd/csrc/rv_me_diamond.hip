// rv_me_diamond.hip -- batched diamond motion search (gfx950).
//
// diamond_me_search (src/me.rs:693-785) with get_best_predictor
// (:655-691), get_mv_rd_cost (:787-838) and compute_mv_rd_cost (:840-856):
// the whole data-dependent search of a block runs inside one workgroup, so
// a tile's blocks advance in parallel with no host round trip per step.
//
// Fast path (SAD, u8/u16, block widths 16/32/64): a workgroup is 4
// wavefronts and every wavefront evaluates one candidate on its own, so the
// 4 points of a diamond step (and up to 4 predictors) run concurrently;
// the step's winner is chosen from LDS in pattern order with the
// reference's strict `<` (first minimum), exactly as the sequential loop.
//  * full-pel: the source block lives in VGPRs (16-byte row chunks); a
//    candidate is 16-byte unaligned loads of the reference block + v_sad_u8
//    / v_sad_u16 + one wave reduction.
//  * sub-pel: predict_inter's put_8tap (src/predict.rs:255-338, REGULAR,
//    PlaneSlice::clamp) runs per wavefront: the (h+7) x (w+7) window is
//    staged in a wave-private LDS slab, lane = output column; the
//    horizontal 8-tap is two v_dot4_i32_i8 (u8, pixels biased by -128) or
//    four v_dot2_i32_i16 (u16), the vertical 8-tap a register ring of the
//    i16 intermediates, and |org - pred| accumulates in registers -- the
//    prediction never leaves the wavefront.
// SATD and square blocks of 8 and 16: ds_grp_kernel (lane groups per job).
// Anything else takes the generic workgroup-per-candidate kernel.
#include <algorithm>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rv_chain.h"
#include "rv_device.h"

namespace rv {

constexpr int kDsThreads = 256;
constexpr int kDsWaves = kDsThreads / 64;

// SUBPEL_FILTERS REGULAR sets (src/mc.rs:70-179): index 0 = 8-tap
// REGULAR, 1 = 4-tap REGULAR (get_filter for length <= 4, src/mc.rs:201-210)
__constant__ int8_t kReg[2][16][8] = {
    {{0, 0, 0, 127, 0, 0, 0, 0}, {0, 2, -6, 126, 8, -2, 0, 0},
     {0, 2, -10, 122, 18, -4, 0, 0}, {0, 2, -12, 116, 28, -8, 2, 0},
     {0, 2, -14, 110, 38, -10, 2, 0}, {0, 2, -14, 102, 48, -12, 2, 0},
     {0, 2, -16, 94, 58, -12, 2, 0}, {0, 2, -14, 84, 66, -12, 2, 0},
     {0, 2, -14, 76, 76, -14, 2, 0}, {0, 2, -12, 66, 84, -14, 2, 0},
     {0, 2, -12, 58, 94, -16, 2, 0}, {0, 2, -12, 48, 102, -14, 2, 0},
     {0, 2, -10, 38, 110, -14, 2, 0}, {0, 2, -8, 28, 116, -12, 2, 0},
     {0, 0, -4, 18, 122, -10, 2, 0}, {0, 0, -2, 8, 126, -6, 2, 0}},
    {{0, 0, 0, 127, 0, 0, 0, 0}, {0, 0, -4, 126, 8, -2, 0, 0},
     {0, 0, -8, 122, 18, -4, 0, 0}, {0, 0, -10, 116, 28, -6, 0, 0},
     {0, 0, -12, 110, 38, -8, 0, 0}, {0, 0, -12, 102, 48, -10, 0, 0},
     {0, 0, -14, 94, 58, -10, 0, 0}, {0, 0, -12, 84, 66, -10, 0, 0},
     {0, 0, -12, 76, 76, -12, 0, 0}, {0, 0, -10, 66, 84, -12, 0, 0},
     {0, 0, -10, 58, 94, -14, 0, 0}, {0, 0, -10, 48, 102, -12, 0, 0},
     {0, 0, -8, 38, 110, -12, 0, 0}, {0, 0, -6, 28, 116, -10, 0, 0},
     {0, 0, -4, 18, 122, -8, 0, 0}, {0, 0, -2, 8, 126, -4, 0, 0}}};

// get_mv_rate's diff_to_rate (src/me.rs:1006-1021)
__device__ __forceinline__ uint32_t ds_diff_to_rate(int16_t diff, int hp) {
  int16_t d = hp ? diff : (int16_t)(diff >> 1);
  if (d == 0) return 0;
  uint32_t a = (uint16_t)(d < 0 ? -d : d);
  return 2u * (16u - (uint32_t)(__builtin_clz(a) - 16));
}

// compute_mv_rd_cost (src/me.rs:840-856) given the distortion
__device__ __forceinline__ uint64_t ds_cost(uint32_t dist, rv_mv mv, const rv_ds_job &jb,
                                            int hp) {
  const uint32_t r1 = ds_diff_to_rate((int16_t)(mv.row - jb.pmv[0].row), hp) +
                      ds_diff_to_rate((int16_t)(mv.col - jb.pmv[0].col), hp);
  const uint32_t r2 = ds_diff_to_rate((int16_t)(mv.row - jb.pmv[1].row), hp) +
                      ds_diff_to_rate((int16_t)(mv.col - jb.pmv[1].col), hp);
  const uint32_t rate = r1 < r2 + 1 ? r1 : r2 + 1;
  return 256ull * dist + (uint64_t)rate * jb.lambda;
}

__device__ __forceinline__ bool ds_in_range(rv_mv mv, const rv_ds_job &jb) {
  return !(mv.col < jb.mvx_min || mv.col > jb.mvx_max || mv.row < jb.mvy_min ||
           mv.row > jb.mvy_max);
}

// blockIdx -> job with consecutive jobs on one XCD (blocks are dealt to
// the 8 XCDs round-robin): neighbouring superblocks share reference rows
// in that XCD's L2.  The grid is rounded up to a multiple of 8.
__device__ __forceinline__ int xcd_job(int n) {
  const int per = (int)gridDim.x >> 3;
  return ((int)blockIdx.x & 7) * per + ((int)blockIdx.x >> 3);
}

struct DsArgs {
  rv_plane org;
  rv_plane ref[RV_MAX_REFS];  // reference of job i = ref[i / n_per_ref]
  const rv_ds_job *jobs;
  rv_fs_result *out;
  int n, n_per_ref, w, h, subpel, satd, hp, bd;
  uint32_t *evals;  // optional: in-range candidate evaluations per job
  // optional (ds_fast_kernel): [0] += the launch's candidate evaluations,
  // [1] += its jobs -- the bench's kernel probe (algorithmic bytes per launch)
  uint32_t *eval_acc;
  // optional (ds_fast_kernel, the kernel probe): the launch's span on the
  // device clock -- every workgroup's first instruction min'd into t0, its
  // last max'd into t1 (wall_clock64 ticks)
  unsigned long long *t0, *t1;
  ChainNext next;   // replay: feed the winner into the next stage's jobs
  int tele;         // 1: telescopic_subpel_search instead of the diamond
  const rv_fs_result *start;  // tele: the search's start (best_mv, lowest_cost)
  // replay rounds: only jobs j with active[j % n_per_ref] set run (null: all)
  const uint8_t *active;
  // replay rounds after the first: the jobs a round's check listed; the
  // grid is a fixed pool of workgroups that loops over them.  lper > 0:
  // alist[0 .. *acount) are superblocks, each with lper consecutive jobs
  // per reference (job = r * n_per_ref + sb * lper + e); lper = 0: alist
  // holds job indices
  const int32_t *alist;
  const int32_t *acount;
  int lper;
  // list-driven rounds: a listed job with dirty[job] == 0 keeps its result
  // (its inputs did not change; null: every listed job runs)
  const uint8_t *dirty;
  // list-driven: the workgroup pool (0: ds_list_grid(); a round expected to
  // list most jobs, e.g. the first after round 0, asks for a full grid)
  int list_grid;
  // RAV1E_HIP_DS_PHASES=1 (diagnostic): list-driven sub-pel jobs add their
  // phase times (wall_clock64 ticks on thread 0) into g_ds_ph
  int ph;
};

// [0] setup (job record, source block to LDS), [1] window staging + filter
// + SAD, [2] the cost exchange, [3] whole job, [4] diamond iterations,
// [5] jobs, [6] window re-stagings, [7] workgroup spans, [8] workgroups
__device__ unsigned long long g_ds_ph[16];

// The ordinal-th job of a list-driven launch (its size: ds_list_total)
__device__ __forceinline__ int ds_list_total(const DsArgs &a) {
  const int cnt = __builtin_amdgcn_readfirstlane(*a.acount);
  return a.lper ? cnt * a.lper * (a.n / a.n_per_ref) : cnt;
}
__device__ __forceinline__ int ds_list_job(const DsArgs &a, int ord) {
  if (!a.lper) return a.alist[ord];
  const int cnt = *a.acount, per = cnt * a.lper;
  const int r = ord / per, rem = ord - r * per, i = rem / a.lper;
  return r * a.n_per_ref + a.alist[i] * a.lper + (rem - i * a.lper);
}

// Workgroups of a list-driven launch: enough to cover a typical round's
// superblocks at once, few enough that a near-empty round costs ~1 us of
// dispatch (a full 4080-workgroup grid of early exits costs ~10 us).
constexpr int kDsListGridDefault = 512;
// RAV1E_HIP_DS_POOL (A/B): the list-driven launches' workgroup pool
static int ds_list_grid() {
  static const int g = [] {
    const char *e = getenv("RAV1E_HIP_DS_POOL");
    const int v = e ? atoi(e) : kDsListGridDefault;
    return v > 0 ? v : kDsListGridDefault;
  }();
  return g;
}

__device__ __forceinline__ void ds_write(const DsArgs &a, int job, rv_mv center,
                                         uint64_t cost) {
  rv_fs_result r;
  r.best_mv = center;
  r.reserved = 0;
  r.cost = cost;
  a.out[job] = r;
}

// ============================ fast path ====================================
// 16-byte chunk helpers: 16 u8 or 8 u16 pixels
__device__ __forceinline__ uint4 ld16(const void *p) {
  uint4 v;
  __builtin_memcpy(&v, p, 16);  // unaligned global_load_dwordx4
  return v;
}
template <typename Px>
__device__ __forceinline__ uint32_t sad16(uint4 a, uint4 b, uint32_t acc) {
  if constexpr (sizeof(Px) == 1) {
    acc = __builtin_amdgcn_sad_u8(a.x, b.x, acc);
    acc = __builtin_amdgcn_sad_u8(a.y, b.y, acc);
    acc = __builtin_amdgcn_sad_u8(a.z, b.z, acc);
    return __builtin_amdgcn_sad_u8(a.w, b.w, acc);
  } else {
    acc = __builtin_amdgcn_sad_u16(a.x, b.x, acc);
    acc = __builtin_amdgcn_sad_u16(a.y, b.y, acc);
    acc = __builtin_amdgcn_sad_u16(a.z, b.z, acc);
    return __builtin_amdgcn_sad_u16(a.w, b.w, acc);
  }
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) { return group_sum<64>(v); }

// Full-pel layout: K 16-byte chunks per block row, R rows per wave
// instruction, I instructions per block.
template <typename Px, int W, int H>
struct FullGeo {
  static constexpr int K = W * (int)sizeof(Px) / 16;
  static constexpr int R = 64 / K;
  static constexpr int I = (H + R - 1) / R;
  static constexpr bool kPartial = (R * I != H);
};

// Sub-pel layout: lane = column c (lane % W), row group g = lane / W of
// RG = H / (64 / W) output rows; the wave-private LDS window is (H + 7)
// rows x P bytes.
template <typename Px, int W, int H>
struct SubGeo {
  static constexpr int G = 64 / W;
  static constexpr int RG = H / G;
  static constexpr int P = sizeof(Px) == 1 ? ((W + 8 + 15) / 16) * 16
                                           : ((2 * (W + 8) + 15) / 16) * 16;
  static constexpr int kWinDwords = (H + 7) * P / 4;
  static constexpr int kOrgDwords = RG * (int)sizeof(Px) / 4;
  // staged window: D px of slack in each direction around the candidates'
  // integer origins, so successive rounds of a search (which stay within a
  // pixel or two) reuse it; pitch UP bytes (+3 px for the dword over-read of
  // the horizontal pass)
  static constexpr int D = 8;
  static constexpr int UP = (((W + 7 + D + 4) * (int)sizeof(Px)) + 15) / 16 * 16;
  static constexpr int kUnionDwords = (H + 7 + D) * UP / 4;
};

// |org - put_8tap| of one lane's column over RG output rows, read from a
// staged window (pitch UP bytes, `win` = the candidate's row -3, `cx` = the
// lane's window column of its output's -3 tap; u8 windows are stored with
// every byte XOR 0x80, i.e. as i8 = pixel - 128, for v_dot4_i32_i8).
// HF / VF: horizontal / vertical filtering active (frac != 0), fixed per
// candidate so the row loop carries no per-row branches (src/mc.rs:232-307
// cases (x,y), (x,0), (0,y), (0,0)).  The vertical 8-tap runs as four
// v_dot2_i32_i16 over a ring of packed (m[j], m[j+1]) intermediate pairs.
// Range: every intermediate fits i16 for REGULAR taps at 8/10/12 bits
// (max 4095 * 136 >> 5), so the reference's `as i16` is the identity here.
template <typename Px, int W, int RG, int UP, bool HF, bool VF>
__device__ __forceinline__ uint32_t sub_sad_rows(const uint32_t *win, const Px *ocol, int cx,
                                                 int grp, const int8_t *xf, const int8_t *yf,
                                                 int ib, int maxv) {
  constexpr int B = (int)sizeof(Px);
  constexpr int PD = UP / 4;  // window pitch in dwords
  uint32_t xp[4] = {0, 0, 0, 0};  // u8: 2 x i8x4; u16: 3 x i16x2
  int xsum = 0;
  if constexpr (HF) {
    if constexpr (B == 1) {
#pragma unroll
      for (int h = 0; h < 2; h++)
        xp[h] = (uint32_t)(uint8_t)xf[4 * h] | ((uint32_t)(uint8_t)xf[4 * h + 1] << 8) |
                ((uint32_t)(uint8_t)xf[4 * h + 2] << 16) | ((uint32_t)(uint8_t)xf[4 * h + 3] << 24);
#pragma unroll
      for (int k = 0; k < 8; k++) xsum += xf[k];
    } else {
#pragma unroll
      for (int h = 0; h < 3; h++)  // taps 1..6 as pairs (taps 0 and 7 are zero)
        xp[h] = (uint32_t)(uint16_t)(int16_t)xf[2 * h + 1] |
                ((uint32_t)(uint16_t)(int16_t)xf[2 * h + 2] << 16);
    }
  }
  // REGULAR taps 0 and 7 are zero for every fraction (src/mc.rs:71-88; the
  // 4-tap set also zeroes 1 and 6), so the vertical pass is three v_dot2
  // over the pairs (1,2), (3,4), (5,6) and window rows 0 and h+6 are never
  // filtered.
  uint32_t tp[3] = {0, 0, 0};  // vertical taps 1..6 as i16 pairs
  if constexpr (VF) {
#pragma unroll
    for (int h = 0; h < 3; h++)
      tp[h] = (uint32_t)(uint16_t)(int16_t)yf[2 * h + 1] |
              ((uint32_t)(uint16_t)(int16_t)yf[2 * h + 2] << 16);
  }
  const int hbias = 128 * xsum;
  const int hround = (1 << (7 - ib)) >> 1, hsh = 7 - ib;
  const uint32_t *base = win + grp * RG * PD;
  // horizontal value of window row t at this lane's column: the 8-tap sum
  // rounded to the intermediate (HF), or the pixel under tap 3
  auto hval = [&](int t) __attribute__((always_inline)) -> int32_t {
    const uint32_t *row = base + t * PD;
    if constexpr (B == 1) {
      if constexpr (!HF) {
        return (int32_t)(reinterpret_cast<const uint8_t *>(row)[cx + 3] ^ 0x80u);
      } else {
        const int d0 = cx >> 2, sh = cx & 3;
        const uint32_t w0 = row[d0], w1 = row[d0 + 1], w2 = row[d0 + 2];
        int32_t s = dot4_i8(__builtin_amdgcn_alignbyte(w1, w0, sh), xp[0], hbias + hround);
        s = dot4_i8(__builtin_amdgcn_alignbyte(w2, w1, sh), xp[1], s);
        return s >> hsh;
      }
    } else {
      if constexpr (!HF) {
        return (int32_t)reinterpret_cast<const uint16_t *>(row)[cx + 3];
      } else {
        const int c1 = cx + 1, d0 = c1 >> 1, sh = (c1 & 1) * 2;  // pixels cx+1 .. cx+6
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; k++) w[k] = row[d0 + k];
        int32_t s = hround;
#pragma unroll
        for (int k = 0; k < 3; k++) s = dot2_i16(__builtin_amdgcn_alignbyte(w[k + 1], w[k], sh), xp[k], s);
        return s >> hsh;
      }
    }
  };
  auto absdiff_acc = [](uint32_t a, uint32_t b, uint32_t acc) __attribute__((always_inline)) {
    return (a > b ? a - b : b - a) + acc;  // v_sad_u32
  };
  uint32_t acc = 0;
  if constexpr (!VF) {
    // (x,0): round_shift(intermediate, ib); (0,0): the pixel itself
#pragma unroll 8
    for (int r = 0; r < RG; r++) {
      int32_t v = hval(r + 3);
      if constexpr (HF) v = clamp_med3(round_shift(v, ib), 0, maxv);
      acc = absdiff_acc((uint32_t)ocol[r * W], (uint32_t)v, acc);
    }
  } else {
    const int vshift = HF ? 7 + ib : 7;
    const int vround = (1 << vshift) >> 1;
    auto pack = [](int32_t lo, int32_t hi) __attribute__((always_inline)) {
      return __builtin_amdgcn_perm((uint32_t)hi, (uint32_t)lo, 0x05040100u);
    };
    uint32_t pr[8];  // pr[j & 7] = (m[j], m[j + 1])
    int32_t prev = hval(1);
#pragma unroll
    for (int t = 2; t < 6; t++) {
      const int32_t m = hval(t);
      pr[t - 1] = pack(prev, m);
      prev = m;
    }
    pr[0] = pr[5] = pr[6] = pr[7] = 0;
#pragma unroll 1
    for (int r0 = 0; r0 < RG; r0 += 8) {
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int r = r0 + u;
        const int32_t m = hval(r + 6);
        pr[(u + 5) & 7] = pack(prev, m);
        prev = m;
        int32_t s = vround;
#pragma unroll
        for (int k = 0; k < 3; k++) s = dot2_i16(pr[(u + 2 * k + 1) & 7], tp[k], s);
        const int v = clamp_med3(s >> vshift, 0, maxv);
        acc = absdiff_acc((uint32_t)ocol[r * W], (uint32_t)v, acc);
      }
    }
  }
  return acc;
}

template <typename Px, int W, int H, bool SUB>
struct DsFast {
  using F = FullGeo<Px, W, H>;
  using S = SubGeo<Px, W, H>;
  static constexpr int kOrgRegs = SUB ? 1 : 4 * F::I;
};

// Returns the search's result MV (uniform).  pred0 (optional): the job's
// first predictor, in place of jobs[job].pred[0] (the fused F3 path hands
// its full-pel winner over without a round trip through memory).
template <typename Px, int W, int H, bool SUB>
__device__ __forceinline__ rv_mv ds_fast_body(const DsArgs &a, const int job, bool has_pred0 = false,
                                              rv_mv pred0 = rv_mv{0, 0}) {
  using F = FullGeo<Px, W, H>;
  using S = SubGeo<Px, W, H>;
  constexpr int B = (int)sizeof(Px);
  static_assert(!SUB || S::RG % 8 == 0, "sub-pel row groups are unrolled by 8");
  __shared__ uint64_t scost[2][kDsWaves];
  __shared__ uint32_t wevals[kDsWaves];
  __shared__ uint32_t win_all[SUB ? S::kUnionDwords : 1];
  __shared__ Px org_lds[SUB ? W * H : 1];  // sub-pel: the source block, shared by all waves

  const bool ph = SUB && a.ph && threadIdx.x == 0;
  const unsigned long long ph_t0 = ph ? wall_clock64() : 0;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const rv_ds_job *jp = a.jobs + job;  // pred[] read through the pointer
  const rv_ds_job jb = *jp;
  const rv_plane &ref = a.ref[job / a.n_per_ref];
  const int ib = a.bd == 12 ? 2 : 4;
  const int maxv = (1 << a.bd) - 1;

  // ---- the source block, in registers ------------------------------------
  uint32_t org[DsFast<Px, W, H, SUB>::kOrgRegs];
  const int col = lane % W, grp = lane / W;  // sub-pel lane mapping
  const int frow = lane / F::K, fchunk = lane % F::K;  // full-pel
  if constexpr (SUB) {
    org[0] = 0;
    const Px *o = plane_ptr<Px>(a.org, jb.po_x, jb.po_y);
    for (int i = threadIdx.x; i < W * H; i += kDsThreads)
      org_lds[i] = o[(int64_t)(i / W) * a.org.stride + (i % W)];
    __syncthreads();
  } else {
    const uint8_t *o = (const uint8_t *)plane_ptr<Px>(a.org, jb.po_x, jb.po_y);
    const int64_t os = (int64_t)a.org.stride * B;
#pragma unroll
    for (int i = 0; i < F::I; i++) {
      const int r = i * F::R + frow;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (!F::kPartial || r < H) v = ld16(o + r * os + fchunk * 16);
      org[4 * i + 0] = v.x;
      org[4 * i + 1] = v.y;
      org[4 * i + 2] = v.z;
      org[4 * i + 3] = v.w;
    }
  }
  uint32_t evals = 0;
  unsigned long long ph_t1 = 0, ph_sub = 0, ph_ex = 0, ph_it = 0, ph_stage = 0;
  if (ph) ph_t1 = wall_clock64();

  // ---- full-pel: one candidate, evaluated by this wavefront -------------
  auto eval_full = [&](rv_mv mv) __attribute__((always_inline)) -> uint64_t {
    if (!ds_in_range(mv, jb)) return ~0ull;
    evals++;
    uint32_t acc = 0;
    // region at po + mv / 8 (Rust `/` truncates toward zero)
    const uint8_t *r =
        (const uint8_t *)plane_ptr<Px>(ref, jb.po_x + mv.col / 8, jb.po_y + mv.row / 8);
    const int64_t rs = (int64_t)ref.stride * B;
#pragma unroll
    for (int i = 0; i < F::I; i++) {
      const int rr = i * F::R + frow;
      if (!F::kPartial || rr < H) {
        const uint4 v = ld16(r + rr * rs + fchunk * 16);
        acc = sad16<Px>(make_uint4(org[4 * i], org[4 * i + 1], org[4 * i + 2], org[4 * i + 3]), v,
                        acc);
      }
    }
    return ds_cost(wave_sum(acc), mv, jb, a.hp);
  };

  // ---- sub-pel: a round of up to 4 candidates (one per wavefront) ------
  // predict_inter / get_params (src/predict.rs:267-283): integer source
  // origin (PlaneSlice::clamp of the -3 origin, src/frame/plane.rs:521-533)
  // and 1/16 fracs.  The candidates of a diamond step lie within 1 px of
  // each other, so the workgroup stages ONE window covering all of them
  // (cooperative, 256 threads) and every wavefront filters its candidate
  // out of it at its own offset.
  struct SubPos {
    int qx, qy, cf, rf, ok;
  };
  auto sub_pos = [&](rv_mv mv) __attribute__((always_inline)) -> SubPos {
    SubPos q;
    q.ok = ds_in_range(mv, jb);
    const int xs = 3 + ref.xdec, ys = 3 + ref.ydec;
    const int roff = (int)mv.row >> ys, coff = (int)mv.col >> xs;
    q.rf = ((int)mv.row - (roff << ys)) << (4 - ys);
    q.cf = ((int)mv.col - (coff << xs)) << (4 - xs);
    q.qx = clampi(jb.po_x + coff - 3, -ref.xorigin, ref.width);
    q.qy = clampi(jb.po_y + roff - 3, -ref.yorigin, ref.height);
    return q;
  };
  // stage the box at (bx, by) of rows x cols pixels into uwin (pitch UP bytes)
  auto load_box = [&](int bx, int by, int rows, int cols) __attribute__((always_inline)) {
    const uint8_t *sp = (const uint8_t *)plane_ptr<Px>(ref, bx, by);
    const int64_t rs = (int64_t)ref.stride * B;
    const int rdw = (cols * B + 3) >> 2, tot = rows * rdw;
    for (int i0 = threadIdx.x; i0 < tot; i0 += 4 * kDsThreads) {
      uint32_t v[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int i = i0 + u * kDsThreads;
        v[u] = 0;
        if (i < tot) {
          const int r = i / rdw, d = i - r * rdw;
          __builtin_memcpy(&v[u], sp + r * rs + 4 * d, 4);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int i = i0 + u * kDsThreads;
        if (i < tot) {
          const int r = i / rdw, d = i - r * rdw;
          // u8: stored as i8 = pixel - 128 (the horizontal v_dot4_i32_i8)
          win_all[r * (S::UP / 4) + d] = B == 1 ? v[u] ^ 0x80808080u : v[u];
        }
      }
    }
  };
  // SAD of this wavefront's candidate from the staged window, the window
  // pixel (dx, dy) being the candidate's (-3, -3) origin; the filter case
  // (horizontal / vertical / both / copy) is resolved once per candidate
  auto sub_sad = [&](int cf, int rf, int dx, int dy) __attribute__((always_inline)) -> uint32_t {
    const uint32_t *w0 = win_all + dy * (S::UP / 4);
    const Px *ocol = org_lds + grp * S::RG * W + col;
    const int8_t *xf = kReg[W <= 4][cf];
    const int8_t *yf = kReg[H <= 4][rf];
    uint32_t acc;
    if (cf && rf)
      acc = sub_sad_rows<Px, W, S::RG, S::UP, true, true>(w0, ocol, col + dx, grp, xf, yf, ib, maxv);
    else if (cf)
      acc = sub_sad_rows<Px, W, S::RG, S::UP, true, false>(w0, ocol, col + dx, grp, xf, yf, ib, maxv);
    else if (rf)
      acc = sub_sad_rows<Px, W, S::RG, S::UP, false, true>(w0, ocol, col + dx, grp, xf, yf, ib, maxv);
    else
      acc = sub_sad_rows<Px, W, S::RG, S::UP, false, false>(w0, ocol, col + dx, grp, xf, yf, ib, maxv);
    return wave_sum(acc);
  };
  // Called by every thread.  Wave w evaluates cands[w] (w < n, w != skip);
  // returns its cost (u64::MAX when out of range, skipped or w >= n).  No trailing barrier: the
  // caller's cost exchange barrier orders the next round's window writes.
  // The window currently staged in win_all: origin (wx, wy), D px of slack;
  // wvalid = false after a far-apart round overwrote it.
  int wx = 0, wy = 0;
  bool wvalid = false;
  auto sub_round = [&](const rv_mv *cands, int n, int skip) __attribute__((always_inline)) -> uint64_t {
    SubPos q[kDsWaves];
    int ux = 1 << 30, uy = 1 << 30, ux2 = -(1 << 30), uy2 = -(1 << 30), any = 0;
#pragma unroll
    for (int k = 0; k < kDsWaves; k++) {
      q[k] = sub_pos(cands[k]);  // (every slot is set; ok masks k >= n)
      q[k].ok = q[k].ok && k < n && k != skip;
      if (q[k].ok) {
        any = 1;
        ux = q[k].qx < ux ? q[k].qx : ux;
        uy = q[k].qy < uy ? q[k].qy : uy;
        ux2 = q[k].qx > ux2 ? q[k].qx : ux2;
        uy2 = q[k].qy > uy2 ? q[k].qy : uy2;
      }
    }
    uint64_t mine = ~0ull;
    if (!any) return mine;
    SubPos me = q[0];
    rv_mv me_mv = cands[0];
#pragma unroll
    for (int k = 1; k < kDsWaves; k++)
      if (wave == k) {
        me = q[k];
        me_mv = cands[k];
      }
    if (ux2 - ux <= S::D && uy2 - uy <= S::D) {
      // Re-stage only when a candidate leaves the staged window.  The last
      // round's cost-exchange barrier follows every read of the old window.
      // The new origin centres the slack on this round's candidates, kept
      // within the origins PlaneSlice::clamp can produce (so the reads stay
      // where a single candidate's window may read).
      if (!(wvalid && ux >= wx && ux2 <= wx + S::D && uy >= wy && uy2 <= wy + S::D)) {
        wx = clampi(ux - ((S::D - (ux2 - ux)) >> 1), max(ux2 - S::D, -ref.xorigin),
                    min(ux, ref.width - S::D));
        wy = clampi(uy - ((S::D - (uy2 - uy)) >> 1), max(uy2 - S::D, -ref.yorigin),
                    min(uy, ref.height - S::D));
        load_box(wx, wy, S::D + H + 7, S::D + W + 7);
        __syncthreads();
        wvalid = true;
        ph_stage++;
      }
      if (me.ok) {
        evals++;
        mine = ds_cost(sub_sad(me.cf, me.rf, me.qx - wx, me.qy - wy), me_mv, jb, a.hp);
      }
    } else {  // far-apart predictors: one window at a time
      wvalid = false;
#pragma unroll 1
      for (int k = 0; k < n; k++) {
        rv_mv ck = cands[0];  // static indices only (no scratch)
#pragma unroll
        for (int j = 1; j < kDsWaves; j++)
          if (k == j) ck = cands[j];
        SubPos qk = sub_pos(ck);
        qk.ok = qk.ok && k != skip;
        __syncthreads();  // previous window consumed
        if (qk.ok) load_box(qk.qx, qk.qy, H + 7, W + 7);
        __syncthreads();
        if (qk.ok && wave == k) {
          evals++;
          mine = ds_cost(sub_sad(qk.cf, qk.rf, 0, 0), ck, jb, a.hp);
        }
      }
    }
    return mine;
  };

  rv_mv center{0, 0};
  uint64_t center_cost = ~0ull;
  // ---- telescopic_subpel_search (src/me.rs:858-941) ---------------------
  // 3x3 grid around the running best at steps 8, 4, 2 (and 1 with hp); the
  // 8 grid points of a step are two rounds of 4; the reference's in-order
  // strict-< updates against a fixed grid centre equal the first minimum
  // of the step compared with the running cost.
  if (a.tele) {
    rv_mv best = a.start[job].best_mv;
    uint64_t lowest = a.start[job].cost;
    int round = 0;
    const int nsteps = a.hp ? 4 : 3;
    for (int st = 0; st < nsteps; st++) {
      const int16_t step = (int16_t)(8 >> st);
      const rv_mv ctr = best;
      uint64_t bc = ~0ull;
      rv_mv bm = ctr;
      for (int half = 0; half < 2; half++, round++) {
        rv_mv c4[kDsWaves];
#pragma unroll
        for (int k = 0; k < kDsWaves; k++) {
          const int gi = half * 4 + k < 4 ? half * 4 + k : half * 4 + k + 1;  // skip the centre
          c4[k] = rv_mv{(int16_t)(ctr.row + step * (gi / 3 - 1)),
                        (int16_t)(ctr.col + step * (gi % 3 - 1))};
        }
        uint64_t c;
        if constexpr (SUB) {
          c = sub_round(c4, kDsWaves, -1);
        } else {
          rv_mv mine = c4[0];
#pragma unroll
          for (int k = 1; k < kDsWaves; k++)
            if (wave == k) mine = c4[k];
          c = eval_full(mine);
        }
        if (lane == 0) scost[round & 1][wave] = c;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kDsWaves; k++) {
          const uint64_t v = scost[round & 1][k];
          if (v < bc) {
            bc = v;
            bm = c4[k];
          }
        }
      }
      if (bc < lowest) {
        lowest = bc;
        best = bm;
      }
    }
    center = best;
    center_cost = lowest;
  } else {
    // ---- get_best_predictor, then diamond steps: one round loop -----------
    // A round evaluates up to 4 candidates, one per wavefront: first the
    // predictors in groups of 4 (the sequential strict-< scan of
    // get_best_predictor, applied group by group in order, is the same
    // first minimum), then the 4 pattern points of each diamond step.  One
    // call site keeps a single inlined copy of the candidate code.
    const int np = jb.n_pred < RV_DS_MAX_PRED ? jb.n_pred : RV_DS_MAX_PRED;
    int16_t radius = a.subpel ? 4 : 16;
    const int16_t radius_end = a.subpel ? (a.hp ? 1 : 2) : 8;
    int p0 = 0;  // next predictor group; >= np once the diamond phase runs
    // After a move along pattern p the step at the same radius contains the
    // previous centre again (pattern (p + 2) & 3).  Its cost is the old
    // centre cost, which the move strictly undercut, so whatever the other
    // three give, it cannot move the centre: the step's outcome (move to the
    // first strict minimum, or halve the radius) is the same without it.
    // (The oracle, orc_diamond_search, evaluates it like the reference.)
    int back = -1;
    // Every diamond move strictly lowers center_cost, so the loop ends; the
    // bound only guarantees the grid drains whatever the inputs.
    for (int iter = 0; iter < 4096 + RV_DS_MAX_PRED; iter++) {
      const bool pred_phase = p0 < np;
      rv_mv c4[kDsWaves];
      int n;
      if (pred_phase) {
        n = np - p0 < kDsWaves ? np - p0 : kDsWaves;
  #pragma unroll
        for (int k = 0; k < kDsWaves; k++) {
          const int pi = p0 + (k < n ? k : 0);
          c4[k] = has_pred0 && pi == 0 ? pred0 : jp->pred[pi];
        }
      } else {
        n = kDsWaves;
        c4[0] = rv_mv{(int16_t)(center.row + radius), center.col};  // diamond_pattern
        c4[1] = rv_mv{center.row, (int16_t)(center.col + radius)};
        c4[2] = rv_mv{(int16_t)(center.row - radius), center.col};
        c4[3] = rv_mv{center.row, (int16_t)(center.col - radius)};
      }
      const int skip = pred_phase ? -1 : back;
      uint64_t c;
      if constexpr (SUB) {
        const unsigned long long ta = ph ? wall_clock64() : 0;
        c = sub_round(c4, n, skip);
        if (ph) {
          ph_sub += wall_clock64() - ta;
          ph_it++;
        }
      } else {
        rv_mv mine = c4[0];
  #pragma unroll
        for (int k = 1; k < kDsWaves; k++)
          if (wave == k) mine = c4[k];
        c = wave < n && wave != skip ? eval_full(mine) : ~0ull;
      }
      const unsigned long long tb = ph ? wall_clock64() : 0;
      if (lane == 0) scost[iter & 1][wave] = c;
      __syncthreads();
      if (ph) ph_ex += wall_clock64() - tb;
      uint64_t best = ~0ull;
      int bp = 0;
  #pragma unroll
      for (int k = 0; k < kDsWaves; k++) {
        const uint64_t v = scost[iter & 1][k];
        if (k < n && v < best) {
          best = v;
          bp = k;
        }
      }
      rv_mv bmv = c4[0];
  #pragma unroll
      for (int k = 1; k < kDsWaves; k++)
        if (bp == k) bmv = c4[k];
      if (pred_phase) {
        if (best < center_cost) {
          center = bmv;
          center_cost = best;
        }
        p0 += kDsWaves;
      } else if (center_cost <= best) {
        if (radius == radius_end) break;
        radius /= 2;
        back = -1;
      } else {
        // the old centre's cost is genuine unless it is the u64::MAX
        // placeholder of a search whose predictors were all out of range
        back = center_cost != ~0ull ? (bp + 2) & 3 : -1;
        center = bmv;
        center_cost = best;
      }
    }
  }
  if (a.evals || a.eval_acc) {
    if (lane == 0) wevals[wave] = evals;
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t ev = wevals[0] + wevals[1] + wevals[2] + wevals[3];
      if (a.evals) a.evals[job] = ev;
      if (a.eval_acc) {
        atomicAdd(a.eval_acc, ev);
        atomicAdd(a.eval_acc + 1, 1u);
      }
    }
  }
  if (threadIdx.x == 0) {
    ds_write(a, job, center, center_cost);
    chain_emit(a.next, job, a.n_per_ref, a.n / a.n_per_ref, center);
  }
  if (ph) {
    atomicAdd(&g_ds_ph[0], ph_t1 - ph_t0);
    atomicAdd(&g_ds_ph[1], ph_sub);
    atomicAdd(&g_ds_ph[2], ph_ex);
    atomicAdd(&g_ds_ph[3], wall_clock64() - ph_t0);
    atomicAdd(&g_ds_ph[4], ph_it);
    atomicAdd(&g_ds_ph[5], 1ull);
    atomicAdd(&g_ds_ph[6], ph_stage);
  }
  return center;
}

// The 4-wavefront search at 5 waves per SIMD (<= 96 VGPRs: the u8 sub-pel
// search fits without spilling), and at the compiler's choice
// (RAV1E_HIP_DS_OCC4=1, A/B).
// The workgroup's jobs: one (xcd_job) on a full grid, or, list-driven, the
// listed superblocks' jobs (every reference's) from blockIdx.x in steps of
// the grid.  Every bound is uniform over the workgroup.
template <typename Px, int W, int H, bool SUB>
__device__ __forceinline__ void ds_fast_jobs(const DsArgs &a) {
  if (!a.alist) {
    const int job = xcd_job(a.n);
    if (job >= a.n) return;                                // whole workgroup, uniformly
    if (a.active && !a.active[job % a.n_per_ref]) return;  // settled this round
    ds_fast_body<Px, W, H, SUB>(a, job);
    return;
  }
  const int total = ds_list_total(a);
  for (int i = blockIdx.x; i < total; i += gridDim.x) {
    const int job = __builtin_amdgcn_readfirstlane(ds_list_job(a, i));
    if (a.dirty && !a.dirty[job]) continue;  // uniform: its inputs are unchanged
    ds_fast_body<Px, W, H, SUB>(a, job);
    __syncthreads();  // the job's LDS reads end before the next job's writes
  }
}

template <typename Px, int W, int H, bool SUB>
__global__ __launch_bounds__(kDsThreads) __attribute__((amdgpu_waves_per_eu(5))) void
ds_fast_kernel(DsArgs a) {
  if (a.t0 && threadIdx.x == 0) atomicMin(a.t0, (unsigned long long)wall_clock64());
  const unsigned long long ph_k = SUB && a.ph && a.alist && threadIdx.x == 0 ? wall_clock64() : 0;
  ds_fast_jobs<Px, W, H, SUB>(a);
  if (ph_k) {
    atomicAdd(&g_ds_ph[7], wall_clock64() - ph_k);
    atomicAdd(&g_ds_ph[8], 1ull);
  }
  if (a.t1) {
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(a.t1, (unsigned long long)wall_clock64());
  }
}
template <typename Px, int W, int H, bool SUB>
__global__ __launch_bounds__(kDsThreads) void ds_fast_kernel_occ4(DsArgs a) {
  ds_fast_jobs<Px, W, H, SUB>(a);
}

// ============================ generic path =================================
template <int N>
__device__ __forceinline__ void ds_had(int32_t *v, int s) {
#pragma unroll
  for (int k = 0; k < N; k += 2) {
    int32_t x = v[k * s], y = v[(k + 1) * s];
    v[k * s] = x + y;
    v[(k + 1) * s] = x - y;
  }
#pragma unroll
  for (int g = 0; g < N; g += 4)
#pragma unroll
    for (int k = 0; k < 2; k++) {
      int32_t x = v[(g + k) * s], y = v[(g + k + 2) * s];
      v[(g + k) * s] = x + y;
      v[(g + k + 2) * s] = x - y;
    }
  if constexpr (N == 8) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      int32_t x = v[k * s], y = v[(k + 4) * s];
      v[k * s] = x + y;
      v[(k + 4) * s] = x - y;
    }
  }
}

__device__ __forceinline__ uint64_t wg_sum(uint64_t v, uint64_t *red) {
  v = group_sum<64>(v);
  __syncthreads();  // red[] may still be read by a previous reduction
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t t = 0;
#pragma unroll
  for (int i = 0; i < kDsWaves; i++) t += red[i];
  return t;
}

// Chunked Hadamard of one N x N difference block (get_satd_ref's butterfly
// order, src/dist.rs:208-272); diff(r, c) supplies org - pred.
template <int N, typename Diff>
__device__ __forceinline__ uint32_t had_abs_sum(Diff diff) {
  int32_t d[N * N];
#pragma unroll
  for (int r = 0; r < N; r++)
#pragma unroll
    for (int c = 0; c < N; c++) d[r * N + c] = diff(r, c);
#pragma unroll
  for (int c = 0; c < N; c++) ds_had<N>(d + c, N);
#pragma unroll
  for (int r = 0; r < N; r++) ds_had<N>(d + r * N, 1);
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < N * N; i++) acc += (uint32_t)(d[i] < 0 ? -d[i] : d[i]);
  return acc;
}

// SAD or SATD (get_sad / get_satd semantics) of org vs pred(r, c),
// evaluated by the whole workgroup; all threads get the result.
template <typename Px, typename Pred>
__device__ uint32_t wg_dist(const Px *o, int ostride, int w, int h, int satd, Pred pred,
                            uint64_t *red) {
  uint64_t acc = 0;
  if (!satd) {
    for (int i = threadIdx.x; i < w * h; i += kDsThreads) {
      const int r = i / w, c = i - r * w;
      const int d = (int)o[(int64_t)r * ostride + c] - pred(r, c);
      acc += (uint32_t)(d < 0 ? -d : d);
    }
    return (uint32_t)wg_sum(acc, red);
  }
  const int n8 = (w < h ? w : h) >= 8;
  const int N = n8 ? 8 : 4, cw = w / N, chunks = cw * (h / N);
  for (int ci = threadIdx.x; ci < chunks; ci += kDsThreads) {
    const int cy = (ci / cw) * N, cx = (ci % cw) * N;
    auto diff = [&](int r, int c) {
      return (int)o[(int64_t)(cy + r) * ostride + cx + c] - pred(cy + r, cx + c);
    };
    acc += n8 ? had_abs_sum<8>(diff) : had_abs_sum<4>(diff);
  }
  const uint64_t s = wg_sum(acc, red);
  const int ln = n8 ? 3 : 2;
  return (uint32_t)((s + ((1ull << ln) >> 1)) >> ln);
}

template <typename Px>
__global__ __launch_bounds__(kDsThreads) void diamond_kernel(DsArgs a) {
  extern __shared__ __align__(16) int16_t lds[];
  __shared__ uint64_t red[kDsWaves];
  const int job = blockIdx.x;
  if (job >= a.n) return;
  if (a.active && !a.active[job % a.n_per_ref]) return;
  const rv_ds_job jb = a.jobs[job];
  const rv_plane &ref = a.ref[job / a.n_per_ref];
  const int w = a.w, h = a.h;
  const Px *o = plane_ptr<Px>(a.org, jb.po_x, jb.po_y);
  const int ib = a.bd == 12 ? 2 : 4;
  const int maxv = (1 << a.bd) - 1;
  const int sw = w + 7, shh = h + 7;
  int16_t *win = lds;             // [h+7][w+7]
  int16_t *mid = lds + sw * shh;  // [h+7][w]
  int16_t *pred = mid + shh * w;  // [h][w]

  // get_mv_rd_cost: range check, prediction, distortion, rate
  uint32_t evals = 0;
  auto rd_cost = [&](rv_mv mv) -> uint64_t {
    if (!ds_in_range(mv, jb)) return ~0ull;
    evals++;
    uint32_t dist;
    if (!a.subpel) {
      const Px *r = plane_ptr<Px>(ref, jb.po_x + mv.col / 8, jb.po_y + mv.row / 8);
      const int rs = ref.stride;
      dist = wg_dist<Px>(o, a.org.stride, w, h, a.satd,
                         [&](int rr, int cc) { return (int)r[(int64_t)rr * rs + cc]; }, red);
    } else {
      const int xs = 3 + ref.xdec, ys = 3 + ref.ydec;
      const int roff = (int)mv.row >> ys, coff = (int)mv.col >> xs;
      const int rf = ((int)mv.row - (roff << ys)) << (4 - ys);
      const int cf = ((int)mv.col - (coff << xs)) << (4 - xs);
      const int qx = clampi(jb.po_x + coff - 3, -ref.xorigin, ref.width);
      const int qy = clampi(jb.po_y + roff - 3, -ref.yorigin, ref.height);
      const Px *sp = plane_ptr<Px>(ref, qx, qy);  // window origin (-3, -3)
      __syncthreads();  // previous candidate done with LDS
      for (int i = threadIdx.x; i < sw * shh; i += kDsThreads) {
        const int r = i / sw, c = i - r * sw;
        win[i] = (int16_t)sp[(int64_t)r * ref.stride + c];
      }
      __syncthreads();
      const int8_t *xf = kReg[w <= 4][cf];
      const int8_t *yf = kReg[h <= 4][rf];
      if (cf) {
        for (int i = threadIdx.x; i < shh * w; i += kDsThreads) {
          const int r = i / w, c = i - r * w;
          const int16_t *p = win + r * sw + c;
          int32_t s = 0;
#pragma unroll
          for (int k = 0; k < 8; k++) s += (int32_t)xf[k] * p[k];
          mid[i] = (int16_t)round_shift(s, 7 - ib);
        }
        __syncthreads();
      }
      for (int i = threadIdx.x; i < w * h; i += kDsThreads) {
        const int r = i / w, c = i - r * w;
        int32_t v;
        if (!cf && !rf) {
          v = win[(r + 3) * sw + c + 3];
        } else if (!cf) {
          const int16_t *p = win + r * sw + c + 3;
          int32_t s = 0;
#pragma unroll
          for (int k = 0; k < 8; k++) s += (int32_t)yf[k] * p[k * sw];
          v = round_shift(s, 7);
        } else if (!rf) {
          v = round_shift((int32_t)mid[(r + 3) * w + c], ib);
        } else {
          const int16_t *p = mid + r * w + c;
          int32_t s = 0;
#pragma unroll
          for (int k = 0; k < 8; k++) s += (int32_t)yf[k] * p[k * w];
          v = round_shift(s, 7 + ib);
        }
        pred[i] = (int16_t)clampi(v, 0, maxv);
      }
      __syncthreads();
      dist = wg_dist<Px>(o, a.org.stride, w, h, a.satd,
                         [&](int rr, int cc) { return (int)pred[rr * w + cc]; }, red);
    }
    return ds_cost(dist, mv, jb, a.hp);
  };

  rv_mv center{0, 0};
  uint64_t center_cost = ~0ull;
  if (a.tele) {  // telescopic_subpel_search (src/me.rs:858-941)
    center = a.start[job].best_mv;
    center_cost = a.start[job].cost;
    const int nsteps = a.hp ? 4 : 3;
    for (int st = 0; st < nsteps; st++) {
      const int16_t step = (int16_t)(8 >> st);
      const rv_mv ctr = center;
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
          if (i == 1 && j == 1) continue;
          const rv_mv cand{(int16_t)(ctr.row + step * (i - 1)), (int16_t)(ctr.col + step * (j - 1))};
          const uint64_t c = rd_cost(cand);
          if (c < center_cost) {
            center_cost = c;
            center = cand;
          }
        }
    }
  } else {
    // get_best_predictor (the predictors read through the job's pointer: a
    // runtime index into the local copy kept it in scratch memory)
    const rv_ds_job *jp = a.jobs + job;
    const int np = jb.n_pred < RV_DS_MAX_PRED ? jb.n_pred : RV_DS_MAX_PRED;
    for (int p = 0; p < np; p++) {
      const rv_mv pm = jp->pred[p];
      const uint64_t c = rd_cost(pm);
      if (c < center_cost) {
        center = pm;
        center_cost = c;
      }
    }
    int16_t radius = a.subpel ? 4 : 16;
    const int16_t radius_end = a.subpel ? (a.hp ? 1 : 2) : 8;
    for (int iter = 0; iter < 4096; iter++) {
      uint64_t best = ~0ull;
      rv_mv best_mv{0, 0};
      for (int p = 0; p < 4; p++) {
        // diamond_pattern {(1, 0), (0, 1), (-1, 0), (0, -1)} without a table
        const int dr = (p == 0) - (p == 2), dc = (p == 1) - (p == 3);
        const rv_mv cand{(int16_t)(center.row + radius * dr), (int16_t)(center.col + radius * dc)};
        const uint64_t c = rd_cost(cand);
        if (c < best) {
          best = c;
          best_mv = cand;
        }
      }
      if (center_cost <= best) {
        if (radius == radius_end) break;
        radius /= 2;
      } else {
        center = best_mv;
        center_cost = best;
      }
    }
  }
  if (threadIdx.x == 0) {
    if (a.evals) a.evals[job] = evals;
    ds_write(a, job, center, center_cost);
    chain_emit(a.next, job, a.n_per_ref, a.n / a.n_per_ref, center);
  }
}

// Full-pel diamond, one wavefront per job.  A round's (up to) 4
// candidates are evaluated together by the one wavefront -- all their row
// loads in flight at once, then four wave reductions -- so the round's
// decision needs no LDS exchange or barrier, and a 64x64 job occupies one
// wave instead of four (the search is a chain of dependent rounds, bound by
// load latency: more jobs in flight per CU is what shortens it).
template <typename Px, int W, int H>
__global__ __launch_bounds__(64) void ds_wave_kernel(DsArgs a) {
  using F = FullGeo<Px, W, H>;
  constexpr int B = (int)sizeof(Px);
  const int job = xcd_job(a.n);
  if (job >= a.n) return;
  if (a.active && !a.active[job % a.n_per_ref]) return;
  const int lane = threadIdx.x;
  const rv_ds_job *jp = a.jobs + job;
  const rv_ds_job jb = *jp;
  const rv_plane &ref = a.ref[job / a.n_per_ref];
  const int frow = lane / F::K, fchunk = lane % F::K;
  uint32_t org[4 * F::I];
  {
    const uint8_t *o = (const uint8_t *)plane_ptr<Px>(a.org, jb.po_x, jb.po_y);
    const int64_t os = (int64_t)a.org.stride * B;
#pragma unroll
    for (int i = 0; i < F::I; i++) {
      const int r = i * F::R + frow;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (!F::kPartial || r < H) v = ld16(o + r * os + fchunk * 16);
      org[4 * i + 0] = v.x;
      org[4 * i + 1] = v.y;
      org[4 * i + 2] = v.z;
      org[4 * i + 3] = v.w;
    }
  }
  const int64_t rs = (int64_t)ref.stride * B;
  uint32_t evals = 0;
  // costs of cands[k], k < n, k != skip (u64::MAX when out of range,
  // skipped or k >= n); wave-uniform
  auto round4 = [&](const rv_mv *cands, int n, int skip, uint64_t *cost)
      __attribute__((always_inline)) {
    bool ok[kDsWaves];
    const uint8_t *rp[kDsWaves];
#pragma unroll
    for (int k = 0; k < kDsWaves; k++) {
      ok[k] = k < n && k != skip && ds_in_range(cands[k], jb);
      // region at po + mv / 8 (Rust `/` truncates toward zero)
      rp[k] = (const uint8_t *)plane_ptr<Px>(ref, jb.po_x + (ok[k] ? cands[k].col / 8 : 0),
                                             jb.po_y + (ok[k] ? cands[k].row / 8 : 0));
      evals += ok[k];
    }
    uint32_t acc[kDsWaves] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < F::I; i++) {
      const int rr = i * F::R + frow;
      if (!F::kPartial || rr < H) {
        uint4 v[kDsWaves];
#pragma unroll
        for (int k = 0; k < kDsWaves; k++)
          v[k] = ok[k] ? ld16(rp[k] + rr * rs + fchunk * 16) : make_uint4(0, 0, 0, 0);
        const uint4 o = make_uint4(org[4 * i], org[4 * i + 1], org[4 * i + 2], org[4 * i + 3]);
#pragma unroll
        for (int k = 0; k < kDsWaves; k++) acc[k] = sad16<Px>(o, v[k], acc[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < kDsWaves; k++)
      cost[k] = ok[k] ? ds_cost(wave_sum(acc[k]), cands[k], jb, a.hp) : ~0ull;
  };

  // get_best_predictor, then the diamond steps: the round loop of
  // ds_fast_kernel (its comments give the exactness arguments), decided in
  // registers.
  rv_mv center{0, 0};
  uint64_t center_cost = ~0ull;
  const int np = jb.n_pred < RV_DS_MAX_PRED ? jb.n_pred : RV_DS_MAX_PRED;
  int16_t radius = 16;
  const int16_t radius_end = 8;
  int p0 = 0;
  int back = -1;
  for (int iter = 0; iter < 4096 + RV_DS_MAX_PRED; iter++) {
    const bool pred_phase = p0 < np;
    rv_mv c4[kDsWaves];
    int n;
    if (pred_phase) {
      n = np - p0 < kDsWaves ? np - p0 : kDsWaves;
#pragma unroll
      for (int k = 0; k < kDsWaves; k++) c4[k] = jp->pred[p0 + (k < n ? k : 0)];
    } else {
      n = kDsWaves;
      c4[0] = rv_mv{(int16_t)(center.row + radius), center.col};  // diamond_pattern
      c4[1] = rv_mv{center.row, (int16_t)(center.col + radius)};
      c4[2] = rv_mv{(int16_t)(center.row - radius), center.col};
      c4[3] = rv_mv{center.row, (int16_t)(center.col - radius)};
    }
    uint64_t c[kDsWaves];
    round4(c4, n, pred_phase ? -1 : back, c);
    uint64_t best = ~0ull;
    int bp = 0;
#pragma unroll
    for (int k = 0; k < kDsWaves; k++)
      if (k < n && c[k] < best) {
        best = c[k];
        bp = k;
      }
    rv_mv bmv = c4[0];
#pragma unroll
    for (int k = 1; k < kDsWaves; k++)
      if (bp == k) bmv = c4[k];
    if (pred_phase) {
      if (best < center_cost) {
        center = bmv;
        center_cost = best;
      }
      p0 += kDsWaves;
    } else if (center_cost <= best) {
      if (radius == radius_end) break;
      radius /= 2;
      back = -1;
    } else {
      back = center_cost != ~0ull ? (bp + 2) & 3 : -1;
      center = bmv;
      center_cost = best;
    }
  }
  if (lane == 0) {
    if (a.evals) a.evals[job] = evals;
    ds_write(a, job, center, center_cost);
    chain_emit(a.next, job, a.n_per_ref, a.n / a.n_per_ref, center);
  }
}

// Square blocks with SATD (use_satd_subpel, src/me.rs:232-253) and the
// small full-pel searches of the speed-6 partition levels: one group of
// L = 4 C lanes per job, 64 / L jobs per wavefront, every round's (up to) 4
// candidates evaluated at once by the group's four C-lane subgroups.  A
// lane owns RPL rows x 8 columns of one 8x8 chunk of its candidate (CPL
// chunks in turn): it forms org - prediction for them (sub-pel: put_8tap
// of its rows, the horizontal pass streamed row by row into per-row
// vertical accumulators), then for SATD the 8-point row Hadamards in-lane
// and the column butterflies in-lane over its rows and across the LPC lanes
// of the chunk by shuffles (get_satd's 8x8 Hadamard, src/dist.rs:208-272:
// the sum of |coefficients| does not depend on the butterfly order).  The
// subgroup's sums meet by shuffles, the four costs by shuffles across the
// group, so a job's rounds need no LDS and no barrier; groups of one
// wavefront diverge freely (a shuffle only reads its own group's lanes).
// SAD-only full-pel searches (SADONLY) give each lane a whole 8x8 chunk: a
// 16x16 job then takes 16 lanes and a wavefront carries 4 jobs, which hides
// the rounds' load latency better than one job per wavefront (FL, F2:
// 0.24 -> 0.13 ms at 2160p).  (Sub-pel tried the same, and a window staged
// in LDS per round: both slower, the sub-pel search is VALU-bound.)
typedef short rv_s16x2 __attribute__((ext_vector_type(2)));
// a.lo * b.lo + a.hi * b.hi + c over packed i16 halves (v_dot2_i32_i16)
__device__ __forceinline__ int32_t sdot2(uint32_t a, uint32_t b, int32_t c) {
  return __builtin_amdgcn_sdot2(__builtin_bit_cast(rv_s16x2, a), __builtin_bit_cast(rv_s16x2, b),
                                c, false);
}
__device__ __forceinline__ uint32_t pk16(int lo, int hi) {
  return (uint32_t)(uint16_t)lo | ((uint32_t)(uint16_t)hi << 16);
}

template <int N, bool SADONLY>
struct GrpGeo {
  static constexpr int C = N == 8 || (SADONLY && N == 16) ? 4 : 16;  // lanes per candidate
  static constexpr int L = 4 * C;                      // lanes per job
  static constexpr int RPL = N == 8 ? 2 : (N == 16 && C == 16) ? 2 : 8;  // chunk rows per lane
  static constexpr int LPC = 8 / RPL;                  // lanes per chunk
  static constexpr int NC = N / 8;                     // chunks per row
  static constexpr int CPL = NC * NC * LPC / C;        // chunks per lane
};

// ord: this lane group's ordinal among nord jobs (the wavefront's first
// ordinal is < nord); the job is ord itself or, list-driven, its list entry
template <typename Px, int N, bool SUB, bool SATD>
__device__ __forceinline__ void ds_grp_body(const DsArgs &a, const int ord, const int nord) {
  using G = GrpGeo<N, !SUB && !SATD>;
  static_assert(G::CPL >= 1 && G::C % G::LPC == 0, "lane layout");
  const int lane = threadIdx.x & 63;
  const int gl = lane % G::L, k = gl / G::C, c = gl % G::C;
  const int gbase = lane - gl;  // the group's first lane
  const int oid = ord < nord ? ord : nord - 1;
  const int job = a.alist ? ds_list_job(a, oid) : oid;
  // a listed job whose inputs did not change keeps its result; a wavefront
  // whose jobs all do leaves (no workgroup barrier below)
  const bool live = ord < nord && !(a.dirty && !a.dirty[job]);
  if (__ballot(live) == 0) return;
  const int jid = job;
  const rv_ds_job *jp = a.jobs + jid;
  const rv_ds_job jb = *jp;
  const rv_plane &ref = a.ref[jid / a.n_per_ref];
  const int ib = a.bd == 12 ? 2 : 4, maxv = (1 << a.bd) - 1;
  const int lic = c % G::LPC;  // lane in chunk

  // distortion of candidate mv for this subgroup (all lanes of the
  // subgroup return it); ok = false: the value is unused (zero work except in the branch-free sub-pel path)
  auto dist = [&](rv_mv mv, bool ok) -> uint32_t {
    int cf = 0, rf = 0, sx = 0, sy = 0;
    if (SUB) {
      const int xs = 3 + ref.xdec, ys = 3 + ref.ydec;
      const int roff = (int)mv.row >> ys, coff = (int)mv.col >> xs;
      rf = ((int)mv.row - (roff << ys)) << (4 - ys);
      cf = ((int)mv.col - (coff << xs)) << (4 - xs);
      sx = clampi(jb.po_x + coff - 3, -ref.xorigin, ref.width);  // window origin (-3, -3)
      sy = clampi(jb.po_y + roff - 3, -ref.yorigin, ref.height);
    } else {
      sx = jb.po_x + (ok ? mv.col / 8 : 0);
      sy = jb.po_y + (ok ? mv.row / 8 : 0);
    }
    // sub-pel: the candidates of one wavefront differ in fraction, so the
    // filter runs branch-free for all of them: a zero fraction takes the
    // identity taps (128 at tap 3), whose 7-bit round trips are exact, so
    // copy / horizontal-only / vertical-only / both equal put_8tap's four
    // cases bit for bit (src/mc.rs:213-274).  Horizontal taps as i16 pairs
    // for v_dot2: odd outputs (1,2) (3,4) (5,6), even outputs (0,1) (2,3)
    // (4,5) (6,7); REGULAR taps 0 and 7 are zero for every fraction
    // (src/mc.rs:71-88), so odd outputs need only 3 pairs.
    uint32_t xp[7];
    int32_t fy[8];
    if (SUB) {
      int32_t fx[8];
      const int8_t *xf = kReg[0][cf];
      const int8_t *yf = kReg[0][rf];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        fx[u] = cf ? (int32_t)xf[u] : (u == 3 ? 128 : 0);
        fy[u] = rf ? (int32_t)yf[u] : (u == 3 ? 128 : 0);
      }
      xp[0] = pk16(fx[1], fx[2]);
      xp[1] = pk16(fx[3], fx[4]);
      xp[2] = pk16(fx[5], fx[6]);
      xp[3] = pk16(fx[0], fx[1]);
      xp[4] = pk16(fx[2], fx[3]);
      xp[5] = pk16(fx[4], fx[5]);
      xp[6] = pk16(fx[6], fx[7]);
    }
    const int32_t hround = (1 << (7 - ib)) >> 1, vround = (1 << (7 + ib)) >> 1;
    uint32_t acc = 0;
#pragma unroll 1
    for (int j = 0; j < G::CPL; j++) {
      const int q = c / G::LPC + j * (G::C / G::LPC);
      const int x0 = (q % G::NC) * 8, y0 = (q / G::NC) * 8 + lic * G::RPL;
      int32_t d[G::RPL][8];
      if (SUB) {
        // output rows y0 .. y0 + RPL - 1 take window rows y0 + 1 .. y0 + RPL + 5
        // (taps 1..6); the window reads stay inside the clamped origin's
        // reach whether or not the candidate is valid (ok only gates use)
        int32_t v[G::RPL][8];
#pragma unroll
        for (int i = 0; i < G::RPL; i++)
#pragma unroll
          for (int t = 0; t < 8; t++) v[i][t] = vround;
#pragma unroll
        for (int m = 1; m < G::RPL + 6; m++) {
          const Px *w = plane_ptr<Px>(ref, sx + x0, sy + y0 + m);
          // pixel pairs (2j, 2j + 1) as packed i16, j < 7 (pixels 0..13)
          uint32_t pp[7];
          if constexpr (sizeof(Px) == 1) {  // 16 bytes, one unaligned load
            const uint4 lv = ld16(w);
            const uint32_t wd[4] = {lv.x, lv.y, lv.z, lv.w};
#pragma unroll
            for (int jj = 0; jj < 7; jj++)
              pp[jj] = __builtin_amdgcn_perm(0u, wd[jj >> 1], jj & 1 ? 0x0c030c02u : 0x0c010c00u);
          } else {  // 32 bytes, two: the dwords already are the pairs
            const uint4 v0 = ld16(w), v1 = ld16(w + 8);
            const uint32_t wd[7] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z};
#pragma unroll
            for (int jj = 0; jj < 7; jj++) pp[jj] = wd[jj];
          }
          int32_t mid[8];
#pragma unroll
          for (int t = 0; t < 8; t++) {
            int32_t hs = hround;
            if (t & 1) {
#pragma unroll
              for (int u = 0; u < 3; u++) hs = sdot2(pp[(t + 1) / 2 + u], xp[u], hs);
            } else {
#pragma unroll
              for (int u = 0; u < 4; u++) hs = sdot2(pp[t / 2 + u], xp[3 + u], hs);
            }
            mid[t] = hs >> (7 - ib);
          }
#pragma unroll
          for (int i = 0; i < G::RPL; i++) {
            const int kk = m - i;
            if (kk >= 1 && kk < 7) {  // taps 1..6
#pragma unroll
              for (int t = 0; t < 8; t++) v[i][t] += __mul24(fy[kk], mid[t]);
            }
          }
        }
#pragma unroll
        for (int i = 0; i < G::RPL; i++) {
          const Px *o = plane_ptr<Px>(a.org, jb.po_x + x0, jb.po_y + y0 + i);
#pragma unroll
          for (int t = 0; t < 8; t++)
            d[i][t] = (int32_t)o[t] - clampi(v[i][t] >> (7 + ib), 0, maxv);
        }
      } else if (ok) {
        if (!SATD) {  // 8-pixel row chunks: unaligned vector loads + v_sad
#pragma unroll
          for (int i = 0; i < G::RPL; i++) {
            const Px *o = plane_ptr<Px>(a.org, jb.po_x + x0, jb.po_y + y0 + i);
            const Px *r = plane_ptr<Px>(ref, sx + x0, sy + y0 + i);
            if constexpr (sizeof(Px) == 1) {
              uint2 ov, rv;
              __builtin_memcpy(&ov, o, 8);
              __builtin_memcpy(&rv, r, 8);
              acc = __builtin_amdgcn_sad_u8(ov.x, rv.x, acc);
              acc = __builtin_amdgcn_sad_u8(ov.y, rv.y, acc);
            } else {
              acc = sad16<Px>(ld16(o), ld16(r), acc);
            }
#pragma unroll
            for (int t = 0; t < 8; t++) d[i][t] = 0;
          }
        } else {
#pragma unroll
          for (int i = 0; i < G::RPL; i++) {
            const Px *o = plane_ptr<Px>(a.org, jb.po_x + x0, jb.po_y + y0 + i);
            const Px *r = plane_ptr<Px>(ref, sx + x0, sy + y0 + i);
#pragma unroll
            for (int t = 0; t < 8; t++) d[i][t] = (int32_t)o[t] - (int32_t)r[t];
          }
        }
      } else {
#pragma unroll
        for (int i = 0; i < G::RPL; i++)
#pragma unroll
          for (int t = 0; t < 8; t++) d[i][t] = 0;
      }
      if (SATD) {
#pragma unroll
        for (int i = 0; i < G::RPL; i++) ds_had<8>(&d[i][0], 1);  // rows
        // columns: row bits inside the lane ...
#pragma unroll
        for (int b = 1; b < G::RPL; b <<= 1)
#pragma unroll
          for (int i = 0; i < G::RPL; i++)
            if (!(i & b))
#pragma unroll
              for (int t = 0; t < 8; t++) {
                const int32_t x = d[i][t], y = d[i + b][t];
                d[i][t] = x + y;
                d[i + b][t] = x - y;
              }
        // ... and across the chunk's lanes
#pragma unroll
        for (int b = 1; b < G::LPC; b <<= 1) {
          const bool up = (lic & b) != 0;
#pragma unroll
          for (int i = 0; i < G::RPL; i++)
#pragma unroll
            for (int t = 0; t < 8; t++) {
              const int32_t p = __shfl_xor(d[i][t], b, 64);
              d[i][t] = up ? p - d[i][t] : d[i][t] + p;
            }
        }
      }
#pragma unroll
      for (int i = 0; i < G::RPL; i++)
#pragma unroll
        for (int t = 0; t < 8; t++) acc += (uint32_t)(d[i][t] < 0 ? -d[i][t] : d[i][t]);
    }
#pragma unroll
    for (int m = G::C / 2; m; m >>= 1) acc += __shfl_xor(acc, m, 64);
    return SATD ? (acc + 4) >> 3 : acc;  // get_satd: (sum + (1 << ln >> 1)) >> ln, ln = 3
  };

  uint32_t evals = 0;
  // costs of cands[0..3] (u64::MAX when out of range, skipped or >= n),
  // uniform over the group
  auto round4 = [&](const rv_mv *cands, int n, int skip, uint64_t *cost)
      __attribute__((always_inline)) {
    bool ok[4];
#pragma unroll
    for (int kk = 0; kk < 4; kk++) {
      ok[kk] = kk < n && kk != skip && ds_in_range(cands[kk], jb);
      evals += ok[kk];
    }
    rv_mv mine = cands[0];
    bool okm = ok[0];
#pragma unroll
    for (int kk = 1; kk < 4; kk++)
      if (k == kk) {
        mine = cands[kk];
        okm = ok[kk];
      }
    const uint32_t dv = dist(mine, okm);
    const uint64_t cm = okm ? ds_cost(dv, mine, jb, a.hp) : ~0ull;
    const uint32_t lo = (uint32_t)cm, hi = (uint32_t)(cm >> 32);
#pragma unroll
    for (int kk = 0; kk < 4; kk++) {
      const uint32_t l = __shfl(lo, gbase + kk * G::C, 64), h = __shfl(hi, gbase + kk * G::C, 64);
      cost[kk] = ((uint64_t)h << 32) | l;
    }
  };

  rv_mv center{0, 0};
  uint64_t center_cost = ~0ull;
  const int np = jb.n_pred < RV_DS_MAX_PRED ? jb.n_pred : RV_DS_MAX_PRED;
  int16_t radius = SUB ? 4 : 16;
  const int16_t radius_end = SUB ? (a.hp ? 1 : 2) : 8;
  int p0 = 0, back = -1;
  for (int iter = 0; iter < 4096 + RV_DS_MAX_PRED; iter++) {
    const bool pred_phase = p0 < np;
    rv_mv c4[4];
    int n;
    if (pred_phase) {
      n = np - p0 < 4 ? np - p0 : 4;
#pragma unroll
      for (int kk = 0; kk < 4; kk++) c4[kk] = jp->pred[p0 + (kk < n ? kk : 0)];
    } else {
      n = 4;
      c4[0] = rv_mv{(int16_t)(center.row + radius), center.col};  // diamond_pattern
      c4[1] = rv_mv{center.row, (int16_t)(center.col + radius)};
      c4[2] = rv_mv{(int16_t)(center.row - radius), center.col};
      c4[3] = rv_mv{center.row, (int16_t)(center.col - radius)};
    }
    uint64_t cst[4];
    round4(c4, n, pred_phase ? -1 : back, cst);
    uint64_t best = ~0ull;
    int bp = 0;
#pragma unroll
    for (int kk = 0; kk < 4; kk++)
      if (kk < n && cst[kk] < best) {
        best = cst[kk];
        bp = kk;
      }
    rv_mv bmv = c4[0];
#pragma unroll
    for (int kk = 1; kk < 4; kk++)
      if (bp == kk) bmv = c4[kk];
    if (pred_phase) {
      if (best < center_cost) {
        center = bmv;
        center_cost = best;
      }
      p0 += 4;
    } else if (center_cost <= best) {
      if (radius == radius_end) break;
      radius /= 2;
      back = -1;
    } else {
      back = center_cost != ~0ull ? (bp + 2) & 3 : -1;
      center = bmv;
      center_cost = best;
    }
  }
  if (gl == 0 && live) {
    if (a.evals) a.evals[job] = evals;
    ds_write(a, job, center, center_cost);
    chain_emit(a.next, job, a.n_per_ref, a.n / a.n_per_ref, center);
  }
}

template <typename Px, int N, bool SUB, bool SATD>
__global__ __launch_bounds__(256) void ds_grp_kernel(DsArgs a) {
  using G = GrpGeo<N, !SUB && !SATD>;
  constexpr int JPW = 64 / G::L;  // jobs per wavefront
  const int lane = threadIdx.x & 63;
  const int w0 = ((int)blockIdx.x * 4 + (int)(threadIdx.x >> 6)) * JPW;  // the wavefront's first
  const int nord = a.alist ? ds_list_total(a) : a.n;
  const int step = (int)gridDim.x * 4 * JPW;  // list-driven: a fixed pool loops
  for (int o = w0; o < nord; o += step) {
    ds_grp_body<Px, N, SUB, SATD>(a, o + lane / G::L, nord);
    if (!a.alist) break;
  }
}
// A round's F2 (16x16 full-pel quadrants at half resolution, ds_grp) and
// F3 full-pel (64x64, ds_fast) in one launch: they are independent, so the
// round pays one search latency for both.  Workgroups below g2 run the F2
// pool, the rest the F3 pool (both list-driven).  The arguments come by
// value (bound by reference to kernel arguments they can land in scratch).
template <typename Px>
__device__ __forceinline__ void ds_grp16_pool(DsArgs a, int b, int gsz) {
  using G = GrpGeo<16, true>;
  constexpr int JPW = 64 / G::L;
  const int lane = threadIdx.x & 63;
  const int nord = ds_list_total(a);
  for (int o = (b * 4 + (int)(threadIdx.x >> 6)) * JPW; o < nord; o += gsz * 4 * JPW)
    ds_grp_body<Px, 16, false, false>(a, o + lane / G::L, nord);
}
// fuse: each F3 job's sub-pel search (f3s, the same job index and dirty
// flag) right after its full-pel search in the same workgroup, from the
// full-pel winner -- the round's separate sub-pel launch and its dependent
// dispatch go away.
template <typename Px>
__device__ __forceinline__ void ds_fast64_pool(DsArgs a, DsArgs sa, bool fuse, int b, int gsz) {
  const int total = ds_list_total(a);
  for (int i = b; i < total; i += gsz) {
    const int job = __builtin_amdgcn_readfirstlane(ds_list_job(a, i));
    if (a.dirty && !a.dirty[job]) continue;
    const rv_mv best = ds_fast_body<Px, 64, 64, false>(a, job);
    __syncthreads();
    if (fuse) {
      ds_fast_body<Px, 64, 64, true>(sa, job, true, best);
      __syncthreads();
    }
  }
}
template <typename Px>
__global__ __launch_bounds__(256) void ds_f2_f3_kernel(
    DsArgs f2, DsArgs f3, DsArgs f3s, int g2, int fuse, unsigned long long *t01) {
  // the kernel probe (fused launches, t01 non-null): the launch's
  // device-clock span; the sub-pel bodies count their candidates into
  // f3s.eval_acc.  (t01 is a parameter of its own: reading it out of an
  // argument struct made the compiler copy the struct to scratch, 704 B.)
  if (t01 && threadIdx.x == 0) atomicMin(t01, (unsigned long long)wall_clock64());
  if ((int)blockIdx.x < g2)
    ds_grp16_pool<Px>(f2, blockIdx.x, g2);
  else
    ds_fast64_pool<Px>(f3, f3s, fuse != 0, (int)blockIdx.x - g2, (int)gridDim.x - g2);
  if (t01) {
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(t01 + 1, (unsigned long long)wall_clock64());
  }
}

template <typename Px>
bool try_grp(const DsArgs &a, hipStream_t s) {
  if (a.tele || a.w != a.h || a.active) return false;
  const int n = a.w;
  const bool small = n == 8 || n == 16;
  if (!(small || (a.satd && (n == 32 || n == 64)))) return false;
  const int jpw = 64 / (n == 8 || (n == 16 && !a.subpel && !a.satd) ? 16 : 64);
  unsigned grid = (unsigned)((a.n + 4 * jpw - 1) / (4 * jpw));
  if (a.alist && grid > (unsigned)(a.list_grid ? a.list_grid : ds_list_grid()))
    grid = (unsigned)(a.list_grid ? a.list_grid : ds_list_grid());
#define RV_GRP(N)                                                                     \
  if (n == N) {                                                                       \
    if (a.subpel) {                                                                   \
      if (a.satd) ds_grp_kernel<Px, N, true, true><<<grid, 256, 0, s>>>(a);           \
      else ds_grp_kernel<Px, N, true, false><<<grid, 256, 0, s>>>(a);                 \
    } else {                                                                          \
      if (a.satd) ds_grp_kernel<Px, N, false, true><<<grid, 256, 0, s>>>(a);          \
      else ds_grp_kernel<Px, N, false, false><<<grid, 256, 0, s>>>(a);                \
    }                                                                                 \
    return true;                                                                      \
  }
  RV_GRP(8)
  RV_GRP(16)
  RV_GRP(32)
  RV_GRP(64)
#undef RV_GRP
  return false;
}

// Blocks up to 32x32 take ds_wave_kernel (2160p F2, 32x32 at half
// resolution: 0.031 -> 0.023 ms); 64x64 stays on the 4-wavefront kernel
// (0.035 vs 0.037 ms: 16 row loads per round from one wavefront issue
// slower than 4 from each of four).  RAV1E_HIP_DS_WG=1: always the
// 4-wavefront kernel (A/B).
static bool ds_full_wave() {
  static const bool on = [] {
    const char *e = getenv("RAV1E_HIP_DS_WG");
    return !(e && e[0] == '1');
  }();
  return on;
}

template <typename Px, int W, int H, bool SUB>
void launch_fast(DsArgs a, hipStream_t s) {
  static const bool phases = getenv("RAV1E_HIP_DS_PHASES") && getenv("RAV1E_HIP_DS_PHASES")[0] == '1';
  a.ph = phases && SUB && a.alist ? 1 : 0;
  const unsigned grid = a.alist ? (unsigned)std::min(a.n, a.list_grid ? a.list_grid : ds_list_grid())
                                 : (unsigned)((a.n + 7) / 8 * 8);
  static const bool occ4 = [] {
    const char *e = getenv("RAV1E_HIP_DS_OCC4");
    return e && e[0] == '1';
  }();
  if (!SUB && !a.tele && W * H <= 32 * 32 && ds_full_wave() && !a.alist)
    ds_wave_kernel<Px, W, H><<<grid, 64, 0, s>>>(a);
  else if (occ4)
    ds_fast_kernel_occ4<Px, W, H, SUB><<<grid, kDsThreads, 0, s>>>(a);
  else
    ds_fast_kernel<Px, W, H, SUB><<<grid, kDsThreads, 0, s>>>(a);
}

template <typename Px>
bool try_fast(const DsArgs &a, hipStream_t s) {
  if (a.satd) return false;
#define RV_DS_CASE(W, H)                                        \
  if (a.w == W && a.h == H) {                                   \
    if (a.subpel)                                               \
      launch_fast<Px, W, H, true>(a, s);                        \
    else                                                        \
      launch_fast<Px, W, H, false>(a, s);                       \
    return true;                                                \
  }
  RV_DS_CASE(64, 64)
  RV_DS_CASE(32, 32)
  RV_DS_CASE(64, 32)
  RV_DS_CASE(32, 64)
  RV_DS_CASE(16, 32)
  RV_DS_CASE(16, 64)
#undef RV_DS_CASE
  return false;
}

}  // namespace rv

using namespace rv;

// RAV1E_HIP_DS_PHASES=1: print the list-driven sub-pel searches' phase
// times (g_ds_ph, microseconds per job / per workgroup) to stderr and clear them
extern "C" int rv_ds_phase_dump(void) {
  unsigned long long h[16];
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpyFromSymbol(h, HIP_SYMBOL(g_ds_ph), sizeof(h)) != hipSuccess)
    return rv_set_error(RV_EHIP, "rv_ds_phase_dump");
  const double us = 0.01;  // wall_clock64: 100 MHz
  const double j = h[5] ? (double)h[5] : 1.0, w = h[8] ? (double)h[8] : 1.0;
  fprintf(stderr,
          "[ds phases] jobs %llu: setup %.2f us, stage+filter+SAD %.2f us, exchange %.2f us, "
          "job %.2f us per job; %.2f iterations, %.2f stagings per job; workgroups %llu: %.2f us each\n",
          h[5], h[0] * us / j, h[1] * us / j, h[2] * us / j, h[3] * us / j, h[4] / j, h[6] / j, h[8],
          h[7] * us / w);
  memset(h, 0, sizeof(h));
  return hipMemcpyToSymbol(HIP_SYMBOL(g_ds_ph), h, sizeof(h)) == hipSuccess ? RV_OK : rv_set_error(RV_EHIP, "rv_ds_phase_dump");
}

// Multi-reference form used by the replay driver: jobs [n_refs][n_per_ref],
// job i searches refs[i / n_per_ref]; evals (optional) receives the
// in-range candidate evaluations per job.
static int ds_dispatch(DsArgs &a, void *stream);

int rv_diamond_search_multi(const rv_plane *org, const rv_plane *refs, int n_refs,
                            const rv_ds_job *d_jobs, int n_per_ref, int blk_w, int blk_h,
                            int subpixel, int use_satd, int allow_hp, int bit_depth,
                            rv_fs_result *d_out, uint32_t *d_evals, const ChainNext *next,
                            void *stream, const uint8_t *active, const int32_t *alist,
                            const int32_t *acount, int lper, const uint8_t *dirty,
                            int list_grid, uint32_t *eval_acc, unsigned long long *t01) {
  auto p2 = [](int v) { return v >= 4 && v <= 128 && (v & (v - 1)) == 0; };
  if (!org || !refs || n_refs < 1 || n_refs > RV_MAX_REFS || n_per_ref < 0 || !p2(blk_w) ||
      !p2(blk_h) || (bit_depth != 8 && bit_depth != 10 && bit_depth != 12) ||
      (!org->hbd && bit_depth != 8))
    return rv_set_error(RV_EINVAL, "rv_diamond_search_batch: bad arguments");
  for (int k = 0; k < n_refs; k++)
    if (refs[k].hbd != org->hbd)
      return rv_set_error(RV_EINVAL, "rv_diamond_search_batch: pixel type mismatch");
  const int n = n_refs * n_per_ref;
  if (n == 0) return RV_OK;
  DsArgs a;
  memset(&a, 0, sizeof(a));
  a.org = *org;
  for (int k = 0; k < n_refs; k++) a.ref[k] = refs[k];
  a.jobs = d_jobs;
  a.out = d_out;
  a.n = n;
  a.n_per_ref = n_per_ref;
  a.w = blk_w;
  a.h = blk_h;
  a.subpel = subpixel ? 1 : 0;
  a.satd = use_satd ? 1 : 0;
  a.hp = allow_hp ? 1 : 0;
  a.bd = bit_depth;
  a.evals = d_evals;
  a.active = active;
  a.alist = alist;
  a.acount = acount;
  a.lper = lper;
  a.dirty = alist ? dirty : nullptr;
  a.list_grid = list_grid;
  a.eval_acc = eval_acc;
  if (t01) {
    a.t0 = t01;
    a.t1 = t01 + 1;
  }
  if (alist && (!acount || lper < 0 || use_satd ||
                !((blk_w == 64 && blk_h == 64) || (blk_w == 16 && blk_h == 16 && !subpixel))))
    return rv_set_error(RV_EINVAL,
                        "rv_diamond_search_multi: list-driven launches: 64x64, or 16x16 full-pel SAD");
  if (next) a.next = *next;
  return ds_dispatch(a, stream);
}

static void ds_fill(DsArgs &a, const rv_plane *org, const rv_plane *refs, int n_refs,
                    const rv_ds_job *d_jobs, int n_per_ref, int blk, rv_fs_result *d_out,
                    int bit_depth, const int32_t *alist, const int32_t *acount, int lper,
                    const uint8_t *dirty) {
  memset(&a, 0, sizeof(a));
  a.org = *org;
  for (int k = 0; k < n_refs; k++) a.ref[k] = refs[k];
  a.jobs = d_jobs;
  a.out = d_out;
  a.n = n_refs * n_per_ref;
  a.n_per_ref = n_per_ref;
  a.w = a.h = blk;
  a.bd = bit_depth;
  a.alist = alist;
  a.acount = acount;
  a.lper = lper;
  a.dirty = dirty;
}

// A round's list-driven F2 (16x16 full-pel SAD on the half-resolution
// planes) and F3 full-pel (64x64 SAD) in one launch (ds_f2_f3_kernel);
// pools of list_grid workgroups each (0: ds_list_grid()).
int rv_diamond_f2_f3(const rv_plane *org_h, const rv_plane *refs_h, const rv_ds_job *jobs_h,
                     rv_fs_result *out_h, const uint8_t *dirty_h, const rv_plane *org,
                     const rv_plane *refs, const rv_ds_job *jobs, rv_fs_result *out,
                     const uint8_t *dirty, const ChainNext *next, int n_refs, int n_per_ref,
                     int bit_depth, const int32_t *alist, const int32_t *acount, int list_grid,
                     void *stream, const rv_ds_job *jobs_sub, rv_fs_result *out_sub,
                     uint32_t *eval_acc, unsigned long long *t01) {
  if (!org_h || !refs_h || !org || !refs || n_refs < 1 || n_refs > RV_MAX_REFS || n_per_ref <= 0 ||
      !alist || !acount || org->hbd != org_h->hbd)
    return rv_set_error(RV_EINVAL, "rv_diamond_f2_f3: bad arguments");
  DsArgs f2, f3;
  ds_fill(f2, org_h, refs_h, n_refs, jobs_h, n_per_ref * 4, 16, out_h, bit_depth, alist, acount, 4,
          dirty_h);
  ds_fill(f3, org, refs, n_refs, jobs, n_per_ref, 64, out, bit_depth, alist, acount, 1, dirty);
  if (next) f3.next = *next;
  // jobs_sub / out_sub (optional): F3's sub-pel searches fused behind the
  // full-pel ones (SAD, no half-pel: the rounds' 64x64 diamond)
  DsArgs f3s;
  ds_fill(f3s, org, refs, n_refs, jobs_sub ? jobs_sub : jobs, n_per_ref, 64, out_sub ? out_sub : out,
          bit_depth, alist, acount, 1, dirty);
  f3s.subpel = 1;
  static const bool phases = getenv("RAV1E_HIP_DS_PHASES") && getenv("RAV1E_HIP_DS_PHASES")[0] == '1';
  f3s.ph = phases ? 1 : 0;
  const int fuse = jobs_sub && out_sub ? 1 : 0;
  if (fuse) f3s.eval_acc = eval_acc;  // the kernel probe (null: off)
  unsigned long long *ts = fuse ? t01 : nullptr;
  const int pool = list_grid ? list_grid : ds_list_grid();
  const int g2 = std::min(pool, (f2.n + 15) / 16), g3 = std::min(f3.n, pool);
  hipStream_t s = rv_resolve_stream(stream);
  if (org->hbd)
    ds_f2_f3_kernel<uint16_t><<<g2 + g3, 256, 0, s>>>(f2, f3, f3s, g2, fuse, ts);
  else
    ds_f2_f3_kernel<uint8_t><<<g2 + g3, 256, 0, s>>>(f2, f3, f3s, g2, fuse, ts);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

// Launch a filled DsArgs: the wavefront-per-candidate fast path where it
// applies (SAD, W,H in {16,32,64}), else the workgroup-per-candidate kernel.
static int ds_dispatch(DsArgs &a, void *stream) {
  const int n = a.n, blk_w = a.w, blk_h = a.h, subpixel = a.subpel;
  const rv_plane *org = &a.org;
  hipStream_t s = rv_resolve_stream(stream);
  // RAV1E_HIP_DS_GENERIC=1: the workgroup-per-candidate kernel for SATD and
  // the small blocks (A/B)
  static const bool grp_on = [] {
    const char *e = getenv("RAV1E_HIP_DS_GENERIC");
    return !(e && e[0] == '1');
  }();
  const bool fast = (grp_on && (org->hbd ? try_grp<uint16_t>(a, s) : try_grp<uint8_t>(a, s))) ||
                    (org->hbd ? try_fast<uint16_t>(a, s) : try_fast<uint8_t>(a, s));
  if (!fast) {
    const size_t lds = subpixel ? (size_t)((blk_w + 7) * (blk_h + 7) + (blk_h + 7) * blk_w +
                                           blk_w * blk_h) * sizeof(int16_t)
                                : 0;
    if (org->hbd)
      diamond_kernel<uint16_t><<<n, kDsThreads, lds, s>>>(a);
    else
      diamond_kernel<uint8_t><<<n, kDsThreads, lds, s>>>(a);
  }
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

extern "C" int rv_diamond_search_batch(const rv_plane *org, const rv_plane *ref,
                                       const rv_ds_job *d_jobs, int n, int blk_w,
                                       int blk_h, int subpixel, int use_satd,
                                       int allow_hp, int bit_depth,
                                       rv_fs_result *d_out, void *stream) {
  if (!ref) return rv_set_error(RV_EINVAL, "rv_diamond_search_batch: null ref");
  return rv_diamond_search_multi(org, ref, 1, d_jobs, n, blk_w, blk_h, subpixel, use_satd,
                                 allow_hp, bit_depth, d_out, nullptr, nullptr, stream, nullptr,
                                 nullptr, nullptr, 0, nullptr, 0, nullptr, nullptr);
}

// telescopic_subpel_search (src/me.rs:858-941) for every job in one launch:
// start[i] = (best_mv, lowest_cost) from the full-pel search (or the
// use_satd recomputation, src/me.rs:232-253); out[i] = the result.
extern "C" int rv_telescopic_subpel_batch(const rv_plane *org, const rv_plane *ref,
                                          const rv_ds_job *d_jobs, const rv_fs_result *d_start,
                                          int n, int blk_w, int blk_h, int use_satd,
                                          int allow_hp, int bit_depth, rv_fs_result *d_out,
                                          void *stream) {
  auto p2 = [](int v) { return v >= 4 && v <= 128 && (v & (v - 1)) == 0; };
  if (!org || !ref || !d_start || n < 0 || !p2(blk_w) || !p2(blk_h) || ref->hbd != org->hbd ||
      (bit_depth != 8 && bit_depth != 10 && bit_depth != 12) || (!org->hbd && bit_depth != 8))
    return rv_set_error(RV_EINVAL, "rv_telescopic_subpel_batch: bad arguments");
  if (n == 0) return RV_OK;
  DsArgs a;
  memset(&a, 0, sizeof(a));
  a.org = *org;
  a.ref[0] = *ref;
  a.jobs = d_jobs;
  a.out = d_out;
  a.n = n;
  a.n_per_ref = n;
  a.w = blk_w;
  a.h = blk_h;
  a.subpel = 1;
  a.satd = use_satd ? 1 : 0;
  a.hp = allow_hp ? 1 : 0;
  a.bd = bit_depth;
  a.tele = 1;
  a.start = d_start;
  return ds_dispatch(a, stream);
}
