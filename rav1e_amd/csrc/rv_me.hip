// rv_me.hip -- batched exhaustive motion search (gfx950).
//
// full_search (src/me.rs:943-990) for many blocks in one launch: one
// workgroup per block.  The reference evaluates every candidate window in
// raster order (y outer, x inner) and keeps the first strict minimum of
// cost = 256 * SAD + rate * lambda; here every lane evaluates a tile of
// candidates and the workgroup reduces (cost, raster index)
// lexicographically, which selects the same candidate.
//
// Fast path (16x16 block, step 1, u8 and u16 -- the quarter-resolution search of
// every 64x64 superblock, estimate_motion_ss4 src/me.rs:1023-1075): the
// search window is staged in LDS in bands, the 16x16 source block lives in
// 64 VGPRs, and each lane computes a 4-wide x 8-tall candidate tile with
// v_sad_u8 on packed dwords (v_alignbyte for the 3 unaligned shifts), so a
// reference row is read from LDS once per 32 candidates.  The search is
// VALU-bound (~256 |a-b| per candidate), not HBM-bound.
#include <stdlib.h>
#include <string.h>

#include "rv_chain.h"
#include "rv_device.h"

namespace rv {

constexpr int kFsThreads = 256;

// get_mv_rate / diff_to_rate (src/me.rs:1006-1021)
__device__ __forceinline__ uint32_t diff_to_rate(int16_t diff, int hp) {
  int16_t d = hp ? diff : (int16_t)(diff >> 1);
  if (d == 0) return 0;
  uint32_t a = (uint16_t)(d < 0 ? -d : d);
  return 2u * (16u - (uint32_t)(__builtin_clz(a) - 16));
}
__device__ __forceinline__ uint32_t mv_rate(int16_t row, int16_t col,
                                            rv_mv p, int hp) {
  return diff_to_rate((int16_t)(row - p.row), hp) +
         diff_to_rate((int16_t)(col - p.col), hp);
}

__device__ __forceinline__ uint64_t group_min_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t w = __shfl_xor(v, o, 64);
    v = w < v ? w : v;
  }
  return v;
}

struct Best {
  uint64_t cost;
  uint32_t idx;
};
__device__ __forceinline__ bool better(uint64_t c, uint32_t i, const Best &b) {
  return c < b.cost || (c == b.cost && i < b.idx);
}

__device__ __forceinline__ uint64_t cand_cost(uint32_t sad, int x, int y,
                                              const rv_fs_job &jb, int hp) {
  const int16_t row = (int16_t)(8 * (y - jb.po_y));
  const int16_t col = (int16_t)(8 * (x - jb.po_x));
  const uint32_t r1 = mv_rate(row, col, jb.pmv[0], hp);
  const uint32_t r2 = mv_rate(row, col, jb.pmv[1], hp);
  const uint32_t rate = r1 < r2 + 1 ? r1 : r2 + 1;
  return 256ull * sad + (uint64_t)rate * jb.lambda;
}

// Workgroup argmin over (cost, idx); lane 0 of wave 0 holds the result.
__device__ __forceinline__ Best block_best(Best b) {
  __shared__ uint64_t sc[kFsThreads / 64];
  __shared__ uint32_t si[kFsThreads / 64];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    uint64_t c = __shfl_xor(b.cost, o, 64);
    uint32_t i = __shfl_xor(b.idx, o, 64);
    if (better(c, i, b)) b = Best{c, i};
  }
  const int wid = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sc[wid] = b.cost;
    si[wid] = b.idx;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    for (int k = 1; k < (int)(blockDim.x >> 6); k++)
      if (better(sc[k], si[k], b)) b = Best{sc[k], si[k]};
  return b;
}

__device__ __forceinline__ rv_fs_result write_result(const rv_fs_job &jb, Best b,
                                             int nx, int step,
                                             rv_fs_result *out) {
  rv_fs_result r;
  r.reserved = 0;
  if (b.cost == ~0ull && b.idx == 0xffffffffu) {
    r.best_mv = rv_mv{0, 0};  // MotionVector::default(), cost u64::MAX
    r.cost = ~0ull;
  } else {
    const int iy = b.idx / nx, ix = b.idx - iy * nx;
    const int x = jb.x_lo + ix * step, y = jb.y_lo + iy * step;
    r.best_mv = rv_mv{(int16_t)(8 * (y - jb.po_y)), (int16_t)(8 * (x - jb.po_x))};
    r.cost = b.cost;
  }
  *out = r;
  return r;
}

struct FsArgs {
  rv_plane org;
  rv_plane ref[RV_MAX_REFS];  // job i searches ref[i / n_per_ref]
  const rv_fs_job *jobs;
  rv_fs_result *out;
  int n, n_per_ref, hp, bw, bh, step;
  ChainNext next;  // replay: feed the winner into the next stage's jobs
  const uint32_t *box[RV_MAX_REFS];  // rv_plane_box_sums of each ref (SEA path)
};

// blockIdx -> job with consecutive jobs on one XCD (blocks are dealt
// round-robin to the 8 XCDs; neighbouring superblocks share reference rows
// in that XCD's L2).  The grid is a multiple of 8.
__device__ __forceinline__ int fs_job_index() {
  const int per = (int)gridDim.x >> 3;
  return ((int)blockIdx.x & 7) * per + ((int)blockIdx.x >> 3);
}

// ---- generic path: one lane per candidate --------------------------------
// The result is valid in thread 0.
template <typename Px>
__device__ rv_fs_result fs_generic_body(const rv_plane &org, const rv_plane &ref,
                                        const rv_fs_job &jb, int bw, int bh,
                                        int step, int hp, rv_fs_result *out) {
  const int nx = jb.x_hi >= jb.x_lo ? (jb.x_hi - jb.x_lo) / step + 1 : 0;
  const int ny = jb.y_hi >= jb.y_lo ? (jb.y_hi - jb.y_lo) / step + 1 : 0;
  const Px *o = plane_ptr<Px>(org, jb.po_x, jb.po_y);
  Best b{~0ull, 0xffffffffu};
  for (int c = threadIdx.x; c < nx * ny; c += blockDim.x) {
    const int iy = c / nx, ix = c - iy * nx;
    const int x = jb.x_lo + ix * step, y = jb.y_lo + iy * step;
    const Px *r = plane_ptr<Px>(ref, x, y);
    uint32_t sad = 0;
    for (int rr = 0; rr < bh; rr++) {
      const Px *po = o + (int64_t)rr * org.stride;
      const Px *pr = r + (int64_t)rr * ref.stride;
      if constexpr (sizeof(Px) == 1) {
        for (int cc = 0; cc < bw; cc += 4)
          sad = sad_u8x4(load_u32_unaligned(po + cc),
                         load_u32_unaligned(pr + cc), sad);
      } else {
        for (int cc = 0; cc < bw; cc++) {
          int d = (int)po[cc] - (int)pr[cc];
          sad += (uint32_t)(d < 0 ? -d : d);
        }
      }
    }
    const uint64_t cost = cand_cost(sad, x, y, jb, hp);
    if (better(cost, (uint32_t)c, b)) b = Best{cost, (uint32_t)c};
  }
  b = block_best(b);
  rv_fs_result res{};
  if (threadIdx.x == 0) res = write_result(jb, b, nx > 0 ? nx : 1, step, out);
  return res;
}

template <typename Px>
__global__ __launch_bounds__(kFsThreads) void fs_generic_kernel(FsArgs a) {
  const int job = fs_job_index();
  if (job >= a.n) return;
  const rv_fs_job jb = a.jobs[job];
  const rv_fs_result res = fs_generic_body<Px>(a.org, a.ref[job / a.n_per_ref], jb, a.bw, a.bh,
                                               a.step, a.hp, a.out + job);
  if (threadIdx.x == 0) chain_emit(a.next, job, a.n_per_ref, a.n / a.n_per_ref, res.best_mv);
}

// ---- fast path: 16x16, step 1 (u8 and u16) --------------------------------
constexpr int kTileRows = 8;  // candidate rows per lane

template <typename Px>
struct Fs16 {
  static constexpr int B = (int)sizeof(Px);
  static constexpr int ODW = 16 * B / 4;        // source dwords per row
  static constexpr int WV = (4 + 16) * B / 4;   // band dwords a 4-wide tile row touches
  // LDS search band: 28 KiB for u8 (5 workgroups per CU), 56 KiB for u16
  // (its rows are twice as long; keeps ~40 candidate rows per band)
  static constexpr int kLdsWords = B == 1 ? 7 * 1024 : 14 * 1024;
};

template <typename Px>
__device__ __forceinline__ uint32_t sad_px(uint32_t a, uint32_t b, uint32_t acc) {
  if constexpr (sizeof(Px) == 1)
    return __builtin_amdgcn_sad_u8(a, b, acc);
  else
    return __builtin_amdgcn_sad_u16(a, b, acc);
}

template <typename Px>
__global__ __launch_bounds__(kFsThreads) void fs16_kernel(FsArgs a) {
  using G = Fs16<Px>;
  constexpr int B = G::B, ODW = G::ODW, WV = G::WV;
  __shared__ uint32_t band[G::kLdsWords];
  const int job = fs_job_index();
  if (job >= a.n) return;
  const rv_fs_job jb = a.jobs[job];
  const rv_plane &ref = a.ref[job / a.n_per_ref];
  const int nx = jb.x_hi >= jb.x_lo ? jb.x_hi - jb.x_lo + 1 : 0;
  const int ny = jb.y_hi >= jb.y_lo ? jb.y_hi - jb.y_lo + 1 : 0;
  const int tid = threadIdx.x;

  // 16x16 source block -> LDS; every lane reads the same row, so the reads
  // are broadcasts and the VGPRs stay with the accumulators
  __shared__ uint32_t orgs[16 * ODW];
  if (tid < 16 * ODW) {
    const uint8_t *o = (const uint8_t *)plane_ptr<Px>(a.org, jb.po_x, jb.po_y);
    orgs[tid] = load_u32_unaligned(o + (int64_t)(tid / ODW) * a.org.stride * B + 4 * (tid % ODW));
  }

  const int tx_n = (nx + 3) >> 2;        // 4-wide candidate columns
  const int rw = tx_n * B + WV - B;      // band row length in dwords
  if (rw * (2 * kTileRows + 15) > G::kLdsWords) {  // window too wide for a band
    const rv_fs_result res = fs_generic_body<Px>(a.org, ref, jb, 16, 16, 1, a.hp, a.out + job);
    if (tid == 0) chain_emit(a.next, job, a.n_per_ref, a.n / a.n_per_ref, res.best_mv);
    return;
  }
  const int vis_w = (nx + 15) * B;       // bytes of a ref row that exist
  int pb = G::kLdsWords / rw - (kTileRows + 15);  // candidate rows per band
  pb = (pb / kTileRows) * kTileRows;

  Best b{~0ull, 0xffffffffu};
  uint64_t bkey = ~0ull;  // (u32 cost << 32 | index) while costs fit u32
  const bool small_cost = jb.lambda < (1u << 25);
  const uint8_t *rbase = (const uint8_t *)plane_ptr<Px>(ref, jb.x_lo, jb.y_lo);
  const int64_t rstride = (int64_t)ref.stride * B;
  for (int y0 = 0; y0 < ny; y0 += pb) {
    const int rows = ny - y0 < pb ? ny - y0 : pb;
    const int lrows = rows + 15;  // ref rows with data
    const int ty_n = (rows + kTileRows - 1) / kTileRows;
    const int brows = ty_n * kTileRows + 15;  // rows the tiles touch
    const int total = brows * rw;
    __syncthreads();
    // band fill: 8 independent loads in flight per thread before the LDS
    // stores, so the fill costs ~one memory round trip, not eight
    for (int i0 = tid; i0 < total; i0 += 8 * kFsThreads) {
      uint32_t v[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int i = i0 + u * kFsThreads;
        const int r = i / rw, c = 4 * (i - r * rw);
        uint32_t x = 0;
        if (i < total && r < lrows) {
          const uint8_t *p = rbase + (int64_t)(y0 + r) * rstride + c;
          if (c + 3 < vis_w) {
            x = load_u32_unaligned(p);
          } else {
#pragma unroll
            for (int k = 0; k < 4; k++)
              if (c + k < vis_w) x |= (uint32_t)p[k] << (8 * k);
          }
        }
        v[u] = x;
      }
#pragma unroll
      for (int u = 0; u < 8; u++)
        if (i0 + u * kFsThreads < total) band[i0 + u * kFsThreads] = v[u];
    }
    __syncthreads();
    const int tasks = tx_n * ty_n;
    for (int t = tid; t < tasks; t += blockDim.x) {
      const int tcy = t / tx_n, tcx = t - tcy * tx_n;
      const int cy0 = tcy * kTileRows;
      uint32_t acc[kTileRows][4];
#pragma unroll
      for (int c = 0; c < kTileRows; c++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[c][j] = 0;
      const uint32_t *bp = band + cy0 * rw + tcx * B;
#pragma unroll 1
      for (int yy = 0; yy < kTileRows + 15; yy++) {
        uint32_t wv[WV];
#pragma unroll
        for (int i = 0; i < WV; i++) wv[i] = bp[yy * rw + i];
        // sh[j][i]: reference dword under source dword i for candidate
        // column j (u8: byte shift j; u16: dword j/2, half-word shift j&1)
        uint32_t sh[4][ODW];
#pragma unroll
        for (int i = 0; i < ODW; i++) {
          if constexpr (B == 1) {
            sh[0][i] = wv[i];
            sh[1][i] = __builtin_amdgcn_alignbyte(wv[i + 1], wv[i], 1);
            sh[2][i] = __builtin_amdgcn_alignbyte(wv[i + 1], wv[i], 2);
            sh[3][i] = __builtin_amdgcn_alignbyte(wv[i + 1], wv[i], 3);
          } else {
            sh[0][i] = wv[i];
            sh[1][i] = __builtin_amdgcn_alignbyte(wv[i + 1], wv[i], 2);
            sh[2][i] = wv[i + 1];
            sh[3][i] = __builtin_amdgcn_alignbyte(wv[i + 2], wv[i + 1], 2);
          }
        }
#pragma unroll
        for (int c = 0; c < kTileRows; c++) {
          const int r = yy - c;  // source row against candidate row c
          if (r >= 0 && r < 16) {
            uint32_t ov[ODW];
#pragma unroll
            for (int i = 0; i < ODW; i += 4) {
              const uint4 o4 = *reinterpret_cast<const uint4 *>(orgs + r * ODW + i);
              ov[i] = o4.x;
              ov[i + 1] = o4.y;
              ov[i + 2] = o4.z;
              ov[i + 3] = o4.w;
            }
#pragma unroll
            for (int j = 0; j < 4; j++)
#pragma unroll
              for (int i = 0; i < ODW; i++) acc[c][j] = sad_px<Px>(ov[i], sh[j][i], acc[c][j]);
          }
        }
      }
      // cost = 256 * sad + rate * lambda (get_mv_rate, src/me.rs:1006-1021):
      // the rate splits into a row part per tile row and a column part per
      // tile column, so a tile needs 24 diff_to_rate instead of 128.  For a
      // 16x16 block 256 * sad < 2^28 (12-bit), so with lambda < 2^25 the
      // cost fits u32 and (cost, raster index) packs into one u64 key whose
      // minimum is the reference's first strict minimum.
      int rr0[kTileRows], rr1[kTileRows], rc0[4], rc1[4];
#pragma unroll
      for (int c = 0; c < kTileRows; c++) {
        const int16_t row = (int16_t)(8 * (jb.y_lo + y0 + cy0 + c - jb.po_y));
        rr0[c] = diff_to_rate((int16_t)(row - jb.pmv[0].row), a.hp);
        rr1[c] = diff_to_rate((int16_t)(row - jb.pmv[1].row), a.hp);
      }
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int16_t col = (int16_t)(8 * (jb.x_lo + 4 * tcx + j - jb.po_x));
        rc0[j] = diff_to_rate((int16_t)(col - jb.pmv[0].col), a.hp);
        rc1[j] = diff_to_rate((int16_t)(col - jb.pmv[1].col), a.hp);
      }
#pragma unroll
      for (int c = 0; c < kTileRows; c++) {
        const int iy = y0 + cy0 + c;
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const int ix = 4 * tcx + j;
          if (ix < nx && cy0 + c < rows) {
            const uint32_t r1 = rr0[c] + rc0[j], r2 = rr1[c] + rc1[j];
            const uint32_t rate = r1 < r2 + 1 ? r1 : r2 + 1;
            const uint32_t idx = (uint32_t)(iy * nx + ix);
            if (small_cost) {
              const uint64_t key =
                  ((uint64_t)((acc[c][j] << 8) + rate * jb.lambda) << 32) | idx;
              bkey = key < bkey ? key : bkey;
            } else {
              const uint64_t cost = 256ull * acc[c][j] + (uint64_t)rate * jb.lambda;
              if (better(cost, idx, b)) b = Best{cost, idx};
            }
          }
        }
      }
    }
  }
  if (bkey != ~0ull && better(bkey >> 32, (uint32_t)bkey, b)) b = Best{bkey >> 32, (uint32_t)bkey};
  b = block_best(b);
  if (tid == 0) {
    const rv_fs_result res = write_result(jb, b, nx > 0 ? nx : 1, 1, a.out + job);
    chain_emit(a.next, job, a.n_per_ref, a.n / a.n_per_ref, res.best_mv);
  }
}

// ---- exact successive-elimination path: 16x16, step 1 ---------------------
// The triangle inequality bounds every candidate from below:
//   SAD(org, cand) >= sum over any partition into blocks q of |S_org,q - S_cand,q|
// (S = pixel sum), so cost >= LB = 256 * that + rate * lambda.  A candidate
// whose LB exceeds an achieved cost UB cannot be the strict first minimum,
// so skipping it leaves the result of full_search (src/me.rs:943-990)
// unchanged bit for bit.  The reference's box sums come from tables built
// once per reference frame (rv_plane_box_sums; every superblock of several
// frames searches the same reference), stored as horizontal pairs
// (S48(x, y) | S48(x + 8, y) << 16 for 4-tall x 8-wide blocks and
// S4(x, y) | S4(x + 4, y) << 16), so one v_sad_u16 against the packed
// source sums gives two block terms: the 8-block bound of a candidate is 4
// v_sad_u16 from four aligned dwords, the sharper 16-block 4x4 bound 8.
// Per job:
//   (1) the 4x4 (kSeaNb) neighbourhood of mv 0, clamped into the window
//       (natural motion puts the minimum there), is evaluated exactly -> UB;
//       a neighbourhood clamped mostly away (mv 0 on a window corner or
//       outside the window) just gives a looser first UB;
//   (2) the window's 4-wide x 8-tall candidate tiles are taken in chunks of
//       one tile per lane: each lane computes its tile's 8-block bounds (20
//       dwordx4 table rows, L2-resident) against the live UB and appends the
//       survivors to an LDS list (on the replay's content ~1 in 150
//       candidates; 8x8 quadrants would keep ~9x more); then the list is
//       spread over all lanes, each survivor checked against the 4x4 bound
//       (which keeps ~1 in 5) and, if it passes, evaluated exactly (which
//       tightens the UB for the next chunk).
// Out-of-window candidates of edge tiles get a bound >= 2^30, above every
// real cost (lambda < 2^23 here; larger lambdas take the exhaustive path).
// Each wavefront's list holds its 64 tiles' worst case (64 x 32), so it
// never overflows.
constexpr int kSeaList = kFsThreads * 32;  // survivors of one chunk, worst case
constexpr uint32_t kSeaOut = 1u << 30;
constexpr int kSeaNb = 4;  // side of the exactly evaluated neighbourhood of mv 0

// Reference rows are read with dword-aligned loads and realigned in
// registers (v_alignbyte): lane addresses that are not 4-byte aligned make a
// multi-dword global load ~3x slower (tools/ubench/load_align.hip).  The
// extra trailing dword is only read when the row is misaligned; it then
// holds needed bytes, so no read leaves a dword-aligned allocation.

// Exact SAD of the 16x16 source block (LDS, 4 * B dwords per row) against
// the reference block at p (global memory, rs bytes per row, rs % 4 == 0).
template <typename Px>
__device__ __forceinline__ uint32_t sad16_global(const uint32_t *orgs, const uint8_t *p,
                                                 int64_t rs) {
  constexpr int B = (int)sizeof(Px);
  const int sh = (int)((uintptr_t)p & 3);
  const uint8_t *pa = p - sh;
  uint32_t sad = 0;
#pragma unroll 8
  for (int r = 0; r < 16; r++) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(pa + r * rs);
    uint32_t v[4 * B + 1];
#pragma unroll
    for (int h = 0; h < B; h++) {
      const uint4 x = *reinterpret_cast<const uint4 *>(w + 4 * h);
      v[4 * h] = x.x;
      v[4 * h + 1] = x.y;
      v[4 * h + 2] = x.z;
      v[4 * h + 3] = x.w;
    }
    v[4 * B] = sh ? w[4 * B] : 0u;
#pragma unroll
    for (int h = 0; h < B; h++) {
      const uint4 o = *reinterpret_cast<const uint4 *>(orgs + r * 4 * B + 4 * h);
      sad = sad_px<Px>(o.x, __builtin_amdgcn_alignbyte(v[4 * h + 1], v[4 * h], sh), sad);
      sad = sad_px<Px>(o.y, __builtin_amdgcn_alignbyte(v[4 * h + 2], v[4 * h + 1], sh), sad);
      sad = sad_px<Px>(o.z, __builtin_amdgcn_alignbyte(v[4 * h + 3], v[4 * h + 2], sh), sad);
      sad = sad_px<Px>(o.w, __builtin_amdgcn_alignbyte(v[4 * h + 4], v[4 * h + 3], sh), sad);
    }
  }
  return sad;
}

struct SeaCtx {
  const uint32_t *box;   // paired 8x8 table at window position (0, 0)
  const uint32_t *box4;  // paired 4x4 table at window position (0, 0)
  int stride;            // table row pitch (elements)
  int nx, ny, tx_n;
  const uint32_t *s48;   // LDS: packed source 4-tall x 8-wide block sums, block row i: cols 0-7 | 8-15
  const uint32_t *s4;    // LDS: packed source 4x4 sums, row i: [2i] = cols 0|1, [2i+1] = cols 2|3
};

// rate * lambda of the tile's candidates (get_mv_rate, src/me.rs:1006-1021)
// as row terms rr and column terms rc; candidates outside the window get
// kSeaOut from both.  SAME: pmv[0] == pmv[1], so min(r0, r1 + 1) is r0 and
// the product splits: rr0 / rc0 already hold rate * lambda.
template <bool SAME>
struct SeaRates {
  uint32_t rr0[kTileRows], rr1[kTileRows], rc0[4], rc1[4];
  __device__ __forceinline__ SeaRates(const SeaCtx &c, const rv_fs_job &jb, int hp, int cy0,
                                      int tcx) {
#pragma unroll
    for (int k = 0; k < kTileRows; k++) {
      const int16_t rw = (int16_t)(8 * (jb.y_lo + cy0 + k - jb.po_y));
      const bool in = cy0 + k < c.ny;
      rr0[k] = in ? diff_to_rate((int16_t)(rw - jb.pmv[0].row), hp) : kSeaOut;
      rr1[k] = SAME ? 0u : (in ? diff_to_rate((int16_t)(rw - jb.pmv[1].row), hp) : kSeaOut);
      if (SAME && in) rr0[k] *= jb.lambda;
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int16_t cl = (int16_t)(8 * (jb.x_lo + 4 * tcx + j - jb.po_x));
      const bool in = 4 * tcx + j < c.nx;
      rc0[j] = in ? diff_to_rate((int16_t)(cl - jb.pmv[0].col), hp) : kSeaOut;
      rc1[j] = SAME ? 0u : (in ? diff_to_rate((int16_t)(cl - jb.pmv[1].col), hp) : kSeaOut);
      if (SAME && in) rc0[j] *= jb.lambda;
    }
  }
  __device__ __forceinline__ uint32_t rl(int k, int j, uint32_t lambda) const {
    if (SAME) return rr0[k] + rc0[j];
    const uint32_t r1 = rr0[k] + rc0[j], r2 = rr1[k] + rc1[j] + 1;
    const uint32_t r = r1 < r2 ? r1 : r2;
    return r >= kSeaOut ? kSeaOut : r * lambda;
  }
};

// Mask of the candidates of tile t whose 4x8 lower bound (eight 4-tall x
// 8-wide blocks) is <= ub: 256 * l + rate * lambda <= ub, tested as
// 256 * l + rc[j] <= ub - rr[k] when SAME.
template <bool SAME>
__device__ __forceinline__ uint32_t sea_tile(const SeaCtx &c, const rv_fs_job &jb, int hp,
                                             int t, uint32_t ub) {
  const int tcy = t / c.tx_n, tcx = t - tcy * c.tx_n;
  const int cy0 = tcy * kTileRows;
  // 8 block terms per candidate: table rows k + 4 i, i = 0..3, in two
  // halves of 12 rows (block rows 0-1, then 2-3)
  uint32_t acc[kTileRows][4];
#pragma unroll
  for (int k = 0; k < kTileRows; k++)
#pragma unroll
    for (int j = 0; j < 4; j++) acc[k][j] = 0;
  // table rows 0..19 in five groups of four, each row loaded once (block
  // row i of candidate row k is table row k + 4 i)
  const uint32_t *bp = c.box + (int64_t)cy0 * c.stride + 4 * tcx;
#pragma unroll
  for (int g = 0; g < 5; g++) {
    uint4 row[4];
#pragma unroll
    for (int u = 0; u < 4; u++)
      row[u] = *reinterpret_cast<const uint4 *>(bp + (int64_t)(4 * g + u) * c.stride);
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const int r = 4 * g + u;
      const uint32_t a[4] = {row[u].x, row[u].y, row[u].z, row[u].w};
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int k = r - 4 * i;
        if (k >= 0 && k < kTileRows) {
#pragma unroll
          for (int j = 0; j < 4; j++) acc[k][j] = __builtin_amdgcn_sad_u16(a[j], c.s48[i], acc[k][j]);
        }
      }
    }
  }
  const SeaRates<SAME> rt(c, jb, hp, cy0, tcx);
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < kTileRows; k++) {
    // SAME: the row term moves to the threshold (out-of-window rows carry
    // kSeaOut > ub and never pass)
    const uint32_t rk = SAME ? rt.rr0[k] : 0u;
    const uint32_t thr = ub >= rk ? ub - rk : 0u;
    const bool row_ok = ub >= rk;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t lb = (acc[k][j] << 8) + (SAME ? rt.rc0[j] : rt.rl(k, j, jb.lambda));
      if (row_ok && lb <= thr) m |= 1u << (k * 4 + j);
    }
  }
  return m;
}

// 4x4 lower bound (sixteen block terms, >= the 8x8 bound) of candidate
// (iy, ix): 8 paired table dwords.
__device__ __forceinline__ uint32_t sea_lb4(const SeaCtx &c, int iy, int ix) {
  const uint32_t *q = c.box4 + (int64_t)iy * c.stride + ix;
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    w[2 * i] = q[(int64_t)(4 * i) * c.stride];
    w[2 * i + 1] = q[(int64_t)(4 * i) * c.stride + 8];
  }
  uint32_t l = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) l = __builtin_amdgcn_sad_u16(w[i], c.s4[i], l);
  return l;
}

template <typename Px, bool SAME>
__device__ __forceinline__ void sea_search(const FsArgs &a, const rv_fs_job &jb, int job,
                                           const rv_plane &ref, const SeaCtx &c,
                                           const uint32_t *orgs, uint32_t *list, uint32_t *cnt,
                                           uint32_t &ub_s) {
  constexpr int B = (int)sizeof(Px);
  const int tid = threadIdx.x;
  const int nx = c.nx, ny = c.ny, tasks = c.tx_n * ((ny + kTileRows - 1) / kTileRows);
  const uint8_t *rbase = (const uint8_t *)plane_ptr<Px>(ref, jb.x_lo, jb.y_lo);
  const int64_t rs = (int64_t)ref.stride * B;
  auto rate_l = [&](int iy, int ix) __attribute__((always_inline)) -> uint32_t {
    const int16_t row = (int16_t)(8 * (jb.y_lo + iy - jb.po_y));
    const int16_t col = (int16_t)(8 * (jb.x_lo + ix - jb.po_x));
    const uint32_t r1 = diff_to_rate((int16_t)(row - jb.pmv[0].row), a.hp) +
                        diff_to_rate((int16_t)(col - jb.pmv[0].col), a.hp);
    const uint32_t r2 = diff_to_rate((int16_t)(row - jb.pmv[1].row), a.hp) +
                        diff_to_rate((int16_t)(col - jb.pmv[1].col), a.hp);
    return (r1 < r2 + 1 ? r1 : r2 + 1) * jb.lambda;
  };
  // exact (u32 cost << 32 | raster index) of candidate (iy, ix)
  auto exact_key = [&](int iy, int ix, uint32_t rl) __attribute__((always_inline)) -> uint64_t {
    const uint32_t sad = sad16_global<Px>(orgs, rbase + iy * rs + ix * B, rs);
    return ((uint64_t)((sad << 8) + rl) << 32) | (uint32_t)(iy * nx + ix);
  };

  // (1) the kSeaNb x kSeaNb candidates around mv 0, clamped into the window
  uint64_t bkey = ~0ull;
  {
    int cx = jb.po_x - jb.x_lo, cy = jb.po_y - jb.y_lo;
    cx = cx < 0 ? 0 : cx >= nx ? nx - 1 : cx;
    cy = cy < 0 ? 0 : cy >= ny ? ny - 1 : cy;
    const int ix = cx - kSeaNb / 2 + tid % kSeaNb, iy = cy - kSeaNb / 2 + tid / kSeaNb;
    if (tid < kSeaNb * kSeaNb && ix >= 0 && ix < nx && iy >= 0 && iy < ny) {
      bkey = exact_key(iy, ix, rate_l(iy, ix));
      atomicMin(&ub_s, (uint32_t)(bkey >> 32));
    }
  }
  __syncthreads();
  // (2) chunks of one tile per lane: 8x8 bounds -> list -> 4x4 bound ->
  // exact.  Each wavefront keeps its own survivor list and works through
  // its tiles with wave-local synchronisation only: the wavefronts of a job
  // run decoupled (one's table loads overlap another's exact evaluations)
  // and share only the bound, which only tightens.
  const int lane = tid & 63;
  uint32_t *wl = list + (tid >> 6) * (kSeaList / (kFsThreads / 64));
  uint32_t *wc = cnt + (tid >> 6);
  for (int base = 0; base < tasks; base += kFsThreads) {
    const int t = base + tid;
    if (t < tasks) {
      uint32_t m = sea_tile<SAME>(c, jb, a.hp, t, *(volatile uint32_t *)&ub_s);
      if (m) {
        const int tcy = t / c.tx_n, tcx = t - tcy * c.tx_n;
        uint32_t slot = atomicAdd(wc, (uint32_t)__builtin_popcount(m));
        while (m) {
          const int bit = __builtin_ctz(m);
          m &= m - 1;
          wl[slot++] = ((uint32_t)(tcy * kTileRows + (bit >> 2)) << 16) | (uint32_t)(4 * tcx + (bit & 3));
        }
      }
    }
    wave_sync();
    const int n = (int)*(volatile uint32_t *)wc;
    for (int e = lane; e < n; e += 64) {
      const uint32_t v = wl[e];
      const int iy = (int)(v >> 16), ix = (int)(v & 0xffff);
      const uint32_t rl = rate_l(iy, ix);
      const uint32_t ub = *(volatile uint32_t *)&ub_s;  // only tightens
      if ((sea_lb4(c, iy, ix) << 8) + rl > ub) continue;
      const uint64_t key = exact_key(iy, ix, rl);
      bkey = key < bkey ? key : bkey;
      atomicMin(&ub_s, (uint32_t)(key >> 32));
    }
    wave_sync();  // every read of the list and the counter done
    if (lane == 0) *wc = 0;
    wave_sync();
  }
  Best b{~0ull, 0xffffffffu};
  if (bkey != ~0ull) b = Best{bkey >> 32, (uint32_t)bkey};
  b = block_best(b);
  if (tid == 0) {
    const rv_fs_result res = write_result(jb, b, nx > 0 ? nx : 1, 1, a.out + job);
    chain_emit(a.next, job, a.n_per_ref, a.n / a.n_per_ref, res.best_mv);
  }
}

template <typename Px>
__device__ __forceinline__ void fs16_sea_body(const FsArgs &a) {
  constexpr int B = (int)sizeof(Px), ODW = 4 * B;
  __shared__ uint32_t orgs[16 * ODW];
  __shared__ uint32_t so4[16], s4p[8], s48p[4];
  __shared__ uint32_t list[kSeaList];
  __shared__ uint32_t cnt[kFsThreads / 64], ub_s;  // survivors per wavefront
  const int job = fs_job_index();
  if (job >= a.n) return;
  const rv_fs_job jb = a.jobs[job];
  const int r_idx = job / a.n_per_ref;
  const rv_plane &ref = a.ref[r_idx];
  SeaCtx c;
  c.nx = jb.x_hi >= jb.x_lo ? jb.x_hi - jb.x_lo + 1 : 0;
  c.ny = jb.y_hi >= jb.y_lo ? jb.y_hi - jb.y_lo + 1 : 0;
  c.tx_n = (c.nx + 3) >> 2;
  // lambdas whose costs could reach the out-of-window marker, or windows
  // wider than the list's 16-bit columns: exhaustive path
  if (jb.lambda >= (1u << 23) || c.nx > 65535) {
    const rv_fs_result res = fs_generic_body<Px>(a.org, ref, jb, 16, 16, 1, a.hp, a.out + job);
    if (threadIdx.x == 0) chain_emit(a.next, job, a.n_per_ref, a.n / a.n_per_ref, res.best_mv);
    return;
  }
  const int tid = threadIdx.x;
  if (tid < 16 * ODW) {
    const uint8_t *o = (const uint8_t *)plane_ptr<Px>(a.org, jb.po_x, jb.po_y);
    orgs[tid] = load_u32_unaligned(o + (int64_t)(tid / ODW) * a.org.stride * B + 4 * (tid % ODW));
  }
  if (tid == 0) {
    ub_s = 0xffffffffu;
    for (int w = 0; w < kFsThreads / 64; w++) cnt[w] = 0;
  }
  __syncthreads();
  if (tid < 16) {  // 4x4 block sums of the source block (row-major blocks)
    uint32_t t = 0;
    for (int r = 0; r < 4; r++)
      for (int i = 0; i < B; i++)
        t = sad_px<Px>(orgs[(4 * (tid >> 2) + r) * ODW + B * (tid & 3) + i], 0u, t);
    so4[tid] = t;
  }
  __syncthreads();
  if (tid < 8) s4p[tid] = so4[2 * tid] | (so4[2 * tid + 1] << 16);
  if (tid < 4)
    s48p[tid] = (so4[4 * tid] + so4[4 * tid + 1]) | ((so4[4 * tid + 2] + so4[4 * tid + 3]) << 16);
  __syncthreads();
  c.s4 = s4p;
  c.s48 = s48p;
  c.stride = ref.stride;
  const int64_t wo = plane_origin_index(ref) + (int64_t)jb.y_lo * ref.stride + jb.x_lo;
  c.box = a.box[r_idx] + wo;
  c.box4 = a.box[r_idx] + (int64_t)ref.stride * ref.alloc_height + wo;
  if (jb.pmv[0].row == jb.pmv[1].row && jb.pmv[0].col == jb.pmv[1].col)
    sea_search<Px, true>(a, jb, job, ref, c, orgs, list, cnt, ub_s);
  else
    sea_search<Px, false>(a, jb, job, ref, c, orgs, list, cnt, ub_s);
}

// u8: capped at 128 VGPRs (4 waves per SIMD) without spilling; u16 keeps
// its registers (the cap would spill).
__global__ __launch_bounds__(kFsThreads) __attribute__((amdgpu_waves_per_eu(4))) void
fs16_sea_kernel_u8(FsArgs a) {
  fs16_sea_body<uint8_t>(a);
}
__global__ __launch_bounds__(kFsThreads) void fs16_sea_kernel_u16(FsArgs a) {
  fs16_sea_body<uint16_t>(a);
}

// Paired box sums (rv_plane_box_sums).  blockIdx.z = 0: 4-tall x 8-wide
// pairs, 1: 4x4 pairs.  A thread computes 4 adjacent positions x 8 rows,
// for x and x + KW, from dword-aligned loads (the pixels under positions
// ax .. ax + 3 + 2 KW - 1 lie in 5 aligned dwords for u8, 10 for u16),
// sliding the vertical KH-row sums over 7 + KH rows of horizontal KW-sums;
// one 16-byte store per row.  Stride is a multiple of 32 bytes (Plane::new).
template <typename Px, int KH, int KW>
__device__ __forceinline__ void box_rows(const rv_plane &p, uint32_t *box, int ax, int ay0) {
  constexpr int B = (int)sizeof(Px);
  constexpr int NDW = 5 * B;
  constexpr int NR = 7 + KH;  // rows of horizontal sums
  const uint32_t *base =
      reinterpret_cast<const uint32_t *>((const uint8_t *)p.data + ((int64_t)ay0 * p.stride + ax) * B);
  const int rdw = p.stride * B / 4;          // dwords per row
  const int ndw = (p.stride - ax) * B / 4;   // dwords left in the row
  uint32_t h[NR][8];  // horizontal KW-sums at ax + j (j < 4) and ax + KW + (j - 4)
#pragma unroll
  for (int k = 0; k < NR; k++) {
    uint32_t w[NDW + 1];
#pragma unroll
    for (int i = 0; i <= NDW; i++)
      w[i] = (ay0 + k < p.alloc_height && i < ndw) ? base[(int64_t)k * rdw + i] : 0u;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const int x = j < 4 ? j : j - 4 + KW;  // pixel offset of the position
      uint32_t t = 0;
#pragma unroll
      for (int g = 0; g < KW; g += 4) {  // 4-pixel groups
        if constexpr (B == 1) {
          const int d = (x + g) >> 2, sh = (x + g) & 3;
          t = __builtin_amdgcn_sad_u8(sh ? __builtin_amdgcn_alignbyte(w[d + 1], w[d], sh) : w[d], 0u, t);
        } else {  // u16: dword (x + g) / 2, half-word (x + g) & 1
          const int d = (x + g) >> 1;
#pragma unroll
          for (int i = 0; i < 2; i++)
            t = __builtin_amdgcn_sad_u16(((x + g) & 1) ? __builtin_amdgcn_alignbyte(w[d + i + 1], w[d + i], 2)
                                                       : w[d + i],
                                         0u, t);
        }
      }
      h[k][j] = t;
    }
  }
  uint32_t acc[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    acc[j] = 0;
#pragma unroll
    for (int k = 0; k < KH; k++) acc[j] += h[k][j];
  }
#pragma unroll
  for (int u = 0; u < 8; u++) {
    const int ay = ay0 + u;
    if (ay < p.alloc_height) {
      // a half whose block leaves the allocation is 0
      const bool vy = ay + KH <= p.alloc_height;
      uint32_t v[4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t lo = vy && ax + j + KW <= p.stride ? acc[j] : 0u;
        const uint32_t hi = vy && ax + j + 2 * KW <= p.stride ? acc[j + 4] : 0u;
        v[j] = lo | (hi << 16);
      }
      *reinterpret_cast<uint4 *>(box + (int64_t)ay * p.stride + ax) = uint4{v[0], v[1], v[2], v[3]};
    }
    if (u < 7)
#pragma unroll
      for (int j = 0; j < 8; j++) acc[j] += h[u + KH][j] - h[u][j];
  }
}

template <typename Px>
__global__ __launch_bounds__(64) void box_sums_kernel(rv_plane p, uint32_t *box) {
  const int ax = ((int)blockIdx.x * 64 + (int)threadIdx.x) * 4;
  const int ay0 = (int)blockIdx.y * 8;
  if (ax >= p.stride || ay0 >= p.alloc_height) return;
  if (blockIdx.z == 0)
    box_rows<Px, 4, 8>(p, box, ax, ay0);
  else
    box_rows<Px, 4, 4>(p, box + (int64_t)p.stride * p.alloc_height, ax, ay0);
}

}  // namespace rv

using namespace rv;

// Multi-reference form used by the replay driver: jobs [n_refs][n_per_ref],
// job i searches refs[i / n_per_ref], all in one launch; `next` (may be
// null) chains each winner into the next stage's jobs.
int rv_full_search_multi(const rv_plane *org, const rv_plane *refs, int n_refs,
                         const rv_fs_job *d_jobs, int n_per_ref, int blk_w, int blk_h,
                         int step, int allow_hp, rv_fs_result *d_out, const ChainNext *next,
                         const uint32_t *const *box, void *stream) {
  if (!org || !refs || n_refs < 1 || n_refs > RV_MAX_REFS || n_per_ref < 0 || blk_w < 4 ||
      blk_h < 4 || blk_w > 128 || blk_h > 128 || (blk_w & 3) || step < 1)
    return rv_set_error(RV_EINVAL, "rv_full_search_batch: bad arguments");
  for (int k = 0; k < n_refs; k++)
    if (refs[k].hbd != org->hbd)
      return rv_set_error(RV_EINVAL, "rv_full_search_batch: pixel type mismatch");
  const int n = n_refs * n_per_ref;
  if (n == 0) return RV_OK;
  hipStream_t s = rv_resolve_stream(stream);
  FsArgs a;
  memset(&a, 0, sizeof(a));
  a.org = *org;
  for (int k = 0; k < n_refs; k++) a.ref[k] = refs[k];
  a.jobs = d_jobs;
  a.out = d_out;
  a.n = n;
  a.n_per_ref = n_per_ref;
  a.hp = allow_hp ? 1 : 0;
  a.bw = blk_w;
  a.bh = blk_h;
  a.step = step;
  if (next) a.next = *next;
  const bool sea = box && blk_w == 16 && blk_h == 16 && step == 1;
  if (sea)
    for (int k = 0; k < n_refs; k++) {
      if (!box[k] || ((uintptr_t)box[k] & 15))
        return rv_set_error(RV_EINVAL, "rv_full_search_sea_batch: box-sum table null or unaligned");
      if (refs[k].stride % 4)
        return rv_set_error(RV_EINVAL, "rv_full_search_sea_batch: ref stride not Plane::new's");
      a.box[k] = box[k];
    }
  const unsigned grid = (unsigned)((n + 7) / 8 * 8);
  if (sea && org->hbd)
    fs16_sea_kernel_u16<<<grid, kFsThreads, 0, s>>>(a);
  else if (sea)
    fs16_sea_kernel_u8<<<grid, kFsThreads, 0, s>>>(a);
  else if (blk_w == 16 && blk_h == 16 && step == 1 && org->hbd)
    fs16_kernel<uint16_t><<<grid, kFsThreads, 0, s>>>(a);
  else if (blk_w == 16 && blk_h == 16 && step == 1)
    fs16_kernel<uint8_t><<<grid, kFsThreads, 0, s>>>(a);
  else if (org->hbd)
    fs_generic_kernel<uint16_t><<<grid, kFsThreads, 0, s>>>(a);
  else
    fs_generic_kernel<uint8_t><<<grid, kFsThreads, 0, s>>>(a);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

extern "C" int rv_full_search_batch(const rv_plane *org, const rv_plane *ref,
                                    const rv_fs_job *d_jobs, int n, int blk_w,
                                    int blk_h, int step, int allow_hp,
                                    rv_fs_result *d_out, void *stream) {
  if (!ref) return rv_set_error(RV_EINVAL, "rv_full_search_batch: null ref");
  return rv_full_search_multi(org, ref, 1, d_jobs, n, blk_w, blk_h, step, allow_hp, d_out,
                              nullptr, nullptr, stream);
}

extern "C" int rv_full_search_sea_batch(const rv_plane *org, const rv_plane *ref,
                                        const uint32_t *d_ref_box, const rv_fs_job *d_jobs, int n,
                                        int allow_hp, rv_fs_result *d_out, void *stream) {
  if (!ref || !d_ref_box || !org)
    return rv_set_error(RV_EINVAL, "rv_full_search_sea_batch: null ref or box-sum table");
  // the packed 16-bit box sums (and the source's 4x8 sums) hold only for
  // pixels <= 10 bits: a u16 plane must say so
  if ((org->hbd && (org->bit_depth < 9 || org->bit_depth > 10)) ||
      (ref->hbd && (ref->bit_depth < 9 || ref->bit_depth > 10)))
    return rv_set_error(RV_EINVAL,
                        "rv_full_search_sea_batch: u16 planes must state bit_depth 9 or 10 "
                        "(12-bit sums overflow the packed tables: use rv_full_search_batch)");
  return rv_full_search_multi(org, ref, 1, d_jobs, n, 16, 16, 1, allow_hp, d_out, nullptr,
                              &d_ref_box, stream);
}

extern "C" int rv_plane_box_sums(const rv_plane *p, uint32_t *d_box, void *stream) {
  if (!p || !p->data || !d_box || p->stride < 1 || p->alloc_height < 1)
    return rv_set_error(RV_EINVAL, "rv_plane_box_sums: bad arguments");
  if (p->hbd && (p->bit_depth < 9 || p->bit_depth > 10))
    return rv_set_error(RV_EINVAL,
                        "rv_plane_box_sums: a u16 plane must state bit_depth 9 or 10 (4x8 "
                        "sums of 12-bit pixels overflow 16 bits)");
  hipStream_t s = rv_resolve_stream(stream);
  if (p->stride % (p->hbd ? 16 : 32) || ((uintptr_t)p->data & 15) || ((uintptr_t)d_box & 15))
    return rv_set_error(RV_EINVAL, "rv_plane_box_sums: plane stride / alignment not Plane::new's");
  const dim3 grid((unsigned)((p->stride / 4 + 63) / 64), (unsigned)((p->alloc_height + 7) / 8), 2);
  if (p->hbd)
    box_sums_kernel<uint16_t><<<grid, 64, 0, s>>>(*p, d_box);
  else
    box_sums_kernel<uint8_t><<<grid, 64, 0, s>>>(*p, d_box);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}
