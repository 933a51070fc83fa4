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
  rv_plane ref[RV_DS_MAX_PRED];  // job i searches ref[i / n_per_ref]
  const rv_fs_job *jobs;
  rv_fs_result *out;
  int n, n_per_ref, hp, bw, bh, step;
  ChainNext next;  // replay: feed the winner into the next stage's jobs
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

// ---- exact successive-elimination path: u8, 16x16, step 1 ----------------
// The triangle inequality bounds every candidate from below:
//   SAD(org, cand) >= sum over the four 8x8 quadrants q of |S_org,q - S_cand,q|
// (S = pixel sum), so cost >= LB = 256 * that + rate * lambda.  A candidate
// whose LB exceeds an achieved cost UB cannot be the strict first minimum,
// so skipping it leaves the result of full_search (src/me.rs:943-990)
// unchanged bit for bit.  Per band: (A) the 8x8 box sums S8 of every
// candidate position go to LDS (horizontal 8-sums by v_sad_u8 against zero,
// vertical by a sliding register ring); (B) every lane takes the
// minimum-LB candidate of its tiles and evaluates it exactly -> UB (carried
// across bands); (C) the candidates with LB <= UB are compacted and
// evaluated exactly, spread over all lanes.
constexpr int kSeaLdsBytes = 48 * 1024;
constexpr int kSeaMaxTiles = 512;

__device__ __forceinline__ uint32_t sum8_u8(const uint32_t *row, int x) {
  const int d = x >> 2, sh = x & 3;
  const uint32_t w0 = row[d], w1 = row[d + 1], w2 = row[d + 2];
  return __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(w1, w0, sh), 0u,
                                 __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(w2, w1, sh), 0u, 0u));
}

__global__ __launch_bounds__(kFsThreads) void fs16_sea_kernel(FsArgs a) {
  extern __shared__ __align__(16) uint32_t sea_lds[];
  __shared__ uint4 orgs[16];
  __shared__ uint32_t so[4];
  __shared__ uint32_t tmin[kSeaMaxTiles];
  __shared__ uint32_t lmask[kSeaMaxTiles], ltile[kSeaMaxTiles], lpre[kSeaMaxTiles + 1];
  __shared__ uint32_t cnt, ub_s;
  const int job = fs_job_index();
  if (job >= a.n) return;
  const rv_fs_job jb = a.jobs[job];
  const rv_plane &ref = a.ref[job / a.n_per_ref];
  const int nx = jb.x_hi >= jb.x_lo ? jb.x_hi - jb.x_lo + 1 : 0;
  const int ny = jb.y_hi >= jb.y_lo ? jb.y_hi - jb.y_lo + 1 : 0;
  const int tid = threadIdx.x;
  if (tid < 64) {
    const uint8_t *o = plane_ptr<uint8_t>(a.org, jb.po_x, jb.po_y);
    reinterpret_cast<uint32_t *>(orgs)[tid] =
        load_u32_unaligned(o + (int64_t)(tid >> 2) * a.org.stride + 4 * (tid & 3));
  }
  if (tid == 0) ub_s = 0xffffffffu;
  __syncthreads();
  if (tid < 4) {  // quadrant sums of the source block
    const uint32_t *ow = reinterpret_cast<const uint32_t *>(orgs);
    uint32_t t = 0;
    for (int r = 0; r < 8; r++)
      for (int i = 0; i < 2; i++)
        t = __builtin_amdgcn_sad_u8(ow[(8 * (tid >> 1) + r) * 4 + 2 * (tid & 1) + i], 0u, t);
    so[tid] = t;
  }
  const int tx_n = (nx + 3) >> 2;
  const int rw = tx_n + 4;             // band row length in dwords (pixels)
  const int sw = 4 * tx_n + 8;         // S8 row length in u16 (candidate cols + 8)
  const int vis_w = nx + 15;
  // band rows: pixels (pb + 15) * rw * 4 + S8 (pb + 8) * sw * 2 <= budget
  int pb = (kSeaLdsBytes - 4 - 15 * rw * 4 - 8 * sw * 2) / (rw * 4 + sw * 2);
  pb = (pb / kTileRows) * kTileRows;
  pb = pb > kSeaMaxTiles / tx_n * kTileRows ? kSeaMaxTiles / tx_n * kTileRows : pb;
  // window too wide for the SEA band, or costs that may not fit u32
  // (256 * sad < 2^24 needs lambda < 2^25): exhaustive path
  if (pb < kTileRows || jb.lambda >= (1u << 25)) {
    const rv_fs_result res = fs_generic_body<uint8_t>(a.org, ref, jb, 16, 16, 1, a.hp, a.out + job);
    if (tid == 0) chain_emit(a.next, job, a.n_per_ref, a.n / a.n_per_ref, res.best_mv);
    return;
  }
  uint32_t *band = sea_lds;
  // S8 rows are read as 8-byte uint2: start the table on an 8-byte boundary
  uint16_t *s8 = reinterpret_cast<uint16_t *>(sea_lds + (((pb + 15) * rw + 1) & ~1));
  uint64_t bkey = ~0ull;  // (u32 cost << 32 | raster index)
  const uint8_t *rbase = plane_ptr<uint8_t>(ref, jb.x_lo, jb.y_lo);
  auto rate_of = [&](int iy, int ix) -> uint32_t {
    const int16_t row = (int16_t)(8 * (jb.y_lo + iy - jb.po_y));
    const int16_t col = (int16_t)(8 * (jb.x_lo + ix - jb.po_x));
    const uint32_t r1 = diff_to_rate((int16_t)(row - jb.pmv[0].row), a.hp) +
                        diff_to_rate((int16_t)(col - jb.pmv[0].col), a.hp);
    const uint32_t r2 = diff_to_rate((int16_t)(row - jb.pmv[1].row), a.hp) +
                        diff_to_rate((int16_t)(col - jb.pmv[1].col), a.hp);
    return r1 < r2 + 1 ? r1 : r2 + 1;
  };
  // exact cost key of the candidate at band row y, column x (raster iy, ix)
  auto exact_key = [&](int y, int x, int iy, int ix) -> uint64_t {
    uint32_t sad = 0;
    const int d = x >> 2, sh = x & 3;
#pragma unroll 4
    for (int r = 0; r < 16; r++) {
      const uint32_t *row = band + (y + r) * rw + d;
      uint32_t w[5];
#pragma unroll
      for (int i = 0; i < 5; i++) w[i] = row[i];
      const uint4 o4 = orgs[r];
      sad = __builtin_amdgcn_sad_u8(o4.x, __builtin_amdgcn_alignbyte(w[1], w[0], sh), sad);
      sad = __builtin_amdgcn_sad_u8(o4.y, __builtin_amdgcn_alignbyte(w[2], w[1], sh), sad);
      sad = __builtin_amdgcn_sad_u8(o4.z, __builtin_amdgcn_alignbyte(w[3], w[2], sh), sad);
      sad = __builtin_amdgcn_sad_u8(o4.w, __builtin_amdgcn_alignbyte(w[4], w[3], sh), sad);
    }
    const uint32_t cost = (sad << 8) + rate_of(iy, ix) * jb.lambda;
    return ((uint64_t)cost << 32) | (uint32_t)(iy * nx + ix);
  };

  for (int y0 = 0; y0 < ny; y0 += pb) {
    const int rows = ny - y0 < pb ? ny - y0 : pb;
    const int lrows = rows + 15;
    const int ty_n = (rows + kTileRows - 1) / kTileRows;
    const int brows = ty_n * kTileRows + 15;
    const int total = brows * rw;
    __syncthreads();
    for (int i0 = tid; i0 < total; i0 += 8 * kFsThreads) {  // band fill
      uint32_t v[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int i = i0 + u * kFsThreads;
        const int r = i / rw, c = 4 * (i - r * rw);
        uint32_t x = 0;
        if (i < total && r < lrows) {
          const uint8_t *p = rbase + (int64_t)(y0 + r) * ref.stride + c;
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
    if (tid == 0) cnt = 0;
    __syncthreads();
    // (A) S8[y][x] = sum of the 8x8 block at band (y, x), y < ty_n*8 + 8
    const int s8rows = ty_n * kTileRows + 8;
    for (int x = tid; x < sw; x += kFsThreads) {
      uint32_t ring[8];
#pragma unroll
      for (int k = 0; k < 8; k++) ring[k] = sum8_u8(band + k * rw, x);
      uint32_t acc = ring[0] + ring[1] + ring[2] + ring[3] + ring[4] + ring[5] + ring[6] + ring[7];
#pragma unroll 1
      for (int y = 0; y < s8rows; y += 8) {
#pragma unroll
        for (int u = 0; u < 8; u++) {
          s8[(y + u) * sw + x] = (uint16_t)acc;
          const uint32_t nxt = y + u + 8 < brows ? sum8_u8(band + (y + u + 8) * rw, x) : 0u;
          acc += nxt - ring[u];
          ring[u] = nxt;
        }
      }
    }
    __syncthreads();
    // (B) tile lower bounds; each lane's minimum-LB candidate
    const uint32_t so0 = so[0], so1 = so[1], so2 = so[2], so3 = so[3];
    const int tasks = tx_n * ty_n;
    uint64_t lbest = ~0ull;  // (LB << 32 | band-local candidate index)
    auto lb_tile = [&](int t, uint32_t thr, uint32_t *mask) -> uint32_t {
      const int tcy = t / tx_n, tcx = t - tcy * tx_n;
      // separable rate terms (get_mv_rate): 24 diff_to_rate per 32 candidates
      uint32_t rr0[kTileRows], rr1[kTileRows], rc0[4], rc1[4];
#pragma unroll
      for (int c = 0; c < kTileRows; c++) {
        const int16_t row = (int16_t)(8 * (jb.y_lo + y0 + tcy * kTileRows + c - jb.po_y));
        rr0[c] = diff_to_rate((int16_t)(row - jb.pmv[0].row), a.hp);
        rr1[c] = diff_to_rate((int16_t)(row - jb.pmv[1].row), a.hp);
      }
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int16_t col = (int16_t)(8 * (jb.x_lo + 4 * tcx + j - jb.po_x));
        rc0[j] = diff_to_rate((int16_t)(col - jb.pmv[0].col), a.hp);
        rc1[j] = diff_to_rate((int16_t)(col - jb.pmv[1].col), a.hp);
      }
      uint32_t tm = 0xffffffffu, m = 0;
#pragma unroll
      for (int c = 0; c < kTileRows; c++) {
        const int y = tcy * kTileRows + c;
        const uint2 t0 = *reinterpret_cast<const uint2 *>(s8 + y * sw + 4 * tcx);
        const uint2 t1 = *reinterpret_cast<const uint2 *>(s8 + y * sw + 4 * tcx + 8);
        const uint2 b0 = *reinterpret_cast<const uint2 *>(s8 + (y + 8) * sw + 4 * tcx);
        const uint2 b1 = *reinterpret_cast<const uint2 *>(s8 + (y + 8) * sw + 4 * tcx + 8);
        const uint32_t tl[4] = {t0.x & 0xffff, t0.x >> 16, t0.y & 0xffff, t0.y >> 16};
        const uint32_t tr[4] = {t1.x & 0xffff, t1.x >> 16, t1.y & 0xffff, t1.y >> 16};
        const uint32_t bl[4] = {b0.x & 0xffff, b0.x >> 16, b0.y & 0xffff, b0.y >> 16};
        const uint32_t br[4] = {b1.x & 0xffff, b1.x >> 16, b1.y & 0xffff, b1.y >> 16};
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const int ix = 4 * tcx + j;
          if (ix >= nx || y >= rows) continue;
          uint32_t l = so0 > tl[j] ? so0 - tl[j] : tl[j] - so0;
          l += so1 > tr[j] ? so1 - tr[j] : tr[j] - so1;
          l += so2 > bl[j] ? so2 - bl[j] : bl[j] - so2;
          l += so3 > br[j] ? so3 - br[j] : br[j] - so3;
          const uint32_t r1 = rr0[c] + rc0[j], r2 = rr1[c] + rc1[j];
          const uint32_t lb = (l << 8) + (r1 < r2 + 1 ? r1 : r2 + 1) * jb.lambda;
          tm = lb < tm ? lb : tm;
          if (mask) {
            if (lb <= thr) m |= 1u << (c * 4 + j);
          } else {
            const uint64_t k = ((uint64_t)lb << 32) | (uint32_t)(y * nx + ix);
            lbest = k < lbest ? k : lbest;
          }
        }
      }
      if (mask) *mask = m;
      return tm;
    };
    for (int t = tid; t < tasks; t += kFsThreads) tmin[t] = lb_tile(t, 0, nullptr);
    if (lbest != ~0ull) {  // evaluate the lane's most promising candidate
      const uint32_t li = (uint32_t)lbest;
      const int y = (int)(li / nx), x = (int)(li - (uint32_t)y * nx);
      const uint64_t k = exact_key(y, x, y0 + y, x);
      bkey = k < bkey ? k : bkey;
      atomicMin(&ub_s, (uint32_t)(k >> 32));
    }
    __syncthreads();
    const uint32_t ub = ub_s;
    // (C) compact the surviving candidates (LB <= UB) and evaluate them
    for (int t = tid; t < tasks; t += kFsThreads) {
      if (tmin[t] > ub) continue;
      uint32_t m;
      lb_tile(t, ub, &m);
      if (m) {
        const uint32_t slot = atomicAdd(&cnt, 1u);
        ltile[slot] = (uint32_t)t;
        lmask[slot] = m;
      }
    }
    __syncthreads();
    const int ns = (int)cnt;
    {  // exclusive prefix of the survivors' popcounts: 2 entries per thread,
       // wave scans by shuffles, wave totals through LDS
      __shared__ uint32_t wsum[kFsThreads / 64];
      const int e0 = 2 * tid;
      const uint32_t p0 = e0 < ns ? __builtin_popcount(lmask[e0]) : 0u;
      const uint32_t p1 = e0 + 1 < ns ? __builtin_popcount(lmask[e0 + 1]) : 0u;
      uint32_t v = p0 + p1, inc = v;
      const int lane = tid & 63;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(inc, o, 64);
        if (lane >= o) inc += u;
      }
      if (lane == 63) wsum[tid >> 6] = inc;
      __syncthreads();
      uint32_t base = 0;
      for (int w = 0; w < (tid >> 6); w++) base += wsum[w];
      const uint32_t ex = base + inc - v;
      if (e0 < ns) lpre[e0] = ex;
      if (e0 + 1 < ns) lpre[e0 + 1] = ex + p0;
      if (tid == kFsThreads - 1) lpre[ns] = base + inc;
      if (ns == 0 && tid == 0) lpre[0] = 0;
    }
    __syncthreads();
    const int nsurv = (int)lpre[ns];
    for (int k = tid; k < nsurv; k += kFsThreads) {
      int lo = 0, hi = ns - 1;  // entry e with lpre[e] <= k < lpre[e + 1]
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (lpre[mid] <= (uint32_t)k) lo = mid;
        else hi = mid - 1;
      }
      uint32_t m = lmask[lo];
      for (uint32_t r = (uint32_t)k - lpre[lo]; r; r--) m &= m - 1;  // r-th set bit
      const int bit = __builtin_ctz(m);
      const int t = (int)ltile[lo], tcy = t / tx_n, tcx = t - tcy * tx_n;
      const int y = tcy * kTileRows + (bit >> 2), x = 4 * tcx + (bit & 3);
      const uint64_t key = exact_key(y, x, y0 + y, x);
      bkey = key < bkey ? key : bkey;
    }
    if (tid < 64) atomicMin(&ub_s, (uint32_t)(group_min_u64(bkey) >> 32));
  }
  Best b{~0ull, 0xffffffffu};
  if (bkey != ~0ull) b = Best{bkey >> 32, (uint32_t)bkey};
  b = block_best(b);
  if (tid == 0) {
    const rv_fs_result res = write_result(jb, b, nx > 0 ? nx : 1, 1, a.out + job);
    chain_emit(a.next, job, a.n_per_ref, a.n / a.n_per_ref, res.best_mv);
  }
}

}  // namespace rv

using namespace rv;

// RAV1E_HIP_FS_SEA=1 selects the successive-elimination u8 path (read per
// launch).  Off by default: measured 2.2x slower than the exhaustive tile
// kernel on the 1080p replay -- the first band's upper bound is loose
// (the window centre, where the best usually is, sits in a middle band)
// and the phase barriers at 2 workgroups per CU cost more than the pruned
// SADs save.  Kept, exact and tested, as the base for a centre-first probe.
static bool sea_enabled() {
  const char *e = getenv("RAV1E_HIP_FS_SEA");
  return e && e[0] == '1';
}

// Multi-reference form used by the replay driver: jobs [n_refs][n_per_ref],
// job i searches refs[i / n_per_ref], all in one launch; `next` (may be
// null) chains each winner into the next stage's jobs.
int rv_full_search_multi(const rv_plane *org, const rv_plane *refs, int n_refs,
                         const rv_fs_job *d_jobs, int n_per_ref, int blk_w, int blk_h,
                         int step, int allow_hp, rv_fs_result *d_out, const ChainNext *next,
                         void *stream) {
  if (!org || !refs || n_refs < 1 || n_refs > RV_DS_MAX_PRED || n_per_ref < 0 || blk_w < 4 ||
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
  const unsigned grid = (unsigned)((n + 7) / 8 * 8);
  if (blk_w == 16 && blk_h == 16 && step == 1 && !org->hbd && sea_enabled())
    fs16_sea_kernel<<<grid, kFsThreads, kSeaLdsBytes, s>>>(a);
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
                              nullptr, stream);
}
