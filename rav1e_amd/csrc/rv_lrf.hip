// rv_lrf.hip -- loop restoration with the self-guided filter (src/lrf.rs) on
// gfx950: rav1e's per-unit decision (rdo_loop_decision's restoration pass,
// src/rdo.rs:1726-2120) and lrf_filter_frame (src/lrf.rs:1345-1444).
//
// Three launches per frame, after the frame's reconstruction:
//  * lrf_rdo_kernel, one workgroup per (superblock, plane) unit -- every
//    unit is one superblock at the replay's quantizers (RestorationState::
//    new, base_q_idx <= 160): the unit's input as rav1e builds it while the
//    tile is coded (the reconstruction so far, 128 where a superblock is not
//    coded yet, CDEF_VERY_LARGE outside the tile, CDEF index 0 on top), its
//    integral images in LDS, then None and each of the 16 parameter sets:
//    the box (a, b) tables in LDS, sgrproj_solve's sums (exact i64 block
//    reductions, the f64 tail on one lane), the filtered unit and its
//    rdo_loop_plane_error -- 17 distortions and 16 xqd pairs to HBM;
//  * lrf_decide_kernel, one lane per tile: the tile's units in coding order,
//    each option priced with count_lrf_switchable at the tile's current
//    restoration CDF and sgrproj_ref, the first cheapest kept, write_lrf's
//    updates after each superblock -- the sequential part, a few hundred
//    integer steps per tile;
//  * lrf_filter_kernel, one workgroup per (stripe, 32-column chunk, plane):
//    setup_integral_image's view of the CDEF output (the deblocked frame
//    above and below the stripe), the unit's set, the restored pixels.
// All of it is integer work but sgrproj_solve's tail, whose f64 operations
// run in the reference's order (IEEE division, no contraction).
#include <string.h>

#include "rv_device.h"
#include "rv_lrf.h"

namespace rv {
namespace {

constexpr int kVeryLarge = 0x8000;
constexpr int kRstBits = 4, kPrjBits = 7, kSgrBits = 8, kMtableBits = 20, kRecipBits = 12;

// SGRPROJ_PARAMS_S (src/lrf.rs:61-78)
__constant__ uint32_t kSgrS[16][2] = {{140, 3236}, {112, 2158}, {93, 1618}, {80, 1438},
                                      {70, 1295},  {58, 1177},  {47, 1079}, {37, 996},
                                      {30, 925},   {25, 863},   {0, 2589},  {0, 1618},
                                      {0, 1177},   {0, 925},    {56, 0},    {22, 0}};
// cdef_directions (src/cdef.rs:164-173): [dir][k] = (dy, dx)
__constant__ int8_t kLrfCdefDirs[8][2][2] = {
    {{-1, 1}, {-2, 2}}, {{0, 1}, {-1, 2}}, {{0, 1}, {0, 2}}, {{0, 1}, {1, 2}},
    {{1, 1}, {2, 2}},   {{1, 0}, {2, 1}},  {{1, 0}, {2, 0}}, {{1, 0}, {2, -1}}};

__device__ __forceinline__ int msb32(int32_t x) { return 31 ^ __clz(x); }
__device__ __forceinline__ int iclamp(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }

// ---- CDEF of one pixel of the unit's padded input (cdef_filter_block,
// src/cdef.rs:134-228) --------------------------------------------------------
__device__ __forceinline__ int cdef_constrain(int diff, int threshold, int damping) {
  if (!threshold) return 0;
  const int shift = max(0, damping - msb32(threshold));
  const int ad = diff < 0 ? -diff : diff;
  const int mag = min(ad, max(0, threshold - (ad >> shift)));
  return diff < 0 ? -mag : mag;
}
__device__ __forceinline__ int cdef_adjust(int strength, int32_t var) {  // :232-239
  const int i = (var >> 6) ? min(msb32(var >> 6), 12) : 0;
  return var ? (strength * (4 + i) + 8) >> 4 : 0;
}
// in: the padded u16 input at the pixel, pitch s
__device__ inline int cdef_px(const uint16_t *in, int s, int pri, int sec, int dir, int damping,
                              int cs) {
  const int x = in[0];
  const int odd = (pri >> cs) & 1;
  int sum = 0, mx = x, mn = x;
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const int pt = odd ? 3 : (k ? 2 : 4), st = k ? 1 : 2;
    const int d0 = kLrfCdefDirs[dir][k][0] * s + kLrfCdefDirs[dir][k][1];
    const int d1 = kLrfCdefDirs[(dir + 2) & 7][k][0] * s + kLrfCdefDirs[(dir + 2) & 7][k][1];
    const int d2 = kLrfCdefDirs[(dir + 6) & 7][k][0] * s + kLrfCdefDirs[(dir + 6) & 7][k][1];
    const int p0 = in[d0], p1 = in[-d0];
    sum += pt * (cdef_constrain(p0 - x, pri, damping) + cdef_constrain(p1 - x, pri, damping));
    if (p0 != kVeryLarge) mx = max(p0, mx);
    if (p1 != kVeryLarge) mx = max(p1, mx);
    mn = min(min(p0, p1), mn);
    const int sv[4] = {in[d1], in[-d1], in[d2], in[-d2]};
#pragma unroll
    for (int e = 0; e < 4; e++) {
      if (sv[e] != kVeryLarge) mx = max(sv[e], mx);
      mn = min(sv[e], mn);
      sum += st * cdef_constrain(sv[e] - x, sec, damping);
    }
  }
  return iclamp(x + ((8 + sum - (sum < 0)) >> 4), mn, mx);
}
// cdef_find_dir (src/cdef.rs:68-126) of the 8x8 luma block at p (pitch s);
// u32 wrapping like the reference's release build
template <typename Px>
__device__ inline int cdef_dir(const Px *p, int64_t s, int cs, int32_t *var) {
  int32_t partial[8][15];
#pragma unroll
  for (int d = 0; d < 8; d++)
#pragma unroll
    for (int k = 0; k < 15; k++) partial[d][k] = 0;
#pragma unroll
  for (int r = 0; r < 8; r++)
#pragma unroll
    for (int c = 0; c < 8; c++) {
      const int32_t x = ((int)p[r * s + c] >> cs) - 128;
      partial[0][r + c] += x;
      partial[1][r + c / 2] += x;
      partial[2][r] += x;
      partial[3][3 + r - c / 2] += x;
      partial[4][7 + r - c] += x;
      partial[5][3 - r / 2 + c] += x;
      partial[6][c] += x;
      partial[7][r / 2 + c] += x;
    }
  constexpr uint32_t div[9] = {0, 840, 420, 280, 210, 168, 140, 120, 105};
  uint32_t cost[8];
#define SQ(v) ((uint32_t)(v) * (uint32_t)(v))
  cost[2] = cost[6] = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    cost[2] += SQ(partial[2][k]);
    cost[6] += SQ(partial[6][k]);
  }
  cost[2] *= div[8];
  cost[6] *= div[8];
  cost[0] = SQ(partial[0][7]) * div[8];
  cost[4] = SQ(partial[4][7]) * div[8];
#pragma unroll
  for (int k = 0; k < 7; k++) {
    cost[0] += (SQ(partial[0][k]) + SQ(partial[0][14 - k])) * div[k + 1];
    cost[4] += (SQ(partial[4][k]) + SQ(partial[4][14 - k])) * div[k + 1];
  }
#pragma unroll
  for (int d = 1; d < 8; d += 2) {
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < 5; k++) c += SQ(partial[d][3 + k]);
    c *= div[8];
#pragma unroll
    for (int k = 0; k < 3; k++) c += (SQ(partial[d][k]) + SQ(partial[d][10 - k])) * div[2 * k + 2];
    cost[d] = c;
  }
#undef SQ
  int best = 0;
  int32_t best_cost = (int32_t)cost[0];
#pragma unroll
  for (int d = 1; d < 8; d++)
    if ((int32_t)cost[d] > best_cost) {
      best = d;
      best_cost = (int32_t)cost[d];
    }
  uint32_t orth = cost[0];
#pragma unroll
  for (int d = 1; d < 8; d++)
    if (d == ((best + 4) & 7)) orth = cost[d];
  *var = (int32_t)((uint32_t)best_cost - orth) >> 10;
  return best;
}

// ---- distortion (src/rdo.rs) -------------------------------------------------
// compute_distortion_bias of an 8x8 at 4x4 block (mi_x, mi_y) (src/rdo.rs:
// 476-508): f32 mean of its importance cells / 3 + 0.65
__device__ inline double lrf_bias(const float *imp, int w_imp, int w_in_b, int h_in_b, int mi_x,
                                  int mi_y) {
  if (!imp) return 0.65;
  const int x2 = min(mi_x + 2, w_in_b), y2 = min(mi_y + 2, h_in_b);
  float tot = 0.f;
  for (int y = mi_y; y < y2; y++)
    for (int x = mi_x; x < x2; x++) tot = __fadd_rn(tot, imp[(y >> 1) * w_imp + (x >> 1)]);
  return (double)__fdiv_rn(__fdiv_rn(tot, 4.0f), 3.0f) + 0.65;
}
__device__ __forceinline__ uint64_t biased(uint64_t v, double b) { return (uint64_t)((double)v * b); }
// cdef_dist_wxh_8x8's f64 tail (src/rdo.rs:219-261) from the moments
__device__ inline uint64_t cdef_dist(int32_t ss, int32_t sd, uint32_t ss2, uint32_t sd2, uint32_t ssd,
                                     int bd) {
  const int cs = bd - 8;
  const int64_t s2 = (int64_t)ss2, d2 = (int64_t)sd2, sdv = (int64_t)ssd;
  const double svar = (double)(s2 - (((int64_t)ss * ss + 32) >> 6));
  const double dvar = (double)(d2 - (((int64_t)sd * sd + 32) >> 6));
  const double sse = (double)(d2 + s2 - 2 * sdv);
  const double boost = (4033.0 / 16384.0) * (svar + dvar + (double)(16384ll << (2 * cs))) /
                       sqrt((double)(16265089ull << (4 * cs)) + svar * dvar);
  const double v = sse * boost + 0.5;
  return v > 0.0 ? (uint64_t)v : 0;
}

// ---- the self-guided filter (src/lrf.rs:156-334) ------------------------------
// sgrproj_sum_finish (:305-323), u32 wrapping
__device__ __forceinline__ void sum_finish(uint32_t ssq, uint32_t sum, uint32_t n, uint32_t one_over_n,
                                           uint32_t s, int bdm8, uint32_t &a, uint32_t &b) {
  const uint32_t sssq = (ssq + ((1u << (2 * bdm8)) >> 1)) >> (2 * bdm8);
  const uint32_t ssum = (sum + ((1u << bdm8) >> 1)) >> bdm8;
  const int32_t pd = (int32_t)(sssq * n - ssum * ssum);  // (i32) - (i32), wrapping
  const uint32_t p = (uint32_t)(pd > 0 ? pd : 0);
  const uint32_t z = (p * s + ((1u << kMtableBits) >> 1)) >> kMtableBits;
  a = z >= 255 ? 256 : z == 0 ? 1 : ((z << kSgrBits) + z / 2) / (z + 1);
  const uint32_t bb = ((1u << kSgrBits) - a) * sum * one_over_n;
  b = (bb + ((1u << kRecipBits) >> 1)) >> kRecipBits;
}
// get_integral_square (:326-334): rows (y, y + d], columns (x, x + d]
__device__ __forceinline__ uint32_t isq(const uint32_t *ii, int s, int x, int y, int d) {
  return ii[y * s + x] + ii[(y + d) * s + x + d] - ii[(y + d) * s + x] - ii[y * s + x + d];
}

// The LDS tables of one region (w x h pixels, w <= W): the integral images
// ((h + 7) x (w + 7)), the r = 1 (a, b) rows 0 .. h + 1 and the r = 2 rows
// 0, 2, .. h (+1), each w + 2 wide.
template <int W, int HMAX>
struct SgrLds {
  static constexpr int IS = W + 7, IR = HMAX + 8;  // image pitch / rows
  static constexpr int AS = W + 2, A1R = HMAX + 2, A2R = HMAX / 2 + 2;
  uint32_t ii[IR * IS], sq[IR * IS];
  uint32_t a1[A1R * AS], b1[A1R * AS];
  uint32_t a2[A2R * AS], b2[A2R * AS];
};

// the (a, b) tables of set s over the region's image (every lane)
template <int W, int HMAX>
__device__ inline void sgr_tables(SgrLds<W, HMAX> &L, int set, int w, int h, int bdm8) {
  using S = SgrLds<W, HMAX>;
  const uint32_t s2 = kSgrS[set][0], s1 = kSgrS[set][1];
  const int n1 = s1 ? (h + 2) * (w + 2) : 0;
  const int r2rows = s2 ? (h + 1) / 2 + 1 + ((h + 1) & 1 ? 0 : 0) : 0;  // rows 0, 2, .., <= h + 1
  const int n2 = r2rows * (w + 2);
  for (int i = threadIdx.x; i < n1 + n2; i += blockDim.x) {
    if (i < n1) {  // box_ab r1: the image from (1, 1) (:626-650, 877-889)
      const int y = i / (w + 2), x = i - y * (w + 2);
      uint32_t a, b;
      sum_finish(isq(L.sq + S::IS + 1, S::IS, x, y, 3), isq(L.ii + S::IS + 1, S::IS, x, y, 3), 9, 455,
                 s1, bdm8, a, b);
      L.a1[y * S::AS + x] = a;
      L.b1[y * S::AS + x] = b;
    } else {  // box_ab r2 at even rows (:611-624, 843-856)
      const int j = i - n1, yr = j / (w + 2), x = j - yr * (w + 2);
      uint32_t a, b;
      sum_finish(isq(L.sq, S::IS, x, 2 * yr, 5), isq(L.ii, S::IS, x, 2 * yr, 5), 25, 164, s2, bdm8, a, b);
      L.a2[yr * S::AS + x] = a;
      L.b2[yr * S::AS + x] = b;
    }
  }
}

// f_r2 and f_r1 of pixel (x, y) with value px (src/lrf.rs:244-301 via the
// row loop :656-733); px0: the pixel of row y & ~1 (box_f_r0 shares it)
template <int W, int HMAX>
__device__ __forceinline__ void sgr_f(const SgrLds<W, HMAX> &L, int set, int x, int y, uint32_t px,
                                      uint32_t px0, uint32_t &f2, uint32_t &f1) {
  using S = SgrLds<W, HMAX>;
  const uint32_t s2 = kSgrS[set][0], s1 = kSgrS[set][1];
  constexpr int sh = 5 + kSgrBits - kRstBits, sho = 4 + kSgrBits - kRstBits;
  if (s2) {
    const int yr = y >> 1;
    const uint32_t *an = L.a2 + (yr + 1) * S::AS, *bn = L.b2 + (yr + 1) * S::AS;
    const uint32_t ao = 5 * (an[x] + an[x + 2]) + 6 * an[x + 1];
    const uint32_t bo = 5 * (bn[x] + bn[x + 2]) + 6 * bn[x + 1];
    if (!(y & 1)) {
      const uint32_t *ap = L.a2 + yr * S::AS, *bp = L.b2 + yr * S::AS;
      const uint32_t a = 5 * (ap[x] + ap[x + 2]) + 6 * ap[x + 1];
      const uint32_t b = 5 * (bp[x] + bp[x + 2]) + 6 * bp[x + 1];
      f2 = ((a + ao) * px + b + bo + ((1u << sh) >> 1)) >> sh;
    } else {
      f2 = (ao * px + bo + ((1u << sho) >> 1)) >> sho;
    }
  } else {
    f2 = px0 << kRstBits;
  }
  if (s1) {
    const uint32_t *A0 = L.a1 + y * S::AS, *A1 = A0 + S::AS, *A2 = A1 + S::AS;
    const uint32_t *B0 = L.b1 + y * S::AS, *B1 = B0 + S::AS, *B2 = B1 + S::AS;
    const uint32_t a = 3 * (A0[x] + A2[x] + A0[x + 2] + A2[x + 2]) +
                       4 * (A1[x] + A0[x + 1] + A1[x + 1] + A2[x + 1] + A1[x + 2]);
    const uint32_t b = 3 * (B0[x] + B2[x] + B0[x + 2] + B2[x + 2]) +
                       4 * (B1[x] + B0[x + 1] + B1[x + 1] + B2[x + 1] + B1[x + 2]);
    f1 = (a * px + b + ((1u << sh) >> 1)) >> sh;
  } else {
    f1 = px << kRstBits;
  }
}
// the restored pixel (:734-746)
__device__ __forceinline__ int sgr_out(uint32_t f2, uint32_t f1, uint32_t px, int w0, int w1, int mx) {
  const int32_t u = (int32_t)(px << kRstBits);
  const int32_t v = w0 * (int32_t)f2 + w1 * u + ((1 << kPrjBits) - w0 - w1) * (int32_t)f1;
  constexpr int sh = kRstBits + kPrjBits;
  return iclamp((v + ((1 << sh) >> 1)) >> sh, 0, mx);
}

// the integral images of a region (w x h, rows / columns of the image from
// pix(r, c)): row prefix sums, then column prefix sums, u32 wrapping
template <int W, int HMAX, typename Pix>
__device__ inline void sgr_integral(SgrLds<W, HMAX> &L, int w, int h, Pix pix) {
  using S = SgrLds<W, HMAX>;
  const int rows = 4 + h + (h & 1) + 2, cols = w + 7;
  for (int i = threadIdx.x; i < rows * cols; i += blockDim.x) {
    const int r = i / cols, c = i - r * cols;
    const uint32_t v = pix(r, c);
    L.ii[r * S::IS + c] = v;
    L.sq[r * S::IS + c] = v * v;
  }
  __syncthreads();
  for (int r = threadIdx.x; r < 2 * rows; r += blockDim.x) {
    uint32_t *p = (r < rows ? L.ii : L.sq) + (r % rows) * S::IS, acc = 0;
    for (int c = 0; c < cols; c++) p[c] = acc += p[c];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * cols; c += blockDim.x) {
    uint32_t *p = (c < cols ? L.ii : L.sq) + c % cols, acc = 0;
    for (int r = 0; r < rows; r++) p[r * S::IS] = acc += p[r * S::IS];
  }
  __syncthreads();
}

// sum of a u64 over the workgroup (LDS slots red[0 .. 8)), result to all lanes
__device__ inline uint64_t wg_sum_u64(uint64_t v, uint64_t *red) {
  v = group_sum<64>(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t t = 0;
  for (int i = 0; i < (int)(blockDim.x >> 6); i++) t += red[i];
  __syncthreads();
  return t;
}
__device__ inline int64_t wg_sum_i64(int64_t v, uint64_t *red) { return (int64_t)wg_sum_u64((uint64_t)v, red); }

// ---- the unit decision's distortions (rdo_loop_decision) -----------------------
struct LrfRdoArgs {
  rv_plane rec[3], src[3];
  const uint8_t *skip;  // per luma 4x4 of the frame
  int mi_stride;
  const float *imp;
  int w_imp, w_in_b, h_in_b;
  LrfGeo g;
  int cdef;                  // CDEF on (strengths at index 0)
  int pri_y, sec_y, pri_uv, sec_uv, damping;
  double ds[3];
  uint64_t *err;             // [3][nsb][17]
  int8_t *xqd;               // [3][nsb][16][2]
};

constexpr int kRdoThreads = 256;

template <typename Px>
__global__ __launch_bounds__(kRdoThreads) void lrf_rdo_kernel(LrfRdoArgs a) {
  using L64 = SgrLds<64, 64>;
  __shared__ L64 L;
  __shared__ uint16_t pad[68 * 68];  // the padded CDEF input (cdef_sb_padded_frame_copy)
  __shared__ uint16_t lin[64 * 64];  // the unit's input (lrf_input)
  __shared__ uint8_t bdir[64], bskip[64];
  __shared__ int32_t bvar[64];
  __shared__ uint64_t red[kRdoThreads / 64];
  __shared__ int8_t sxqd[2];
  const LrfGeo &g = a.g;
  const int p = blockIdx.y, sb = blockIdx.x;
  const int sbc = g.sbc, fsx = sb % sbc, fsy = sb / sbc;
  if (fsx >= g.cols[p] || fsy >= g.rows[p]) return;  // no unit (uniform)
  const int t0x = fsx - fsx % g.tws, t0y = fsy - fsy % g.ths, sx = fsx - t0x, sy = fsy - t0y;
  const int xd = p ? g.xdec : 0, yd = p ? g.ydec : 0, bw = 64 >> xd, bh = 64 >> yd;
  const int tw_px = min(g.tws * 64, g.W - t0x * 64), th_px = min(g.ths * 64, g.H - t0y * 64);
  const int pw_t = (tw_px + xd) >> xd, ph_t = (th_px + yd) >> yd;
  const int mi_cols = tw_px >> 2, mi_rows = th_px >> 2;
  const int ox = (sx * 64) >> xd, oy = (sy * 64) >> yd, fx0 = (t0x * 64) >> xd, fy0 = (t0y * 64) >> yd;
  const int bd = g.bd, cs = bd - 8, mx = (1 << bd) - 1;
  const rv_plane &rec = a.rec[p], &src = a.src[p];
  auto recpx = [&](int x, int y) -> int {  // frame plane coordinates
    return (int)((const Px *)rec.data)[(int64_t)(rec.yorigin + y) * rec.stride + rec.xorigin + x];
  };
  // 1. the padded copy and the unit's input
  for (int i = threadIdx.x; i < (bh + 4) * (bw + 4); i += blockDim.x) {
    const int y = i / (bw + 4) - 2, x = i % (bw + 4) - 2, tx = ox + x, ty = oy + y;
    int v = kVeryLarge;
    if (tx >= 0 && tx < pw_t && ty >= 0 && ty < ph_t) {
      const int csx = (tx << xd) >> 6, csy = (ty << yd) >> 6;
      v = (csy < sy || (csy == sy && csx <= sx)) ? recpx(fx0 + tx, fy0 + ty) : 128;
    }
    pad[i] = (uint16_t)v;
  }
  const int vw = min(bw, pw_t - ox), vh = min(bh, ph_t - oy);
  for (int i = threadIdx.x; i < bw * bh; i += blockDim.x) {
    const int y = i / bw, x = i - y * bw;
    lin[i] = (uint16_t)recpx(fx0 + ox + min(x, vw - 1), fy0 + oy + min(y, vh - 1));
  }
  // 2. CDEF index 0 on the 8x8 blocks inside the tile (cdef_filter_superblock)
  if (a.cdef) {
    if (threadIdx.x < 64) {
      const int bx = threadIdx.x & 7, by = threadIdx.x >> 3, gx = sx * 16 + 2 * bx, gy = sy * 16 + 2 * by;
      uint8_t sk = 2, dir = 0;
      int32_t var = 0;
      if (gx < mi_cols && gy < mi_rows) {
        const uint8_t *k = a.skip + (int64_t)(t0y * 16 + gy) * a.mi_stride + t0x * 16 + gx;
        sk = k[0] & k[1] & k[a.mi_stride] & k[a.mi_stride + 1];
        if (!sk) {
          const rv_plane &yl = a.rec[0];
          const Px *bp = (const Px *)yl.data + (int64_t)(yl.yorigin + t0y * 64 + sy * 64 + 8 * by) * yl.stride +
                         yl.xorigin + t0x * 64 + sx * 64 + 8 * bx;
          dir = (uint8_t)cdef_dir<Px>(bp, yl.stride, cs, &var);
        }
      }
      bskip[threadIdx.x] = sk;
      bdir[threadIdx.x] = dir;
      bvar[threadIdx.x] = var;
    }
    __syncthreads();
    const int bxs = 8 >> xd, bys = 8 >> yd;
    for (int i = threadIdx.x; i < bw * bh; i += blockDim.x) {
      const int y = i / bw, x = i - y * bw, blk = (y / bys) * 8 + x / bxs;
      if (bskip[blk]) continue;  // skip: the copy (equal to lin); 2: outside the tile
      int pri, sec, dmp = a.damping + cs, d;
      if (p == 0) {
        pri = cdef_adjust(a.pri_y << cs, bvar[blk]);
        sec = a.sec_y << cs;
        d = a.pri_y ? bdir[blk] : 0;
      } else {
        pri = a.pri_uv << cs;
        sec = a.sec_uv << cs;
        dmp -= 1;
        d = a.pri_uv ? bdir[blk] : 0;
      }
      lin[i] = (uint16_t)cdef_px(pad + (y + 2) * (bw + 4) + x + 2, bw + 4, pri, sec, d, dmp, cs);
    }
  }
  __syncthreads();
  // 3. the unit (unit size clipped at the tile-relative offset, the
  // reference's quirk) and its integral image: lrf_input alone, replicated
  const int pw = p ? (g.W + xd) >> xd : g.W, ph = p ? (g.H + yd) >> yd : g.H;
  const int uw = min(bw, pw - ox), uh = min(bh, ph - oy);
  sgr_integral<64, 64>(L, uw, uh, [&](int r, int c) -> uint32_t {
    return lin[iclamp(r - 4, 0, uh - 1) * bw + iclamp(c - 4, 0, uw - 1)];
  });
  // 4. the distortions: rdo_loop_plane_error over the superblock's 8x8s in
  // the tile; lane = 8x8 block (64), the option's pixels from `val`
  const int64_t ss_ = src.stride;
  const Px *sbase = (const Px *)src.data + (int64_t)(src.yorigin + fy0 + oy) * ss_ + src.xorigin + fx0 + ox;
  auto plane_err = [&](auto val) -> uint64_t {
    uint64_t e = 0;
    if (threadIdx.x < 64) {
      const int bx = threadIdx.x & 7, by = threadIdx.x >> 3, gx = sx * 16 + 2 * bx, gy = sy * 16 + 2 * by;
      if (gx < mi_cols && gy < mi_rows) {
        const double bias = lrf_bias(a.imp, a.w_imp, a.w_in_b, a.h_in_b, t0x * 16 + gx, t0y * 16 + gy);
        const int qx = (8 * bx) >> xd, qy = (8 * by) >> yd;
        if (p == 0) {
          int32_t ss = 0, sd = 0;
          uint32_t ss2 = 0, sd2 = 0, ssd = 0;
          for (int j = 0; j < 8; j++)
            for (int i = 0; i < 8; i++) {
              const int32_t s = sbase[(int64_t)(qy + j) * ss_ + qx + i], d = val(qx + i, qy + j);
              ss += s;
              sd += d;
              ss2 += (uint32_t)(s * s);
              sd2 += (uint32_t)(d * d);
              ssd += (uint32_t)(s * d);
            }
          e = biased(cdef_dist(ss, sd, ss2, sd2, ssd, bd), bias);
        } else {  // sse_wxh of (8 >> xdec) x (8 >> ydec) in parts of the importance block
          const int w8 = 8 >> xd, h8 = 8 >> yd, pbw = min(8, w8) >> xd, pbh = min(8, h8) >> yd;
          for (int py = 0; py < h8 / pbh; py++)
            for (int px_ = 0; px_ < w8 / pbw; px_++) {
              uint64_t v = 0;
              for (int j = 0; j < pbh; j++) {
                uint32_t row = 0;
                for (int i = 0; i < pbw; i++) {
                  const int c = (int)(int16_t)sbase[(int64_t)(qy + py * pbh + j) * ss_ + qx + px_ * pbw + i] -
                                (int)(int16_t)val(qx + px_ * pbw + i, qy + py * pbh + j);
                  row += (uint32_t)(c * c);
                }
                v += row;
              }
              e += biased(v, bias);
            }
        }
      }
    }
    const uint64_t t = wg_sum_u64(e, red);
    return (uint64_t)((double)t * a.ds[p]);
  };
  uint64_t *eo = a.err + ((size_t)p * g.nsb + sb) * 17;
  int8_t *xo = a.xqd + ((size_t)p * g.nsb + sb) * 32;
  {
    const uint64_t e = plane_err([&](int x, int y) { return (int32_t)lin[y * bw + x]; });
    if (threadIdx.x == 0) eo[0] = e;
  }
  // 5. the 16 sets: tables, solve sums, xqd, the filtered unit's distortion
  for (int set = 0; set < 16; set++) {
    sgr_tables<64, 64>(L, set, uw, uh, cs);
    __syncthreads();
    int64_t H00 = 0, H11 = 0, H01 = 0, C0 = 0, C1 = 0;
    for (int i = threadIdx.x; i < uw * uh; i += blockDim.x) {
      const int y = i / uw, x = i - y * uw;
      const uint32_t px = lin[y * bw + x], px0 = lin[(y & ~1) * bw + x];
      uint32_t f2, f1;
      sgr_f<64, 64>(L, set, x, y, px, px0, f2, f1);
      // sgrproj_solve reads the source at the unit's tile-relative offset
      // of the whole frame (ts.input with loop_tile_po, src/rdo.rs:2028-2033)
      const int64_t u = (int64_t)px << kRstBits;
      const int64_t s = ((int64_t)((const Px *)src.data)[(int64_t)(src.yorigin + oy + y) * ss_ + src.xorigin +
                                                         ox + x]
                         << kRstBits) - u;
      const int64_t e2 = (int64_t)(int32_t)f2 - u, e1 = (int64_t)(int32_t)f1 - u;
      H00 += e2 * e2;
      H11 += e1 * e1;
      H01 += e1 * e2;
      C0 += e2 * s;
      C1 += e1 * s;
    }
    H00 = wg_sum_i64(H00, red);
    H11 = wg_sum_i64(H11, red);
    H01 = wg_sum_i64(H01, red);
    C0 = wg_sum_i64(C0, red);
    C1 = wg_sum_i64(C1, red);
    if (threadIdx.x == 0) {
      int8_t q[2];
      lrf_solve_finish(set, uw, uh, H00, H01, H11, C0, C1, q);
      sxqd[0] = q[0];
      sxqd[1] = q[1];
      xo[2 * set] = q[0];
      xo[2 * set + 1] = q[1];
    }
    __syncthreads();
    const int w0 = sxqd[0], w1 = sxqd[1];
    const uint64_t e = plane_err([&](int x, int y) -> int32_t {
      if (x >= uw || y >= uh) return 128;  // lrf_output's fill (never inside the frame)
      const uint32_t px = lin[y * bw + x], px0 = lin[(y & ~1) * bw + x];
      uint32_t f2, f1;
      sgr_f<64, 64>(L, set, x, y, px, px0, f2, f1);
      return sgr_out(f2, f1, px, w0, w1, mx);
    });
    if (threadIdx.x == 0) eo[1 + set] = e;
    __syncthreads();  // the tables are rewritten by the next set
  }
}

// ---- the sequential decisions (count_lrf_switchable, write_lrf) -----------------
struct LrfDecideArgs {
  LrfGeo g;
  const uint64_t *err;
  const int8_t *xqd;
  double lambda;
  int8_t *units;  // [3][rows][cols][3]: set (-1 None), xqd0, xqd1
};

__global__ void lrf_decide_kernel(LrfDecideArgs a) {
  const LrfGeo &g = a.g;
  const int ntx = (g.sbc + g.tws - 1) / g.tws, nty = (g.sbr + g.ths - 1) / g.ths;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntx * nty) return;
  const int t0x = (t % ntx) * g.tws, t0y = (t / ntx) * g.ths;
  const int tsw = min(g.tws, g.sbc - t0x), tsh = min(g.ths, g.sbr - t0y);
  LrfTileState st;
  lrf_tile_init(st);
  for (int sy = 0; sy < tsh; sy++)
    for (int sx = 0; sx < tsw; sx++) {
      const int fsx = t0x + sx, fsy = t0y + sy, sb = fsy * g.sbc + fsx;
      int8_t pick[3][3];
      bool has[3];
      for (int p = 0; p < 3; p++) {
        has[p] = fsx < g.cols[p] && fsy < g.rows[p];
        if (!has[p]) {  // stretched into its neighbour's unit: none of its own
          int8_t *u = a.units + (((size_t)p * g.urows_max + fsy) * g.ucols_max + fsx) * 3;
          u[0] = -1;
          u[1] = u[2] = 0;
          continue;
        }
        const uint64_t *e = a.err + ((size_t)p * g.nsb + sb) * 17;
        const int8_t *xq = a.xqd + ((size_t)p * g.nsb + sb) * 32;
        int best = -1;
        double best_cost = (double)e[0] + a.lambda * ((double)lrf_rate(st, p, -1, nullptr) / 8.0);
        for (int s = 0; s < 16; s++) {
          const double c = (double)e[1 + s] + a.lambda * ((double)lrf_rate(st, p, s, xq + 2 * s) / 8.0);
          if (c < best_cost) {
            best_cost = c;
            best = s;
          }
        }
        pick[p][0] = (int8_t)best;
        pick[p][1] = best < 0 ? 0 : xq[2 * best];
        pick[p][2] = best < 0 ? 0 : xq[2 * best + 1];
        int8_t *u = a.units + (((size_t)p * g.urows_max + fsy) * g.ucols_max + fsx) * 3;
        u[0] = pick[p][0];
        u[1] = pick[p][1];
        u[2] = pick[p][2];
      }
      for (int p = 0; p < 3; p++)
        if (has[p]) lrf_commit(st, p, pick[p][0], pick[p] + 1);
    }
}

// ---- lrf_filter_frame (src/lrf.rs:1345-1444) ------------------------------------
struct LrfFilterArgs {
  rv_plane cd[3], db[3], out[3];  // the CDEF output, the deblocked frame, the restored frame
  LrfGeo g;
  const int8_t *units;
  int enable_cdef;
  int nchunk[3], nstripe;  // 32-column chunks per plane row, stripes
};

template <typename Px>
__global__ __launch_bounds__(256) void lrf_filter_kernel(LrfFilterArgs a) {
  using L32 = SgrLds<32, 64>;
  __shared__ L32 L;
  __shared__ uint16_t blk[64 * 32];  // the stripe chunk's CDEF output
  const LrfGeo &g = a.g;
  const int p = blockIdx.z, si = blockIdx.y, ck = blockIdx.x;
  if (ck >= a.nchunk[p]) return;
  const int xd = p ? g.xdec : 0, yd = p ? g.ydec : 0;
  const int crop_w = (g.W + ((1 << xd) >> 1)) >> xd, crop_h = (g.H + ((1 << yd) >> 1)) >> yd;
  int y0, sz;
  if (si == 0) {
    y0 = 0;
    sz = (64 - 8) >> yd;
  } else {
    y0 = (si * 64 - 8) >> yd;
    sz = min(64 >> yd, crop_h - y0);
  }
  const int x = ck * 32, w = min(32, crop_w - x);
  if (sz <= 0 || w <= 0) return;
  const int us = g.unit[p], rux = min(x / us, g.cols[p] - 1);
  const int ruy = min(si * g.stripe_h[p] / us, g.rows[p] - 1);
  const int8_t *u = a.units + (((size_t)p * g.urows_max + ruy) * g.ucols_max + rux) * 3;
  const rv_plane &cd = a.cd[p], &db = a.db[p], &out = a.out[p];
  auto at = [](const rv_plane &pl, int xx, int yy) -> int {
    return (int)((const Px *)pl.data)[(int64_t)(pl.yorigin + yy) * pl.stride + pl.xorigin + xx];
  };
  Px *op = (Px *)out.data + (int64_t)(out.yorigin + y0) * out.stride + out.xorigin + x;
  if (u[0] < 0 || !a.enable_cdef) {  // None: the CDEF output as it is
    for (int i = threadIdx.x; i < w * sz; i += blockDim.x) {
      const int yy = i / w, xx = i - yy * w;
      op[(int64_t)yy * out.stride + xx] = (Px)at(cd, x + xx, y0 + yy);
    }
    return;
  }
  // setup_integral_image's view (VertPaddedIter / HorzPaddedIter): columns
  // clamp to the frame (the unit's own right limit reaches 3 past it),
  // rows to the frame and the stripe's +-2 extension, deblocked outside
  const int sh = sz + (sz & 1), crop = crop_h;
  sgr_integral<32, 64>(L, w, sz, [&](int r, int c) -> uint32_t {
    const int cy = iclamp(y0 - 4 + r, 0, crop - 1), ly = iclamp(cy, y0 - 2, y0 + sh + 1);
    const int xx = iclamp(x - 4 + c, 0, crop_w - 1);
    return (uint32_t)((ly >= y0 && ly < y0 + sh) ? at(cd, xx, ly) : at(db, xx, ly));
  });
  for (int i = threadIdx.x; i < w * sz; i += blockDim.x) {
    const int yy = i / w, xx = i - yy * w;
    blk[yy * 32 + xx] = (uint16_t)at(cd, x + xx, y0 + yy);
  }
  const int set = u[0];
  sgr_tables<32, 64>(L, set, w, sz, g.bd - 8);
  __syncthreads();
  const int mx = (1 << g.bd) - 1;
  for (int i = threadIdx.x; i < w * sz; i += blockDim.x) {
    const int yy = i / w, xx = i - yy * w;
    const uint32_t px = blk[yy * 32 + xx], px0 = blk[(yy & ~1) * 32 + xx];
    uint32_t f2, f1;
    sgr_f<32, 64>(L, set, xx, yy, px, px0, f2, f1);
    op[(int64_t)yy * out.stride + xx] = (Px)sgr_out(f2, f1, px, u[1], u[2], mx);
  }
}

}  // namespace
}  // namespace rv

using namespace rv;

int lrf_geometry(int width, int height, int xdec, int ydec, int bit_depth, int base_q_idx,
                 int tile_w_sb, int tile_h_sb, LrfGeo *g) {
  memset(g, 0, sizeof(*g));
  g->W = width;
  g->H = height;
  g->xdec = xdec;
  g->ydec = ydec;
  g->bd = bit_depth;
  g->sbc = (width + 63) / 64;
  g->sbr = (height + 63) / 64;
  g->nsb = g->sbc * g->sbr;
  g->tws = tile_w_sb > 0 ? tile_w_sb : g->sbc;
  g->ths = tile_h_sb > 0 ? tile_h_sb : g->sbr;
  const int tiled = (g->sbc + g->tws - 1) / g->tws > 1 || (g->sbr + g->ths - 1) / g->ths > 1;
  LrfPlaneCfg c[3];
  lrf_config(width, height, xdec, ydec, base_q_idx, tiled, g->tws, g->ths, c);
  for (int p = 0; p < 3; p++) {
    // one superblock per unit, the shape of every BASELINE config (a last
    // superblock row / column narrower than half a unit is stretched into
    // the unit before it: it has no unit of its own)
    if (c[p].sb_h_shift || c[p].sb_v_shift || c[p].cols > g->sbc || c[p].rows > g->sbr)
      return rv_set_error(RV_EINVAL, "loop restoration: units of one superblock only");
    g->unit[p] = c[p].unit_size;
    g->cols[p] = c[p].cols;
    g->rows[p] = c[p].rows;
    g->stripe_h[p] = c[p].stripe_h;
  }
  g->ucols_max = g->sbc;
  g->urows_max = g->sbr;
  return RV_OK;
}

int lrf_rdo_launch(const rv_plane rec[3], const rv_plane src[3], const uint8_t *skip, int mi_stride,
                   const float *imp, int w_imp, int w_in_b, int h_in_b, const LrfGeo &g, int cdef,
                   const uint8_t cdef_str[2], const double ds[3], uint64_t *err, int8_t *xqd,
                   double lambda, int8_t *units, hipStream_t s) {
  LrfRdoArgs a;
  memset(&a, 0, sizeof(a));
  for (int p = 0; p < 3; p++) {
    a.rec[p] = rec[p];
    a.src[p] = src[p];
    a.ds[p] = ds[p];
  }
  a.skip = skip;
  a.mi_stride = mi_stride;
  a.imp = imp;
  a.w_imp = w_imp;
  a.w_in_b = w_in_b;
  a.h_in_b = h_in_b;
  a.g = g;
  a.cdef = cdef;
  a.pri_y = cdef_str[0] / 4;
  a.sec_y = cdef_str[0] % 4 == 3 ? 4 : cdef_str[0] % 4;
  a.pri_uv = cdef_str[1] / 4;
  a.sec_uv = cdef_str[1] % 4 == 3 ? 4 : cdef_str[1] % 4;
  a.damping = 3;  // cdef_damping (src/encoder.rs:665)
  a.err = err;
  a.xqd = xqd;
  const dim3 grid((unsigned)g.nsb, 3);
  if (rec[0].hbd)
    lrf_rdo_kernel<uint16_t><<<grid, kRdoThreads, 0, s>>>(a);
  else
    lrf_rdo_kernel<uint8_t><<<grid, kRdoThreads, 0, s>>>(a);
  RV_HIP_CHECK_LAUNCH();
  LrfDecideArgs d;
  d.g = g;
  d.err = err;
  d.xqd = xqd;
  d.lambda = lambda;
  d.units = units;
  const int nt = ((g.sbc + g.tws - 1) / g.tws) * ((g.sbr + g.ths - 1) / g.ths);
  lrf_decide_kernel<<<(nt + 63) / 64, 64, 0, s>>>(d);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

int lrf_filter_launch(const rv_plane cd[3], const rv_plane db[3], const rv_plane out[3], const LrfGeo &g,
                      const int8_t *units, int enable_cdef, hipStream_t s) {
  LrfFilterArgs a;
  memset(&a, 0, sizeof(a));
  int most = 0;
  for (int p = 0; p < 3; p++) {
    a.cd[p] = cd[p];
    a.db[p] = db[p];
    a.out[p] = out[p];
    const int xd = p ? g.xdec : 0;
    const int cw = (g.W + ((1 << xd) >> 1)) >> xd;
    a.nchunk[p] = (cw + 31) / 32;
    most = a.nchunk[p] > most ? a.nchunk[p] : most;
  }
  a.g = g;
  a.units = units;
  a.enable_cdef = enable_cdef;
  a.nstripe = (g.H + 7) / 64 + 1;
  const dim3 grid((unsigned)most, (unsigned)a.nstripe, 3);
  if (cd[0].hbd)
    lrf_filter_kernel<uint16_t><<<grid, 256, 0, s>>>(a);
  else
    lrf_filter_kernel<uint8_t><<<grid, 256, 0, s>>>(a);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}
