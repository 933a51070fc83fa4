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
#include <stddef.h>
#include <stdlib.h>
#include <algorithm>
#include <mutex>
#include <type_traits>
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
// the taps' offsets in a buffer of pitch s: [dir][k][primary, the two
// secondaries], from cdef_directions (one lane per entry)
__device__ __forceinline__ void cdef_offsets(int16_t *offs, int s) {
  const int t = threadIdx.x;
  if (t < 48) {
    const int dir = t / 6, k = (t / 3) & 1, j = t % 3;
    const int d = j == 0 ? dir : j == 1 ? (dir + 2) & 7 : (dir + 6) & 7;
    offs[t] = (int16_t)(kLrfCdefDirs[d][k][0] * s + kLrfCdefDirs[d][k][1]);
  }
}
// in: the padded u16 input at the pixel; off: cdef_offsets of its direction
__device__ inline int cdef_px(const uint16_t *in, const int16_t *off, int pri, int sec, int damping, int cs) {
  const int x = in[0];
  const int odd = (pri >> cs) & 1;
  int sum = 0, mx = x, mn = x;
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const int pt = odd ? 3 : (k ? 2 : 4), st = k ? 1 : 2;
    const int d0 = off[3 * k], d1 = off[3 * k + 1], d2 = off[3 * k + 2];
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
// The LDS of one region (w x h pixels, w <= W): the integral images
// ((h + 7) x (w + 7), ii then sq), the r = 1 (a, b) rows 0 .. h + 1 and the
// r = 2 rows 0, 2, .. h (+1), each w + 2 wide, (a, b) side by side (one
// 8-byte read), and x_by_xplus1 of z.
template <int W, int HMAX>
struct SgrLds {
  static constexpr int IS = W + 7, IR = HMAX + 8;  // image pitch / rows
  static constexpr int AS = W + 2, A1R = HMAX + 2, A2R = HMAX / 2 + 2;
  static constexpr int TAB = (A1R + A2R) * AS;
  uint32_t ii[IR * IS], sq[IR * IS];
  uint2 tab[TAB];  // r = 1 rows then r = 2 rows
  uint16_t xz[256];
};
using SgrL64 = SgrLds<64, 64>;
using SgrL32 = SgrLds<32, 64>;
// the loops below walk ii and sq as one array by integer offsets (a select
// of two LDS constants trips the compiler here)
static_assert(offsetof(SgrL32, sq) == sizeof(uint32_t) * SgrL32::IR * SgrL32::IS, "");

// x_by_xplus1 (the a of sgrproj_sum_finish for z < 255); every lane, a
// barrier before the first use
__device__ __forceinline__ void sgr_init_xz(uint16_t *xz) {
  for (int z = threadIdx.x; z < 256; z += blockDim.x)
    xz[z] = (uint16_t)(z == 255 ? 256 : z == 0 ? 1 : ((z << kSgrBits) + z / 2) / (z + 1));
}
// sgrproj_sum_finish (:305-323), u32 wrapping, in its two halves: the box's
// p (the set-independent variance term) with its sum, then a and b of
// strength s
__device__ __forceinline__ uint2 sgr_box(uint32_t ssq, uint32_t sum, uint32_t n, int bdm8) {
  const uint32_t sssq = (ssq + ((1u << (2 * bdm8)) >> 1)) >> (2 * bdm8);
  const uint32_t ssum = (sum + ((1u << bdm8) >> 1)) >> bdm8;
  const int32_t pd = (int32_t)(sssq * n - ssum * ssum);  // (i32) - (i32), wrapping
  return make_uint2((uint32_t)(pd > 0 ? pd : 0), sum);
}
__device__ __forceinline__ uint2 sgr_ab(uint2 ps, uint32_t s, uint32_t one_over_n, const uint16_t *xz) {
  const uint32_t z = (ps.x * s + ((1u << kMtableBits) >> 1)) >> kMtableBits;
  const uint32_t a = xz[z < 255 ? z : 255];
  const uint32_t bb = ((1u << kSgrBits) - a) * ps.y * one_over_n;
  return make_uint2(a, (bb + ((1u << kRecipBits) >> 1)) >> kRecipBits);
}
// get_integral_square (:326-334): rows (y, y + d], columns (x, x + d] of
// the image at ii + o (o = y * s + x)
__device__ __forceinline__ uint32_t isq(const uint32_t *ii, int s, int o, int d) {
  return ii[o] + ii[o + d * s + d] - ii[o + d * s] - ii[o + d];
}

// A lane's fixed place in a region's (w + 2)-wide tables: column tx, first
// row ty, row step tstep (lanes past tstep full rows idle).
struct SgrLane {
  int tx, ty, tstep;
};
__device__ __forceinline__ SgrLane sgr_lane(int w, int t, int nt) {  // lane t of nt
  const int cw = w + 2, step = nt / cw;
  return {t % cw, t >= 0 && t < step * cw ? t / cw : 1 << 20, step};
}
__device__ __forceinline__ SgrLane sgr_lane(int w) { return sgr_lane(w, (int)threadIdx.x, (int)blockDim.x); }
// where table row r of a set with r1rows rows of r = 1 lives, and its box
// in the image: r = 1 boxes from (1, 1) (:626-650, 877-889), r = 2 at even
// rows (:611-624, 843-856)
template <int IS, int AS, int A1R>
__device__ __forceinline__ void sgr_row(int r, int r1rows, int tx, int &to, int &o, int &d) {
  if (r < r1rows) {
    to = r * AS + tx;
    o = (r + 1) * IS + tx + 1;
    d = 3;
  } else {
    const int yr = r - r1rows;
    to = (A1R + yr) * AS + tx;
    o = 2 * yr * IS + tx;
    d = 5;
  }
}

// A table entry: (a, b) side by side, or packed in one word ((a << 20) | b:
// a <= 256, b < 2^20 since it is a u32 >> 12) where LDS is short.
constexpr uint32_t kBMask = (1u << 20) - 1;
__device__ __forceinline__ uint2 tab_get(uint2 v) { return v; }
__device__ __forceinline__ uint2 tab_get(uint32_t v) { return make_uint2(v >> 20, v & kBMask); }
__device__ __forceinline__ void tab_put(uint2 &d, uint2 v) { d = v; }
__device__ __forceinline__ void tab_put(uint32_t &d, uint2 v) { d = (v.x << 20) | v.y; }

// the (a, b) tables of set s straight from the integral images (every lane)
template <int IS, int IR, int AS, int A1R, typename T>
__device__ __forceinline__ void sgr_tables(const uint32_t *img, T *tab, const uint16_t *xz,
                                           const SgrLane &ln, int set, int h, int bdm8) {
  const uint32_t s2 = kSgrS[set][0], s1 = kSgrS[set][1];
  const int r1rows = s1 ? h + 2 : 0, r2rows = s2 ? (h + 1) / 2 + 1 : 0;  // r = 2: rows 0, 2, .., <= h + 1
  for (int r = ln.ty; r < r1rows + r2rows; r += ln.tstep) {
    int to, o, d;
    sgr_row<IS, AS, A1R>(r, r1rows, ln.tx, to, o, d);
    const bool one = r < r1rows;
    tab_put(tab[to], sgr_ab(sgr_box(isq(img, IS, IR * IS + o, d), isq(img, IS, o, d), one ? 9 : 25, bdm8),
                            one ? s1 : s2, one ? 455 : 164, xz));
  }
}
// the boxes' (p, sum) of both radii, once per region (every lane) ...
template <int IS, int IR, int AS, int A1R>
__device__ __forceinline__ void sgr_boxes(const uint32_t *img, uint2 *ps, const SgrLane &ln, int h, int bdm8) {
  const int r1rows = h + 2, r2rows = (h + 1) / 2 + 1;
  for (int r = ln.ty; r < r1rows + r2rows; r += ln.tstep) {
    int to, o, d;
    sgr_row<IS, AS, A1R>(r, r1rows, ln.tx, to, o, d);
    ps[to] = sgr_box(isq(img, IS, IR * IS + o, d), isq(img, IS, o, d), r < r1rows ? 9 : 25, bdm8);
  }
}
// ... and each set's tables from them (the same places)
template <int AS, int A1R>
__device__ __forceinline__ void sgr_tables_ps(const uint2 *ps, uint2 *tab, const uint16_t *xz,
                                              const SgrLane &ln, int set, int h) {
  const uint32_t s2 = kSgrS[set][0], s1 = kSgrS[set][1];
  const int r1rows = s1 ? h + 2 : 0, r2rows = s2 ? (h + 1) / 2 + 1 : 0;
#pragma unroll 2
  for (int r = ln.ty; r < r1rows + r2rows; r += ln.tstep) {
    const bool one = r < r1rows;
    const int to = (one ? r : A1R + r - r1rows) * AS + ln.tx;
    tab[to] = sgr_ab(ps[to], one ? s1 : s2, one ? 455 : 164, xz);
  }
}

// 5 * (t[x] + t[x + 2]) + 6 * t[x + 1], a and b
template <typename T>
__device__ __forceinline__ void sgr_row3(const T *t, int x, uint32_t &a, uint32_t &b) {
  const uint2 v0 = tab_get(t[x]), v1 = tab_get(t[x + 1]), v2 = tab_get(t[x + 2]);
  a = 5 * (v0.x + v2.x) + 6 * v1.x;
  b = 5 * (v0.y + v2.y) + 6 * v1.y;
}
// f_r2 and f_r1 of pixel (x, y) with value px (src/lrf.rs:244-301 via the
// row loop :656-733); px0: the pixel of row y & ~1 (box_f_r0 shares it)
template <int AS, int A1R>
__device__ __forceinline__ void sgr_f(const uint2 *tab, int set, int x, int y, uint32_t px, uint32_t px0,
                                      uint32_t &f2, uint32_t &f1) {
  const uint32_t s2 = kSgrS[set][0], s1 = kSgrS[set][1];
  constexpr int sh = 5 + kSgrBits - kRstBits, sho = 4 + kSgrBits - kRstBits;
  if (s2) {
    const int yr = y >> 1;
    uint32_t ao, bo;
    sgr_row3(tab + (A1R + yr + 1) * AS, x, ao, bo);
    if (!(y & 1)) {
      uint32_t a, b;
      sgr_row3(tab + (A1R + yr) * AS, x, a, b);
      f2 = ((a + ao) * px + b + bo + ((1u << sh) >> 1)) >> sh;
    } else {
      f2 = (ao * px + bo + ((1u << sho) >> 1)) >> sho;
    }
  } else {
    f2 = px0 << kRstBits;
  }
  if (s1) {
    const uint2 *T0 = tab + y * AS + x, *T1 = T0 + AS, *T2 = T1 + AS;
    const uint2 c0 = T0[0], c1 = T0[1], c2 = T0[2], c3 = T1[0], c4 = T1[1], c5 = T1[2], c6 = T2[0],
                c7 = T2[1], c8 = T2[2];
    // corners weigh 3, the cross 4
    const uint32_t a = 3 * (c0.x + c6.x + c2.x + c8.x) + 4 * (c3.x + c1.x + c4.x + c7.x + c5.x);
    const uint32_t b = 3 * (c0.y + c6.y + c2.y + c8.y) + 4 * (c3.y + c1.y + c4.y + c7.y + c5.y);
    f1 = (a * px + b + ((1u << sh) >> 1)) >> sh;
  } else {
    f1 = px << kRstBits;
  }
}
// sgr_f of the four pixels (x, y0 .. y0 + 3) of a column strip (y0 a
// multiple of 4): the table rows they share are read once
template <int AS, int A1R, typename T>
__device__ __forceinline__ void sgr_f4(const T *tab, int set, int x, int y0, const uint32_t px[4],
                                       uint32_t f2[4], uint32_t f1[4]) {
  const uint32_t s2 = kSgrS[set][0], s1 = kSgrS[set][1];
  constexpr int sh = 5 + kSgrBits - kRstBits, sho = 4 + kSgrBits - kRstBits;
  constexpr uint32_t rnd = (1u << sh) >> 1, rndo = (1u << sho) >> 1;
  // (the results go to scalars in both branches and to the arrays after
  // them: array stores inside the branches sent the arrays to scratch)
  uint32_t g0, g1, g2, g3, h0, h1, h2, h3;
  if (s2) {  // r = 2 rows y0 / 2 .. y0 / 2 + 2: even pixels use two, odd ones the second
    uint32_t wa[3], wb[3];
#pragma unroll
    for (int j = 0; j < 3; j++) sgr_row3(tab + (A1R + (y0 >> 1) + j) * AS, x, wa[j], wb[j]);
    g0 = ((wa[0] + wa[1]) * px[0] + wb[0] + wb[1] + rnd) >> sh;
    g1 = (wa[1] * px[1] + wb[1] + rndo) >> sho;
    g2 = ((wa[1] + wa[2]) * px[2] + wb[1] + wb[2] + rnd) >> sh;
    g3 = (wa[2] * px[3] + wb[2] + rndo) >> sho;
  } else {  // box_f_r0: the pixel of the even row
    g0 = g1 = px[0] << kRstBits;
    g2 = g3 = px[2] << kRstBits;
  }
  if (s1) {  // r = 1 rows y0 .. y0 + 5: each row's corner pair and middle
    uint32_t ca[6], cb[6], ma[6], mb[6], o[4];
#pragma unroll
    for (int j = 0; j < 6; j++) {
      const T *t = tab + (y0 + j) * AS + x;
      const uint2 v0 = tab_get(t[0]), v1 = tab_get(t[1]), v2 = tab_get(t[2]);
      ca[j] = v0.x + v2.x;
      cb[j] = v0.y + v2.y;
      ma[j] = v1.x;
      mb[j] = v1.y;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {  // corners weigh 3, the cross 4
      const uint32_t a = 3 * (ca[k] + ca[k + 2]) + 4 * (ma[k] + ca[k + 1] + ma[k + 1] + ma[k + 2]);
      const uint32_t b = 3 * (cb[k] + cb[k + 2]) + 4 * (mb[k] + cb[k + 1] + mb[k + 1] + mb[k + 2]);
      o[k] = (a * px[k] + b + rnd) >> sh;
    }
    h0 = o[0];
    h1 = o[1];
    h2 = o[2];
    h3 = o[3];
  } else {
    h0 = px[0] << kRstBits;
    h1 = px[1] << kRstBits;
    h2 = px[2] << kRstBits;
    h3 = px[3] << kRstBits;
  }
  f2[0] = g0;
  f2[1] = g1;
  f2[2] = g2;
  f2[3] = g3;
  f1[0] = h0;
  f1[1] = h1;
  f1[2] = h2;
  f1[3] = h3;
}
// the restored pixel (:734-746)
__device__ __forceinline__ int sgr_out(uint32_t f2, uint32_t f1, uint32_t px, int w0, int w1, int mx) {
  const int32_t u = (int32_t)(px << kRstBits);
  const int32_t v = w0 * (int32_t)f2 + w1 * u + ((1 << kPrjBits) - w0 - w1) * (int32_t)f1;
  constexpr int sh = kRstBits + kPrjBits;
  return iclamp((v + ((1 << sh) >> 1)) >> sh, 0, mx);
}

// inclusive u32 prefix sums (wrapping) of the image's lines -- rows of ii
// and sq, or their columns -- 8 lanes per line, each a chunk of up to 9
// consecutive elements in registers, the chunk totals scanned by shuffles
// within the 8 (lines up to 72 long)
template <int IS, int IR>
__device__ __forceinline__ void img_prefix(uint32_t *img, int rows, int cols, bool along_rows) {
  const int nline = along_rows ? 2 * rows : 2 * cols, len = along_rows ? cols : rows;
  const int chunk = (len + 7) >> 3, g = threadIdx.x & 7;
  for (int line = threadIdx.x >> 3; line < nline; line += blockDim.x >> 3) {
    uint32_t *p;
    int st;
    if (along_rows) {
      p = img + (line < rows ? line : IR + line - rows) * IS;
      st = 1;
    } else {
      p = img + (line < cols ? line : IR * IS + line - cols);
      st = IS;
    }
    uint32_t v[9], acc = 0;
#pragma unroll
    for (int k = 0; k < 9; k++) {
      const int idx = g * chunk + k;
      v[k] = (k < chunk && idx < len) ? p[idx * st] : 0;
      acc += v[k];
      v[k] = acc;
    }
    uint32_t t = acc;
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) {
      const uint32_t u = __shfl_up(t, o, 8);
      if (g >= o) t += u;
    }
    const uint32_t off = t - acc;
#pragma unroll
    for (int k = 0; k < 9; k++) {
      const int idx = g * chunk + k;
      if (k < chunk && idx < len) p[idx * st] = v[k] + off;
    }
  }
}
// the integral images of a region (w x h, rows / columns of the image from
// pix(r, c)) at img (ii) and img + IR * IS (sq): the values, then row and
// column prefix sums
template <int IS, int IR, typename Pix>
__device__ __forceinline__ void sgr_integral(uint32_t *img, int w, int h, Pix pix) {
  const int rows = 4 + h + (h & 1) + 2, cols = w + 7;
  for (int i = threadIdx.x; i < rows * cols; i += blockDim.x) {
    const int r = i / cols, c = i - r * cols;
    const uint32_t v = pix(r, c);
    img[r * IS + c] = v;
    img[IR * IS + r * IS + c] = v * v;
  }
  __syncthreads();
  img_prefix<IS, IR>(img, rows, cols, true);
  __syncthreads();
  img_prefix<IS, IR>(img, rows, cols, false);
  __syncthreads();
}

// ---- wave sums on the DPP lane network (VALU, no LDS traffic) --------------
// lanes' values moved by DPP control CTRL; rows outside ROWS read 0
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xf, false);
}
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ uint64_t dpp64(uint64_t v) {
  return (uint64_t)dpp32<CTRL, ROWS>((uint32_t)(v >> 32)) << 32 | dpp32<CTRL, ROWS>((uint32_t)v);
}
template <typename T, int CTRL, int ROWS = 0xf>
__device__ __forceinline__ T dpp_t(T v) {
  if constexpr (sizeof(T) == 8)
    return (T)dpp64<CTRL, ROWS>((uint64_t)v);
  else
    return (T)dpp32<CTRL, ROWS>((uint32_t)v);
}
// the sum over each aligned 8 lanes, to all of them: quad_perm [1,0,3,2],
// [2,3,0,1], row_half_mirror (wrapping)
template <typename T>
__device__ __forceinline__ T dpp_sum8(T v) {
  v += dpp_t<T, 0xB1>(v);
  v += dpp_t<T, 0x4E>(v);
  v += dpp_t<T, 0x141>(v);
  return v;
}
// the sum over the wave, to all lanes: the rows of 16 (row_mirror), then
// row_bcast:15 / :31 carry them up to lane 63
__device__ __forceinline__ uint64_t dpp_sum64(uint64_t v) {
  v = dpp_sum8(v);
  v += dpp64<0x140>(v);
  v += dpp64<0x142, 0xa>(v);
  v += dpp64<0x143, 0xc>(v);
  return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63) << 32 |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32 |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
  return __longlong_as_double((long long)readlane64((uint64_t)__double_as_longlong(v), l));
}
// lrf_solve_finish on a whole wave: the independent divisions on separate
// lanes (each IEEE-rounded as on one), the same operations in the same order
__device__ __forceinline__ void lrf_solve_finish_wave(int set, int w, int h, int64_t H00, int64_t H01,
                                                      int64_t H11, int64_t C0, int64_t C1, int8_t xqd[2]) {
  const int lane = threadIdx.x & 63;
  const bool r2 = lrf_set_has(set, 0), r1 = lrf_set_has(set, 1);
  const double n = (double)w * (double)h;
  const double num = lane == 0 ? (double)H00 : lane == 1 ? (double)H01 : lane == 2 ? (double)H11 : 128.0;
  const double q = num / n;
  const double h00 = readlane_f64(q, 0), h01 = readlane_f64(q, 1), h11 = readlane_f64(q, 2);
  const double sc = readlane_f64(q, 3);
  const double h10 = h01;
  const double c0 = (double)C0 * sc, c1 = (double)C1 * sc;
  int xq0, xq1;
  if (!r2) {
    xq0 = 0;
    xq1 = h11 == 0. ? 0 : (int)round(c1 / h11);
  } else if (!r1) {
    xq0 = h00 == 0. ? 0 : (int)round(c0 / h00);
    xq1 = 0;
  } else {
    const double det = h00 * h11 - h01 * h10;
    if (det == 0.) {
      xq0 = xq1 = 0;
    } else {
      const double d1 = h11 * c0 - h01 * c1, d2 = h00 * c1 - h10 * c0;
      const double r = (lane == 0 ? d1 : d2) / det;
      xq0 = (int)round(readlane_f64(r, 0));
      xq1 = (int)round(readlane_f64(r, 1));
    }
  }
  const int x0 = xq0 < -96 ? -96 : xq0 > 31 ? 31 : xq0;
  const int t = 128 - x0 - xq1, x1 = t < -32 ? -32 : t > 95 ? 95 : t;
  xqd[0] = (int8_t)x0;
  xqd[1] = (int8_t)x1;
}

// sum of a u64 over the workgroup (LDS slots red[0 .. 16)), result to all lanes
__device__ __forceinline__ uint64_t wg_sum_u64(uint64_t v, uint64_t *red) {
  v = dpp_sum64(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t t = 0;
  for (int i = 0; i < (int)(blockDim.x >> 6); i++) t += red[i];
  __syncthreads();
  return t;
}

// ---- the unit decision's distortions (rdo_loop_decision) -----------------------
struct LrfRdoArgs {
  rv_plane rec[3], src[3];
  const uint8_t *skip;  // per luma 4x4 of the frame
  int mi_stride;
  const float *imp;
  int w_imp, w_in_b, h_in_b;
  LrfGeo g;
  int p0;                    // the launch's first plane (blockIdx.y + p0)
  int gx0, gy0, gx1, gy1;    // the superblocks decided here (a tile group's)
  int cdef;                  // CDEF on (strengths at index 0)
  const uint8_t *dir;        // cdef_analyze_superblock of the unit's input: per 8x8 luma block,
  const int32_t *var;        // pitch dstride (rv_cdef_find_dirs)
  int dstride;
  int pri_y, sec_y, pri_uv, sec_uv, damping;
  double ds[3];
  uint64_t *err;             // [3][nsb][17]
  int8_t *xqd;               // [3][nsb][16][2]
};

// One workgroup per unit, BW * BH / 4 lanes: a lane owns a column strip of
// 4 pixels (x, y0 .. y0 + 3) -- one table read serves all four -- and keeps
// its f values in registers from the solve sums to the filtered pixels.
// 64 x 64 units (luma, 4:4:4 chroma): 1024 lanes, ~135 KB of LDS, one per
// CU; 32 x 32 (4:2:0 chroma): 256 lanes, ~36 KB, several per CU. The
// boxes' (p, sum) are set-independent: computed once, each set's (a, b)
// tables are a multiply and a table lookup per entry. The distortion of an
// option comes from the lanes' registers: 64-wide units sum half blocks
// over 8 lanes and the last wave joins the halves; 4:2:0 chroma sums 2x2
// parts over lane pairs.
#ifdef LRF_PHASES  // tools/ubench/lrf_bench.hip: one workgroup's phase clocks
__device__ unsigned long long lrf_phase_t[96];
#define PHASE(k) \
  if (tid == 0 && blockIdx.x == LRF_PHASES && p == 0) lrf_phase_t[k] = wall_clock64()
#else
#define PHASE(k)
#endif

template <int BW, int BH>
struct RdoLds {
  using L = SgrLds<BW, BH>;
  static constexpr int NT = BW * BH / 4, NW = NT / 64;
  union {
    uint32_t img[2 * L::IR * L::IS];  // ii, sq
    uint2 tab[L::TAB];                // then each set's (a, b)
  } a;
  union {
    uint16_t lin[BW * BH];  // the unit's input (lrf_input)
    uint2 ps[L::TAB];       // then the boxes' (p, sum)
  } b;
  uint16_t xz[256];
  int16_t coffs[48];                     // cdef_offsets at the pad's pitch
  uint16_t pad[(BW + 4) * (BH + 4)];     // the padded CDEF input
  uint16_t ssolve[BW * BH], esrc[BW * BH];  // the source at the solve's / the distortion's place
  uint8_t bdir[64], bskip[64];
  int32_t bvar[64];
  int64_t red5[5][NW];
  uint3 hm[(BH / 4) * 8];  // 64-wide: each half block's (sd, sd2, ssd) / (sse), [strip][block column]
  uint64_t wsum[NW];       // 4:2:0 chroma: each wave's biased part errors
  int32_t bss[64];         // luma: each block's source sum and sum of squares
  uint32_t bss2[64];
  int8_t sxqd[2];
};

template <typename Px, int BW, int BH>
__global__ __launch_bounds__(BW * BH / 4) void lrf_rdo_kernel(LrfRdoArgs a) {
  using Lds = RdoLds<BW, BH>;
  using SL = SgrLds<BW, BH>;
  constexpr int NT = Lds::NT, NW = Lds::NW, AS = SL::AS, A1R = SL::A1R;
  constexpr int LBW = BW == 64 ? 6 : 5;
  constexpr bool WIDE = BW == 64;  // luma / 4:4:4 chroma; else 4:2:0 chroma
  __shared__ Lds S;
  const LrfGeo &g = a.g;
  const int p = a.p0 + blockIdx.y, sb = blockIdx.x, tid = threadIdx.x;
  const int sbc = g.sbc, fsx = sb % sbc, fsy = sb / sbc;
  if (fsx >= g.cols[p] || fsy >= g.rows[p]) return;  // no unit (uniform)
  if (fsx < a.gx0 || fsx >= a.gx1 || fsy < a.gy0 || fsy >= a.gy1) return;  // another group's
  const int t0x = fsx - fsx % g.tws, t0y = fsy - fsy % g.ths, sx = fsx - t0x, sy = fsy - t0y;
  const int xd = p ? g.xdec : 0, yd = p ? g.ydec : 0;
  constexpr int npx = BW * BH;
  const int tw_px = min(g.tws * 64, g.W - t0x * 64), th_px = min(g.ths * 64, g.H - t0y * 64);
  const int pw_t = (tw_px + xd) >> xd, ph_t = (th_px + yd) >> yd;
  const int mi_cols = tw_px >> 2, mi_rows = th_px >> 2;
  const int ox = (sx * 64) >> xd, oy = (sy * 64) >> yd, fx0 = (t0x * 64) >> xd, fy0 = (t0y * 64) >> yd;
  const int bd = g.bd, cs = bd - 8, mx = (1 << bd) - 1;
  const rv_plane &rec = a.rec[p], &src = a.src[p];
  auto recpx = [&](int x, int y) -> int {  // frame plane coordinates
    return (int)((const Px *)rec.data)[(int64_t)(rec.yorigin + y) * rec.stride + rec.xorigin + x];
  };
  PHASE(0);
  sgr_init_xz(S.xz);
  cdef_offsets(S.coffs, BW + 4);
  // 1. the padded copy and the unit's input
  for (int i = tid; i < (BH + 4) * (BW + 4); i += NT) {
    const int y = i / (BW + 4) - 2, x = i % (BW + 4) - 2, tx = ox + x, ty = oy + y;
    int v = kVeryLarge;
    if (tx >= 0 && tx < pw_t && ty >= 0 && ty < ph_t) {
      const int csx = (tx << xd) >> 6, csy = (ty << yd) >> 6;
      v = (csy < sy || (csy == sy && csx <= sx)) ? recpx(fx0 + tx, fy0 + ty) : 128;
    }
    S.pad[i] = (uint16_t)v;
  }
  const int vw = min(BW, pw_t - ox), vh = min(BH, ph_t - oy);
  for (int i = tid; i < npx; i += NT) {
    const int y = i >> LBW, x = i & (BW - 1);
    S.b.lin[i] = (uint16_t)recpx(fx0 + ox + min(x, vw - 1), fy0 + oy + min(y, vh - 1));
  }
  // the unit (unit size clipped at the tile-relative offset, the
  // reference's quirk) and the two source tiles: sgrproj_solve's, read at
  // the unit's tile-relative offset of the whole frame (ts.input with
  // loop_tile_po, src/rdo.rs:2028-2033), and the distortion's, over the 8x8
  // blocks inside the tile (a block reaches at most 7 past the frame, into
  // the plane's padding)
  const int pw = p ? (g.W + xd) >> xd : g.W, ph = p ? (g.H + yd) >> yd : g.H;
  const int uw = min(BW, pw - ox), uh = min(BH, ph - oy);
  const int64_t ss_ = src.stride;
  const Px *const sp = (const Px *)src.data;
  const int elx = (min(8, max(0, (mi_cols - sx * 16 + 1) / 2)) * 8) >> xd;
  const int ely = (min(8, max(0, (mi_rows - sy * 16 + 1) / 2)) * 8) >> yd;
  {
    const Px *const ssolve = sp + (int64_t)(src.yorigin + oy) * ss_ + src.xorigin + ox;
    const Px *const sdist = sp + (int64_t)(src.yorigin + fy0 + oy) * ss_ + src.xorigin + fx0 + ox;
    for (int i = tid; i < npx; i += NT) {
      const int y = i >> LBW, x = i & (BW - 1);
      S.ssolve[i] = (x < uw && y < uh) ? (uint16_t)ssolve[(int64_t)y * ss_ + x] : 0;
      S.esrc[i] = (x < elx && y < ely) ? (uint16_t)sdist[(int64_t)y * ss_ + x] : 0;
    }
  }
  // 2. CDEF index 0 on the 8x8 blocks inside the tile (cdef_filter_superblock)
  PHASE(1);
  if (a.cdef) {
    if (tid < 64) {
      const int bx = tid & 7, by = tid >> 3, gx = sx * 16 + 2 * bx, gy = sy * 16 + 2 * by;
      uint8_t sk = 2, dir = 0;
      int32_t var = 0;
      if (gx < mi_cols && gy < mi_rows) {
        const uint8_t *k = a.skip + (int64_t)(t0y * 16 + gy) * a.mi_stride + t0x * 16 + gx;
        sk = k[0] & k[1] & k[a.mi_stride] & k[a.mi_stride + 1];
        if (!sk) {
          const int64_t o = (int64_t)(fsy * 8 + by) * a.dstride + fsx * 8 + bx;
          dir = a.dir[o];
          var = a.var[o];
        }
      }
      S.bskip[tid] = sk;
      S.bdir[tid] = dir;
      S.bvar[tid] = var;
    }
    __syncthreads();
    const int bxs = 8 >> xd, bys = 8 >> yd;
    for (int i = tid; i < npx; i += NT) {
      const int y = i >> LBW, x = i & (BW - 1), blk = (y / bys) * 8 + x / bxs;
      if (S.bskip[blk]) continue;  // skip: the copy (equal to lin); 2: outside the tile
      int pri, sec, dmp = a.damping + cs, d;
      if (p == 0) {
        pri = cdef_adjust(a.pri_y << cs, S.bvar[blk]);
        sec = a.sec_y << cs;
        d = a.pri_y ? S.bdir[blk] : 0;
      } else {
        pri = a.pri_uv << cs;
        sec = a.sec_uv << cs;
        dmp -= 1;
        d = a.pri_uv ? S.bdir[blk] : 0;
      }
      S.b.lin[i] = (uint16_t)cdef_px(S.pad + (y + 2) * (BW + 4) + x + 2, S.coffs + 6 * d, pri, sec, dmp, cs);
    }
  }
  __syncthreads();
  // 3. the unit's integral image: lrf_input alone, replicated
  PHASE(2);
  sgr_integral<SL::IS, SL::IR>(S.a.img, uw, uh, [&](int r, int c) -> uint32_t {
    return S.b.lin[iclamp(r - 4, 0, uh - 1) * BW + iclamp(c - 4, 0, uw - 1)];
  });
  // the lane's column strip (qx, qy0 .. qy0 + 3): its input pixels
  PHASE(3);
  const int qx = tid & (BW - 1), qy0 = (tid >> LBW) * 4;
  uint32_t pxr[4], lnr[4];  // the unit's pixels (0 outside it), lrf_input's
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int y = qy0 + k, i = y * BW + qx;
    lnr[k] = S.b.lin[i];
    pxr[k] = (qx < uw && y < uh) ? lnr[k] : 0;
  }
  __syncthreads();  // lin is read: the boxes take its place
  PHASE(4);
  const SgrLane ln = sgr_lane(uw, tid, NT);
  sgr_boxes<SL::IS, SL::IR, AS, A1R>(S.a.img, S.b.ps, ln, uh, cs);
  // 4. the distortion: rdo_loop_plane_error over the superblock's 8x8s in
  // the tile (cdef_dist_wxh_8x8 for luma, sse_wxh in the importance
  // block's parts for chroma), each weighted by its distortion bias
  const int wave = tid >> 6;
  const bool fin = wave == NW - 1;  // the last wave joins the parts
  const int fb = tid & 63, fgx = sx * 16 + 2 * (fb & 7), fgy = sy * 16 + 2 * (fb >> 3);
  const bool fblk = fin && fgx < mi_cols && fgy < mi_rows;  // lane fb of the last wave: block fb
  const double fbias = fblk ? lrf_bias(a.imp, a.w_imp, a.w_in_b, a.h_in_b, t0x * 16 + fgx, t0y * 16 + fgy) : 0.0;
  // 4:2:0 chroma: lane (qx, strip by) covers column qx of the 4x4 block
  // (qx / 4, by); the even lane of a pair adds up its two 2x2 parts
  const int cgx = sx * 16 + 2 * (qx >> 2), cgy = sy * 16 + 2 * (qy0 >> 2);
  const bool cblk = !WIDE && !(qx & 1) && cgx < mi_cols && cgy < mi_rows;
  const double cbias = cblk ? lrf_bias(a.imp, a.w_imp, a.w_in_b, a.h_in_b, t0x * 16 + cgx, t0y * 16 + cgy) : 0.0;
  if (WIDE && p == 0 && tid < 64) {  // luma blocks' source moments (every option reuses them)
    int32_t ss = 0;
    uint32_t ss2 = 0;
    for (int j = 0; j < 8; j++)
      for (int i = 0; i < 8; i++) {
        const int32_t v = S.esrc[(8 * (tid >> 3) + j) * BW + 8 * (tid & 7) + i];
        ss += v;
        ss2 += (uint32_t)(v * v);
      }
    S.bss[tid] = ss;
    S.bss2[tid] = ss2;
  }
  // an option's pixels d[4] (the lane's strip) -> its partial sums in LDS
  auto err_part = [&](const int32_t d[4]) {
    if (WIDE) {
      if (p == 0) {
        int32_t sd = 0;
        uint32_t sd2 = 0, ssd = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int32_t sv = S.esrc[(qy0 + k) * BW + qx];
          sd += d[k];
          sd2 += (uint32_t)(d[k] * d[k]);
          ssd += (uint32_t)(sv * d[k]);
        }
        sd = dpp_sum8(sd);
        sd2 = dpp_sum8(sd2);
        ssd = dpp_sum8(ssd);
        if ((qx & 7) == 0) S.hm[(qy0 >> 2) * 8 + (qx >> 3)] = make_uint3((uint32_t)sd, sd2, ssd);
      } else {  // 4:4:4 chroma: one 8x8 part per block
        uint32_t v = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int c = (int)(int16_t)S.esrc[(qy0 + k) * BW + qx] - (int)(int16_t)d[k];
          v += (uint32_t)(c * c);
        }
        v = dpp_sum8(v);
        if ((qx & 7) == 0) S.hm[(qy0 >> 2) * 8 + (qx >> 3)] = make_uint3(v, 0, 0);
      }
    } else {
      uint32_t top = 0, bot = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int c = (int)(int16_t)S.esrc[(qy0 + k) * BW + qx] - (int)(int16_t)d[k];
        if (k < 2)
          top += (uint32_t)(c * c);
        else
          bot += (uint32_t)(c * c);
      }
      top += dpp32<0xB1>(top);  // the lane pair (quad_perm [1,0,3,2])
      bot += dpp32<0xB1>(bot);
      uint64_t e = cblk ? biased(top, cbias) + biased(bot, cbias) : 0;
      e = dpp_sum64(e);
      if ((tid & 63) == 0) S.wsum[wave] = e;
    }
  };
  uint64_t *eo = a.err + ((size_t)p * g.nsb + sb) * 17;
  int8_t *xo = a.xqd + ((size_t)p * g.nsb + sb) * 32;
  // option o's distortion from the parts: the last wave, after the next
  // barrier (the parts are rewritten two barriers later)
  auto err_finish = [&](int o) {
    uint64_t e = 0;
    if (WIDE) {
      if (fblk) {
        const uint3 u0 = S.hm[(2 * (fb >> 3)) * 8 + (fb & 7)], u1 = S.hm[(2 * (fb >> 3) + 1) * 8 + (fb & 7)];
        e = p == 0 ? biased(cdef_dist(S.bss[fb], (int32_t)(u0.x + u1.x), S.bss2[fb], u0.y + u1.y, u0.z + u1.z, bd),
                            fbias)
                   : biased((uint64_t)u0.x + u1.x, fbias);
      }
      e = dpp_sum64(e);
    } else {
      for (int w = 0; w < NW; w++) e += S.wsum[w];
    }
    if (fb == 0) eo[o] = (uint64_t)((double)e * a.ds[p]);
  };
  {
    int32_t d[4];
#pragma unroll
    for (int k = 0; k < 4; k++) d[k] = (int32_t)lnr[k];  // None: the input as it is
    err_part(d);
  }
  // 5. the 16 sets: tables, solve sums, xqd, the filtered unit's
  // distortion; wave 0 solves set s while the other waves build set s + 1's
  // tables (the f values of s are in registers by then)
  using Acc = typename std::conditional<sizeof(Px) == 1, int32_t, int64_t>::type;  // 8-bit: 4 products fit
  const SgrLane ln_rest = sgr_lane(uw, tid - 64, NT - 64);
  __syncthreads();  // the boxes and the None parts
  if (fin) err_finish(0);
  sgr_tables_ps<AS, A1R>(S.b.ps, S.a.tab, S.xz, ln, 0, uh);
  PHASE(5);
  for (int set = 0; set < 16; set++) {
    __syncthreads();
    PHASE(6 + 5 * set);
    if (set > 0 && fin) err_finish(set);  // set - 1's, at eo[set]
    uint32_t f2r[4] = {0, 0, 0, 0}, f1r[4] = {0, 0, 0, 0};
    Acc H00 = 0, H11 = 0, H01 = 0, C0 = 0, C1 = 0;
    if (qx < uw) {
      sgr_f4<AS, A1R>(S.a.tab, set, qx, qy0, pxr, f2r, f1r);
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (qy0 + k < uh) {
          const Acc u = (Acc)pxr[k] << kRstBits;
          const Acc sv = ((Acc)S.ssolve[(qy0 + k) * BW + qx] << kRstBits) - u;
          const Acc e2 = (Acc)(int32_t)f2r[k] - u, e1 = (Acc)(int32_t)f1r[k] - u;
          H00 += e2 * e2;
          H11 += e1 * e1;
          H01 += e1 * e2;
          C0 += e2 * sv;
          C1 += e1 * sv;
        }
    }
    {
      const int64_t v[5] = {H00, H11, H01, C0, C1};
#pragma unroll
      for (int q = 0; q < 5; q++) {
        const int64_t t = (int64_t)dpp_sum64((uint64_t)v[q]);
        if ((tid & 63) == 0) S.red5[q][wave] = t;
      }
    }
    __syncthreads();
    PHASE(7 + 5 * set);
    if (wave == 0) {  // the solve (lanes 0 .. 4 add up one sum each)
      int64_t t = 0;
      if (tid < 5)
        for (int w = 0; w < NW; w++) t += S.red5[tid][w];
      const int64_t h00 = readlane64((uint64_t)t, 0), h11 = readlane64((uint64_t)t, 1),
                    h01 = readlane64((uint64_t)t, 2), c0 = readlane64((uint64_t)t, 3),
                    c1 = readlane64((uint64_t)t, 4);
      int8_t q[2];
      lrf_solve_finish_wave(set, uw, uh, h00, h01, h11, c0, c1, q);
      if (tid == 0) {
        S.sxqd[0] = q[0];
        S.sxqd[1] = q[1];
        xo[2 * set] = q[0];
        xo[2 * set + 1] = q[1];
      }
    } else if (set < 15) {
      sgr_tables_ps<AS, A1R>(S.b.ps, S.a.tab, S.xz, ln_rest, set + 1, uh);
    }
    __syncthreads();
    PHASE(8 + 5 * set);
    const int w0 = S.sxqd[0], w1 = S.sxqd[1];
    int32_t d[4];
#pragma unroll
    for (int k = 0; k < 4; k++)  // 128 outside the unit: lrf_output's fill (never inside the frame)
      d[k] = (qx < uw && qy0 + k < uh) ? sgr_out(f2r[k], f1r[k], pxr[k], w0, w1, mx) : 128;
    err_part(d);
    PHASE(9 + 5 * set);
    PHASE(10 + 5 * set);
  }
  __syncthreads();
  if (fin) err_finish(16);
}

// 64 x 64 units (luma, 4:4:4 chroma) in 512-lane workgroups with ~71 KB of
// LDS, two per CU: a lane owns two column strips (rows y0 .. y0 + 3 and
// y0 + 32 .. y0 + 35), the source pixels it needs sit in its registers, and
// each set's (a, b) tables are built from the integral images (which stay)
// into packed words. Otherwise as lrf_rdo_kernel.
// Region `raw` by phase (word offsets): the integral images at 0 and the
// unit's input + padded copy after them; then, 8-bit, the packed tables at
// 0 and the boxes' p (u32) and sum (u16) after them, over the images (the
// boxes go through registers); 10/12-bit (a box sum can exceed 16 bits), the
// images stay and the tables sit after them, over the input.
template <bool PS>
struct RdoWideMap {
  using L = SgrL64;
  static constexpr int IMG = 0, IMGW = 2 * L::IR * L::IS;
  static constexpr int LIN = IMGW, PAD = LIN + 64 * 64 / 2;  // u16 pairs
  static constexpr int INW = PAD + 68 * 68 / 2;
  static constexpr int TAB = PS ? 0 : IMGW, PP = L::TAB, P16 = 2 * L::TAB;
  static constexpr int TABW = PS ? 2 * L::TAB + (L::TAB + 1) / 2 : IMGW + L::TAB;
  static constexpr int WORDS = TABW > INW ? TABW : INW;
};
template <bool PS>
struct RdoWideLds {
  uint32_t raw[RdoWideMap<PS>::WORDS];
  uint16_t xz[256];
  int16_t coffs[48];
  uint8_t bdir[64], bskip[64];
  int32_t bvar[64];
  int64_t red5[5][8];
  uint3 hm[16 * 8];  // each half block's (sd, sd2, ssd) / (sse), [strip][block column]
  int2 bsh[16 * 8];  // luma: each half block's source (sum, sum of squares)
  int8_t sxqd[2];
};

// each set's tables from the boxes' p and sum (the same places)
template <int AS, int A1R>
__device__ __forceinline__ void sgr_tables_pp(const uint32_t *pp, const uint16_t *p16, uint32_t *tab,
                                              const uint16_t *xz, const SgrLane &ln, int set, int h) {
  const uint32_t s2 = kSgrS[set][0], s1 = kSgrS[set][1];
  const int r1rows = s1 ? h + 2 : 0, r2rows = s2 ? (h + 1) / 2 + 1 : 0;
#pragma unroll 2
  for (int r = ln.ty; r < r1rows + r2rows; r += ln.tstep) {
    const bool one = r < r1rows;
    const int to = (one ? r : A1R + r - r1rows) * AS + ln.tx;
    tab_put(tab[to], sgr_ab(make_uint2(pp[to], p16[to]), one ? s1 : s2, one ? 455 : 164, xz));
  }
}

template <typename Px>
__global__ __launch_bounds__(512, 4) void lrf_rdo_wide_kernel(LrfRdoArgs a) {
  using SL = SgrL64;
  constexpr int BW = 64, BH = 64, NT = 512, NW = 8, AS = SL::AS, A1R = SL::A1R;
  constexpr bool PS = sizeof(Px) == 1;  // 8-bit: the boxes' p and sum kept (see RdoWideMap)
  using M = RdoWideMap<PS>;
  __shared__ RdoWideLds<PS> S;
  uint32_t *const img = S.raw + M::IMG, *const tab = S.raw + M::TAB;
  uint16_t *const lin = (uint16_t *)(S.raw + M::LIN), *const pad = (uint16_t *)(S.raw + M::PAD);
  const LrfGeo &g = a.g;
  const int p = a.p0 + blockIdx.y, sb = blockIdx.x, tid = threadIdx.x;
  const int sbc = g.sbc, fsx = sb % sbc, fsy = sb / sbc;
  if (fsx >= g.cols[p] || fsy >= g.rows[p]) return;  // no unit (uniform)
  if (fsx < a.gx0 || fsx >= a.gx1 || fsy < a.gy0 || fsy >= a.gy1) return;  // another group's
  const int t0x = fsx - fsx % g.tws, t0y = fsy - fsy % g.ths, sx = fsx - t0x, sy = fsy - t0y;
  const int xd = p ? g.xdec : 0, yd = p ? g.ydec : 0;
  const int tw_px = min(g.tws * 64, g.W - t0x * 64), th_px = min(g.ths * 64, g.H - t0y * 64);
  const int pw_t = (tw_px + xd) >> xd, ph_t = (th_px + yd) >> yd;
  const int mi_cols = tw_px >> 2, mi_rows = th_px >> 2;
  const int ox = (sx * 64) >> xd, oy = (sy * 64) >> yd, fx0 = (t0x * 64) >> xd, fy0 = (t0y * 64) >> yd;
  const int bd = g.bd, cs = bd - 8, mx = (1 << bd) - 1;
  const rv_plane &rec = a.rec[p], &src = a.src[p];
  auto recpx = [&](int x, int y) __attribute__((always_inline)) -> int {  // frame plane coordinates
    return (int)((const Px *)rec.data)[(int64_t)(rec.yorigin + y) * rec.stride + rec.xorigin + x];
  };
  PHASE(0);
  sgr_init_xz(S.xz);
  cdef_offsets(S.coffs, BW + 4);
  // 1. the padded copy and the unit's input
  for (int i = tid; i < (BH + 4) * (BW + 4); i += NT) {
    const int y = i / (BW + 4) - 2, x = i % (BW + 4) - 2, tx = ox + x, ty = oy + y;
    int v = kVeryLarge;
    if (tx >= 0 && tx < pw_t && ty >= 0 && ty < ph_t) {
      const int csx = (tx << xd) >> 6, csy = (ty << yd) >> 6;
      v = (csy < sy || (csy == sy && csx <= sx)) ? recpx(fx0 + tx, fy0 + ty) : 128;
    }
    pad[i] = (uint16_t)v;
  }
  const int vw = min(BW, pw_t - ox), vh = min(BH, ph_t - oy);
  for (int i = tid; i < BW * BH; i += NT) {
    const int y = i >> 6, x = i & 63;
    lin[i] = (uint16_t)recpx(fx0 + ox + min(x, vw - 1), fy0 + oy + min(y, vh - 1));
  }
  // the unit (size clipped at the tile-relative offset, the reference's
  // quirk) and the lane's source pixels: sgrproj_solve's at the unit's
  // tile-relative offset of the whole frame (src/rdo.rs:2028-2033), the
  // distortion's over the 8x8 blocks inside the tile (two u16 per word)
  const int pw = p ? (g.W + xd) >> xd : g.W, ph = p ? (g.H + yd) >> yd : g.H;
  const int uw = min(BW, pw - ox), uh = min(BH, ph - oy);
  const int elx = (min(8, max(0, (mi_cols - sx * 16 + 1) / 2)) * 8) >> xd;
  const int ely = (min(8, max(0, (mi_rows - sy * 16 + 1) / 2)) * 8) >> yd;
  const int qx = tid & 63, qy0 = (tid >> 6) * 4;  // strips (qx, qy0 + 32 j + k)
  uint32_t ssw[4], esw[4];
  {
    const int64_t ss_ = src.stride;
    const Px *const sp = (const Px *)src.data;
    const Px *const ssolve = sp + (int64_t)(src.yorigin + oy) * ss_ + src.xorigin + ox;
    const Px *const sdist = sp + (int64_t)(src.yorigin + fy0 + oy) * ss_ + src.xorigin + fx0 + ox;
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      uint32_t sv[2], ev[2];
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int y = qy0 + 32 * ((j + h) >> 2) + ((j + h) & 3);
        sv[h] = (qx < uw && y < uh) ? (uint32_t)ssolve[(int64_t)y * ss_ + qx] : 0;
        ev[h] = (qx < elx && y < ely) ? (uint32_t)sdist[(int64_t)y * ss_ + qx] : 0;
      }
      ssw[j >> 1] = sv[0] | sv[1] << 16;
      esw[j >> 1] = ev[0] | ev[1] << 16;
    }
  }
  auto srcv = [&](const uint32_t *w, int i) __attribute__((always_inline)) -> int32_t {  // pixel i (0 .. 7) of the lane's strips
    return (int32_t)((w[i >> 1] >> (16 * (i & 1))) & 0xffff);
  };
  // 2. CDEF index 0 on the 8x8 blocks inside the tile (cdef_filter_superblock)
  PHASE(1);
  if (a.cdef) {
    if (tid < 64) {
      const int bx = tid & 7, by = tid >> 3, gx = sx * 16 + 2 * bx, gy = sy * 16 + 2 * by;
      uint8_t sk = 2, dir = 0;
      int32_t var = 0;
      if (gx < mi_cols && gy < mi_rows) {
        const uint8_t *k = a.skip + (int64_t)(t0y * 16 + gy) * a.mi_stride + t0x * 16 + gx;
        sk = k[0] & k[1] & k[a.mi_stride] & k[a.mi_stride + 1];
        if (!sk) {
          const int64_t o = (int64_t)(fsy * 8 + by) * a.dstride + fsx * 8 + bx;
          dir = a.dir[o];
          var = a.var[o];
        }
      }
      S.bskip[tid] = sk;
      S.bdir[tid] = dir;
      S.bvar[tid] = var;
    }
    __syncthreads();
    const int bxs = 8 >> xd, bys = 8 >> yd;
    for (int i = tid; i < BW * BH; i += NT) {
      const int y = i >> 6, x = i & 63, blk = (y / bys) * 8 + x / bxs;
      if (S.bskip[blk]) continue;  // skip: the copy (equal to lin); 2: outside the tile
      int pri, sec, dmp = a.damping + cs, d;
      if (p == 0) {
        pri = cdef_adjust(a.pri_y << cs, S.bvar[blk]);
        sec = a.sec_y << cs;
        d = a.pri_y ? S.bdir[blk] : 0;
      } else {
        pri = a.pri_uv << cs;
        sec = a.sec_uv << cs;
        dmp -= 1;
        d = a.pri_uv ? S.bdir[blk] : 0;
      }
      lin[i] = (uint16_t)cdef_px(pad + (y + 2) * (BW + 4) + x + 2, S.coffs + 6 * d, pri, sec, dmp, cs);
    }
  }
  __syncthreads();
  // 3. the unit's integral image: lrf_input alone, replicated
  PHASE(2);
  sgr_integral<SL::IS, SL::IR>(img, uw, uh, [&](int r, int c) -> uint32_t {
    return lin[iclamp(r - 4, 0, uh - 1) * BW + iclamp(c - 4, 0, uw - 1)];
  });
  PHASE(3);
  uint32_t pxr[8], lnr[8];  // the unit's pixels (0 outside it), lrf_input's
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int y = qy0 + 32 * (i >> 2) + (i & 3);
    lnr[i] = lin[y * BW + qx];
    pxr[i] = (qx < uw && y < uh) ? lnr[i] : 0;
  }
  // 4. the distortion (as lrf_rdo_kernel): half blocks over 8 lanes, the
  // last wave joins them
  const int wave = tid >> 6;
  const bool fin = wave == NW - 1;
  const int fb = tid & 63, fgx = sx * 16 + 2 * (fb & 7), fgy = sy * 16 + 2 * (fb >> 3);
  const bool fblk = fin && fgx < mi_cols && fgy < mi_rows;
  const double fbias = fblk ? lrf_bias(a.imp, a.w_imp, a.w_in_b, a.h_in_b, t0x * 16 + fgx, t0y * 16 + fgy) : 0.0;
  if (p == 0) {  // the luma half blocks' source moments (every option reuses them)
#pragma unroll
    for (int j = 0; j < 2; j++) {
      int32_t ss = 0;
      uint32_t ss2 = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int32_t v = srcv(esw, 4 * j + k);
        ss += v;
        ss2 += (uint32_t)(v * v);
      }
      ss = dpp_sum8(ss);
      ss2 = dpp_sum8(ss2);
      if ((qx & 7) == 0) S.bsh[((qy0 >> 2) + 8 * j) * 8 + (qx >> 3)] = make_int2(ss, (int32_t)ss2);
    }
  }
  auto err_part = [&](const int32_t d[8]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; j++) {
      const int slot = ((qy0 >> 2) + 8 * j) * 8 + (qx >> 3);
      if (p == 0) {
        int32_t sd = 0;
        uint32_t sd2 = 0, ssd = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int32_t dv = d[4 * j + k], sv = srcv(esw, 4 * j + k);
          sd += dv;
          sd2 += (uint32_t)(dv * dv);
          ssd += (uint32_t)(sv * dv);
        }
        sd = dpp_sum8(sd);
        sd2 = dpp_sum8(sd2);
        ssd = dpp_sum8(ssd);
        if ((qx & 7) == 0) S.hm[slot] = make_uint3((uint32_t)sd, sd2, ssd);
      } else {  // 4:4:4 chroma: one 8x8 part per block
        uint32_t v = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int c = (int)(int16_t)srcv(esw, 4 * j + k) - (int)(int16_t)d[4 * j + k];
          v += (uint32_t)(c * c);
        }
        v = dpp_sum8(v);
        if ((qx & 7) == 0) S.hm[slot] = make_uint3(v, 0, 0);
      }
    }
  };
  uint64_t *eo = a.err + ((size_t)p * g.nsb + sb) * 17;
  int8_t *xo = a.xqd + ((size_t)p * g.nsb + sb) * 32;
  auto err_finish = [&](int o) __attribute__((always_inline)) {
    uint64_t e = 0;
    if (fblk) {
      const int h0 = (2 * (fb >> 3)) * 8 + (fb & 7), h1 = h0 + 8;
      const uint3 u0 = S.hm[h0], u1 = S.hm[h1];
      if (p == 0) {
        const int2 s0 = S.bsh[h0], s1 = S.bsh[h1];
        e = biased(cdef_dist(s0.x + s1.x, (int32_t)(u0.x + u1.x), (uint32_t)s0.y + (uint32_t)s1.y, u0.y + u1.y,
                             u0.z + u1.z, bd),
                   fbias);
      } else {
        e = biased((uint64_t)u0.x + u1.x, fbias);
      }
    }
    e = dpp_sum64(e);
    if (fb == 0) eo[o] = (uint64_t)((double)e * a.ds[p]);
  };
  {
    int32_t d[8];
#pragma unroll
    for (int i = 0; i < 8; i++) d[i] = (int32_t)lnr[i];  // None: the input as it is
    err_part(d);
  }
  // 5. the 16 sets (wave 0 solves set s while the others build s + 1's tables)
  using Acc = typename std::conditional<sizeof(Px) == 1, int32_t, int64_t>::type;  // 8-bit: 8 products fit
  const SgrLane ln = sgr_lane(uw, tid, NT), ln_rest = sgr_lane(uw, tid - 64, NT - 64);
  uint32_t *const pp = S.raw + M::PP;
  uint16_t *const p16 = (uint16_t *)(S.raw + M::P16);
  if (PS) {  // the boxes' p and sum, through registers (they land on the images)
    constexpr int KMAX = (SL::A1R + SL::A2R + NT / SL::AS - 1) / (NT / SL::AS) + 1;
    uint32_t bp[KMAX], bs[KMAX];
    const int r1rows = uh + 2, r2rows = (uh + 1) / 2 + 1;
#pragma unroll
    for (int k = 0; k < KMAX; k++) {
      const int r = ln.ty + k * ln.tstep;
      bp[k] = bs[k] = 0;
      if (r < r1rows + r2rows) {
        int to, o, dd;
        sgr_row<SL::IS, AS, A1R>(r, r1rows, ln.tx, to, o, dd);
        const uint2 v = sgr_box(isq(img, SL::IS, SL::IR * SL::IS + o, dd), isq(img, SL::IS, o, dd),
                                r < r1rows ? 9 : 25, cs);
        bp[k] = v.x;
        bs[k] = v.y;
      }
    }
    __syncthreads();  // the images and lin are read
#pragma unroll
    for (int k = 0; k < KMAX; k++) {
      const int r = ln.ty + k * ln.tstep;
      if (r < r1rows + r2rows) {
        const int to = (r < r1rows ? r : A1R + r - r1rows) * AS + ln.tx;
        pp[to] = bp[k];
        p16[to] = (uint16_t)bs[k];  // <= 25 x 255
      }
    }
  }
  __syncthreads();  // lin is read (the tables take its place); the None parts; the boxes
  PHASE(4);
  if (fin) err_finish(0);
  if (PS)
    sgr_tables_pp<AS, A1R>(pp, p16, tab, S.xz, ln, 0, uh);
  else
    sgr_tables<SL::IS, SL::IR, AS, A1R>(img, tab, S.xz, ln, 0, uh, cs);
  PHASE(5);
  for (int set = 0; set < 16; set++) {
    __syncthreads();
    PHASE(6 + 5 * set);
    if (set > 0 && fin) err_finish(set);  // set - 1's, at eo[set]
    uint32_t f2r[8], f1r[8];
    Acc H00 = 0, H11 = 0, H01 = 0, C0 = 0, C1 = 0;
#pragma unroll
    for (int j = 0; j < 2; j++) {
      sgr_f4<AS, A1R>(tab, set, qx, qy0 + 32 * j, pxr + 4 * j, f2r + 4 * j, f1r + 4 * j);
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (qx < uw && qy0 + 32 * j + k < uh) {
          const int i = 4 * j + k;
          const Acc u = (Acc)pxr[i] << kRstBits;
          const Acc sv = ((Acc)srcv(ssw, i) << kRstBits) - u;
          const Acc e2 = (Acc)(int32_t)f2r[i] - u, e1 = (Acc)(int32_t)f1r[i] - u;
          H00 += e2 * e2;
          H11 += e1 * e1;
          H01 += e1 * e2;
          C0 += e2 * sv;
          C1 += e1 * sv;
        }
    }
    {
      const int64_t v[5] = {H00, H11, H01, C0, C1};
#pragma unroll
      for (int q = 0; q < 5; q++) {
        const int64_t t = (int64_t)dpp_sum64((uint64_t)v[q]);
        if ((tid & 63) == 0) S.red5[q][wave] = t;
      }
    }
    __syncthreads();
    PHASE(7 + 5 * set);
    if (wave == 0) {
      int64_t t = 0;
      if (tid < 5)
        for (int w = 0; w < NW; w++) t += S.red5[tid][w];
      const int64_t h00 = readlane64((uint64_t)t, 0), h11 = readlane64((uint64_t)t, 1),
                    h01 = readlane64((uint64_t)t, 2), c0 = readlane64((uint64_t)t, 3),
                    c1 = readlane64((uint64_t)t, 4);
      int8_t q[2];
      lrf_solve_finish_wave(set, uw, uh, h00, h01, h11, c0, c1, q);
      if (tid == 0) {
        S.sxqd[0] = q[0];
        S.sxqd[1] = q[1];
        xo[2 * set] = q[0];
        xo[2 * set + 1] = q[1];
      }
    } else if (set < 15) {
      if (PS)
        sgr_tables_pp<AS, A1R>(pp, p16, tab, S.xz, ln_rest, set + 1, uh);
      else
        sgr_tables<SL::IS, SL::IR, AS, A1R>(img, tab, S.xz, ln_rest, set + 1, uh, cs);
    }
    __syncthreads();
    PHASE(8 + 5 * set);
    const int w0 = S.sxqd[0], w1 = S.sxqd[1];
    int32_t d[8];
#pragma unroll
    for (int i = 0; i < 8; i++)  // 128 outside the unit: lrf_output's fill (never inside the frame)
      d[i] = (qx < uw && qy0 + 32 * (i >> 2) + (i & 3) < uh) ? sgr_out(f2r[i], f1r[i], pxr[i], w0, w1, mx) : 128;
    err_part(d);
    PHASE(9 + 5 * set);
    PHASE(10 + 5 * set);
  }
  __syncthreads();
  if (fin) err_finish(16);
}

// ---- the sequential decisions (count_lrf_switchable, write_lrf) -----------------
struct LrfDecideArgs {
  LrfGeo g;
  int gx0, gy0, gx1, gy1;  // the superblocks decided here (whole tiles)
  const uint64_t *err;
  const int8_t *xqd;
  double lambda;
  int8_t *units;  // [3][rows][cols][3]: set (-1 None), xqd0, xqd1
  int fix_passes;  // lrf_decide_fix_kernel: parallel passes before the serial rest
};

// (key, set) lexicographic minimum with the lane DPP control CTRL reads
template <int CTRL>
__device__ __forceinline__ void dpp_min_step(uint64_t &bk, int &bs) {
  const uint64_t ok = dpp64<CTRL>(bk);
  const int os = (int)dpp32<CTRL>((uint32_t)bs);
  if (ok < bk || (ok == bk && os < bs)) {
    bk = ok;
    bs = os;
  }
}

// One wave per tile: lane 16 p + s prices set s of plane p, lane 48 + p
// plane p's None, at the tile's current state; a (cost, set) minimum over
// each 16-lane group on the DPP network, then None (first in the reference's order:
// it wins ties) picks the first cheapest, and every lane applies the same
// write_lrf updates (the state stays uniform). No LDS and no barrier: the
// next superblock's distortions load while this one is decided.
#ifdef LRF_PHASES
__device__ unsigned long long lrf_dphase[5];
#endif
// count_signed_subexp_with_ref of each (xqd, ref) pair, per radius (bits *
// 8; uploaded once by lrf_lut_upload)
__device__ uint8_t g_lrf_subexp[2][128][128];
constexpr int kDecideAhead = 8;        // superblocks of distortions in flight
constexpr int kDecideBuf = 4096;        // superblocks whose picks wait in LDS

__global__ __launch_bounds__(64) void lrf_decide_kernel(LrfDecideArgs a) {
  __shared__ int8_t ubuf[kDecideBuf][3][3];
  __shared__ uint8_t slut[2][128][128];  // g_lrf_subexp
  __shared__ uint16_t sbl[2][520];       // symbol_bits of None / Sgrproj by cdf[0] / cdf[1] >> 6
  const LrfGeo &g = a.g;
  const int ntx = (g.sbc + g.tws - 1) / g.tws;
  const int t = blockIdx.x, lane = threadIdx.x;
  const int t0x = (t % ntx) * g.tws, t0y = (t / ntx) * g.ths;
  if (t0x < a.gx0 || t0x >= a.gx1 || t0y < a.gy0 || t0y >= a.gy1) return;  // another group's tile
  const int tsw = min(g.tws, g.sbc - t0x), tsh = min(g.ths, g.sbr - t0y), n = tsw * tsh;
  const bool none = lane >= 48, live = lane < 51;
  const int lp = none ? lane - 48 : lane >> 4, ls = none ? -1 : lane & 15;  // plane, set (-1: None)
  const bool buffered = n <= kDecideBuf;
  {
    const uint4 *gl = (const uint4 *)&g_lrf_subexp[0][0][0];
    uint4 *sl = (uint4 *)&slut[0][0][0];
    for (int i = lane; i < 2 * 128 * 128 / 16; i += 64) sl[i] = gl[i];
    for (int f = lane; f < 520; f += 64) {
      const uint16_t c0[4] = {(uint16_t)(f << 6), 0, 0, 0}, c1[4] = {0, (uint16_t)(f << 6), 0, 0};
      sbl[0][f] = (uint16_t)lrf_symbol_bits(0, c0, 3);
      sbl[1][f] = (uint16_t)lrf_symbol_bits(2, c1, 3);
    }
    __syncthreads();
  }
  LrfTileState st;
  lrf_tile_init(st);
#ifdef LRF_PHASES  // cycles per part of a step, summed over the tile (s_memtime)
  unsigned long long dacc[5] = {0, 0, 0, 0, 0}, dlast = clock64();
#define DPHASE(i)                             \
  {                                           \
    const unsigned long long now = clock64(); \
    dacc[i] += now - dlast;                   \
    dlast = now;                              \
  }
#else
#define DPHASE(i)
#endif
  // superblock k = (kx, ky): unconditional loads (indices clamped; the
  // dead lanes' and None's xqd are never used) kept raw until their step,
  // so the wait for them is the only one
  const int lpc = lp < 3 ? lp : 2, lsc = ls > 0 ? ls : 0;
  auto load = [&](int k, int kx, int ky, uint64_t &e, uint32_t &xq) {
    if (k >= n) kx = ky = 0;
    const size_t u = (size_t)lpc * g.nsb + (t0y + ky) * g.sbc + t0x + kx;
    e = a.err[u * 17 + 1 + ls];
    xq = *(const uint32_t *)(a.xqd + u * 32 + 4 * (lsc >> 1));  // an aligned word: two pairs
  };
  uint64_t ev[kDecideAhead];
  uint32_t xv[kDecideAhead];
#pragma unroll
  for (int d = 0; d < kDecideAhead; d++) load(d, d % tsw, d / tsw, ev[d], xv[d]);
  int sx = 0, sy = 0;                                            // the superblock in the tile
  int lx = kDecideAhead % tsw, ly = kDecideAhead / tsw;          // the next one to load
  for (int k0 = 0; k0 < n; k0 += kDecideAhead) {
#pragma unroll
    for (int d = 0; d < kDecideAhead; d++) {
      const int k = k0 + d;
      if (k >= n) break;
      const int fsx = t0x + sx, fsy = t0y + sy;
      DPHASE(0);
      const uint32_t xw = (lsc & 1) ? xv[d] >> 16 : xv[d];
      const int x0 = none ? 0 : (int)(int8_t)(xw & 0xff), x1 = none ? 0 : (int)(int8_t)((xw >> 8) & 0xff);
      const int r0 = lp == 0 ? st.ref[0][0] : lp == 1 ? st.ref[1][0] : st.ref[2][0];
      const int r1 = lp == 0 ? st.ref[0][1] : lp == 1 ? st.ref[1][1] : st.ref[2][1];
      // count_lrf_switchable (lrf_rate_at) from the tables
      uint32_t bits;
      if (none) {
        bits = sbl[0][st.cdf[0] >> 6];
      } else {
        bits = sbl[1][st.cdf[1] >> 6] + (4u << 3);
        if (lrf_set_has(ls, 0)) bits += slut[0][x0 + 96][r0 + 96];
        if (lrf_set_has(ls, 1)) bits += slut[1][x1 + 32][r1 + 32];
      }
      const double c = (double)ev[d] + a.lambda * ((double)bits / 8.0);
      // costs are >= 0: their bit patterns order like the values
      const uint64_t key = live ? (uint64_t)__double_as_longlong(c) : ~0ull;
      DPHASE(1);
      uint64_t bk = key;
      int bs = ls;
      // the first cheapest set of each 16 lanes: quad pairs, quads, halves
      // (any pairing reaches all 16 for a minimum)
      dpp_min_step<0xB1>(bk, bs);
      dpp_min_step<0x4E>(bk, bs);
      dpp_min_step<0x141>(bk, bs);
      dpp_min_step<0x140>(bk, bs);
      // lanes 0 .. 2, plane p = lane: its best set (lane 16 p) against its
      // None (lane 48 + p), its xqd, packed; then uniform by lane reads
      int packed;
      {
        const int pl = lane < 3 ? lane : 0;
        auto shfl64 = [](uint64_t v, int l) {
          return (uint64_t)(uint32_t)__shfl((int)(uint32_t)(v >> 32), l, 64) << 32 |
                 (uint32_t)__shfl((int)(uint32_t)v, l, 64);
        };
        const uint64_t sk = shfl64(bk, 16 * pl), nk = shfl64(key, 48 + pl);
        const int sbest = __shfl(bs, 16 * pl, 64);
        const int best = nk <= sk ? -1 : sbest;
        const int src = 16 * pl + (best < 0 ? 0 : best);
        const int q0 = __shfl(x0, src, 64), q1 = __shfl(x1, src, 64);
        // a stretched superblock has no unit of its own
        const int cols = pl == 0 ? g.cols[0] : pl == 1 ? g.cols[1] : g.cols[2];
        const int rows = pl == 0 ? g.rows[0] : pl == 1 ? g.rows[1] : g.rows[2];
        const bool has = fsx < cols && fsy < rows;
        packed = has ? (best & 0xff) | (best >= 0 ? (q0 & 0xff) << 8 | (q1 & 0xff) << 16 : 0) : 0xfe;
      }
      int pick[3][3];
#pragma unroll
      for (int p = 0; p < 3; p++) {
        const int v = __builtin_amdgcn_readlane(packed, p);
        pick[p][0] = (int8_t)(v & 0xff);
        pick[p][1] = (int8_t)((v >> 8) & 0xff);
        pick[p][2] = (int8_t)((v >> 16) & 0xff);
      }
      DPHASE(2);
      load(k + kDecideAhead, lx, ly, ev[d], xv[d]);  // this slot's next superblock
      if (++lx == tsw) {
        lx = 0;
        ly++;
      }
      if (lane < 9) {  // the picks wait in LDS (a store would hold up the loads' counter)
        const int p = lane / 3, j = lane % 3;
        const int v = p == 0 ? (j == 0 ? pick[0][0] : j == 1 ? pick[0][1] : pick[0][2])
                    : p == 1 ? (j == 0 ? pick[1][0] : j == 1 ? pick[1][1] : pick[1][2])
                             : (j == 0 ? pick[2][0] : j == 1 ? pick[2][1] : pick[2][2]);
        const int8_t b = (int8_t)(j == 0 && v < 0 ? -1 : v);
        if (buffered)
          ubuf[k][p][j] = b;
        else
          a.units[(((size_t)p * g.urows_max + fsy) * g.ucols_max + fsx) * 3 + j] = b;
      }
      DPHASE(3);
#pragma unroll
      for (int p = 0; p < 3; p++)
        if (pick[p][0] > -2) {
          const int8_t q[2] = {(int8_t)pick[p][1], (int8_t)pick[p][2]};
          lrf_commit(st, p, pick[p][0], q);
        }
      DPHASE(4);
      if (++sx == tsw) {
        sx = 0;
        sy++;
      }
    }
  }
#ifdef LRF_PHASES
  if (lane == 0 && t == 0)
    for (int i = 0; i < 5; i++) lrf_dphase[i] = dacc[i];
#endif
  if (buffered) {
    __syncthreads();
    for (int i = lane; i < n * 9; i += 64) {
      const int k = i / 9, p = (i / 3) % 3, j = i % 3;
      const int fsx = t0x + k % tsw, fsy = t0y + k / tsw;
      a.units[(((size_t)p * g.urows_max + fsy) * g.ucols_max + fsx) * 3 + j] = ubuf[k][p][j];
    }
  }
}

// The same decisions by a fixed point (tiles of at most kFixMax superblocks):
// the tile's restoration state before each superblock -- the CDF and each
// plane's sgrproj_ref -- is a cheap serial function of the decisions before
// it, and each decision a parallel function of its state. Guess every state
// (the initial one), decide every (superblock, plane) in parallel, run the
// states from the first decision that changed, repeat. Decisions before the
// first change are final (their states are), so an iteration settles at
// least one more superblock, and the fixed point is the sequential result;
// after kFixIter iterations the rest is decided in order.
constexpr int kFixMax = 1024, kFixIter = 12, kFixThreads = 1024;
#ifdef LRF_PHASES
__device__ int lrf_fix_stats[8], lrf_fix_iters[8], lrf_fix_trace[8][kFixIter];
__device__ unsigned long long lrf_fix_clk[40];
#define FIXCLK(i) \
  if (tid == 0 && t == 0) lrf_fix_clk[i] = wall_clock64()
#else
#define FIXCLK(i)
#endif
struct FixState {
  uint16_t c0, c1, c3;  // lrf_switchable_cdf[0], [1] and its counter
  int8_t ref[3][2];
};
__device__ __forceinline__ void fix_load(LrfTileState &st, const FixState &f) {
  st.cdf[0] = f.c0;
  st.cdf[1] = f.c1;
  st.cdf[2] = 0;
  st.cdf[3] = f.c3;
  for (int p = 0; p < 3; p++)
    for (int i = 0; i < 2; i++) st.ref[p][i] = f.ref[p][i];
}
__device__ __forceinline__ void fix_store(FixState &f, const LrfTileState &st) {
  f.c0 = st.cdf[0];
  f.c1 = st.cdf[1];
  f.c3 = st.cdf[3];
  for (int p = 0; p < 3; p++)
    for (int i = 0; i < 2; i++) f.ref[p][i] = st.ref[p][i];
}
// one unit's choice at a state: None, then the 16 sets, the first cheapest
// (the costs of lrf_decide_kernel's lanes, in the reference's order);
// packed as set | xqd0 << 8 | xqd1 << 16 (set -1: None)
// (the unit's 17 distortions and 16 xqd pairs in registers: ev, xw)
struct FixUnit {
  uint64_t ev[17];
  uint32_t xw[8];
};
__device__ __forceinline__ void fix_load_unit(FixUnit &fu, const uint64_t *e, const int8_t *xq) {
#pragma unroll
  for (int s = 0; s < 17; s++) fu.ev[s] = e[s];
#pragma unroll
  for (int w = 0; w < 8; w++) fu.xw[w] = ((const uint32_t *)xq)[w];
}
__device__ __forceinline__ int fix_decide(const FixUnit &fu, const FixState &f, int p, double lambda,
                                          const uint8_t (*slut)[128][128], const uint16_t (*sbl)[520]) {
  int best = -1, bx0 = 0, bx1 = 0;
  double bc = (double)fu.ev[0] + lambda * ((double)sbl[0][f.c0 >> 6] / 8.0);
  const uint32_t base = sbl[1][f.c1 >> 6] + (4u << 3);
  const int r0 = f.ref[p][0], r1 = f.ref[p][1];
#pragma unroll
  for (int s = 0; s < 16; s++) {
    const uint32_t pr = (fu.xw[s >> 1] >> (16 * (s & 1))) & 0xffff;
    const int x0 = (int)(int8_t)(pr & 0xff), x1 = (int)(int8_t)(pr >> 8);
    uint32_t bits = base;
    if (lrf_set_has(s, 0)) bits += slut[0][x0 + 96][r0 + 96];
    if (lrf_set_has(s, 1)) bits += slut[1][x1 + 32][r1 + 32];
    const double c = (double)fu.ev[1 + s] + lambda * ((double)bits / 8.0);
    if (c < bc) {
      bc = c;
      best = s;
      bx0 = x0;
      bx1 = x1;
    }
  }
  return best < 0 ? 0xff : (best & 0xff) | (bx0 & 0xff) << 8 | (bx1 & 0xff) << 16;
}
// the same from memory, one option at a time (no registers held)
__device__ __noinline__ int fix_decide_mem(const uint64_t *e, const int8_t *xq, const FixState &f, int p,
                                           double lambda, const uint8_t (*slut)[128][128],
                                           const uint16_t (*sbl)[520]) {
  int best = -1, bx0 = 0, bx1 = 0;
  double bc = (double)e[0] + lambda * ((double)sbl[0][f.c0 >> 6] / 8.0);
  const uint32_t base = sbl[1][f.c1 >> 6] + (4u << 3);
  const int r0 = f.ref[p][0], r1 = f.ref[p][1];
  for (int s = 0; s < 16; s++) {
    const int x0 = xq[2 * s], x1 = xq[2 * s + 1];
    uint32_t bits = base;
    if (lrf_set_has(s, 0)) bits += slut[0][x0 + 96][r0 + 96];
    if (lrf_set_has(s, 1)) bits += slut[1][x1 + 32][r1 + 32];
    const double c = (double)e[1 + s] + lambda * ((double)bits / 8.0);
    if (c < bc) {
      bc = c;
      best = s;
      bx0 = x0;
      bx1 = x1;
    }
  }
  return best < 0 ? 0xff : (best & 0xff) | (bx0 & 0xff) << 8 | (bx1 & 0xff) << 16;
}
constexpr int kFixNoUnit = 0xfe;  // a stretched superblock (no unit of its own)

__global__ __launch_bounds__(kFixThreads) void lrf_decide_fix_kernel(LrfDecideArgs a) {
  __shared__ uint8_t slut[2][128][128];
  __shared__ uint16_t sbl[2][520];
  __shared__ FixState fs[kFixMax];
  __shared__ int dec[kFixMax][3];
  __shared__ int first;
  const LrfGeo &g = a.g;
  const int ntx = (g.sbc + g.tws - 1) / g.tws;
  const int t = blockIdx.x, tid = threadIdx.x;
  FIXCLK(0);
  const int t0x = (t % ntx) * g.tws, t0y = (t / ntx) * g.ths;
  if (t0x < a.gx0 || t0x >= a.gx1 || t0y < a.gy0 || t0y >= a.gy1) return;  // another group's tile
  const int tsw = min(g.tws, g.sbc - t0x), tsh = min(g.ths, g.sbr - t0y), n = tsw * tsh;
  {
    const uint4 *gl = (const uint4 *)&g_lrf_subexp[0][0][0];
    uint4 *sl = (uint4 *)&slut[0][0][0];
    for (int i = tid; i < 2 * 128 * 128 / 16; i += kFixThreads) sl[i] = gl[i];
    for (int f = tid; f < 520; f += kFixThreads) {
      const uint16_t c0[4] = {(uint16_t)(f << 6), 0, 0, 0}, c1[4] = {0, (uint16_t)(f << 6), 0, 0};
      sbl[0][f] = (uint16_t)lrf_symbol_bits(0, c0, 3);
      sbl[1][f] = (uint16_t)lrf_symbol_bits(2, c1, 3);
    }
    LrfTileState st;
    lrf_tile_init(st);
    for (int k = tid; k < n; k += kFixThreads) {
      fix_store(fs[k], st);  // the guess: every state the initial one
      dec[k][0] = dec[k][1] = dec[k][2] = -1;
    }
  }
  auto unit_of = [&](int i, int &k, int &p, bool &has, size_t &u) {
    k = i / 3;
    p = i - 3 * k;
    const int fsx = t0x + k % tsw, fsy = t0y + k / tsw;
    has = fsx < (p == 0 ? g.cols[0] : p == 1 ? g.cols[1] : g.cols[2]) &&
          fsy < (p == 0 ? g.rows[0] : p == 1 ? g.rows[1] : g.rows[2]);
    u = (size_t)p * g.nsb + (size_t)fsy * g.sbc + fsx;
  };
  // serial: the states from superblock k0 on (k0's own is final), wave 0.
  // Batches of 64 superblocks: lane j holds superblock k + j's decisions
  // (read in one LDS access) and receives the state before it (a lane
  // select), so the chain itself is scalar: lane reads and the updates.
  auto run_states = [&](int k0) {
    auto uni = [](int v) { return __builtin_amdgcn_readfirstlane(v); };
    // the state in three scalar words, updated without branches: cc =
    // lrf_switchable_cdf[0] | [1] << 16 (both entries move the same way, and
    // each half stays within 0..32768, so one subtract serves both), c3 its
    // counter, rp the planes' sgrproj_ref as bytes (ref0 | ref1 << 8 each)
    uint32_t cc = (uint32_t)uni(fs[k0].c0) | (uint32_t)uni(fs[k0].c1) << 16;
    int c3 = uni(fs[k0].c3);
    uint32_t rp[3];
#pragma unroll
    for (int q = 0; q < 3; q++)
      rp[q] = ((uint32_t)uni(fs[k0].ref[q][0]) & 0xff) | ((uint32_t)uni(fs[k0].ref[q][1]) & 0xff) << 8;
    for (int kb = k0; kb < n; kb += 64) {
      const int kk = kb + tid, m = min(64, n - kb);
      const int d0 = kk < n ? dec[kk][0] : kFixNoUnit, d1 = kk < n ? dec[kk][1] : kFixNoUnit,
                d2 = kk < n ? dec[kk][2] : kFixNoUnit;
      uint32_t w0 = 0, w1 = 0, w2 = 0;  // the state before superblock kk
      for (int j = 0; j < m; j++) {
        const bool me = tid == j;
        w0 = me ? cc : w0;
        w1 = me ? (uint32_t)c3 | rp[2] << 16 : w1;
        w2 = me ? rp[0] | rp[1] << 16 : w2;
        const int dd[3] = {__builtin_amdgcn_readlane(d0, j), __builtin_amdgcn_readlane(d1, j),
                           __builtin_amdgcn_readlane(d2, j)};
#pragma unroll
        for (int p = 0; p < 3; p++) {
          // lrf_commit: update_cdf (src/ec.rs:891-905) with symbol 0 (None:
          // the entries fall) or 2 (a set: they rise towards 32768), and the
          // set's sgrproj_ref
          const uint32_t d = (uint32_t)dd[p], set = d & 0xff;
          const bool valid = set != kFixNoUnit, rise = valid && set < 16;
          const uint32_t sh = 4 + ((uint32_t)c3 >> 4), msk = (0xffffu >> sh) * 0x10001u;
          uint32_t x = rise ? 0x80008000u - cc : cc;
          x -= (x >> sh) & msk;
          x = rise ? 0x80008000u - x : x;
          cc = valid ? x : cc;
          c3 = valid ? min(c3 + 1, 32) : c3;
          // (masks, not selects: the compiler would branch on them)
          const uint32_t h0 = 0u - (uint32_t)(set - 10u > 3u), h1 = 0u - (uint32_t)(set < 14u),
                         rm = 0u - (uint32_t)rise;
          const uint32_t nr = ((d >> 8) & 0xffu & h0) | ((d >> 8) & 0xff00u & h1) | (95u << 8 & ~h1);
          rp[p] = (nr & rm) | (rp[p] & ~rm);
        }
      }
      if (kk > k0 && kk < n) {
        FixState &f = fs[kk];
        f.c0 = (uint16_t)(w0 & 0xffff);
        f.c1 = (uint16_t)(w0 >> 16);
        f.c3 = (uint16_t)(w1 & 0xffff);
        f.ref[0][0] = (int8_t)(w2 & 0xff);
        f.ref[0][1] = (int8_t)((w2 >> 8) & 0xff);
        f.ref[1][0] = (int8_t)((w2 >> 16) & 0xff);
        f.ref[1][1] = (int8_t)(w2 >> 24);
        f.ref[2][0] = (int8_t)((w1 >> 16) & 0xff);
        f.ref[2][1] = (int8_t)(w1 >> 24);
      }
    }
  };
  __syncthreads();
  bool settled = false;
  int from = 0;
  // the lane's first item stays in registers across the passes
  FixUnit mine;
  int mk = 0, mp = 0;
  bool mhas = false;
  if (tid < 3 * n) {
    size_t u;
    unit_of(tid, mk, mp, mhas, u);
    if (mhas) fix_load_unit(mine, a.err + u * 17, a.xqd + u * 32);
  }
  FIXCLK(1);
  for (int it = 0; it < a.fix_passes; it++) {
    if (tid == 0) first = n;
    __syncthreads();
    FIXCLK(2 + 3 * it);
    for (int i = tid; i < 3 * n; i += kFixThreads) {
      int k, p, d;
      if (i == tid) {
        k = mk;
        p = mp;
        if (k < from) continue;
        d = mhas ? fix_decide(mine, fs[k], p, a.lambda, slut, sbl) : kFixNoUnit;
      } else {  // tiles past 341 superblocks: the other items straight from memory
        bool has;
        size_t u;
        unit_of(i, k, p, has, u);
        if (k < from) continue;
        d = has ? fix_decide_mem(a.err + u * 17, a.xqd + u * 32, fs[k], p, a.lambda, slut, sbl) : kFixNoUnit;
      }
      if (d != dec[k][p]) {
        dec[k][p] = d;
        atomicMin(&first, k);
      }
    }
    __syncthreads();
    FIXCLK(3 + 3 * it);
    from = first;
#ifdef LRF_PHASES
    if (tid == 0 && t < 8) lrf_fix_trace[t][it] = from;
#endif
    if (from == n) {
      settled = true;
      break;
    }
    if (tid < 64) run_states(from);
    __syncthreads();
    FIXCLK(4 + 3 * it);
  }
#ifdef LRF_PHASES
  if (tid == 0 && t < 8) lrf_fix_iters[t] = settled ? 0 : -1;
#endif
  if (!settled && tid == 0) {  // the rest in order (from: its state is final)
    LrfTileState st;
    fix_load(st, fs[from]);
    for (int k = from; k < n; k++) {
      FixState f;
      fix_store(f, st);
#pragma unroll
      for (int p = 0; p < 3; p++) {
        int kk, pp;
        bool has;
        size_t u;
        unit_of(3 * k + p, kk, pp, has, u);
        dec[k][p] = has ? fix_decide_mem(a.err + u * 17, a.xqd + u * 32, f, p, a.lambda, slut, sbl) : kFixNoUnit;
      }
#pragma unroll
      for (int p = 0; p < 3; p++) {
        const int d = dec[k][p];
        if (d != kFixNoUnit) {
          const int8_t q[2] = {(int8_t)((d >> 8) & 0xff), (int8_t)((d >> 16) & 0xff)};
          lrf_commit(st, p, (int8_t)(d & 0xff), q);
        }
      }
    }
  }
#ifdef LRF_PHASES
  if (tid == 0 && t < 8) lrf_fix_stats[t] = (settled ? 0 : 1000) + from;  // where it settled / fell back
#endif
  FIXCLK(39);
  __syncthreads();
  for (int i = tid; i < 9 * n; i += kFixThreads) {
    const int k = i / 9, p = (i / 3) % 3, j = i % 3;
    const int fsx = t0x + k % tsw, fsy = t0y + k / tsw, d = dec[k][p];
    int8_t b;
    if (d == kFixNoUnit)
      b = j == 0 ? -1 : 0;
    else
      b = (int8_t)((d >> (8 * j)) & 0xff);
    a.units[(((size_t)p * g.urows_max + fsy) * g.ucols_max + fsx) * 3 + j] = b;
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

// The restored chunk: columns x .. x + w - 1 (w <= 32) of the stripe at rows
// y0 .. y0 + sz - 1 (sz <= 64) of a crop_w x crop_h plane, set `set`,
// weights (w0, w1) = xqd, into op (row pitch ostride) -- lrf_filter_kernel's
// body, shared with the golden-stripe test kernel.
template <typename Px>
__device__ __forceinline__ void lrf_filter_chunk(SgrLds<32, 64> &L, uint16_t *blk, const rv_plane &cd,
                                                 const rv_plane &db, int x, int w, int y0, int sz,
                                                 int crop_w, int crop_h, int set, int w0, int w1, int bd,
                                                 Px *op, int64_t ostride) {
  using L32 = SgrLds<32, 64>;
  auto at = [](const rv_plane &pl, int xx, int yy) -> int {
    return (int)((const Px *)pl.data)[(int64_t)(pl.yorigin + yy) * pl.stride + pl.xorigin + xx];
  };
  // setup_integral_image's view (VertPaddedIter / HorzPaddedIter): columns
  // clamp to the frame (the unit's own right limit reaches 3 past it),
  // rows to the frame and the stripe's +-2 extension, deblocked outside
  const int sh = sz + (sz & 1), crop = crop_h;
  sgr_init_xz(L.xz);
  sgr_integral<L32::IS, L32::IR>(L.ii, w, sz, [&](int r, int c) -> uint32_t {
    const int cy = iclamp(y0 - 4 + r, 0, crop - 1), ly = iclamp(cy, y0 - 2, y0 + sh + 1);
    const int xx = iclamp(x - 4 + c, 0, crop_w - 1);
    return (uint32_t)((ly >= y0 && ly < y0 + sh) ? at(cd, xx, ly) : at(db, xx, ly));
  });
  for (int i = threadIdx.x; i < w * sz; i += blockDim.x) {
    const int yy = i / w, xx = i - yy * w;
    blk[yy * 32 + xx] = (uint16_t)at(cd, x + xx, y0 + yy);
  }
  sgr_tables<L32::IS, L32::IR, L32::AS, L32::A1R>(L.ii, L.tab, L.xz, sgr_lane(w), set, sz, bd - 8);
  __syncthreads();
  const int mx = (1 << bd) - 1;
  for (int i = threadIdx.x; i < w * sz; i += blockDim.x) {
    const int yy = i / w, xx = i - yy * w;
    const uint32_t px = blk[yy * 32 + xx], px0 = blk[(yy & ~1) * 32 + xx];
    uint32_t f2, f1;
    sgr_f<L32::AS, L32::A1R>(L.tab, set, xx, yy, px, px0, f2, f1);
    op[(int64_t)yy * ostride + xx] = (Px)sgr_out(f2, f1, px, w0, w1, mx);
  }
}

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
  lrf_filter_chunk<Px>(L, blk, cd, db, x, w, y0, sz, crop_w, crop_h, u[0], u[1], u[2], g.bd, op,
                       out.stride);
}

// One golden stripe (tests/golden/ref_lrf.npz, rv_lrf_stripe_filter): the
// stripe at (x0, y0) of sw x sz pixels inside a cw x ch crop, restored with
// set `set` and weights (w0, w1) by the product's chunk code, 32 columns per
// workgroup, into out (row pitch sw).
template <typename Px>
__global__ __launch_bounds__(256) void lrf_stripe_case_kernel(rv_plane cd, rv_plane db, int x0, int y0,
                                                               int sw, int sz, int cw, int ch, int set,
                                                               int w0, int w1, int bd, Px *out) {
  using L32 = SgrLds<32, 64>;
  __shared__ L32 L;
  __shared__ uint16_t blk[64 * 32];
  const int c = (int)blockIdx.x * 32;
  if (c >= sw) return;
  lrf_filter_chunk<Px>(L, blk, cd, db, x0 + c, min(32, sw - c), y0, sz, cw, ch, set, w0, w1, bd,
                       out + c, sw);
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

// g_lrf_subexp, once per process (the table is a constant of the codec)
static int lrf_lut_upload() {
  static std::once_flag once;
  static int rc = RV_OK;
  std::call_once(once, [] {
    static uint8_t t[2][128][128];
    for (int i = 0; i < 2; i++)
      for (int x = 0; x < 128; x++)
        for (int r = 0; r < 128; r++) {
          const int lo = i ? -32 : -96;
          const uint32_t b = lrf_subexp_ref(x + lo, lo, lo + 128, 4, r + lo);
          if (b > 255) rc = RV_EINVAL;
          t[i][x][r] = (uint8_t)b;
        }
    if (rc == RV_OK && hipMemcpyToSymbol(HIP_SYMBOL(g_lrf_subexp), t, sizeof(t)) != hipSuccess) rc = RV_EHIP;
  });
  return rc == RV_OK ? RV_OK : rv_set_error(rc, "loop restoration: subexp table upload failed");
}

int lrf_rdo_launch(const rv_plane rec[3], const rv_plane src[3], const uint8_t *skip, int mi_stride,
                   const float *imp, int w_imp, int w_in_b, int h_in_b, const LrfGeo &g, int cdef,
                   const uint8_t *dir, const int32_t *var, const uint8_t cdef_str[2], const double ds[3],
                   uint64_t *err, int8_t *xqd, const int32_t *rect, hipStream_t s) {
  if (g.xdec != g.ydec) return rv_set_error(RV_EINVAL, "loop restoration: 4:2:0, 4:4:4 (4:2:2 has none)");
  if (lrf_lut_upload() != RV_OK) return RV_EHIP;
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
  a.dir = dir;
  a.var = var;
  a.dstride = (g.W + 7) / 8;
  a.pri_y = cdef_str[0] / 4;
  a.sec_y = cdef_str[0] % 4 == 3 ? 4 : cdef_str[0] % 4;
  a.pri_uv = cdef_str[1] / 4;
  a.sec_uv = cdef_str[1] % 4 == 3 ? 4 : cdef_str[1] % 4;
  a.damping = 3;  // cdef_damping (src/encoder.rs:665)
  a.err = err;
  a.xqd = xqd;
  a.gx0 = rect ? rect[0] : 0;
  a.gy0 = rect ? rect[1] : 0;
  a.gx1 = rect ? rect[0] + rect[2] : g.sbc;
  a.gy1 = rect ? rect[1] + rect[3] : g.sbr;
  // 64 x 64 units: luma (and 4:4:4 chroma); 32 x 32: 4:2:0 chroma
  const bool c420 = g.xdec && g.ydec;
  a.p0 = 0;
  const dim3 grid64((unsigned)g.nsb, c420 ? 1 : 3), grid32((unsigned)g.nsb, 2);
  // RAV1E_LRF_WIDE=0 (A/B): the 1024-lane, 135 KB workgroup for 64 x 64 units
  static const bool wide = [] {
    const char *e = getenv("RAV1E_LRF_WIDE");
    return !(e && e[0] == '0');
  }();
  if (wide) {
    if (rec[0].hbd)
      lrf_rdo_wide_kernel<uint16_t><<<grid64, 512, 0, s>>>(a);
    else
      lrf_rdo_wide_kernel<uint8_t><<<grid64, 512, 0, s>>>(a);
  } else {
    if (rec[0].hbd)
      lrf_rdo_kernel<uint16_t, 64, 64><<<grid64, 1024, 0, s>>>(a);
    else
      lrf_rdo_kernel<uint8_t, 64, 64><<<grid64, 1024, 0, s>>>(a);
  }
  RV_HIP_CHECK_LAUNCH();
  if (c420) {
    a.p0 = 1;
    if (rec[0].hbd)
      lrf_rdo_kernel<uint16_t, 32, 32><<<grid32, 256, 0, s>>>(a);
    else
      lrf_rdo_kernel<uint8_t, 32, 32><<<grid32, 256, 0, s>>>(a);
    RV_HIP_CHECK_LAUNCH();
  }
  return RV_OK;
}

// the sequential decisions over the units lrf_rdo_launch priced (rect: the
// same superblocks)
int lrf_decide_launch(const LrfGeo &g, const uint64_t *err, const int8_t *xqd, double lambda, int8_t *units,
                      const int32_t *rect, int fix_passes, hipStream_t s) {
  LrfDecideArgs d;
  d.g = g;
  d.err = err;
  d.xqd = xqd;
  d.lambda = lambda;
  d.units = units;
  d.gx0 = rect ? rect[0] : 0;
  d.gy0 = rect ? rect[1] : 0;
  d.gx1 = rect ? rect[0] + rect[2] : g.sbc;
  d.gy1 = rect ? rect[1] + rect[3] : g.sbr;
  const int nt = ((g.sbc + g.tws - 1) / g.tws) * ((g.sbr + g.ths - 1) / g.ths);
  // fix_passes: 0 the one-wave serial decision, else the fixed point with at
  // most that many parallel passes (capped at kFixIter) before its serial rest
  d.fix_passes = std::min(std::max(fix_passes, 1), kFixIter);
  if (fix_passes > 0 && g.tws * g.ths <= kFixMax)
    lrf_decide_fix_kernel<<<nt, kFixThreads, 0, s>>>(d);
  else
    lrf_decide_kernel<<<nt, 64, 0, s>>>(d);
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

// One stripe of the golden loop-restoration vectors through the device's
// filter code (lrf_filter_kernel's chunk body): tests/test_lrf.py -m gpu.
extern "C" int rv_lrf_stripe_filter(const rv_plane *cd, const rv_plane *db, int x0, int y0, int sw,
                                    int sh, int cw, int ch, int set, int xqd0, int xqd1, int bit_depth,
                                    void *d_out, void *stream) {
  if (!cd || !db || !d_out || cd->hbd != db->hbd || sw < 1 || sw > 256 || sh < 1 || sh > 64 ||
      set < 0 || set > 15 || x0 < 0 || y0 < 0 || x0 + sw > cw || y0 + sh > ch || cw > cd->width ||
      ch > cd->height || cw > db->width || ch > db->height ||
      (bit_depth != 8 && bit_depth != 10 && bit_depth != 12) || (!cd->hbd && bit_depth != 8))
    return rv_set_error(RV_EINVAL, "rv_lrf_stripe_filter: bad arguments");
  hipStream_t s = rv_resolve_stream(stream);
  const unsigned grid = (unsigned)((sw + 31) / 32);
  if (cd->hbd)
    lrf_stripe_case_kernel<uint16_t><<<grid, 256, 0, s>>>(*cd, *db, x0, y0, sw, sh, cw, ch, set, xqd0, xqd1,
                                                          bit_depth, (uint16_t *)d_out);
  else
    lrf_stripe_case_kernel<uint8_t><<<grid, 256, 0, s>>>(*cd, *db, x0, y0, sw, sh, cw, ch, set, xqd0, xqd1,
                                                         bit_depth, (uint8_t *)d_out);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}
