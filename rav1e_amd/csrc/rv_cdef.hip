// rv_cdef.hip -- the CDEF filter of a reconstructed frame (cdef_filter_frame,
// src/cdef.rs:542-641) on gfx950.
//
// Two launches per frame, both HBM-bound byte work:
//  * cdef_dir_kernel: one lane per 8x8 luma block (cdef_analyze_superblock,
//    :278-317): cdef_find_dir (:68-126) over the block, dir / var to HBM.
//  * cdef_filter_kernel: one lane per visible output pixel of a plane, a
//    64-lane row segment per wavefront (coalesced stores), the block's
//    strengths from the per-64x64 cdef_index and the per-8x8 dir / var /
//    skip (cdef_filter_superblock, :411-534), the 12 taps of
//    cdef_filter_block (:152-228) read through L1/L2.
// The reference's padded u16 copy (:550-609) is never materialised: a tap
// outside the visible plane reads CDEF_VERY_LARGE inside the 2-pixel ring
// and Plane::new's fill value 128 beyond it, exactly the copy's contents.
// Out of place: src is the unfiltered reconstruction, dst receives it
// filtered (the reference writes back into rec from its copy).
#include "rv_device.h"

namespace rv {

constexpr int kCdefVeryLarge = 0x8000;

struct CdefArgs {
  rv_plane src, dst;
  const uint8_t *skip, *cdef_index, *dir;
  const int32_t *var;
  uint8_t *dir_out;
  int32_t *var_out;
  int pw, ph, xdec, ydec, pli, cols8, rows8, mi_stride, fb_w, damping, bd;
  uint8_t ystr[8], uvstr[8];
};
// the filter of up to three planes in one launch: plane p owns the 64x4
// tiles [blk[p], blk[p + 1]), tx[p] of them per row
struct CdefPlanes {
  CdefArgs pl[3];
  unsigned blk[4];
  int tx[3];
};

template <typename T>
__device__ __forceinline__ int cdef_px(const rv_plane &p, int pw, int ph, int x, int y) {
  if ((unsigned)x < (unsigned)pw && (unsigned)y < (unsigned)ph)
    return ((const T *)p.data)[(int64_t)(p.yorigin + y) * p.stride + p.xorigin + x];
  return (x >= -2 && x < pw + 2 && y >= -2 && y < ph + 2) ? kCdefVeryLarge : 128;
}

__device__ __forceinline__ int cdef_msb(int32_t x) { return 31 ^ __clz(x); }

__device__ __forceinline__ bool cdef_skip8(const uint8_t *skip, int mi_stride, int bx, int by) {
  const uint8_t *s = skip + (int64_t)(2 * by) * mi_stride + 2 * bx;
  return (s[0] & s[1] & s[mi_stride] & s[mi_stride + 1]) != 0;
}

// cdef_find_dir (src/cdef.rs:68-126); wrapping u32 arithmetic like the
// reference's release build (partial edge blocks sum CDEF_VERY_LARGE).
template <typename T>
__global__ __launch_bounds__(256) void cdef_dir_kernel(CdefArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.cols8 * a.rows8) return;
  const int bx = i % a.cols8, by = i / a.cols8;
  uint8_t dir = 0;
  int32_t var = 0;
  if (!cdef_skip8(a.skip, a.mi_stride, bx, by)) {
    const int cs = a.bd - 8;
    int32_t partial[8][15];
#pragma unroll
    for (int d = 0; d < 8; d++)
#pragma unroll
      for (int k = 0; k < 15; k++) partial[d][k] = 0;
#pragma unroll
    for (int r = 0; r < 8; r++)
#pragma unroll
      for (int c = 0; c < 8; c++) {
        const int32_t x = (cdef_px<T>(a.src, a.pw, a.ph, 8 * bx + c, 8 * by + r) >> cs) - 128;
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
    dir = (uint8_t)best;
    var = (int32_t)((uint32_t)best_cost - orth) >> 10;
  }
  a.dir_out[i] = dir;
  a.var_out[i] = var;
}

// constrain (src/cdef.rs:134-148)
__device__ __forceinline__ int cdef_constrain(int diff, int threshold, int damping) {
  if (!threshold) return 0;
  const int shift = max(0, damping - cdef_msb(threshold));
  const int ad = diff < 0 ? -diff : diff;
  const int mag = min(ad, max(0, threshold - (ad >> shift)));
  return diff < 0 ? -mag : mag;
}

// adjust_strength (src/cdef.rs:232-239)
__device__ __forceinline__ int cdef_adjust(int strength, int32_t var) {
  const int i = (var >> 6) ? min(cdef_msb(var >> 6), 12) : 0;
  return var ? (strength * (4 + i) + 8) >> 4 : 0;
}

// tap offsets (dy, dx) of cdef_directions (src/cdef.rs:164-173): [dir][k]
__constant__ int8_t kCdefDirs[8][2][2] = {
    {{-1, 1}, {-2, 2}}, {{0, 1}, {-1, 2}}, {{0, 1}, {0, 2}},  {{0, 1}, {1, 2}},
    {{1, 1}, {2, 2}},   {{1, 0}, {2, 1}},  {{1, 0}, {2, 0}},  {{1, 0}, {2, -1}}};

template <typename T>
__global__ __launch_bounds__(256) void cdef_filter_kernel(CdefPlanes P) {
  const int pi = blockIdx.x >= P.blk[1] ? (blockIdx.x >= P.blk[2] ? 2 : 1) : 0;
  const CdefArgs &a = P.pl[pi];
  const int t = (int)(blockIdx.x - P.blk[pi]), ty = t / P.tx[pi];
  const int x = (t - ty * P.tx[pi]) * 64 + threadIdx.x;
  const int y = ty * 4 + threadIdx.y;
  if (x >= a.pw || y >= a.ph) return;
  const int bx = (x << a.xdec) >> 3, by = (y << a.ydec) >> 3;
  const int px = cdef_px<T>(a.src, a.pw, a.ph, x, y);
  int v = px;
  if (!cdef_skip8(a.skip, a.mi_stride, bx, by)) {
    const int idx = a.cdef_index[(by >> 3) * a.fb_w + (bx >> 3)] & 7;  // cdef_bits <= 3
    const int str = a.pli ? a.uvstr[idx] : a.ystr[idx];
    const int pri0 = str >> 2;
    int sec = str & 3;
    if (sec == 3) sec++;
    const int cs = a.bd - 8;
    const int b = by * a.cols8 + bx;
    const int pri = a.pli ? pri0 << cs : cdef_adjust(pri0 << cs, a.var[b]);
    sec <<= cs;
    const int damping = a.damping + cs - (a.pli ? 1 : 0);
    const int dir = pri0 ? a.dir[b] & 7 : 0;
    const int odd = (pri >> cs) & 1;
    int sum = 0, mx = px, mn = px;
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const int pt = odd ? 3 : (k ? 2 : 4), st = k ? 1 : 2;
      const int dy0 = kCdefDirs[dir][k][0], dx0 = kCdefDirs[dir][k][1];
      const int dy1 = kCdefDirs[(dir + 2) & 7][k][0], dx1 = kCdefDirs[(dir + 2) & 7][k][1];
      const int dy2 = kCdefDirs[(dir + 6) & 7][k][0], dx2 = kCdefDirs[(dir + 6) & 7][k][1];
      const int p[2] = {cdef_px<T>(a.src, a.pw, a.ph, x + dx0, y + dy0),
                        cdef_px<T>(a.src, a.pw, a.ph, x - dx0, y - dy0)};
#pragma unroll
      for (int e = 0; e < 2; e++) {
        sum += pt * cdef_constrain(p[e] - px, pri, damping);
        if (p[e] != kCdefVeryLarge) mx = max(p[e], mx);
        mn = min(p[e], mn);
      }
      const int s[4] = {cdef_px<T>(a.src, a.pw, a.ph, x + dx1, y + dy1),
                        cdef_px<T>(a.src, a.pw, a.ph, x - dx1, y - dy1),
                        cdef_px<T>(a.src, a.pw, a.ph, x + dx2, y + dy2),
                        cdef_px<T>(a.src, a.pw, a.ph, x - dx2, y - dy2)};
#pragma unroll
      for (int e = 0; e < 4; e++) {
        if (s[e] != kCdefVeryLarge) mx = max(s[e], mx);
        mn = min(s[e], mn);
        sum += st * cdef_constrain(s[e] - px, sec, damping);
      }
    }
    v = clampi(px + ((8 + sum - (sum < 0)) >> 4), mn, mx);
  }
  ((T *)a.dst.data)[(int64_t)(a.dst.yorigin + y) * a.dst.stride + a.dst.xorigin + x] = (T)v;
}

}  // namespace rv

using namespace rv;

static bool cdef_bd_ok(const rv_plane *p, int bd) {
  return (bd == 8 || bd == 10 || bd == 12) && p->hbd == (bd > 8);
}

// cdef_analyze_superblock over the frame (src/cdef.rs:278-317, called per
// superblock by cdef_filter_frame :622-628): dir / var per 8x8 luma block,
// pitch ceil(width / 8); skip blocks get dir 0, var 0.  The frame size
// must be a multiple of 8: rav1e's reconstruction always is (Frame::new
// aligns it, src/frame/mod.rs:58-59), so a ragged plane has no reference
// counterpart.
extern "C" int rv_cdef_find_dirs(const rv_plane *luma, int width, int height,
                                 const uint8_t *d_skip, int mi_stride, uint8_t *d_dir,
                                 int32_t *d_var, int bit_depth, void *stream) {
  const int cols8 = (width + 7) / 8, rows8 = (height + 7) / 8;
  if (!luma || !d_skip || !d_dir || !d_var || width <= 0 || height <= 0 || (width & 7) ||
      (height & 7) || mi_stride < 2 * cols8 || !cdef_bd_ok(luma, bit_depth) || luma->width < width ||
      luma->height < height)
    return rv_set_error(RV_EINVAL, "rv_cdef_find_dirs: bad arguments");
  CdefArgs a = {};
  a.src = *luma;
  a.skip = d_skip;
  a.dir_out = d_dir;
  a.var_out = d_var;
  a.pw = width;
  a.ph = height;
  a.cols8 = cols8;
  a.rows8 = rows8;
  a.mi_stride = mi_stride;
  a.bd = bit_depth;
  const unsigned grid = (unsigned)((cols8 * rows8 + 255) / 256);
  hipStream_t s = rv_resolve_stream(stream);
  if (luma->hbd)
    cdef_dir_kernel<uint16_t><<<grid, 256, 0, s>>>(a);
  else
    cdef_dir_kernel<uint8_t><<<grid, 256, 0, s>>>(a);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

// The arguments of cdef_filter_superblock over plane pli (cdef_bits <= 3).
static int cdef_plane_args(CdefArgs &a, const rv_plane *src, const rv_plane *dst, int pli,
                           int width, int height, const uint8_t *d_skip, int mi_stride,
                           const uint8_t *d_dir, const int32_t *d_var, const uint8_t *d_cdef_index,
                           const uint8_t *y_strengths, const uint8_t *uv_strengths, int damping,
                           int bit_depth) {
  if (!src || !dst || !d_skip || !d_dir || !d_var || !d_cdef_index || !y_strengths ||
      !uv_strengths || pli < 0 || pli > 2 || width <= 0 || height <= 0 || (width & 7) ||
      (height & 7) || damping < 0 ||
      mi_stride < 2 * ((width + 7) / 8) || !cdef_bd_ok(src, bit_depth) || dst->hbd != src->hbd ||
      src->data == dst->data)
    return rv_set_error(RV_EINVAL, "rv_cdef_filter_plane: bad arguments");
  a = CdefArgs{};
  a.src = *src;
  a.dst = *dst;
  a.xdec = pli ? src->xdec : 0;
  a.ydec = pli ? src->ydec : 0;
  if (a.xdec > 1 || a.ydec > 1 || dst->xdec != src->xdec || dst->ydec != src->ydec)
    return rv_set_error(RV_EINVAL, "rv_cdef_filter_plane: plane decimation");
  a.pw = pli ? (width + a.xdec) >> a.xdec : width;
  a.ph = pli ? (height + a.ydec) >> a.ydec : height;
  if (src->width < a.pw || src->height < a.ph || dst->width < a.pw || dst->height < a.ph)
    return rv_set_error(RV_EINVAL, "rv_cdef_filter_plane: plane smaller than the frame");
  for (int k = 0; k < 8; k++)
    if (y_strengths[k] > 63 || uv_strengths[k] > 63)
      return rv_set_error(RV_EINVAL, "rv_cdef_filter_plane: strength above 15 * 4 + 3");
  a.skip = d_skip;
  a.cdef_index = d_cdef_index;
  a.dir = d_dir;
  a.var = d_var;
  a.pli = pli;
  a.cols8 = (width + 7) / 8;
  a.rows8 = (height + 7) / 8;
  a.mi_stride = mi_stride;
  a.fb_w = (width + 63) / 64;
  a.damping = damping;
  a.bd = bit_depth;
  for (int k = 0; k < 8; k++) {
    a.ystr[k] = y_strengths[k];
    a.uvstr[k] = uv_strengths[k];
  }
  return RV_OK;
}

static void cdef_filter_launch(CdefPlanes &P, int np, hipStream_t s) {
  unsigned blocks = 0;
  for (int p = 0; p < np; p++) {
    P.tx[p] = (P.pl[p].pw + 63) / 64;
    P.blk[p] = blocks;
    blocks += (unsigned)(P.tx[p] * ((P.pl[p].ph + 3) / 4));
  }
  for (int p = np; p < 4; p++) P.blk[p] = blocks;
  const dim3 block(64, 4);
  if (P.pl[0].src.hbd)
    cdef_filter_kernel<uint16_t><<<blocks, block, 0, s>>>(P);
  else
    cdef_filter_kernel<uint8_t><<<blocks, block, 0, s>>>(P);
}

// cdef_filter_superblock over every superblock of plane pli (src/cdef.rs:
// 411-534 via cdef_filter_frame :614-640), src -> dst (distinct planes).
extern "C" int rv_cdef_filter_plane(const rv_plane *src, const rv_plane *dst, int pli, int width,
                                    int height, const uint8_t *d_skip, int mi_stride,
                                    const uint8_t *d_dir, const int32_t *d_var,
                                    const uint8_t *d_cdef_index, const uint8_t *y_strengths,
                                    const uint8_t *uv_strengths, int damping, int bit_depth,
                                    void *stream) {
  CdefPlanes P = {};
  const int e = cdef_plane_args(P.pl[0], src, dst, pli, width, height, d_skip, mi_stride, d_dir,
                                d_var, d_cdef_index, y_strengths, uv_strengths, damping, bit_depth);
  if (e != RV_OK) return e;
  cdef_filter_launch(P, 1, rv_resolve_stream(stream));
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

// cdef_filter_frame's filter pass over the three planes (src/cdef.rs:
// 614-640) in one launch, src[p] -> dst[p].
int rv_cdef_filter_frame_dev(const rv_plane src[3], const rv_plane dst[3], int width, int height,
                             const uint8_t *d_skip, int mi_stride, const uint8_t *d_dir,
                             const int32_t *d_var, const uint8_t *d_cdef_index,
                             const uint8_t *y_strengths, const uint8_t *uv_strengths, int damping,
                             int bit_depth, hipStream_t s) {
  CdefPlanes P = {};
  for (int p = 0; p < 3; p++) {
    const int e = cdef_plane_args(P.pl[p], &src[p], &dst[p], p, width, height, d_skip, mi_stride,
                                  d_dir, d_var, d_cdef_index, y_strengths, uv_strengths, damping,
                                  bit_depth);
    if (e != RV_OK) return e;
  }
  cdef_filter_launch(P, 3, s);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}
