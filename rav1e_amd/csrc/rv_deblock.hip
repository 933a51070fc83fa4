// rv_deblock.hip -- the deblocking filter of a reconstructed plane
// (deblock_plane, src/deblock.rs:1174-1335) on gfx950.
//
// One lane per pixel row (vertical edges) or column (horizontal edges) of a
// 4-pixel edge segment.  Within a pass no filter reads a pixel another one
// writes (the transform grid keeps edges >= 8 pixels apart and the widest
// filter writes 6 on a side), so a pass is one launch; rav1e's interleaved
// order (horizontal edges lagging one 4x4 row and two columns) is
// equivalent to all vertical edges, then all horizontal ones.  Blocks come
// as per-4x4 bytes: log2 of the square block's width in 4x4 units and the
// skip flag (every block inter, loop-filter deltas off).
#include "rv_device.h"

namespace rv {

struct DbArgs {
  rv_plane p;
  const uint8_t *lg, *skip;
  const uint8_t *dlev;  // null: `level`; else the device levels [Y v, Y h, U, V]
  int mi_stride, cols, rows, xdec, ydec, pli, level, bd, vert;
};
// one pass (vertical or horizontal edges) over up to three planes in one
// launch: plane p owns workgroups [blk[p], blk[p + 1])
struct DbPlanes {
  DbArgs pl[3];
  unsigned blk[4];
};

__device__ __forceinline__ int db_abs(int v) { return v < 0 ? -v : v; }
__device__ __forceinline__ int db_max(int a, int b) { return a > b ? a : b; }
__device__ __forceinline__ int lim_lv(int v, int s) { return (v + (1 << s) - 1) >> s; }
__device__ __forceinline__ int blim_lv(int v, int s) { return (((v + (1 << s) - 1) >> s) - 2) / 3; }
__device__ __forceinline__ int thr_lv(int v, int s) { return (v + (1 << s) - 1) >> s << 4; }

// filter_narrow2_4 / filter_narrow4_4 (src/deblock.rs:165-240) on p1 p0 q0 q1
__device__ __forceinline__ void db_narrow(int32_t *v, int s, bool four) {
  const int lo = -(128 << s), hi = (128 << s) - 1, mx = (256 << s) - 1;
  const int f0 = four ? 0 : clampi(v[0] - v[3], lo, hi);
  const int f1 = clampi(f0 + 3 * (v[2] - v[1]) + 4, lo, hi) >> 3;
  const int f2 = clampi(f0 + 3 * (v[2] - v[1]) + 3, lo, hi) >> 3;
  if (four) {
    const int f3 = (f1 + 1) >> 1;
    v[0] = clampi(v[0] + f3, 0, mx);
    v[3] = clampi(v[3] - f3, 0, mx);
  }
  v[1] = clampi(v[1] + f2, 0, mx);
  v[2] = clampi(v[2] - f1, 0, mx);
}
__device__ __forceinline__ void db_narrow_sel(int32_t *c, int s, int level) {
  const int nhev = thr_lv(db_max(db_abs(c[0] - c[1]), db_abs(c[3] - c[2])), s);
  db_narrow(c, s, nhev <= level);
}
__device__ __forceinline__ int db_blim(const int32_t *c, int s) {
  return blim_lv(db_abs(c[1] - c[2]) * 2 + db_abs(c[0] - c[3]) / 2, s);
}

// deblock_size{4,6,8,14}_inner (:382-995) on N taps across the edge
template <int N>
__device__ __forceinline__ void db_filter(int32_t *t, int level, int bd) {
  const int s = bd - 8, flat = 1 << s;
  if constexpr (N == 4) {
    const int m = db_max(lim_lv(db_max(db_abs(t[0] - t[1]), db_abs(t[3] - t[2])), s), db_blim(t, s));
    if (m <= level) db_narrow_sel(t, s, level);
  } else if constexpr (N == 6) {
    const int m = db_max(lim_lv(db_max(db_max(db_abs(t[0] - t[1]), db_abs(t[1] - t[2])),
                                       db_max(db_abs(t[5] - t[4]), db_abs(t[4] - t[3]))), s),
                         db_blim(t + 1, s));
    if (m > level) return;
    const int f = db_max(db_max(db_abs(t[1] - t[2]), db_abs(t[4] - t[3])),
                         db_max(db_abs(t[0] - t[2]), db_abs(t[5] - t[3])));
    if (f <= flat) {  // filter_wide6_4
      const int p2 = t[0], p1 = t[1], p0 = t[2], q0 = t[3], q1 = t[4], q2 = t[5];
      t[1] = (p2 * 3 + p1 * 2 + p0 * 2 + q0 + 4) >> 3;
      t[2] = (p2 + p1 * 2 + p0 * 2 + q0 * 2 + q1 + 4) >> 3;
      t[3] = (p1 + p0 * 2 + q0 * 2 + q1 * 2 + q2 + 4) >> 3;
      t[4] = (p0 + q0 * 2 + q1 * 2 + q2 * 3 + 4) >> 3;
    } else {
      db_narrow_sel(t + 1, s, level);
    }
  } else {
    int32_t *in = N == 8 ? t : t + 3;  // p3 .. q3
    const int m = db_max(
        lim_lv(db_max(db_max(db_max(db_abs(in[0] - in[1]), db_abs(in[1] - in[2])), db_abs(in[2] - in[3])),
                      db_max(db_max(db_abs(in[7] - in[6]), db_abs(in[6] - in[5])), db_abs(in[5] - in[4]))),
               s),
        db_blim(in + 2, s));
    if (m > level) return;
    const int f8 = db_max(db_max(db_max(db_abs(in[2] - in[3]), db_abs(in[5] - in[4])),
                                 db_max(db_abs(in[1] - in[3]), db_abs(in[6] - in[4]))),
                          db_max(db_abs(in[0] - in[3]), db_abs(in[7] - in[4])));
    if (f8 > flat) {
      db_narrow_sel(in + 2, s, level);
      return;
    }
    bool wide14 = false;
    if constexpr (N == 14) {
      const int f14 = db_max(db_max(db_max(db_abs(t[2] - t[6]), db_abs(t[11] - t[7])),
                                    db_max(db_abs(t[1] - t[6]), db_abs(t[12] - t[7]))),
                             db_max(db_abs(t[0] - t[6]), db_abs(t[13] - t[7])));
      wide14 = f14 <= flat;
    }
    if (wide14) {  // filter_wide14_12
      const int p6 = t[0], p5 = t[1], p4 = t[2], p3 = t[3], p2 = t[4], p1 = t[5], p0 = t[6];
      const int q0 = t[7], q1 = t[8], q2 = t[9], q3 = t[10], q4 = t[11], q5 = t[12], q6 = t[13];
      t[1] = (p6 * 7 + p5 * 2 + p4 * 2 + p3 + p2 + p1 + p0 + q0 + 8) >> 4;
      t[2] = (p6 * 5 + p5 * 2 + p4 * 2 + p3 * 2 + p2 + p1 + p0 + q0 + q1 + 8) >> 4;
      t[3] = (p6 * 4 + p5 + p4 * 2 + p3 * 2 + p2 * 2 + p1 + p0 + q0 + q1 + q2 + 8) >> 4;
      t[4] = (p6 * 3 + p5 + p4 + p3 * 2 + p2 * 2 + p1 * 2 + p0 + q0 + q1 + q2 + q3 + 8) >> 4;
      t[5] = (p6 * 2 + p5 + p4 + p3 + p2 * 2 + p1 * 2 + p0 * 2 + q0 + q1 + q2 + q3 + q4 + 8) >> 4;
      t[6] = (p6 + p5 + p4 + p3 + p2 + p1 * 2 + p0 * 2 + q0 * 2 + q1 + q2 + q3 + q4 + q5 + 8) >> 4;
      t[7] = (p5 + p4 + p3 + p2 + p1 + p0 * 2 + q0 * 2 + q1 * 2 + q2 + q3 + q4 + q5 + q6 + 8) >> 4;
      t[8] = (p4 + p3 + p2 + p1 + p0 + q0 * 2 + q1 * 2 + q2 * 2 + q3 + q4 + q5 + q6 * 2 + 8) >> 4;
      t[9] = (p3 + p2 + p1 + p0 + q0 + q1 * 2 + q2 * 2 + q3 * 2 + q4 + q5 + q6 * 3 + 8) >> 4;
      t[10] = (p2 + p1 + p0 + q0 + q1 + q2 * 2 + q3 * 2 + q4 * 2 + q5 + q6 * 4 + 8) >> 4;
      t[11] = (p1 + p0 + q0 + q1 + q2 + q3 * 2 + q4 * 2 + q5 * 2 + q6 * 5 + 8) >> 4;
      t[12] = (p0 + q0 + q1 + q2 + q3 + q4 * 2 + q5 * 2 + q6 * 7 + 8) >> 4;
    } else {  // filter_wide8_6 on p3 .. q3
      const int p3 = in[0], p2 = in[1], p1 = in[2], p0 = in[3], q0 = in[4], q1 = in[5], q2 = in[6],
                q3 = in[7];
      in[1] = (p3 * 3 + p2 * 2 + p1 + p0 + q0 + 4) >> 3;
      in[2] = (p3 * 2 + p2 + p1 * 2 + p0 + q0 + q1 + 4) >> 3;
      in[3] = (p3 + p2 + p1 + p0 * 2 + q0 + q1 + q2 + 4) >> 3;
      in[4] = (p2 + p1 + p0 + q0 * 2 + q1 + q2 + q3 + 4) >> 3;
      in[5] = (p1 + p0 + q0 + q1 * 2 + q2 + q3 * 2 + 4) >> 3;
      in[6] = (p0 + q0 + q1 + q2 * 2 + q3 * 3 + 4) >> 3;
    }
  }
}

// transform width / height in 4x4 units: luma = the block, chroma =
// largest_chroma_tx_size (coded size <= 32, src/partition.rs:288-297)
__device__ __forceinline__ int db_tx_mi(int lg, int pli, int dec) {
  if (pli == 0) return 1 << lg;
  int px = (4 << lg) >> dec;
  px = px > 32 ? 32 : px;
  return px >= 4 ? px >> 2 : 1;
}

template <typename Px, int N>
__device__ __forceinline__ void db_apply(const DbArgs &a, int ox, int oy, int k, int level) {
  const int h = N >> 1;
  Px *base = a.vert ? plane_ptr_mut<Px>(a.p, ox - h, oy + k) : plane_ptr_mut<Px>(a.p, ox + k, oy - h);
  const int64_t step = a.vert ? 1 : a.p.stride;
  int32_t t[N];
#pragma unroll
  for (int i = 0; i < N; i++) t[i] = base[i * step];
  db_filter<N>(t, level, a.bd);
#pragma unroll
  for (int i = 0; i < N; i++) base[i * step] = (Px)t[i];
}

// thread = (edge segment, pixel row / column k of its 4)
template <typename Px>
__global__ __launch_bounds__(256) void deblock_kernel(DbPlanes P) {
  const int pi = blockIdx.x >= P.blk[1] ? (blockIdx.x >= P.blk[2] ? 2 : 1) : 0;
  const DbArgs &a = P.pl[pi];
  const int i = (blockIdx.x - P.blk[pi]) * 256 + threadIdx.x;
  const int k = i & 3, seg = i >> 2;
  const int sx = a.vert ? (a.cols >> a.xdec) - 1 : (a.cols >> a.xdec);  // segments per row
  const int sy = a.vert ? (a.rows >> a.ydec) : (a.rows >> a.ydec) - 1;
  if (seg >= sx * sy) return;
  int level = a.level;
  if (a.dlev) {
    if (!(a.dlev[0] | a.dlev[1])) return;  // src/encoder.rs:2790-2793
    level = a.pli == 0 ? a.dlev[a.vert ? 0 : 1] : a.dlev[a.pli + 1];
    if (!level) return;
  }
  const int gy = seg / sx, gx = seg - gy * sx;
  const int x = (gx + (a.vert ? 1 : 0)) << a.xdec, y = (gy + (a.vert ? 0 : 1)) << a.ydec;
  const int b = y * a.mi_stride + x;
  const int lgb = a.lg[b], n4 = 1 << lgb;
  const int pos = a.vert ? x : y, dec = a.vert ? a.xdec : a.ydec;
  if (((pos >> dec) & (db_tx_mi(lgb, a.pli, dec) - 1)) != 0) return;  // not a transform edge
  const int px = (x | a.xdec) - (a.vert ? 1 << a.xdec : 0);
  const int py = (y | a.ydec) - (a.vert ? 0 : 1 << a.ydec);
  const int pb = py * a.mi_stride + px;
  const bool block_edge = (pos & (n4 - 1)) == 0;
  if (!(block_edge || !a.skip[b] || !a.skip[pb])) return;
  const int tn = db_tx_mi(lgb, a.pli, dec), tp = db_tx_mi(a.lg[pb], a.pli, dec);
  int size = (tn < tp ? tn : tp) << 2;
  const int cap = a.pli == 0 ? 14 : 6;
  size = size < cap ? size : cap;
  const int ox = (x * 4) >> a.xdec, oy = (y * 4) >> a.ydec;
  if (size == 4)
    db_apply<Px, 4>(a, ox, oy, k, level);
  else if (size == 6)
    db_apply<Px, 6>(a, ox, oy, k, level);
  else if (size == 8)
    db_apply<Px, 8>(a, ox, oy, k, level);
  else
    db_apply<Px, 14>(a, ox, oy, k, level);
}

// ---- sse_optimize (src/deblock.rs:1418-1475): the level search below
// speed 8.  One lane per row of a 4-pixel edge segment, the vertical and the
// horizontal segments of all three planes in one launch (blockIdx.y = plane);
// a lane measures its row unfiltered and with each filter variant against
// the source and adds at most three tally deltas into the workgroup's LDS
// tallies (64-bit LDS atomics), which are added to the frame's tallies once
// per workgroup.  Integer sums: the result is order-independent.
struct SsePlane {
  rv_plane rec, src;
  int xdec, ydec, pli, nvx, nvy, nhx, nhy;  // vertical / horizontal segment grids
};
struct SseArgs {
  SsePlane pl[3];
  const uint8_t *lg, *skip;
  int mi_stride, bd;
  int64_t *tally;  // [plane][v 65 | h 65]
};

// the pixel at (x, y) of a plane, 128 outside its width: the fill of a
// fresh plane (src/frame/plane.rs:130-134); rav1e pads neither the
// reconstruction nor the input before the loop filters
template <typename Px>
__device__ __forceinline__ int32_t sse_px(const rv_plane &p, int x, int y) {
  return (x < 0 || x >= p.width) ? 128 : (int32_t)plane_ptr<Px>(p, x, y)[0];
}

// the SSE of the compared outputs (taps [o, N-o), o = 0 for 4 taps else 1;
// stride_sse, :337-344)
template <int N>
__device__ __forceinline__ int64_t sse_cmp(const int32_t *t, const int32_t *a) {
  constexpr int o = N == 4 ? 0 : 1;
  int32_t acc = 0;
#pragma unroll
  for (int i = o; i < N - o; i++) acc += (a[i] - t[i]) * (a[i] - t[i]);
  return acc;
}

// sse_size{4,6,8,14} (:425-999) of one row: taps t (rec), a (src)
template <int N>
__device__ __forceinline__ void sse_row(const int32_t *t, const int32_t *a, int bd, int d_idx[3],
                                        int64_t d_val[3]) {
  const int s = bd - 8, fl = 1 << s;
  constexpr int ci = N == 4 ? 0 : N == 6 ? 1 : N == 8 ? 2 : 5;  // p1 of p1 p0 q0 q1
  const int32_t *c = t + ci;
  int m, flat = 0;
  if constexpr (N == 4) {
    m = db_max(lim_lv(db_max(db_abs(t[0] - t[1]), db_abs(t[3] - t[2])), s), db_blim(t, s));
  } else if constexpr (N == 6) {
    m = db_max(lim_lv(db_max(db_max(db_abs(t[0] - t[1]), db_abs(t[1] - t[2])),
                             db_max(db_abs(t[5] - t[4]), db_abs(t[4] - t[3]))), s),
               db_blim(c, s));
    flat = db_max(db_max(db_abs(t[1] - t[2]), db_abs(t[4] - t[3])),
                  db_max(db_abs(t[0] - t[2]), db_abs(t[5] - t[3]))) <= fl;
  } else {
    const int32_t *in = N == 8 ? t : t + 3;
    m = db_max(lim_lv(db_max(db_max(db_max(db_abs(in[0] - in[1]), db_abs(in[1] - in[2])),
                                    db_abs(in[2] - in[3])),
                             db_max(db_max(db_abs(in[7] - in[6]), db_abs(in[6] - in[5])),
                                    db_abs(in[5] - in[4]))), s),
               db_blim(in + 2, s));
    flat = db_max(db_max(db_max(db_abs(in[2] - in[3]), db_abs(in[5] - in[4])),
                         db_max(db_abs(in[1] - in[3]), db_abs(in[6] - in[4]))),
                  db_max(db_abs(in[0] - in[3]), db_abs(in[7] - in[4]))) <= fl;
  }
  const int mask = m < 1 ? 1 : m > 64 ? 64 : m;
  int nhev = thr_lv(db_max(db_abs(c[0] - c[1]), db_abs(c[3] - c[2])), s);
  nhev = nhev < mask ? mask : nhev > 64 ? 64 : nhev;
  const int64_t none = sse_cmp<N>(t, a);
  int32_t v[N];
  d_idx[0] = 0;
  d_val[0] = none;
  d_idx[1] = mask;
  d_idx[2] = nhev;
  if (flat) {
    int64_t w = none;
    if (mask <= 63) {  // the wide filter: level 63 passes the mask, flatness picks it
#pragma unroll
      for (int i = 0; i < N; i++) v[i] = t[i];
      db_filter<N>(v, 63, bd);
      w = sse_cmp<N>(v, a);
    }
    d_val[1] = w - none;
    d_val[2] = 0;
  } else {
    int64_t n2 = none, n4 = none;
    if (nhev != mask) {
#pragma unroll
      for (int i = 0; i < N; i++) v[i] = t[i];
      db_narrow(v + ci, s, false);
      n2 = sse_cmp<N>(v, a);
    }
    if (nhev <= 63) {
#pragma unroll
      for (int i = 0; i < N; i++) v[i] = t[i];
      db_narrow(v + ci, s, true);
      n4 = sse_cmp<N>(v, a);
    }
    d_val[1] = n2 - none;
    d_val[2] = n4 - n2;
  }
}

template <typename Px, int N>
__device__ __forceinline__ void sse_gather(const SsePlane &P, int ox, int oy, int bd, int d_idx[3],
                                           int64_t d_val[3]) {
  int32_t t[N], a[N];
#pragma unroll
  for (int i = 0; i < N; i++) {
    t[i] = sse_px<Px>(P.rec, ox - N / 2 + i, oy);
    a[i] = sse_px<Px>(P.src, ox - N / 2 + i, oy);
  }
  sse_row<N>(t, a, bd, d_idx, d_val);
}

template <typename Px>
__global__ __launch_bounds__(256) void sse_tally_kernel(SseArgs a) {
  __shared__ unsigned long long lt[130];
  const SsePlane &P = a.pl[blockIdx.y];
  for (int i = threadIdx.x; i < 130; i += 256) lt[i] = 0;
  __syncthreads();
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int k = i & 3, seg = i >> 2;
  const int nv = P.nvx * P.nvy, nh = P.nhx * P.nhy;
  if (seg < nv + nh) {
    // sse_plane's walk (:1351-1406): vertical edges x >= 1 << xdec on every
    // row, horizontal edges y >= 1 << ydec on every column
    const bool vert = seg < nv;
    const int sg = vert ? seg : seg - nv, sx = vert ? P.nvx : P.nhx;
    const int gy = sg / sx, gx = sg - gy * sx;
    const int x = (gx + (vert ? 1 : 0)) << P.xdec, y = (gy + (vert ? 0 : 1)) << P.ydec;
    const int b = y * a.mi_stride + x;
    const int lgb = a.lg[b];
    const int pos = vert ? x : y, dec = vert ? P.xdec : P.ydec;
    const int px = (x | P.xdec) - (vert ? 1 << P.xdec : 0);
    const int py = (y | P.ydec) - (vert ? 0 : 1 << P.ydec);
    const int pb = py * a.mi_stride + px;
    if (((pos >> dec) & (db_tx_mi(lgb, P.pli, dec) - 1)) == 0 &&
        ((pos & ((1 << lgb) - 1)) == 0 || !a.skip[b] || !a.skip[pb])) {
      // both directions size the filter by width (sse_h_edge passes
      // vertical = true to deblock_size) and tally the row's horizontal taps
      const int tn = db_tx_mi(lgb, P.pli, P.xdec), tp = db_tx_mi(a.lg[pb], P.pli, P.xdec);
      int size = (tn < tp ? tn : tp) << 2;
      const int cap = P.pli == 0 ? 14 : 6;
      size = size < cap ? size : cap;
      const int ox = (x * 4) >> P.xdec, oy = ((y * 4) >> P.ydec) + k;
      int di[3];
      int64_t dv[3];
      if (size == 4)
        sse_gather<Px, 4>(P, ox, oy, a.bd, di, dv);
      else if (size == 6)
        sse_gather<Px, 6>(P, ox, oy, a.bd, di, dv);
      else if (size == 8)
        sse_gather<Px, 8>(P, ox, oy, a.bd, di, dv);
      else
        sse_gather<Px, 14>(P, ox, oy, a.bd, di, dv);
      const int base = vert ? 0 : 65;
#pragma unroll
      for (int j = 0; j < 3; j++)
        if (dv[j]) atomicAdd(&lt[base + di[j]], (unsigned long long)dv[j]);
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < 130; j += 256)
    if (lt[j]) atomicAdd((unsigned long long *)&a.tally[blockIdx.y * 130 + j], lt[j]);
}

// sse_optimize's choice (:1441-1473): prefix sums to MAX_LOOP_FILTER and the
// first minimum; luma per direction, chroma over both directions.  One lane
// per plane.
__global__ void sse_levels_kernel(const int64_t *tally, uint8_t *levels) {
  const int p = threadIdx.x;
  if (p >= 3) return;
  const int64_t *v = tally + p * 130, *h = v + 65;
  int64_t sv = 0, sh = 0, bvv = 0, bhv = 0, bcv = 0;
  int bv = 0, bh = 0, bc = 0;
  for (int i = 0; i < 64; i++) {
    sv += v[i];
    sh += h[i];
    if (i == 0 || bvv > sv) { bv = i; bvv = sv; }
    if (i == 0 || bhv > sh) { bh = i; bhv = sh; }
    if (i == 0 || bcv > sv + sh) { bc = i; bcv = sv + sh; }
  }
  if (p == 0) {
    levels[0] = (uint8_t)bv;
    levels[1] = (uint8_t)bh;
  } else {
    levels[p + 1] = (uint8_t)bc;
  }
}

}  // namespace rv

using namespace rv;

int rv_deblock_sse_dev(const rv_plane rec[3], const rv_plane src[3], int width, int height,
                       const uint8_t *d_lg, const uint8_t *d_skip, int mi_stride,
                       int64_t *d_tally, uint8_t *d_levels, int bit_depth, hipStream_t s) {
  SseArgs a;
  a.lg = d_lg;
  a.skip = d_skip;
  a.mi_stride = mi_stride;
  a.bd = bit_depth;
  a.tally = d_tally;
  const int cols = (width + 3) >> 2, rows = (height + 3) >> 2;  // sse_plane (:1347-1348)
  int64_t most = 0;
  for (int p = 0; p < 3; p++) {
    SsePlane &P = a.pl[p];
    P.rec = rec[p];
    P.src = src[p];
    P.pli = p;
    P.xdec = p ? rec[p].xdec : 0;
    P.ydec = p ? rec[p].ydec : 0;
    const int nx = (cols + (1 << P.xdec) - 1) >> P.xdec;  // x = 0, 1 << xdec, .. < cols
    const int ny = (rows + (1 << P.ydec) - 1) >> P.ydec;
    P.nvx = nx - 1 > 0 ? nx - 1 : 0;
    P.nvy = ny;
    P.nhx = nx;
    P.nhy = ny - 1 > 0 ? ny - 1 : 0;
    const int64_t n = ((int64_t)P.nvx * P.nvy + (int64_t)P.nhx * P.nhy) * 4;
    most = n > most ? n : most;
  }
  if (hipMemsetAsync(d_tally, 0, 3 * 130 * sizeof(int64_t), s) != hipSuccess)
    return rv_set_error(RV_EHIP, "rv_deblock_sse: hipMemsetAsync");
  if (most > 0) {
    const dim3 grid((unsigned)((most + 255) / 256), 3);
    if (rec[0].hbd)
      sse_tally_kernel<uint16_t><<<grid, 256, 0, s>>>(a);
    else
      sse_tally_kernel<uint8_t><<<grid, 256, 0, s>>>(a);
  }
  sse_levels_kernel<<<1, 64, 0, s>>>(d_tally, d_levels);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

// One pass of the deblocking over planes pl[0 .. np) in one launch (the
// passes of different planes touch different memory).  levels: the host
// levels [Y v, Y h, U, V] (a plane whose level is 0 is left out), or null
// with d_levels the device ones (every lane reads its level).
static int deblock_pass(const rv_plane *planes, const int *pli, int np, int width, int height,
                        const uint8_t *d_lg, const uint8_t *d_skip, int mi_stride,
                        const uint8_t *levels, const uint8_t *d_levels, int bit_depth, bool vert,
                        hipStream_t s) {
  DbPlanes P = {};
  unsigned blocks = 0;
  int k = 0;
  for (int j = 0; j < np; j++) {
    const rv_plane *p = &planes[j];
    DbArgs &a = P.pl[k];
    a.p = *p;
    a.lg = d_lg;
    a.skip = d_skip;
    a.dlev = levels ? nullptr : d_levels;
    a.mi_stride = mi_stride;
    a.xdec = p->xdec;
    a.ydec = p->ydec;
    a.cols = ((((width + 3) >> 2) + ((1 << a.xdec) >> 1)) >> a.xdec) << a.xdec;
    a.rows = ((((height + 3) >> 2) + ((1 << a.ydec) >> 1)) >> a.ydec) << a.ydec;
    a.pli = pli[j];
    a.bd = bit_depth;
    a.vert = vert;
    a.level = levels ? (a.pli == 0 ? levels[vert ? 0 : 1] : levels[a.pli + 1]) : 0;
    if (levels && a.level == 0) continue;
    const int sx = vert ? (a.cols >> a.xdec) - 1 : (a.cols >> a.xdec);
    const int sy = vert ? (a.rows >> a.ydec) : (a.rows >> a.ydec) - 1;
    const int64_t n = (int64_t)(sx > 0 ? sx : 0) * (sy > 0 ? sy : 0) * 4;
    if (n == 0) continue;
    P.blk[k] = blocks;
    blocks += (unsigned)((n + 255) / 256);
    k++;
  }
  for (int j = k; j < 4; j++) P.blk[j] = blocks;
  if (!blocks) return RV_OK;
  if (planes[0].hbd)
    deblock_kernel<uint16_t><<<blocks, 256, 0, s>>>(P);
  else
    deblock_kernel<uint8_t><<<blocks, 256, 0, s>>>(P);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

// deblock_filter_frame (src/deblock.rs:1337-1345 via src/encoder.rs:
// 2789-2793) of a frame's three planes: all vertical edges, then all
// horizontal ones, each pass one launch over the planes.  d_levels: the
// device levels (sse_optimize's; nothing is filtered unless a luma level is
// non-zero, every lane reads its level) or, with levels, the host ones.
int rv_deblock_frame_dev(const rv_plane planes[3], int width, int height, const uint8_t *d_lg,
                         const uint8_t *d_skip, int mi_stride, const uint8_t *d_levels,
                         int bit_depth, hipStream_t s, const uint8_t *levels) {
  static const int pli[3] = {0, 1, 2};
  for (int pass = 0; pass < 2; pass++)
    if (const int e = deblock_pass(planes, pli, 3, width, height, d_lg, d_skip, mi_stride, levels,
                                   d_levels, bit_depth, pass == 0, s))
      return e;
  return RV_OK;
}

// The deblocking of one plane (pli 0 = Y, 1 = U, 2 = V) of a frame of
// width x height luma pixels; lg / skip per luma 4x4 block (row pitch
// mi_stride >= the frame's 4x4 columns, device memory); levels = the
// DeblockState levels [Y vertical, Y horizontal, U, V].
int rv_deblock_plane_dev(const rv_plane *p, int pli, int width, int height, const uint8_t *d_lg,
                         const uint8_t *d_skip, int mi_stride, const uint8_t levels[4],
                         int bit_depth, hipStream_t s) {
  for (int pass = 0; pass < 2; pass++)
    if (const int e = deblock_pass(p, &pli, 1, width, height, d_lg, d_skip, mi_stride, levels,
                                   nullptr, bit_depth, pass == 0, s))
      return e;
  return RV_OK;
}

extern "C" int rv_deblock_plane(const rv_plane *plane, int pli, int width, int height,
                                const uint8_t *d_lg, const uint8_t *d_skip, int mi_stride,
                                const uint8_t *levels, int bit_depth, void *stream) {
  if (!plane || !levels || pli < 0 || pli > 2 || width <= 0 || height <= 0 || !d_lg || !d_skip ||
      mi_stride < (width + 3) / 4 || (bit_depth != 8 && bit_depth != 10 && bit_depth != 12) ||
      (plane->hbd != (bit_depth > 8)))
    return rv_set_error(RV_EINVAL, "rv_deblock_plane: bad arguments");
  return rv_deblock_plane_dev(plane, pli, width, height, d_lg, d_skip, mi_stride, levels,
                              bit_depth, rv_resolve_stream(stream));
}

extern "C" int rv_deblock_sse(const rv_plane *rec, const rv_plane *src, int width, int height,
                              const uint8_t *d_lg, const uint8_t *d_skip, int mi_stride,
                              int64_t *d_tally, uint8_t *d_levels, int bit_depth, void *stream) {
  bool ok = rec && src && width > 0 && height > 0 && d_lg && d_skip && d_tally && d_levels &&
            mi_stride >= (width + 3) / 4 && (bit_depth == 8 || bit_depth == 10 || bit_depth == 12);
  for (int p = 0; ok && p < 3; p++)
    ok = rec[p].hbd == (bit_depth > 8) && src[p].hbd == rec[p].hbd &&
         rec[p].width == src[p].width && rec[p].height == src[p].height &&
         (p == 0 ? !rec[0].xdec && !rec[0].ydec
                 : rec[p].xdec == rec[1].xdec && rec[p].ydec == rec[1].ydec) &&
         rec[p].width == (width + (p ? rec[p].xdec : 0)) >> (p ? rec[p].xdec : 0) &&
         rec[p].height == (height + (p ? rec[p].ydec : 0)) >> (p ? rec[p].ydec : 0);
  if (!ok) return rv_set_error(RV_EINVAL, "rv_deblock_sse: bad arguments");
  return rv_deblock_sse_dev(rec, src, width, height, d_lg, d_skip, mi_stride, d_tally, d_levels,
                            bit_depth, rv_resolve_stream(stream));
}

extern "C" int rv_deblock_frame(const rv_plane *planes, int width, int height, const uint8_t *d_lg,
                                const uint8_t *d_skip, int mi_stride, const uint8_t *d_levels,
                                int bit_depth, void *stream) {
  bool ok = planes && width > 0 && height > 0 && d_lg && d_skip && d_levels &&
            mi_stride >= (width + 3) / 4 && (bit_depth == 8 || bit_depth == 10 || bit_depth == 12);
  for (int p = 0; ok && p < 3; p++) ok = planes[p].hbd == (bit_depth > 8);
  if (!ok) return rv_set_error(RV_EINVAL, "rv_deblock_frame: bad arguments");
  return rv_deblock_frame_dev(planes, width, height, d_lg, d_skip, mi_stride, d_levels, bit_depth,
                              rv_resolve_stream(stream), nullptr);
}

// deblock_filter_optimize's fast path (src/deblock.rs:1477-1517, speed >=
// 8): the level of every plane and direction from the frame's ac quantizer
extern "C" int rv_deblock_fast_level(int ac_q, int bit_depth, int is_key) {
  int v;
  if (bit_depth == 8)
    v = is_key ? (ac_q * 17563 - 421574 + (1 << 17)) >> 18 : (ac_q * 6017 + 650707 + (1 << 17)) >> 18;
  else if (bit_depth == 10)
    v = ((ac_q * 20723 + 4060632 + (1 << 19)) >> 20) - (is_key ? 4 : 0);
  else
    v = ((ac_q * 20723 + 16242526 + (1 << 21)) >> 22) - (is_key ? 4 : 0);
  return v < 0 ? 0 : v > 63 ? 63 : v;
}
