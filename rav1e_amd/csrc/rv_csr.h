// rv_csr.h -- stable grouping of (target, entry) pairs by target, hand-written
// for gfx950 (the importance propagation's target lists, rv_impwin.hip and
// rv_lookahead.hip).
//
// compute_block_importances (src/api/internal.rs:823-1081) adds every
// source block's four contributions into the target blocks with f32 `+=` in
// source raster order, so each target needs its entries in ascending entry
// order (entry j = 4 * source + corner).  The keys are bounded block indices
// (0 .. n, n = "off the frame"), so a counting sort fits:
//   count    the producer kernel adds 1 to cnt[key] for every valid entry;
//   scan     off[t] = the exclusive prefix sum of cnt, cur[t] = off[t] (one
//            workgroup per 4096 targets, each adding up its own carry);
//   scatter  entry j goes to src[atomicAdd(&cur[key], 1)]: grouped, but in
//            arrival order;
//   order    one thread per target sorts its (short) list ascending, which is
//            the source order a stable sort would keep.
// Three launches per frame after the producer, every reference of the frame
// in the same launches (blockIdx.y / blockIdx.x = the set).
#pragma once

#include "rv_device.h"

namespace rv {
namespace {  // each including file gets its own kernels

constexpr int kCsrScanThreads = 1024;

// cnt / cur: [sets][n] (stride n); off: [sets][n + 1].  Workgroup (chunk,
// set) scans counts [chunk * kCsrTile, +kCsrTile), four per lane; its carry
// is the sum of the counts before the chunk, which it adds up itself (L2
// reads, no second launch): the scan is one launch of n / 4096 x sets
// workgroups instead of one serial workgroup per set.
constexpr int kCsrTile = 4 * kCsrScanThreads;
__global__ __launch_bounds__(kCsrScanThreads) void csr_scan_kernel(const int32_t *cnt, int32_t *cur,
                                                                   int32_t *off, int n) {
  const int set = blockIdx.y, base = blockIdx.x * kCsrTile;
  const int32_t *c = cnt + (size_t)set * n;
  int32_t *cu = cur + (size_t)set * n;
  int32_t *o = off + (size_t)set * (n + 1);
  __shared__ int32_t wsum[kCsrScanThreads / 64];
  __shared__ int32_t wpre[kCsrScanThreads / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int32_t pre = 0;
  for (int i = threadIdx.x; i < base; i += kCsrScanThreads) pre += c[i];
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) pre += __shfl_xor(pre, d, 64);
  const int t0 = base + 4 * threadIdx.x;
  int32_t v[4];
#pragma unroll
  for (int u = 0; u < 4; u++) v[u] = t0 + u < n ? c[t0 + u] : 0;
  const int32_t mine = v[0] + v[1] + v[2] + v[3];
  int32_t inc = mine;  // inclusive scan over the wavefront
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int32_t y = __shfl_up(inc, d, 64);
    if (lane >= d) inc += y;
  }
  if (lane == 63) {
    wsum[wave] = inc;
    wpre[wave] = pre;
  }
  __syncthreads();
  int32_t before = 0;
  for (int w = 0; w < kCsrScanThreads / 64; w++) {
    before += wpre[w];
    if (w < wave) before += wsum[w];
  }
  int32_t run = before + inc - mine;
#pragma unroll
  for (int u = 0; u < 4; u++)
    if (t0 + u < n) {
      o[t0 + u] = run;
      cu[t0 + u] = run;
      run += v[u];
    }
  if (t0 < n && t0 + 4 >= n) o[n] = run;  // the lane holding the last count
}

// entries [sets][m] with keys[set * m + j] (n: none): j goes to its
// target's group in src[set * m + ...] (arrival order)
__global__ __launch_bounds__(256) void csr_scatter_kernel(const uint32_t *keys, int m, int n,
                                                          int32_t *cur, int32_t *src) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  const int set = blockIdx.y;
  if (j >= m) return;
  const uint32_t k = keys[(size_t)set * m + j];
  if (k >= (uint32_t)n) return;
  const int pos = atomicAdd(cur + (size_t)set * n + k, 1);
  src[(size_t)set * m + pos] = j;
}

// each target's list ascending (insertion sort: a target holds a handful of
// entries -- the sources whose displaced block overlaps it)
__global__ __launch_bounds__(256) void csr_order_kernel(const int32_t *off, int n, int m,
                                                        int32_t *src) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int set = blockIdx.y;
  if (t >= n) return;
  const int32_t *o = off + (size_t)set * (n + 1);
  int32_t *s = src + (size_t)set * m;
  const int a = o[t], b = o[t + 1];
  for (int i = a + 1; i < b; i++) {
    const int32_t v = s[i];
    int j = i - 1;
    while (j >= a && s[j] > v) {
      s[j + 1] = s[j];
      j--;
    }
    s[j + 1] = v;
  }
}

// After the producer counted (cnt zeroed before it ran): off / src of `sets`
// sets of m entries over n targets.
inline int csr_build(const uint32_t *keys, int m, int n, int sets, int32_t *cnt, int32_t *cur,
                     int32_t *off, int32_t *src, hipStream_t st) {
  csr_scan_kernel<<<dim3((unsigned)((n + kCsrTile - 1) / kCsrTile), (unsigned)sets),
                    kCsrScanThreads, 0, st>>>(cnt, cur, off, n);
  RV_HIP_CHECK_LAUNCH();
  csr_scatter_kernel<<<dim3((unsigned)((m + 255) / 256), (unsigned)sets), 256, 0, st>>>(
      keys, m, n, cur, src);
  RV_HIP_CHECK_LAUNCH();
  csr_order_kernel<<<dim3((unsigned)((n + 255) / 256), (unsigned)sets), 256, 0, st>>>(off, n, m,
                                                                                      src);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

}  // namespace
}  // namespace rv
