// lrf_bench.hip -- loop restoration's decision kernels alone on a 2160p
// 4:2:0 8-bit frame of synthetic content: the per-unit distortion kernel's
// duration (full grid, HIP events) and one workgroup's phase clocks.
// Build (tools/ubench/Makefile):  hipcc -DLRF_PHASES=... includes the
// kernel source so the harness launches it directly.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#include "../../rav1e_amd/csrc/rv_lrf.hip"

extern "C" int rv_cdef_find_dirs(const rv_plane *luma, int width, int height, const uint8_t *d_skip,
                                 int mi_stride, uint8_t *d_dir, int32_t *d_var, int bit_depth, void *stream);

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

static rv_plane plane(int w, int h, int xdec, int ydec, unsigned seed) {
  rv_plane p{};
  const int pad = 80;
  p.stride = w + 2 * pad;
  p.alloc_height = h + 2 * pad;
  p.width = w;
  p.height = h;
  p.xorigin = pad;
  p.yorigin = pad;
  p.xdec = xdec;
  p.ydec = ydec;
  p.hbd = 0;
  p.bit_depth = 8;
  std::vector<uint8_t> v((size_t)p.stride * p.alloc_height);
  srand(seed);
  for (int y = 0; y < p.alloc_height; y++)
    for (int x = 0; x < p.stride; x++) {
      int t = 96 + ((x * 3 + y * 2) >> 4) % 64 + (rand() % 17) - 8 + (((x >> 5) ^ (y >> 5)) & 1) * 30;
      v[(size_t)y * p.stride + x] = (uint8_t)(t < 0 ? 0 : t > 255 ? 255 : t);
    }
  CK(hipMalloc(&p.data, v.size()));
  CK(hipMemcpy(p.data, v.data(), v.size(), hipMemcpyHostToDevice));
  return p;
}

int main(int argc, char **argv) {
  const int W = 3840, H = 2160, reps = argc > 1 ? atoi(argv[1]) : 5;
  rv_plane rec[3], src[3];
  for (int p = 0; p < 3; p++) {
    const int d = p ? 1 : 0;
    rec[p] = plane(W >> d, H >> d, d, d, 1 + p);
    src[p] = plane(W >> d, H >> d, d, d, 11 + p);
  }
  LrfGeo g;
  if (lrf_geometry(W, H, 1, 1, 8, 100, 8, 34, &g) != RV_OK) return 1;
  const int mi_stride = W / 4 + 8;
  uint8_t *skip;
  CK(hipMalloc(&skip, (size_t)mi_stride * (H / 4 + 8)));
  CK(hipMemset(skip, 0, (size_t)mi_stride * (H / 4 + 8)));
  uint64_t *err;
  int8_t *xqd, *units;
  CK(hipMalloc(&err, sizeof(uint64_t) * 3 * g.nsb * 17));
  CK(hipMalloc(&xqd, 3 * g.nsb * 32));
  CK(hipMalloc(&units, 3 * g.urows_max * g.ucols_max * 3));
  uint8_t *dir;
  int32_t *var;
  const int n8 = (W / 8) * (H / 8);
  CK(hipMalloc(&dir, n8));
  CK(hipMalloc(&var, n8 * 4));
  if (rv_cdef_find_dirs(&rec[0], W, H, skip, mi_stride, dir, var, 8, nullptr) != RV_OK) return 1;
  LrfRdoArgs a;
  memset(&a, 0, sizeof(a));
  for (int p = 0; p < 3; p++) {
    a.rec[p] = rec[p];
    a.src[p] = src[p];
    a.ds[p] = 1.0;
  }
  a.skip = skip;
  a.mi_stride = mi_stride;
  a.g = g;
  a.cdef = 1;
  a.gx1 = g.sbc;
  a.gy1 = g.sbr;
  a.dir = dir;
  a.var = var;
  a.dstride = W / 8;
  a.pri_y = 2;
  a.sec_y = 1;
  a.pri_uv = 1;
  a.sec_uv = 1;
  a.damping = 3;
  a.err = err;
  a.xqd = xqd;
  LrfDecideArgs d;
  d.g = g;
  d.err = err;
  d.xqd = xqd;
  d.lambda = 300.0;
  d.units = units;
  d.fix_passes = kFixIter;
  d.gx0 = d.gy0 = 0;
  d.gx1 = g.sbc;
  d.gy1 = g.sbr;
  const int nt = ((g.sbc + g.tws - 1) / g.tws) * ((g.sbr + g.ths - 1) / g.ths);
  hipEvent_t e0, e1, e2, em;
  CK(hipEventCreate(&em));
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&e2));
  if (lrf_lut_upload() != RV_OK) return 1;
  for (int r = 0; r < reps; r++) {
    CK(hipEventRecord(e0, 0));
    a.p0 = 0;
    if (r & 1)  // odd reps: the 1024-lane luma kernel (RAV1E_LRF_WIDE=0)
      lrf_rdo_kernel<uint8_t, 64, 64><<<dim3(g.nsb, 1), 1024>>>(a);
    else
      lrf_rdo_wide_kernel<uint8_t><<<dim3(g.nsb, 1), 512>>>(a);
    CK(hipEventRecord(em, 0));
    a.p0 = 1;
    lrf_rdo_kernel<uint8_t, 32, 32><<<dim3(g.nsb, 2), 256>>>(a);
    CK(hipEventRecord(e1, 0));
    if (r & 1)
      lrf_decide_kernel<<<nt, 64>>>(d);
    else
      lrf_decide_fix_kernel<<<nt, kFixThreads>>>(d);
    CK(hipEventRecord(e2, 0));
    CK(hipEventSynchronize(e2));
    float t1, t2;
    CK(hipEventElapsedTime(&t1, e0, e1));
    CK(hipEventElapsedTime(&t2, e1, e2));
    float tl;
    CK(hipEventElapsedTime(&tl, e0, em));
    printf("rep %d (%s luma, %s decision): rdo %.3f ms (luma %.3f; %d x 3 workgroups), decide %.3f ms (%d tiles)\n",
           r, r & 1 ? "1024-lane" : "512-lane", r & 1 ? "serial" : "fixed-point", t1, tl, g.nsb, t2, nt);
    {  // the distortions and solutions, hashed (compare builds)
      std::vector<uint64_t> he((size_t)3 * g.nsb * 17);
      std::vector<int8_t> hx((size_t)3 * g.nsb * 32);
      CK(hipMemcpy(he.data(), err, he.size() * 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hx.data(), xqd, hx.size(), hipMemcpyDeviceToHost));
      uint64_t h = 1469598103934665603ull;
      for (uint64_t v : he) h = (h ^ v) * 1099511628211ull;
      for (int8_t v : hx) h = (h ^ (uint8_t)v) * 1099511628211ull;
      printf("  err/xqd hash %016llx\n", (unsigned long long)h);
    }
    // the two decisions agree unit for unit
    static std::vector<int8_t> prev;
    std::vector<int8_t> cur((size_t)3 * g.urows_max * g.ucols_max * 3);
    CK(hipMemcpy(cur.data(), units, cur.size(), hipMemcpyDeviceToHost));
    if (!prev.empty()) {
      size_t bad = 0;
      for (size_t i = 0; i < cur.size(); i++) bad += cur[i] != prev[i];
      printf("  units vs the previous rep's decision: %zu of %zu bytes differ\n", bad, cur.size());
    }
    prev = cur;
  }
#ifdef LRF_PHASES
  {  // the fixed point's passes (the last rep with it)
    lrf_decide_fix_kernel<<<nt, kFixThreads>>>(d);
    CK(hipDeviceSynchronize());
    int st[8], tr[8][kFixIter];
    CK(hipMemcpyFromSymbol(st, HIP_SYMBOL(lrf_fix_stats), sizeof(st)));
    CK(hipMemcpyFromSymbol(tr, HIP_SYMBOL(lrf_fix_trace), sizeof(tr)));
    unsigned long long ck[40];
    CK(hipMemcpyFromSymbol(ck, HIP_SYMBOL(lrf_fix_clk), sizeof(ck)));
    printf("  tile 0 clocks (us): setup %.2f", (ck[1] - ck[0]) / 100.0);
    for (int j = 0; j < 3; j++)
      printf(" | pass %d: decide %.2f states %.2f", j, (ck[3 + 3 * j] - ck[2 + 3 * j]) / 100.0,
             (ck[4 + 3 * j] - ck[3 + 3 * j]) / 100.0);
    printf(" | total %.2f\n", (ck[39] - ck[0]) / 100.0);
    for (int i = 0; i < 8 && i < nt; i++) {
      printf("  tile %d: %s at %d; first change per pass:", i, st[i] >= 1000 ? "fell back" : "settled",
             st[i] % 1000);
      for (int j = 0; j < kFixIter; j++) printf(" %d", tr[i][j]);
      printf("\n");
    }
  }
  // one workgroup alone: its phases in wall_clock64 ticks (100 MHz)
  a.p0 = 0;
  if (getenv("LRF_BENCH_OLD"))
    lrf_rdo_kernel<uint8_t, 64, 64><<<dim3(LRF_PHASES + 1, 1), 1024>>>(a);
  else
    lrf_rdo_wide_kernel<uint8_t><<<dim3(LRF_PHASES + 1, 1), 512>>>(a);
  CK(hipDeviceSynchronize());
  unsigned long long t[96];
  CK(hipMemcpyFromSymbol(t, HIP_SYMBOL(lrf_phase_t), sizeof(t)));
  printf("one workgroup (unit %d, luma), us:\n", LRF_PHASES);
  const char *names[6] = {"start", "pad+lin", "cdef", "integral", "pixels", "boxes/tables0+none"};  // (stamps before barriers)
  for (int k = 1; k < 6; k++) printf("  %-12s %8.2f\n", names[k], (t[k] - t[k - 1]) / 100.0);
  for (int s = 0; s < 16; s++) {
    const unsigned long long *q = t + 6 + 5 * s, prev = s ? q[-1] : t[5];
    printf("  set %2d: tables %6.2f f+sums %6.2f solve %6.2f out %6.2f err %6.2f\n", s, (q[0] - prev) / 100.0,
           (q[1] - q[0]) / 100.0, (q[2] - q[1]) / 100.0, (q[3] - q[2]) / 100.0, (q[4] - q[3]) / 100.0);
  }
  printf("  total %8.2f\n", (t[6 + 5 * 15 + 4] - t[0]) / 100.0);
  unsigned long long dp[5];
  CK(hipMemcpyFromSymbol(dp, HIP_SYMBOL(lrf_dphase), sizeof(dp)));
  printf("decide, tile 0, shader clocks per step: wait+loads %.0f rate %.0f min+picks %.0f stores %.0f commit %.0f\n",
         dp[0] / 272.0, dp[1] / 272.0, dp[2] / 272.0, dp[3] / 272.0, dp[4] / 272.0);
#endif
  return 0;
}
