// rv_impwin.hip -- the lookahead window's block importances
// (compute_block_importances, src/api/internal.rs:823-1081); see
// rv_impwin.h for the decomposition.  f32 arithmetic in the reference's
// operation order: products and sums round separately (-ffp-contract=off),
// divisions are correctly rounded (__fdiv_rn), as in Rust.
#include <string.h>

#include "rv_csr.h"
#include "rv_impwin.h"

namespace rv {

namespace {

constexpr int kImpB = 8, kMvUnits = 8, kBMv = kImpB * kMvUnits, kAreaMv = kBMv * kBMv;

size_t al256(size_t v) { return (v + 255) & ~(size_t)255; }

// impwin_lists' scratch: the entries' keys [R][4 n], the per-target
// counts and cursors [R][n] (rv_csr.h)
struct CsrScratch {
  size_t keys, cnt, cur, total;
};

CsrScratch csr_scratch(int n) {
  CsrScratch s;
  const size_t m = 4 * (size_t)n;
  s.keys = 0;
  s.cnt = al256(s.keys + 4 * m * kImpMaxRefs);
  s.cur = al256(s.cnt + 4 * (size_t)n * kImpMaxRefs);
  s.total = al256(s.cur + 4 * (size_t)n * kImpMaxRefs);
  return s;
}

// The four targets of a source block at (x, y) with lookahead MV mv (MV
// units): target block index (n: off the frame) and area fraction, in the
// order top-left, top-right, bottom-left, bottom-right (:967-1043).
__device__ inline void corners(int x, int y, rv_mv mv, int w, int h, int tgt[4], float f[4]) {
  const int64_t rx = (int64_t)x * kBMv + mv.col, ry = (int64_t)y * kBMv + mv.row;
  // (reference_x - (BLOCK - 1 if negative)) / BLOCK * BLOCK: i64 `/` truncates
  const int64_t tlx = (rx - (rx < 0 ? kBMv - 1 : 0)) / kBMv * kBMv;
  const int64_t tly = (ry - (ry < 0 ? kBMv - 1 : 0)) / kBMv * kBMv;
  const int64_t trx = tlx + kBMv, bly = tly + kBMv;
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const int64_t tx = (c & 1) ? trx : tlx, ty = (c & 2) ? bly : tly;
    const int64_t fx = (c & 1) ? rx + kBMv - trx : trx - rx;
    const int64_t fy = (c & 2) ? ry + kBMv - bly : bly - ry;
    f[c] = __fdiv_rn((float)(fx * fy), (float)kAreaMv);
    const int64_t bx = tx / kBMv, by = ty / kBMv;
    tgt[c] = bx >= 0 && by >= 0 && bx < w && by < h ? (int)(by * w + bx) : w * h;
  }
}

template <typename Px>
__device__ inline uint32_t satd8(const Px *o, int64_t os, const Px *r, int64_t rs, int base) {
  int32_t d[64];
#pragma unroll
  for (int rr = 0; rr < 8; rr++)
#pragma unroll
    for (int cc = 0; cc < 8; cc++)
      d[rr * 8 + cc] = (int32_t)o[rr * os + cc] - (r ? (int32_t)r[rr * rs + cc] : base);
  return (uint32_t)((satd_chunk<8>(d) + 4) >> 3);  // get_satd 8x8: ln = msb(8)
}

// One thread per 8x8 block of the group's rectangle and reference
// (blockIdx.y): lookahead_intra_costs (pred_dc_128, :680-765; reference 0
// stores them), the lookahead MV of the 16x16 holding the block, get_satd
// against the reference's original block at that MV (:911-931) and the
// propagate fraction (:939).  A block whose reference region would leave
// the allocation (the reference would panic; the search windows prevent
// it) gets fraction 0.
struct DataArgs {
  rv_plane cur, ref[kImpMaxRefs];
  int base, w, h;       // the frame's 8x8 blocks
  int bx0, by0, bw, bh; // the group's blocks
  int tx0, ty0, tw, nsb;  // the group's superblocks (look is [R][nsb][16] over them)
  const rv_fs_result *look;
  ImpFrame f;
};

template <typename Px>
__global__ __launch_bounds__(256) void data_kernel(DataArgs a) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  const int k = blockIdx.y;
  if (j >= a.bw * a.bh) return;
  const int n = a.w * a.h;
  const int x = a.bx0 + j % a.bw, y = a.by0 + j / a.bw, i = y * a.w + x;
  const Px *o = plane_ptr<Px>(a.cur, x * kImpB, y * kImpB);
  const uint32_t intra = satd8<Px>(o, a.cur.stride, (const Px *)nullptr, 0, a.base);
  if (k == 0) a.f.intra[i] = intra;
  const int sb = (y / 8 - a.ty0) * a.tw + x / 8 - a.tx0, b = ((y % 8) / 2) * 4 + (x % 8) / 2;
  const rv_plane &ref = a.ref[k];
  const rv_mv mv = a.look[((size_t)k * a.nsb + sb) * 16 + b].best_mv;
  a.f.mv8[(size_t)k * n + i] = mv;
  const int64_t px_x = ((int64_t)x * kBMv + mv.col) / kMvUnits;  // isize `/`
  const int64_t px_y = ((int64_t)y * kBMv + mv.row) / kMvUnits;
  const bool inside = px_x >= -ref.xorigin && px_y >= -ref.yorigin &&
                      px_x + kImpB <= ref.stride - ref.xorigin &&
                      px_y + kImpB <= ref.alloc_height - ref.yorigin;
  float frac = 0.f;
  if (inside) {
    const float inter = (float)satd8<Px>(o, a.cur.stride, plane_ptr<Px>(ref, (int)px_x, (int)px_y),
                                         ref.stride, 0);
    // f32::max(NaN, 0) = 0, as fmaxf
    frac = fmaxf(1.0f - __fdiv_rn(inter, (float)intra), 0.0f);
  }
  a.f.frac[(size_t)k * n + i] = frac;
}

// One thread per 8x8 block of the frame and reference (blockIdx.y): its four
// (target, 4 * block + corner) entries, counted per target.  A block with
// fraction 0 adds exactly +0.0f to each target (its amount is +0 and every
// importance is >= +0), which leaves the target unchanged, so it is not
// listed: the lists hold the blocks that change something.
__global__ __launch_bounds__(256) void keys_kernel(ImpFrame f, int w, int h, uint32_t *keys,
                                                   int32_t *cnt) {
  const int n = w * h;
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int k = blockIdx.y;
  if (i >= n) return;
  const bool live = f.frac[(size_t)k * n + i] > 0.f;
  int tgt[4];
  float fr[4];
  corners(i % w, i / w, f.mv8[(size_t)k * n + i], w, h, tgt, fr);
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const uint32_t key = live ? (uint32_t)tgt[c] : (uint32_t)n;
    keys[(size_t)k * 4 * n + 4 * (size_t)i + c] = key;
    if (key < (uint32_t)n) atomicAdd(cnt + (size_t)k * n + key, 1);
  }
}

// A group's part of the frame data for the exchange (multi-group runs): per
// block of the rectangle in raster order the intra cost, then per reference
// slot k < 3 the MV and the fraction (kImpPartBytes).  unpack: the reverse.
__global__ __launch_bounds__(256) void part_kernel(ImpFrame f, int w, int h, int R, int bx0,
                                                   int by0, int bw, int bh, uint32_t *buf,
                                                   int unpack) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= bw * bh) return;
  const int n = w * h;
  const size_t i = (size_t)(by0 + j / bw) * w + bx0 + j % bw;
  uint32_t *p = buf + (size_t)j * (kImpPartBytes / 4);
  if (!unpack) {
    p[0] = f.intra[i];
#pragma unroll
    for (int k = 0; k < kImpMaxRefs; k++) {
      const bool on = k < R;
      rv_mv mv = on ? f.mv8[(size_t)k * n + i] : rv_mv{0, 0};
      uint32_t mw;
      __builtin_memcpy(&mw, &mv, 4);
      p[1 + 2 * k] = mw;
      p[2 + 2 * k] = on ? __float_as_uint(f.frac[(size_t)k * n + i]) : 0u;
    }
  } else {
    f.intra[i] = p[0];
    for (int k = 0; k < R; k++) {
      rv_mv mv;
      const uint32_t mw = p[1 + 2 * k];
      __builtin_memcpy(&mv, &mw, 4);
      f.mv8[(size_t)k * n + i] = mv;
      f.frac[(size_t)k * n + i] = __uint_as_float(p[2 + 2 * k]);
    }
  }
}

// One window pass: target t of the reference frame adds its sources'
// contributions in source order (:936-963).  blockIdx.y picks one of the
// launch's passes: a source frame's passes into its distinct references
// write different frames and read only the source, so they share a launch.
struct PassSet {
  const uint32_t *intra;
  const float *imp;
  const rv_mv *mv8[kImpMaxRefs];
  const float *frac[kImpMaxRefs];
  const int32_t *off[kImpMaxRefs], *src[kImpMaxRefs];
  float *ref_imp[kImpMaxRefs];
  int nu;
};
__global__ __launch_bounds__(256) void pass_kernel(PassSet p, int w, int h) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= w * h) return;
  const int y = blockIdx.y;
  const int32_t *off = p.off[y], *src = p.src[y];
  const rv_mv *mv8 = p.mv8[y];
  const float *frac = p.frac[y];
  const int j0 = off[t], j1 = off[t + 1];
  if (j0 == j1) return;
  float *ref_imp = p.ref_imp[y];
  float acc = ref_imp[t];
  for (int j = j0; j < j1; j++) {
    const int e = src[j], s = e >> 2, c = e & 3;
    const float ic = (float)p.intra[s];
    const float amount = __fdiv_rn((ic + p.imp[s]) * frac[s], (float)p.nu);
    int tgt[4];
    float fr[4];
    corners(s % w, s / w, mv8[s], w, h, tgt, fr);
    acc = acc + amount * fr[c];
  }
  ref_imp[t] = acc;
}

// The window's frames' propagated importances to zero, up to 64 frames a launch
struct ZeroSet {
  float *p[64];
};
__global__ __launch_bounds__(256) void zero_kernel(ZeroSet z, int n) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t < n) z.p[blockIdx.y][t] = 0.f;
}

// f32::log2 as the reference gets it on x86-64 Linux: glibc's log2f
// (sysdeps/ieee754/flt-32/e_log2f.c, its published algorithm, the FMA
// build), restated in oracle/orc_lookahead.c orc_log2f and pinned there
// against the host's log2f over every float in [1, 2) and a stride of the
// rest.  x >= 1 here (1 + importance / intra cost); +inf passes through.
__constant__ double kLog2fT[16][2] = {
    {0x1.661ec79f8f3bep+0, -0x1.efec65b963019p-2}, {0x1.571ed4aaf883dp+0, -0x1.b0b6832d4fca4p-2},
    {0x1.49539f0f010b0p+0, -0x1.7418b0a1fb77bp-2}, {0x1.3c995b0b80385p+0, -0x1.39de91a6dcf7bp-2},
    {0x1.30d190c8864a5p+0, -0x1.01d9bf3f2b631p-2}, {0x1.25e227b0b8ea0p+0, -0x1.97c1d1b3b7af0p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.2f9e393af3c9fp-3}, {0x1.12358f08ae5bap+0, -0x1.960cbbf788d5cp-4},
    {0x1.0953f419900a7p+0, -0x1.a6f9db6475fcep-5}, {0x1.0000000000000p+0, 0x0.0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.338ca9f24f53dp-4}, {0x1.ca4b31f026aa0p-1, 0x1.476a9543891bap-3},
    {0x1.b2036576afce6p-1, 0x1.e840b4ac4e4d2p-3}, {0x1.9c2d163a1aa2dp-1, 0x1.40645f0c6651cp-2},
    {0x1.886e6037841edp-1, 0x1.88e9c2c1b9ff8p-2}, {0x1.767dcf5534862p-1, 0x1.ce0a44eb17bccp-2}};
__constant__ double kLog2fA[4] = {-0x1.712b6f70a7e4dp-2, 0x1.ecabf496832e0p-2,
                                  -0x1.715479ffae3dep-1, 0x1.715475f35c8b8p+0};

__device__ inline float log2f_ref(float x) {
  const uint32_t ix = __float_as_uint(x);
  if (ix == 0x3f800000u) return 0.0f;
  if (ix >= 0x7f800000u) return x;  // +inf / NaN
  const uint32_t tmp = ix - 0x3f330000u;
  const int i = (int)((tmp >> 19) % 16);
  const uint32_t iz = ix - (tmp & 0xff800000u);
  const int k = (int32_t)tmp >> 23;
  const double z = (double)__uint_as_float(iz), invc = kLog2fT[i][0], logc = kLog2fT[i][1];
  const double r = fma(z, invc, -1.0);
  const double y0 = logc + (double)k, r2 = r * r;
  double y = fma(kLog2fA[1], r, kLog2fA[2]);
  y = fma(kLog2fA[0], r2, y);
  const double p = fma(kLog2fA[3], r, y0);
  return (float)fma(y, r2, p);
}

// :1052-1070: log2(1 + importance / intra cost), 0 where the intra cost is 0
__global__ __launch_bounds__(256) void final_kernel(const uint32_t *intra, const float *imp, int n,
                                                    float *fin) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= n) return;
  const float ic = (float)intra[t];
  fin[t] = ic > 0.f ? log2f_ref(1.0f + __fdiv_rn(imp[t], ic)) : 0.f;
}

}  // namespace

size_t impwin_frame_bytes(int n, int R) {
  return al256((size_t)n * 4) + al256((size_t)R * n * sizeof(rv_mv)) + al256((size_t)R * n * 4) +
         al256((size_t)R * (n + 1) * 4) + al256((size_t)R * 4 * n * 4) + 2 * al256((size_t)n * 4);
}

void impwin_frame_carve(ImpFrame &f, void *base, int n, int R) {
  uint8_t *m = (uint8_t *)base;
  f.intra = (uint32_t *)m;
  m += al256((size_t)n * 4);
  f.mv8 = (rv_mv *)m;
  m += al256((size_t)R * n * sizeof(rv_mv));
  f.frac = (float *)m;
  m += al256((size_t)R * n * 4);
  f.off = (int32_t *)m;
  m += al256((size_t)R * (n + 1) * 4);
  f.src = (int32_t *)m;
  m += al256((size_t)R * 4 * n * 4);
  f.imp = (float *)m;
  m += al256((size_t)n * 4);
  f.fin = (float *)m;
}

size_t impwin_scratch_bytes(int n) { return csr_scratch(n).total; }

int impwin_group_data(const rv_plane &cur, const rv_plane *refs, int R, int bit_depth,
                      const rv_fs_result *look, int tx0, int ty0, int tw, int th, int w_imp,
                      int h_imp, const ImpFrame &f, hipStream_t st) {
  const int n = w_imp * h_imp;
  int bx0, by0, bw, bh;
  impwin_group_blocks(tx0, ty0, tw, th, w_imp, h_imp, bx0, by0, bw, bh);
  if (R < 1 || R > kImpMaxRefs || n <= 0 || bw <= 0 || bh <= 0 ||
      cur.xorigin + w_imp * 8 > cur.stride || cur.yorigin + h_imp * 8 > cur.alloc_height)
    return rv_set_error(RV_EINVAL, "impwin_group_data: bad geometry");
  DataArgs a;
  memset(&a, 0, sizeof(a));
  a.cur = cur;
  for (int k = 0; k < R; k++) a.ref[k] = refs[k];
  a.base = 128 << (bit_depth - 8);
  a.w = w_imp;
  a.h = h_imp;
  a.bx0 = bx0;
  a.by0 = by0;
  a.bw = bw;
  a.bh = bh;
  a.tx0 = tx0;
  a.ty0 = ty0;
  a.tw = tw;
  a.nsb = tw * th;
  a.look = look;
  a.f = f;
  const dim3 grid((unsigned)((bw * bh + 255) / 256), (unsigned)R);
  if (cur.hbd)
    data_kernel<uint16_t><<<grid, 256, 0, st>>>(a);
  else
    data_kernel<uint8_t><<<grid, 256, 0, st>>>(a);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

int impwin_lists(const ImpFrame &f, int R, int w_imp, int h_imp, void *scratch,
                 size_t scratch_bytes, hipStream_t st) {
  const int n = w_imp * h_imp;
  if (R < 1 || R > kImpMaxRefs || n <= 0) return rv_set_error(RV_EINVAL, "impwin_lists: bad arguments");
  const CsrScratch s = csr_scratch(n);
  if (!scratch || scratch_bytes < s.total) return rv_set_error(RV_EINVAL, "impwin_lists: scratch");
  uint8_t *base = (uint8_t *)scratch;
  uint32_t *keys = (uint32_t *)(base + s.keys);
  int32_t *cnt = (int32_t *)(base + s.cnt), *cursor = (int32_t *)(base + s.cur);
  {
    const hipError_t e = hipMemsetAsync(cnt, 0, (size_t)R * n * 4, st);
    if (e != hipSuccess) return rv_set_hip_error(e, "impwin_lists");
  }
  keys_kernel<<<dim3((unsigned)((n + 255) / 256), (unsigned)R), 256, 0, st>>>(f, w_imp, h_imp, keys,
                                                                            cnt);
  RV_HIP_CHECK_LAUNCH();
  // every reference's target lists, in source order within a target
  return csr_build(keys, 4 * n, n, R, cnt, cursor, f.off, f.src, st);
}

int impwin_part(const ImpFrame &f, int R, int tx0, int ty0, int tw, int th, int w_imp, int h_imp,
                void *buf, bool unpack, hipStream_t st) {
  int bx0, by0, bw, bh;
  impwin_group_blocks(tx0, ty0, tw, th, w_imp, h_imp, bx0, by0, bw, bh);
  if (R < 1 || R > kImpMaxRefs || bw <= 0 || bh <= 0 || !buf)
    return rv_set_error(RV_EINVAL, "impwin_part: bad arguments");
  part_kernel<<<(unsigned)((bw * bh + 255) / 256), 256, 0, st>>>(f, w_imp, h_imp, R, bx0, by0, bw,
                                                                 bh, (uint32_t *)buf, unpack ? 1 : 0);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

int impwin_pass(const ImpFrame &src, const int *ks, float *const *ref_imp, int np, int nu,
                int w_imp, int h_imp, hipStream_t st) {
  const int n = w_imp * h_imp;
  if (nu < 1 || nu > kImpMaxRefs || n <= 0 || np < 1 || np > kImpMaxRefs)
    return rv_set_error(RV_EINVAL, "impwin_pass: bad arguments");
  PassSet p;
  p.intra = src.intra;
  p.imp = src.imp;
  p.nu = nu;
  for (int i = 0; i < np; i++) {
    const int k = ks[i];
    p.mv8[i] = src.mv8 + (size_t)k * n;
    p.frac[i] = src.frac + (size_t)k * n;
    p.off[i] = src.off + (size_t)k * (n + 1);
    p.src[i] = src.src + (size_t)k * 4 * n;
    p.ref_imp[i] = ref_imp[i];
  }
  pass_kernel<<<dim3((unsigned)((n + 255) / 256), (unsigned)np), 256, 0, st>>>(p, w_imp, h_imp);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

int impwin_zero(float *const *imp, int count, int n, hipStream_t st) {
  for (int i0 = 0; i0 < count; i0 += 64) {
    ZeroSet z;
    const int c = count - i0 < 64 ? count - i0 : 64;
    for (int i = 0; i < c; i++) z.p[i] = imp[i0 + i];
    zero_kernel<<<dim3((unsigned)((n + 255) / 256), (unsigned)c), 256, 0, st>>>(z, n);
    RV_HIP_CHECK_LAUNCH();
  }
  return RV_OK;
}

int impwin_final(const ImpFrame &f, int w_imp, int h_imp, hipStream_t st) {
  const int n = w_imp * h_imp;
  final_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(f.intra, f.imp, n, f.fin);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

}  // namespace rv
