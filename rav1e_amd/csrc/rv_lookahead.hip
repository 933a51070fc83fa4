// rv_lookahead.hip -- the importance propagation of the lookahead
// (compute_block_importances, src/api/internal.rs:823-1010), one (frame,
// reference) pass, bit-exact in f32.
//
// The reference walks the frame's 8x8 importance blocks in raster order;
// each block measures its inter cost (get_satd against the reference at its
// lookahead MV), turns it into a propagate amount and adds amount * area
// fraction to the four reference blocks its MV-displaced area overlaps
// (top-left, top-right, bottom-left, bottom-right).  A float accumulation
// depends on its order, so the device does not scatter with atomics:
//   1. one thread per source block writes its four (target, amount *
//      fraction) contributions at [4 * source + k] -- the reference's order;
//   2. a counting sort by target (rv_csr.h: the keys are bounded block
//      indices) groups them, keeping that order within a target;
//   3. one thread per target adds its contributions in order onto the
//      target's current value, as the reference's `+=` sequence does.
// Products and sums are separate roundings (-ffp-contract=off) and the
// divisions are correctly rounded (__fdiv_rn), as in Rust.
#include "rv_csr.h"
#include "rv_device.h"

namespace rv {

constexpr int kImpB = 8, kMvUnits = 8, kBMv = kImpB * kMvUnits, kAreaMv = kBMv * kBMv;

template <typename Px>
__global__ __launch_bounds__(256) void importance_contrib_kernel(
    rv_plane org, rv_plane ref, int nbx, int nby, const rv_mv *mvs, const uint32_t *intra,
    const float *imp, int n_unique, uint32_t *keys, float *vals, int32_t *cnt) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int n = nbx * nby;
  if (i >= n) return;
  const int x = i % nbx, y = i / nbx;
  const rv_mv mv = mvs[i];
  const int64_t rx = (int64_t)x * kBMv + mv.col, ry = (int64_t)y * kBMv + mv.row;
  const int64_t px_x = rx / kMvUnits, px_y = ry / kMvUnits;  // isize `/`: toward zero
  // the 8x8 reference block must lie inside the allocation (the reference's
  // region would panic otherwise); a block that leaves it contributes nothing
  const bool inside = px_x >= -ref.xorigin && px_y >= -ref.yorigin &&
                      px_x + kImpB <= ref.stride - ref.xorigin &&
                      px_y + kImpB <= ref.alloc_height - ref.yorigin;
  uint32_t key[4] = {(uint32_t)n, (uint32_t)n, (uint32_t)n, (uint32_t)n};
  float val[4] = {0.f, 0.f, 0.f, 0.f};
  if (inside) {
    const Px *o = plane_ptr<Px>(org, x * kImpB, y * kImpB);

    const Px *r = plane_ptr<Px>(ref, (int)px_x, (int)px_y);
    int32_t d[64];
#pragma unroll
    for (int rr = 0; rr < 8; rr++)
#pragma unroll
      for (int cc = 0; cc < 8; cc++)
        d[rr * 8 + cc] = (int32_t)o[(int64_t)rr * org.stride + cc] -
                         (int32_t)r[(int64_t)rr * ref.stride + cc];
    const float inter_cost = (float)(uint32_t)((satd_chunk<8>(d) + 4) >> 3);
    const float intra_cost = (float)intra[i];
    // f32::max(NaN, 0) = 0, as fmaxf
    const float fraction = fmaxf(1.0f - __fdiv_rn(inter_cost, intra_cost), 0.0f);
    const float amount = __fdiv_rn((intra_cost + imp[i]) * fraction, (float)n_unique);
    const int64_t tlx = (rx - (rx < 0 ? kBMv - 1 : 0)) / kBMv * kBMv;
    const int64_t tly = (ry - (ry < 0 ? kBMv - 1 : 0)) / kBMv * kBMv;
    const int64_t trx = tlx + kBMv, bly = tly + kBMv;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int64_t tx = (k & 1) ? trx : tlx, ty = (k & 2) ? bly : tly;
      const int64_t fx = (k & 1) ? rx + kBMv - trx : trx - rx;
      const int64_t fy = (k & 2) ? ry + kBMv - bly : bly - ry;
      const float f = __fdiv_rn((float)(fx * fy), (float)kAreaMv);
      const int64_t bx = tx / kBMv, by = ty / kBMv;
      if (bx >= 0 && by >= 0 && bx < nbx && by < nby) {
        key[k] = (uint32_t)(by * nbx + bx);
        val[k] = amount * f;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 4; k++) {
    keys[4 * (int64_t)i + k] = key[k];
    vals[4 * (int64_t)i + k] = val[k];
    if (key[k] < (uint32_t)n) atomicAdd(cnt + key[k], 1);
  }
}

// One thread per target: its value plus its contributions (src: entry
// indices in source order), one rounding per addition, in the reference's
// order.
__global__ __launch_bounds__(256) void importance_accumulate_kernel(const int32_t *off,
                                                                    const int32_t *src,
                                                                    const float *vals, int n,
                                                                    float *ref_imp) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= n) return;
  const int a = off[t], b = off[t + 1];
  if (a == b) return;
  float acc = ref_imp[t];
  for (int j = a; j < b; j++) acc = acc + vals[src[j]];
  ref_imp[t] = acc;
}

struct ImpScratch {
  size_t keys, vals, cnt, cur, off, src, total;
};

static size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

static ImpScratch imp_scratch(int n) {
  ImpScratch s;
  const size_t m = 4 * (size_t)n;
  s.keys = 0;
  s.vals = align256(s.keys + 4 * m);
  s.cnt = align256(s.vals + 4 * m);
  s.cur = align256(s.cnt + 4 * (size_t)n);
  s.off = align256(s.cur + 4 * (size_t)n);
  s.src = align256(s.off + 4 * ((size_t)n + 1));
  s.total = align256(s.src + 4 * m);
  return s;
}

}  // namespace rv

using namespace rv;

extern "C" size_t rv_propagate_importances_scratch(int w_imp, int h_imp) {
  if (w_imp <= 0 || h_imp <= 0) return 0;
  return imp_scratch(w_imp * h_imp).total;
}

extern "C" int rv_propagate_importances(const rv_plane *org, const rv_plane *ref,
                                        const rv_mv *d_mvs, const uint32_t *d_intra_costs,
                                        const float *d_importances, int n_unique,
                                        float *d_ref_importances, void *d_scratch,
                                        size_t scratch_bytes, void *stream) {
  if (!org || !ref || !d_mvs || !d_intra_costs || !d_importances || !d_ref_importances ||
      n_unique < 1 || n_unique > 3 || org->hbd != ref->hbd || org->xdec || org->ydec ||
      org->width <= 0 || org->height <= 0)
    return rv_set_error(RV_EINVAL, "rv_propagate_importances: bad arguments");
  // w_in_imp_b = w_in_b / 2 (src/encoder.rs:624-625): ceil(width / 8)
  const int nbx = (org->width + 7) >> 3, nby = (org->height + 7) >> 3, n = nbx * nby;
  if (org->xorigin + nbx * 8 > org->stride || org->yorigin + nby * 8 > org->alloc_height)
    return rv_set_error(RV_EINVAL, "rv_propagate_importances: blocks leave the allocation");
  const ImpScratch s = imp_scratch(n);
  if (!d_scratch || scratch_bytes < s.total)
    return rv_set_error(RV_EINVAL, "rv_propagate_importances: scratch below "
                                   "rv_propagate_importances_scratch()");
  uint8_t *base = (uint8_t *)d_scratch;
  uint32_t *keys = (uint32_t *)(base + s.keys);
  float *vals = (float *)(base + s.vals);
  int32_t *cnt = (int32_t *)(base + s.cnt), *cur = (int32_t *)(base + s.cur);
  int32_t *off = (int32_t *)(base + s.off), *src = (int32_t *)(base + s.src);
  hipStream_t st = rv_resolve_stream(stream);
  {
    const hipError_t e = hipMemsetAsync(cnt, 0, (size_t)n * 4, st);
    if (e != hipSuccess) return rv_set_hip_error(e, "rv_propagate_importances");
  }
  const unsigned g1 = (unsigned)((n + 255) / 256);
  if (org->hbd)
    importance_contrib_kernel<uint16_t><<<g1, 256, 0, st>>>(*org, *ref, nbx, nby, d_mvs,
                                                            d_intra_costs, d_importances,
                                                            n_unique, keys, vals, cnt);
  else
    importance_contrib_kernel<uint8_t><<<g1, 256, 0, st>>>(*org, *ref, nbx, nby, d_mvs,
                                                           d_intra_costs, d_importances,
                                                           n_unique, keys, vals, cnt);
  RV_HIP_CHECK_LAUNCH();
  {
    const int e = csr_build(keys, 4 * n, n, 1, cnt, cur, off, src, st);
    if (e != RV_OK) return e;
  }
  importance_accumulate_kernel<<<g1, 256, 0, st>>>(off, src, vals, n, d_ref_importances);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}
