// rv_me_diamond.hip -- batched diamond motion search, one persistent
// workgroup per (block, reference) (gfx950).
//
// diamond_me_search (src/me.rs:693-785) with get_best_predictor
// (:655-691), get_mv_rd_cost (:787-838) and compute_mv_rd_cost (:840-856):
// the whole data-dependent search loop of a block runs inside one
// workgroup, so a tile's blocks advance in parallel without a host round
// trip per diamond step.  Full-pel candidates read the reference region
// straight from HBM; sub-pel candidates run predict_inter's put_8tap
// (src/predict.rs:255-338, REGULAR filters) into LDS first.  Every block
// evaluation is a workgroup-wide SAD / SATD reduced through LDS.
#include "rv_device.h"

namespace rv {

constexpr int kDsThreads = 256;

// SUBPEL_FILTERS REGULAR sets (src/mc.rs:70-179): index 0 = 8-tap
// REGULAR, 1 = 4-tap REGULAR (get_filter for length <= 4, src/mc.rs:201-210)
__constant__ int8_t kReg[2][16][8] = {
    {{0, 0, 0, 127, 0, 0, 0, 0}, {0, 2, -6, 126, 8, -2, 0, 0},
     {0, 2, -10, 122, 18, -4, 0, 0}, {0, 2, -12, 116, 28, -8, 2, 0},
     {0, 2, -14, 110, 38, -10, 2, 0}, {0, 2, -14, 102, 48, -12, 2, 0},
     {0, 2, -16, 94, 58, -12, 2, 0}, {0, 2, -14, 84, 66, -12, 2, 0},
     {0, 2, -14, 76, 76, -14, 2, 0}, {0, 2, -12, 66, 84, -14, 2, 0},
     {0, 2, -12, 58, 94, -16, 2, 0}, {0, 2, -12, 48, 102, -14, 2, 0},
     {0, 2, -10, 38, 110, -14, 2, 0}, {0, 2, -8, 28, 116, -12, 2, 0},
     {0, 0, -4, 18, 122, -10, 2, 0}, {0, 0, -2, 8, 126, -6, 2, 0}},
    {{0, 0, 0, 127, 0, 0, 0, 0}, {0, 0, -4, 126, 8, -2, 0, 0},
     {0, 0, -8, 122, 18, -4, 0, 0}, {0, 0, -10, 116, 28, -6, 0, 0},
     {0, 0, -12, 110, 38, -8, 0, 0}, {0, 0, -12, 102, 48, -10, 0, 0},
     {0, 0, -14, 94, 58, -10, 0, 0}, {0, 0, -12, 84, 66, -10, 0, 0},
     {0, 0, -12, 76, 76, -12, 0, 0}, {0, 0, -10, 66, 84, -12, 0, 0},
     {0, 0, -10, 58, 94, -14, 0, 0}, {0, 0, -10, 48, 102, -12, 0, 0},
     {0, 0, -8, 38, 110, -12, 0, 0}, {0, 0, -6, 28, 116, -10, 0, 0},
     {0, 0, -4, 18, 122, -8, 0, 0}, {0, 0, -2, 8, 126, -4, 0, 0}}};

__device__ __forceinline__ uint32_t ds_diff_to_rate(int16_t diff, int hp) {
  int16_t d = hp ? diff : (int16_t)(diff >> 1);
  if (d == 0) return 0;
  uint32_t a = (uint16_t)(d < 0 ? -d : d);
  return 2u * (16u - (uint32_t)(__builtin_clz(a) - 16));
}

template <int N>
__device__ __forceinline__ void ds_had(int32_t *v, int s) {
#pragma unroll
  for (int k = 0; k < N; k += 2) {
    int32_t a = v[k * s], b = v[(k + 1) * s];
    v[k * s] = a + b;
    v[(k + 1) * s] = a - b;
  }
#pragma unroll
  for (int g = 0; g < N; g += 4)
#pragma unroll
    for (int k = 0; k < 2; k++) {
      int32_t a = v[(g + k) * s], b = v[(g + k + 2) * s];
      v[(g + k) * s] = a + b;
      v[(g + k + 2) * s] = a - b;
    }
  if constexpr (N == 8) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      int32_t a = v[k * s], b = v[(k + 4) * s];
      v[k * s] = a + b;
      v[(k + 4) * s] = a - b;
    }
  }
}

__device__ __forceinline__ uint64_t wg_sum(uint64_t v, uint64_t *red) {
  v = group_sum<64>(v);
  __syncthreads();  // red[] may still be read by a previous reduction
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t t = 0;
#pragma unroll
  for (int i = 0; i < kDsThreads / 64; i++) t += red[i];
  return t;
}

// SAD or SATD (get_sad / get_satd semantics) of org vs pred(r, c),
// evaluated by the whole workgroup; all threads get the result.
template <typename Px, typename Pred>
__device__ uint32_t wg_dist(const Px *o, int ostride, int w, int h, int satd,
                            Pred pred, uint64_t *red) {
  uint64_t acc = 0;
  if (!satd) {
    for (int i = threadIdx.x; i < w * h; i += kDsThreads) {
      const int r = i / w, c = i - r * w;
      const int d = (int)o[(int64_t)r * ostride + c] - pred(r, c);
      acc += (uint32_t)(d < 0 ? -d : d);
    }
    return (uint32_t)wg_sum(acc, red);
  }
  const int n8 = (w < h ? w : h) >= 8;
  const int N = n8 ? 8 : 4, cw = w / N, chunks = cw * (h / N);
  for (int ci = threadIdx.x; ci < chunks; ci += kDsThreads) {
    const int cy = (ci / cw) * N, cx = (ci % cw) * N;
    if (n8) {
      int32_t d[64];
#pragma unroll
      for (int r = 0; r < 8; r++)
#pragma unroll
        for (int c = 0; c < 8; c++)
          d[r * 8 + c] = (int)o[(int64_t)(cy + r) * ostride + cx + c] - pred(cy + r, cx + c);
#pragma unroll
      for (int c = 0; c < 8; c++) ds_had<8>(d + c, 8);
#pragma unroll
      for (int r = 0; r < 8; r++) ds_had<8>(d + r * 8, 1);
#pragma unroll
      for (int i = 0; i < 64; i++) acc += (uint32_t)(d[i] < 0 ? -d[i] : d[i]);
    } else {
      int32_t d[16];
#pragma unroll
      for (int r = 0; r < 4; r++)
#pragma unroll
        for (int c = 0; c < 4; c++)
          d[r * 4 + c] = (int)o[(int64_t)(cy + r) * ostride + cx + c] - pred(cy + r, cx + c);
#pragma unroll
      for (int c = 0; c < 4; c++) ds_had<4>(d + c, 4);
#pragma unroll
      for (int r = 0; r < 4; r++) ds_had<4>(d + r * 4, 1);
#pragma unroll
      for (int i = 0; i < 16; i++) acc += (uint32_t)(d[i] < 0 ? -d[i] : d[i]);
    }
  }
  const uint64_t s = wg_sum(acc, red);
  const int ln = n8 ? 3 : 2;
  return (uint32_t)((s + ((1ull << ln) >> 1)) >> ln);
}

struct DsArgs {
  rv_plane org, ref;
  const rv_ds_job *jobs;
  rv_fs_result *out;
  int n, w, h, subpel, satd, hp, bd;
  unsigned long long *evals;  // optional: candidate evaluations (a counter)
};

template <typename Px>
__global__ __launch_bounds__(kDsThreads) void diamond_kernel(DsArgs a) {
  extern __shared__ __align__(16) int16_t lds[];
  __shared__ uint64_t red[kDsThreads / 64];
  const int job = blockIdx.x;
  if (job >= a.n) return;
  const rv_ds_job jb = a.jobs[job];
  const int w = a.w, h = a.h;
  const Px *o = plane_ptr<Px>(a.org, jb.po_x, jb.po_y);
  const int ib = a.bd == 12 ? 2 : 4;
  const int maxv = (1 << a.bd) - 1;
  const int sw = w + 7, shh = h + 7;
  int16_t *win = lds;               // [h+7][w+7]
  int16_t *mid = lds + sw * shh;    // [h+7][w]
  int16_t *pred = mid + shh * w;    // [h][w]

  // get_mv_rd_cost: range check, prediction, distortion, rate
  unsigned evals = 0;
  auto rd_cost = [&](rv_mv mv) -> uint64_t {
    if (mv.col < jb.mvx_min || mv.col > jb.mvx_max || mv.row < jb.mvy_min ||
        mv.row > jb.mvy_max)
      return ~0ull;
    evals++;
    uint32_t dist;
    if (!a.subpel) {
      // region at po + mv / 8 (Rust `/` truncates toward zero)
      const Px *r = plane_ptr<Px>(a.ref, jb.po_x + mv.col / 8, jb.po_y + mv.row / 8);
      const int rs = a.ref.stride;
      dist = wg_dist<Px>(o, a.org.stride, w, h, a.satd,
                         [&](int rr, int cc) { return (int)r[(int64_t)rr * rs + cc]; }, red);
    } else {
      // predict_inter / get_params (src/predict.rs:267-283), luma plane
      const int xs = 3 + a.ref.xdec, ys = 3 + a.ref.ydec;
      const int roff = (int)mv.row >> ys, coff = (int)mv.col >> xs;
      const int rf = ((int)mv.row - (roff << ys)) << (4 - ys);
      const int cf = ((int)mv.col - (coff << xs)) << (4 - xs);
      // PlaneSlice::clamp (src/frame/plane.rs:521-533) of the -3 origin
      const int qx = clampi(jb.po_x + coff - 3, -a.ref.xorigin, a.ref.width);
      const int qy = clampi(jb.po_y + roff - 3, -a.ref.yorigin, a.ref.height);
      const Px *sp = plane_ptr<Px>(a.ref, qx, qy);  // window origin (-3, -3)
      __syncthreads();  // previous candidate done with LDS
      for (int i = threadIdx.x; i < sw * shh; i += kDsThreads) {
        const int r = i / sw, c = i - r * sw;
        win[i] = (int16_t)sp[(int64_t)r * a.ref.stride + c];
      }
      __syncthreads();
      const int8_t *xf = kReg[w <= 4][cf];
      const int8_t *yf = kReg[h <= 4][rf];
      if (cf) {
        for (int i = threadIdx.x; i < shh * w; i += kDsThreads) {
          const int r = i / w, c = i - r * w;
          const int16_t *p = win + r * sw + c;
          int32_t s = 0;
#pragma unroll
          for (int k = 0; k < 8; k++) s += (int32_t)xf[k] * p[k];
          mid[i] = (int16_t)round_shift(s, 7 - ib);
        }
        __syncthreads();
      }
      for (int i = threadIdx.x; i < w * h; i += kDsThreads) {
        const int r = i / w, c = i - r * w;
        int32_t v;
        if (!cf && !rf) {
          v = win[(r + 3) * sw + c + 3];
        } else if (!cf) {
          const int16_t *p = win + r * sw + c + 3;
          int32_t s = 0;
#pragma unroll
          for (int k = 0; k < 8; k++) s += (int32_t)yf[k] * p[k * sw];
          v = round_shift(s, 7);
        } else if (!rf) {
          v = round_shift((int32_t)mid[(r + 3) * w + c], ib);
        } else {
          const int16_t *p = mid + r * w + c;
          int32_t s = 0;
#pragma unroll
          for (int k = 0; k < 8; k++) s += (int32_t)yf[k] * p[k * w];
          v = round_shift(s, 7 + ib);
        }
        pred[i] = (int16_t)clampi(v, 0, maxv);
      }
      __syncthreads();
      dist = wg_dist<Px>(o, a.org.stride, w, h, a.satd,
                         [&](int rr, int cc) { return (int)pred[rr * w + cc]; }, red);
    }
    const uint32_t r1 = ds_diff_to_rate((int16_t)(mv.row - jb.pmv[0].row), a.hp) +
                        ds_diff_to_rate((int16_t)(mv.col - jb.pmv[0].col), a.hp);
    const uint32_t r2 = ds_diff_to_rate((int16_t)(mv.row - jb.pmv[1].row), a.hp) +
                        ds_diff_to_rate((int16_t)(mv.col - jb.pmv[1].col), a.hp);
    const uint32_t rate = r1 < r2 + 1 ? r1 : r2 + 1;
    return 256ull * dist + (uint64_t)rate * jb.lambda;
  };

  // get_best_predictor
  rv_mv center{0, 0};
  uint64_t center_cost = ~0ull;
  const int np = jb.n_pred < RV_DS_MAX_PRED ? jb.n_pred : RV_DS_MAX_PRED;
  for (int p = 0; p < np; p++) {
    const uint64_t c = rd_cost(jb.pred[p]);
    if (c < center_cost) {
      center = jb.pred[p];
      center_cost = c;
    }
  }
  int16_t radius = a.subpel ? 4 : 16;
  const int16_t radius_end = a.subpel ? (a.hp ? 1 : 2) : 8;
  const int16_t pat[4][2] = {{1, 0}, {0, 1}, {-1, 0}, {0, -1}};
  // Every move strictly lowers center_cost, so the loop ends; the bound
  // only guarantees the grid drains whatever the inputs.
  for (int iter = 0; iter < 4096; iter++) {
    uint64_t best = ~0ull;
    rv_mv best_mv{0, 0};
    for (int p = 0; p < 4; p++) {
      const rv_mv cand{(int16_t)(center.row + radius * pat[p][0]),
                       (int16_t)(center.col + radius * pat[p][1])};
      const uint64_t c = rd_cost(cand);
      if (c < best) {
        best = c;
        best_mv = cand;
      }
    }
    if (center_cost <= best) {
      if (radius == radius_end) break;
      radius /= 2;
    } else {
      center = best_mv;
      center_cost = best;
    }
  }
  if (threadIdx.x == 0) {
    if (a.evals) atomicAdd(a.evals, (unsigned long long)evals);
    rv_fs_result r;
    r.best_mv = center;
    r.reserved = 0;
    r.cost = center_cost;
    a.out[job] = r;
  }
}

}  // namespace rv

using namespace rv;

int rv_diamond_search_batch_counted(const rv_plane *org, const rv_plane *ref,
                                    const rv_ds_job *d_jobs, int n, int blk_w, int blk_h,
                                    int subpixel, int use_satd, int allow_hp, int bit_depth,
                                    rv_fs_result *d_out, unsigned long long *evals,
                                    void *stream) {
  auto p2 = [](int v) { return v >= 4 && v <= 128 && (v & (v - 1)) == 0; };
  if (!org || !ref || n < 0 || !p2(blk_w) || !p2(blk_h) ||
      org->hbd != ref->hbd ||
      (bit_depth != 8 && bit_depth != 10 && bit_depth != 12) ||
      (!org->hbd && bit_depth != 8))
    return rv_set_error(RV_EINVAL, "rv_diamond_search_batch: bad arguments");
  if (n == 0) return RV_OK;
  DsArgs a{*org, *ref, d_jobs, d_out, n, blk_w, blk_h, subpixel ? 1 : 0,
           use_satd ? 1 : 0, allow_hp ? 1 : 0, bit_depth, evals};
  const size_t lds = subpixel ? (size_t)((blk_w + 7) * (blk_h + 7) + (blk_h + 7) * blk_w +
                                         blk_w * blk_h) * sizeof(int16_t)
                              : 0;
  hipStream_t s = rv_resolve_stream(stream);
  if (org->hbd)
    diamond_kernel<uint16_t><<<n, kDsThreads, lds, s>>>(a);
  else
    diamond_kernel<uint8_t><<<n, kDsThreads, lds, s>>>(a);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

extern "C" int rv_diamond_search_batch(const rv_plane *org, const rv_plane *ref,
                                       const rv_ds_job *d_jobs, int n, int blk_w,
                                       int blk_h, int subpixel, int use_satd,
                                       int allow_hp, int bit_depth,
                                       rv_fs_result *d_out, void *stream) {
  return rv_diamond_search_batch_counted(org, ref, d_jobs, n, blk_w, blk_h, subpixel,
                                         use_satd, allow_hp, bit_depth, d_out, nullptr,
                                         stream);
}
