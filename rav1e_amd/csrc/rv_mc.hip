// rv_mc.hip -- batched 8-tap motion compensation (gfx950).
//
// put_8tap_ref / prep_8tap_ref / mc_avg_ref (src/mc.rs:213-408) as one
// workgroup per block: the (h+7) x (w+7) source window is loaded once with
// coalesced row reads into LDS, the horizontal pass writes the i16
// intermediate (round_shift(sum, 7 - ib)) into LDS, the vertical pass reads
// it back.  The same pipeline feeds the fused MC+distortion kernel, whose
// prediction never touches HBM.
#include "rv_device.h"

namespace rv {

constexpr int kMcThreads = 256;

// SUBPEL_FILTERS (src/mc.rs:70-179), 6 sets x 16 fracs x 8 taps.
__constant__ int8_t kSubpel[6][16][8] = {
    {{0, 0, 0, 127, 0, 0, 0, 0}, {0, 2, -6, 126, 8, -2, 0, 0},
     {0, 2, -10, 122, 18, -4, 0, 0}, {0, 2, -12, 116, 28, -8, 2, 0},
     {0, 2, -14, 110, 38, -10, 2, 0}, {0, 2, -14, 102, 48, -12, 2, 0},
     {0, 2, -16, 94, 58, -12, 2, 0}, {0, 2, -14, 84, 66, -12, 2, 0},
     {0, 2, -14, 76, 76, -14, 2, 0}, {0, 2, -12, 66, 84, -14, 2, 0},
     {0, 2, -12, 58, 94, -16, 2, 0}, {0, 2, -12, 48, 102, -14, 2, 0},
     {0, 2, -10, 38, 110, -14, 2, 0}, {0, 2, -8, 28, 116, -12, 2, 0},
     {0, 0, -4, 18, 122, -10, 2, 0}, {0, 0, -2, 8, 126, -6, 2, 0}},
    {{0, 0, 0, 127, 0, 0, 0, 0}, {0, 2, 28, 62, 34, 2, 0, 0},
     {0, 0, 26, 62, 36, 4, 0, 0}, {0, 0, 22, 62, 40, 4, 0, 0},
     {0, 0, 20, 60, 42, 6, 0, 0}, {0, 0, 18, 58, 44, 8, 0, 0},
     {0, 0, 16, 56, 46, 10, 0, 0}, {0, -2, 16, 54, 48, 12, 0, 0},
     {0, -2, 14, 52, 52, 14, -2, 0}, {0, 0, 12, 48, 54, 16, -2, 0},
     {0, 0, 10, 46, 56, 16, 0, 0}, {0, 0, 8, 44, 58, 18, 0, 0},
     {0, 0, 6, 42, 60, 20, 0, 0}, {0, 0, 4, 40, 62, 22, 0, 0},
     {0, 0, 4, 36, 62, 26, 0, 0}, {0, 0, 2, 34, 62, 28, 2, 0}},
    {{0, 0, 0, 127, 0, 0, 0, 0}, {-2, 2, -6, 126, 8, -2, 2, 0},
     {-2, 6, -12, 124, 16, -6, 4, -2}, {-2, 8, -18, 120, 26, -10, 6, -2},
     {-4, 10, -22, 116, 38, -14, 6, -2}, {-4, 10, -22, 108, 48, -18, 8, -2},
     {-4, 10, -24, 100, 60, -20, 8, -2}, {-4, 10, -24, 90, 70, -22, 10, -2},
     {-4, 12, -24, 80, 80, -24, 12, -4}, {-2, 10, -22, 70, 90, -24, 10, -4},
     {-2, 8, -20, 60, 100, -24, 10, -4}, {-2, 8, -18, 48, 108, -22, 10, -4},
     {-2, 6, -14, 38, 116, -22, 10, -4}, {-2, 6, -10, 26, 120, -18, 8, -2},
     {-2, 4, -6, 16, 124, -12, 6, -2}, {0, 2, -2, 8, 126, -6, 2, -2}},
    {{0, 0, 0, 127, 0, 0, 0, 0}, {0, 0, 0, 120, 8, 0, 0, 0},
     {0, 0, 0, 112, 16, 0, 0, 0}, {0, 0, 0, 104, 24, 0, 0, 0},
     {0, 0, 0, 96, 32, 0, 0, 0}, {0, 0, 0, 88, 40, 0, 0, 0},
     {0, 0, 0, 80, 48, 0, 0, 0}, {0, 0, 0, 72, 56, 0, 0, 0},
     {0, 0, 0, 64, 64, 0, 0, 0}, {0, 0, 0, 56, 72, 0, 0, 0},
     {0, 0, 0, 48, 80, 0, 0, 0}, {0, 0, 0, 40, 88, 0, 0, 0},
     {0, 0, 0, 32, 96, 0, 0, 0}, {0, 0, 0, 24, 104, 0, 0, 0},
     {0, 0, 0, 16, 112, 0, 0, 0}, {0, 0, 0, 8, 120, 0, 0, 0}},
    {{0, 0, 0, 127, 0, 0, 0, 0}, {0, 0, -4, 126, 8, -2, 0, 0},
     {0, 0, -8, 122, 18, -4, 0, 0}, {0, 0, -10, 116, 28, -6, 0, 0},
     {0, 0, -12, 110, 38, -8, 0, 0}, {0, 0, -12, 102, 48, -10, 0, 0},
     {0, 0, -14, 94, 58, -10, 0, 0}, {0, 0, -12, 84, 66, -10, 0, 0},
     {0, 0, -12, 76, 76, -12, 0, 0}, {0, 0, -10, 66, 84, -12, 0, 0},
     {0, 0, -10, 58, 94, -14, 0, 0}, {0, 0, -10, 48, 102, -12, 0, 0},
     {0, 0, -8, 38, 110, -12, 0, 0}, {0, 0, -6, 28, 116, -10, 0, 0},
     {0, 0, -4, 18, 122, -8, 0, 0}, {0, 0, -2, 8, 126, -4, 0, 0}},
    {{0, 0, 0, 127, 0, 0, 0, 0}, {0, 0, 30, 62, 34, 2, 0, 0},
     {0, 0, 26, 62, 36, 4, 0, 0}, {0, 0, 22, 62, 40, 4, 0, 0},
     {0, 0, 20, 60, 42, 6, 0, 0}, {0, 0, 18, 58, 44, 8, 0, 0},
     {0, 0, 16, 56, 46, 10, 0, 0}, {0, 0, 14, 54, 48, 12, 0, 0},
     {0, 0, 12, 52, 52, 12, 0, 0}, {0, 0, 12, 48, 54, 14, 0, 0},
     {0, 0, 10, 46, 56, 16, 0, 0}, {0, 0, 8, 44, 58, 18, 0, 0},
     {0, 0, 6, 42, 60, 20, 0, 0}, {0, 0, 4, 40, 62, 22, 0, 0},
     {0, 0, 4, 36, 62, 26, 0, 0}, {0, 0, 2, 34, 62, 30, 0, 0}}};
// frac 0 (the {0,0,0,128,...} row) is never filtered (every path
// special-cases a zero frac), so its 128 is stored as 127 to fit int8.

// get_filter (src/mc.rs:201-210)
__device__ __forceinline__ int filter_set(int mode, int length) {
  return (mode == 3 || length > 4) ? mode : ((mode < 1 ? mode : 1) + 4);
}

enum McKind { kPut = 0, kPrep = 1, kDistSad = 2, kDistSatd = 3 };

struct McArgs {
  rv_plane src, dst;  // dst: put destination, or org for the dist kinds
  const rv_mc_job *jobs;
  int n, w, h, mode_x, mode_y, bit_depth;
  int16_t *tmp;     // prep output
  uint32_t *dist;   // dist output
};

template <int N>
__device__ __forceinline__ void had1d_i(int32_t *v, int s) {
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

// Block-wide u64 sum (256 threads = 4 wavefronts).
__device__ __forceinline__ uint64_t block_sum(uint64_t v, uint64_t *red) {
  v = group_sum<64>(v);
  const int wid = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[wid] = v;
  __syncthreads();
  uint64_t t = 0;
  for (int i = 0; i < (int)(blockDim.x >> 6); i++) t += red[i];
  return t;
}

template <typename Px, int KIND>
__global__ __launch_bounds__(kMcThreads) void mc_kernel(McArgs a) {
  extern __shared__ __align__(16) int16_t lds[];
  const int job = blockIdx.x;
  if (job >= a.n) return;
  const rv_mc_job jb = a.jobs[job];
  const int w = a.w, h = a.h;
  const int cf = jb.col_frac, rf = jb.row_frac;
  const int ox = cf ? 3 : 0, oy = rf ? 3 : 0;  // window margins
  const int sw = w + 2 * ox + (cf ? 1 : 0);    // -3..w+4 when filtered
  const int sh = h + 2 * oy + (rf ? 1 : 0);
  const int ib = a.bit_depth == 12 ? 2 : 4;  // intermediate_bits
  const int maxv = (1 << a.bit_depth) - 1;
  int16_t *win = lds;              // [sh][sw] source pixels
  int16_t *mid = lds + sh * sw;    // [sh][w] horizontal pass
  const int nt = blockDim.x, tid = threadIdx.x;

  // 1. source window -> LDS (row-contiguous, coalesced)
  const Px *sp = plane_ptr<Px>(a.src, jb.src_x - ox, jb.src_y - oy);
  for (int i = tid; i < sh * sw; i += nt) {
    const int r = i / sw, c = i - r * sw;
    win[i] = (int16_t)sp[(int64_t)r * a.src.stride + c];
  }
  __syncthreads();

  const int8_t *xf = kSubpel[filter_set(a.mode_x, w)][cf];
  const int8_t *yf = kSubpel[filter_set(a.mode_y, h)][rf];

  // 2. horizontal pass: mid = round_shift(sum xf * src, 7 - ib)
  if (cf) {
    int32_t f[8];
#pragma unroll
    for (int k = 0; k < 8; k++) f[k] = xf[k];
    for (int i = tid; i < sh * w; i += nt) {
      const int r = i / w, c = i - r * w;
      const int16_t *p = win + r * sw + c;  // column c - 3 .. c + 4
      int32_t s = 0;
#pragma unroll
      for (int k = 0; k < 8; k++) s += f[k] * p[k];
      mid[i] = (int16_t)round_shift(s, 7 - ib);
    }
    __syncthreads();
  }

  // 3. vertical pass / output
  int32_t fy[8];
#pragma unroll
  for (int k = 0; k < 8; k++) fy[k] = yf[k];
  auto pixel_at = [&](int r, int c) -> int32_t {
    // value of put (clamped pixel) or prep (i16 intermediate) at (r, c)
    int32_t v;
    if (!cf && !rf) {
      v = win[r * sw + c];
      if (KIND == kPrep) v = (int32_t)(int16_t)(v << ib);
    } else if (!cf) {
      const int16_t *p = win + r * sw + c;  // rows r-3 .. r+4
      int32_t s = 0;
#pragma unroll
      for (int k = 0; k < 8; k++) s += fy[k] * p[k * sw];
      v = KIND == kPrep ? round_shift(s, 7 - ib) : round_shift(s, 7);
    } else if (!rf) {
      const int32_t m = mid[r * w + c];
      v = KIND == kPrep ? m : round_shift(m, ib);
    } else {
      const int16_t *p = mid + r * w + c;
      int32_t s = 0;
#pragma unroll
      for (int k = 0; k < 8; k++) s += fy[k] * p[k * w];
      v = KIND == kPrep ? round_shift(s, 7) : round_shift(s, 7 + ib);
    }
    if (KIND != kPrep) v = clampi(v, 0, maxv);
    return v;
  };

  if constexpr (KIND == kPut) {
    Px *dp = plane_ptr_mut<Px>(a.dst, jb.dst_x, jb.dst_y);
    for (int i = tid; i < w * h; i += nt) {
      const int r = i / w, c = i - r * w;
      dp[(int64_t)r * a.dst.stride + c] = (Px)pixel_at(r, c);
    }
  } else if constexpr (KIND == kPrep) {
    int16_t *tp = a.tmp + (int64_t)job * w * h;
    for (int i = tid; i < w * h; i += nt) {
      const int r = i / w, c = i - r * w;
      tp[i] = (int16_t)pixel_at(r, c);
    }
  } else {
    // fused distortion against org (= a.dst) at (dst_x, dst_y)
    __shared__ uint64_t red[kMcThreads / 64];
    const Px *op = plane_ptr<Px>(a.dst, jb.dst_x, jb.dst_y);
    uint64_t acc = 0;
    if constexpr (KIND == kDistSad) {
      for (int i = tid; i < w * h; i += nt) {
        const int r = i / w, c = i - r * w;
        int d = (int)op[(int64_t)r * a.dst.stride + c] - pixel_at(r, c);
        acc += (uint32_t)(d < 0 ? -d : d);
      }
      acc = block_sum(acc, red);
      if (tid == 0) a.dist[job] = (uint32_t)acc;
    } else {
      const int n8 = (w < h ? w : h) >= 8;
      const int N = n8 ? 8 : 4;
      const int cw = w / N, chunks = cw * (h / N);
      for (int ci = tid; ci < chunks; ci += nt) {
        const int cy = (ci / cw) * N, cx = (ci % cw) * N;
        if (n8) {
          int32_t d[64];
#pragma unroll
          for (int rr = 0; rr < 8; rr++)
#pragma unroll
            for (int cc = 0; cc < 8; cc++)
              d[rr * 8 + cc] =
                  (int32_t)op[(int64_t)(cy + rr) * a.dst.stride + cx + cc] -
                  pixel_at(cy + rr, cx + cc);
#pragma unroll
          for (int c = 0; c < 8; c++) had1d_i<8>(d + c, 8);
#pragma unroll
          for (int r = 0; r < 8; r++) had1d_i<8>(d + r * 8, 1);
#pragma unroll
          for (int i = 0; i < 64; i++) acc += (uint32_t)(d[i] < 0 ? -d[i] : d[i]);
        } else {
          int32_t d[16];
#pragma unroll
          for (int rr = 0; rr < 4; rr++)
#pragma unroll
            for (int cc = 0; cc < 4; cc++)
              d[rr * 4 + cc] =
                  (int32_t)op[(int64_t)(cy + rr) * a.dst.stride + cx + cc] -
                  pixel_at(cy + rr, cx + cc);
#pragma unroll
          for (int c = 0; c < 4; c++) had1d_i<4>(d + c, 4);
#pragma unroll
          for (int r = 0; r < 4; r++) had1d_i<4>(d + r * 4, 1);
#pragma unroll
          for (int i = 0; i < 16; i++) acc += (uint32_t)(d[i] < 0 ? -d[i] : d[i]);
        }
      }
      acc = block_sum(acc, red);
      const int ln = n8 ? 3 : 2;
      if (tid == 0) a.dist[job] = (uint32_t)((acc + ((1ull << ln) >> 1)) >> ln);
    }
  }
}

// mc_avg_ref (src/mc.rs:389-408): clamp(round_shift(t1 + t2, ib + 1))
template <typename Px>
__global__ __launch_bounds__(kMcThreads) void avg_kernel(
    rv_plane dst, const int16_t *__restrict__ t1,
    const int16_t *__restrict__ t2, const rv_mc_job *__restrict__ jobs, int n,
    int w, int h, int bit_depth) {
  const int job = blockIdx.x;
  if (job >= n) return;
  const rv_mc_job jb = jobs[job];
  const int ib = bit_depth == 12 ? 2 : 4;
  const int maxv = (1 << bit_depth) - 1;
  const int16_t *a = t1 + (int64_t)job * w * h;
  const int16_t *b = t2 + (int64_t)job * w * h;
  Px *dp = plane_ptr_mut<Px>(dst, jb.dst_x, jb.dst_y);
  for (int i = threadIdx.x; i < w * h; i += blockDim.x) {
    const int r = i / w, c = i - r * w;
    const int32_t v = round_shift((int32_t)a[i] + (int32_t)b[i], ib + 1);
    dp[(int64_t)r * dst.stride + c] = (Px)clampi(v, 0, maxv);
  }
}

static bool mc_args_ok(int n, int w, int h, int mx, int my, int bd) {
  auto p2 = [](int v) { return v >= 2 && v <= 128 && (v & (v - 1)) == 0; };
  return n >= 0 && p2(w) && p2(h) && mx >= 0 && mx < 4 && my >= 0 && my < 4 &&
         (bd == 8 || bd == 10 || bd == 12);
}

template <int KIND>
static int launch_mc(const McArgs &a, int hbd, hipStream_t s) {
  const int sw = a.w + 7, sh = a.h + 7;
  const size_t lds = (size_t)(sh * sw + sh * a.w) * sizeof(int16_t);
  int threads = a.w * a.h;
  threads = threads < 64 ? 64 : (threads > kMcThreads ? kMcThreads : threads);
  if (hbd)
    mc_kernel<uint16_t, KIND><<<a.n, threads, lds, s>>>(a);
  else
    mc_kernel<uint8_t, KIND><<<a.n, threads, lds, s>>>(a);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

}  // namespace rv

using namespace rv;

extern "C" {

int rv_put_8tap_batch(const rv_plane *dst, const rv_plane *src,
                      const rv_mc_job *d_jobs, int n, int w, int h,
                      int mode_x, int mode_y, int bit_depth, void *stream) {
  if (!dst || !src || !mc_args_ok(n, w, h, mode_x, mode_y, bit_depth) ||
      dst->hbd != src->hbd || (!src->hbd && bit_depth != 8))
    return rv_set_error(RV_EINVAL, "rv_put_8tap_batch: bad arguments");
  if (n == 0) return RV_OK;
  McArgs a{*src, *dst, d_jobs, n, w, h, mode_x, mode_y, bit_depth, nullptr,
           nullptr};
  return launch_mc<kPut>(a, src->hbd, rv_resolve_stream(stream));
}

int rv_prep_8tap_batch(int16_t *d_tmp, const rv_plane *src,
                       const rv_mc_job *d_jobs, int n, int w, int h,
                       int mode_x, int mode_y, int bit_depth, void *stream) {
  if (!src || !mc_args_ok(n, w, h, mode_x, mode_y, bit_depth) ||
      (!src->hbd && bit_depth != 8))
    return rv_set_error(RV_EINVAL, "rv_prep_8tap_batch: bad arguments");
  if (n == 0) return RV_OK;
  McArgs a{*src, *src, d_jobs, n, w, h, mode_x, mode_y, bit_depth, d_tmp,
           nullptr};
  return launch_mc<kPrep>(a, src->hbd, rv_resolve_stream(stream));
}

int rv_mc_avg_batch(const rv_plane *dst, const int16_t *d_tmp1,
                    const int16_t *d_tmp2, const rv_mc_job *d_jobs, int n,
                    int w, int h, int bit_depth, void *stream) {
  if (!dst || !mc_args_ok(n, w, h, 0, 0, bit_depth) ||
      (!dst->hbd && bit_depth != 8))
    return rv_set_error(RV_EINVAL, "rv_mc_avg_batch: bad arguments");
  if (n == 0) return RV_OK;
  hipStream_t s = rv_resolve_stream(stream);
  if (dst->hbd)
    avg_kernel<uint16_t><<<n, kMcThreads, 0, s>>>(*dst, d_tmp1, d_tmp2, d_jobs,
                                                  n, w, h, bit_depth);
  else
    avg_kernel<uint8_t><<<n, kMcThreads, 0, s>>>(*dst, d_tmp1, d_tmp2, d_jobs,
                                                 n, w, h, bit_depth);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

int rv_mc_dist_batch(const rv_plane *org, const rv_plane *ref,
                     const rv_mc_job *d_jobs, int n, int w, int h, int mode_x,
                     int mode_y, int bit_depth, int metric, uint32_t *d_out,
                     void *stream) {
  if (!org || !ref || !mc_args_ok(n, w, h, mode_x, mode_y, bit_depth) ||
      w < 4 || h < 4 || org->hbd != ref->hbd || (metric != 0 && metric != 1) ||
      (!ref->hbd && bit_depth != 8))
    return rv_set_error(RV_EINVAL, "rv_mc_dist_batch: bad arguments");
  if (n == 0) return RV_OK;
  McArgs a{*ref, *org, d_jobs, n, w, h, mode_x, mode_y, bit_depth, nullptr,
           d_out};
  hipStream_t s = rv_resolve_stream(stream);
  return metric ? launch_mc<kDistSatd>(a, ref->hbd, s)
                : launch_mc<kDistSad>(a, ref->hbd, s);
}

}  // extern "C"
