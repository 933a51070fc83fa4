// rv_dist.hip -- batched SAD / SATD / SSE / cdef-moment kernels (gfx950).
//
// One launch covers every job of a tile-step; all jobs share (w, h), so the
// work split is static: a job's block is cut into fixed work units (SAD: 4
// pixels of one row; SATD: one 4x4 / 8x8 Hadamard chunk) and a power-of-two
// group of G lanes of one 64-wide wavefront owns one job, G = min(64,
// units).  Groups reduce with xor-shuffles (no LDS, no atomics), so small
// blocks pack 64 / G jobs per wavefront and large blocks use whole waves.
#include "rv_device.h"
#include "rv_tx.h"

namespace rv {

constexpr int kBlock = 256;  // 4 wavefronts per workgroup

__host__ __device__ constexpr int ilog2(int v) {
  int r = 0;
  while ((1 << r) < v) r++;
  return r;
}

// ---- SAD: get_sad_ref (src/dist.rs:25-46) ---------------------------------
template <typename Px, int LG>
__global__ __launch_bounds__(kBlock) void sad_kernel(
    rv_plane org, rv_plane ref, const rv_dist_job *__restrict__ jobs, int n,
    int w, int h, int upt, uint32_t *__restrict__ out) {
  constexpr int G = 1 << LG;
  const int tid = blockIdx.x * kBlock + threadIdx.x;
  const int job = tid >> LG;
  const int t = tid & (G - 1);
  const bool live = job < n;
  uint32_t acc = 0;
  if (live) {
    const rv_dist_job jb = jobs[job];
    const Px *o = plane_ptr<Px>(org, jb.org_x, jb.org_y);
    const Px *r = plane_ptr<Px>(ref, jb.ref_x, jb.ref_y);
    const int qw = w >> 2;  // 4-pixel units per row
    for (int k = 0; k < upt; k++) {
      const int u = t + k * G;
      const int row = u / qw, c4 = (u - row * qw) << 2;
      const Px *po = o + (int64_t)row * org.stride + c4;
      const Px *pr = r + (int64_t)row * ref.stride + c4;
      if constexpr (sizeof(Px) == 1) {
        acc = sad_u8x4(load_u32_unaligned((const uint8_t *)po),
                       load_u32_unaligned((const uint8_t *)pr), acc);
      } else {
#pragma unroll
        for (int i = 0; i < 4; i++) {
          int d = (int)po[i] - (int)pr[i];
          acc += (uint32_t)(d < 0 ? -d : d);
        }
      }
    }
  }
  acc = group_sum<G>(acc);
  if (live && t == 0) out[job] = acc;
}

// ---- SATD: get_satd_ref (src/dist.rs:197-328); had1d / satd_chunk live in
// rv_device.h (the replay's importance kernel uses them too)
template <typename Px, int N, int LG>
__global__ __launch_bounds__(kBlock) void satd_kernel(
    rv_plane org, rv_plane ref, const rv_dist_job *__restrict__ jobs, int n,
    int w, int h, int cpt, uint32_t *__restrict__ out) {
  constexpr int G = 1 << LG;
  const int tid = blockIdx.x * kBlock + threadIdx.x;
  const int job = tid >> LG;
  const int t = tid & (G - 1);
  const bool live = job < n;
  uint64_t acc = 0;
  if (live) {
    const rv_dist_job jb = jobs[job];
    const Px *o = plane_ptr<Px>(org, jb.org_x, jb.org_y);
    const Px *r = plane_ptr<Px>(ref, jb.ref_x, jb.ref_y);
    const int cw = w / N;
    for (int k = 0; k < cpt; k++) {
      const int cidx = t + k * G;
      const int cy = (cidx / cw) * N, cx = (cidx % cw) * N;
      int32_t d[N * N];
#pragma unroll
      for (int rr = 0; rr < N; rr++)
#pragma unroll
        for (int cc = 0; cc < N; cc++)
          d[rr * N + cc] =
              (int32_t)o[(int64_t)(cy + rr) * org.stride + cx + cc] -
              (int32_t)r[(int64_t)(cy + rr) * ref.stride + cx + cc];
      acc += satd_chunk<N>(d);
    }
  }
  acc = group_sum<G>(acc);
  if (live && t == 0) {
    constexpr int ln = N == 8 ? 3 : 2;
    out[job] = (uint32_t)((acc + ((1ull << ln) >> 1)) >> ln);
  }
}

// ---- SSE: sse_wxh raw partials (src/rdo.rs:286-335) ------------------------
// One lane per importance sub-block: each output is one u64.
template <typename Px>
__global__ __launch_bounds__(kBlock) void sse_kernel(
    rv_plane a, rv_plane b, const rv_dist_job *__restrict__ jobs, int n,
    int bw, int bh, int sub_x, int nsub, uint64_t *__restrict__ out) {
  const int tid = blockIdx.x * kBlock + threadIdx.x;
  if (tid >= n * nsub) return;
  const int job = tid / nsub, k = tid - job * nsub;
  const int by = k / sub_x, bx = k - by * sub_x;
  const rv_dist_job jb = jobs[job];
  const Px *pa = plane_ptr<Px>(a, jb.org_x + bx * bw, jb.org_y + by * bh);
  const Px *pb = plane_ptr<Px>(b, jb.ref_x + bx * bw, jb.ref_y + by * bh);
  uint64_t value = 0;
  for (int j = 0; j < bh; j++) {
    uint32_t row = 0;
    for (int i = 0; i < bw; i++) {
      // (i16::cast_from(a) - i16::cast_from(b)) as i32, squared as u32
      int32_t c = (int32_t)(int16_t)pa[(int64_t)j * a.stride + i] -
                  (int32_t)(int16_t)pb[(int64_t)j * b.stride + i];
      row += (uint32_t)wmul24(c, c);
    }
    value += row;
  }
  out[tid] = value;
}

// ---- cdef_dist_wxh_8x8 moments (src/rdo.rs:219-241) ------------------------
// 8 lanes per 8x8 (one row each), reduced by shuffles within the 8-group.
template <typename Px>
__global__ __launch_bounds__(kBlock) void cdef_moments_kernel(
    rv_plane a, rv_plane b, const rv_dist_job *__restrict__ jobs, int n,
    int sub_x, int nsub, int64_t *__restrict__ out) {
  const int tid = blockIdx.x * kBlock + threadIdx.x;
  const int blk = tid >> 3, j = tid & 7;
  const bool live = blk < n * nsub;
  int32_t ss = 0, sd = 0;
  int64_t ss2 = 0, sd2 = 0, ssd = 0;
  if (live) {
    const int job = blk / nsub, k = blk - job * nsub;
    const int by = k / sub_x, bx = k - by * sub_x;
    const rv_dist_job jb = jobs[job];
    const Px *pa = plane_ptr<Px>(a, jb.org_x + bx * 8, jb.org_y + by * 8 + j);
    const Px *pb = plane_ptr<Px>(b, jb.ref_x + bx * 8, jb.ref_y + by * 8 + j);
#pragma unroll
    for (int i = 0; i < 8; i++) {
      int32_t s = pa[i], d = pb[i];
      ss += s;
      sd += d;
      ss2 += (int64_t)wmul24(s, s);
      sd2 += (int64_t)wmul24(d, d);
      ssd += (int64_t)wmul24(s, d);
    }
  }
  ss = group_sum<8>(ss);
  sd = group_sum<8>(sd);
  ss2 = group_sum<8>(ss2);
  sd2 = group_sum<8>(sd2);
  ssd = group_sum<8>(ssd);
  if (live && j == 0) {
    int64_t *o = out + (int64_t)blk * 5;
    o[0] = ss;
    o[1] = sd;
    o[2] = ss2;
    o[3] = sd2;
    o[4] = ssd;
  }
}

// ---- tx-domain distortion (src/encoder.rs:1210-1224) ------------------------
// One wavefront per transform block: sum over the coded area of
// ((c - rc) * (c - rc)) as u64 (i32 wrapping square, sign-extended), then
// (d + (1 << (bits - 1))) >> bits, bits = 2 * (3 - get_log_tx_scale).
__global__ __launch_bounds__(kBlock) void tx_dist_kernel(const int32_t *__restrict__ coeffs,
                                                         int cstride,
                                                         const int32_t *__restrict__ rcoeffs,
                                                         int n, int area, int bits,
                                                         uint64_t *__restrict__ out) {
  const int blk = (int)((blockIdx.x * kBlock + threadIdx.x) >> 6), lane = threadIdx.x & 63;
  if (blk >= n) return;  // whole wavefront
  const int32_t *c = coeffs + (int64_t)blk * cstride;
  const int32_t *rc = rcoeffs + (int64_t)blk * area;
  uint64_t d = 0;
  for (int i = lane; i < area; i += 64) {
    const int32_t e = wsub(c[i], rc[i]);
    d += (uint64_t)(int64_t)wmul(e, e);
  }
  d = group_sum<64>(d);
  if (lane == 0) out[blk] = (d + (1ull << (bits - 1))) >> bits;
}

// ---- launch helpers -------------------------------------------------------
static bool valid_block(int w, int h) {
  auto p2 = [](int v) { return v >= 4 && v <= 128 && (v & (v - 1)) == 0; };
  return p2(w) && p2(h);
}

template <typename Px>
static void launch_sad(const rv_plane &o, const rv_plane &r,
                       const rv_dist_job *jobs, int n, int w, int h,
                       uint32_t *out, hipStream_t s) {
  const int units = (w / 4) * h;
  const int lg = units >= 64 ? 6 : ilog2(units);
  const int upt = units >> lg;
  const long threads = (long)n << lg;
  dim3 grid((unsigned)((threads + kBlock - 1) / kBlock));
  switch (lg) {
#define RV_CASE(L)                                                         \
  case L:                                                                  \
    sad_kernel<Px, L><<<grid, kBlock, 0, s>>>(o, r, jobs, n, w, h, upt, out); \
    break;
    RV_CASE(0) RV_CASE(1) RV_CASE(2) RV_CASE(3) RV_CASE(4) RV_CASE(5) RV_CASE(6)
#undef RV_CASE
  }
}

template <typename Px, int N>
static void launch_satd(const rv_plane &o, const rv_plane &r,
                        const rv_dist_job *jobs, int n, int w, int h,
                        uint32_t *out, hipStream_t s) {
  const int chunks = (w / N) * (h / N);
  const int lg = chunks >= 64 ? 6 : ilog2(chunks);
  const int cpt = chunks >> lg;
  const long threads = (long)n << lg;
  dim3 grid((unsigned)((threads + kBlock - 1) / kBlock));
  switch (lg) {
#define RV_CASE(L)                                                       \
  case L:                                                                \
    satd_kernel<Px, N, L><<<grid, kBlock, 0, s>>>(o, r, jobs, n, w, h, cpt, \
                                                  out);                  \
    break;
    RV_CASE(0) RV_CASE(1) RV_CASE(2) RV_CASE(3) RV_CASE(4) RV_CASE(5) RV_CASE(6)
#undef RV_CASE
  }
}

// compute_lookahead_intra_costs (src/api/internal.rs:680-765): for every
// 8x8 importance block, DC_PRED into a copy of the plane, then get_satd of
// the source block against it.  predict_intra is handed a tile rect that
// starts at the block itself (:731-736), so its position relative to the
// "tile" is (0, 0), PredictionVariant::NONE, and DC_PRED becomes pred_dc_128
// (src/predict.rs:214-221, 552-557, 623-633): the prediction is the constant
// 128 << (bd - 8) whatever the edges hold.  One thread per block.
template <typename Px>
__global__ __launch_bounds__(kBlock) void intra_cost_kernel(rv_plane p, int nbx, int nby,
                                                            int base, uint32_t *out) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= nbx * nby) return;
  const int bx = i % nbx, by = i / nbx;
  const Px *o = plane_ptr<Px>(p, bx * 8, by * 8);
  int32_t d[64];
#pragma unroll
  for (int r = 0; r < 8; r++)
#pragma unroll
    for (int c = 0; c < 8; c++) d[r * 8 + c] = (int32_t)o[(int64_t)r * p.stride + c] - base;
  out[i] = (uint32_t)((satd_chunk<8>(d) + 4) >> 3);  // ln = msb(8)
}

}  // namespace rv

using namespace rv;

extern "C" {

int rv_lookahead_intra_costs(const rv_plane *p, int bit_depth, uint32_t *d_costs,
                             void *stream) {
  if (!p || !d_costs || (bit_depth != 8 && bit_depth != 10 && bit_depth != 12) ||
      (!p->hbd && bit_depth != 8) || p->width <= 0 || p->height <= 0 || p->xdec || p->ydec)
    return rv_set_error(RV_EINVAL, "rv_lookahead_intra_costs: bad arguments");
  // w_in_imp_b = w_in_b / 2 (src/encoder.rs:624-625): ceil(width / 8); the
  // last column / row of blocks may read the plane's padding, as the
  // reference's region does
  const int nbx = (p->width + 7) >> 3, nby = (p->height + 7) >> 3;
  if (p->xorigin + nbx * 8 > p->stride || p->yorigin + nby * 8 > p->alloc_height)
    return rv_set_error(RV_EINVAL, "rv_lookahead_intra_costs: blocks leave the allocation");
  const int n = nbx * nby;
  hipStream_t s = rv_resolve_stream(stream);
  const int base = 128 << (bit_depth - 8);
  if (p->hbd)
    intra_cost_kernel<uint16_t><<<(n + kBlock - 1) / kBlock, kBlock, 0, s>>>(*p, nbx, nby, base,
                                                                           d_costs);
  else
    intra_cost_kernel<uint8_t><<<(n + kBlock - 1) / kBlock, kBlock, 0, s>>>(*p, nbx, nby, base,
                                                                          d_costs);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

int rv_sad_batch(const rv_plane *org, const rv_plane *ref,
                 const rv_dist_job *d_jobs, int n, int w, int h,
                 uint32_t *d_out, void *stream) {
  if (!org || !ref || n < 0 || !valid_block(w, h) || org->hbd != ref->hbd)
    return rv_set_error(RV_EINVAL, "rv_sad_batch: bad arguments");
  if (n == 0) return RV_OK;
  hipStream_t s = rv_resolve_stream(stream);
  if (org->hbd)
    launch_sad<uint16_t>(*org, *ref, d_jobs, n, w, h, d_out, s);
  else
    launch_sad<uint8_t>(*org, *ref, d_jobs, n, w, h, d_out, s);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

int rv_satd_batch(const rv_plane *org, const rv_plane *ref,
                  const rv_dist_job *d_jobs, int n, int w, int h,
                  uint32_t *d_out, void *stream) {
  if (!org || !ref || n < 0 || !valid_block(w, h) || org->hbd != ref->hbd)
    return rv_set_error(RV_EINVAL, "rv_satd_batch: bad arguments");
  if (n == 0) return RV_OK;
  hipStream_t s = rv_resolve_stream(stream);
  const bool n4 = (w < h ? w : h) == 4;
  if (org->hbd) {
    if (n4) launch_satd<uint16_t, 4>(*org, *ref, d_jobs, n, w, h, d_out, s);
    else launch_satd<uint16_t, 8>(*org, *ref, d_jobs, n, w, h, d_out, s);
  } else {
    if (n4) launch_satd<uint8_t, 4>(*org, *ref, d_jobs, n, w, h, d_out, s);
    else launch_satd<uint8_t, 8>(*org, *ref, d_jobs, n, w, h, d_out, s);
  }
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

int rv_sse_batch(const rv_plane *org, const rv_plane *ref,
                 const rv_dist_job *d_jobs, int n, int w, int h,
                 uint64_t *d_out, void *stream) {
  // assert!(w & (MI_SIZE - 1) == 0) etc. (src/rdo.rs:290-291)
  if (!org || !ref || n < 0 || w <= 0 || h <= 0 || (w & 3) || (h & 3) ||
      org->hbd != ref->hbd)
    return rv_set_error(RV_EINVAL, "rv_sse_batch: bad arguments");
  const int bw = (w < 8 ? w : 8) >> org->xdec, bh = (h < 8 ? h : 8) >> org->ydec;
  if (bw <= 0 || bh <= 0 || (w % bw) || (h % bh))
    return rv_set_error(RV_EINVAL, "rv_sse_batch: bad sub-block");
  if (n == 0) return RV_OK;
  const int sub_x = w / bw, nsub = sub_x * (h / bh);
  const long threads = (long)n * nsub;
  dim3 grid((unsigned)((threads + kBlock - 1) / kBlock));
  hipStream_t s = rv_resolve_stream(stream);
  if (org->hbd)
    sse_kernel<uint16_t><<<grid, kBlock, 0, s>>>(*org, *ref, d_jobs, n, bw, bh,
                                                 sub_x, nsub, d_out);
  else
    sse_kernel<uint8_t><<<grid, kBlock, 0, s>>>(*org, *ref, d_jobs, n, bw, bh,
                                                sub_x, nsub, d_out);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

int rv_cdef_moments_batch(const rv_plane *org, const rv_plane *ref,
                          const rv_dist_job *d_jobs, int n, int w, int h,
                          int64_t *d_out, void *stream) {
  // assert!(w & 0x7 == 0) / (h & 0x7 == 0) (src/rdo.rs:262-263)
  if (!org || !ref || n < 0 || w <= 0 || h <= 0 || (w & 7) || (h & 7) ||
      org->hbd != ref->hbd)
    return rv_set_error(RV_EINVAL, "rv_cdef_moments_batch: bad arguments");
  if (n == 0) return RV_OK;
  const int sub_x = w / 8, nsub = sub_x * (h / 8);
  const long threads = (long)n * nsub * 8;
  dim3 grid((unsigned)((threads + kBlock - 1) / kBlock));
  hipStream_t s = rv_resolve_stream(stream);
  if (org->hbd)
    cdef_moments_kernel<uint16_t><<<grid, kBlock, 0, s>>>(
        *org, *ref, d_jobs, n, sub_x, nsub, d_out);
  else
    cdef_moments_kernel<uint8_t><<<grid, kBlock, 0, s>>>(*org, *ref, d_jobs, n,
                                                         sub_x, nsub, d_out);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

// tx-domain distortion of a batch of transform blocks: coeffs [n] at
// coeff_stride (e.g. the W*H raster of rv_fwd_txfm_batch), rcoeffs [n][coded
// area] (the packed dequantized coefficients).
int rv_tx_dist_batch(const int32_t *d_coeffs, int coeff_stride, const int32_t *d_rcoeffs, int n,
                     int tx_size, uint64_t *d_out, void *stream) {
  if (!d_coeffs || !d_rcoeffs || !d_out || n < 0 || tx_size < 0 || tx_size > 18)
    return rv_set_error(RV_EINVAL, "rv_tx_dist_batch: bad arguments");
  const int w = 1 << tx_w_log2(tx_size), h = 1 << tx_h_log2(tx_size);
  const int area = (w < 32 ? w : 32) * (h < 32 ? h : 32);  // coded_tx_area
  if (coeff_stride < area) return rv_set_error(RV_EINVAL, "rv_tx_dist_batch: stride < coded area");
  const int log_scale = (w * h > 256) + (w * h > 1024);  // get_log_tx_scale
  if (n == 0) return RV_OK;
  const unsigned grid = (unsigned)((n + 3) / 4);
  tx_dist_kernel<<<grid, kBlock, 0, rv_resolve_stream(stream)>>>(
      d_coeffs, coeff_stride, d_rcoeffs, n, area, 2 * (3 - log_scale), d_out);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

}  // extern "C"
