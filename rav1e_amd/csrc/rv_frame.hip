// rv_frame.hip -- frame-layout kernels: Plane::pad and
// Plane::downsample_from (src/frame/plane.rs:269-314, 399-423).
#include "rv_device.h"

namespace rv {

// Plane::pad: left/right replicate the first/last visible pixel of each
// visible row, then the top/bottom padding rows copy the first/last padded
// row.  Per pixel that is "read the visible pixel at the clamped
// coordinate", which this kernel does for every padding pixel (interior
// pixels are left untouched, so reads and writes never overlap).
template <typename Px>
__global__ __launch_bounds__(256) void pad_kernel(rv_plane p) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)p.stride * p.alloc_height;
  if (i >= total) return;
  const int y = (int)(i / p.stride), x = (int)(i - (int64_t)y * p.stride);
  const int x0 = p.xorigin, y0 = p.yorigin;
  if (x >= x0 && x < x0 + p.width && y >= y0 && y < y0 + p.height) return;
  const int sx = clampi(x, x0, x0 + p.width - 1);
  const int sy = clampi(y, y0, y0 + p.height - 1);
  Px *d = reinterpret_cast<Px *>(p.data);
  d[i] = d[(int64_t)sy * p.stride + sx];
}

// The three planes of a frame in one launch (plane p owns workgroups
// [blk[p], blk[p + 1])).  Without src: Plane::pad of dst, one lane per
// padding pixel only (the top rows, the visible rows' left and right
// margins, the bottom rows).  With src (same geometry): every allocation
// pixel of dst = src's visible pixel at the clamped coordinate -- copying a
// frame and padding it in one pass.
struct PadPlanes {
  rv_plane dst[3], src[3];
  unsigned blk[4];
  int copy;
};
template <typename Px>
__global__ __launch_bounds__(256) void pad3_kernel(PadPlanes P) {
  const int pi = blockIdx.x >= P.blk[1] ? (blockIdx.x >= P.blk[2] ? 2 : 1) : 0;
  const rv_plane &d = P.dst[pi];
  int64_t i = (int64_t)(blockIdx.x - P.blk[pi]) * 256 + threadIdx.x;
  const int x0 = d.xorigin, y0 = d.yorigin, w = d.width, h = d.height;
  const int64_t st = d.stride;
  int x, y;
  if (P.copy) {
    if (i >= st * d.alloc_height) return;
    y = (int)(i / st);
    x = (int)(i - y * st);
  } else {
    const int64_t top = (int64_t)y0 * st, side = (int64_t)h * (st - w);
    if (i < top) {
      y = (int)(i / st);
      x = (int)(i - y * st);
    } else if ((i -= top) < side) {
      const int r = (int)(i / (st - w)), c = (int)(i - r * (st - w));
      y = y0 + r;
      x = c < x0 ? c : c + w;
    } else {
      i -= side;
      if (i >= (int64_t)(d.alloc_height - y0 - h) * st) return;
      const int r = (int)(i / st);
      y = y0 + h + r;
      x = (int)(i - r * st);
    }
  }
  const int sx = clampi(x, x0, x0 + w - 1), sy = clampi(y, y0, y0 + h - 1);
  const Px *sp = reinterpret_cast<const Px *>(P.copy ? P.src[pi].data : d.data);
  reinterpret_cast<Px *>(d.data)[(int64_t)y * st + x] = sp[(int64_t)sy * st + sx];
}

// downsample_from: (sum of the 2x2 source pixels + 2) >> 2
template <typename Px>
__global__ __launch_bounds__(256) void downsample_kernel(rv_plane dst,
                                                         rv_plane src) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)dst.width * dst.height) return;
  const int r = (int)(i / dst.width), c = (int)(i - (int64_t)r * dst.width);
  const Px *s = plane_ptr<Px>(src, 2 * c, 2 * r);
  const uint32_t sum = (uint32_t)s[0] + (uint32_t)s[1] + (uint32_t)s[src.stride] +
                       (uint32_t)s[src.stride + 1];
  *plane_ptr_mut<Px>(dst, c, r) = (Px)((sum + 2) >> 2);
}

// The replay's per-frame F0 in one launch: input_hres and input_qres
// (src/encoder.rs:3382-3385: downsample_from twice, each followed by pad)
// computed straight from the full-resolution plane.  Every allocation pixel
// of hres (blockIdx.y = 0) / qres (1) is the downsampled value at the
// clamped visible coordinate -- exactly what downsample + pad leave there;
// qres pixels recompute their four hres parents with the same rounding.
template <typename Px>
__device__ __forceinline__ uint32_t ds2x2(const Px *s, int stride) {
  return ((uint32_t)s[0] + (uint32_t)s[1] + (uint32_t)s[stride] + (uint32_t)s[stride + 1] + 2) >> 2;
}
template <typename Px>
__global__ __launch_bounds__(256) void pyramid_kernel(rv_plane y, rv_plane h, rv_plane q) {
  const rv_plane &d = blockIdx.y ? q : h;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)d.stride * d.alloc_height) return;
  const int ay = (int)(i / d.stride), ax = (int)(i - (int64_t)ay * d.stride);
  const int c = clampi(ax - d.xorigin, 0, d.width - 1), r = clampi(ay - d.yorigin, 0, d.height - 1);
  uint32_t v;
  if (blockIdx.y == 0) {
    v = ds2x2(plane_ptr<Px>(y, 2 * c, 2 * r), y.stride);
  } else {
    const Px *s = plane_ptr<Px>(y, 4 * c, 4 * r);
    const int st = y.stride;
    v = (ds2x2(s, st) + ds2x2(s + 2, st) + ds2x2(s + 2 * st, st) + ds2x2(s + 2 * st + 2, st) + 2) >> 2;
  }
  reinterpret_cast<Px *>(d.data)[i] = (Px)v;
}

// ---- synthetic input (integer form) --------------------------
// The bench's y4m stand-in, generated in HBM (the inputs are resident before
// the timed region, as an uploaded clip would be).  Pure integer arithmetic,
// so rav1e_amd/replay.py:synth_frame (numpy) produces the same planes bit
// for bit: a 2-D wave times a moving value-noise texture plus +-2 noise,
// moving (1.25, 0.75) luma px per frame (sub-pel motion), per plane p at
// luma-space quarter-pel coordinates.
__host__ __device__ inline uint32_t synth_hash(uint32_t x) {  // lowbias32
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// integer parabola standing in for a sine of period P (amplitude 64)
__host__ __device__ inline int synth_wave(int q, int P) {
  const int h = P / 2;
  return q < h ? 256 * q * (h - q) / (h * h) : -(256 * (q - h) * (P - q) / (h * h));
}
__host__ __device__ inline int synth_lat(int ix, int iy) {
  return (int)(synth_hash((uint32_t)ix * 0x9E3779B1u ^ (uint32_t)iy * 0x85EBCA77u ^ 0x5EEDu) & 511) -
         256;
}
template <typename Px>
__global__ __launch_bounds__(256) void synth_kernel(rv_plane p, int t, int pidx, int bd) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)p.width * p.height) return;
  const int y = (int)(i / p.width), x = (int)(i - (int64_t)y * p.width);
  const int X4 = ((4 * x) << p.xdec) - 5 * t + 64 * pidx, Y4 = ((4 * y) << p.ydec) - 3 * t;
  const int ix = X4 >> 5, fx = X4 & 31, iy = Y4 >> 5, fy = Y4 & 31;
  const int v = (synth_lat(ix, iy) * (32 - fx) + synth_lat(ix + 1, iy) * fx) * (32 - fy) +
                (synth_lat(ix, iy + 1) * (32 - fx) + synth_lat(ix + 1, iy + 1) * fx) * fy;
  const int ta = pidx ? 12 : 24, wa = pidx ? 30 : 60;
  const int tex = (v * ta) >> 18;
  const int px = ((X4 % 388) + 388) % 388, py = ((Y4 % 244) + 244) % 244;
  const int wave = (synth_wave(px, 388) * synth_wave(py, 244) * wa) >> 12;
  const uint32_t hs = synth_hash((uint32_t)x * 0x27D4EB2Du ^ (uint32_t)y * 0x165667B1u ^
                                 (uint32_t)t * 0x9E3779B9u ^ (uint32_t)pidx * 0x85EBCA6Bu);
  const int noise = (int)(hs % 5u) - 2;
  int v8 = 128 + wave + tex + noise;
  v8 = v8 < 0 ? 0 : v8 > 255 ? 255 : v8;
  const int val = (v8 << (bd - 8)) | (int)(synth_hash(hs ^ 0xABCDu) & ((1u << (bd - 8)) - 1));
  *plane_ptr_mut<Px>(p, x, y) = (Px)val;
}

}  // namespace rv

using namespace rv;

// One synthetic frame t into planes y, u, v (visible area), then padded.
int rv_synth_frame(const rv_plane *y, const rv_plane *u, const rv_plane *v, int t, int bit_depth,
                   void *stream) {
  const rv_plane *pl[3] = {y, u, v};
  hipStream_t s = rv_resolve_stream(stream);
  for (int k = 0; k < 3; k++) {
    const int64_t n = (int64_t)pl[k]->width * pl[k]->height;
    const unsigned g = (unsigned)((n + 255) / 256);
    if (pl[k]->hbd)
      synth_kernel<uint16_t><<<g, 256, 0, s>>>(*pl[k], t, k, bit_depth);
    else
      synth_kernel<uint8_t><<<g, 256, 0, s>>>(*pl[k], t, k, bit_depth);
    RV_HIP_CHECK_LAUNCH();
    const int e = rv_plane_pad(pl[k], stream);
    if (e != RV_OK) return e;
  }
  return RV_OK;
}

// Plane::pad of a frame's three planes, or (src) src copied into dst and
// padded, in one launch (pad3_kernel).  src's planes have dst's geometry.
int rv_frame_pad_dev(const rv_plane dst[3], const rv_plane *src, hipStream_t s) {
  PadPlanes P = {};
  P.copy = src != nullptr;
  unsigned blocks = 0;
  for (int p = 0; p < 3; p++) {
    const rv_plane &d = dst[p];
    if (!d.data || d.width <= 0 || d.height <= 0 || d.hbd != dst[0].hbd ||
        (src && (src[p].stride != d.stride || src[p].xorigin != d.xorigin ||
                 src[p].yorigin != d.yorigin || src[p].width != d.width ||
                 src[p].height != d.height || src[p].hbd != d.hbd)))
      return rv_set_error(RV_EINVAL, "rv_frame_pad: bad planes");
    P.dst[p] = d;
    if (src) P.src[p] = src[p];
    const int64_t n = src ? (int64_t)d.stride * d.alloc_height
                          : (int64_t)d.stride * d.alloc_height - (int64_t)d.width * d.height;
    P.blk[p] = blocks;
    blocks += (unsigned)((n + 255) / 256);
  }
  P.blk[3] = blocks;
  if (dst[0].hbd)
    pad3_kernel<uint16_t><<<blocks, 256, 0, s>>>(P);
  else
    pad3_kernel<uint8_t><<<blocks, 256, 0, s>>>(P);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

// hres = downsample(y) + pad, qres = downsample(hres) + pad, one launch.
int rv_plane_pyramid(const rv_plane *y, const rv_plane *h, const rv_plane *q, void *stream) {
  if (!y || !h || !q || y->hbd != h->hbd || h->hbd != q->hbd || h->width * 2 != y->width ||
      h->height * 2 != y->height || q->width * 2 != h->width || q->height * 2 != h->height)
    return rv_set_error(RV_EINVAL, "rv_plane_pyramid: size mismatch");
  const int64_t th = (int64_t)h->stride * h->alloc_height;
  dim3 grid((unsigned)((th + 255) / 256), 2);
  hipStream_t s = rv_resolve_stream(stream);
  if (y->hbd)
    pyramid_kernel<uint16_t><<<grid, 256, 0, s>>>(*y, *h, *q);
  else
    pyramid_kernel<uint8_t><<<grid, 256, 0, s>>>(*y, *h, *q);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

extern "C" {

int rv_plane_pad(const rv_plane *p, void *stream) {
  if (!p || !p->data || p->width <= 0 || p->height <= 0)
    return rv_set_error(RV_EINVAL, "rv_plane_pad: bad plane");
  const int64_t total = (int64_t)p->stride * p->alloc_height;
  dim3 grid((unsigned)((total + 255) / 256));
  hipStream_t s = rv_resolve_stream(stream);
  if (p->hbd)
    pad_kernel<uint16_t><<<grid, 256, 0, s>>>(*p);
  else
    pad_kernel<uint8_t><<<grid, 256, 0, s>>>(*p);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

int rv_plane_downsample(const rv_plane *dst, const rv_plane *src,
                        void *stream) {
  // assert!(width * 2 == src.cfg.width) (src/frame/plane.rs:406-407)
  if (!dst || !src || dst->hbd != src->hbd || dst->width * 2 != src->width ||
      dst->height * 2 != src->height)
    return rv_set_error(RV_EINVAL, "rv_plane_downsample: size mismatch");
  const int64_t total = (int64_t)dst->width * dst->height;
  dim3 grid((unsigned)((total + 255) / 256));
  hipStream_t s = rv_resolve_stream(stream);
  if (dst->hbd)
    downsample_kernel<uint16_t><<<grid, 256, 0, s>>>(*dst, *src);
  else
    downsample_kernel<uint8_t><<<grid, 256, 0, s>>>(*dst, *src);
  RV_HIP_CHECK_LAUNCH();
  return rv_plane_pad(dst, stream);
}

}  // extern "C"
