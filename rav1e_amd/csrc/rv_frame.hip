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

}  // namespace rv

using namespace rv;

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
