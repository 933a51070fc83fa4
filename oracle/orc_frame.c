/* Frame-layout restatements (test infrastructure only), src/frame/. */
#include <string.h>

#include "orc_common.h"

static inline int align_pow2(int x, int n) {
  return (x + (1 << n) - 1) & ~((1 << n) - 1);
}

/* Plane::new, src/frame/plane.rs:215-244: STRIDE_ALIGNMENT_LOG2 = 5, so
 * xorigin and stride are aligned to 32 bytes (2^(5+1-sizeof(T)) pixels). */
void orc_plane_geometry(int width, int height, int xpad, int ypad, int hbd,
                        int out[4]) {
  int al = 5 + 1 - (hbd ? 2 : 1);
  int xorigin = align_pow2(xpad, al);
  int yorigin = ypad;
  int stride = align_pow2(xorigin + width + xpad, al);
  out[0] = stride;
  out[1] = yorigin + height + ypad;
  out[2] = xorigin;
  out[3] = yorigin;
}

/* Plane::pad, src/frame/plane.rs:269-314 */
void orc_plane_pad(void *data, int stride, int alloc_height, int xorigin,
                   int yorigin, int xdec, int ydec, int w, int h, int hbd) {
  int width = (w + xdec) >> xdec, height = (h + ydec) >> ydec;
  size_t px = hbd ? 2 : 1;
  char *d = (char *)data;
  if (xorigin > 0)
    for (int y = 0; y < height; y++) {
      ptrdiff_t base = (ptrdiff_t)(yorigin + y) * stride;
      int32_t fill = orc_px(data, hbd, base + xorigin);
      for (int x = 0; x < xorigin; x++) orc_px_store(data, hbd, base + x, fill);
    }
  if (xorigin + width < stride)
    for (int y = 0; y < height; y++) {
      ptrdiff_t base = (ptrdiff_t)(yorigin + y) * stride + xorigin + width;
      int32_t fill = orc_px(data, hbd, base - 1);
      for (int x = 0; x < stride - (xorigin + width); x++)
        orc_px_store(data, hbd, base + x, fill);
    }
  if (yorigin > 0)
    for (int y = 0; y < yorigin; y++)
      memcpy(d + (size_t)y * stride * px, d + (size_t)yorigin * stride * px,
             (size_t)stride * px);
  if (yorigin + height < alloc_height)
    for (int y = yorigin + height; y < alloc_height; y++)
      memcpy(d + (size_t)y * stride * px,
             d + (size_t)(yorigin + height - 1) * stride * px,
             (size_t)stride * px);
}

/* Plane::downsample_from, src/frame/plane.rs:399-423: 2x2 box, (s+2)>>2 */
void orc_downsample(void *dst, ptrdiff_t dst_stride, int dst_w, int dst_h,
                    const void *src, ptrdiff_t src_stride, int hbd) {
  for (int r = 0; r < dst_h; r++)
    for (int c = 0; c < dst_w; c++) {
      uint32_t s = (uint32_t)orc_px(src, hbd, 2 * r * src_stride + 2 * c) +
                   (uint32_t)orc_px(src, hbd, 2 * r * src_stride + 2 * c + 1) +
                   (uint32_t)orc_px(src, hbd, (2 * r + 1) * src_stride + 2 * c) +
                   (uint32_t)orc_px(src, hbd,
                                    (2 * r + 1) * src_stride + 2 * c + 1);
      orc_px_store(dst, hbd, r * dst_stride + c, (int32_t)((s + 2) >> 2));
    }
}
