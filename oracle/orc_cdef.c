/* CDEF (test infrastructure only): cdef_find_dir (src/cdef.rs:68-126),
 * cdef_filter_block's native path (:134-228), adjust_strength (:232-239),
 * and the frame driver cdef_filter_frame (:542-641) with
 * cdef_analyze_superblock (:278-317) and cdef_filter_superblock (:411-534).
 *
 * The frame driver builds the padded u16 copy exactly as the reference
 * does (:550-609): Plane::new fills with 128 (src/frame/plane.rs:133-140),
 * a 2-pixel ring around the visible plane holds CDEF_VERY_LARGE, and the
 * filter reads that copy and writes the output frame (out of place here;
 * the reference writes back into rec).  Arithmetic in cdef_find_dir wraps
 * like Rust's release build: a partial 8x8 block at the frame's edge sums
 * CDEF_VERY_LARGE samples whose squares exceed i32. */
#include <stdlib.h>
#include <string.h>

#include "orc_common.h"

#define CDEF_VERY_LARGE 0x8000
static const int32_t cdef_div_table[9] = {0, 840, 420, 280, 210, 168, 140, 120, 105};

static int imax(int a, int b) { return a > b ? a : b; }
static int imin(int a, int b) { return a < b ? a : b; }
/* msb (src/util/mod.rs:235-238) for x != 0 */
static int msb32(int32_t x) { return 31 ^ __builtin_clz((uint32_t)x); }

/* cdef_find_dir (src/cdef.rs:68-126) on the padded u16 copy */
int orc_cdef_find_dir(const uint16_t *img, ptrdiff_t stride, int32_t *var, int coeff_shift) {
  uint32_t cost[8] = {0};
  int32_t partial[8][15];
  memset(partial, 0, sizeof partial);
  for (int i = 0; i < 8; i++)
    for (int j = 0; j < 8; j++) {
      const int32_t x = (int32_t)(img[i * stride + j] >> coeff_shift) - 128;
      partial[0][i + j] += x;
      partial[1][i + j / 2] += x;
      partial[2][i] += x;
      partial[3][3 + i - j / 2] += x;
      partial[4][7 + i - j] += x;
      partial[5][3 - i / 2 + j] += x;
      partial[6][j] += x;
      partial[7][i / 2 + j] += x;
    }
#define SQ(v) ((uint32_t)(v) * (uint32_t)(v))
  for (int i = 0; i < 8; i++) {
    cost[2] += SQ(partial[2][i]);
    cost[6] += SQ(partial[6][i]);
  }
  cost[2] *= (uint32_t)cdef_div_table[8];
  cost[6] *= (uint32_t)cdef_div_table[8];
  for (int i = 0; i < 7; i++) {
    cost[0] += (SQ(partial[0][i]) + SQ(partial[0][14 - i])) * (uint32_t)cdef_div_table[i + 1];
    cost[4] += (SQ(partial[4][i]) + SQ(partial[4][14 - i])) * (uint32_t)cdef_div_table[i + 1];
  }
  cost[0] += SQ(partial[0][7]) * (uint32_t)cdef_div_table[8];
  cost[4] += SQ(partial[4][7]) * (uint32_t)cdef_div_table[8];
  for (int i = 1; i < 8; i += 2) {
    for (int j = 0; j < 5; j++) cost[i] += SQ(partial[i][3 + j]);
    cost[i] *= (uint32_t)cdef_div_table[8];
    for (int j = 0; j < 3; j++)
      cost[i] += (SQ(partial[i][j]) + SQ(partial[i][10 - j])) * (uint32_t)cdef_div_table[2 * j + 2];
  }
#undef SQ
  /* first_max_element (:54-59): the first maximum, compared as i32 */
  int best = 0;
  for (int d = 1; d < 8; d++)
    if ((int32_t)cost[d] > (int32_t)cost[best]) best = d;
  *var = (int32_t)(cost[best] - cost[(best + 4) & 7]) >> 10;
  return best;
}

/* constrain (:134-148) */
static int constrain(int diff, int threshold, int damping) {
  if (!threshold) return 0;
  const int shift = imax(0, damping - msb32(threshold));
  const int ad = abs(diff);
  const int mag = imin(ad, imax(0, threshold - (ad >> shift)));
  return diff < 0 ? -mag : mag;
}

/* cdef_filter_block, native (:152-228) */
void orc_cdef_filter_block(void *dst, ptrdiff_t dstride, int hbd, const uint16_t *in,
                           ptrdiff_t istride, int pri, int sec, int dir, int damping, int bd,
                           int xdec, int ydec) {
  const int xsize = 8 >> xdec, ysize = 8 >> ydec, cs = bd - 8;
  static const int pri_taps_t[2][2] = {{4, 2}, {3, 3}};
  static const int sec_taps_t[2][2] = {{2, 1}, {2, 1}};
  const int *pri_taps = pri_taps_t[(pri >> cs) & 1];
  const int *sec_taps = sec_taps_t[(pri >> cs) & 1];
  const ptrdiff_t s = istride;
  const ptrdiff_t dirs[8][2] = {{-1 * s + 1, -2 * s + 2}, {0 * s + 1, -1 * s + 2},
                                {0 * s + 1, 0 * s + 2},   {0 * s + 1, 1 * s + 2},
                                {1 * s + 1, 2 * s + 2},   {1 * s + 0, 2 * s + 1},
                                {1 * s + 0, 2 * s + 0},   {1 * s + 0, 2 * s - 1}};
  for (int i = 0; i < ysize; i++)
    for (int j = 0; j < xsize; j++) {
      const uint16_t *p = in + i * s + j;
      const int x = *p;
      int sum = 0, mx = x, mn = x;
      for (int k = 0; k < 2; k++) {
        const ptrdiff_t d0 = dirs[dir][k], d1 = dirs[(dir + 2) & 7][k], d2 = dirs[(dir + 6) & 7][k];
        const int pv[2] = {p[d0], p[-d0]};
        for (int e = 0; e < 2; e++) {
          sum += pri_taps[k] * constrain(pv[e] - x, pri, damping);
          if (pv[e] != CDEF_VERY_LARGE) mx = imax(pv[e], mx);
          mn = imin(pv[e], mn);
        }
        const int sv[4] = {p[d1], p[-d1], p[d2], p[-d2]};
        for (int e = 0; e < 4; e++) {
          if (sv[e] != CDEF_VERY_LARGE) mx = imax(sv[e], mx);
          mn = imin(sv[e], mn);
          sum += sec_taps[k] * constrain(sv[e] - x, sec, damping);
        }
      }
      int v = x + ((8 + sum - (sum < 0)) >> 4);
      v = v < mn ? mn : v > mx ? mx : v;
      if (hbd)
        ((uint16_t *)dst)[i * dstride + j] = (uint16_t)v;
      else
        ((uint8_t *)dst)[i * dstride + j] = (uint8_t)v;
    }
}

/* adjust_strength (:232-239) */
int orc_cdef_adjust_strength(int strength, int32_t var) {
  const int i = (var >> 6) ? imin(msb32(var >> 6), 12) : 0;
  return var ? (strength * (4 + i) + 8) >> 4 : 0;
}

/* cdef_filter_frame (:542-641): planes[p] / strides[p] at the visible
 * origin of plane p (luma width x height, chroma (width + xdec) >> xdec),
 * out of place.  skip per luma 4x4 block (pitch mi_stride, >= the frame's
 * 2 * ceil(width / 8) columns); cdef_index per 64x64 superblock (pitch
 * ceil(width / 64)); strengths = FrameInvariants::cdef_{y,uv}_strengths;
 * damping = cdef_damping.  dirs / vars (optional, pitch ceil(width / 8))
 * receive cdef_analyze_superblock's result per 8x8 block. */
void orc_cdef_filter_frame(const void *const in[3], const ptrdiff_t istride[3], void *const out[3],
                           const ptrdiff_t ostride[3], int hbd, int bd, int width, int height,
                           int xdec, int ydec, const uint8_t *skip, int mi_stride,
                           const uint8_t *cdef_index, const uint8_t y_str[8],
                           const uint8_t uv_str[8], int damping, uint8_t *dirs, int32_t *vars) {
  const int fb_w = (width + 63) / 64, fb_h = (height + 63) / 64;
  const int cols8 = (width + 7) / 8, rows8 = (height + 7) / 8;
  const int cs = bd - 8;
  uint16_t *pad[3];
  ptrdiff_t pstride[3];
  int pw[3], ph[3], xd[3], yd[3];
  for (int p = 0; p < 3; p++) {
    xd[p] = p ? xdec : 0;
    yd[p] = p ? ydec : 0;
    pw[p] = p ? (width + xdec) >> xdec : width;
    ph[p] = p ? (height + ydec) >> ydec : height;
    /* Plane::new((fb_w * 64) >> xdec, (fb_h * 64) >> ydec, xdec, ydec, 2, 2) */
    const int aw = ((fb_w * 64) >> xd[p]) + 4, ah = ((fb_h * 64) >> yd[p]) + 4;
    pstride[p] = aw;
    pad[p] = (uint16_t *)malloc(sizeof(uint16_t) * (size_t)aw * ah);
    for (size_t k = 0; k < (size_t)aw * ah; k++) pad[p][k] = 128;
    for (int y = -2; y < ph[p] + 2; y++)
      for (int x = -2; x < pw[p] + 2; x++) {
        uint16_t v = CDEF_VERY_LARGE;
        if (x >= 0 && x < pw[p] && y >= 0 && y < ph[p])
          v = hbd ? ((const uint16_t *)in[p])[y * istride[p] + x]
                  : ((const uint8_t *)in[p])[y * istride[p] + x];
        pad[p][(y + 2) * aw + x + 2] = v;
      }
  }
  for (int by8 = 0; by8 < rows8; by8++)
    for (int bx8 = 0; bx8 < cols8; bx8++) {
      const uint8_t *sk = skip + (size_t)(2 * by8) * mi_stride + 2 * bx8;
      const int is_skip = sk[0] & sk[1] & sk[mi_stride] & sk[mi_stride + 1];
      int dir = 0;
      int32_t var = 0;
      if (!is_skip)
        dir = orc_cdef_find_dir(pad[0] + (size_t)(8 * by8 + 2) * pstride[0] + 8 * bx8 + 2,
                                pstride[0], &var, cs);
      if (dirs) dirs[by8 * cols8 + bx8] = (uint8_t)dir;
      if (vars) vars[by8 * cols8 + bx8] = var;
      const int idx = cdef_index[(by8 / 8) * fb_w + bx8 / 8];
      const int ys = y_str[idx], uvs = uv_str[idx];
      const int pri_y = ys / 4, pri_uv = uvs / 4;
      int sec_y = ys % 4, sec_uv = uvs % 4;
      if (sec_y == 3) sec_y++;
      if (sec_uv == 3) sec_uv++;
      for (int p = 0; p < 3; p++) {
        const int xsize = 8 >> xd[p], ysize = 8 >> yd[p];
        const int x0 = (8 * bx8) >> xd[p], y0 = (8 * by8) >> yd[p];
        const uint16_t *src = pad[p] + (size_t)(y0 + 2) * pstride[p] + x0 + 2;
        /* only the visible part of the block (the reference also writes the
         * rec plane's padding columns / rows, which pad_frame overwrites) */
        uint16_t blk[64];
        if (!is_skip) {
          int pri, sec, dmp = damping + cs, d;
          if (p == 0) {
            pri = orc_cdef_adjust_strength(pri_y << cs, var);
            sec = sec_y << cs;
            d = pri_y ? dir : 0;
          } else {
            pri = pri_uv << cs;
            sec = sec_uv << cs;
            dmp -= 1;
            d = pri_uv ? dir : 0;
          }
          orc_cdef_filter_block(blk, 8, 1, src, pstride[p], pri, sec, d, dmp, bd, xd[p], yd[p]);
        } else {
          for (int i = 0; i < ysize; i++)
            for (int j = 0; j < xsize; j++) blk[i * 8 + j] = src[i * pstride[p] + j];
        }
        for (int i = 0; i < ysize && y0 + i < ph[p]; i++)
          for (int j = 0; j < xsize && x0 + j < pw[p]; j++) {
            const size_t o = (size_t)(y0 + i) * ostride[p] + x0 + j;
            if (hbd)
              ((uint16_t *)out[p])[o] = blk[i * 8 + j];
            else
              ((uint8_t *)out[p])[o] = (uint8_t)blk[i * 8 + j];
          }
      }
    }
  for (int p = 0; p < 3; p++) free(pad[p]);
}
