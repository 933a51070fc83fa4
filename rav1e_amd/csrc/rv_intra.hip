// rv_intra.hip -- batched intra prediction: PredictionMode::predict_intra
// without CfL (src/predict.rs:202-241) over the native Intra trait
// (src/predict.rs:538-1035), one wavefront per block.
//
// Every job brings rav1e's edge_buf (4 * MAX_TX_SIZE + 1 pixels, built by
// get_intra_edges, src/recon_intra.rs): left pixels bottom-to-top and
// right-aligned in [0, 128), the top-left pixel at 128, the above row from
// 129.  The wavefront stages it in LDS as i32 and writes the predicted
// block (up to 64 x 64) row-major, lanes across columns, into the
// destination plane.  Modes and variants are uniform per wavefront.
#include "rv_device.h"

namespace rv {

// sm_weight_arrays (src/predict.rs:406-424)
__constant__ uint8_t kSmW[128] = {
    0,   0,   255, 128, 255, 149, 85,  64,  255, 197, 146, 105, 73,  50,  37,  32,
    255, 225, 196, 170, 145, 123, 102, 84,  68,  54,  43,  33,  26,  20,  17,  16,
    255, 240, 225, 210, 196, 182, 169, 157, 145, 133, 122, 111, 101, 92,  83,  74,
    66,  59,  52,  45,  39,  34,  29,  25,  21,  17,  14,  12,  10,  9,   8,   8,
    255, 248, 240, 233, 225, 218, 210, 203, 196, 189, 182, 176, 169, 163, 156, 150,
    144, 138, 133, 127, 121, 116, 111, 106, 101, 96,  91,  86,  82,  77,  73,  69,
    65,  61,  57,  54,  50,  47,  44,  41,  38,  35,  32,  29,  27,  25,  22,  20,
    18,  16,  15,  13,  12,  10,  9,   8,   7,   6,   6,   5,   5,   4,   4,   4};

// dr_intra_derivative (src/predict.rs:912-944) for the six angles rav1e uses
__device__ __forceinline__ int dr_deriv(int a) {
  switch (a) {
    case 45: return 64;
    case 23: return 151;
    case 67: return 27;
    default: return 0;
  }
}

constexpr int kEdge = 4 * 64 + 1;
constexpr uint8_t kTxW[19] = {4, 8, 16, 32, 64, 4, 8, 8, 16, 16, 32, 32, 64, 4, 16, 8, 32, 16, 64};
constexpr uint8_t kTxH[19] = {4, 8, 16, 32, 64, 8, 4, 16, 8, 32, 16, 64, 32, 16, 4, 32, 8, 64, 16};

template <typename Px>
__global__ __launch_bounds__(64) void intra_kernel(rv_plane dst, const rv_intra_job *jobs,
                                                    const Px *edges, int w, int h, int bd) {
  __shared__ int32_t e[kEdge + 3];
  const int lane = threadIdx.x;
  const rv_intra_job j = jobs[blockIdx.x];
  const Px *eb = edges + (int64_t)blockIdx.x * kEdge;
  for (int i = lane; i < kEdge; i += 64) e[i] = eb[i];
  __syncthreads();
  // predict_intra's remaps (src/predict.rs:214-233)
  int mode = j.mode;
  const int variant = j.variant;
  if (mode == 12) mode = variant == 0 ? 0 : variant == 1 ? 2 : variant == 2 ? 1 : 12;
  const int angle = mode == 3 ? 45 : mode == 4 ? 135 : mode == 5 ? 113 : mode == 6 ? 157
                  : mode == 7 ? 203 : mode == 8 ? 67 : 0;
  const int maxv = (1 << bd) - 1;
  const int L0 = 128 - h, LB = 128 - h - w, A0 = 129;
  const int32_t tl = e[128];
  int32_t dcv = 0;
  if (mode == 0) {  // DC_PRED: the sums over the edges, one wave reduction
    uint32_t s = 0;
    if (variant & 1)
      for (int k = lane; k < h; k += 64) s += (uint32_t)e[L0 + k];
    if (variant & 2)
      for (int k = lane; k < w; k += 64) s += (uint32_t)e[A0 + k];
    s = group_sum<64>(s);
    const uint32_t len = (variant & 1 ? h : 0) + (variant & 2 ? w : 0);
    dcv = variant == 0 ? (128 << (bd - 8)) : (int32_t)((s + (len >> 1)) / len);
  }
  const int dx = angle < 90 ? dr_deriv(angle) : (angle > 90 && angle < 180 ? dr_deriv(180 - angle) : 0);
  const int dy = (angle > 90 && angle < 180) ? dr_deriv(angle - 90)
                                             : (angle > 180 ? dr_deriv(270 - angle) : 0);
  for (int i = lane; i < w * h; i += 64) {
    const int r = i / w, c = i - r * w;
    int32_t v;
    switch (mode) {
      case 0: v = dcv; break;
      case 1: v = e[A0 + c]; break;                 // V_PRED
      case 2: v = e[L0 + h - 1 - r]; break;         // H_PRED
      case 12: {                                    // PAETH_PRED
        const int32_t l = e[L0 + h - 1 - r], t = e[A0 + c];
        const int32_t base = t + l - tl;
        const int32_t pl = abs(base - l), pt = abs(base - t), ptl = abs(base - tl);
        v = (pl <= pt && pl <= ptl) ? l : (pt <= ptl ? t : tl);
        break;
      }
      case 9: {  // SMOOTH_PRED: weights scaled by 2^8, log2_scale 9
        const uint32_t wh = kSmW[h + r], ww = kSmW[w + c];
        const uint32_t s = wh * (uint32_t)e[A0 + c] + (256 - wh) * (uint32_t)e[L0] +
                           ww * (uint32_t)e[L0 + h - 1 - r] + (256 - ww) * (uint32_t)e[A0 + w - 1];
        v = (int32_t)((s + 256) >> 9);
        break;
      }
      case 11: {  // SMOOTH_H_PRED
        const uint32_t ww = kSmW[w + c];
        v = (int32_t)((ww * (uint32_t)e[L0 + h - 1 - r] + (256 - ww) * (uint32_t)e[A0 + w - 1] + 128) >> 8);
        break;
      }
      case 10: {  // SMOOTH_V_PRED
        const uint32_t wh = kSmW[h + r];
        v = (int32_t)((wh * (uint32_t)e[A0 + c] + (256 - wh) * (uint32_t)e[L0] + 128) >> 8);
        break;
      }
      default: {  // pred_directional (src/predict.rs:894-1034), no edge filter / upsampling
        if (angle < 90) {
          const int idx = (r + 1) * dx, base = (idx >> 6) + c, shift = (idx >> 1) & 31;
          const int mb = h + w - 1;
          v = base < mb ? round_shift(e[A0 + base] * (32 - shift) + e[A0 + base + 1] * shift, 5)
                        : e[A0 + mb];
        } else if (angle < 180) {
          const int idx = (c << 6) - (r + 1) * dx, base = idx >> 6;
          if (base >= -1) {
            const int shift = (idx >> 1) & 31;
            const int32_t a = base < 0 ? tl : e[A0 + base];
            v = round_shift(a * (32 - shift) + e[A0 + base + 1] * shift, 5);
          } else {
            const int idy = (r << 6) - (c + 1) * dy, bl = idy >> 6, shift = (idy >> 1) & 31;
            const int32_t a = bl < 0 ? tl : e[LB + w + h - 1 - bl];
            v = round_shift(a * (32 - shift) + e[LB + w + h - 2 - bl] * shift, 5);
          }
        } else {
          const int idx = (c + 1) * dy, base = (idx >> 6) + r, shift = (idx >> 1) & 31;
          v = round_shift(e[LB + w + h - 1 - base] * (32 - shift) + e[LB + w + h - 2 - base] * shift, 5);
        }
        v = v < 0 ? 0 : (v > maxv ? maxv : v);
        break;
      }
    }
    *plane_ptr_mut<Px>(dst, j.x + c, j.y + r) = (Px)v;
  }
}

}  // namespace rv

using namespace rv;

extern "C" int rv_predict_intra_batch(const rv_plane *dst, const rv_intra_job *d_jobs,
                                      const void *d_edges, int n, int tx_size, int bit_depth,
                                      void *stream) {
  if (!dst || n < 0 || tx_size < 0 || tx_size > 18 ||
      (bit_depth != 8 && bit_depth != 10 && bit_depth != 12) || (dst->hbd != (bit_depth > 8)) ||
      (n > 0 && (!d_jobs || !d_edges)))
    return rv_set_error(RV_EINVAL, "rv_predict_intra_batch: bad arguments");
  if (n == 0) return RV_OK;
  hipStream_t s = rv_resolve_stream(stream);
  const int w = kTxW[tx_size], h = kTxH[tx_size];
  if (dst->hbd)
    intra_kernel<uint16_t><<<n, 64, 0, s>>>(*dst, d_jobs, (const uint16_t *)d_edges, w, h, bit_depth);
  else
    intra_kernel<uint8_t><<<n, 64, 0, s>>>(*dst, d_jobs, (const uint8_t *)d_edges, w, h, bit_depth);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}
