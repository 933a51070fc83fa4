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
#include "rv_intra.h"

namespace rv {

constexpr uint8_t kTxW[19] = {4, 8, 16, 32, 64, 4, 8, 8, 16, 16, 32, 32, 64, 4, 16, 8, 32, 16, 64};
constexpr uint8_t kTxH[19] = {4, 8, 16, 32, 64, 8, 4, 16, 8, 32, 16, 64, 32, 16, 4, 32, 8, 64, 16};

template <typename Px>
__global__ __launch_bounds__(64) void intra_kernel(rv_plane dst, const rv_intra_job *jobs,
                                                    const Px *edges, int w, int h, int bd) {
  __shared__ int32_t e[kIntraEdge + 3];
  const int lane = threadIdx.x;
  const rv_intra_job j = jobs[blockIdx.x];
  const Px *eb = edges + (int64_t)blockIdx.x * kIntraEdge;
  for (int i = lane; i < kIntraEdge; i += 64) e[i] = eb[i];
  __syncthreads();
  IntraSetup st = intra_setup(j.mode, j.variant);
  if (st.mode == 0) st.dcv = intra_dc<64>(e, j.variant, w, h, bd, lane);
  const int maxv = (1 << bd) - 1;
  for (int i = lane; i < w * h; i += 64) {
    const int r = i / w, c = i - r * w;
    *plane_ptr_mut<Px>(dst, j.x + c, j.y + r) = (Px)intra_px(st, e, w, h, r, c, maxv);
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
