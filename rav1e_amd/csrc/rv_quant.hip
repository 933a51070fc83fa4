// rv_quant.hip -- batched quantize / dequantize (src/quantize.rs), one
// wavefront per transform block (rv_quant.h has the algorithm).
#include "rv_quant.h"
#include "rv_rdo.h"

namespace rv {

constexpr uint8_t kQTxWLog2[19] = {2, 3, 4, 5, 6, 2, 3, 3, 4, 4, 5, 5, 6, 2, 4, 3, 5, 4, 6};
constexpr uint8_t kQTxHLog2[19] = {2, 3, 4, 5, 6, 3, 2, 4, 3, 5, 4, 6, 5, 4, 2, 5, 3, 6, 4};

struct QArgs {
  const int32_t *coeffs;
  int cstride, n, area, coded, tx_index;  // tx_index = tx_size * 16 + tx_type
  int qindex, bd, is_intra, dc_delta_q, ac_delta_q;
  int32_t *qcoeffs, *rcoeffs;
  uint32_t *eob;
};

template <int N>
__global__ __launch_bounds__(64) void quantize_kernel(QArgs a) {
  const int blk = blockIdx.x;
  if (blk >= a.n) return;
  const QCtx c = q_ctx(a.qindex, a.area, a.is_intra, a.bd, a.dc_delta_q, a.ac_delta_q);
  const int32_t *co = a.coeffs + (int64_t)blk * a.cstride;
  int32_t *q = a.qcoeffs + (int64_t)blk * a.coded;
  int32_t *r = a.rcoeffs ? a.rcoeffs + (int64_t)blk * a.coded : nullptr;
  const int eob = quantize_block<N, 64>(
      c, RV_SCANS + RV_SCAN_OFF[a.tx_index], [&](int pos) { return co[pos]; },
      [&](int pos, int32_t qv, int32_t rv) {
        q[pos] = qv;
        if (r) r[pos] = rv;
      });
  if (a.eob && threadIdx.x == 0) a.eob[blk] = (uint32_t)eob;
}

__global__ __launch_bounds__(256) void dequantize_kernel(const int32_t *q, int total, int coded,
                                                         int lts, int qindex, int bd,
                                                         int dc_delta_q, int ac_delta_q,
                                                         int32_t *r) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int32_t v = q[i];
  const int32_t quant = (i % coded) == 0 ? q_lookup(0, qindex, dc_delta_q, bd)
                                         : q_lookup(1, qindex, ac_delta_q, bd);
  r[i] = wadd(wmul(v, quant), (v >> 31) & ((1 << lts) - 1)) >> lts;
}

// estimate_rate (src/rdo.rs:204-216), one block per thread (q_estimate_rate).
__global__ __launch_bounds__(256) void estimate_rate_kernel(const uint64_t *dist, int n,
                                                            int qindex, int tx_size,
                                                            uint64_t *rate) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  rate[i] = q_estimate_rate(qindex, tx_size, dist[i]);
}

__global__ void q_ctx_kernel(int qindex, int area, int is_intra, int bd, int dc_delta_q,
                             int ac_delta_q, QCtx *out) {
  *out = q_ctx(qindex, area, is_intra, bd, dc_delta_q, ac_delta_q);
}

}  // namespace rv

using namespace rv;

int rv_quant_ctx(int qindex, int tx_area, int is_intra, int bit_depth, int dc_delta_q,
                 int ac_delta_q, QCtx *out) {
  QCtx *d = nullptr;
  if (hipMalloc((void **)&d, sizeof(QCtx)) != hipSuccess)
    return rv_set_error(RV_EHIP, "rv_quant_ctx: alloc");
  q_ctx_kernel<<<1, 1>>>(qindex, tx_area, is_intra, bit_depth, dc_delta_q, ac_delta_q, d);
  const bool ok = hipMemcpy(out, d, sizeof(QCtx), hipMemcpyDeviceToHost) == hipSuccess;
  (void)hipFree(d);
  return ok ? RV_OK : rv_set_error(RV_EHIP, "rv_quant_ctx");
}

extern "C" int rv_quantize_batch(const int32_t *d_coeffs, int coeff_stride, int n, int tx_size,
                                 int tx_type, int qindex, int bit_depth, int is_intra,
                                 int dc_delta_q, int ac_delta_q, int32_t *d_qcoeffs,
                                 int32_t *d_rcoeffs, uint32_t *d_eob, void *stream) {
  if (n < 0 || tx_size < 0 || tx_size > 18 || tx_type < 0 || tx_type > 15 || qindex < 1 ||
      qindex > 255 || (bit_depth != 8 && bit_depth != 10 && bit_depth != 12) ||
      (n > 0 && (!d_coeffs || !d_qcoeffs)))
    return rv_set_error(RV_EINVAL, "rv_quantize_batch: bad arguments");
  const int w = 1 << kQTxWLog2[tx_size], h = 1 << kQTxHLog2[tx_size];
  const int coded = (w < 32 ? w : 32) * (h < 32 ? h : 32);
  if (coeff_stride < coded)
    return rv_set_error(RV_EINVAL, "rv_quantize_batch: coeff_stride below the coded area");
  if (n == 0) return RV_OK;
  QArgs a{d_coeffs, coeff_stride, n, w * h, coded, tx_size * 16 + tx_type, qindex, bit_depth,
          is_intra ? 1 : 0, dc_delta_q, ac_delta_q, d_qcoeffs, d_rcoeffs, d_eob};
  hipStream_t st = rv_resolve_stream(stream);
  switch (coded) {  // coded areas of the 19 TxSizes: 16 .. 1024
#define RV_QCASE(N) \
  case N:           \
    quantize_kernel<N><<<n, 64, 0, st>>>(a); \
    break;
    RV_QCASE(16) RV_QCASE(32) RV_QCASE(64) RV_QCASE(128) RV_QCASE(256) RV_QCASE(512) RV_QCASE(1024)
#undef RV_QCASE
    default:
      return rv_set_error(RV_EINVAL, "rv_quantize_batch: coded area");
  }
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

extern "C" int rv_dequantize_batch(const int32_t *d_qcoeffs, int n, int tx_size, int qindex,
                                   int bit_depth, int dc_delta_q, int ac_delta_q,
                                   int32_t *d_rcoeffs, void *stream) {
  if (n < 0 || tx_size < 0 || tx_size > 18 || qindex < 1 || qindex > 255 ||
      (bit_depth != 8 && bit_depth != 10 && bit_depth != 12) ||
      (n > 0 && (!d_qcoeffs || !d_rcoeffs)))
    return rv_set_error(RV_EINVAL, "rv_dequantize_batch: bad arguments");
  if (n == 0) return RV_OK;
  const int w = 1 << kQTxWLog2[tx_size], h = 1 << kQTxHLog2[tx_size];
  const int coded = (w < 32 ? w : 32) * (h < 32 ? h : 32);
  const int total = n * coded;
  dequantize_kernel<<<(total + 255) / 256, 256, 0, rv_resolve_stream(stream)>>>(
      d_qcoeffs, total, coded, q_log_tx_scale(w * h), qindex, bit_depth, dc_delta_q, ac_delta_q,
      d_rcoeffs);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

extern "C" int rv_estimate_rate_batch(const uint64_t *d_tx_dist, int n, int qindex, int tx_size,
                                      uint64_t *d_rate, void *stream) {
  if (n < 0 || qindex < 0 || qindex > 255 || tx_size < 0 || tx_size > 18 ||
      (n > 0 && (!d_tx_dist || !d_rate)))
    return rv_set_error(RV_EINVAL, "rv_estimate_rate_batch: bad arguments");
  if (n == 0) return RV_OK;
  estimate_rate_kernel<<<(n + 255) / 256, 256, 0, rv_resolve_stream(stream)>>>(
      d_tx_dist, n, qindex, tx_size, d_rate);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

// dc_q / ac_q (src/quantize.rs:42-62) on the host: the fixed-quantizer
// parameters (rav1e_amd/rate.py, src/rate.rs:746-775) select qindices from
// these lookups.  ac = 0: dc_qlookup*_Q3, 1: ac_qlookup*_Q3; -1 on bad args.
extern "C" int rv_q_lookup(int ac, int qindex, int bit_depth) {
  if ((ac != 0 && ac != 1) || qindex < 0 || qindex > 255 ||
      (bit_depth != 8 && bit_depth != 10 && bit_depth != 12))
    return -1;
  return RV_QLOOKUP_HOST[(3 * ac + (bit_depth - 8) / 2) * 256 + qindex];
}
