// rv_tx_inv.hip -- batched inverse 2-D transform + add (gfx950).
//
// NativeInvTxfm2D::inv_txfm2d_add (src/transform/inverse.rs:1939-2114):
// row transforms over the first min(H, 32) rows of min(W, 32) coefficients
// (rectangular 2:1 sizes pre-scaled by 1/sqrt2 = 2896 >> 12, inputs clamped
// to bd + 8 bits), INTERMEDIATE_SHIFT rounding + clamp to max(bd + 6, 16)
// bits, column transforms, round_shift 4, add into the destination with a
// clip to [0, 2^bd - 1].  Same wavefront layout as the forward launch:
// 64 / max(W, H) blocks per wavefront, LDS rows padded to W + 1.
#include "rv_tx.h"

namespace rv {

// InvBlock::INTERMEDIATE_SHIFT (inverse.rs:1643-1666) by TxSize.
__constant__ uint8_t kInvShift[19] = {0, 1, 2, 2, 2, 0, 0, 1, 1, 1,
                                      1, 1, 1, 1, 1, 2, 2, 2, 2};

struct InvArgs {
  const int32_t *coeffs;
  rv_plane dst;
  const rv_tx_job *jobs;
  int n, tx_size, ck, rk, bd;
};

template <int KIND, int N>
__device__ __forceinline__ void inv_dispatch(int32_t *v, int range) {
  if constexpr (tx::inv_supported(KIND, N)) tx::inv1d<KIND, N>(v, range);
}
template <int N>
__device__ __forceinline__ void inv_kind(int kind, int32_t *v, int range) {
  switch (kind) {
    case 0: inv_dispatch<0, N>(v, range); break;
    case 1: inv_dispatch<1, N>(v, range); break;
    default: inv_dispatch<2, N>(v, range); break;
  }
}

template <int W, int H, typename Px>
__global__ __launch_bounds__(64) void inv_tx_kernel(InvArgs a) {
  constexpr int L = W > H ? W : H;
  constexpr int TPW = 64 / L;
  constexpr int S = W + 1;
  constexpr int CW = W < 32 ? W : 32, CH = H < 32 ? H : 32;
  constexpr int WL = tx::lg2<W>(), HL = tx::lg2<H>();
  constexpr bool RECT2 = (WL - HL == 1) || (HL - WL == 1);
  __shared__ int32_t buf[TPW * H * S];
  const int lane = threadIdx.x;
  const int tx0 = blockIdx.x * TPW;
  const int range = a.bd + 8;

  // 1. coefficients (row stride CW) -> LDS rows; zero the rest
  for (int i = lane; i < TPW * H * W; i += 64) {
    const int sub = i / (H * W), e = i - sub * (H * W);
    const int r = e / W, c = e - r * W;
    const int t = tx0 + sub;
    int32_t v = 0;
    if (t < a.n && r < CH && c < CW) {
      const int32_t raw = a.coeffs[(int64_t)t * CW * CH + r * CW + c];
      v = RECT2 ? round_shift(wmul(raw, 2896), 12) : raw;
      v = tx::clampv(v, range);
    }
    buf[sub * H * S + r * S + c] = v;
  }
  __syncthreads();
  const int sub = lane / L, l = lane - sub * L;
  int32_t *blk = buf + sub * H * S;
  // 2. row pass (rows >= 32 are all zero and transform to zero)
  if (l < CH) {
    int32_t v[W];
#pragma unroll
    for (int c = 0; c < W; c++) v[c] = blk[l * S + c];
    inv_kind<W>(a.rk, v, range);
#pragma unroll
    for (int c = 0; c < W; c++) blk[l * S + c] = v[c];
  }
  __syncthreads();
  // 3. column pass + add
  const int t = tx0 + sub;
  if (l < W && t < a.n) {
    const int crange = a.bd + 6 > 16 ? a.bd + 6 : 16;
    const int shift = kInvShift[a.tx_size];
    int32_t v[H];
#pragma unroll
    for (int r = 0; r < H; r++) v[r] = tx::clampv(round_shift(blk[r * S + l], shift), crange);
    inv_kind<H>(a.ck, v, crange);
    const rv_tx_job jb = a.jobs[t];
    Px *dp = plane_ptr_mut<Px>(a.dst, jb.pred_x + l, jb.pred_y);
    const int32_t maxv = (1 << a.bd) - 1;
#pragma unroll
    for (int r = 0; r < H; r++) {
      Px *p = dp + (int64_t)r * a.dst.stride;
      *p = (Px)clampi(wadd((int32_t)*p, round_shift(v[r], 4)), 0, maxv);
    }
  }
}

template <typename Px>
static int launch_inv(InvArgs a, hipStream_t s) {
  const int wl = tx_w_log2(a.tx_size), hl = tx_h_log2(a.tx_size);
  const int L = 1 << (wl > hl ? wl : hl);
  const int tpw = 64 / L;
  dim3 grid((a.n + tpw - 1) / tpw);
  switch (a.tx_size) {
#define RV_CASE(ID, W, H)                              \
  case ID:                                             \
    inv_tx_kernel<W, H, Px><<<grid, 64, 0, s>>>(a);    \
    break;
    RV_CASE(0, 4, 4) RV_CASE(1, 8, 8) RV_CASE(2, 16, 16) RV_CASE(3, 32, 32)
    RV_CASE(4, 64, 64) RV_CASE(5, 4, 8) RV_CASE(6, 8, 4) RV_CASE(7, 8, 16)
    RV_CASE(8, 16, 8) RV_CASE(9, 16, 32) RV_CASE(10, 32, 16) RV_CASE(11, 32, 64)
    RV_CASE(12, 64, 32) RV_CASE(13, 4, 16) RV_CASE(14, 16, 4) RV_CASE(15, 8, 32)
    RV_CASE(16, 32, 8) RV_CASE(17, 16, 64) RV_CASE(18, 64, 16)
#undef RV_CASE
  }
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

}  // namespace rv

using namespace rv;

extern "C" int rv_inv_txfm_add_batch(const int32_t *d_coeffs,
                                     const rv_plane *dst,
                                     const rv_tx_job *d_jobs, int n,
                                     int tx_size, int tx_type, int bit_depth,
                                     void *stream) {
  if (!dst || n < 0 || tx_size < 0 || tx_size > 18 || tx_type < 0 ||
      tx_type > 15 || (bit_depth != 8 && bit_depth != 10 && bit_depth != 12) ||
      (!dst->hbd && bit_depth != 8))
    return rv_set_error(RV_EINVAL, "rv_inv_txfm_add_batch: bad arguments");
  const int ck = tx_col_kind(tx_type), rk = tx_row_kind(tx_type);
  const int w = 1 << tx_w_log2(tx_size), h = 1 << tx_h_log2(tx_size);
  // the native 2-D path implements no FlipAdst, no Adst32/64, no Id64
  if (!tx::inv_supported(ck, h) || !tx::inv_supported(rk, w))
    return rv_set_error(RV_ENOTSUP, "rv_inv_txfm_add_batch: unsupported type");
  if (n == 0) return RV_OK;
  InvArgs a{d_coeffs, *dst, d_jobs, n, tx_size, ck, rk, bit_depth};
  hipStream_t s = rv_resolve_stream(stream);
  return dst->hbd ? launch_inv<uint16_t>(a, s) : launch_inv<uint8_t>(a, s);
}
