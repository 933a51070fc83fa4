// rv_tx_fwd.hip -- batched forward 2-D transform (gfx950).
//
// FwdTxfm2D::fht (src/transform/forward.rs:1804-1899) for a batch of
// same-size, same-type transform blocks.  One 64-lane wavefront owns
// 64 / max(W, H) blocks; the block is staged in LDS (row stride W + 1, so
// both the column pass and the row pass are bank-conflict free), each lane
// runs one 1-D transform of one column, then of one row, entirely in VGPRs,
// and the W x H raster leaves through coalesced stores.  Integer only: these
// are lifting networks, not dense GEMMs, so MFMA does not apply.
//
// The fused form reads src - pred (diff, src/encoder.rs:1044-1058) straight
// from the planes, so the i16 residual never exists in HBM.
#include "rv_tx.h"

namespace rv {

// FWD_SHIFT_* (forward.rs:22-40) by TxSize, shift_idx = (bd - 8) / 2.
__constant__ int8_t kFwdShift[19][3][3] = {
    {{3, 0, 0}, {2, 0, 1}, {0, 0, 3}},    {{4, -1, 0}, {2, 0, 1}, {0, 0, 3}},
    {{4, -1, 0}, {2, 0, 1}, {0, 0, 3}},   {{4, -2, 0}, {2, 0, 0}, {0, 0, 2}},
    {{4, -1, -2}, {2, 0, -1}, {0, 0, 1}}, {{4, -1, 0}, {2, 0, 1}, {0, 0, 3}},
    {{4, -1, 0}, {2, 0, 1}, {0, 0, 3}},   {{4, -1, 0}, {2, 0, 1}, {0, 0, 3}},
    {{4, -1, 0}, {2, 0, 1}, {0, 0, 3}},   {{4, -2, 0}, {2, 0, 0}, {0, 0, 2}},
    {{4, -2, 0}, {2, 0, 0}, {0, 0, 2}},   {{4, -1, -2}, {2, 0, -1}, {0, 0, 1}},
    {{4, -1, -2}, {2, 0, -1}, {0, 0, 1}}, {{4, -1, 0}, {2, 0, 1}, {0, 0, 3}},
    {{4, -1, 0}, {2, 0, 1}, {0, 0, 3}},   {{4, -1, 0}, {2, 0, 1}, {0, 0, 3}},
    {{4, -1, 0}, {2, 0, 1}, {0, 0, 3}},   {{4, -2, 0}, {2, 0, 0}, {0, 0, 2}},
    {{4, -2, 0}, {2, 0, 0}, {0, 0, 2}}};

// round_shift_array (src/transform/mod.rs:499-521): bit > 0 rounds right,
// bit < 0 shifts left.
__device__ __forceinline__ int32_t rsa(int32_t v, int bit) {
  if (bit > 0) return round_shift(v, bit);
  if (bit < 0) return (int32_t)((uint32_t)v << -bit);
  return v;
}

enum FwdSrc { kFromResidual = 0, kFromPlanesU8 = 1, kFromPlanesU16 = 2 };

struct FwdArgs {
  const int16_t *residual;
  rv_plane src, pred;
  const rv_tx_job *jobs;
  int32_t *coeffs;
  int n, tx_size, ck, rk, shift_idx;
};

template <int KIND, int N>
__device__ __forceinline__ void fwd_dispatch(int32_t *v) {
  if constexpr (tx::fwd_supported(KIND, N)) tx::fwd1d<KIND, N>(v, v);
}

template <int N>
__device__ __forceinline__ void fwd_kind(int kind, int32_t *v) {
  switch (kind) {
    case 0: fwd_dispatch<0, N>(v); break;
    case 1: fwd_dispatch<1, N>(v); break;
    default: fwd_dispatch<2, N>(v); break;  // Adst and FlipAdst (flip is 2-D)
  }
}

template <int W, int H, int SRC>
__global__ __launch_bounds__(64) void fwd_tx_kernel(FwdArgs a) {
  constexpr int L = W > H ? W : H;  // lanes per block
  constexpr int TPW = 64 / L;       // blocks per wavefront
  constexpr int S = W + 1;          // padded LDS row stride
  __shared__ int32_t buf[TPW * H * S];
  const int lane = threadIdx.x;
  const int tx0 = blockIdx.x * TPW;
  const int8_t *sh = kFwdShift[a.tx_size][a.shift_idx];
  const int s0 = sh[0], s1 = sh[1], s2 = sh[2];

  // 1. stage the residual block(s) into LDS, coalesced, << -shift[0]
  for (int i = lane; i < TPW * W * H; i += 64) {
    const int sub = i / (W * H), e = i - sub * (W * H);
    const int r = e / W, c = e - r * W;
    const int t = tx0 + sub;
    int32_t v = 0;
    if (t < a.n) {
      if constexpr (SRC == kFromResidual) {
        v = a.residual[(int64_t)t * W * H + e];
      } else {
        const rv_tx_job jb = a.jobs[t];
        if constexpr (SRC == kFromPlanesU8) {
          v = (int32_t)(int16_t)((int16_t)*plane_ptr<uint8_t>(a.src, jb.src_x + c, jb.src_y + r) -
                                 (int16_t)*plane_ptr<uint8_t>(a.pred, jb.pred_x + c, jb.pred_y + r));
        } else {
          v = (int32_t)(int16_t)((int16_t)*plane_ptr<uint16_t>(a.src, jb.src_x + c, jb.src_y + r) -
                                 (int16_t)*plane_ptr<uint16_t>(a.pred, jb.pred_x + c, jb.pred_y + r));
        }
      }
    }
    buf[sub * H * S + r * S + c] = rsa(v, -s0);
  }
  __syncthreads();

  const int sub = lane / L, l = lane - sub * L;
  int32_t *blk = buf + sub * H * S;
  // 2. column pass (Col::FLIPPED flips upside down, forward.rs:1829-1836)
  if (l < W) {
    int32_t v[H];
#pragma unroll
    for (int r = 0; r < H; r++)
      v[r] = blk[(a.ck == 3 ? H - 1 - r : r) * S + l];
    fwd_kind<H>(a.ck, v);
#pragma unroll
    for (int r = 0; r < H; r++) blk[r * S + l] = rsa(v[r], -s1);
  }
  __syncthreads();
  // 3. row pass
  if (l < H) {
    int32_t v[W];
#pragma unroll
    for (int c = 0; c < W; c++) v[c] = blk[l * S + c];
    fwd_kind<W>(a.rk, v);
#pragma unroll
    for (int c = 0; c < W; c++) blk[l * S + c] = rsa(v[c], -s2);
  }
  __syncthreads();
  // 4. coalesced store of the W-stride raster(s)
  for (int i = lane; i < TPW * W * H; i += 64) {
    const int sb = i / (W * H), e = i - sb * (W * H);
    const int r = e / W, c = e - r * W;
    if (tx0 + sb < a.n)
      a.coeffs[(int64_t)(tx0 + sb) * W * H + e] = buf[sb * H * S + r * S + c];
  }
}

template <int SRC>
static int launch_fwd(FwdArgs a, hipStream_t s) {
  const int wl = tx_w_log2(a.tx_size), hl = tx_h_log2(a.tx_size);
  const int L = 1 << (wl > hl ? wl : hl);
  const int tpw = 64 / L;
  dim3 grid((a.n + tpw - 1) / tpw);
  switch (a.tx_size) {
#define RV_CASE(ID, W, H)                                   \
  case ID:                                                  \
    fwd_tx_kernel<W, H, SRC><<<grid, 64, 0, s>>>(a);        \
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

// Validates (size, type, bd) exactly as FwdTxfm2D::fht + txfm_types would
// accept them: both 1-D kernels must exist, no row FlipAdst (the flipped-row
// branch is unreachable in the reference, forward.rs:1858-1862).
static int fwd_check(int tx_size, int tx_type, int bd, int *ck, int *rk) {
  if (tx_size < 0 || tx_size > 18 || tx_type < 0 || tx_type > 15 ||
      (bd != 8 && bd != 10 && bd != 12))
    return RV_EINVAL;
  *ck = tx_col_kind(tx_type);
  *rk = tx_row_kind(tx_type);
  const int w = 1 << tx_w_log2(tx_size), h = 1 << tx_h_log2(tx_size);
  if (*rk == 3 || !tx::fwd_supported(*ck, h) || !tx::fwd_supported(*rk, w))
    return RV_ENOTSUP;
  return RV_OK;
}

}  // namespace rv

using namespace rv;

extern "C" {

int rv_fwd_txfm_batch(const int16_t *d_residual, int32_t *d_coeffs, int n,
                      int tx_size, int tx_type, int bit_depth, void *stream) {
  int ck, rk;
  int e = fwd_check(tx_size, tx_type, bit_depth, &ck, &rk);
  if (e || n < 0)
    return rv_set_error(e ? e : RV_EINVAL, "rv_fwd_txfm_batch: unsupported");
  if (n == 0) return RV_OK;
  FwdArgs a{};
  a.residual = d_residual;
  a.coeffs = d_coeffs;
  a.n = n;
  a.tx_size = tx_size;
  a.ck = ck;
  a.rk = rk;
  a.shift_idx = (bit_depth - 8) / 2;
  return launch_fwd<kFromResidual>(a, rv_resolve_stream(stream));
}

int rv_diff_fwd_txfm_batch(const rv_plane *src, const rv_plane *pred,
                           const rv_tx_job *d_jobs, int n, int tx_size,
                           int tx_type, int bit_depth, int32_t *d_coeffs,
                           void *stream) {
  int ck, rk;
  int e = fwd_check(tx_size, tx_type, bit_depth, &ck, &rk);
  if (e || n < 0 || !src || !pred || src->hbd != pred->hbd)
    return rv_set_error(e ? e : RV_EINVAL,
                        "rv_diff_fwd_txfm_batch: bad arguments");
  if (n == 0) return RV_OK;
  FwdArgs a{};
  a.src = *src;
  a.pred = *pred;
  a.jobs = d_jobs;
  a.coeffs = d_coeffs;
  a.n = n;
  a.tx_size = tx_size;
  a.ck = ck;
  a.rk = rk;
  a.shift_idx = (bit_depth - 8) / 2;
  hipStream_t s = rv_resolve_stream(stream);
  return src->hbd ? launch_fwd<kFromPlanesU16>(a, s)
                  : launch_fwd<kFromPlanesU8>(a, s);
}

}  // extern "C"
