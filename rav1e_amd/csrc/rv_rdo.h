// rv_rdo.h -- the fused RDO inter-candidate launch (rv_rdo.hip), used by the
// replay driver's stage F4.
#pragma once

#include "rv_device.h"
#include "rv_quant.h"

namespace rv {

struct RdoPlane {
  rv_plane org;                  // source plane
  rv_plane ref[RV_DS_MAX_PRED];  // reference planes of this plane type
  rv_plane dst;                  // tall prediction / reconstruction plane
  const rv_mc_job *mc;           // per candidate
  const rv_tx_job *tx;           // per (candidate, transform block)
  int32_t *packed;               // per transform block: min(N,32)^2 i32
  void *dist;                    // luma: i64 x 5 per 8x8; chroma: u64 per sub-block
};

struct RdoArgs {
  RdoPlane p[2];      // blockIdx.y selects the plane (chroma: U, V)
  int n_tx;           // transform blocks per plane in this launch
  int k_sel;          // -1: every candidate; 0 / 1: only candidates 2r + k_sel
  int nsb;            // superblocks (candidate c of SB sb = c * nsb + sb)
  int ntx_per_cand;   // transform blocks per candidate
  int cands_per_ref;  // candidates of one reference (job arrays are ref-major)
  int bd;
  int mb_w, mb_h;     // MC block size (filter choice, distortion grid)
  int sub_w, sub_h;   // distortion sub-block (SSE); moments use 8x8
  QCtx q;             // QuantizationContext of this plane type's transform
  int q_tx_index;     // tx_size * 16 + tx_type: av1_scan_orders entry
};

}  // namespace rv

// QuantizationContext::update (src/quantize.rs:205-253) evaluated on the
// device (the lookups live there), for the replay's launch arguments.
int rv_quant_ctx(int qindex, int tx_area, int is_intra, int bit_depth, int dc_delta_q,
                 int ac_delta_q, rv::QCtx *out);

// Luma candidates (64x64 transform, cdef moments) and the chroma transform
// blocks of planes U and V (32x32, SSE partials) in one launch.
int rv_rdo_candidates(const rv::RdoArgs &luma, const rv::RdoArgs &chroma, int hbd,
                      hipStream_t s, hipStream_t chroma_stream = nullptr);
