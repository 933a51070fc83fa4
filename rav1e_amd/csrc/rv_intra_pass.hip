// rv_intra_pass.hip -- the intra-mode screening and intra RDO of the replay
// (rdo_mode_decision, src/rdo.rs:1008-1152) for the 64x64 superblocks whose
// inter winner is not skip (speed 10, 4:2:0).
//
// rav1e codes the superblocks of a tile in raster order, so an intra
// candidate sees the final reconstruction of its left, top, top-right and
// top-left neighbours.  The replay evaluates every eligible superblock of
// the frame at once against the reconstruction the inter commit (F6) left
// (round 1), commits the intra winners, and re-evaluates only those whose
// neighbours' reconstruction changed (the superblocks to the right, below,
// below-left and below-right of a changed one, in the same tile) until no
// decision changes: a fixed point over the dependency DAG, equal to the
// sequential order's result (every round settles at least the earliest
// superblock, in coding order, that was still evaluated on stale edges).
//
// Kernels (one launch each per round):
//   intra_elig_kernel     the eligible superblocks (non-skip inter winner,
//                         fully inside the frame: rav1e splits edge
//                         superblocks, must_split) -> round 1's list
//   intra_screen_kernel   per listed superblock, one 256-thread workgroup:
//                         get_intra_edges of Y, U, V (opt_mode None) from the
//                         current reconstruction -> HBM; the 13
//                         RAV1E_INTRA_MODES predicted at TX_64X64 and their
//                         get_satd (8x8 Hadamard chunks, one lane each);
//                         stable sort; the modes to try
//   (rv_rdo_intra)        the intra chains: 3 luma modes x (chroma mode, DC)
//   intra_decide_kernel   compute_rd_cost of each (luma, chroma) pair in
//                         rav1e's order against the inter winner (strict <);
//                         result words; the commit / revert lists; the next
//                         round's list
#include "rv_intra.h"
#include "rv_intra_pass.h"

namespace rv {

__device__ __forceinline__ void sb_tile_geo(const IntraGeo &g, int sb, int &fx, int &fy, int &tx,
                                            int &ty, int &tw, int &th) {
  const int sx = sb % g.tw, sy = sb / g.tw;
  fx = g.tx0 + sx;
  fy = g.ty0 + sy;
  const int t0x = fx - fx % g.tws, t0y = fy - fy % g.ths;
  tx = t0x * 64;
  ty = t0y * 64;
  tw = g.W - tx < g.tws * 64 ? g.W - tx : g.tws * 64;
  th = g.H - ty < g.ths * 64 ? g.H - ty : g.ths * 64;
}

// Wave-aggregated append of flag v of this lane to list / *count.
__device__ __forceinline__ void wave_append(bool v, int item, int32_t *list, int32_t *count) {
  const uint64_t m = __ballot(v);
  const int lane = threadIdx.x & 63;
  int base = 0;
  if (lane == 0 && m) base = atomicAdd(count, (int)__popcll(m));
  base = __shfl(base, 0, 64);
  if (v) list[base + __popcll(m & ((1ull << lane) - 1))] = item;
}

// Round 1: every superblock whose inter winner is not skip and that lies
// inside the frame; resets the per-frame intra state.
__global__ __launch_bounds__(256) void intra_elig_kernel(IntraGeo g, const RdoWinner *win,
                                                         uint8_t *elig, uint8_t *iwas,
                                                         int32_t *mark, int32_t *list,
                                                         int32_t *count) {
  const int sb = blockIdx.x * 256 + threadIdx.x;
  bool v = false;
  if (sb < g.nsb) {
    const int sx = sb % g.tw, sy = sb / g.tw;
    const int px = (g.tx0 + sx) * 64, py = (g.ty0 + sy) * 64;
    v = win[sb].skip == 0 && px + 64 <= g.W && py + 64 <= g.H;
    elig[sb] = v;
    iwas[sb] = 0;
    mark[sb] = 0;
  }
  wave_append(v, sb, list, count);
}

// Screening of the listed superblocks (workgroup b = list entry b).
template <typename Px>
__global__ __launch_bounds__(256) void intra_screen_kernel(IntraScreenArgs a) {
  __shared__ int32_t e[3][kIntraEdge + 3];
  __shared__ uint32_t satd[16];
  const int b = blockIdx.x;
  if (b >= __builtin_amdgcn_readfirstlane(*a.count)) return;
  const int sb = a.list[b];
  int fx, fy, tx, ty, tw, th;
  sb_tile_geo(a.g, sb, fx, fy, tx, ty, tw, th);
  const int x = fx * 64 - tx, y = fy * 64 - ty;  // tile-relative
  const int have_top = y > 0;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int bd = a.g.bd;
  // get_intra_edges of Y (n 64), U, V (n 32 in 4:2:0; the chroma tile region
  // is the luma one decimated, src/tiling/plane_region.rs:30-37)
  if (wave < 3) {
    const rv_plane &p = a.rec[wave];
    const int dec = wave ? 1 : 0;
    intra_edges_sb<Px, 64>(p, tx >> dec, ty >> dec, tw >> dec, x >> dec, y >> dec, 64 >> dec,
                           have_top, bd, e[wave], lane);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 3 * kIntraEdge; i += 256) {
    const int pl = i / kIntraEdge, k = i - pl * kIntraEdge;
    ((Px *)a.edges)[((size_t)sb * 3 + pl) * kIntraEdge + k] = (Px)e[pl][k];
  }
  // the 13 RAV1E_INTRA_MODES (src/predict.rs:32-46) at TX_64X64: get_satd
  // = (sum of the 8x8 chunks' Hadamard sums + 4) >> 3 (src/dist.rs:197-328)
  const int var = x == 0 && y == 0 ? 0 : y == 0 ? 1 : x == 0 ? 2 : 3;
  const int maxv = (1 << bd) - 1;
  const Px *o = plane_ptr<Px>(a.org, fx * 64, fy * 64);
  const int64_t os = a.org.stride;
  const int cy = (lane >> 3) * 8, cx = (lane & 7) * 8;  // this lane's 8x8 chunk
  for (int k = wave; k < kIntraModes; k += 4) {
    IntraSetup st = intra_setup(kIntraModeOrder[k], var);
    if (st.mode == 0) st.dcv = intra_dc<64>(e[0], var, 64, 64, bd, lane);
    int32_t d[64];
#pragma unroll
    for (int r = 0; r < 8; r++)
#pragma unroll
      for (int c = 0; c < 8; c++)
        d[r * 8 + c] = (int32_t)o[(int64_t)(cy + r) * os + cx + c] -
                       intra_px(st, e[0], 64, 64, cy + r, cx + c, maxv);
    const uint64_t s = group_sum<64>(satd_chunk<8>(d));
    if (lane == 0) satd[k] = (uint32_t)((s + 4) >> 3);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    // satds.sort_by_key (stable); modes = [DC_PRED (the most probable under
    // the unadapted default_if_y_mode_cdf)] + the 3 lowest not yet in; take 3
    int order[kIntraModes];
    for (int k = 0; k < kIntraModes; k++) order[k] = k;
    for (int i = 1; i < kIntraModes; i++)
      for (int j = i; j > 0 && satd[order[j]] < satd[order[j - 1]]; j--) {
        const int t = order[j];
        order[j] = order[j - 1];
        order[j - 1] = t;
      }
    uint8_t m[4];
    int n = 0;
    m[n++] = 0;
    for (int i = 0; i < 3; i++) {
      const int md = kIntraModeOrder[order[i]];
      bool seen = false;
      for (int j = 0; j < n; j++) seen |= m[j] == md;
      if (!seen) m[n++] = (uint8_t)md;
    }
    n = n > 3 ? 3 : n;
    uint8_t *w = a.modes + (size_t)sb * 4;
    w[0] = (uint8_t)n;
    for (int i = 0; i < 3; i++) w[1 + i] = i < n ? m[i] : 0;
  }
}

// The decision of every listed superblock (one thread each): rav1e's order
// of (luma mode, chroma mode) pairs, compute_rd_cost = ScaledDistortion +
// lambda * rate / 8 (src/rdo.rs:563-569, the replay's estimate_rate model),
// strict < against the running best, which starts at the inter winner's
// cost.  Writes the result words, the commit list (intra winners) and the
// revert list (intra before, inter now), and appends the superblocks that
// depend on a changed reconstruction to the next round's list.
__global__ __launch_bounds__(256) void intra_decide_kernel(IntraDecideArgs a) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int n = *a.count;
  const bool live = i < n;
  const int sb = live ? a.list[i] : 0;
  bool commit = false, revert = false, changed = false;
  if (live) {
    const RdoWinner w = a.win[sb];
    const uint8_t *md = a.modes + (size_t)sb * 4;
    double best = w.cost;
    int bl = -1, bc = 0;
    uint64_t bd = 0;
    for (int k = 0; k < md[0]; k++) {
      const int m = md[1 + k];
      const uint64_t *lo = a.lout + ((size_t)sb * 3 + k) * 3;
      for (int j = 0; j < (m ? 2 : 1); j++) {
        const uint64_t *uo = a.uout + ((size_t)sb * 6 + 2 * k + j) * 3;
        const uint64_t *vo = a.vout + ((size_t)sb * 6 + 2 * k + j) * 3;
        const uint32_t rate = (uint32_t)lo[2] + (uint32_t)uo[2] + (uint32_t)vo[2];
        const uint64_t d = (uint64_t)((double)lo[1] * 1.0) + (uint64_t)((double)uo[1] * a.ds_u) +
                           (uint64_t)((double)vo[1] * a.ds_v);
        const double rd = (double)d + a.lambda * ((double)rate / 8.0);
        if (rd < best) {
          best = rd;
          bl = m;
          bc = j ? 0 : m;
          bd = d;
        }
      }
    }
    const bool was = a.iwas[sb] != 0;
    uint64_t *wd = a.words + (size_t)sb * a.words_per_sb + a.win_off;
    if (bl >= 0) {
      a.iwin[sb * 2 + 0] = (uint8_t)bl;
      a.iwin[sb * 2 + 1] = (uint8_t)bc;
      a.iwas[sb] = 1;
      uint64_t cb;
      __builtin_memcpy(&cb, &best, 8);
      wd[0] = (uint64_t)(kIntraWord + 16 * bl + bc);
      wd[1] = 0;
      wd[2] = cb;
      wd[3] = bd;
      commit = true;
    } else {
      if (was) {  // back to the inter winner
        uint64_t cb;
        __builtin_memcpy(&cb, &w.cost, 8);
        wd[0] = (uint64_t)w.c;
        wd[1] = (uint64_t)w.skip;
        wd[2] = cb;
        wd[3] = w.dist;
        revert = true;
      }
      a.iwas[sb] = 0;
      a.iwin[sb * 2 + 0] = a.iwin[sb * 2 + 1] = 0;
    }
    changed = commit || was;
  }
  wave_append(commit, sb, a.commit_list, a.commit_count);
  wave_append(revert, sb, a.revert_list, a.revert_count);
  // the superblocks reading this one's pixels as edges: right, below-left,
  // below, below-right, in the same tile; eligible ones join the next round
  int fx = 0, fy = 0, tx = 0, ty = 0, tw = 0, th = 0;
  if (live) sb_tile_geo(a.g, sb, fx, fy, tx, ty, tw, th);
  const int tx1 = (tx + tw + 63) / 64, ty1 = (ty + th + 63) / 64;  // tile end (superblocks)
  const int dxs[4] = {1, -1, 0, 1}, dys[4] = {0, 1, 1, 1};
  for (int k = 0; k < 4; k++) {
    const int nx = fx + dxs[k], ny = fy + dys[k];
    bool add = false;
    int nsb = 0;
    if (changed && nx >= tx / 64 && nx < tx1 && ny < ty1) {
      nsb = (ny - a.g.ty0) * a.g.tw + (nx - a.g.tx0);
      add = a.elig[nsb] && atomicMax(&a.mark[nsb], a.round + 1) < a.round + 1;
    }
    wave_append(add, nsb, a.next_list, a.next_count);
  }
}

// Intra candidates of the frame: [screened (round 1), intra winners].
__global__ __launch_bounds__(256) void intra_stats_kernel(int nsb, const uint8_t *elig,
                                                          const uint8_t *iwas, uint32_t *out) {
  uint32_t s = 0, w = 0;
  for (int i = threadIdx.x; i < nsb; i += 256) {
    s += elig[i];
    w += iwas[i];
  }
  s = group_sum<64>(s);
  w = group_sum<64>(w);
  __shared__ uint32_t red[2][4];
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s;
    red[1][threadIdx.x >> 6] = w;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    out[0] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    out[1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}

}  // namespace rv

using namespace rv;

int rv_intra_elig(const IntraGeo &g, const RdoWinner *win, uint8_t *elig, uint8_t *iwas,
                  int32_t *mark, int32_t *list, int32_t *count, hipStream_t s) {
  intra_elig_kernel<<<(g.nsb + 255) / 256, 256, 0, s>>>(g, win, elig, iwas, mark, list, count);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

int rv_intra_screen(const IntraScreenArgs &a, int n, int hbd, hipStream_t s) {
  // one workgroup per listed superblock (n = the list's count, read by the
  // host; the kernel re-reads it from the device)
  const unsigned grid = (unsigned)(n < a.g.nsb ? n : a.g.nsb);
  if (grid == 0) return RV_OK;
  if (hbd)
    intra_screen_kernel<uint16_t><<<grid, 256, 0, s>>>(a);
  else
    intra_screen_kernel<uint8_t><<<grid, 256, 0, s>>>(a);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

int rv_intra_decide(const IntraDecideArgs &a, hipStream_t s) {
  intra_decide_kernel<<<(a.g.nsb + 255) / 256, 256, 0, s>>>(a);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

int rv_intra_stats(int nsb, const uint8_t *elig, const uint8_t *iwas, uint32_t *out, hipStream_t s) {
  intra_stats_kernel<<<1, 256, 0, s>>>(nsb, elig, iwas, out);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}
