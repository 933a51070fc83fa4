// rv_ec.hip -- coefficient entropy coding: a device tokenizer for
// ContextWriter::write_coeffs_lv_map (src/context.rs:3965-4220) and the host
// range coder of WriterBase<WriterEncoder> (src/ec.rs:100-600).
//
// The work splits where the reference's data dependencies split:
//  * Everything write_coeffs_lv_map derives from a transform block's own
//    coefficients and its neighbours' final coefficient contexts -- the
//    scan, eob, eob_pt / eob_extra, the nz-map and base-range contexts, the
//    txb_skip / dc_sign contexts, the symbol values -- is data-parallel
//    across transform blocks once the blocks are committed.  The block
//    context a block reads (BlockContext::get_txb_ctx, :1776-1868) is the
//    value set_coeff_context (:1594-1609) stored for the block directly
//    above / left of it in the same tile (z-order coding never revisits a
//    column above or a row to the left; a skip leaf stores 0 through
//    reset_skip_context, :1651-1679; a tile starts from zero, the left
//    context restarts every superblock row, :1681-1688).  So one launch
//    stores every block's context value into a per-plane 4x4 map, a second
//    reads its neighbours' values and emits the block's symbols.
//  * What stays sequential is the range coder and the CDF adaptation
//    (update_cdf, src/ec.rs:891-905): the host runs them over the symbol
//    stream of each tile ("tokens": CDF offset + length + symbol, or a raw
//    bit), tiles independently.
//
// Device layout: jobs in coding order (rv_ec_job), token offsets from an
// exclusive scan of the per-job token counts, tokens u32:
//   symbol  bits 0-12 CDF offset (u16 units, rv_ec_tables.h layout),
//           bits 13-17 CDF length (nsymbs + 1), bits 18-22 symbol
//   raw bit bit 31 set, bit 0 the bit (Writer::bit, bool at 16384)
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "rv_device.h"
#include "rv_ec.h"
#include "rv_ec_tables.h"
#include "rv_quant_tables.h"

namespace rv {

constexpr int kEcPadHor = 4;  // TX_PAD_HOR (src/context.rs:253)
constexpr int kEcLds = 36 * 36 + 16;  // levels of a coded 32x32 block + its pad

__host__ __device__ inline uint32_t ec_sym(int off, int len, int s) {
  return (uint32_t)off | ((uint32_t)len << 13) | ((uint32_t)s << 18);
}
__host__ __device__ inline uint32_t ec_raw(int b) { return 0x80000000u | (uint32_t)(b & 1); }

__device__ inline int coded_w(int tx) { return tx == 4 ? 32 : 4 << tx; }
__device__ inline int golomb_bits(uint32_t level) {  // write_golomb(level - 15): 2 len - 1 bits
  const uint32_t x = level - 14;
  const int len = 32 - __clz(x);
  return 2 * len - 1;
}
__device__ inline int br_count(uint32_t level) {  // coeff_br symbols (src/context.rs:4145-4170)
  if (level <= 2) return 0;
  const int n = (int)(level - 3) / 3 + 1;
  return n < 4 ? n : 4;
}
__device__ inline int eob_pos_token(int eob, int *extra) {  // src/context.rs:3778-3789
  int t;
  if (eob < 33) {
    t = RV_eob_to_pos_small[eob];
  } else {
    int e = (eob - 1) >> 5;
    t = RV_eob_to_pos_large[e < 16 ? e : 16];
  }
  *extra = eob - RV_k_eob_group_start[t];
  return t;
}
__device__ inline int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ inline int wave_or(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o, 64);
  return v;
}
__device__ inline int wave_max(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ inline int wave_incl_scan(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

struct EcArgs {
  const rv_ec_job *jobs;
  int n, xdec, ydec, map_w4, map_h4;
  const uint32_t *dn;  // non-null: the job count is *dn (<= n, device-generated jobs)
  uint8_t *map;
  uint32_t *count;  // [n] token counts, then exclusive offsets [n + 1]
  int32_t *eob;     // [n]
  uint32_t *tokens;
  uint32_t cap;
  uint32_t *status;  // [0] total tokens, [1] overflow flag
};

__device__ inline uint8_t *ec_map(const EcArgs &a, int tile, int p) {
  return a.map + ((size_t)tile * 3 + p) * a.map_h4 * a.map_w4;
}

// Pass 1, one wavefront per job: eob, the stored context value (cul_level
// with the dc sign, src/context.rs:4209-4217; 0 for eob == 0 and for a skip
// leaf's planes) into the map, and the job's token count.
__device__ void ec_prep_job(const EcArgs &a, int j, int lane);
__global__ __launch_bounds__(256) void ec_prep_kernel(EcArgs a) {
  const int lane = threadIdx.x & 63;
  const int n = a.dn ? (int)*a.dn : a.n;
  for (int j = blockIdx.x * 4 + (threadIdx.x >> 6); j < n; j += gridDim.x * 4) ec_prep_job(a, j, lane);
}
__device__ void ec_prep_job(const EcArgs &a, int j, int lane) {
  const rv_ec_job jb = a.jobs[j];
  if (jb.kind == 1) {
    for (int p = 0; p < 3; p++) {
      const int xd = p ? a.xdec : 0, yd = p ? a.ydec : 0;
      const int w4 = max(1, (1 << (jb.bw_lg - 2)) >> xd), h4 = max(1, (1 << (jb.bh_lg - 2)) >> yd);
      uint8_t *m = ec_map(a, jb.tile, p);
      const int x0 = jb.bx >> xd, y0 = jb.by >> yd;
      for (int i = lane; i < w4 * h4; i += 64)
        m[(size_t)(y0 + i / w4) * a.map_w4 + x0 + i % w4] = 0;
    }
  }
  if (jb.kind != 0) {
    if (lane == 0) {
      a.count[j] = 0;
      a.eob[j] = 0;
    }
    return;
  }
  const int tx = jb.tx_size, cw = coded_w(tx), area = cw * cw;
  const uint16_t *scan = RV_SCANS + RV_SCAN_OFF[tx * 16 + jb.tx_type];
  const int32_t *co = jb.coeffs;
  uint32_t sum = 0;
  int last = 0;
  for (int i = lane; i < area; i += 64) {
    const int32_t v = co[scan[i]];
    sum += (uint32_t)(v < 0 ? -v : v);
    if (v != 0) last = i + 1;
  }
  sum = (uint32_t)wave_sum((int)sum);
  const int eob = sum ? wave_max(last) : 0;
  int cnt = 0;
  for (int i = lane; i < eob; i += 64) {
    const int32_t v = co[scan[i]];
    const uint32_t level = (uint32_t)(v < 0 ? -v : v);
    cnt += 1 + br_count(level) + (level > 0) + (level > 14 ? golomb_bits(level) : 0);
  }
  cnt = wave_sum(cnt);
  int hdr = 1;
  uint8_t val = 0;
  if (eob) {
    int extra;
    const int pt = eob_pos_token(eob, &extra);
    hdr += (jb.plane == 0 && tx < 4 && jb.is_inter) + 1 + RV_k_eob_offset_bits[pt];
    uint32_t cul = sum < 63 ? sum : 63;
    const int32_t dc = co[0];
    if (dc < 0)
      cul |= 1u << 6;
    else if (dc > 0)
      cul += 2u << 6;
    val = (uint8_t)cul;
  }
  const int xd = jb.plane ? a.xdec : 0, yd = jb.plane ? a.ydec : 0;
  const int n4 = 1 << tx;
  uint8_t *m = ec_map(a, jb.tile, jb.plane);
  const int x0 = jb.bx >> xd, y0 = jb.by >> yd;
  for (int i = lane; i < n4 * n4; i += 64) m[(size_t)(y0 + i / n4) * a.map_w4 + x0 + i % n4] = val;
  if (lane == 0) {
    a.count[j] = (uint32_t)(hdr + cnt);
    a.eob[j] = eob;
  }
}

// Exclusive scan of the counts in place (n <= 1024 * 1024; dn non-null:
// the count is *dn <= n): per-1024 block scans, a scan of the block sums,
// the block offsets added.  v[count] = the total, status[0] too.
__device__ inline int scan_n(int n, const uint32_t *dn) { return dn ? (int)*dn : n; }
__global__ __launch_bounds__(1024) void ec_scan_blocks(uint32_t *v, int n, const uint32_t *dn,
                                                       uint32_t *bsum) {
  __shared__ uint32_t s[1024];
  n = scan_n(n, dn);
  const int i = blockIdx.x * 1024 + threadIdx.x;
  const uint32_t x = i < n ? v[i] : 0;
  s[threadIdx.x] = x;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const uint32_t t = threadIdx.x >= o ? s[threadIdx.x - o] : 0;
    __syncthreads();
    s[threadIdx.x] += t;
    __syncthreads();
  }
  if (i < n) v[i] = s[threadIdx.x] - x;
  if (threadIdx.x == 1023) bsum[blockIdx.x] = s[1023];
}
__global__ __launch_bounds__(1024) void ec_scan_top(uint32_t *bsum, int n, const uint32_t *dn,
                                                    uint32_t *v, uint32_t *status) {
  __shared__ uint32_t s[1024];
  n = scan_n(n, dn);
  const int nb = (n + 1023) / 1024;
  const uint32_t x = (int)threadIdx.x < nb ? bsum[threadIdx.x] : 0;
  s[threadIdx.x] = x;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const uint32_t t = threadIdx.x >= o ? s[threadIdx.x - o] : 0;
    __syncthreads();
    s[threadIdx.x] += t;
    __syncthreads();
  }
  if ((int)threadIdx.x < nb) bsum[threadIdx.x] = s[threadIdx.x] - x;
  if (threadIdx.x == 0) {
    v[n] = s[1023];
    if (status) {
      status[0] = s[1023];
      status[1] = 0;
    }
  }
}
__global__ __launch_bounds__(1024) void ec_scan_add(uint32_t *v, int n, const uint32_t *dn,
                                                    const uint32_t *bsum) {
  n = scan_n(n, dn);
  const int i = blockIdx.x * 1024 + threadIdx.x;
  if (i < n) v[i] += bsum[blockIdx.x];
}

void ec_scan(uint32_t *v, int n, const uint32_t *dn, uint32_t *bsum, uint32_t *status,
             hipStream_t st) {
  const int nb = (n + 1023) / 1024;
  ec_scan_blocks<<<nb, 1024, 0, st>>>(v, n, dn, bsum);
  ec_scan_top<<<1, 1024, 0, st>>>(bsum, n, dn, v, status);
  if (nb > 1) ec_scan_add<<<nb, 1024, 0, st>>>(v, n, dn, bsum);
}

struct TokW {
  uint32_t *t;
  uint32_t cap;
  uint32_t *status;
  __device__ void put(uint32_t idx, uint32_t v) const {
    if (idx < cap)
      t[idx] = v;
    else
      status[1] = 1;
  }
};

// get_nz_map_ctx, TX_CLASS_2D (src/context.rs:3791-3878), over the LDS levels
__device__ inline int nz_ctx(const uint8_t *lv, int pos, int bwl, int height, int c, int eob,
                             int tx) {
  if (c == eob - 1) {
    if (c == 0) return 0;
    if (c <= (height << bwl) / 8) return 1;
    if (c <= (height << bwl) / 4) return 2;
    return 3;
  }
  if (pos == 0) return 0;
  const uint8_t *l = lv + pos + ((pos >> bwl) << 2);
  const int st = (1 << bwl) + kEcPadHor;
  int mag = min((int)l[1], 3) + min((int)l[st], 3) + min((int)l[st + 1], 3) + min((int)l[2], 3) +
            min((int)l[2 * st], 3);
  const int row = pos >> bwl, col = pos - (row << bwl);
  const int ctx = min((mag + 1) >> 1, 4);
  return ctx + RV_av1_nz_map_ctx_offset[tx * 25 + min(row, 4) * 5 + min(col, 4)];
}
// get_br_ctx, TX_CLASS_2D (src/context.rs:3901-3948)
__device__ inline int br_ctx(const uint8_t *lv, int c, int bwl) {
  const int row = c >> bwl, col = c - (row << bwl);
  const int st = (1 << bwl) + kEcPadHor;
  const int pos = row * st + col;
  int mag = lv[pos + 1] + lv[pos + st] + lv[pos + st + 1];
  mag = min((mag + 1) >> 1, 6);
  if (c == 0) return mag;
  if (row < 2 && col < 2) return mag + 7;
  return mag + 14;
}

// Pass 2, one wavefront per transform-block job: its symbols, in
// write_coeffs_lv_map's order, from its token offset.
__device__ void ec_token_job(const EcArgs &a, int j, int lane, uint8_t *lv);
__global__ __launch_bounds__(256) void ec_token_kernel(EcArgs a) {
  __shared__ uint8_t lds[4][kEcLds];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int n = a.dn ? (int)*a.dn : a.n;
  for (int j = blockIdx.x * 4 + wv; j < n; j += gridDim.x * 4) {
    ec_token_job(a, j, lane, lds[wv]);
    wave_sync();
  }
}
__device__ void ec_token_job(const EcArgs &a, int j, int lane, uint8_t *lv) {
  const rv_ec_job jb = a.jobs[j];
  if (jb.kind != 0) return;
  const TokW w{a.tokens, a.cap, a.status};
  const int tx = jb.tx_size, cw = coded_w(tx), area = cw * cw, bwl = tx == 4 ? 5 : tx + 2;
  const int eob = a.eob[j];
  uint32_t o = a.count[j];
  const int p = jb.plane, ptype = p ? 1 : 0;
  const int xd = p ? a.xdec : 0, yd = p ? a.ydec : 0;
  // get_txb_ctx from the neighbours' stored values (zero outside the tile)
  const int n4 = 1 << tx, x0 = jb.bx >> xd, y0 = jb.by >> yd;
  const uint8_t *m = ec_map(a, jb.tile, p);
  const int ab = (lane < n4 && y0 > 0) ? m[(size_t)(y0 - 1) * a.map_w4 + x0 + lane] : 0;
  const int lf = (lane < n4 && x0 > 0) ? m[(size_t)(y0 + lane) * a.map_w4 + x0 - 1] : 0;
  const int sgn = (lane < n4 ? ((ab >> 6) == 1 ? -1 : (ab >> 6) == 2 ? 1 : 0) +
                                   ((lf >> 6) == 1 ? -1 : (lf >> 6) == 2 ? 1 : 0)
                             : 0);
  const int dc_sign = wave_sum(sgn);
  const int top = wave_or(ab), left = wave_or(lf);
  const int dc_ctx = dc_sign < 0 ? 1 : dc_sign > 0 ? 2 : 0;
  const int tx_lg = 2 * (tx + 2), plane_lg = jb.bw_lg + jb.bh_lg;
  int skip_ctx;
  if (p == 0) {
    if (plane_lg == tx_lg) {
      skip_ctx = 0;
    } else {
      const int t = top & 63, l = left & 63;
      const int mx = min(t | l, 4), mn = min(min(t, l), 4);
      // skip_contexts[min][max] (src/context.rs:1832-1838)
      skip_ctx = mx == 0 ? 1 : mn == 0 ? 2 + (mx > 3) : mx <= 3 ? 4 : mn <= 3 ? 5 : 6;
    }
  } else {
    skip_ctx = (top != 0) + (left != 0) + (plane_lg > tx_lg ? 10 : 7);
  }
  const int txs = tx;
  if (lane == 0) w.put(o, ec_sym(RV_EC_TXB_SKIP + (txs * 13 + skip_ctx) * 3, 3, eob == 0));
  o++;
  if (eob == 0) return;
  // txb_init_levels into LDS (pad columns / rows zero)
  const int st = cw + kEcPadHor;
  for (int i = lane; i < st * (cw + 4); i += 64) lv[i] = 0;
  wave_sync();
  const int32_t *co = jb.coeffs;
  for (int i = lane; i < area; i += 64) {
    const int32_t v = co[i];
    const int32_t av = v < 0 ? -v : v;
    lv[(i >> bwl) * st + (i & (cw - 1))] = (uint8_t)min(av, 127);
  }
  wave_sync();
  if (p == 0 && tx < 4 && jb.is_inter) {
    // write_tx_type: TX_SET_DCT_IDTX (set 1) -> inter_tx_cdf[3][sqr][..=2]
    if (lane == 0)
      w.put(o, ec_sym(RV_EC_INTER_TX + (RV_tx_set_index_inter[1] * 4 + tx) * 17,
                      RV_num_tx_set[1] + 1, RV_av1_tx_ind[16 + jb.tx_type]));
    o++;
  }
  int extra;
  const int pt = eob_pos_token(eob, &extra);
  const int em = min(2 * (tx + 2) - 4, 6), elen = 6 + em;
  int eoff;
  switch (em) {
    case 0: eoff = RV_EC_EOB16; break;
    case 1: eoff = RV_EC_EOB32; break;
    case 2: eoff = RV_EC_EOB64; break;
    case 3: eoff = RV_EC_EOB128; break;
    case 4: eoff = RV_EC_EOB256; break;
    case 5: eoff = RV_EC_EOB512; break;
    default: eoff = RV_EC_EOB1024; break;
  }
  if (lane == 0) w.put(o, ec_sym(eoff + ptype * 2 * elen, elen, pt - 1));
  o++;
  const int ebits = RV_k_eob_offset_bits[pt];
  if (ebits > 0) {
    if (lane == 0)
      w.put(o, ec_sym(RV_EC_EOB_EXTRA + ((txs * 2 + ptype) * 9 + (pt - 3)) * 3, 3,
                      (extra >> (ebits - 1)) & 1));
    if (lane >= 1 && lane < ebits) w.put(o + lane, ec_raw(extra >> (ebits - 1 - lane)));
    o += ebits;
  }
  // the coefficients: lane chunks of the scan, K positions each
  const uint16_t *scan = RV_SCANS + RV_SCAN_OFF[tx * 16 + jb.tx_type];
  const int K = (eob + 63) >> 6;
  const int c0 = min(lane * K, eob), c1 = min(c0 + K, eob);
  int sa = 0, sb = 0;
  for (int c = c0; c < c1; c++) {
    const int32_t v = co[scan[c]];
    const uint32_t level = (uint32_t)(v < 0 ? -v : v);
    sa += 1 + br_count(level);
    sb += (level > 0) + (level > 14 ? golomb_bits(level) : 0);
  }
  const int pa = wave_incl_scan(sa, lane), pb = wave_incl_scan(sb, lane);
  const int ta = __shfl(pa, 63, 64);
  // base / base-range symbols, reverse scan order (src/context.rs:4120-4172)
  uint32_t oa = o + (uint32_t)(ta - pa);
  const int btx = min(txs, 3);
  for (int c = c1 - 1; c >= c0; c--) {
    const int pos = scan[c];
    const int32_t v = co[pos];
    const uint32_t level = (uint32_t)(v < 0 ? -v : v);
    const int ctx = nz_ctx(lv, pos, bwl, cw, c, eob, tx);
    if (c == eob - 1)
      w.put(oa++, ec_sym(RV_EC_BASE_EOB + ((txs * 2 + ptype) * 4 + ctx) * 4, 4,
                         (int)min(level, 3u) - 1));
    else
      w.put(oa++, ec_sym(RV_EC_BASE + ((txs * 2 + ptype) * 42 + ctx) * 5, 5, (int)min(level, 3u)));
    if (level > 2) {
      const int bctx = br_ctx(lv, pos, bwl);
      const int off = RV_EC_BR + ((btx * 2 + ptype) * 21 + bctx) * 5;
      const int br = (int)level - 3;
      for (int idx = 0; idx < 12; idx += 3) {
        const int k = min(br - idx, 3);
        w.put(oa++, ec_sym(off, 5, k));
        if (k < 3) break;
      }
    }
  }
  // signs (dc through dc_sign_cdf) and golomb remainders, scan order
  uint32_t ob = o + (uint32_t)ta + (uint32_t)(pb - sb);
  for (int c = c0; c < c1; c++) {
    const int32_t v = co[scan[c]];
    const uint32_t level = (uint32_t)(v < 0 ? -v : v);
    if (level == 0) continue;
    if (c == 0)
      w.put(ob++, ec_sym(RV_EC_DC_SIGN + (ptype * 3 + dc_ctx) * 3, 3, v < 0));
    else
      w.put(ob++, ec_raw(v < 0));
    if (level > 14) {
      const uint32_t x = level - 14;
      const int len = 32 - __clz(x);
      for (int k = 0; k < len - 1; k++) w.put(ob++, ec_raw(0));
      for (int k = len - 1; k >= 0; k--) w.put(ob++, ec_raw((int)(x >> k)));
    }
  }
}


// ---- the replay's job list -------------------------------------------------
// One thread per superblock of the group in coding order (tiles in raster
// order, superblocks in raster order inside a tile; encode_tile_group /
// encode_tile, src/encoder.rs:2766-2781, 3160-3340): its jobs are [tile
// start] [superblock-row start] then its leaves in z-order
// (encode_partition_topdown, :2392-2470): the Morton walk of the
// superblock's 256 luma 4x4 positions meets each leaf's top-left first.
// pass 0 counts, pass 1 writes at the scanned offsets.
__device__ inline void ec_sb_of(const EcFrameArgs &a, int i, int &sx, int &sy, int &t, int &first,
                                int &rowstart, int &t0x, int &t0y) {
  const int ntx = (a.tw + a.tws - 1) / a.tws;
  int base = 0;
  for (t = 0;; t++) {
    const int tx = t % ntx, ty = t / ntx;
    const int w = min(a.tws, a.tw - tx * a.tws), h = min(a.ths, a.th - ty * a.ths);
    if (i < base + w * h) {
      const int k = i - base;
      t0x = a.tx0 + tx * a.tws;
      t0y = a.ty0 + ty * a.ths;
      sx = t0x + k % w;
      sy = t0y + k / w;
      first = k == 0;
      rowstart = k % w == 0;
      return;
    }
    base += w * h;
  }
}

// The jobs of superblock i (coding order): count (out == nullptr) or write
// them from out[0].  Leaves in z-order: a walk over the superblock's 8x8
// cells in z-order (the depth-first order of the partition tree) that reads
// the block map's leaf size at a cell and, at a leaf's top-left cell, emits
// the leaf and steps over its cells (a 64x64 leaf costs one read).  No
// stack: the explicit depth-first stack it replaces was indexed at run time
// and lived in scratch memory (208 B per lane).
__device__ int ec_sb_jobs(const EcFrameArgs &a, int i, rv_ec_job *out, int cap) {
  int sx, sy, t, first, rowstart, t0x, t0y;
  ec_sb_of(a, i, sx, sy, t, first, rowstart, t0x, t0y);
  int n = 0;
  auto put = [&](const rv_ec_job &jb) {
    if (out && n < cap) out[n] = jb;
    n++;
  };
  rv_ec_job z{};
  z.tile = t;
  if (first) {
    rv_ec_job j3 = z;
    j3.kind = 3;
    put(j3);
  }
  if (rowstart) {
    rv_ec_job j2 = z;
    j2.kind = 2;
    put(j2);
  }
  const int sb = (sy - a.ty0) * a.tw + (sx - a.tx0);
  for (int zc = 0; zc < 64;) {
    // cell zc of the superblock in z-order: de-interleave its bits
    const int cx = (zc & 1) | ((zc >> 1) & 2) | ((zc >> 2) & 4);
    const int cy = ((zc >> 1) & 1) | ((zc >> 2) & 2) | ((zc >> 3) & 4);
    const int x4 = sx * 16 + 2 * cx, y4 = sy * 16 + 2 * cy;
    if (x4 >= a.mi_cols || y4 >= a.mi_rows) {  // outside the frame: no block starts here
      zc++;
      continue;
    }
    const int code = a.mi_lg[(size_t)y4 * a.mi_stride + x4];  // log2 of the leaf's 4x4 units
    const int n4 = 1 << code, lg = code + 2;
    if (((x4 | y4) & (n4 - 1)) != 0) {  // not the leaf's first cell (never for a consistent map)
      zc++;
      continue;
    }
    zc += (n4 >> 1) * (n4 >> 1);  // the leaf's cells
    rv_ec_job jb = z;
    jb.bx = x4 - t0x * 16;
    jb.by = y4 - t0y * 16;
    if (a.mi_skip[(size_t)y4 * a.mi_stride + x4]) {
      jb.kind = 1;
      jb.bw_lg = jb.bh_lg = lg;
      put(jb);
      continue;
    }
    const int l = 6 - lg;
    const EcGenLevel &L = a.lv[l];
    int bi, inter = 1;
    if (l == 0) {
      bi = sb;
      inter = a.words[(size_t)sb * a.words_per_sb + a.win_off] < 1000;
    } else {
      bi = (y4 / n4 - L.y0) * L.gw + (x4 / n4 - L.x0);
    }
    jb.kind = 0;
    jb.is_inter = inter;
    jb.plane = 0;
    jb.tx_size = min(lg - 2, 4);
    jb.bw_lg = jb.bh_lg = lg;
    jb.coeffs = L.l_lev + (size_t)bi * (l == 0 ? 1024 : L.B * L.B);
    put(jb);
    const int plg = lg - a.xdec;
    const int ntc = plg == 6 ? 4 : 1;
    const int ctx_ = plg == 6 ? 3 : plg - 2;
    const int carea = plg == 6 ? 1024 : L.bc * L.bc;
    for (int p = 1; p < 3; p++)
      for (int c = 0; c < ntc; c++) {
        rv_ec_job jc = jb;
        jc.plane = p;
        jc.tx_size = ctx_;
        jc.bw_lg = jc.bh_lg = plg;
        jc.bx = jb.bx + (ntc == 4 ? (c % 2) * 8 : 0);
        jc.by = jb.by + (ntc == 4 ? (c / 2) * 8 : 0);
        if (l == 0)
          jc.coeffs = L.c_lev + (size_t)(p - 1) * a.nsb * a.ntx_c * 1024 +
                      ((size_t)bi * a.ntx_c + c) * 1024;
        else
          jc.coeffs = L.c_lev + (size_t)(p - 1) * L.n * carea + (size_t)bi * carea;
        put(jc);
      }
  }
  return n;
}

// block-wide exclusive scan of one value per thread (1024 threads)
__device__ inline uint32_t block_scan_1024(uint32_t x, uint32_t *s, uint32_t &total) {
  s[threadIdx.x] = x;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const uint32_t t = threadIdx.x >= o ? s[threadIdx.x - o] : 0;
    __syncthreads();
    s[threadIdx.x] += t;
    __syncthreads();
  }
  total = s[1023];
  const uint32_t r = s[threadIdx.x] - x;
  __syncthreads();
  return r;
}

// Every superblock's job count (pass 0) / its jobs at the scanned offset
// (pass 1), one thread per superblock.
__global__ __launch_bounds__(64) void ec_gen_kernel(EcFrameArgs a, EcFrameBufs b, int pass) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= a.nsb) return;
  if (!pass) {
    b.sb_off[i] = (uint32_t)ec_sb_jobs(a, i, nullptr, 0);
    return;
  }
  const uint32_t o = b.sb_off[i];
  if (o < (uint32_t)b.max_jobs) ec_sb_jobs(a, i, b.jobs + o, b.max_jobs - (int)o);
}

// One workgroup: the exclusive scan of the superblocks' job counts;
// sb_off[nsb] = the job count (clamped to max_jobs, overflow flagged)
__global__ __launch_bounds__(1024) void ec_sb_scan_kernel(EcFrameArgs a, EcFrameBufs b) {
  __shared__ uint32_t s[1024];
  uint32_t carry = 0;
  for (int c0 = 0; c0 < a.nsb; c0 += 1024) {
    const int i = c0 + threadIdx.x;
    const uint32_t x = i < a.nsb ? b.sb_off[i] : 0;
    uint32_t total;
    const uint32_t o = carry + block_scan_1024(x, s, total);
    if (i < a.nsb) b.sb_off[i] = o;
    carry += total;
  }
  if (threadIdx.x == 0) {
    b.sb_off[a.nsb] = carry < (uint32_t)b.max_jobs ? carry : b.max_jobs;
    if (carry > (uint32_t)b.max_jobs) b.dstat[1] = 1;
  }
}

// One workgroup: the exclusive scan of the jobs' token counts, then the
// host-mapped stat: [total, overflow, jobs, first token of every tile, total]
__global__ __launch_bounds__(1024) void ec_scan_frame_kernel(EcFrameArgs a, EcFrameBufs b) {
  __shared__ uint32_t s[1024];
  const int n = (int)b.sb_off[a.nsb];
  uint32_t carry = 0;
  for (int c0 = 0; c0 < n; c0 += 1024) {
    const int i = c0 + threadIdx.x;
    const uint32_t x = i < n ? b.offsets[i] : 0;
    uint32_t total;
    const uint32_t o = carry + block_scan_1024(x, s, total);
    if (i < n) b.offsets[i] = o;
    carry += total;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    b.offsets[n] = carry;
    b.dstat[0] = carry;
    const bool over = b.dstat[1] || carry > b.cap;
    b.dstat[1] = over;
    b.stat[0] = carry;
    b.stat[1] = over;
    b.stat[2] = (uint32_t)n;
    b.stat[3 + b.ntiles] = carry;
  }
  if ((int)threadIdx.x < b.ntiles) {  // tile t's first superblock -> its first job's token
    const int t = threadIdx.x;
    const int ntx = (a.tw + a.tws - 1) / a.tws;
    int base = 0;
    for (int k = 0; k < t; k++) {
      const int tx = k % ntx, ty = k / ntx;
      base += min(a.tws, a.tw - tx * a.tws) * min(a.ths, a.th - ty * a.ths);
    }
    // sb_off holds unclamped prefix sums: past an overflow (dstat[1]) the
    // index is clamped to the job count (the host drops the frame anyway)
    const uint32_t j = b.sb_off[base];
    b.stat[3 + t] = b.offsets[j < (uint32_t)n ? j : (uint32_t)n];
  }
}

int ec_frame_tokens(const EcFrameArgs &a, const EcFrameBufs &b, hipStream_t st) {
  if (b.ntiles > 1024) return rv_set_error(RV_EINVAL, "ec_frame_tokens: more than 1024 tiles");
  EcArgs e;
  e.jobs = b.jobs;
  e.n = b.max_jobs;
  e.dn = b.sb_off + a.nsb;
  e.xdec = a.xdec;
  e.ydec = a.ydec;
  e.map_w4 = b.map_w4;
  e.map_h4 = b.map_h4;
  e.map = b.map;  // every visible 4x4 of a tile is stored by its leaf before it is read
  e.count = b.offsets;
  e.eob = (int32_t *)b.scratch;
  e.tokens = b.tokens;
  e.cap = b.cap;
  e.status = b.dstat;
  if (hipMemsetAsync(b.dstat, 0, 8, st) != hipSuccess)
    return rv_set_error(RV_EHIP, "ec_frame_tokens: status");
  ec_gen_kernel<<<(a.nsb + 63) / 64, 64, 0, st>>>(a, b, 0);
  ec_sb_scan_kernel<<<1, 1024, 0, st>>>(a, b);
  ec_gen_kernel<<<(a.nsb + 63) / 64, 64, 0, st>>>(a, b, 1);
  // grid-stride over the device-side job count
  ec_prep_kernel<<<1024, 256, 0, st>>>(e);
  ec_scan_frame_kernel<<<1, 1024, 0, st>>>(a, b);
  ec_token_kernel<<<1024, 256, 0, st>>>(e);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

}  // namespace rv

using namespace rv;

// ------------------------------------------------------------ host coder
namespace {

struct EcWriter {  // WriterBase<WriterEncoder> (src/ec.rs:100-600)
  uint32_t low = 0;
  uint16_t rng = 0x8000;
  int16_t cnt = -9;
  std::vector<uint16_t> pre;

  // lr_compute + store (src/ec.rs:270-295, 339-364)
  inline void store(uint32_t fl, uint32_t fh, uint32_t nms) {
    const uint32_t r = rng;
    uint32_t l, rr;
    if (fl < 32768) {
      const uint32_t u = (((r >> 8) * (fl >> 6)) >> 1) + 4 * nms;
      const uint32_t v = (((r >> 8) * (fh >> 6)) >> 1) + 4 * (nms - 1);
      l = r - u;
      rr = (u - v) & 0xFFFF;
    } else {
      l = 0;
      rr = (r - ((((r >> 8) * (fh >> 6)) >> 1) + 4 * (nms - 1))) & 0xFFFF;
    }
    uint32_t lo = l + low;
    int c = cnt;
    const int d = __builtin_clz(rr) - 16;  // 16 - ilog(u16)
    int s = c + d;
    if (s >= 0) {
      c += 16;
      uint32_t m = (1u << c) - 1;
      if (s >= 8) {
        pre.push_back((uint16_t)(lo >> c));
        lo &= m;
        c -= 8;
        m >>= 8;
      }
      pre.push_back((uint16_t)(lo >> c));
      s = c + d - 24;
      lo &= m;
    }
    low = lo << d;
    rng = (uint16_t)(rr << d);
    cnt = (int16_t)s;
  }
  // symbol_with_update: cdf of len entries (nsymbs + 1), update_cdf after
  inline void symbol_update(uint32_t s, uint16_t *cdf, int len) {
    const int n = len - 1;
    const uint32_t fl = s > 0 ? cdf[s - 1] : 32768u;
    store(fl, cdf[s], (uint32_t)(n - (int)s));
    const int nsymbs = n;
    const int rate = 3 + (nsymbs >> 1 < 2 ? nsymbs >> 1 : 2) + (cdf[nsymbs] >> 4);
    cdf[nsymbs] = (uint16_t)(cdf[nsymbs] + 1 - (cdf[nsymbs] >> 5));
    for (int i = 0; i < nsymbs - 1; i++)
      cdf[i] = (uint32_t)i >= s ? (uint16_t)(cdf[i] - (cdf[i] >> rate))
                                : (uint16_t)(cdf[i] + ((32768 - cdf[i]) >> rate));
  }
  inline void bit(uint32_t b) {  // bool(b, 16384): symbol over [16384, 0]
    store(b ? 16384u : 32768u, b ? 0u : 16384u, b ? 1u : 2u);
  }
  // done() (src/ec.rs:444-486)
  size_t finish() {
    int c = cnt;
    int s = 10 + c;
    const uint32_t m = 0x3FFF;
    uint32_t e = ((low + m) & ~m) | (m + 1);
    if (s > 0) {
      uint32_t n = (1u << (c + 16)) - 1;
      for (;;) {
        pre.push_back((uint16_t)(e >> (c + 16)));
        e &= n;
        s -= 8;
        c -= 8;
        n >>= 8;
        if (s <= 0) break;
      }
    }
    return pre.size();
  }
  void bytes(uint8_t *out) const {
    uint16_t cc = 0;
    for (size_t offs = pre.size(); offs > 0;) {
      offs--;
      cc = (uint16_t)(cc + pre[offs]);
      out[offs] = (uint8_t)cc;
      cc >>= 8;
    }
  }
};

}  // namespace

extern "C" {

long rv_ec_code_tokens(const uint32_t *tok, size_t n, uint16_t *cdf, uint8_t *out, size_t cap) {
  if (!tok && n) return rv_set_error(RV_EINVAL, "rv_ec_code_tokens: null tokens");
  if (!cdf) return rv_set_error(RV_EINVAL, "rv_ec_code_tokens: null cdf");
  EcWriter w;
  w.pre.reserve(n / 4 + 64);
  for (size_t i = 0; i < n; i++) {
    const uint32_t t = tok[i];
    if (t >> 31) {
      w.bit(t & 1);
    } else {
      const int off = (int)(t & 0x1FFF), len = (int)((t >> 13) & 31), s = (int)((t >> 18) & 31);
      if (off + len > RV_EC_TOTAL || len < 2 || s >= len - 1)
        return rv_set_error(RV_EINVAL, "rv_ec_code_tokens: bad token");
      w.symbol_update((uint32_t)s, cdf + off, len);
    }
  }
  const size_t nb = w.finish();
  if (out && nb <= cap) w.bytes(out);
  return (long)nb;
}

int rv_ec_default_cdf(int qctx, uint16_t *out) {
  if (qctx < 0 || qctx > 3 || !out) return rv_set_error(RV_EINVAL, "rv_ec_default_cdf");
  memcpy(out, RV_EC_DEFAULT_CDF[qctx], sizeof(RV_EC_DEFAULT_CDF[qctx]));
  return RV_OK;
}

int rv_ec_cdf_total(void) { return RV_EC_TOTAL; }

// CDFContext::reset_counts (src/context.rs:851-) over the coefficient CDFs
void rv_ec_reset_counts(uint16_t *cdf) {
  static const int fam[][3] = {{RV_EC_TXB_SKIP, 65, 3},   {RV_EC_EOB16, 4, 6},
                               {RV_EC_EOB32, 4, 7},       {RV_EC_EOB64, 4, 8},
                               {RV_EC_EOB128, 4, 9},      {RV_EC_EOB256, 4, 10},
                               {RV_EC_EOB512, 4, 11},     {RV_EC_EOB1024, 4, 12},
                               {RV_EC_EOB_EXTRA, 90, 3},  {RV_EC_BASE_EOB, 40, 4},
                               {RV_EC_BASE, 420, 5},      {RV_EC_BR, 210, 5},
                               {RV_EC_DC_SIGN, 6, 3},     {RV_EC_INTER_TX, 16, 17}};
  for (const auto &f : fam)
    for (int i = 0; i < f[1]; i++) cdf[f[0] + i * f[2] + f[2] - 1] = 0;
}

size_t rv_ec_scratch_bytes(int n_jobs) {
  const size_t nb = ((size_t)n_jobs + 1023) / 1024;
  return (size_t)n_jobs * 4 /* eob */ + ((size_t)n_jobs + 1) * 4 /* counts / offsets */ +
         (nb + 1) * 4 + 16;
}

int rv_ec_tokenize(const rv_ec_job *d_jobs, int n, int xdec, int ydec, int n_tiles, int map_w4,
                   int map_h4, uint8_t *d_map, void *d_scratch, uint32_t *d_offsets,
                   uint32_t *d_tokens, uint32_t token_cap, uint32_t *d_status, void *stream) {
  if (n < 0 || n > 1024 * 1024 || n_tiles < 1 || map_w4 < 1 || map_h4 < 1 || !d_map ||
      !d_scratch || !d_offsets || !d_status || (token_cap && !d_tokens) || (n && !d_jobs))
    return rv_set_error(RV_EINVAL, "rv_ec_tokenize: bad arguments");
  hipStream_t st = rv_resolve_stream(stream);
  if (hipMemsetAsync(d_map, 0, (size_t)n_tiles * 3 * map_w4 * map_h4, st) != hipSuccess)
    return rv_set_error(RV_EHIP, "rv_ec_tokenize: map clear");
  if (n == 0) {
    if (hipMemsetAsync(d_status, 0, 8, st) != hipSuccess ||
        hipMemsetAsync(d_offsets, 0, 4, st) != hipSuccess)
      return rv_set_error(RV_EHIP, "rv_ec_tokenize: status");
    return RV_OK;
  }
  EcArgs a;
  a.jobs = d_jobs;
  a.n = n;
  a.xdec = xdec;
  a.ydec = ydec;
  a.map_w4 = map_w4;
  a.map_h4 = map_h4;
  a.map = d_map;
  a.count = d_offsets;
  a.eob = (int32_t *)d_scratch;
  uint32_t *bsum = (uint32_t *)((char *)d_scratch + (size_t)n * 4);
  a.tokens = d_tokens;
  a.cap = token_cap;
  a.status = d_status;
  a.dn = nullptr;
  const int grid = (n + 3) / 4 < 4096 ? (n + 3) / 4 : 4096;
  ec_prep_kernel<<<grid, 256, 0, st>>>(a);
  ec_scan(d_offsets, n, nullptr, bsum, d_status, st);
  ec_token_kernel<<<grid, 256, 0, st>>>(a);
  RV_HIP_CHECK_LAUNCH();
  return RV_OK;
}

}  // extern "C"
