/*
 * rav1e_oracle.h -- CPU restatement of the rav1e encode hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the
 * MI355X product path (rav1e_amd/, include/rav1e_hip.h).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product never links, calls or falls back to it.
 *
 * Every function restates a reference function of geobacter-rs/rav1e
 * (/root/reference); the file:line each one follows is cited next to its
 * definition.  Parity pins ("Oracle"):
 *   - SAD / SATD: the 88 known-answer values of src/dist.rs:379-460;
 *   - 1-D and 2-D transforms: golden vectors produced by evaluating the
 *     reference's own transform source (tools/refeval/, tests/golden/);
 *   - MC put/prep/avg: restated from src/mc.rs:213-408 (no KATs exist in
 *     the reference: "parity unpinned" beyond the restatement itself).
 *
 * Conventions: pixel buffers are `const void*` + stride in ELEMENTS + an
 * `hbd` flag (0 = u8, 1 = u16), mirroring the generated-kernel ABI of the
 * reference (build/kernel/gen/dist.rs:132-139).  All i32 arithmetic wraps
 * (Rust release semantics).
 */
#ifndef RAV1E_ORACLE_H
#define RAV1E_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- distortion (src/dist.rs, src/rdo.rs) ---------------------------- */
uint32_t orc_get_sad(const void *org, ptrdiff_t org_stride, const void *ref,
                     ptrdiff_t ref_stride, int w, int h, int hbd);
/* emulate_gen: 0 = get_satd_ref (src/dist.rs:197-328);
 *              1 = generated i16-lane kernel (build/kernel/gen/dist.rs:173-357) */
uint32_t orc_get_satd(const void *org, ptrdiff_t org_stride, const void *ref,
                      ptrdiff_t ref_stride, int w, int h, int hbd,
                      int emulate_gen);
/* compute_lookahead_intra_costs (src/api/internal.rs:680-765): ceil(w/8) x
 * ceil(h/8) costs, org = the plane's pixel (0, 0), stride in elements. */
void orc_lookahead_intra_costs(const void *org, ptrdiff_t stride, int w, int h, int hbd, int bd,
                               uint32_t *out);
/* sse_wxh raw partials (src/rdo.rs:286-335): one u64 per importance
 * sub-block, raster order, (w/bw)*(h/bh) values, bw = min(8,w)>>xdec. */
int orc_sse_wxh(const void *a, ptrdiff_t sa, const void *b, ptrdiff_t sb,
                int w, int h, int xdec, int ydec, int hbd, uint64_t *out);
/* cdef_dist_wxh_8x8 integer moments (src/rdo.rs:219-253):
 * out[0]=sum_s out[1]=sum_d out[2]=sum_s2 out[3]=sum_d2 out[4]=sum_sd */
void orc_cdef_moments_8x8(const void *a, ptrdiff_t sa, const void *b,
                          ptrdiff_t sb, int hbd, int64_t out[5]);
/* f64 tail of cdef_dist_wxh_8x8 (src/rdo.rs:242-252) */
uint64_t orc_cdef_dist_from_moments(const int64_t m[5], int bit_depth);

/* ---- motion compensation (src/mc.rs) ---------------------------------- */
/* src points at the block's integer position; reads rows -3..h+4 and
 * columns -3..w+4 around it (src/mc.rs:232, 251, 273).
 * emulate_gen: 1 = generated u8 kernels' missing upper clamp
 * (build/kernel/gen/mc.rs:253-261, 281-290, 337-344). */
void orc_put_8tap(void *dst, ptrdiff_t dst_stride, const void *src,
                  ptrdiff_t src_stride, int w, int h, int col_frac,
                  int row_frac, int mode_x, int mode_y, int bit_depth,
                  int hbd, int emulate_gen);
void orc_prep_8tap(int16_t *tmp, const void *src, ptrdiff_t src_stride, int w,
                   int h, int col_frac, int row_frac, int mode_x, int mode_y,
                   int bit_depth, int hbd);
void orc_mc_avg(void *dst, ptrdiff_t dst_stride, const int16_t *tmp1,
                const int16_t *tmp2, int w, int h, int bit_depth, int hbd,
                int emulate_gen);
/* PredictionMode::predict_intra without CfL (src/predict.rs:202-241, 538-1035):
 * mode = PredictionMode (0 DC .. 12 PAETH), variant = PredictionVariant,
 * edge = rav1e's 257-pixel edge_buf. */
void orc_predict_intra(int mode, int variant, void *dst, ptrdiff_t stride, int w, int h,
                       int bit_depth, int hbd, const void *edge);
/* get_intra_edges (src/partition.rs:500-693), opt_mode None, for the
 * transform block of a superblock-level partition at tile-relative pixel
 * (x, y) of a tw x th tile region (pixel (0, 0) at `tile`); edge = 257 px. */
void orc_intra_edges_sb(const void *tile, ptrdiff_t stride, int hbd, int bd, int tw, int th,
                        int x, int y, int n, int have_top, int have_left, void *edge);
/* deblock_plane (src/deblock.rs:1174-1335) of plane pli at origin (visible
 * (0, 0)); lg / skip per luma 4x4 block (row pitch mi_stride): log2 of the
 * square block's width in 4x4 units, skip flag; levels = [Y vertical, Y
 * horizontal, U, V] */
void orc_deblock_plane(void *origin, ptrdiff_t stride, int hbd, int bd, int width, int height,
                       int xdec, int ydec, int pli, const uint8_t *lg, const uint8_t *skip,
                       int mi_stride, const uint8_t levels[4]);
int orc_deblock_fast_level(int ac_q, int bd, int is_key);
/* sse_plane (src/deblock.rs:1337-1407) of plane pli: the vertical and
 * horizontal level tallies (65 entries) of the unfiltered reconstruction
 * `rec` against the source `src` (visible origins; reads outside the
 * plane's width are 128, the fill of a fresh plane) */
void orc_deblock_sse_plane(const void *rec, ptrdiff_t rstride, const void *src, ptrdiff_t sstride,
                           int hbd, int bd, int width, int height, int xdec, int ydec, int pli,
                           const uint8_t *lg, const uint8_t *skip, int mi_stride,
                           int64_t v_tally[65], int64_t h_tally[65]);
/* sse_optimize's level choice (src/deblock.rs:1441-1473) from the three
 * planes' tallies */
void orc_deblock_sse_levels(const int64_t v_tally[3][65], const int64_t h_tally[3][65],
                            uint8_t levels[4]);
/* CDEF (src/cdef.rs): cdef_find_dir (:68-126) of the 8x8 block at img
 * (the padded u16 copy), cdef_filter_block (:152-228), adjust_strength
 * (:232-239), and cdef_filter_frame (:542-641) out of place: planes at
 * their visible origins, skip per luma 4x4 (pitch mi_stride), cdef_index
 * per 64x64 superblock (pitch ceil(width / 64)); dirs / vars (optional,
 * pitch ceil(width / 8)) receive the per-8x8 directions and variances. */
int orc_cdef_find_dir(const uint16_t *img, ptrdiff_t stride, int32_t *var, int coeff_shift);
void orc_cdef_filter_block(void *dst, ptrdiff_t dstride, int hbd, const uint16_t *in,
                           ptrdiff_t istride, int pri, int sec, int dir, int damping, int bd,
                           int xdec, int ydec);
int orc_cdef_adjust_strength(int strength, int32_t var);
void orc_cdef_filter_frame(const void *const in[3], const ptrdiff_t istride[3], void *const out[3],
                           const ptrdiff_t ostride[3], int hbd, int bd, int width, int height,
                           int xdec, int ydec, const uint8_t *skip, int mi_stride,
                           const uint8_t *cdef_index, const uint8_t y_str[8],
                           const uint8_t uv_str[8], int damping, uint8_t *dirs, int32_t *vars);
/* SUBPEL_FILTERS + get_filter (src/mc.rs:70-179, 201-210) */
const int32_t *orc_get_filter(int mode, int frac, int length);

/* ---- transforms (src/transform/) -------------------------------------- */
/* 1-D kernel ids: 0 = Id, 1 = Dct, 2 = Adst, 3 = FlipAdst (TBL_IDX order,
 * src/transform/mod.rs:158-173). Return 0 on success, -1 if the reference
 * leaves the (kind, n) pair unimplemented. */
int orc_fwd_txfm1d(int kind, int n, const int32_t *in, int32_t *out);
int orc_inv_txfm1d(int kind, int n, const int32_t *in, int32_t *out,
                   int range);
/* tx_size: TxSize enum order (src/transform/mod.rs:225-247);
 * tx_type: TxType enum order (src/transform/mod.rs:123-140).
 * forward: FwdTxfm2D::fht (src/transform/forward.rs:1804-1899); output is a
 * W-stride raster of W*H i32. */
int orc_fwd_txfm2d(const int16_t *residual, int32_t *coeffs, int tx_size,
                   int tx_type, int bit_depth);
/* inverse + add: NativeInvTxfm2D (src/transform/inverse.rs:1939-2114);
 * coeffs are min(W,32)*min(H,32) i32, row stride min(W,32). */
int orc_inv_txfm2d_add(const int32_t *coeffs, void *dst, ptrdiff_t dst_stride,
                       int tx_size, int tx_type, int bit_depth, int hbd);
/* ---- quantize / dequantize (src/quantize.rs) --------------------------- */
typedef struct {
  int log_tx_scale;
  uint32_t dc_quant;
  int32_t dc_offset;
  uint32_t dc_mul_add[3];
  uint32_t ac_quant;
  int32_t ac_offset_eob, ac_offset0, ac_offset1;
  uint32_t ac_mul_add[3];
} orc_qctx; /* QuantizationContext (src/quantize.rs:108-120) */
int orc_get_log_tx_scale(int tx_size);
int orc_coded_tx_area(int tx_size);
int orc_dc_q(int qindex, int delta_q, int bd);
int orc_ac_q(int qindex, int delta_q, int bd);
void orc_divu_gen(uint32_t d, uint32_t out[3]);
int32_t orc_divu_pair(int32_t x, const uint32_t d[3]);
void orc_qctx_update(orc_qctx *c, int qindex, int tx_size, int is_intra, int bd,
                     int dc_delta_q, int ac_delta_q);
/* coeffs indexed by scan position (the forward transform's W-stride raster,
 * first coded_tx_area entries); returns eob. */
int orc_quantize(const orc_qctx *c, const int32_t *coeffs, int32_t *qcoeffs, int tx_size,
                 int tx_type);
void orc_dequantize(int qindex, const int32_t *coeffs, int32_t *rcoeffs, int tx_size, int bd,
                    int dc_delta_q, int ac_delta_q);
/* estimate_rate (src/rdo.rs:204-216) */
uint64_t orc_estimate_rate(int qindex, int tx_size, uint64_t fast_distortion);
/* diff (src/encoder.rs:1044-1058) */
void orc_diff(int16_t *dst, const void *a, ptrdiff_t sa, const void *b,
              ptrdiff_t sb, int w, int h, int hbd);

/* ---- motion search (src/me.rs) ---------------------------------------- */
typedef struct { int16_t row, col; } orc_mv;

/* ---- lookahead (src/api/internal.rs) ------------------------------------ */
/* compute_block_importances' propagation (:823-1010), one (frame, reference)
 * pass; see orc_lookahead.c. */
void orc_propagate_importances(const void *org, ptrdiff_t org_stride, const void *ref,
                               ptrdiff_t ref_stride, int w_imp, int h_imp, int hbd,
                               const orc_mv *mvs, const uint32_t *intra_costs,
                               const float *importances, int n_unique,
                               float *ref_importances);
void orc_propagate_importances_costs(int w_imp, int h_imp, const orc_mv *mvs,
                                     const uint32_t *inter_costs, const uint32_t *intra_costs,
                                     const float *importances, int n_unique,
                                     float *ref_importances);
void orc_importance_inter_costs(const void *org, ptrdiff_t org_stride, const void *ref,
                                ptrdiff_t ref_stride, int w_imp, int h_imp, int hbd,
                                const orc_mv *mvs, uint32_t *inter_costs);
/* glibc's log2f restated (f32::log2 on x86-64 Linux), see orc_lookahead.c */
float orc_log2f(float x);
uint32_t orc_get_mv_rate(orc_mv a, orc_mv b, int allow_hp);
/* full_search (src/me.rs:943-990). org/ref point at plane (0,0) (the data
 * origin); x/y in pixels relative to it; may be negative (padding). */
void orc_full_search(const void *org, ptrdiff_t org_stride, const void *ref,
                     ptrdiff_t ref_stride, int hbd, int po_x, int po_y,
                     int x_lo, int x_hi, int y_lo, int y_hi, int blk_w,
                     int blk_h, int step, uint32_t lambda, orc_mv pmv0,
                     orc_mv pmv1, int allow_hp, orc_mv *best_mv,
                     uint64_t *lowest_cost);

/* diamond_me_search (src/me.rs:655-856).  org / ref point at their
 * plane's data origin (visible (0,0)); the ref geometry feeds
 * PlaneSlice::clamp for sub-pel prediction. */
typedef struct {
  const void *org;
  ptrdiff_t org_stride;
  const void *ref;
  ptrdiff_t ref_stride;
  int ref_width, ref_height, ref_xorigin, ref_yorigin, ref_xdec, ref_ydec;
  int hbd, bit_depth;
  int po_x, po_y, w, h;
  int mvx_min, mvx_max, mvy_min, mvy_max;
  orc_mv pmv[2];
  uint32_t lambda;
  int subpel, satd, allow_hp;
} orc_ds_ctx;
void orc_diamond_search(const orc_ds_ctx *c, const orc_mv *pred, int n_pred,
                        orc_mv *best_mv, uint64_t *best_cost);
/* get_subset_predictors (src/me.rs:82-174, ArrayVec capacity 17) */
#define ORC_MAX_PRED 17
int orc_subset_predictors(int bx, int by, const orc_mv *cmvs, int ncmv, const orc_mv *tile,
                          int tp, int tc, const orc_mv *prev, int pp, int fc, int fr, int fx,
                          int fy, orc_mv *out);
/* telescopic_subpel_search (src/me.rs:858-941): best_mv / lowest_cost are
 * the search's start (in) and result (out). */
void orc_telescopic_subpel(const orc_ds_ctx *c, orc_mv *best_mv, uint64_t *lowest_cost);
/* ---- MV reference stack (src/context.rs:2308-2965), orc_mvref.c -------- */
/* RefType codes: INTRA_FRAME 0, reference k of the replay 1 + k, NONE 8 */
#define ORC_INTRA_FRAME 0
#define ORC_NONE_FRAME 8
/* the fields of Block (src/context.rs:1395-1440) the scans read; newmv: the
 * mode counts as a NEWMV one in add_ref_mv_candidate */
typedef struct {
  int8_t ref[2];
  uint8_t n4_w, n4_h, newmv, pad_[3];
  orc_mv mv[2];
} orc_blk;
typedef struct {
  orc_mv this_mv, comp_mv;
  uint32_t weight;
} orc_mv_cand; /* CandidateMV */
/* find_mvrefs of the block at tile 4x4 offset (bx, by), bw4 x bh4, over a
 * tile grid (pitch stride, tile size cols x rows in 4x4 units, origin
 * tile_mi_x / y in the frame, frame size frame_cols x frame_rows);
 * ref_frames[1] = ORC_NONE_FRAME for a single reference; sign_bias[k] of
 * reference k.  Writes the stack (<= 9 entries) and its length; returns
 * the mode context. */
int orc_find_mvrefs(const orc_blk *grid, int stride, int cols, int rows, int tile_mi_x,
                    int tile_mi_y, int frame_cols, int frame_rows, int bx, int by, int bw4,
                    int bh4, const int ref_frames[2], const uint8_t *sign_bias,
                    orc_mv_cand stack[9], int *n_out);

/* tx-domain distortion (src/encoder.rs:1210-1224). */
uint64_t orc_tx_dist(const int32_t *coeffs, const int32_t *rcoeffs, int coded_area,
                     int tx_w, int tx_h);

/* ---- frame layout (src/frame/) --------------------------------------- */
/* Plane::new geometry (src/frame/plane.rs:215-244). Writes
 * {stride, alloc_height, xorigin, yorigin}. */
void orc_plane_geometry(int width, int height, int xpad, int ypad, int hbd,
                        int out[4]);
/* Plane::pad (src/frame/plane.rs:269-314) on a buffer of stride*alloc_h */
void orc_plane_pad(void *data, int stride, int alloc_height, int xorigin,
                   int yorigin, int xdec, int ydec, int w, int h, int hbd);
/* Plane::downsample_from (src/frame/plane.rs:399-423); both pointers at
 * their plane's data origin. */
void orc_downsample(void *dst, ptrdiff_t dst_stride, int dst_w, int dst_h,
                    const void *src, ptrdiff_t src_stride, int hbd);


/* ---- entropy coding (src/ec.rs, src/context.rs) --------------------- */
/* WriterBase<WriterEncoder> (src/ec.rs:100-600) */
typedef struct {
  uint16_t rng;
  int16_t cnt;
  uint32_t low;        /* ec_window */
  uint16_t *pre;       /* precarry */
  size_t n, cap;
} orc_ecw;
/* the Reader of src/ec.rs's test module (:914-1010) */
typedef struct {
  const uint8_t *buf;
  size_t len, bptr;
  uint32_t dif;
  uint16_t rng;
  int16_t cnt;
} orc_ecr;
/* the coefficient CDFs of CDFContext (flat, orc_ec_tables.h layout) and
 * BlockContext's above / left coefficient contexts */
#define ORC_EC_CDF_TOTAL 4317
typedef struct {
  uint16_t cdf[ORC_EC_CDF_TOTAL];
  uint8_t above[3][1024];  /* COEFF_CONTEXT_MAX_WIDTH */
  uint8_t left[3][16];     /* MIB_SIZE */
} orc_ec_ctx;
/* one step of a tile's coefficient coding (orc_ec_code_jobs) */
typedef struct {
  int32_t kind;       /* 0 tx block, 1 skip leaf, 2 superblock row, 3 new tile */
  int32_t plane;
  int32_t bx, by;     /* TileBlockOffset (luma 4x4 units) */
  int32_t tx_size;    /* TX_4X4 .. TX_64X64 (square) */
  int32_t tx_type;
  int32_t is_inter;
  int32_t bw_lg, bh_lg;  /* tx job: plane block log2 w / h; skip job: the leaf's (luma) */
  int32_t coeff_off;
} orc_ec_job;
void orc_ecw_init(orc_ecw *w);
void orc_ecw_free(orc_ecw *w);
void orc_ecw_symbol(orc_ecw *w, uint32_t s, const uint16_t *cdf, int n);
void orc_update_cdf(uint16_t *cdf, int len, uint32_t val);
void orc_ecw_symbol_update(orc_ecw *w, uint32_t s, uint16_t *cdf, int len);
void orc_ecw_bool(orc_ecw *w, int val, uint16_t f);
void orc_ecw_bit(orc_ecw *w, int bit);
void orc_ecw_literal(orc_ecw *w, int bits, uint32_t s);
void orc_ecw_golomb(orc_ecw *w, uint16_t level);
size_t orc_ecw_finish(orc_ecw *w);
void orc_ecw_bytes(const orc_ecw *w, uint8_t *out);
size_t orc_ecw_done(orc_ecw *w, uint8_t *out, size_t cap);
void orc_ecr_init(orc_ecr *r, const uint8_t *buf, size_t len);
int orc_ecr_bool(orc_ecr *r, uint32_t f);
int orc_ecr_symbol(orc_ecr *r, const uint16_t *icdf, int n_entries);
void orc_ec_ctx_init(orc_ec_ctx *c, int qctx);
void orc_ec_reset_counts(uint16_t *cdf);
void orc_ec_reset_skip(orc_ec_ctx *c, int bx, int by, int bw_lg, int bh_lg, int xdec, int ydec);
void orc_ec_reset_left(orc_ec_ctx *c);
int orc_ec_write_coeffs(orc_ecw *w, orc_ec_ctx *cx, int plane, int bx, int by,
                        const int32_t *coeffs_in, int is_inter, int tx, int tx_type,
                        int plane_lg, int xdec, int ydec, int reduced, uint8_t *cul_out);
long orc_ec_code_jobs(const orc_ec_job *jobs, int n, const int32_t *coeffs, const uint16_t *cdf_init,
                      int xdec, int ydec, uint8_t *out, long cap, int32_t *tile_bytes,
                      uint16_t *ret, uint16_t *cdf_out);
const uint16_t *orc_ec_default_cdf(int qctx);
struct orc_replay;
int orc_replay_set_entropy(struct orc_replay *r, int on);
void orc_replay_entropy_stats(const struct orc_replay *r, uint64_t out[4]);

/* ---- loop restoration, self-guided filter (orc_lrf.c) ---- */
typedef struct {
  int unit_size, sb_h_shift, sb_v_shift, stripe_h, cols, rows;
} orc_lrf_plane_cfg;
typedef struct {
  int8_t set;     /* -1: RestorationFilter::None, else the Sgrproj set */
  int8_t xqd[2];
} orc_lrf_unit;
extern const uint32_t ORC_SGRPROJ_PARAMS_S[16][2];
void orc_lrf_config(int width, int height, int xdec, int ydec, int base_q_idx, int tiled,
                    int tile_w_sb, int tile_h_sb, orc_lrf_plane_cfg out[3]);
void orc_lrf_integral(const void *cdeffed, ptrdiff_t cs, const void *deblocked, ptrdiff_t ds,
                      int hbd, int x0, int y0, int crop_w, int crop_h, int stripe_w, int stripe_h,
                      uint32_t *ii, uint32_t *sq, int iis);
void orc_sgr_stripe_filter(int set, const int8_t xqd[2], int bd, const uint32_t *ii,
                           const uint32_t *sq, int iis, int w, int h, const void *cd, ptrdiff_t cs,
                           void *out, ptrdiff_t os, int hbd);
void orc_sgr_solve(int set, int bd, const uint32_t *ii, const uint32_t *sq, int iis,
                   const void *in, ptrdiff_t is, const void *cd, ptrdiff_t cs, int hbd, int w, int h,
                   int8_t xqd[2]);
void orc_sgr_solve_finish(int set, int w, int h, int64_t H00, int64_t H01, int64_t H11, int64_t C0,
                          int64_t C1, int8_t xqd[2]);
void orc_lrf_filter_frame(void *const out[3], const void *const pre[3], const ptrdiff_t stride[3],
                          int hbd, int bd, int width, int height, int xdec, int ydec,
                          const orc_lrf_plane_cfg cfg[3], const orc_lrf_unit *const units[3],
                          int enable_cdef);
uint32_t orc_symbol_bits(uint32_t s, const uint16_t *cdf, int nsym);
uint32_t orc_lrf_rate(const uint16_t cdf[4], const int8_t ref[2], int set, const int8_t xqd[2]);
void orc_lrf_commit(uint16_t cdf[4], int8_t ref[2], int set, const int8_t xqd[2]);
void orc_lrf_tile_init(uint16_t cdf[4], int8_t ref[3][2]);
int orc_replay_set_lrf(struct orc_replay *r, int on);
void orc_replay_lrf_units(const struct orc_replay *r, int plane, int8_t *out, int cap);

#ifdef __cplusplus
}
#endif
#endif
