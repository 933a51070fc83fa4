/*
 * rav1e_hip.h -- C ABI of the MI355X (gfx950) encode hot path for rav1e.
 *
 * Two layers, both plain C (no torch / HIP types in any signature; a
 * stream is an opaque `void *` that is a hipStream_t, NULL = the library's
 * per-thread default stream):
 *
 *  1. Drop-in "asm backend" entry points, one symbol per (kernel, block
 *     size, pixel type), with exactly the signatures rav1e's x86 FFI binds
 *     (byte strides, `isize`, `i32`), so a src/asm/hip/{dist,mc}.rs table can
 *     point at them the way src/asm/x86/{dist,mc}.rs point at NASM.  They
 *     take HOST pointers, stage the block through the device and block
 *     until the result is back: correct, reentrant, latency bound.  They
 *     exist for drop-in parity (the reference's `check_asm` pattern); the
 *     production path is layer 2.
 *
 *  2. Batched entry points (`rv_*_batch`): one launch per tile-step over
 *     all candidate blocks, device-resident planes (`rv_plane`) and job
 *     arrays, results left in device memory, asynchronous on `stream`.
 *
 * Semantics follow the reference's declared ground truth (the `*_ref`
 * functions that `feature = "check_asm"` cross-checks against) bit for bit;
 * each entry point cites the reference function it replaces.
 * Reference = geobacter-rs/rav1e; paths below are relative to its root.
 *
 * Errors: batched entry points return 0 on success, RV_EINVAL for
 * arguments the reference's safe wrappers would `assert!` on, RV_EHIP for
 * a HIP runtime failure (rv_last_error() has the text).  The asm-shaped
 * entry points have no error channel (neither has NASM): on a HIP failure
 * they print the error and abort(), they never return a wrong value.
 */
#ifndef RAV1E_HIP_H
#define RAV1E_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RV_OK 0
#define RV_EINVAL (-1)
#define RV_EHIP (-2)
#define RV_ENOTSUP (-3)

/* ---------------------------------------------------------------------
 * Dispatch level.  Mirrors CpuFeatureLevel (src/cpu_features/x86.rs:13-61)
 * with one more level, HIP, selected like the others through
 * RAV1E_CPU_TARGET (src/cpu_features/x86.rs:44-59): RAV1E_CPU_TARGET=hip.
 * ------------------------------------------------------------------- */
typedef enum rv_cpu_feature_level {
  RV_CPU_NATIVE = 0,
  RV_CPU_SSE2 = 1,
  RV_CPU_SSSE3 = 2,
  RV_CPU_AVX2 = 3,
  RV_CPU_HIP = 4,
  RV_CPU_LEVELS = 5
} rv_cpu_feature_level;

/* CpuFeatureLevel::default() + the RAV1E_CPU_TARGET override
 * (src/cpu_features/x86.rs:34-61); "hip" selects RV_CPU_HIP. */
int rv_cpu_feature_level_default(void);
/* CpuFeatureLevel::as_index (src/cpu_features/x86.rs:26-30) */
int rv_cpu_feature_level_index(int level);

/* ---------------------------------------------------------------------
 * Runtime
 * ------------------------------------------------------------------- */
/* Number of visible gfx950 devices (0 if none; never aborts). */
int rv_device_count(void);
/* Select the device for the calling thread (hipSetDevice). */
int rv_set_device(int device);
const char *rv_last_error(void);
/* Library build string, e.g. "rav1e_hip gfx950 <date>". */
const char *rv_version(void);

void *rv_malloc(size_t bytes);            /* device memory, NULL on error */
void rv_free(void *p);
void *rv_host_alloc(size_t bytes);        /* pinned host memory */
void rv_host_free(void *p);
int rv_memcpy_h2d(void *dst, const void *src, size_t bytes, void *stream);
int rv_memcpy_d2h(void *dst, const void *src, size_t bytes, void *stream);
int rv_memcpy_d2d(void *dst, const void *src, size_t bytes, void *stream);
int rv_memset(void *dst, int value, size_t bytes, void *stream);
void *rv_stream_create(void);
/* A stream at a priority: < 0 the highest, > 0 the lowest, 0 the default
 * (HIP serves each priority from a hardware-queue pool of its own). */
void *rv_stream_create_priority(int priority);
int rv_stream_destroy(void *stream);
int rv_stream_sync(void *stream);
int rv_device_sync(void);
/* An empty kernel on `stream` (null: the default stream), for finding a
 * region in a kernel trace: bench.py launches one right before and one right
 * after its timed region (tools/prof_json.py restricts the occupancy figures
 * to what lies between). */
int rv_trace_marker(void *stream);
void *rv_event_create(void);
int rv_event_destroy(void *ev);
int rv_event_record(void *ev, void *stream);
int rv_event_sync(void *ev);
/* work submitted to `stream` after this call waits for `ev`'s last record
 * (hipStreamWaitEvent) */
int rv_stream_wait_event(void *stream, void *ev);
/* milliseconds between two recorded events (hipEventElapsedTime) */
float rv_event_elapsed_ms(void *start, void *stop);

/* ---------------------------------------------------------------------
 * Data model: a padded plane in device memory.  Reproduces PlaneConfig
 * (src/frame/plane.rs:22-47, geometry Plane::new :215-244): pixel (x, y)
 * of the visible area lives at data[(yorigin + y) * stride + xorigin + x];
 * x, y may be negative down to -xorigin / -yorigin (the padding).
 * ------------------------------------------------------------------- */
typedef struct rv_plane {
  void *data;         /* device pointer to element 0 of the allocation */
  int32_t stride;     /* in elements */
  int32_t alloc_height;
  int32_t width;      /* visible width / height */
  int32_t height;
  int32_t xorigin;
  int32_t yorigin;
  int32_t xdec;
  int32_t ydec;
  int32_t hbd;        /* 0: u8 pixels, 1: u16 pixels */
  int32_t bit_depth;  /* 8 / 10 / 12; rv_plane_geometry sets 8 for u8 planes
                         and 0 ("not stated") for u16 ones.  Entry points
                         whose exactness depends on the range (the SEA box
                         sums) require it on u16 planes. */
} rv_plane;

/* Plane::new geometry (src/frame/plane.rs:215-244): fills stride,
 * alloc_height, xorigin, yorigin, width, height, xdec, ydec, hbd; data is
 * left NULL.  Returns the allocation size in bytes. */
size_t rv_plane_geometry(rv_plane *p, int width, int height, int xdec,
                         int ydec, int xpad, int ypad, int hbd);
/* Plane::pad (src/frame/plane.rs:269-314): replicate edges into padding. */
int rv_plane_pad(const rv_plane *p, void *stream);
/* Plane::downsample_from (src/frame/plane.rs:399-423): 2x2 box filter
 * (s + 2) >> 2 of src's visible area into dst (dst->width x dst->height),
 * followed by dst padding like Frame::new's callers do. */
int rv_plane_downsample(const rv_plane *dst, const rv_plane *src,
                        void *stream);

/* ---------------------------------------------------------------------
 * Batched distortion.  All jobs of one call share (w, h).
 * Block positions are in the plane's visible coordinates.
 * ------------------------------------------------------------------- */
typedef struct rv_dist_job {
  int32_t org_x, org_y; /* block in `org` */
  int32_t ref_x, ref_y; /* block in `ref` */
} rv_dist_job;

/* get_sad (src/dist.rs:48-111) == get_sad_ref (src/dist.rs:25-46):
 * out[i] = sum |org - ref| over the w x h block of job i. */
int rv_sad_batch(const rv_plane *org, const rv_plane *ref,
                 const rv_dist_job *d_jobs, int n, int w, int h,
                 uint32_t *d_out, void *stream);
/* get_satd (src/dist.rs:121-193) == get_satd_ref (src/dist.rs:197-328):
 * 4x4 (min(w,h) == 4) or 8x8 Hadamard, sum |.| then
 * (sum + (1 << ln >> 1)) >> ln, ln = msb(min(w, h, 8)). */
int rv_satd_batch(const rv_plane *org, const rv_plane *ref,
                  const rv_dist_job *d_jobs, int n, int w, int h,
                  uint32_t *d_out, void *stream);
/* compute_lookahead_intra_costs (src/api/internal.rs:680-765) of a luma
 * plane: d_costs[by * ceil(width / 8) + bx] = get_satd of the 8x8 block at
 * (8 bx, 8 by) against its DC_PRED prediction, which the reference's tile
 * rect makes pred_dc_128 (the constant 128 << (bit_depth - 8)).  Blocks of
 * a partial last column / row read the plane's padding, as the reference's
 * region does. */
int rv_lookahead_intra_costs(const rv_plane *p, int bit_depth, uint32_t *d_costs,
                             void *stream);

/* sse_wxh raw partials (src/rdo.rs:286-335): per job, one u64 per
 * importance sub-block (bw x bh = (min(w,8) >> xdec) x (min(h,8) >> ydec),
 * xdec/ydec taken from `org`), raster order: d_out[i * nsub + k],
 * nsub = (w / bw) * (h / bh).  The f64 bias stays with the caller
 * (src/rdo.rs:325-331). */
int rv_sse_batch(const rv_plane *org, const rv_plane *ref,
                 const rv_dist_job *d_jobs, int n, int w, int h,
                 uint64_t *d_out, void *stream);
/* cdef_dist_wxh_8x8 integer moments (src/rdo.rs:219-241) for every 8x8 of
 * a w x h block (w, h multiples of 8): d_out[(i * nsub + k) * 5 + m],
 * m = {sum_s, sum_d, sum_s2, sum_d2, sum_sd}, nsub = (w/8) * (h/8). */
int rv_cdef_moments_batch(const rv_plane *org, const rv_plane *ref,
                          const rv_dist_job *d_jobs, int n, int w, int h,
                          int64_t *d_out, void *stream);

/* Transform-domain distortion of encode_tx_block (src/encoder.rs:1210-1224,
 * tune = Psnr): per block, sum over the coded area (min(W,32) *
 * min(H,32)) of ((c - rc) * (c - rc)) as u64 -- i32 wrapping square,
 * sign-extended -- then (d + (1 << (s - 1))) >> s, s = 2 * (3 -
 * get_log_tx_scale(tx_size)) (src/quantize.rs:34-39).  coeffs: block i at
 * d_coeffs + i * coeff_stride (the fht raster); rcoeffs: [n][coded area]. */
int rv_tx_dist_batch(const int32_t *d_coeffs, int coeff_stride,
                     const int32_t *d_rcoeffs, int n, int tx_size,
                     uint64_t *d_out, void *stream);

/* ---------------------------------------------------------------------
 * Batched motion compensation.  FilterMode (src/mc.rs:58-66):
 * 0 REGULAR, 1 SMOOTH, 2 SHARP, 3 BILINEAR.  Fracs are 1/16 pel (0..15).
 * The source block's integer position is (src_x, src_y); the filters read
 * rows -3..h+4 and columns -3..w+4 around it (src/mc.rs:232-273), which
 * must lie inside the padded allocation (PlaneSlice::clamp,
 * src/frame/plane.rs:521-533, is the caller's job as in predict_inter).
 * ------------------------------------------------------------------- */
typedef struct rv_mc_job {
  int32_t src_x, src_y;   /* integer source position in `src` */
  int32_t dst_x, dst_y;   /* destination block in `dst` (put/avg) */
  int32_t col_frac, row_frac;
} rv_mc_job;

/* put_8tap (src/mc.rs:410-519) == put_8tap_ref (src/mc.rs:213-307). */
int rv_put_8tap_batch(const rv_plane *dst, const rv_plane *src,
                      const rv_mc_job *d_jobs, int n, int w, int h,
                      int mode_x, int mode_y, int bit_depth, void *stream);
/* prep_8tap (src/mc.rs:520-616) == prep_8tap_ref (src/mc.rs:310-387):
 * d_tmp[i * w * h + r * w + c], i16. */
int rv_prep_8tap_batch(int16_t *d_tmp, const rv_plane *src,
                       const rv_mc_job *d_jobs, int n, int w, int h,
                       int mode_x, int mode_y, int bit_depth, void *stream);
/* mc_avg (src/mc.rs:617-706) == mc_avg_ref (src/mc.rs:389-408) of the
 * i-th w*h tiles of tmp1 / tmp2 into dst at (dst_x, dst_y) of job i. */
int rv_mc_avg_batch(const rv_plane *dst, const int16_t *d_tmp1,
                    const int16_t *d_tmp2, const rv_mc_job *d_jobs, int n,
                    int w, int h, int bit_depth, void *stream);

/* Fused sub-pel candidate evaluation: predict_inter's put_8tap into
 * on-chip memory, then get_sad / get_satd against org -- the pair
 * compute_mv_rd_cost runs per sub-pel candidate (src/me.rs:811-838).
 * job.dst_x/dst_y = the org block; out[i] = SAD (metric 0) or SATD (1). */
int rv_mc_dist_batch(const rv_plane *org, const rv_plane *ref,
                     const rv_mc_job *d_jobs, int n, int w, int h,
                     int mode_x, int mode_y, int bit_depth, int metric,
                     uint32_t *d_out, void *stream);

/* ---------------------------------------------------------------------
 * Batched transforms.  TxSize order = src/transform/mod.rs:225-247
 * (0 TX_4X4 ... 18 TX_64X16); TxType order = src/transform/mod.rs:123-140
 * (0 DCT_DCT ... 15 H_FLIPADST).
 * ------------------------------------------------------------------- */
/* forward_transform (src/transform/mod.rs:556-566) = FwdTxfm2D::fht
 * (src/transform/forward.rs:1804-1899): residual [n][W*H] i16 ->
 * coeffs [n][W*H] i32 (W-stride raster, full W x H also for 64-point
 * sizes, forward.rs:1885-1889).  RV_ENOTSUP for (size, type) pairs the
 * reference leaves unimplemented. */
int rv_fwd_txfm_batch(const int16_t *d_residual, int32_t *d_coeffs, int n,
                      int tx_size, int tx_type, int bit_depth, void *stream);
typedef struct rv_tx_job {
  int32_t src_x, src_y;   /* source block (org) */
  int32_t pred_x, pred_y; /* prediction block */
} rv_tx_job;
/* diff (src/encoder.rs:1044-1058) fused with forward_transform: the
 * residual src - pred never leaves the chip.  coeffs as above. */
int rv_diff_fwd_txfm_batch(const rv_plane *src, const rv_plane *pred,
                           const rv_tx_job *d_jobs, int n, int tx_size,
                           int tx_type, int bit_depth, int32_t *d_coeffs,
                           void *stream);
/* inverse_transform_add (src/transform/mod.rs:568-580) =
 * NativeInvTxfm2D::inv_txfm2d_add (src/transform/inverse.rs:1939-2114):
 * coeffs [n][min(W,32)*min(H,32)] (row stride min(W,32)) added into dst
 * at (pred_x, pred_y) of job i with clip to [0, 2^bd - 1]. */
int rv_inv_txfm_add_batch(const int32_t *d_coeffs, const rv_plane *dst,
                          const rv_tx_job *d_jobs, int n, int tx_size,
                          int tx_type, int bit_depth, void *stream);

/* ---------------------------------------------------------------------
 * Quantisation, the step of encode_tx_block between the transforms
 * (src/encoder.rs:1170, 1192).  One wavefront per block.
 * ------------------------------------------------------------------- */
/* QuantizationContext::update + quantize (src/quantize.rs:205-316) of n
 * blocks of one (tx_size, tx_type): block i at d_coeffs + i * coeff_stride,
 * read at the scan positions of av1_scan_orders[tx_size][tx_type]
 * (src/scan_order.rs:892) -- i.e. the forward transform's W-stride raster,
 * first coded_tx_area = min(W,32) * min(H,32) entries, as encode_tx_block
 * hands it over.  d_qcoeffs: [n][coded area] levels; d_rcoeffs (may be
 * NULL): the same blocks dequantized (src/quantize.rs:319-333), the
 * inverse transform's input; d_eob (may be NULL): eob per block as the
 * reference computes it.  qindex 1..255 (lossless is unsupported, as in
 * src/encoder.rs:1099). */
int rv_quantize_batch(const int32_t *d_coeffs, int coeff_stride, int n, int tx_size,
                      int tx_type, int qindex, int bit_depth, int is_intra,
                      int dc_delta_q, int ac_delta_q, int32_t *d_qcoeffs,
                      int32_t *d_rcoeffs, uint32_t *d_eob, void *stream);
/* dequantize (src/quantize.rs:319-333): [n][coded area] levels -> values. */
int rv_dequantize_batch(const int32_t *d_qcoeffs, int n, int tx_size, int qindex,
                        int bit_depth, int dc_delta_q, int ac_delta_q,
                        int32_t *d_rcoeffs, void *stream);

/* estimate_rate (src/rdo.rs:204-216) for n blocks of one TxSize: d_rate[i] =
 * the rate the reference reads off RDO_RATE_TABLE for tx-domain distortion
 * d_tx_dist[i] (rv_tx_dist_batch's output, src/encoder.rs:1210-1224) at the
 * frame's base qindex (0..255).  Replaces the call at src/encoder.rs:1231. */
int rv_estimate_rate_batch(const uint64_t *d_tx_dist, int n, int qindex, int tx_size,
                           uint64_t *d_rate, void *stream);

/* ---------------------------------------------------------------------
 * Motion search
 * ------------------------------------------------------------------- */
/* ---- intra prediction (src/predict.rs:202-241, 538-1035) ---------------
 * PredictionMode::predict_intra without CfL for every job: mode is the
 * PredictionMode (0 DC_PRED, 1 V, 2 H, 3 D45, 4 D135, 5 D117, 6 D153,
 * 7 D207, 8 D63, 9 SMOOTH, 10 SMOOTH_V, 11 SMOOTH_H, 12 PAETH), variant the
 * PredictionVariant of the block's tile position (0 NONE, 1 LEFT, 2 TOP,
 * 3 BOTH, src/predict.rs:175-184); the predicted tx_size block is written at
 * (x, y) of dst.  d_edges: per job rav1e's edge_buf, 4 * 64 + 1 pixels of
 * dst's pixel type (left bottom-to-top right-aligned in [0, 128), top-left
 * at 128, above from 129; get_intra_edges, src/recon_intra.rs). */
typedef struct rv_intra_job {
  int32_t x, y;
  int32_t mode, variant;
} rv_intra_job;
int rv_predict_intra_batch(const rv_plane *dst, const rv_intra_job *d_jobs, const void *d_edges,
                           int n, int tx_size, int bit_depth, void *stream);

/* ---- deblocking (src/deblock.rs) ---------------------------------------
 * deblock_plane (src/deblock.rs:1174-1335, replaces the per-edge loop of
 * deblock_filter_frame :1410-1416) of plane pli (0 Y, 1 U, 2 V) of a frame
 * width x height luma pixels, in place: every transform edge of the 4x4
 * grid, vertical then horizontal, with the 4 / 6 / 8 / 14-tap filters and
 * their masks.  d_lg / d_skip: per luma 4x4 block (row pitch mi_stride,
 * device memory) log2 of the square block's width in 4x4 units (1 = 8x8 ..
 * 4 = 64x64; the transform is the block's size) and its skip flag; every
 * block inter, loop-filter deltas off.  levels (host) = DeblockState.levels
 * [Y vertical, Y horizontal, U, V]. */
int rv_deblock_plane(const rv_plane *plane, int pli, int width, int height, const uint8_t *d_lg,
                     const uint8_t *d_skip, int mi_stride, const uint8_t *levels, int bit_depth,
                     void *stream);
/* deblock_filter_optimize's fast path (src/deblock.rs:1477-1517, speed >= 8):
 * the level from the frame's ac quantizer (ac_q(base_q_idx, 0, bd)). */
int rv_deblock_fast_level(int ac_q, int bit_depth, int is_key);
/* sse_optimize (src/deblock.rs:1418-1475, deblock_filter_optimize below
 * speed 8; replaces sse_plane :1337-1407 and its sse_v_edge / sse_h_edge /
 * sse_size{4,6,8,14}): rec[3] / src[3] = the frame's unfiltered
 * reconstruction and its source (Y U V, the chroma planes' width / height =
 * the luma's rounded up >> xdec / ydec); reads outside a plane's width are
 * 128, the fill of a fresh plane.  d_tally (device, 3 x 130 int64) receives
 * each plane's vertical then horizontal level tallies (65 each, not prefix
 * summed), d_levels (device, 4 bytes) the chosen DeblockState.levels [Y
 * vertical, Y horizontal, U, V].  Block map as rv_deblock_plane. */
int rv_deblock_sse(const rv_plane *rec, const rv_plane *src, int width, int height,
                   const uint8_t *d_lg, const uint8_t *d_skip, int mi_stride, int64_t *d_tally,
                   uint8_t *d_levels, int bit_depth, void *stream);
/* deblock_filter_frame (src/deblock.rs:1410-1416) of planes[3] with the
 * levels in device memory (d_levels, e.g. from rv_deblock_sse); nothing is
 * filtered when both luma levels are 0 (src/encoder.rs:2790-2793). */
int rv_deblock_frame(const rv_plane *planes, int width, int height, const uint8_t *d_lg,
                     const uint8_t *d_skip, int mi_stride, const uint8_t *d_levels, int bit_depth,
                     void *stream);

/* ---- CDEF (src/cdef.rs) ------------------------------------------------
 * cdef_filter_frame (src/cdef.rs:542-641) as two steps on device planes.
 * rv_cdef_find_dirs: cdef_analyze_superblock (:278-317) over the frame --
 * cdef_find_dir (:68-126) of every 8x8 luma block that is not skip (skip =
 * all four of its 4x4 blocks skip), dir 0 / var 0 otherwise; d_dir / d_var
 * per 8x8 block, pitch ceil(width / 8).  d_skip per luma 4x4 block, pitch
 * mi_stride >= 2 * ceil(width / 8), rows 2 * ceil(height / 8).
 * rv_cdef_filter_plane: cdef_filter_superblock (:411-534) over every
 * superblock of plane pli, src -> dst (distinct planes): cdef_filter_block
 * (:152-228) on non-skip blocks with the strengths of the block's 64x64
 * cdef_index (d_cdef_index, pitch ceil(width / 64)), a copy on skip ones.
 * y_strengths / uv_strengths / damping: FrameInvariants::cdef_{y,uv}_
 * strengths (host, 8 entries <= 63) and cdef_damping.  Taps outside the
 * visible plane read what the reference's padded copy holds there
 * (CDEF_VERY_LARGE in the 2-pixel ring, 128 beyond). */
int rv_cdef_find_dirs(const rv_plane *luma, int width, int height, const uint8_t *d_skip,
                      int mi_stride, uint8_t *d_dir, int32_t *d_var, int bit_depth, void *stream);
int rv_cdef_filter_plane(const rv_plane *src, const rv_plane *dst, int pli, int width, int height,
                         const uint8_t *d_skip, int mi_stride, const uint8_t *d_dir,
                         const int32_t *d_var, const uint8_t *d_cdef_index,
                         const uint8_t *y_strengths, const uint8_t *uv_strengths, int damping,
                         int bit_depth, void *stream);

/* ---- loop restoration (src/lrf.rs) --------------------------------------
 * The frame's restoration runs inside the replay (RV_REPLAY_LRF).  This
 * entry runs one stripe through the same device code as lrf_filter_frame's
 * kernel: setup_integral_image's view of the stripe at (x0, y0), sw x sh
 * pixels (sh <= 64) of a cw x ch crop (cd inside the stripe, db outside its
 * rows, clamped), then sgrproj_stripe_filter (src/lrf.rs:677-760) with set
 * `set` and xqd (xqd0, xqd1), into d_out (u8 / u16, row pitch sw). */
int rv_lrf_stripe_filter(const rv_plane *cd, const rv_plane *db, int x0, int y0, int sw, int sh,
                         int cw, int ch, int set, int xqd0, int xqd1, int bit_depth, void *d_out,
                         void *stream);

/* ---- stream containers ---------------------------------
 * The y4m input rav1e reads (src/bin/decoder/y4m.rs through the y4m crate)
 * and the IVF file it writes (ivf/src/lib.rs:6-30).  Host code.
 * rv_y4m_read_frame reads the next frame's planar samples (Y, then U, V;
 * 16-bit little endian above 8 bits: the packed layout rv_replay_set_input
 * takes, rv_y4m_frame_bytes of them) and returns RV_OK, or 1 at the end of
 * the stream. */
typedef struct rv_y4m_info {
  int width, height, bit_depth, xdec, ydec, fps_num, fps_den;
} rv_y4m_info;
typedef struct rv_y4m rv_y4m;
typedef struct rv_ivf rv_ivf;
int rv_y4m_parse_header(const char *line, rv_y4m_info *out);
rv_y4m *rv_y4m_open(const char *path);
int rv_y4m_get_info(const rv_y4m *y, rv_y4m_info *out);
size_t rv_y4m_frame_bytes(const rv_y4m *y);
int rv_y4m_read_frame(rv_y4m *y, void *host_yuv);
void rv_y4m_close(rv_y4m *y);
/* write_ivf_header (version 0, header size 32, "AV01", width, height,
 * framerate num / den), then write_ivf_frame per frame (length, pts, bytes). */
rv_ivf *rv_ivf_create(const char *path, int width, int height, int fps_num, int fps_den);
int rv_ivf_write_frame(rv_ivf *v, uint64_t pts, const uint8_t *data, size_t len);
int rv_ivf_close(rv_ivf *v);

/* ---- entropy coding (src/ec.rs, src/context.rs) -------------------------
 * Coefficient coding = ContextWriter::write_coeffs_lv_map (src/context.rs:
 * 3965-4220) for square transforms (TX_4X4 .. TX_64X64, the sizes the
 * replay codes), split into a device tokenizer and the host range coder.
 *
 * rv_ec_job: one step of a tile's coding, in coding order (the shape of
 * encode_tile's superblock loop, src/encoder.rs:3160-3340, down to
 * write_tx_tree / write_tx_blocks, :1757-2030):
 *   kind 0 a transform block: write_coeffs_lv_map(plane, bo = (bx, by),
 *          coeffs, is_inter ? NEARESTMV : DC_PRED, tx_size, tx_type,
 *          plane_bsize = (1 << bw_lg) x (1 << bh_lg), xdec, ydec,
 *          reduced tx set); coeffs = the quantised coefficients, raster of the
 *          coded size (min(w, 32) square), device pointer;
 *   kind 1 a skip leaf of (1 << bw_lg) x (1 << bh_lg) luma pixels at (bx, by):
 *          reset_skip_context (:1651-1679);
 *   kind 2 a superblock row starts: reset_left_contexts;
 *   kind 3 a tile starts (a fresh BlockContext; its own range coder).
 * (bx, by) are TileBlockOffsets: luma 4x4 units relative to the tile.
 * `tile` indexes the tile's context map (jobs of a tile share it). */
typedef struct rv_ec_job {
  int32_t kind, plane, bx, by, tx_size, tx_type, is_inter, bw_lg, bh_lg, tile;
  const int32_t *coeffs;
} rv_ec_job;
/* rv_ec_tokenize: the symbols of every kind-0 job.  Device buffers: d_map
 * n_tiles * 3 * map_w4 * map_h4 bytes (cleared here; map_w4 / map_h4 >= the
 * largest tile in luma 4x4 units), d_scratch rv_ec_scratch_bytes(n) bytes,
 * d_offsets n + 1 u32 (job j's tokens start at d_offsets[j]; [n] = total),
 * d_tokens token_cap u32, d_status 2 u32 ([0] total tokens, [1] 1 if the
 * total exceeded token_cap: tokens past it were dropped).  Token format in
 * rav1e_amd/csrc/rv_ec.hip.  Returns 0 or an error (n <= 2^20). */
size_t rv_ec_scratch_bytes(int n_jobs);
int rv_ec_tokenize(const rv_ec_job *d_jobs, int n, int xdec, int ydec, int n_tiles, int map_w4,
                   int map_h4, uint8_t *d_map, void *d_scratch, uint32_t *d_offsets,
                   uint32_t *d_tokens, uint32_t token_cap, uint32_t *d_status, void *stream);
/* rv_ec_code_tokens (host): one tile's tokens through WriterBase<
 * WriterEncoder> (symbol_with_update on cdf, which adapts; Writer::bit),
 * then done(): returns the byte count, the bytes go to out if they fit in
 * cap.  cdf: the tile's CDFs (rv_ec_cdf_total() u16, updated in place). */
long rv_ec_code_tokens(const uint32_t *tokens, size_t n, uint16_t *cdf, uint8_t *out, size_t cap);
/* CDFContext::new(quantizer) coefficient CDFs for q context qctx 0..3
 * (src/context.rs:793-850: base_q_idx <= 20, <= 60, <= 120, else 3) and
 * CDFContext::reset_counts (:851-) over them. */
int rv_ec_cdf_total(void);
int rv_ec_default_cdf(int qctx, uint16_t *out);
void rv_ec_reset_counts(uint16_t *cdf);

/* dc_q / ac_q lookups (src/quantize.rs:42-62) on the host: ac = 0 for
 * dc_qlookup*_Q3, 1 for ac_qlookup*_Q3; -1 on bad arguments. */
int rv_q_lookup(int ac, int qindex, int bit_depth);

typedef struct rv_mv {
  int16_t row, col; /* 1/8 pel (MotionVector, src/mc.rs:28-31) */
} rv_mv;
typedef struct rv_fs_job {
  int32_t po_x, po_y;            /* block origin in org (plane coords) */
  int32_t x_lo, x_hi, y_lo, y_hi; /* inclusive candidate window in ref */
  rv_mv pmv[2];
  uint32_t lambda;
  int32_t reserved;
} rv_fs_job;
typedef struct rv_fs_result {
  rv_mv best_mv;
  uint32_t reserved;
  uint64_t cost;
} rv_fs_result;

/* The importance propagation of compute_block_importances
 * (src/api/internal.rs:823-1010) for one (frame, reference) pass, bit-exact
 * in f32.  org: the frame's luma plane; ref: the reference's; d_mvs,
 * d_intra_costs, d_importances: the frame's [ceil(h / 8)][ceil(w / 8)]
 * lookahead MVs (lookahead_mvs sampled at [2y][2x]), intra costs
 * (rv_lookahead_intra_costs) and block importances; n_unique: the number of
 * distinct references of the frame (1..3).  Every block adds
 * amount * overlap fraction to the four blocks of d_ref_importances its
 * MV-displaced area overlaps, in the reference's order (source raster
 * order; top-left, top-right, bottom-left, bottom-right), so the float sums
 * round exactly as the reference's.  A block whose 8x8 reference area
 * leaves the allocation (where the reference's region panics) contributes
 * nothing.  d_scratch: device memory of rv_propagate_importances_scratch()
 * bytes. */
size_t rv_propagate_importances_scratch(int w_imp, int h_imp);
int rv_propagate_importances(const rv_plane *org, const rv_plane *ref, const rv_mv *d_mvs,
                             const uint32_t *d_intra_costs, const float *d_importances,
                             int n_unique, float *d_ref_importances, void *d_scratch,
                             size_t scratch_bytes, void *stream);
/* full_search (src/me.rs:943-990): every candidate (x, y), y outer,
 * x inner, step `step`: cost = 256 * SAD + rate * lambda,
 * rate = min(rate(mv - pmv0), rate(mv - pmv1) + 1) (get_mv_rate,
 * src/me.rs:1006-1021); strict-< argmin in raster order. */
int rv_full_search_batch(const rv_plane *org, const rv_plane *ref,
                         const rv_fs_job *d_jobs, int n, int blk_w,
                         int blk_h, int step, int allow_hp,
                         rv_fs_result *d_out, void *stream);

/* Paired box sums of a plane (bit depth <= 10, so every sum fits 16
 * bits; a u16 plane must state bit_depth 9 or 10, else RV_EINVAL), for the successive-elimination search below.  d_box (16-byte
 * aligned) holds two tables with the plane's geometry, n = stride *
 * alloc_height u32 each: entry (ax, ay) of the allocation in [0, n) is
 * S48(ax, ay) | S48(ax + 8, ay) << 16, in [n, 2n) S4(ax, ay) | S4(ax + 4, ay)
 * << 16; S48 / S4 = the sum of the 4-tall x 8-wide / 4x4 pixels whose
 * top-left corner is there (0 where that block would leave the allocation).  A reference frame needs
 * them once (rav1e searches each input_qres as a reference for several
 * frames). */
int rv_plane_box_sums(const rv_plane *p, uint32_t *d_box, void *stream);

/* rv_full_search_batch for 16x16 blocks, step 1 (estimate_motion_ss4's
 * quarter-resolution search, src/me.rs:1023-1075) with exact successive
 * elimination: SAD >= sum over the eight 4x8 blocks (and over the sixteen
 * 4x4 blocks) of |S_org - S_ref|, so every candidate whose lower bound
 * exceeds an achieved cost is skipped.  Results are identical to
 * rv_full_search_batch (same cost, same first raster minimum).
 * d_ref_box = rv_plane_box_sums of ref. */
int rv_full_search_sea_batch(const rv_plane *org, const rv_plane *ref,
                             const uint32_t *d_ref_box, const rv_fs_job *d_jobs,
                             int n, int allow_hp, rv_fs_result *d_out,
                             void *stream);

/* diamond_me_search (src/me.rs:693-785) with get_best_predictor
 * (:655-691), get_mv_rd_cost (:787-838), compute_mv_rd_cost (:840-856):
 * one persistent workgroup per job runs the whole data-dependent search.
 * Full-pel (subpixel = 0): radius 16 -> 8 (1/8 pel units), candidates are
 * the reference region at po + mv / 8.  Sub-pel (subpixel = 1): radius
 * 4 -> 2 (1 with allow_hp), candidates are predict_inter (REGULAR 8-tap,
 * src/predict.rs:255-338, PlaneSlice::clamp included) into on-chip memory.
 * Distortion: SAD (use_satd = 0) or SATD; cost = 256 * dist + rate *
 * lambda; candidates outside [mv*_min, mv*_max] cost u64::MAX. */
/* ArrayVec<[MotionVector; 17]>: get_subset_predictors' capacity
 * (src/me.rs:82-88: zero, <= 7 coarse MVs, 3 + 1 of subsets A / B, 5 of
 * subset C) */
#define RV_DS_MAX_PRED 17
/* references of one multi-reference launch (job i: ref[i / n_per_ref]) */
#define RV_MAX_REFS 8
typedef struct rv_ds_job {
  int32_t po_x, po_y;                 /* block origin (plane coords) */
  int32_t mvx_min, mvx_max;           /* get_mv_range, 1/8 pel */
  int32_t mvy_min, mvy_max;
  rv_mv pmv[2];                       /* rate predictors */
  uint32_t lambda;
  int32_t n_pred;                     /* predictors used (<= 17) */
  rv_mv pred[RV_DS_MAX_PRED];         /* search start candidates */
} rv_ds_job;
int rv_diamond_search_batch(const rv_plane *org, const rv_plane *ref,
                            const rv_ds_job *d_jobs, int n, int blk_w,
                            int blk_h, int subpixel, int use_satd,
                            int allow_hp, int bit_depth,
                            rv_fs_result *d_out, void *stream);

/* telescopic_subpel_search (src/me.rs:858-941, the FullSearch sub-pel
 * stage): 3x3 grids around the running best at steps 8, 4, 2 (and 1 with
 * allow_hp), REGULAR 8-tap prediction, SAD or SATD; start[i] = the full-pel
 * (best_mv, lowest_cost) the search refines, out[i] = the result.  Job
 * fields used: po, MV range, pmv, lambda. */
int rv_telescopic_subpel_batch(const rv_plane *org, const rv_plane *ref,
                               const rv_ds_job *d_jobs,
                               const rv_fs_result *d_start, int n, int blk_w,
                               int blk_h, int use_satd, int allow_hp,
                               int bit_depth, rv_fs_result *d_out,
                               void *stream);

/* ---------------------------------------------------------------------
 * Hot-path replay driver (see DESIGN.md "Replay driver"): the per-frame
 * call structure of a speed-10 encode of a stream for the accelerated
 * stages -- motion search, every RDO inter candidate (skip / non-skip),
 * the winners' reconstruction, which becomes the next frames' reference --
 * in the coding order of rav1e's reorder pyramid, frames resident in HBM.
 * One instance encodes one tile group (a rectangle of whole AV1 tiles).
 * ------------------------------------------------------------------- */
typedef struct rv_replay_cfg {
  int32_t width, height;      /* luma, visible */
  int32_t xdec, ydec;         /* chroma subsampling (1,1 = 4:2:0) */
  int32_t bit_depth;          /* 8, 10 or 12 (12: exhaustive full search) */
  int32_t tile_x0, tile_y0;   /* tile group rectangle in 64x64 superblocks */
  int32_t tile_w, tile_h;     /* (a whole frame: 0, 0, 0, 0) */
  int32_t n_refs;             /* reference frames searched per frame: 1 or 2 */
  int32_t tile_w_sb, tile_h_sb; /* uniform AV1 tile size (TilingInfo::
                                 * tile_width_sb / tile_height_sb,
                                 * src/tiling/tiler.rs:49-126); 0 = one tile */
  int32_t n_inputs;           /* input frames resident in HBM; display d
                               * reads input d % n_inputs */
  int32_t flags;              /* RV_REPLAY_* bits, 0 = default */
} rv_replay_cfg;
/* flags: F1 coarse search exhaustively (rv_full_search_batch) instead of
 * by successive elimination over box-sum tables (rv_full_search_sea_batch;
 * same results, the default for bit depth <= 10). */
#define RV_REPLAY_EXHAUSTIVE_FS 4
/* flags: the speed-6 schedule (config D; SpeedSettings::from_preset(6),
 * src/api/config.rs:309-460): every inter frame also searches and scores
 * 32x32, 16x16 and 8x8 blocks (motion_estimation per block, SATD sub-pel),
 * picks the partition top-down (PARTITION_NONE vs PARTITION_SPLIT,
 * rdo_partition_decision, src/rdo.rs:1500-1668; must_split past the frame
 * edge, src/encoder.rs:2392-2470) and commits the leaves.  Needs xdec ==
 * ydec.  Result words: the 64x64 words, then per 32x32 / 16x16 / 8x8 block
 * of the group [(full-pel MV, cost, sub-pel MV, cost) per reference,
 * winner, skip, cost bits, distortion], then one partition mask per
 * superblock (bit 0: 64x64 split, 1 + q: 32x32 quadrant q split, 5 + 4 *
 * row + col: 16x16 split), then the 5 tail words. */
#define RV_REPLAY_SPEED6 8
/* flags: deblock every coded frame before it becomes a reference
 * (deblock_filter_optimize's fast levels + deblock_filter_frame,
 * src/encoder.rs:2789-2793).  With several tile groups the exchange
 * also carries each group's block map (log2 block size and skip per luma
 * 4x4) and every group deblocks the whole frame after the import. */
#define RV_REPLAY_DEBLOCK 16
/* flags (with RV_REPLAY_DEBLOCK, as rav1e always deblocks before CDEF):
 * CDEF every coded frame after deblocking (cdef_filter_frame,
 * src/encoder.rs:2795-2802; enable_cdef at every speed, src/api/config.rs:
 * 421-423) with cdef_bits 0, i.e. every superblock at cdef_index 0 and the
 * level's strengths of FrameInvariants::set_quantizers (src/encoder.rs:
 * 882-941, rv_replay_level_params.cdef_strengths).  Width and height must
 * be multiples of 8. */
#define RV_REPLAY_CDEF 32
/* flags: no intra-mode screening.  By default (speed 10, 4:2:0) every
 * superblock whose inter winner is not skip and that lies inside the frame
 * runs rdo_mode_decision's intra screening and intra RDO (src/rdo.rs:
 * 1008-1152): get_intra_edges of the current reconstruction, the 13
 * RAV1E_INTRA_MODES at TX_64X64 + get_satd, the three modes to try, each
 * with chroma modes [mode, DC_PRED]; an intra winner's result words are
 * [1000 + 16 * luma mode + chroma mode, 0, cost bits, distortion] and its
 * reconstruction and levels replace the inter winner's.  rav1e's tile
 * raster order is reproduced by re-evaluating, round after round, the
 * superblocks whose left / top / top-right / top-left neighbour changed. */
#define RV_REPLAY_NO_INTRA 64
/* flags: code the coefficients of every coded frame (stage F8): the
 * committed transform blocks of each tile in coding order through
 * write_coeffs_lv_map (src/context.rs:3965) -- tokenized on the device,
 * range-coded on a host thread beside the next frames (rv_ec_*) -- with the
 * frame's CDFs from the previous frame of its pyramid level (primary
 * reference LAST3, src/encoder.rs:776-830, 2750-2761) and the biggest
 * tile's CDFs kept (:2824-2833).  xdec == ydec.  With several tile groups
 * each instance codes its own tiles and keeps its own biggest tile's CDFs
 * (the frame's biggest tile in rav1e: exact with one group).
 * rv_replay_entropy_stats reads the result. */
#define RV_REPLAY_ENTROPY 128
/* flags: speed 10 takes the MV stacks of the superblocks' candidates and
 * of their 64x64 search's rate predictors from rav1e's find_mvrefs over the
 * blocks coded before them (src/context.rs:2650-2965) by default, in
 * coding-order rounds (a round re-evaluates the superblocks whose stacks
 * changed, until none does).  This flag substitutes the neighbours'
 * motion-search MVs (every superblock independent, one pass; zero rate
 * predictors): an A/B of the rounds' cost, not rav1e's decisions. */
#define RV_REPLAY_MVREF_STANDIN 256
/* flags (with RV_REPLAY_CDEF): loop restoration of every coded frame, the
 * self-guided filter (rav1e evaluates no Wiener filter): each unit's choice
 * as rdo_loop_decision makes it while the tile is coded (src/rdo.rs:
 * 1726-2120; the unit's input is the reconstruction so far with CDEF index
 * 0, None and the 16 parameter sets solved, filtered and priced with
 * count_lrf_switchable), then lrf_filter_frame after CDEF (src/lrf.rs:
 * 1345-1444, src/encoder.rs:2803-2806).  Units of one superblock in every
 * plane (RestorationState::new at base_q_idx <= 160, every level of the
 * default quantizer).  With tile groups each group decides its own units
 * before the exchange and they travel with its reconstruction (the choices
 * are tile-local).  The symbol prices assume a range coder in its initial
 * state (the replay codes no other symbols). */
#define RV_REPLAY_LRF 512
typedef struct rv_replay_frame_info {
  int32_t display;            /* display index of the coded frame */
  int32_t me_range_scale;     /* 4 >> pyramid level (src/encoder.rs:838) */
  int32_t level;              /* pyramid level */
  int32_t is_key;             /* 1: the key frame (input taken as recon) */
  int32_t ref_display[2];     /* display index of each reference */
  int32_t compound;           /* 1: compound candidates (reference_mode SELECT
                               * with a forward and a backward reference) */
} rv_replay_frame_info;
/* The frame parameters of one pyramid level (FrameInvariants::
 * set_quantizers, src/encoder.rs:865-880): base_q_idx, per-plane dc / ac
 * qindex deltas, lambda (bit-depth scaled), me_lambda = sqrt(lambda),
 * dist_scale per plane.  rav1e_amd/rate.py computes them for a fixed
 * --quantizer (src/rate.rs:546-606, 746-775). */
typedef struct rv_replay_level_params {
  int32_t base_q_idx;
  int32_t dc_delta_q[3];
  int32_t ac_delta_q[3];
  int32_t cdef_strengths;     /* cdef_y_strengths[0] | cdef_uv_strengths[0] << 8
                               * (set_quantizers, src/encoder.rs:882-941) */
  double lambda, me_lambda;
  double dist_scale[3];
} rv_replay_level_params;
typedef struct rv_replay rv_replay;
/* Allocate the device state of one tile group: n_inputs input frames, a
 * 12-frame DPB (reconstruction + input hres / qres + box sums).  NULL on
 * failure (rv_last_error). */
rv_replay *rv_replay_create(const rv_replay_cfg *cfg, void *stream);
void rv_replay_destroy(rv_replay *r);
/* A second instance of `primary`'s tile group that shares its DPB and input
 * frames (device memory owned by `primary`, which must outlive it) and has
 * its own per-frame state, stream (`stream`, NULL = its own) and timing: it
 * codes the pyramid's level-2 frames (display 4g+1, 4g+3), which no later
 * frame references, concurrently with `primary`'s levels 0 / 1.  Level
 * parameters, importances and the loop-filter settings are copied from
 * `primary` at creation.  The caller orders the two streams
 * (rv_replay_stream, rv_stream_wait_event): a level-2 frame of group g
 * after `primary`'s level-1 frame of group g, and `primary`'s level-0 frame
 * of group g + 2 (whose DPB slot is display 4g's) after both level-2 frames
 * of group g. */
rv_replay *rv_replay_create_twin(rv_replay *primary, void *stream);
/* The next rv_replay_frame codes coding-order frame n (>= 1; n = 0 is the key
 * frame): display 4g + {4, 2, 1, 3}[j] for n = 1 + 4g + j. */
int rv_replay_seek(rv_replay *r, long n);
/* The instance's replay stream (a hipStream_t). */
void *rv_replay_stream(rv_replay *r);
/* Set the parameters of pyramid level 0..2 (all three before the first
 * inter frame). */
int rv_replay_set_level_params(rv_replay *r, int level, const rv_replay_level_params *p);
/* Generate input i = synthetic frame t0 + i (integer form;
 * rav1e_amd/replay.py synth_frame is its bit-exact numpy twin) for every
 * input slot, in HBM. */
int rv_replay_synth_inputs(rv_replay *r, int t0);
/* Upload / download input `idx` (planar, tightly packed: Y w*h, then the two
 * chroma planes); the upload pads it. */
int rv_replay_set_input(rv_replay *r, int idx, const void *host_yuv);
int rv_replay_get_input(rv_replay *r, int idx, void *host_yuv);
/* The reconstruction of display frame `display` (one of the last 12). */
int rv_replay_get_recon(rv_replay *r, int display, void *host_yuv);
/* block_importances (f32, w_imp x h_imp = ceil(w/8) x ceil(h/8)) that bias
 * the RDO distortion (compute_distortion_bias, src/rdo.rs:476-508); NULL =
 * all zero (the default). */
int rv_replay_set_importances(rv_replay *r, const float *host, int n);
/* The importance window (rdo_lookahead_frames, src/api/config.rs:158;
 * compute_block_importances, src/api/internal.rs:823-1081): window > 0 runs
 * every frame's lookahead `window` coded frames ahead on a lookahead engine
 * (its own host thread and stream) and biases each frame's RDO with the
 * importances propagated over [n, n + window] (replaces
 * rv_replay_set_importances); limit = the stream's length in coded frames
 * (the window shrinks at its end; 0: unbounded).  The inputs of frame n +
 * window must be in place when frame n is coded.  Before the first frame,
 * on a primary instance replaying the whole frame as one group; a twin
 * (rv_replay_create_twin) created afterwards shares the engine.  0 removes
 * the window.  Replaces the reference's lookahead bookkeeping in
 * ContextInner::compute_lookahead_data / receive_packet
 * (src/api/internal.rs:767-823, 1116). */
int rv_replay_set_imp_window(rv_replay *r, int window, long limit);
/* The inputs of displays 0 .. displays - 1 are in place (rv_replay_input /
 * set) and stay until their frames are coded: the lookahead engine may run
 * every frame they cover as far ahead as its ring allows (W + 1 +
 * kLaSlack = W + 29 frames past the oldest frame still being coded), instead of starting frame
 * n + window only when frame n is asked for.  rav1e computes a frame's
 * lookahead data as soon as the frame arrives (compute_lookahead_data,
 * src/api/internal.rs:767-820).  At most the instance's n_inputs; no
 * effect without a window.  Results are unchanged. */
int rv_replay_set_inputs_ready(rv_replay *r, long displays);
/* Tile groups with an importance window: the propagation reads the whole
 * frame, so every group's engine computes its own blocks' lookahead part of
 * each coded frame (intra costs, lookahead MVs, fractions: 28 bytes per 8x8
 * block) and the parts are all-gathered before the frame's target lists are
 * built -- over RCCL (comm from rv_comm_create: one rank per group) or, for
 * several groups in one process, through an in-process hub.  After
 * rv_replay_set_groups and rv_replay_set_imp_window, before the first frame,
 * on every group's primary instance (exactly one of comm / hub). */
typedef struct rv_la_hub rv_la_hub;
rv_la_hub *rv_la_hub_create(int n_groups);
void rv_la_hub_destroy(rv_la_hub *hub);
int rv_replay_set_la_exchange(rv_replay *r, void *comm, rv_la_hub *hub);
/* The block importances (f32 [h_imp][w_imp]) the last coded frame's RDO
 * used (zero without a window or input). */
int rv_replay_get_importances(rv_replay *r, float *host, int n);
/* Code the next frame of the stream (asynchronous on the replay's stream):
 * the key frame first, then the pyramid's coding order.  info may be NULL. */
int rv_replay_frame(rv_replay *r, rv_replay_frame_info *info);
/* Tile-parallel runs (one instance per rank): every rank's tile-group
 * rectangle (4 x i32 in superblocks per group, rank order), this instance's
 * group, and an RCCL communicator from rv_comm_create (or NULL: the caller
 * all-gathers the packed regions from rv_replay_exchange_buffers' send
 * buffer into its recv buffer, group k at k * bytes_per_group, and calls
 * rv_replay_import after every rv_replay_frame). */
int rv_replay_set_groups(rv_replay *r, int n_groups, const int32_t *rects, int my_group,
                         void *comm);
int rv_replay_exchange_buffers(rv_replay *r, void **send, void **recv, size_t *bytes_per_group);
int rv_replay_import(rv_replay *r);
/* RCCL (over xGMI) for the per-frame reconstruction all-gather: rank 0 gets
 * an id (returns its size), every rank creates the communicator with it. */
int rv_comm_unique_id(uint8_t *out, int cap);
void *rv_comm_create(const uint8_t *id, int nranks, int rank);
void rv_comm_destroy(void *comm);
/* Copy the last coded frame's results to host: per superblock and
 * reference the search results as (mv, cost) pairs -- coarse, the four
 * half-res quadrants, full-pel, sub-pel, the 16 lookahead 16x16 blocks (46
 * words) -- and the RDO winner [candidate, skip, rd cost bits,
 * distortion]; (speed 6: the level words and partition masks); then
 * [levels checksum, group reconstruction sum, importance SATD sum,
 * importance blocks, frame reconstruction sum].
 * Returns the number of u64 written (<= cap). */
int rv_replay_results(rv_replay *r, uint64_t *host_out, int cap);
/* RV_REPLAY_ENTROPY: waits for the host coder to finish every frame coded
 * so far, then out[0..3] = the last frame's coefficient bytes, tiles,
 * FNV-1a 64 of its tiles' bytes in tile order, frames coded; out[4] =
 * coefficient bytes summed over every coded frame (cap >= 5).  Returns the
 * count written, RV_EINVAL without the flag or when a frame's tokens
 * overflowed the buffer. */
int rv_replay_entropy_stats(rv_replay *r, uint64_t *out, int cap);
/* Record the timing events only on frames f with (f / block) % stride == 0
 * (stride 1 = every frame, the default; 0 = never).  Each event record
 * leaves the GPU idle for a few microseconds between kernels, so timed runs
 * instrument a sample: block = the GOP length keeps every me_range_scale
 * equally represented. */
int rv_replay_set_timing(rv_replay *r, int stride, int block);
/* Kernel-time breakdown of the last instrumented frame (HIP events), ms:
 * [0] F0 pyramid + box sums, [1] F1 full search, [2] F2 half-res diamond,
 * [3] FL on the main stream (the fork to the side stream; the whole
 * lookahead with RAV1E_HIP_REPLAY_SERIAL=1), [4] F3 full-pel diamond, [5]
 * F3 sub-pel diamond + the candidate lists (speed 6: + every level's
 * searches), [6] F4 fused single-reference candidate launch (luma: MC +
 * skip distortion + diff + fwd TX_64X64 + quantize + estimate_rate +
 * inverse + add + non-skip distortion; chroma U and V: the same with
 * TX_32X32 and SSE), [7] F4 compound candidates, [8] F4 rd cost + argmin
 * (+ the join with the lookahead), [9] F6 commit, [10] F6b intra-mode
 * screening + intra RDO rounds, [11] F5 importance, [12] F7 loop filters /
 * pad / exchange, [13] the lookahead's own span (FL, on the side stream,
 * overlapping [4]..[7]), [14] the speed-10 frame-edge levels' own span (their
 * searches, candidates and scores on the edge stream, beside [4]..[8]; 0
 * without edge superblocks).  [0] .. [12] tile the frame's span on the replay
 * stream.  Returns the count written (<= 15). */
int rv_replay_stage_times(rv_replay *r, float *ms_out, int cap);
/* Same breakdown summed over the last `last_frames` instrumented frames
 * (<= 64). */
int rv_replay_stage_times_sum(rv_replay *r, int last_frames, float *ms_out,
                              int cap);
/* Kernel probes for the bench's roofline: with on != 0, every F3 sub-pel
 * launch (ds_fast_kernel, 64x64, speed 10: round 0 and the MV-stack rounds)
 * and every F4 candidate-list launch (rdo_quad_list_kernel: round 0's single
 * and compound launches, each round's pair) of an instrumented frame
 * (rv_replay_set_timing) is bracketed by a HIP event pair on the stream it
 * runs on and adds its units to device counters.  (Re)starting drops the
 * sums so far.  rv_replay_kernel_probe: out[0] F3 sub-pel launches, out[1]
 * their summed ms (event pairs), out[2] candidate evaluations, out[3] jobs
 * since the last start, (cap >= 5) out[4] the launches' summed ms on the
 * device clock (first workgroup's start to last workgroup's end,
 * wall_clock64); (cap >= 12) out[5] F4 list launches, out[6] their event
 * ms, out[7] their device-clock ms, out[8] / out[9] single-reference /
 * compound luma candidates, out[10] / out[11] single-reference / compound
 * chroma transform blocks.  Returns the count written; waits for the
 * launches. */
int rv_replay_set_kernel_probe(rv_replay *r, int on);
/* Host-only test hook (no device call): the slots the round ring gives
 * round check q -- out[0] its device count slot, out[1] the slot it zeroes
 * for check q + 1, out[2] its host publication slot -- then out[3] the
 * rounds queued ahead of the host's reads, out[4] / out[5] the ring sizes.
 * Returns 6. */
int rv_round_ring_slots(uint32_t q, int32_t *out, int cap);
/* Host-only test hook: the importance window's reference slots of coded
 * frame m >= 1 (rav1e's distinct DPB slots of fi.ref_frames,
 * src/api/internal.rs:875-882; with 2 references a frame above pyramid
 * level 0 adds LAST3): out[0] = their count, out[1..3] their displays,
 * out[4..6] the propagation order.  Returns 0. */
/* RV_REPLAY_LRF: the last coded frame's loop-restoration units of plane p,
 * (set, xqd0, xqd1) int8 triples in raster order of the superblocks (set -1:
 * RestorationFilter::None); cap >= 3 x superblocks.  Synchronous. */
int rv_replay_lrf_units(rv_replay *r, int plane, int8_t *out, int cap);
int rv_replay_la_refs(long m, int R, int32_t *out);
int rv_replay_kernel_probe(rv_replay *r, double *out, int cap);
/* Diagnostic (RAV1E_HIP_DS_PHASES=1 in the environment): the MV-stack
 * rounds' 64x64 sub-pel searches add their phase times (setup, window +
 * filter + SAD, cost exchange, whole job; iterations, window stagings) on
 * the device clock; this prints the per-job means to stderr and clears them. */
int rv_ds_phase_dump(void);
/* Diagnostic (RAV1E_HIP_RDO_PHASES=1): the MV-stack rounds' F4 items
 * (luma quads per set, chroma triples) add their phase spans; this prints
 * the per-item means to stderr and clears them. */
int rv_rdo_phase_dump(void);
/* Candidate evaluations summed over the last min(frames, 64) coded frames:
 * out[0] F3 full-pel 64x64 diamond, out[1] F3 sub-pel 64x64 diamond, out[2]
 * = the number of frames summed (cap >= 3); with cap >= 5, out[3] / out[4]
 * the F4 single-reference / compound RDO candidates; with cap >= 11, out[5
 * .. 10] those of the 32x32, 16x16 and 8x8 blocks (speed 6); with cap >=
 * 14, out[11] superblocks intra-screened, out[12] intra winners, out[13]
 * intra rounds; with cap >= 17 (speed 10, since creation) out[14] the
 * MV-stack evaluation rounds, out[15] the superblocks they re-evaluated,
 * out[16] the frames this instance coded (a twin codes some of the
 * stream's); with cap >= 18, out[17] the round runs (1 + the MV /
 * intra passes of each frame); with cap >= 20, out[18] the lookahead's
 * EPZS rounds (round 0 included) and out[19] the jobs they re-ran (the
 * engine's, on the primary, with an importance window); with cap >= 21,
 * out[20] the frames whose lookahead those rounds ran (the engine runs up to
 * W frames ahead of the encode).  Returns the count. */
int rv_replay_counters(rv_replay *r, uint64_t *out, int cap);

/* The replay's DPB: reconstructions (and their saved motion fields) live in
 * slot display % rv_replay_dpb_slots().  A frame that reuses a slot must
 * follow every frame that reads the slot's previous occupant (display -
 * slots); instances coding frames concurrently (PipelinedReplay) order
 * themselves by it. */
int rv_replay_dpb_slots(void);

/* ---------------------------------------------------------------------
 * Layer 1: drop-in asm-shaped entry points.  Signatures = the reference's
 * FFI declarations; strides in BYTES (T::to_asm_stride,
 * src/util/mod.rs:185-187).  Host pointers.
 * ------------------------------------------------------------------- */

/* Each calling thread stages its blocks through its own stream, device
 * scratch and pinned buffer, created on first use.  They are never freed
 * from a thread-exit destructor (which may run after the HIP runtime is
 * gone): rv_shims_release() frees the calling thread's context (call it
 * from a worker before it exits); rv_shims_shutdown() frees every thread's
 * context (call it once, while HIP is alive, after all threads have stopped
 * calling the shims).  Unreleased contexts are left to process teardown. */
void rv_shims_release(void);
void rv_shims_shutdown(void);

#define RV_DIST_SIZES(X) \
  X(4, 4) X(4, 8) X(8, 4) X(8, 8) X(8, 16) X(16, 8) X(16, 16) X(16, 32) \
  X(32, 16) X(32, 32) X(32, 64) X(64, 32) X(64, 64) X(64, 128) X(128, 64) \
  X(128, 128) X(4, 16) X(16, 4) X(8, 32) X(32, 8) X(16, 64) X(64, 16)

/* SadFn / SadHBDFn / SatdFn (src/asm/x86/dist.rs:16-32, externs :34-98):
 *   rav1e_sad{W}x{H}_hip, rav1e_sad{W}x{H}_hbd_hip,
 *   rav1e_satd_{W}x{H}_hip, rav1e_satd_{W}x{H}_hbd_hip */
#define RV_DECL_DIST(W, H)                                                   \
  uint32_t rav1e_sad##W##x##H##_hip(const uint8_t *src, ptrdiff_t src_stride, \
                                    const uint8_t *dst, ptrdiff_t dst_stride); \
  uint32_t rav1e_sad##W##x##H##_hbd_hip(const uint16_t *src,                  \
                                        ptrdiff_t src_stride,                 \
                                        const uint16_t *dst,                  \
                                        ptrdiff_t dst_stride);                \
  uint32_t rav1e_satd_##W##x##H##_hip(const uint8_t *src,                     \
                                      ptrdiff_t src_stride,                   \
                                      const uint8_t *dst,                     \
                                      ptrdiff_t dst_stride);                  \
  uint32_t rav1e_satd_##W##x##H##_hbd_hip(const uint16_t *src,                \
                                          ptrdiff_t src_stride,               \
                                          const uint16_t *dst,                \
                                          ptrdiff_t dst_stride);
RV_DIST_SIZES(RV_DECL_DIST)
#undef RV_DECL_DIST

/* PutFn / PutHBDFn / PrepFn / PrepHBDFn / AvgFn / AvgHBDFn
 * (src/asm/x86/mc.rs:17-78; tables :300-439, index mode_x + 4 * mode_y,
 * get_2d_mode_idx :81-83):
 *   rav1e_put_8tap_{mx}_{my}_hip  (u8)   rav1e_put_8tap_{mx}_{my}_16bpc_hip
 *   rav1e_prep_8tap_{mx}_{my}_hip (u8)   rav1e_prep_8tap_{mx}_{my}_16bpc_hip
 *   rav1e_avg_hip / rav1e_avg_16bpc_hip
 * with {mx},{my} in regular, smooth, sharp, bilinear. */
#define RV_FILTER_PAIRS(X)                                                  \
  X(regular, regular, 0, 0) X(smooth, regular, 1, 0)                       \
  X(sharp, regular, 2, 0) X(bilinear, regular, 3, 0)                       \
  X(regular, smooth, 0, 1) X(smooth, smooth, 1, 1) X(sharp, smooth, 2, 1)  \
  X(bilinear, smooth, 3, 1) X(regular, sharp, 0, 2) X(smooth, sharp, 1, 2) \
  X(sharp, sharp, 2, 2) X(bilinear, sharp, 3, 2)                           \
  X(regular, bilinear, 0, 3) X(smooth, bilinear, 1, 3)                     \
  X(sharp, bilinear, 2, 3) X(bilinear, bilinear, 3, 3)

#define RV_DECL_MC(NX, NY, MX, MY)                                            \
  void rav1e_put_8tap_##NX##_##NY##_hip(                                      \
      uint8_t *dst, ptrdiff_t dst_stride, const uint8_t *src,                 \
      ptrdiff_t src_stride, int32_t w, int32_t h, int32_t mx, int32_t my);    \
  void rav1e_put_8tap_##NX##_##NY##_16bpc_hip(                                \
      uint16_t *dst, ptrdiff_t dst_stride, const uint16_t *src,               \
      ptrdiff_t src_stride, int32_t w, int32_t h, int32_t mx, int32_t my,     \
      int32_t bit_depth);                                                     \
  void rav1e_prep_8tap_##NX##_##NY##_hip(int16_t *tmp, const uint8_t *src,    \
                                         ptrdiff_t src_stride, int32_t w,     \
                                         int32_t h, int32_t mx, int32_t my);  \
  void rav1e_prep_8tap_##NX##_##NY##_16bpc_hip(                               \
      int16_t *tmp, const uint16_t *src, ptrdiff_t src_stride, int32_t w,     \
      int32_t h, int32_t mx, int32_t my, int32_t bit_depth);
RV_FILTER_PAIRS(RV_DECL_MC)
#undef RV_DECL_MC

void rav1e_avg_hip(uint8_t *dst, ptrdiff_t dst_stride, const int16_t *tmp1,
                   const int16_t *tmp2, int32_t w, int32_t h);
void rav1e_avg_16bpc_hip(uint16_t *dst, ptrdiff_t dst_stride,
                         const int16_t *tmp1, const int16_t *tmp2, int32_t w,
                         int32_t h, int32_t bit_depth);

/* Transforms.  The reference has no asm/generated forward transform
 * (src/encoder.rs:1166-1168 calls the generic Rust), so the HIP level adds
 * the table FWD_TX[TxSize][TxType]:
 *   void rav1e_fwd_txfm_hip(const int16_t *residual, int32_t *coeffs,
 *                           int32_t tx_size, int32_t tx_type, int32_t bd)
 * and replaces InvTxAddF (build/kernel/gen/tx.rs:1365-1370) with
 *   rav1e_inv_txfm_add_hip(coeffs, dst, byte stride, size, type, bd)
 * which covers every pair the native fallback covers (incl. 64-point).
 * Return 0 or RV_ENOTSUP. */
int rav1e_fwd_txfm_hip(const int16_t *residual, int32_t *coeffs,
                       int32_t tx_size, int32_t tx_type, int32_t bit_depth);
int rav1e_inv_txfm_add_hip(const int32_t *coeffs, void *dst,
                           ptrdiff_t dst_stride, int32_t tx_size,
                           int32_t tx_type, int32_t bit_depth);

/* Dispatch tables in the reference's shape (SAD_FNS / SATD_FNS,
 * src/asm/x86/dist.rs:193-327, indexed [cpu][bsize & 31]; PUT_FNS /
 * PREP_FNS, src/asm/x86/mc.rs:300-439, indexed [cpu][mode_x + 4*mode_y]).
 * Entries for levels other than RV_CPU_HIP are NULL (= "use native").
 * BlockSize order: src/partition.rs:116-140. */
typedef uint32_t (*rv_dist_fn)(const void *src, ptrdiff_t src_stride,
                               const void *dst, ptrdiff_t dst_stride);
rv_dist_fn rv_sad_fn(int cpu_level, int bsize, int hbd);
rv_dist_fn rv_satd_fn(int cpu_level, int bsize, int hbd);
typedef void (*rv_put_fn)(void *dst, ptrdiff_t dst_stride, const void *src,
                          ptrdiff_t src_stride, int32_t w, int32_t h,
                          int32_t mx, int32_t my);
rv_put_fn rv_put_fn_get(int cpu_level, int mode_x, int mode_y);

#ifdef __cplusplus
}
#endif
#endif /* RAV1E_HIP_H */
