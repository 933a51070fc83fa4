"""ctypes binding of the CPU oracle (oracle/), for tests only.

The oracle is the parity checker; nothing in the product imports this.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
# RAV1E_ORACLE_LIB: another build of the same sources (tools/sanitize_oracle.sh
# points it at the ASan + UBSan one)
_LIB = os.environ.get("RAV1E_ORACLE_LIB") or os.path.join(ROOT, "oracle", "build",
                                                           "librav1e_oracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = C.CDLL(_LIB)
        vp, sz, i32 = C.c_void_p, C.c_ssize_t, C.c_int
        L.orc_get_sad.restype = C.c_uint32
        L.orc_get_sad.argtypes = [vp, sz, vp, sz, i32, i32, i32]
        L.orc_get_satd.restype = C.c_uint32
        L.orc_get_satd.argtypes = [vp, sz, vp, sz, i32, i32, i32, i32]
        L.orc_sse_wxh.restype = i32
        L.orc_sse_wxh.argtypes = [vp, sz, vp, sz, i32, i32, i32, i32, i32, vp]
        L.orc_cdef_moments_8x8.argtypes = [vp, sz, vp, sz, i32, vp]
        L.orc_cdef_dist_from_moments.restype = C.c_uint64
        L.orc_cdef_dist_from_moments.argtypes = [vp, i32]
        L.orc_put_8tap.argtypes = [vp, sz, vp, sz] + [i32] * 9
        L.orc_predict_intra.argtypes = [i32, i32, vp, sz, i32, i32, i32, i32, vp]
        L.orc_prep_8tap.argtypes = [vp, vp, sz] + [i32] * 8
        L.orc_mc_avg.argtypes = [vp, sz, vp, vp] + [i32] * 5
        L.orc_fwd_txfm1d.restype = i32
        L.orc_fwd_txfm1d.argtypes = [i32, i32, vp, vp]
        L.orc_inv_txfm1d.restype = i32
        L.orc_inv_txfm1d.argtypes = [i32, i32, vp, vp, i32]
        L.orc_fwd_txfm2d.restype = i32
        L.orc_fwd_txfm2d.argtypes = [vp, vp, i32, i32, i32]
        L.orc_inv_txfm2d_add.restype = i32
        L.orc_inv_txfm2d_add.argtypes = [vp, vp, sz, i32, i32, i32, i32]
        L.orc_diff.argtypes = [vp, vp, sz, vp, sz, i32, i32, i32]
        L.orc_plane_geometry.argtypes = [i32] * 5 + [vp]
        L.orc_plane_pad.argtypes = [vp] + [i32] * 9
        L.orc_downsample.argtypes = [vp, sz, i32, i32, vp, sz, i32]
        L.orc_get_mv_rate.restype = C.c_uint32
        L.orc_divu_pair.restype = i32
        L.orc_divu_pair.argtypes = [i32, vp]
        L.orc_divu_gen.argtypes = [C.c_uint32, vp]
        L.orc_qctx_update.argtypes = [vp] + [i32] * 6
        L.orc_quantize.restype = i32
        L.orc_quantize.argtypes = [vp, vp, vp, i32, i32]
        L.orc_dequantize.argtypes = [i32, vp, vp, i32, i32, i32, i32]
        L.orc_coded_tx_area.restype = i32
        L.orc_estimate_rate.restype = C.c_uint64
        L.orc_lookahead_intra_costs.argtypes = [vp, sz, i32, i32, i32, i32, vp]
        L.orc_propagate_importances.argtypes = [vp, sz, vp, sz, i32, i32, i32, vp, vp, vp, i32,
                                                vp]
        L.orc_estimate_rate.argtypes = [i32, i32, C.c_uint64]
        L.orc_get_log_tx_scale.restype = i32
        L.orc_deblock_plane.argtypes = [vp, sz, i32, i32, i32, i32, i32, i32, i32, vp, vp, i32,
                                        vp]
        L.orc_deblock_fast_level.argtypes = [i32, i32, i32]
        L.orc_deblock_sse_plane.argtypes = [vp, sz, vp, sz] + [i32] * 7 + [vp, vp, i32, vp, vp]
        L.orc_deblock_sse_levels.argtypes = [vp, vp, vp]
        L.orc_cdef_find_dir.restype = i32
        L.orc_cdef_find_dir.argtypes = [vp, sz, vp, i32]
        L.orc_cdef_filter_block.argtypes = [vp, sz, i32, vp, sz] + [i32] * 7
        L.orc_cdef_adjust_strength.restype = i32
        L.orc_cdef_adjust_strength.argtypes = [i32, i32]
        L.orc_cdef_filter_frame.argtypes = [vp, vp, vp, vp] + [i32] * 6 + [vp, i32, vp, vp, vp,
                                                                          i32, vp, vp]
        _lib = L
    return _lib


def ptr(a, offset=0):
    """Pointer to element `offset` (flat, in elements) of a numpy array."""
    return C.c_void_p(int(a.ctypes.data) + int(offset) * a.itemsize)


def hbd_of(a):
    return 1 if a.dtype == np.uint16 else 0


# ---- thin wrappers (arrays are 2-D numpy, regions addressed by (y, x)) ----
def get_sad(org, oy, ox, ref, ry, rx, w, h):
    L = lib()
    return L.orc_get_sad(ptr(org, oy * org.shape[1] + ox), org.shape[1],
                         ptr(ref, ry * ref.shape[1] + rx), ref.shape[1], w, h, hbd_of(org))


def get_satd(org, oy, ox, ref, ry, rx, w, h, emulate_gen=0):
    L = lib()
    return L.orc_get_satd(ptr(org, oy * org.shape[1] + ox), org.shape[1],
                          ptr(ref, ry * ref.shape[1] + rx), ref.shape[1], w, h,
                          hbd_of(org), emulate_gen)


def put_8tap(src, sy, sx, w, h, col_frac, row_frac, mode_x=0, mode_y=0, bd=8, emulate_gen=0):
    dst = np.zeros((h, w), dtype=src.dtype)
    lib().orc_put_8tap(ptr(dst), w, ptr(src, sy * src.shape[1] + sx), src.shape[1], w, h,
                       col_frac, row_frac, mode_x, mode_y, bd, hbd_of(src), emulate_gen)
    return dst


def predict_intra(mode, variant, w, h, edge, bd=8):
    """orc_predict_intra: PredictionMode::predict_intra (no CfL) of a w x h
    block from a 257-pixel edge_buf."""
    edge = np.ascontiguousarray(edge, dtype=np.uint16 if bd > 8 else np.uint8)
    dst = np.zeros((h, w), dtype=edge.dtype)
    lib().orc_predict_intra(mode, variant, ptr(dst), w, w, h, bd, 1 if bd > 8 else 0, ptr(edge))
    return dst


def deblock_plane(full, yo, xo, width, height, xdec, ydec, pli, lg, skip, levels, bd=8):
    """orc_deblock_plane on a full (padded) plane array, visible origin (xo,
    yo), in place."""
    lg = np.ascontiguousarray(lg, dtype=np.uint8)
    skip = np.ascontiguousarray(skip, dtype=np.uint8)
    lv = np.ascontiguousarray(np.asarray(levels, dtype=np.uint8))
    lib().orc_deblock_plane(ptr(full, yo * full.shape[1] + xo), full.shape[1], hbd_of(full), bd,
                            width, height, xdec, ydec, pli, ptr(lg), ptr(skip), lg.shape[1],
                            ptr(lv))
    return full


def deblock_sse_plane(rec, src, width, height, xdec, ydec, pli, lg, skip, bd=8):
    """orc_deblock_sse_plane on visible planes rec / src (same shape): the
    (vertical, horizontal) tallies, 65 int64 each."""
    lg = np.ascontiguousarray(lg, dtype=np.uint8)
    skip = np.ascontiguousarray(skip, dtype=np.uint8)
    rec = np.ascontiguousarray(rec)
    src = np.ascontiguousarray(src, dtype=rec.dtype)
    v = np.zeros(65, np.int64)
    h = np.zeros(65, np.int64)
    lib().orc_deblock_sse_plane(ptr(rec), rec.shape[1], ptr(src), src.shape[1], hbd_of(rec), bd,
                                width, height, xdec, ydec, pli, ptr(lg), ptr(skip), lg.shape[1],
                                ptr(v), ptr(h))
    return v, h


def deblock_sse_levels(v, h):
    """orc_deblock_sse_levels: levels [Y vertical, Y horizontal, U, V] from
    the three planes' tallies (3 x 65 each)."""
    v = np.ascontiguousarray(v, dtype=np.int64)
    h = np.ascontiguousarray(h, dtype=np.int64)
    lv = np.zeros(4, np.uint8)
    lib().orc_deblock_sse_levels(ptr(v), ptr(h), ptr(lv))
    return [int(x) for x in lv]


def deblock_fast_level(ac_q, bd, is_key=False):
    return int(lib().orc_deblock_fast_level(int(ac_q), bd, 1 if is_key else 0))


def cdef_find_dir(img, coeff_shift=0):
    """orc_cdef_find_dir of an 8x8 u16 block (the padded copy's samples):
    (dir, var)."""
    img = np.ascontiguousarray(img, dtype=np.uint16)
    var = np.zeros(1, np.int32)
    d = lib().orc_cdef_find_dir(ptr(img), img.shape[1], ptr(var), coeff_shift)
    return int(d), int(var[0])


def cdef_adjust_strength(strength, var):
    return int(lib().orc_cdef_adjust_strength(int(strength), int(var)))


def cdef_filter_frame(planes, width, height, xdec, ydec, skip, cdef_index, y_str, uv_str,
                      damping=3, bd=8):
    """orc_cdef_filter_frame on three visible planes (numpy); returns the
    filtered planes and the per-8x8 (dir, var)."""
    ins = [np.ascontiguousarray(p) for p in planes]
    outs = [np.zeros_like(p) for p in ins]
    skip = np.ascontiguousarray(skip, dtype=np.uint8)
    cdef_index = np.ascontiguousarray(cdef_index, dtype=np.uint8)
    ys = np.ascontiguousarray(np.asarray(y_str, dtype=np.uint8))
    us = np.ascontiguousarray(np.asarray(uv_str, dtype=np.uint8))
    cols8, rows8 = (width + 7) // 8, (height + 7) // 8
    dirs = np.zeros((rows8, cols8), np.uint8)
    vars_ = np.zeros((rows8, cols8), np.int32)
    ip = (C.c_void_p * 3)(*[p.ctypes.data for p in ins])
    op = (C.c_void_p * 3)(*[p.ctypes.data for p in outs])
    ist = (C.c_ssize_t * 3)(*[p.shape[1] for p in ins])
    ost = (C.c_ssize_t * 3)(*[p.shape[1] for p in outs])
    lib().orc_cdef_filter_frame(ip, ist, op, ost, hbd_of(ins[0]), bd, width, height, xdec, ydec,
                                ptr(skip), skip.shape[1], ptr(cdef_index), ptr(ys), ptr(us),
                                damping, ptr(dirs), ptr(vars_))
    return outs, dirs, vars_


def prep_8tap(src, sy, sx, w, h, col_frac, row_frac, mode_x=0, mode_y=0, bd=8):
    tmp = np.zeros((h, w), dtype=np.int16)
    lib().orc_prep_8tap(ptr(tmp), ptr(src, sy * src.shape[1] + sx), src.shape[1], w, h,
                        col_frac, row_frac, mode_x, mode_y, bd, hbd_of(src))
    return tmp


def mc_avg(t1, t2, bd=8, hbd=0, emulate_gen=0):
    h, w = t1.shape
    dst = np.zeros((h, w), dtype=np.uint16 if hbd else np.uint8)
    lib().orc_mc_avg(ptr(dst), w, ptr(np.ascontiguousarray(t1)), ptr(np.ascontiguousarray(t2)),
                     w, h, bd, hbd, emulate_gen)
    return dst


def fwd_txfm1d(kind, vec):
    v = np.ascontiguousarray(vec, dtype=np.int32)
    out = np.zeros_like(v)
    rc = lib().orc_fwd_txfm1d(kind, v.size, ptr(v), ptr(out))
    return None if rc else out


def inv_txfm1d(kind, vec, rng):
    v = np.ascontiguousarray(vec, dtype=np.int32)
    out = np.zeros_like(v)
    rc = lib().orc_inv_txfm1d(kind, v.size, ptr(v), ptr(out), rng)
    return None if rc else out


def fwd_txfm2d(residual, tx_size, tx_type, bd):
    r = np.ascontiguousarray(residual, dtype=np.int16).ravel()
    out = np.zeros(r.size, dtype=np.int32)
    rc = lib().orc_fwd_txfm2d(ptr(r), ptr(out), tx_size, tx_type, bd)
    return None if rc else out


def divu_gen(d):
    out = np.zeros(3, dtype=np.uint32)
    lib().orc_divu_gen(d, ptr(out))
    return out


def divu_pair(x, dgen):
    return lib().orc_divu_pair(int(x), ptr(dgen))


QCTX_BYTES = 64  # >= sizeof(orc_qctx)


def quantize(coeffs, tx_size, tx_type, qindex, bd, is_intra=False, dc_delta_q=0,
             ac_delta_q=0):
    """QuantizationContext::update + quantize (src/quantize.rs:205-316):
    (qcoeffs[coded_tx_area], eob)."""
    ctx = np.zeros(QCTX_BYTES, dtype=np.uint8)
    lib().orc_qctx_update(ptr(ctx), qindex, tx_size, int(is_intra), bd, dc_delta_q, ac_delta_q)
    c = np.ascontiguousarray(coeffs, dtype=np.int32).ravel()
    q = np.zeros(lib().orc_coded_tx_area(tx_size), dtype=np.int32)
    eob = lib().orc_quantize(ptr(ctx), ptr(c), ptr(q), tx_size, tx_type)
    return q, eob


def dequantize(qcoeffs, tx_size, qindex, bd, dc_delta_q=0, ac_delta_q=0):
    """dequantize (src/quantize.rs:319-333)"""
    q = np.ascontiguousarray(qcoeffs, dtype=np.int32).ravel()
    r = np.zeros(q.size, dtype=np.int32)
    lib().orc_dequantize(qindex, ptr(q), ptr(r), tx_size, bd, dc_delta_q, ac_delta_q)
    return r


def lookahead_intra_costs(full, yo, xo, w, h, bd):
    """compute_lookahead_intra_costs of the plane whose pixel (0, 0) is
    full[yo, xo] (the padded allocation): u32 [ceil(h / 8), ceil(w / 8)]."""
    nbx, nby = (w + 7) // 8, (h + 7) // 8
    out = np.zeros(nbx * nby, dtype=np.uint32)
    lib().orc_lookahead_intra_costs(ptr(full, yo * full.shape[1] + xo), full.shape[1], w, h,
                                    hbd_of(full), bd, ptr(out))
    return out.reshape(nby, nbx)


def propagate_importances(org_full, oyo, oxo, ref_full, ryo, rxo, w, h, mvs, intra_costs,
                          importances, n_unique, ref_importances):
    """compute_block_importances' propagation, one (frame, reference) pass:
    org_full / ref_full are padded allocations whose pixel (0, 0) is at
    [yo, xo]; mvs is an int16 [h_imp, w_imp, 2] (row, col) array.  Returns
    the reference's importances after the pass."""
    nbx, nby = (w + 7) // 8, (h + 7) // 8
    mv = np.ascontiguousarray(mvs, dtype=np.int16).reshape(nby * nbx * 2)
    ic = np.ascontiguousarray(intra_costs, dtype=np.uint32).ravel()
    imp = np.ascontiguousarray(importances, dtype=np.float32).ravel()
    out = np.array(ref_importances, dtype=np.float32).ravel().copy()
    lib().orc_propagate_importances(ptr(org_full, oyo * org_full.shape[1] + oxo),
                                    org_full.shape[1],
                                    ptr(ref_full, ryo * ref_full.shape[1] + rxo),
                                    ref_full.shape[1], nbx, nby, hbd_of(org_full), ptr(mv),
                                    ptr(ic), ptr(imp), int(n_unique), ptr(out))
    return out.reshape(nby, nbx)


def estimate_rate(qindex, tx_size, fast_distortion):
    """estimate_rate (src/rdo.rs:204-216)"""
    return int(lib().orc_estimate_rate(int(qindex), int(tx_size), int(fast_distortion)))


def inv_txfm2d_add(coeffs, dst, tx_size, tx_type, bd):
    c = np.ascontiguousarray(coeffs, dtype=np.int32).ravel()
    d = np.array(dst, copy=True)
    rc = lib().orc_inv_txfm2d_add(ptr(c), ptr(d), d.shape[1], tx_size, tx_type, bd, hbd_of(d))
    return None if rc else d


def sse_wxh(a, b, w, h, xdec=0, ydec=0):
    out = np.zeros(w * h, dtype=np.uint64)  # >= sub-block count
    n = lib().orc_sse_wxh(ptr(a), a.shape[1], ptr(b), b.shape[1], w, h, xdec, ydec,
                          hbd_of(a), ptr(out))
    return out[:n]


def cdef_moments(a, b):
    out = np.zeros(5, dtype=np.int64)
    lib().orc_cdef_moments_8x8(ptr(a), a.shape[1], ptr(b), b.shape[1], hbd_of(a), ptr(out))
    return out


def cdef_dist(moments, bd):
    m = np.ascontiguousarray(moments, dtype=np.int64)
    return lib().orc_cdef_dist_from_moments(ptr(m), bd)


def plane_geometry(width, height, xpad, ypad, hbd):
    out = np.zeros(4, dtype=np.int32)
    lib().orc_plane_geometry(width, height, xpad, ypad, hbd, ptr(out))
    return tuple(int(x) for x in out)  # stride, alloc_height, xorigin, yorigin


TX_W_LOG2 = [2, 3, 4, 5, 6, 2, 3, 3, 4, 4, 5, 5, 6, 2, 4, 3, 5, 4, 6]
TX_H_LOG2 = [2, 3, 4, 5, 6, 3, 2, 4, 3, 5, 4, 6, 5, 4, 2, 5, 3, 6, 4]
TX_NAMES = ["4x4", "8x8", "16x16", "32x32", "64x64", "4x8", "8x4", "8x16", "16x8",
            "16x32", "32x16", "32x64", "64x32", "4x16", "16x4", "8x32", "32x8",
            "16x64", "64x16"]
TX_TYPES = ["DCT_DCT", "ADST_DCT", "DCT_ADST", "ADST_ADST", "FLIPADST_DCT",
            "DCT_FLIPADST", "FLIPADST_FLIPADST", "ADST_FLIPADST", "FLIPADST_ADST",
            "IDTX", "V_DCT", "H_DCT", "V_ADST", "H_ADST", "V_FLIPADST", "H_FLIPADST"]
BLOCKS = ["4x4", "4x8", "8x4", "8x8", "8x16", "16x8", "16x16", "16x32", "32x16",
          "32x32", "32x64", "64x32", "64x64", "64x128", "128x64", "128x128",
          "4x16", "16x4", "8x32", "32x8", "16x64", "64x16"]


def block_wh(name):
    w, h = name.split("x")
    return int(w), int(h)


def dist_kat_planes(dtype):
    """setup_planes of src/dist.rs:342-375, in the reference's exact layout."""
    hbd = 1 if dtype == np.uint16 else 0
    planes = []
    for pad, pattern in ((128 + 8, "sum"), (2 * 128 + 8, "diff")):
        stride, alloc_h, xorigin, yorigin = plane_geometry(640, 480, pad, pad, hbd)
        xpad_off = (xorigin - pad) - 8
        i = np.arange(alloc_h)[:, None]
        j = np.arange(stride)[None, :]
        v = ((j + i) - xpad_off) & 255 if pattern == "sum" else (j - i - xpad_off) & 255
        planes.append((v.astype(dtype), xorigin, yorigin))
    return planes


class _Mv(C.Structure):
    _fields_ = [("row", C.c_int16), ("col", C.c_int16)]


def full_search(org_full, ref_full, xorigin, yorigin, job, blk_w, blk_h, step, allow_hp):
    """orc_full_search on full padded arrays; job = one FS_JOB record
    (coordinates relative to the plane origin).  Returns ((row, col), cost)."""
    L = lib()
    L.orc_full_search.argtypes = [C.c_void_p, C.c_ssize_t, C.c_void_p, C.c_ssize_t, C.c_int,
                                  C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                  C.c_int, C.c_int, C.c_int, C.c_uint32, _Mv, _Mv, C.c_int,
                                  C.POINTER(_Mv), C.POINTER(C.c_uint64)]
    o = ptr(org_full, yorigin * org_full.shape[1] + xorigin)
    r = ptr(ref_full, yorigin * ref_full.shape[1] + xorigin)
    best = _Mv(0, 0)
    cost = C.c_uint64(2 ** 64 - 1)
    L.orc_full_search(o, org_full.shape[1], r, ref_full.shape[1], hbd_of(org_full),
                      int(job["po_x"]), int(job["po_y"]), int(job["x_lo"]), int(job["x_hi"]),
                      int(job["y_lo"]), int(job["y_hi"]), blk_w, blk_h, step,
                      int(job["lambda_"]), _Mv(int(job["pmv0_row"]), int(job["pmv0_col"])),
                      _Mv(int(job["pmv1_row"]), int(job["pmv1_col"])), allow_hp,
                      C.byref(best), C.byref(cost))
    return (best.row, best.col), cost.value


class _DsCtx(C.Structure):
    _fields_ = [("org", C.c_void_p), ("org_stride", C.c_ssize_t), ("ref", C.c_void_p),
                ("ref_stride", C.c_ssize_t)] + [(f, C.c_int) for f in (
                    "ref_width", "ref_height", "ref_xorigin", "ref_yorigin", "ref_xdec",
                    "ref_ydec", "hbd", "bit_depth", "po_x", "po_y", "w", "h", "mvx_min",
                    "mvx_max", "mvy_min", "mvy_max")] + [
                ("pmv", _Mv * 2), ("lambda_", C.c_uint32), ("subpel", C.c_int),
                ("satd", C.c_int), ("allow_hp", C.c_int)]


def _ds_ctx(org_full, ref_full, xorigin, yorigin, width, height, job, w, h, subpel, satd,
            allow_hp, bd):
    c = _DsCtx()
    c.org = ptr(org_full, yorigin * org_full.shape[1] + xorigin)
    c.org_stride = org_full.shape[1]
    c.ref = ptr(ref_full, yorigin * ref_full.shape[1] + xorigin)
    c.ref_stride = ref_full.shape[1]
    c.ref_width, c.ref_height, c.ref_xorigin, c.ref_yorigin = width, height, xorigin, yorigin
    c.ref_xdec = c.ref_ydec = 0
    c.hbd, c.bit_depth = hbd_of(org_full), bd
    c.po_x, c.po_y, c.w, c.h = int(job["po_x"]), int(job["po_y"]), w, h
    c.mvx_min, c.mvx_max = int(job["mvx_min"]), int(job["mvx_max"])
    c.mvy_min, c.mvy_max = int(job["mvy_min"]), int(job["mvy_max"])
    c.pmv[0] = _Mv(int(job["pmv0_row"]), int(job["pmv0_col"]))
    c.pmv[1] = _Mv(int(job["pmv1_row"]), int(job["pmv1_col"]))
    c.lambda_ = int(job["lambda_"])
    c.subpel, c.satd, c.allow_hp = int(subpel), int(satd), int(allow_hp)
    return c


def diamond_search(org_full, ref_full, xorigin, yorigin, width, height, job, w, h, subpel,
                   satd, allow_hp, bd):
    """orc_diamond_search for one DS_JOB record on full padded arrays (both
    planes share the geometry).  Returns ((row, col), cost)."""
    L = lib()
    L.orc_diamond_search.argtypes = [C.POINTER(_DsCtx), C.POINTER(_Mv), C.c_int,
                                     C.POINTER(_Mv), C.POINTER(C.c_uint64)]
    c = _ds_ctx(org_full, ref_full, xorigin, yorigin, width, height, job, w, h, subpel, satd,
                allow_hp, bd)
    n = int(job["n_pred"])
    preds = (_Mv * max(1, n))(*[_Mv(int(job["pred"][k][0]), int(job["pred"][k][1]))
                                for k in range(n)])
    best = _Mv(0, 0)
    cost = C.c_uint64(0)
    L.orc_diamond_search(C.byref(c), preds, n, C.byref(best), C.byref(cost))
    return (best.row, best.col), cost.value


def telescopic_subpel(org_full, ref_full, xorigin, yorigin, width, height, job, w, h, satd,
                      allow_hp, bd, start_mv, start_cost):
    """orc_telescopic_subpel for one DS_JOB record; returns ((row, col), cost)."""
    L = lib()
    L.orc_telescopic_subpel.argtypes = [C.POINTER(_DsCtx), C.POINTER(_Mv), C.POINTER(C.c_uint64)]
    c = _ds_ctx(org_full, ref_full, xorigin, yorigin, width, height, job, w, h, True, satd,
                allow_hp, bd)
    best = _Mv(int(start_mv[0]), int(start_mv[1]))
    cost = C.c_uint64(int(start_cost))
    L.orc_telescopic_subpel(C.byref(c), C.byref(best), C.byref(cost))
    return (best.row, best.col), cost.value


def tx_dist(coeffs, rcoeffs, tx_w, tx_h):
    L = lib()
    L.orc_tx_dist.restype = C.c_uint64
    L.orc_tx_dist.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int]
    coeffs = np.ascontiguousarray(coeffs, dtype=np.int32)
    rcoeffs = np.ascontiguousarray(rcoeffs, dtype=np.int32)
    return int(L.orc_tx_dist(coeffs.ctypes.data, rcoeffs.ctypes.data, rcoeffs.size, tx_w, tx_h))


_V4_FLAGS = {"avx512f", "avx512bw", "avx512cd", "avx512dq", "avx512vl"}
_baseline = None


def baseline_lib():
    """The oracle build for the bench's CPU baseline: x86-64-v4 (AVX-512)
    when this host has it, else the x86-64-v3 (AVX2) build the tests use --
    "-march=native" resolved on the host that runs the bench (the GPU box's
    CPU is not this container's).  Returns (ctypes lib, ISA label)."""
    global _baseline
    if _baseline is None:
        flags = set()
        try:
            with open("/proc/cpuinfo") as f:
                for line in f:
                    if line.startswith("flags"):
                        flags = set(line.split(":", 1)[1].split())
                        break
        except OSError:
            pass
        v4 = os.path.join(ROOT, "oracle", "build", "librav1e_oracle_v4.so")
        if _V4_FLAGS <= flags and os.path.exists(v4):
            _baseline = (C.CDLL(v4), "x86-64-v4")
        else:
            _baseline = (lib(), "x86-64-v3")
    return _baseline


def cpu_share() -> int:
    """Host threads this process may use: its affinity mask, capped at 16
    (the GPU box's per-GPU CPU share; os.cpu_count() there reports the whole
    machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    return max(1, min(16, n))


class OrcFrameInfo(C.Structure):
    _fields_ = [("display", C.c_int32), ("me_range_scale", C.c_int32), ("level", C.c_int32),
                ("is_key", C.c_int32), ("ref_display", C.c_int32 * 2), ("compound", C.c_int32)]


class CpuReplay:
    """orc_replay_* (oracle/orc_replay.c): the replay schedule on the CPU,
    the same API as rav1e_amd.replay.HipReplay.  `L` selects the oracle
    build (default: the tests' build; the bench's baseline passes
    baseline_lib()[0])."""

    def __init__(self, width, height, xdec=1, ydec=1, bit_depth=8, n_refs=2, group=None,
                 tile_size=(0, 0), n_inputs=8, threads=1, L=None, quantizer=100, speed=10,
                 deblock=False, cdef=False, intra=True, entropy=False, mvref_standin=False,
                 imp_window=0, imp_limit=0, lrf=False):
        from rav1e_amd import rate as RT
        L = L or lib()
        self.L = L
        L.orc_replay_create.restype = C.c_void_p
        L.orc_replay_create.argtypes = [C.c_int] * 14
        L.orc_replay_destroy.argtypes = [C.c_void_p]
        L.orc_replay_set_input.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        L.orc_replay_get_recon.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
        L.orc_replay_set_importances.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        L.orc_replay_frame.argtypes = [C.c_void_p, C.POINTER(OrcFrameInfo), C.c_int, C.c_int]
        L.orc_replay_results.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        L.orc_replay_xcopy.restype = C.c_int64
        L.orc_replay_xcopy.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        L.orc_replay_pad_recon.argtypes = [C.c_void_p]
        I3, D3 = C.c_int32 * 3, C.c_double * 3
        L.orc_replay_set_level_params.argtypes = [C.c_void_p, C.c_int, C.c_int, I3, I3,
                                                  C.c_double, C.c_double, D3]
        self.group = tuple(group) if group else None
        tx0, ty0, tw, th = group or (0, 0, 0, 0)
        self.h = L.orc_replay_create(width, height, xdec, ydec, bit_depth, tx0, ty0, tw, th,
                                     tile_size[0], tile_size[1], n_refs, n_inputs, threads)
        assert self.h, "orc_replay_create failed"
        from rav1e_amd.replay import result_words
        L.orc_replay_set_speed.argtypes = [C.c_void_p, C.c_int]
        assert L.orc_replay_set_speed(self.h, speed) == 0, "orc_replay_set_speed"
        L.orc_replay_set_deblock.argtypes = [C.c_void_p, C.c_int]
        assert L.orc_replay_set_deblock(self.h, 1 if deblock else 0) == 0, "orc_replay_set_deblock"
        self.speed = speed
        L.orc_replay_set_mvref_standin.argtypes = [C.c_void_p, C.c_int]
        assert L.orc_replay_set_mvref_standin(self.h, 1 if mvref_standin else 0) == 0
        # intra-mode screening of non-skip superblocks: speed 10, 4:2:0 (the
        # replay's default; RV_REPLAY_NO_INTRA turns it off on the GPU)
        self.intra = bool(intra and speed == 10 and xdec == 1 and ydec == 1)
        L.orc_replay_set_intra.argtypes = [C.c_void_p, C.c_int]
        assert L.orc_replay_set_intra(self.h, 1 if self.intra else 0) == 0
        L.orc_replay_intra_stats.argtypes = [C.c_void_p, C.c_void_p]
        L.orc_replay_set_entropy.argtypes = [C.c_void_p, C.c_int]
        L.orc_replay_entropy_stats.argtypes = [C.c_void_p, C.c_void_p]
        self.entropy = bool(entropy)
        assert L.orc_replay_set_entropy(self.h, 1 if entropy else 0) == 0, "orc_replay_set_entropy"
        self.n_words = result_words(width, height, n_refs, tw, th, tx0, ty0, speed, xdec, ydec)
        self.geom = (width, height, xdec, ydec, bit_depth)
        self.levels = RT.level_params(quantizer, bit_depth)
        L.orc_replay_set_cdef.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int]
        for lv, d in enumerate(self.levels):
            if cdef:
                assert L.orc_replay_set_cdef(self.h, lv, d["cdef_y"], d["cdef_uv"]) == 0
            assert L.orc_replay_set_level_params(
                self.h, lv, d["base_q_idx"], I3(*d["dc_delta_q"]), I3(*d["ac_delta_q"]),
                d["lambda"], d["me_lambda"], D3(*d["dist_scale"])) == 0
        L.orc_replay_set_imp_window.argtypes = [C.c_void_p, C.c_int, C.c_long]
        assert L.orc_replay_set_imp_window(self.h, imp_window, imp_limit) == 0, \
            "orc_replay_set_imp_window"
        L.orc_replay_set_lrf.argtypes = [C.c_void_p, C.c_int]
        assert L.orc_replay_set_lrf(self.h, 1 if lrf else 0) == 0, "orc_replay_set_lrf"
        self.imp_window = imp_window
        self.imp_shape = ((height + 7) // 8, (width + 7) // 8)

    def lrf_units(self, plane, n):
        """The last frame's loop-restoration units of plane p: (set, xqd0,
        xqd1) per unit, set -1 = None."""
        out = np.zeros(3 * n, np.int8)
        self.L.orc_replay_lrf_units.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int]
        self.L.orc_replay_lrf_units(self.h, plane, out.ctypes.data, out.size)
        return out.reshape(n, 3)

    def importances(self):
        """The block importances the last coded frame's RDO used
        ([h_imp][w_imp] f32; the window's, or the input's)."""
        out = np.zeros(self.imp_shape, np.float32)
        self.L.orc_replay_get_importances.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        assert self.L.orc_replay_get_importances(self.h, out.ctypes.data, out.size) == 0
        return out

    def set_input(self, idx, yuv):
        yuv = np.ascontiguousarray(yuv)
        assert self.L.orc_replay_set_input(self.h, idx, yuv.ctypes.data) == 0

    def deblock_levels(self):
        """deblock_filter_optimize's levels of the last deblocked frame."""
        out = np.zeros(4, np.uint8)
        self.L.orc_replay_deblock_levels.argtypes = [C.c_void_p, C.c_void_p]
        self.L.orc_replay_deblock_levels(self.h, out.ctypes.data)
        return [int(v) for v in out]

    def intra_stats(self):
        """(superblocks screened, intra winners) of the last coded frame."""
        out = np.zeros(2, np.uint64)
        self.L.orc_replay_intra_stats(self.h, out.ctypes.data)
        return int(out[0]), int(out[1])

    def entropy_stats(self):
        """[bytes, tiles, FNV-1a of the tiles' bytes, frames coded] of the
        last frame's coefficient coding."""
        out = np.zeros(4, np.uint64)
        self.L.orc_replay_entropy_stats(self.h, out.ctypes.data)
        return [int(v) for v in out]

    def set_importances(self, imp):
        if imp is None:
            assert self.L.orc_replay_set_importances(self.h, None, 0) == 0
            return
        imp = np.ascontiguousarray(imp, dtype=np.float32)
        assert self.L.orc_replay_set_importances(self.h, imp.ctypes.data, imp.size) == 0

    # ---- a tile group's importance window (orc_replay_la_due / _group /
    # _import): each group computes its own blocks' lookahead part, the
    # caller exchanges the parts before frame()
    def la_due(self):
        """(next coded frame whose part is due, the last one the next frame
        needs, the part's bytes); None without a group window"""
        out = (C.c_long * 3)()
        self.L.orc_replay_la_due.argtypes = [C.c_void_p, C.c_void_p]
        if self.L.orc_replay_la_due(self.h, out) != 0:
            return None
        return int(out[0]), int(out[1]), int(out[2])

    def la_group(self, m, nbytes) -> np.ndarray:
        out = np.zeros(nbytes, np.uint8)
        self.L.orc_replay_la_group.argtypes = [C.c_void_p, C.c_long, C.c_void_p]
        assert self.L.orc_replay_la_group(self.h, m, out.ctypes.data) == 0, "orc_replay_la_group"
        return out

    def la_import(self, m, rect, buf):
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        self.L.orc_replay_la_import.argtypes = [C.c_void_p, C.c_long] + [C.c_int] * 4 + [C.c_void_p]
        assert self.L.orc_replay_la_import(self.h, m, *[int(v) for v in rect],
                                           buf.ctypes.data) == 0, "orc_replay_la_import"

    def la_part_bytes(self, rect) -> int:
        """bytes of a group's lookahead part (28 per 8x8 block of its rect)"""
        tx0, ty0, tw, th = rect
        hi, wi = self.imp_shape
        bw = min((tx0 + tw) * 8, wi) - tx0 * 8
        bh = min((ty0 + th) * 8, hi) - ty0 * 8
        return 28 * bw * bh

    def frame(self, sb_limit=0, pad=True) -> dict:
        fi = OrcFrameInfo()
        assert self.L.orc_replay_frame(self.h, C.byref(fi), sb_limit, 1 if pad else 0) == 0
        return {"display": fi.display, "me_range_scale": fi.me_range_scale, "level": fi.level,
                "is_key": fi.is_key, "ref_display": list(fi.ref_display),
                "compound": fi.compound}

    def region_bytes(self, rect) -> int:
        r = np.ascontiguousarray(np.asarray(rect, dtype=np.int32))
        return int(self.L.orc_replay_xcopy(self.h, r.ctypes.data, None, 1))

    def export(self, rect) -> np.ndarray:
        """The packed reconstruction of tile group `rect` of the last frame."""
        r = np.ascontiguousarray(np.asarray(rect, dtype=np.int32))
        out = np.zeros(self.region_bytes(rect), dtype=np.uint8)
        self.L.orc_replay_xcopy(self.h, r.ctypes.data, out.ctypes.data, 1)
        return out

    def import_(self, rect, buf: np.ndarray):
        r = np.ascontiguousarray(np.asarray(rect, dtype=np.int32))
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        self.L.orc_replay_xcopy(self.h, r.ctypes.data, buf.ctypes.data, 0)

    def pad_recon(self):
        self.L.orc_replay_pad_recon(self.h)

    def get_recon(self, display) -> np.ndarray:
        from rav1e_amd.replay import frame_bytes
        w, h, xd, yd, bd = self.geom
        out = np.zeros(frame_bytes(w, h, xd, yd, bd) // (2 if bd > 8 else 1),
                       dtype=np.uint16 if bd > 8 else np.uint8)
        assert self.L.orc_replay_get_recon(self.h, display, out.ctypes.data) == 0
        return out

    def results(self):
        out = np.zeros(self.n_words, dtype=np.uint64)
        n = self.L.orc_replay_results(self.h, out.ctypes.data, out.size)
        assert n == out.size
        return out

    def close(self):
        if self.h:
            self.L.orc_replay_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


# ---------------------------------------------------------------- entropy coder
EC_CDF_TOTAL = 4317  # oracle/orc_ec_tables.h ORC_EC_TOTAL
EC_JOB = np.dtype([(n, np.int32) for n in ("kind", "plane", "bx", "by", "tx_size", "tx_type",
                                            "is_inter", "bw_lg", "bh_lg", "coeff_off")])


def ec_lib():
    """The oracle's range coder / coefficient coder (oracle/orc_ec.c)."""
    L = lib()
    if not getattr(L, "_ec_ready", False):
        vp, i32 = C.c_void_p, C.c_int
        for n, a in (("orc_ecw_init", [vp]), ("orc_ecw_free", [vp]),
                     ("orc_ecw_symbol_update", [vp, C.c_uint32, vp, i32]),
                     ("orc_ecw_bool", [vp, i32, C.c_uint16]), ("orc_ecw_bit", [vp, i32]),
                     ("orc_ecw_literal", [vp, i32, C.c_uint32]),
                     ("orc_ecw_golomb", [vp, C.c_uint16]), ("orc_ecw_bytes", [vp, vp]),
                     ("orc_ecr_init", [vp, vp, C.c_size_t]),
                     ("orc_ec_reset_counts", [vp])):
            getattr(L, n).argtypes = a
            getattr(L, n).restype = None
        L.orc_ecw_finish.argtypes = [vp]
        L.orc_ecw_finish.restype = C.c_size_t
        L.orc_ecr_bool.argtypes = [vp, C.c_uint32]
        L.orc_ecr_bool.restype = i32
        L.orc_ecr_symbol.argtypes = [vp, vp, i32]
        L.orc_ecr_symbol.restype = i32
        L.orc_ec_default_cdf.argtypes = [i32]
        L.orc_ec_default_cdf.restype = C.POINTER(C.c_uint16)
        L.orc_ec_code_jobs.argtypes = [vp, i32, vp, vp, i32, i32, vp, C.c_long, vp, vp, vp]
        L.orc_ec_code_jobs.restype = C.c_long
        L._ec_ready = True
    return L


def ec_default_cdf(qctx):
    L = ec_lib()
    p = L.orc_ec_default_cdf(qctx)
    return np.ctypeslib.as_array(p, (EC_CDF_TOTAL,)).copy()


class EcWriter:
    """orc_ecw (WriterBase<WriterEncoder>) behind ctypes."""

    def __init__(self):
        self.L = ec_lib()
        self.buf = C.create_string_buffer(64)
        self.L.orc_ecw_init(self.buf)

    def symbol_update(self, s, cdf, off, n):
        arr = cdf[off:off + n]  # a view: update_cdf writes through
        self.L.orc_ecw_symbol_update(self.buf, s, arr.ctypes.data, n)

    def bool(self, v, f):
        self.L.orc_ecw_bool(self.buf, int(v), int(f))

    def bit(self, b):
        self.L.orc_ecw_bit(self.buf, int(b))

    def literal(self, nb, v):
        self.L.orc_ecw_literal(self.buf, int(nb), int(v))

    def golomb(self, v):
        self.L.orc_ecw_golomb(self.buf, int(v))

    def done(self):
        n = self.L.orc_ecw_finish(self.buf)
        out = np.zeros(n, np.uint8)
        self.L.orc_ecw_bytes(self.buf, out.ctypes.data)
        self.L.orc_ecw_free(self.buf)
        return out


def ec_replay_ops(ops):
    """Replay a gen_ec_ref op stream ((kind, a, b, c, d) rows) through the
    oracle's writer; returns the bytes."""
    w = EcWriter()
    state = {}
    for k, a, b, c, d in ops:
        if k == 0:
            if a not in state:
                state[a] = ec_default_cdf(int(a))
            w.symbol_update(int(d), state[a], int(b), int(c))
        elif k == 1:
            w.bool(b, a)
        elif k == 2:
            w.bit(a)
        elif k == 3:
            w.literal(a, b)
        else:
            w.golomb(a)
    return w.done()


def ec_code_jobs(jobs, coeffs, cdf_init, xdec, ydec, cap=1 << 24):
    """orc_ec_code_jobs: (bytes, tile byte counts, per-job returns, final CDFs)."""
    L = ec_lib()
    jobs = np.ascontiguousarray(jobs, np.int32)
    n = jobs.shape[0]
    coeffs = np.ascontiguousarray(coeffs, np.int32)
    cdf_init = np.ascontiguousarray(cdf_init, np.uint16)
    out = np.zeros(cap, np.uint8)
    ntiles = int((jobs[:, 0] == 3).sum()) + 1
    tb = np.zeros(ntiles, np.int32)
    ret = np.zeros(n, np.uint16)
    fin = np.zeros(EC_CDF_TOTAL, np.uint16)
    total = L.orc_ec_code_jobs(jobs.ctypes.data, n, coeffs.ctypes.data, cdf_init.ctypes.data,
                               xdec, ydec, out.ctypes.data, cap, tb.ctypes.data, ret.ctypes.data,
                               fin.ctypes.data)
    assert total >= 0, total
    return out[:total].copy(), tb, ret, fin


BLK = np.dtype([("ref", np.int8, 2), ("n4_w", np.uint8), ("n4_h", np.uint8), ("newmv", np.uint8),
                ("pad", np.uint8, 3), ("mv", np.int16, (2, 2))])
CAND = np.dtype([("this_mv", np.int16, 2), ("comp_mv", np.int16, 2), ("weight", np.uint32)])


def find_mvrefs(grid, cols, rows, tile_x, tile_y, frame_cols, frame_rows, bx, by, bw4, bh4,
                ref_frames, sign_bias):
    """orc_find_mvrefs (src/context.rs:2650-2965) over grid, a (rows, pitch)
    array of BLK: (mode_context, the stack's CAND entries)."""
    L = lib()
    if not getattr(L, "_mvref_bound", False):
        L.orc_find_mvrefs.argtypes = [C.c_void_p] + [C.c_int] * 11 + [C.c_void_p] * 4
        L.orc_find_mvrefs.restype = C.c_int
        L._mvref_bound = True
    g = np.ascontiguousarray(grid, dtype=BLK)
    rf = np.array(ref_frames, np.int32)
    sb = np.array(sign_bias, np.uint8)
    st = np.zeros(9, CAND)
    n = C.c_int(0)
    ctx = L.orc_find_mvrefs(ptr(g), g.shape[1], cols, rows, tile_x, tile_y, frame_cols, frame_rows,
                            bx, by, bw4, bh4, ptr(rf), ptr(sb), ptr(st), C.addressof(n))
    return ctx, st[:n.value]
