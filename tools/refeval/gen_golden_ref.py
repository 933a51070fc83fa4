"""Golden vectors produced by RUNNING the reference's own Rust function text.

Run in the build container (needs /root/reference):
    python tools/refeval/gen_golden_ref.py [section ...]

`rsinterp.py` parses the named reference functions out of
/root/reference/src and evaluates them; `rshost.py` supplies rav1e's frame
types over Python lists.  Only the resulting numbers are written
(tests/golden/ref_*.npz).  Functions evaluated, by section:

  mc    src/mc.rs:182-408      run_filter, get_filter, put_8tap_ref,
                               prep_8tap_ref, mc_avg_ref (+ SUBPEL_FILTERS)
  dist  src/dist.rs:25-46,197-328  get_sad_ref, get_satd_ref (8/10/12-bit,
                               random and maximum-residual planes)
  rdo   src/rdo.rs:219-335, 511-560  cdef_dist_wxh_8x8, cdef_dist_wxh,
                               sse_wxh, RawDistortion/Distortion arithmetic
  me    src/me.rs:943-1021     full_search, get_mv_rate (get_sad -> get_sad_ref)
  ds    src/me.rs:654-941      get_best_predictor, diamond_me_search,
                               get_mv_rd_cost, compute_mv_rd_cost,
                               telescopic_subpel_search; src/predict.rs:255-338
                               predict_inter (+ get_params); TileRect
                               (src/tiling/tile.rs); put/prep/avg -> *_ref
  quant src/quantize.rs:34-160, 205-333  QuantizationContext::update /
                               quantize, dequantize, divu_gen/divu_pair,
                               dc_q/ac_q, get_log_tx_scale (+ av1_scan_orders)
  cdef  src/cdef.rs:54-239      cdef_find_dir (+ first_max_element),
                               native::cdef_filter_block (+ constrain),
                               adjust_strength (+ msb, src/util/mod.rs)
  tx    src/transform/forward.rs:1771-1900 FwdTxfm2D::fht and
        src/transform/inverse.rs:1939-2114 inv_txfm2d_add / inv_txfm2d, over
        the reference's 1-D kernels (rs2py.py); round_shift_array,
        get_rect_tx_log_ratio, clamp_value from src/transform/mod.rs.

SIMD note (tx): fht is written over packed_simd lanes (`S::ColSimd::LANES`);
every operation on those vectors is lane-wise, so the
function is evaluated with LANES = 1.
"""
import os
import random
import re
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(__file__))
import rs2py  # noqa: E402
import rshost as H  # noqa: E402
import rsinterp as RI  # noqa: E402

REF = "/root/reference/src/"
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
OUT = os.path.join(ROOT, "tests", "golden")

TX_W_LOG2 = [2, 3, 4, 5, 6, 2, 3, 3, 4, 4, 5, 5, 6, 2, 4, 3, 5, 4, 6]
TX_H_LOG2 = [2, 3, 4, 5, 6, 3, 2, 4, 3, 5, 4, 6, 5, 4, 2, 5, 3, 6, 4]
# TxType -> (column 1-D kind, row 1-D kind): 0 Id, 1 Dct, 2 Adst, 3 FlipAdst
# (src/transform/mod.rs:123-160 TxType order; tx_2d_types)
TX_COL = [1, 2, 1, 2, 3, 1, 3, 2, 3, 0, 1, 0, 2, 0, 3, 0]
TX_ROW = [1, 1, 2, 2, 1, 3, 3, 3, 2, 0, 0, 1, 0, 2, 0, 3]
KIND = {"Id": 0, "Dct": 1, "Adst": 2, "FlipAdst": 3}


class TxSizeV(int):
    """A TxSize enum value (src/transform/mod.rs:162-247)."""

    def __new__(cls, idx):
        o = int.__new__(cls, idx)
        o.w, o.h = 1 << TX_W_LOG2[idx], 1 << TX_H_LOG2[idx]
        return o

    def width(self):
        return RI.TInt(self.w, "usize")

    def height(self):
        return RI.TInt(self.h, "usize")

    def area(self):
        return RI.TInt(self.w * self.h, "usize")

    def width_log2(self):
        return RI.TInt(TX_W_LOG2[int(self)], "usize")

    def height_log2(self):
        return RI.TInt(TX_H_LOG2[int(self)], "usize")


class _Mem:
    @staticmethod
    def size_of_val(v):
        v = RI.deref(v)
        return RI.TInt(RI.INT_BITS[RI.ty_of(v)] // 8, "usize")


class Fi:
    """The FrameInvariants fields full_search reads."""

    def __init__(self, bd):
        self.sequence = RI.Struct("Sequence", {"bit_depth": RI.TInt(bd, "usize")})
        self.cpu_feature_level = 0


def make_interp():
    env = H.base_env()
    env.update({"IMPORTANCE_BLOCK_SIZE": RI.TInt(8, "usize"),  # src/encoder.rs:58
                "MI_SIZE": RI.TInt(4, "usize"),  # src/context.rs:51
                "mem": _Mem,
                "Into": type("Into", (), {"into": staticmethod(
                    lambda v: RI.TInt(int(RI.deref(v)), "usize"))}),
                "RawDistortion": RI.StructType("RawDistortion"),
                "Distortion": RI.StructType("Distortion"),
                "ScaledDistortion": RI.StructType("ScaledDistortion"),
                "QuantizationContext": RI.StructType("QuantizationContext"),
                "SUBPEL_FILTER_SIZE": RI.TInt(8, "usize")})
    I = RI.Interp(env)
    I.sources = [RI.Source(REF + p) for p in (
        "util/mod.rs", "mc.rs", "dist.rs", "rdo.rs", "me.rs", "quantize.rs",
        "transform/mod.rs", "transform/forward.rs", "transform/inverse.rs", "scan_order.rs")]
    return I


def F(I, name, src=None, after=None):
    if src is not None:
        I.define_fn(I.sources[[s.path.endswith(src) for s in I.sources].index(True)]
                    .fn(name, after))
    elif name not in I.globals.vars:
        assert I.resolve(name), name
    return I.globals.vars[name]


def src_of(I, tail):
    return [s for s in I.sources if s.path.endswith(tail)][0]


def region_at(plane, x, y):
    return plane.region(RI.Struct("Area::StartingAt", {"x": x, "y": y}))


def prim(bd):
    return RI.PrimType("u8" if bd == 8 else "u16")


def rand_plane(rng, h, w, bd):
    return rng.integers(0, 1 << bd, (h, w)).astype(np.int64)


# ---------------------------------------------------------------- MC
MC_SIZES = [(4, 4), (8, 4), (4, 8), (8, 8), (16, 16), (16, 8), (8, 16), (4, 16), (16, 4),
            (32, 32), (32, 8), (64, 64)]


def gen_mc(I, rng, out):
    put, prep, avg = F(I, "put_8tap_ref"), F(I, "prep_8tap_ref"), F(I, "mc_avg_ref")
    for bd in (8, 10, 12):
        H_, W_ = 96, 112
        src = rand_plane(rng, H_, W_, bd)
        mx = (1 << bd) - 1
        src[:, 40:48] = np.array([0, 1, 0, 1, 1, 0, 1, 0]) * mx  # clamp stripes
        src[60:66, :] = mx
        plane = H.Plane.from_full(src, 0, 0, W_, H_)
        cases, puts, preps = [], [], []
        for (w, h) in MC_SIZES:
            fr = [(0, 0), (int(rng.integers(1, 16)), 0), (0, int(rng.integers(1, 16))),
                  (int(rng.integers(1, 16)), int(rng.integers(1, 16))),
                  (int(rng.integers(1, 16)), int(rng.integers(1, 16)))]
            modes = [(0, 0), (0, 0), (1, 2), (int(rng.integers(0, 4)), int(rng.integers(0, 4))),
                     (int(rng.integers(0, 4)), int(rng.integers(0, 4)))]
            for (cf, rf), (mdx, mdy) in zip(fr, modes):
                x = int(rng.integers(3, W_ - w - 4))
                y = int(rng.integers(3, H_ - h - 4))
                if len(cases) % 3 == 0:
                    x = 38 - w // 2 if w < 40 else 3  # across the stripes
                dst = H.Plane.from_full(np.zeros((h, w), np.int64), 0, 0, w, h)
                put(region_at(dst, 0, 0), plane.slice(RI.Struct("PlaneOffset", {"x": x, "y": y})),
                    RI.TInt(w, "usize"), RI.TInt(h, "usize"), cf, rf, mdx, mdy,
                    RI.TInt(bd, "usize"), 0, generics={"T": prim(bd)})
                tmp = [RI.TInt(0, "i16")] * (w * h)
                prep(RI.Slice(tmp), plane.slice(RI.Struct("PlaneOffset", {"x": x, "y": y})),
                     RI.TInt(w, "usize"), RI.TInt(h, "usize"), cf, rf, mdx, mdy,
                     RI.TInt(bd, "usize"), 0, generics={"T": prim(bd)})
                cases.append((w, h, cf, rf, mdx, mdy, x, y))
                puts.extend(dst.data)
                preps.extend(int(v) for v in tmp)
        # mc_avg over pairs of prep outputs of equal size
        offs = np.cumsum([0] + [c[0] * c[1] for c in cases])
        avg_cases, avgs = [], []
        for i in range(len(cases)):
            j = (i + 3) % len(cases)
            while (cases[j][0], cases[j][1]) != (cases[i][0], cases[i][1]):
                j = (j + 1) % len(cases)
            w, h = cases[i][0], cases[i][1]
            t1 = preps[offs[i]:offs[i + 1]]
            t2 = preps[offs[j]:offs[j + 1]]
            dst = H.Plane.from_full(np.zeros((h, w), np.int64), 0, 0, w, h)
            avg(region_at(dst, 0, 0), RI.Slice([RI.TInt(v, "i16") for v in t1]),
                RI.Slice([RI.TInt(v, "i16") for v in t2]), RI.TInt(w, "usize"),
                RI.TInt(h, "usize"), RI.TInt(bd, "usize"), 0, generics={"T": prim(bd)})
            avg_cases.append((i, j))
            avgs.extend(dst.data)
        k = "mc_bd%d_" % bd
        out[k + "src"] = src.astype(np.uint16)
        out[k + "cases"] = np.array(cases, np.int32)
        out[k + "put"] = np.array(puts, np.uint16)
        out[k + "prep"] = np.array(preps, np.int16)
        out[k + "avg_cases"] = np.array(avg_cases, np.int32)
        out[k + "avg"] = np.array(avgs, np.uint16)
        print("mc bd%d: %d put/prep, %d avg" % (bd, len(cases), len(avg_cases)))


# ---------------------------------------------------------------- dist
def gen_dist(I, rng, out):
    sad, satd = F(I, "get_sad_ref"), F(I, "get_satd_ref")
    for bd in (8, 10, 12):
        mx = (1 << bd) - 1
        H_, W_ = 200, 200
        org = rand_plane(rng, H_, W_, bd)
        ref = rand_plane(rng, H_, W_, bd)
        # maximum-residual corner: org = max, ref = 0 / checkerboard
        org[:64, :64] = mx
        ref[:64, :64] = 0
        yy, xx = np.mgrid[0:64, 0:64]
        ref[:64, 64:128] = ((yy + xx) & 1) * mx
        org[:64, 64:128] = (1 - ((yy + xx) & 1)) * mx
        po = H.Plane.from_full(org, 0, 0, W_, H_)
        pr = H.Plane.from_full(ref, 0, 0, W_, H_)
        cases, sads, satds = [], [], []
        for bs in range(22):
            b = H.BlockSize.from_width_and_height(*map(int, H.BLOCK_NAMES[bs].split("X")))
            w, h = b.w, b.h
            pos = [(0, 0), (64, 0) if w <= 64 and h <= 64 else (0, 0)]
            pos.append((int(rng.integers(0, W_ - w + 1)), int(rng.integers(0, H_ - h + 1))))
            for (x, y) in pos:
                rx, ry = (x, y) if len(cases) % 2 == 0 else (
                    int(rng.integers(0, W_ - w + 1)), int(rng.integers(0, H_ - h + 1)))
                a = region_at(po, x, y)
                r = region_at(pr, rx, ry)
                g = {"T": prim(bd)}
                sads.append(int(sad(a, r, b, RI.TInt(bd, "usize"), 0, generics=g)))
                satds.append(int(satd(a, r, b, RI.TInt(bd, "usize"), 0, generics=g)))
                cases.append((bs, x, y, rx, ry))
        k = "dist_bd%d_" % bd
        out[k + "org"] = org.astype(np.uint16)
        out[k + "ref"] = ref.astype(np.uint16)
        out[k + "cases"] = np.array(cases, np.int32)
        out[k + "sad"] = np.array(sads, np.uint32)
        out[k + "satd"] = np.array(satds, np.uint32)
        print("dist bd%d: %d cases" % (bd, len(cases)))


# ---------------------------------------------------------------- rdo distortion
def bias_of(area):
    """A deterministic non-trivial compute_bias closure (the device returns
    raw partials; the f64 bias is host arithmetic, src/rdo.rs:525-530)."""
    x, y = int(area.x), int(area.y)
    return 0.65 + ((x * 7 + y * 3) % 11) / 8.0


def gen_rdo(I, rng, out):
    rdo = src_of(I, "rdo.rs")
    for n in ("RawDistortion", "Distortion", "ScaledDistortion"):
        fns = []
        for m in re.finditer(r"\bimpl\b[^{;]*\b%s\s*\{" % n, rdo.src):
            fns += RI.parse_impl_fns(RI.find_item(rdo.src, "impl", n, m.start()))
        I.define_impl(n, fns)
    c8 = F(I, "cdef_dist_wxh_8x8", "rdo.rs")
    cdef = F(I, "cdef_dist_wxh", "rdo.rs")
    sse = F(I, "sse_wxh", "rdo.rs")
    for bd in (8, 10, 12):
        H_, W_ = 96, 96
        a = rand_plane(rng, H_, W_, bd)
        b = np.clip(a + rng.integers(-40, 41, a.shape) * (1 << (bd - 8)), 0, (1 << bd) - 1)
        b[:16, :16] = rand_plane(rng, 16, 16, bd)  # uncorrelated corner
        pa = H.Plane.from_full(a, 0, 0, W_, H_)
        pb = H.Plane.from_full(b, 0, 0, W_, H_)
        c8_cases, c8_vals = [], []
        for (x, y) in [(0, 0), (8, 0), (40, 24), (88, 88)] + \
                [(int(rng.integers(0, 89)), int(rng.integers(0, 89))) for _ in range(8)]:
            v = c8(region_at(pa, x, y), region_at(pb, x, y), RI.TInt(bd, "usize"),
                   generics={"T": prim(bd)})
            c8_cases.append((x, y))
            c8_vals.append(int(v._f["0"]))
        blk_cases, cdef_vals, sse_vals = [], [], []
        for (w, h, x, y) in [(8, 8, 0, 0), (64, 64, 0, 0), (32, 16, 40, 24), (16, 32, 8, 56),
                             (64, 32, 32, 64)]:
            bias = (lambda area, bsize: bias_of(area))
            d = cdef(region_at(pa, x, y), region_at(pb, x, y), RI.TInt(w, "usize"),
                     RI.TInt(h, "usize"), RI.TInt(bd, "usize"), bias, generics={"T": prim(bd)})
            s = sse(region_at(pa, x, y), region_at(pb, x, y), RI.TInt(w, "usize"),
                    RI.TInt(h, "usize"), bias, generics={"T": prim(bd)})
            blk_cases.append((w, h, x, y))
            cdef_vals.append(int(d._f["0"]))
            sse_vals.append(int(s._f["0"]))
        # chroma planes (4:2:0 and 4:2:2): sse over importance sub-blocks >> dec
        ch_cases, ch_vals = [], []
        for xdec, ydec in ((1, 1), (1, 0)):
            qa = H.Plane.from_full(a, 0, 0, W_, H_, xdec, ydec)
            qb = H.Plane.from_full(b, 0, 0, W_, H_, xdec, ydec)
            for (w, h, x, y) in [(32, 32, 0, 0), (16, 16, 12, 20), (8, 8, 40, 4)]:
                s = sse(region_at(qa, x, y), region_at(qb, x, y), RI.TInt(w, "usize"),
                        RI.TInt(h, "usize"), lambda area, bsize: bias_of(area),
                        generics={"T": prim(bd)})
                ch_cases.append((xdec, ydec, w, h, x, y))
                ch_vals.append(int(s._f["0"]))
        k = "rdo_bd%d_" % bd
        out[k + "a"] = a.astype(np.uint16)
        out[k + "b"] = b.astype(np.uint16)
        out[k + "c8_cases"] = np.array(c8_cases, np.int32)
        out[k + "c8"] = np.array(c8_vals, np.uint64)
        out[k + "blk_cases"] = np.array(blk_cases, np.int32)
        out[k + "cdef"] = np.array(cdef_vals, np.uint64)
        out[k + "sse"] = np.array(sse_vals, np.uint64)
        out[k + "ch_cases"] = np.array(ch_cases, np.int32)
        out[k + "ch_sse"] = np.array(ch_vals, np.uint64)
        print("rdo bd%d" % bd)


# ---------------------------------------------------------------- motion search
def gen_me(I, rng, out):
    fs = F(I, "full_search", "me.rs")
    sad_ref = F(I, "get_sad_ref")
    for bd in (8, 10):
        pad = 24
        H_, W_ = 64, 96
        org = rand_plane(rng, H_, W_, bd)
        ref = np.roll(org, (3, -5), (0, 1))
        ref = np.clip(ref + rng.integers(-2, 3, ref.shape), 0, (1 << bd) - 1)
        ref[40:, 60:] = 77 << (bd - 8)  # flat area: ties resolve to the first raster candidate
        org[40:, 60:] = 77 << (bd - 8)
        fo = np.pad(org, pad, mode="edge")
        fr = np.pad(ref, pad, mode="edge")
        po = H.Plane.from_full(fo, pad, pad, W_, H_)
        pr = H.Plane.from_full(fr, pad, pad, W_, H_)
        I.globals.vars["get_sad"] = (
            lambda a, b, bs, bd_, cpu, _g={"T": prim(bd)}: sad_ref(a, b, bs, bd_, cpu, generics=_g))
        cases, res = [], []
        for k in range(10):
            blk = [8, 16, 16, 8, 16, 16, 16, 8, 16, 16][k]
            step = [1, 1, 2, 1, 1, 1, 1, 3, 1, 1][k]
            if k == 5:
                px, py = 64, 44  # inside the flat area
            elif k == 6:
                px, py = 0, 0  # window crosses the padding
            else:
                px, py = int(rng.integers(0, W_ - blk)), int(rng.integers(0, H_ - blk))
            rx, ry = int(rng.integers(4, 14)), int(rng.integers(3, 9))
            x_lo, x_hi = max(px - rx, -pad + 4), min(px + rx, W_ - blk + pad - 4)
            y_lo, y_hi = max(py - ry, -pad + 4), min(py + ry, H_ - blk + pad - 4)
            pm0 = (int(rng.integers(-40, 40)), int(rng.integers(-40, 40)))
            pm1 = (int(rng.integers(-40, 40)), int(rng.integers(-40, 40)))
            lam = int(rng.integers(0, 3000)) if k != 4 else 0
            hp = k % 2
            best = [H.motion_vector(0, 0)]
            cost = [RI.TInt(2 ** 64 - 1, "u64")]
            best_ref = RI.Ref(lambda: best[0], lambda v: best.__setitem__(0, v))
            cost_ref = RI.Ref(lambda: cost[0], lambda v: cost.__setitem__(0, v))
            bsize = H.BlockSize.from_width_and_height(blk, blk)
            fs(Fi(bd), RI.TInt(x_lo, "isize"), RI.TInt(x_hi, "isize"), RI.TInt(y_lo, "isize"),
               RI.TInt(y_hi, "isize"), bsize, po, pr, best_ref, cost_ref,
               RI.Struct("PlaneOffset", {"x": RI.TInt(px, "isize"), "y": RI.TInt(py, "isize")}),
               RI.TInt(step, "usize"), RI.TInt(lam, "u32"),
               [H.motion_vector(*pm0), H.motion_vector(*pm1)], bool(hp), generics={"T": prim(bd)})
            cases.append((blk, step, hp, px, py, x_lo, x_hi, y_lo, y_hi, pm0[0], pm0[1],
                          pm1[0], pm1[1], lam))
            res.append((int(best[0].row), int(best[0].col), int(cost[0])))
        kk = "me_bd%d_" % bd
        out[kk + "org"] = fo.astype(np.uint16)
        out[kk + "ref"] = fr.astype(np.uint16)
        out[kk + "geom"] = np.array([pad, pad, W_, H_], np.int32)
        out[kk + "cases"] = np.array(cases, np.int64)
        out[kk + "mv"] = np.array([r[:2] for r in res], np.int16)
        out[kk + "cost"] = np.array([r[2] for r in res], np.uint64)
        print("me bd%d: %d searches" % (bd, len(cases)))
    # get_mv_rate on its own over a grid of differences
    rate = F(I, "get_mv_rate", "me.rs")
    g = []
    for hp in (False, True):
        for dr in (-300, -17, -8, -1, 0, 1, 2, 3, 7, 8, 255, 4000):
            for dc in (-9, 0, 5, 64):
                g.append((int(hp), dr, dc, int(rate(H.motion_vector(dr, dc), H.motion_vector(0, 0),
                                                    hp))))
    out["me_mv_rate"] = np.array(g, np.int32)


# ---------------------------------------------------------------- diamond / sub-pel
class RefV(int):
    """RefType (src/frame/mod.rs / context: INTRA_FRAME = 0 .. NONE_FRAME)."""

    def to_index(self):
        return RI.TInt(int(self) - 1, "usize")


class _RefType:
    INTRA_FRAME, LAST_FRAME, NONE_FRAME = RefV(0), RefV(1), RefV(8)


class PredModeV(int):
    """PredictionMode::NEWMV; is_intra() is `self < NEARESTMV` (predict.rs:243)."""
    interp = None

    def is_intra(self):
        return False

    def predict_inter(self, *args):
        return PredModeV.fn(self, *args, generics={"T": PredModeV.pixel})


class DsFi(Fi):
    """FrameInvariants fields the diamond / sub-pel searches and predict_inter read."""

    def __init__(self, bd, ref_plane, allow_hp):
        super().__init__(bd)
        self.allow_high_precision_mv = bool(allow_hp)
        self.default_filter = RI.TInt(0, "usize")  # REGULAR (src/encoder.rs:705)
        rec = RI.Struct("ReferenceFrame", {"frame": RI.Struct("Frame", {"planes": [ref_plane]})})
        self.rec_buffer = RI.Struct("ReferenceFramesSet", {"frames": [rec] * 8})
        self.ref_frames = [RI.TInt(0, "u8")] * 7


def gen_ds(I, rng, out):
    tile = RI.Source(REF + "tiling/tile.rs")
    I.define_impl("TileRect", tile.impl("TileRect"))
    I.globals.vars["TileRect"] = RI.StructType("TileRect")
    I.globals.vars["RefType"] = _RefType
    I.globals.vars["NONE_FRAME"] = _RefType.NONE_FRAME
    I.globals.vars["PredictionMode"] = type("PM", (), {"NEWMV": PredModeV(16)})
    I.globals.vars["Plane"] = type("PlaneNS", (), {"new": staticmethod(
        lambda w, h, xd, yd, xp, yp: H.Plane.from_full(np.zeros((int(h), int(w)), np.int64),
                                                       0, 0, int(w), int(h)))})
    pred = RI.Source(REF + "predict.rs")
    PredModeV.fn = I.make_fn(pred.fn("predict_inter"), I.globals)
    ds = F(I, "diamond_me_search", "me.rs")
    tel = F(I, "telescopic_subpel_search", "me.rs")
    sad_ref, satd_ref = F(I, "get_sad_ref"), F(I, "get_satd_ref")
    put_ref, prep_ref, avg_ref = F(I, "put_8tap_ref"), F(I, "prep_8tap_ref"), F(I, "mc_avg_ref")
    for bd in (8, 10):
        g = {"T": prim(bd)}
        PredModeV.pixel = prim(bd)
        I.globals.vars["get_sad"] = lambda *a, _g=g: sad_ref(*a, generics=_g)
        I.globals.vars["get_satd"] = lambda *a, _g=g: satd_ref(*a, generics=_g)
        I.globals.vars["put_8tap"] = lambda *a, _g=g: put_ref(*a, generics=_g)
        I.globals.vars["prep_8tap"] = lambda *a, _g=g: prep_ref(*a, generics=_g)
        I.globals.vars["mc_avg"] = lambda *a, _g=g: avg_ref(*a, generics=_g)
        pad, H_, W_ = 88, 96, 128
        org = rand_plane(rng, H_, W_, bd)
        ref = np.roll(org, (2, -3), (0, 1))
        ref = np.clip(ref + rng.integers(-3, 4, ref.shape), 0, (1 << bd) - 1)
        ref[:, 100:128:2] = (1 << bd) - 1  # 0/max stripes near the right edge
        ref[:, 101:128:2] = 0
        fo = np.pad(org, pad, mode="edge")
        fr = np.pad(ref, pad, mode="edge")
        po = H.Plane.from_full(fo, pad, pad, W_, H_)
        pr = H.Plane.from_full(fr, pad, pad, W_, H_)
        cases, res = [], []
        specs = [  # (w, h, subpel, satd, hp, kind) kind 0 diamond, 1 telescopic
            (64, 64, 0, 0, 0, 0), (32, 32, 0, 0, 0, 0), (16, 16, 0, 1, 0, 0), (32, 16, 0, 0, 0, 0),
            (8, 8, 1, 0, 0, 0), (8, 8, 1, 0, 1, 0), (16, 16, 1, 0, 0, 0), (16, 8, 1, 1, 1, 0),
            (8, 16, 1, 0, 1, 0), (8, 8, 0, 0, 0, 1), (8, 8, 0, 1, 1, 1), (16, 16, 0, 0, 1, 1),
            (16, 8, 0, 0, 0, 1)]
        for n, (w, h, sub, satd, hp, kind) in enumerate(specs):
            px_ = int(rng.integers(-4, W_ - w + 4)) if n % 4 else W_ - w + 2
            py_ = int(rng.integers(-4, H_ - h + 4)) if n % 4 else 0
            span = 8 * int(rng.integers(3, 10))
            rng_ = (-span, span, -span // 2, span // 2)
            pm0 = [int(v) for v in rng.integers(-40, 40, 2)]
            pm1 = [int(v) for v in rng.integers(-40, 40, 2)]
            lam = int(rng.integers(0, 4000))
            npred = int(rng.integers(1, 6))
            step = 1 if sub else 8
            preds = [[int(v) * step for v in rng.integers(-6, 6, 2)] for _ in range(npred)]
            if n % 5 == 2:
                preds[0] = [span + 8, 0]  # out of range
            start = (8 * int(rng.integers(-2, 3)), 8 * int(rng.integers(-2, 3)))
            start_cost = int(rng.integers(0, 1 << 22)) if n % 3 else 2 ** 64 - 1
            fi = DsFi(bd, pr, hp)
            best = [H.motion_vector(*start) if kind else H.motion_vector(0, 0)]
            cost = [RI.TInt(start_cost if kind else 0, "u64")]
            bref = RI.Ref(lambda: best[0], lambda v: best.__setitem__(0, v))
            cref = RI.Ref(lambda: cost[0], lambda v: cost.__setitem__(0, v))
            po_ = RI.Struct("PlaneOffset", {"x": RI.TInt(px_, "isize"), "y": RI.TInt(py_, "isize")})
            pmv = [H.motion_vector(*pm0), H.motion_vector(*pm1)]
            bs = H.BlockSize.from_width_and_height(w, h)
            lo = [RI.TInt(v, "isize") for v in rng_]
            if kind == 0:
                ds(fi, po_, po, pr, [H.motion_vector(*p) for p in preds], RI.TInt(bd, "usize"),
                   pmv, RI.TInt(lam, "u32"), lo[0], lo[1], lo[2], lo[3], bs, bool(satd), bref,
                   cref, bool(sub), _RefType.LAST_FRAME, generics=g)
            else:
                ts = RI.Struct("TileStateMut", {"input": RI.Struct("Frame", {"planes": [po]})})
                tel(fi, ts, po_, RI.TInt(lam, "u32"), _RefType.LAST_FRAME, pmv, lo[0], lo[1],
                    lo[2], lo[3], bs, bool(satd), bref, cref, generics=g)
            pp = preds + [[0, 0]] * (8 - npred)
            cases.append([w, h, sub, satd, hp, kind, px_, py_] + list(rng_) + pm0 + pm1 +
                         [lam, npred] + [v for p in pp for v in p] + list(start) +
                         [start_cost & 0xFFFFFFFF, start_cost >> 32])
            res.append((int(best[0].row), int(best[0].col), int(cost[0])))
            print("  ds bd%d case %d: %s -> %s" % (bd, n, specs[n], res[-1]))
        kk = "ds_bd%d_" % bd
        out[kk + "org"] = fo.astype(np.uint16)
        out[kk + "ref"] = fr.astype(np.uint16)
        out[kk + "geom"] = np.array([pad, pad, W_, H_], np.int32)
        out[kk + "cases"] = np.array(cases, np.int64)
        out[kk + "mv"] = np.array([r[:2] for r in res], np.int16)
        out[kk + "cost"] = np.array([r[2] for r in res], np.uint64)


# ---------------------------------------------------------------- quantizer
def gen_quant(I, rng, out):
    q = src_of(I, "quantize.rs")
    I.define_impl("QuantizationContext", q.impl("QuantizationContext", "impl QuantizationContext"))
    deq = F(I, "dequantize", "quantize.rs")
    I.globals.vars["TxSize"] = type("TxSizeNS", (), {})
    cases, qout, dqout, coeffs_all = [], [], [], []
    for ts in range(19):
        w, h = 1 << TX_W_LOG2[ts], 1 << TX_H_LOG2[ts]
        area = min(w, 32) * min(h, 32)
        types = [0, 9] if max(w, h) <= 16 else [0]
        if max(w, h) <= 16:
            types += [int(rng.integers(1, 16))]
        for tt in types:
            if max(w, h) == 64 and tt != 0:
                continue
            for bd in (8, 10, 12):
                for qi, intra in ((100, False), (int(rng.integers(1, 256)), True),
                                  (int(rng.integers(1, 256)), False)):
                    sc = 1 << (bd - 8)
                    co = (rng.laplace(0, 40 * sc, area) * np.exp(-np.arange(area) / (area / 4)))
                    co = co.astype(np.int64)
                    co[0] = int(rng.integers(-2000 * sc, 2000 * sc))
                    ctx = RI.Struct("QuantizationContext", {
                        "log_tx_scale": RI.TInt(0, "usize"), "dc_quant": RI.TInt(0, "u32"),
                        "dc_offset": RI.TInt(0, "i32"), "dc_mul_add": (0, 0, 0),
                        "ac_quant": RI.TInt(0, "u32"), "ac_offset_eob": RI.TInt(0, "i32"),
                        "ac_offset0": RI.TInt(0, "i32"), "ac_offset1": RI.TInt(0, "i32"),
                        "ac_mul_add": (0, 0, 0)})
                    upd = I.make_method("QuantizationContext", "update", ctx, I.globals)
                    upd(RI.TInt(qi, "u8"), TxSizeV(ts), intra, RI.TInt(bd, "usize"),
                        RI.TInt(0, "i8"), RI.TInt(0, "i8"))
                    quant = I.make_fn(q.fn("quantize", "impl QuantizationContext"), I.globals)
                    cin = [RI.TInt(int(v), "i32") for v in co]
                    qc = [RI.TInt(0, "i32")] * area
                    quant(ctx, RI.Slice(cin), RI.Slice(qc), TxSizeV(ts), RI.TInt(tt, "usize"),
                          generics={"T": RI.PrimType("i32")},
                          bind={"Self": I.globals.vars["QuantizationContext"]})
                    rc = [RI.TInt(0, "i32")] * area
                    deq(RI.TInt(qi, "u8"), RI.Slice(list(qc)), RI.Slice(rc), TxSizeV(ts),
                        RI.TInt(bd, "usize"), RI.TInt(0, "i8"), RI.TInt(0, "i8"))
                    cases.append((ts, tt, bd, qi, int(intra), len(coeffs_all)))
                    coeffs_all.extend(int(v) for v in co)
                    qout.extend(int(v) for v in qc)
                    dqout.extend(int(v) for v in rc)
    out["quant_cases"] = np.array(cases, np.int32)
    out["quant_coeffs"] = np.array(coeffs_all, np.int32)
    out["quant_q"] = np.array(qout, np.int32)
    out["quant_dq"] = np.array(dqout, np.int32)
    divu = []
    gen, pair = F(I, "divu_gen", "quantize.rs"), F(I, "divu_pair", "quantize.rs")
    for d in (1, 2, 3, 4, 7, 8, 100, 1000, 1337, 21387, 65535):
        dg = gen(RI.TInt(d, "u32"))
        for x in (-70000, -1001, -1, 0, 1, 5, 999, 123456, 2 ** 20 + 3):
            divu.append((d, x, int(pair(RI.TInt(x, "i32"), dg))))
    out["quant_divu"] = np.array(divu, np.int64)
    print("quant: %d blocks" % len(cases))


# ---------------------------------------------------------------- transforms
class Lane1:
    """packed_simd vector types at LANES = 1 (see module docstring)."""
    LANES = RI.TInt(1, "usize")

    @staticmethod
    def load_from_slice(s):
        return RI.as_slice(s)[0]

    @staticmethod
    def slice_cast_ref(s):
        return s

    slice_cast_mut = slice_cast_ref

    @staticmethod
    def _splat(v):
        return v


class AlignedArray:
    def __init__(self, arr):
        self.array = arr

    @staticmethod
    def uninitialized():
        return AlignedArray([RI.TInt(0, "i32")] * (64 * 64))

    @staticmethod
    def new(arr):
        return AlignedArray(arr)

    def index_range(self, r):
        return RI.index_get(self.array, r)

    def as_slice(self):
        return RI.Slice(self.array)


def tx_tables(I):
    fwd = src_of(I, "transform/forward.rs")
    inv = src_of(I, "transform/inverse.rs")
    ns = rs2py.load()
    # 1-D forward kernel per (kind, n): the reference's txfm_types::d! table
    blk = fwd.raw[fwd.raw.index("pub mod txfm_types"):]
    f1 = {}
    for m in re.finditer(r"\((Dct|Adst|FlipAdst|Id),\s*(\d+),\s*(\w+),\s*\)", blk):
        f1[(KIND[m.group(1)], int(m.group(2)))] = ns[m.group(3)]
    # inverse 1-D kernel per (kind, n): inverse.rs txfm_types::d! (FlipAdst and
    # the 32/64-point Adst are `unimplemented!` there, so never reached)
    iblk = inv.raw[inv.raw.index("mod txfm_types"):]
    iblk = iblk[:iblk.index("unimplemented inversions")]
    i1 = {}
    for m in re.finditer(r"\((Dct|Adst|FlipAdst|Id),\s*(\d+),\s*(\w+),\s*\)", iblk):
        i1[(KIND[m.group(1)], int(m.group(2)))] = ns[m.group(3)]
    # InvBlock::INTERMEDIATE_SHIFT from the impl_inv_txs! invocations
    ish = {}
    for m in re.finditer(r"impl_inv_txs!\s*\{\s*([^}]*)\}", inv.src):
        body = m.group(1)
        if "$" in body:
            continue
        sh = int(body.strip().split()[-1])
        for w, h in re.findall(r"\((\d+),\s*(\d+)\)", body):
            ish[(int(w), int(h))] = sh
    return f1, i1, ish


class _NS:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def tx_fns(I):
    """(fwd, inv): the reference's FwdTxfm2D::fht and inv_txfm2d_add bound to
    one (TxSize, TxType), as gen_tx evaluates them.
      fwd(ts, tt, residual (list, W*H), bd) -> W-stride raster of W*H ints
      inv(ts, tt, coeffs (min(W,32)*min(H,32)), dst (H x W array), bd, "u8"|"u16")
        -> the reconstruction (H x W array)"""
    f1, i1, ish = tx_tables(I)
    fwd_src = src_of(I, "transform/forward.rs")
    inv_src = src_of(I, "transform/inverse.rs")
    fht = fwd_src.fn("fht", "impl<P, S, T> FwdTxfm2D<P> for (S, T)")
    itx2 = inv_src.fn("inv_txfm2d", "type ColTxfm = ")
    itx_add = inv_src.fn("inv_txfm2d_add", "type ColTxfm = ")
    I.globals.vars["AlignedArray"] = AlignedArray
    I.globals.vars["round_shift_array"] = I.make_fn(
        src_of(I, "transform/mod.rs").fn("round_shift_array"), I.globals)
    I.globals.vars["PixelType"] = _NS(U8=0, U16=1)
    nocall = [[None] * 4 for _ in range(4)]
    I.globals.vars["kernels"] = _NS(U8_INV_TX_ADD_KERNELS=[[nocall] * 22],
                                    U16_INV_TX_ADD_KERNELS=[[nocall] * 22])

    def size_of(ts):
        w, h = 1 << TX_W_LOG2[ts], 1 << TX_H_LOG2[ts]
        return w, h, _NS(W=RI.TInt(w, "usize"), H=RI.TInt(h, "usize"), WIDTH=RI.TInt(w, "usize"),
                         HEIGHT=RI.TInt(h, "usize"), AREA=RI.TInt(w * h, "usize"),
                         ColSimd=Lane1, RowSimd=Lane1, IColSimd=Lane1,
                         INTERMEDIATE_SHIFT=RI.TInt(ish[(w, h)], "u16"))

    def fwd(ts, tt, res, bd):
        w, h, size = size_of(ts)
        ck, rk = TX_COL[tt], TX_ROW[tt]
        shift = fwd_src.load_static(I, "FWD_SHIFT_%dX%d" % (w, h))
        ctx = _NS(Size=size, SHIFT=shift, Col=_NS(FLIPPED=ck == 3), Row=_NS(FLIPPED=rk == 3),
                  ColTx=_NS(forward=lambda i, o, f=f1[(ck, h)]: f(i, o)),
                  RowTx=_NS(forward=lambda i, o, f=f1[(rk, w)]: f(i, o)))
        co = [RI.TInt(0, "i32")] * (w * h)
        I.make_fn(fht, I.globals)(RI.Slice([RI.TInt(int(v), "i16") for v in res]), RI.Slice(co),
                                  RI.TInt(bd, "usize"), bind={"Self": ctx, "S": size})
        return [int(v) for v in co]

    def inv(ts, tt, co, dst, bd, px):
        w, h, size = size_of(ts)
        ck, rk = TX_COL[tt], TX_ROW[tt]
        pd = H.Plane.from_full(np.asarray(dst, np.int64).copy(), 0, 0, w, h)
        ictx = _NS(Size=size, RowTxfm=_NS(inverse=lambda i, o, r, f=i1[(rk, w)]: f(i, o, r)),
                   ColTxfm=_NS(inverse=lambda i, o, r, f=i1[(ck, h)]: f(i, o, r)))
        tt_ns = _NS(Row=_NS(TBL_IDX=0), Col=_NS(TBL_IDX=0), TX_TYPE=tt)
        inner = I.make_fn(itx2, I.globals)
        ictx.inv_txfm2d = (lambda *a, _f=inner, _c=ictx, _s=size: _f(*a, bind={"Self": _c, "S": _s}))
        pt = RI.PrimType(px)
        pt.type_enum = lambda: 0 if px == "u8" else 1
        I.make_fn(itx_add, I.globals)(
            RI.Slice([RI.TInt(int(v), "i32") for v in co] + [RI.TInt(0, "i32")] * 32),
            region_at(pd, 0, 0), RI.TInt(bd, "usize"), H.base_env()["CpuFeatureLevel"],
            bind={"Self": ictx, "S": size, "T": tt_ns, "P": pt})
        return np.array(pd.data, np.int64).reshape(h, w)
    return fwd, inv


def gen_tx(I, rng, out):
    f1, i1, ish = tx_tables(I)
    fwd = src_of(I, "transform/forward.rs")
    inv = src_of(I, "transform/inverse.rs")
    fht = fwd.fn("fht", "impl<P, S, T> FwdTxfm2D<P> for (S, T)")
    itx2 = inv.fn("inv_txfm2d", "type ColTxfm = ")
    itx_add = inv.fn("inv_txfm2d_add", "type ColTxfm = ")
    I.globals.vars["AlignedArray"] = AlignedArray
    I.globals.vars["round_shift_array"] = I.make_fn(
        src_of(I, "transform/mod.rs").fn("round_shift_array"), I.globals)
    I.globals.vars["PixelType"] = _NS(U8=0, U16=1)
    nocall = [[None] * 4 for _ in range(4)]
    I.globals.vars["kernels"] = _NS(U8_INV_TX_ADD_KERNELS=[[nocall] * 22],
                                    U16_INV_TX_ADD_KERNELS=[[nocall] * 22])
    cases_f, fin, fout, cases_i, icoef, idst, iout = [], [], [], [], [], [], []
    for ts in range(19):
        w, h = 1 << TX_W_LOG2[ts], 1 << TX_H_LOG2[ts]
        shift = fwd.load_static(I, "FWD_SHIFT_%dX%d" % (w, h))
        size = _NS(W=RI.TInt(w, "usize"), H=RI.TInt(h, "usize"), WIDTH=RI.TInt(w, "usize"),
                   HEIGHT=RI.TInt(h, "usize"), AREA=RI.TInt(w * h, "usize"),
                   ColSimd=Lane1, RowSimd=Lane1, IColSimd=Lane1,
                   INTERMEDIATE_SHIFT=RI.TInt(ish[(w, h)], "u16"))
        for tt in range(16):
            ck, rk = TX_COL[tt], TX_ROW[tt]
            for bd in (8, 10, 12):
                if rk != 3 and (ck, h) in f1 and (rk, w) in f1:
                    ctx = _NS(Size=size, SHIFT=shift,
                              Col=_NS(FLIPPED=ck == 3), Row=_NS(FLIPPED=rk == 3),
                              ColTx=_NS(forward=lambda i, o, f=f1[(ck, h)]: f(i, o)),
                              RowTx=_NS(forward=lambda i, o, f=f1[(rk, w)]: f(i, o)))
                    amp = (1 << bd) - 1
                    res = [int(v) for v in rng.integers(-amp, amp + 1, w * h)]
                    if len(cases_f) % 4 == 0:  # extreme residuals
                        res = [amp if (k * 7 + k // w) % 3 else -amp for k in range(w * h)]
                    co = [RI.TInt(0, "i32")] * (w * h)
                    fn = I.make_fn(fht, I.globals)
                    fn(RI.Slice([RI.TInt(v, "i16") for v in res]), RI.Slice(co),
                       RI.TInt(bd, "usize"), bind={"Self": ctx, "S": size})
                    cases_f.append((ts, tt, bd, len(fin)))
                    fin.extend(res)
                    fout.extend(int(v) for v in co)
                if (ck, h) in i1 and (rk, w) in i1 and bd in (8, 10, 12):
                    cw, ch = min(w, 32), min(h, 32)
                    co = [0] * (cw * ch)
                    for k in range(cw * ch):
                        if rng.random() < 0.3:
                            co[k] = int(rng.integers(-(1 << (bd + 3)), 1 << (bd + 3)))
                    co[0] = int(rng.integers(-(1 << (bd + 6)), 1 << (bd + 6)))
                    dst = rand_plane(rng, h, w, bd)
                    pd = H.Plane.from_full(dst.copy(), 0, 0, w, h)
                    ictx = _NS(Size=size, RowTxfm=_NS(inverse=lambda i, o, r, f=i1[(rk, w)]:
                                                      f(i, o, r)),
                               ColTxfm=_NS(inverse=lambda i, o, r, f=i1[(ck, h)]: f(i, o, r)))
                    tt_ns = _NS(Row=_NS(TBL_IDX=0), Col=_NS(TBL_IDX=0), TX_TYPE=tt)
                    inner = I.make_fn(itx2, I.globals)
                    ictx.inv_txfm2d = (lambda *a, _f=inner, _c=ictx, _s=size:
                                       _f(*a, bind={"Self": _c, "S": _s}))
                    pt = prim(bd)
                    pt.type_enum = lambda _b=bd: 0 if _b == 8 else 1
                    fn = I.make_fn(itx_add, I.globals)
                    fn(RI.Slice([RI.TInt(v, "i32") for v in co] + [RI.TInt(0, "i32")] * 32),
                       region_at(pd, 0, 0), RI.TInt(bd, "usize"), H.base_env()["CpuFeatureLevel"],
                       bind={"Self": ictx, "S": size, "T": tt_ns, "P": pt})
                    cases_i.append((ts, tt, bd, len(icoef), len(idst)))
                    icoef.extend(co)
                    idst.extend(int(v) for v in dst.reshape(-1))
                    iout.extend(pd.data)
        print("tx size %d done (%d fwd, %d inv)" % (ts, len(cases_f), len(cases_i)))
    out["tx_fwd_cases"] = np.array(cases_f, np.int32)
    out["tx_fwd_in"] = np.array(fin, np.int16)
    out["tx_fwd_out"] = np.array(fout, np.int32)
    out["tx_inv_cases"] = np.array(cases_i, np.int32)
    out["tx_inv_coeffs"] = np.array(icoef, np.int32)
    out["tx_inv_dst"] = np.array(idst, np.uint16)
    out["tx_inv_out"] = np.array(iout, np.uint16)


# ---------------------------------------------------------------- cdef
def _cdef_content(rng, h, w, bd):
    """Directional ramps + an edge + small noise: taps land inside
    constrain's active range at every strength."""
    yy, xx = np.mgrid[0:h, 0:w]
    a = rng.uniform(0, np.pi)
    base = (np.cos(a) * xx + np.sin(a) * yy) * rng.uniform(2, 12)
    img = base + rng.integers(-6, 7, (h, w)) + (xx > w // 2) * rng.integers(0, 40)
    img = img * (1 << (bd - 8)) + (1 << bd) // 3
    return np.clip(img, 0, (1 << bd) - 1).astype(np.int64)


def gen_cdef(I, rng, out):
    I.sources.append(RI.Source(REF + "cdef.rs"))
    # release semantics: cdef_find_dir's debug_assert!(p >> coeff_shift <= 255)
    # is compiled out, and a partial edge block of the padded copy sums
    # CDEF_VERY_LARGE with i32 wrap-around (typed ints wrap in the interpreter)
    I.release = True
    I.globals.vars["CDEF_VERY_LARGE"] = RI.TInt(0x8000, "u16")
    fd = F(I, "cdef_find_dir", "cdef.rs")
    fb = F(I, "cdef_filter_block", "cdef.rs")
    adj = F(I, "adjust_strength", "cdef.rs")

    def u(v):
        return RI.TInt(int(v), "usize")

    def i32(v):
        return RI.TInt(int(v), "i32")

    imgs, shifts, dirs, vars_ = [], [], [], []
    for n in range(96):
        bd = (8, 10, 12)[n % 3]
        img = _cdef_content(rng, 8, 8, bd)
        if n % 8 == 5:  # a partial edge block of the padded copy
            img[:, 8 - 1 - (n // 8) % 4:] = 0x8000
        if n % 8 == 6:
            img[5:, :] = 128
            img[3:5, :] = 0x8000
        plane = H.Plane.from_full(img, 0, 0, 8, 8)
        v = [RI.TInt(0, "i32")]
        d = fd(plane.slice(RI.Struct("PlaneOffset", {"x": 0, "y": 0})),
               RI.Ref(lambda: v[0], lambda x: v.__setitem__(0, x)), u(bd - 8),
               generics={"T": RI.PrimType("u16")})
        imgs.append(img.astype(np.uint16))
        shifts.append(bd - 8)
        dirs.append(int(d))
        vars_.append(int(v[0]))
    out["dir_img"] = np.array(imgs, np.uint16)
    out["dir_shift"] = np.array(shifts, np.int32)
    out["dir_dir"] = np.array(dirs, np.int32)
    out["dir_var"] = np.array(vars_, np.int32)
    cases, srcs, dsts = [], [], []
    for n in range(120):
        bd = (8, 10, 12)[n % 3]
        xdec, ydec = ((0, 0), (1, 1), (1, 0))[(n // 3) % 3]
        cs = bd - 8
        src = _cdef_content(rng, 12, 12, bd)
        if n % 5 == 1:
            src[:2, :] = 0x8000
        if n % 5 == 2:
            src[:, -3:] = 0x8000
            src[-2:, :] = 128
        pri = int(rng.integers(0, 16)) << cs
        if n % 4 == 0:
            pri = int(rng.integers(0, 16 << cs))  # adjust_strength output: any value
        sec = (0, 1, 2, 4)[int(rng.integers(0, 4))] << cs
        damping = 3 + cs - (1 if (xdec or ydec) else 0) + int(rng.integers(0, 4))
        dr = int(rng.integers(0, 8))
        flat = [RI.TInt(int(x), "u16") for x in src.ravel()]
        dst = H.Plane.from_full(np.zeros((8, 8), np.int64), 0, 0, 8, 8)
        fb(region_at(dst, 0, 0), RI.Ptr(flat, 2 * 12 + 2), RI.TInt(12, "isize"), i32(pri),
           i32(sec), u(dr), i32(damping), u(bd), u(xdec), u(ydec), 0,
           generics={"T": prim(bd)})
        cases.append((bd, xdec, ydec, pri, sec, dr, damping))
        srcs.append(src.astype(np.uint16))
        dsts.append(np.array(dst.data, np.int64).reshape(8, 8).astype(np.uint16))
    out["filt_cases"] = np.array(cases, np.int32)
    out["filt_src"] = np.array(srcs, np.uint16)
    out["filt_dst"] = np.array(dsts, np.uint16)
    adj_cases = [(s, v) for s in (0, 1, 5, 15, 60) for v in
                 (0, 1, 63, 64, 100, 1 << 12, 1 << 18, (1 << 30) + 5, 977)]
    out["adj_cases"] = np.array(adj_cases, np.int32)
    out["adj_out"] = np.array([int(adj(i32(s), i32(v))) for s, v in adj_cases], np.int32)
    print("cdef: %d find_dir, %d filter_block, %d adjust" % (len(imgs), len(cases),
                                                             len(adj_cases)))

# ---------------------------------------------------------------- deblocking
class _RefV(int):
    def to_index(self):
        return RI.TInt(int(self) - 1, "usize")


class FrameBlocksV:
    """FrameBlocks (src/context.rs): the Block of every luma 4x4, indexed by
    PlaneBlockOffset; the fields deblock.rs reads (bsize, txsize, n4_w,
    n4_h, skip, ref_frames, mode, deblock_deltas)."""

    def __init__(self, cols, rows):
        self.cols, self.rows = cols, rows
        self.b = [[None] * cols for _ in range(rows)]

    def place(self, x4, y4, w4, h4, skip, intra):
        bs = H.BlockSize.from_width_and_height(w4 * 4, h4 * 4)
        blk = RI.Struct("Block", {
            "bsize": bs, "txsize": H.TxDims(min(w4 * 4, 64), min(h4 * 4, 64)),
            "n4_w": RI.TInt(w4, "usize"), "n4_h": RI.TInt(h4, "usize"), "skip": bool(skip),
            "ref_frames": [_RefV(0 if intra else 1), _RefV(8)],
            "mode": RI.TInt(0 if intra else 19, "usize"),  # DC_PRED / NEWMV
            "deblock_deltas": [RI.TInt(0, "i8")] * 4})
        for y in range(y4, min(y4 + h4, self.rows)):
            for x in range(x4, min(x4 + w4, self.cols)):
                self.b[y][x] = blk

    def index_any(self, bo):
        o = bo._f["0"]
        return self.b[int(o.y)][int(o.x)]


def _deblock_map(rng, cols, rows, min_lg):
    """A random quadtree of square blocks (64x64 down to 4 << min_lg px):
    per 4x4, lg = log2(width in 4x4 units) and skip."""
    lg = np.zeros((rows, cols), np.uint8)
    sk = np.zeros((rows, cols), np.uint8)
    intra = np.zeros((rows, cols), np.uint8)

    def split(x, y, l):
        n = 1 << l
        if x >= cols or y >= rows:
            return
        if l > min_lg and (rng.random() < 0.55 or x + n > cols or y + n > rows):
            h = n // 2
            for dy in (0, h):
                for dx in (0, h):
                    split(x + dx, y + dy, l - 1)
            return
        lg[y:y + n, x:x + n] = l
        sk[y:y + n, x:x + n] = rng.random() < 0.35
    for y in range(0, rows, 16):
        for x in range(0, cols, 16):
            split(x, y, 4)
    return lg, sk, intra


def _deblock_content(rng, h, w, bd, lg):
    """Smooth ramps with small steps on the 4x4 grid (inside the filters'
    masks at moderate levels) + noise."""
    yy, xx = np.mgrid[0:h, 0:w]
    base = (xx * rng.uniform(0.2, 2) + yy * rng.uniform(0.2, 2)) + 60
    step = np.kron(rng.integers(-6, 7, ((h + 3) // 4, (w + 3) // 4)), np.ones((4, 4)))[:h, :w]
    img = base + step + rng.integers(-2, 3, (h, w))
    img[:, w // 3: w // 3 + 2] += rng.integers(10, 40)  # a real edge
    img = img * (1 << (bd - 8))
    return np.clip(img, 0, (1 << bd) - 1).astype(np.int64)


def gen_deblock(I, rng, out):
    dsrc = RI.Source(REF + "deblock.rs")
    ctx = RI.Source(REF + "context.rs")
    I.sources.append(dsrc)
    I.release = True
    for n in ("BlockOffset", "PlaneBlockOffset"):
        I.globals.vars[n] = RI.StructType(n)
        I.define_impl(n, ctx.impl(n))
    I.globals.vars.update({
        "MI_SIZE_LOG2": RI.TInt(2, "usize"), "MI_SIZE": RI.TInt(4, "usize"),
        "BLOCK_TO_PLANE_SHIFT": RI.TInt(2, "usize"), "SUPERBLOCK_TO_BLOCK_SHIFT": RI.TInt(4, "usize"),
        "MAX_LOOP_FILTER": RI.TInt(63, "usize"),
        "INTRA_FRAME": _RefV(0), "NEARESTMV": RI.TInt(14, "usize"),
        "GLOBALMV": RI.TInt(18, "usize"), "GLOBAL_GLOBALMV": RI.TInt(26, "usize")})
    dp = F(I, "deblock_plane", "deblock.rs")
    cases, planes_in, planes_out, lgs, sks = [], [], [], [], []
    shapes = [(80, 56, 1, 1, 8), (72, 48, 0, 0, 10), (64, 40, 1, 0, 12), (96, 64, 1, 1, 10),
              (56, 72, 0, 0, 8), (88, 48, 1, 1, 12), (64, 64, 1, 1, 8), (48, 40, 0, 0, 12)]
    for n, (W_, H_, xdec, ydec, bd) in enumerate(shapes):
        cols, rows = (W_ + 3) // 4, (H_ + 3) // 4
        min_lg = 0 if n % 2 else 1
        lg, sk, _ = _deblock_map(rng, cols, rows, min_lg)
        fb = FrameBlocksV(cols, rows)
        for y in range(rows):
            for x in range(cols):
                n4 = 1 << int(lg[y, x])
                if x % n4 == 0 and y % n4 == 0:
                    fb.place(x, y, n4, n4, sk[y, x], False)
        levels = [int(v) for v in rng.integers(0, 64, 4)]
        if n % 3 == 0:
            levels[int(rng.integers(0, 4))] = 0
        deb = RI.Struct("DeblockState", {
            "levels": [RI.TInt(v, "u8") for v in levels], "sharpness": RI.TInt(0, "u8"),
            "deltas_enabled": False, "delta_updates_enabled": False,
            "ref_deltas": [RI.TInt(v, "i8") for v in (1, 0, 0, 0, 0, -1, -1, -1)],
            "mode_deltas": [RI.TInt(0, "i8")] * 2, "block_deltas_enabled": False,
            "block_delta_shift": RI.TInt(0, "u8"), "block_delta_multi": False})
        fi = RI.Struct("FrameInvariants", {
            "width": RI.TInt(W_, "usize"), "height": RI.TInt(H_, "usize"),
            "sequence": RI.Struct("Sequence", {"bit_depth": RI.TInt(bd, "usize")})})
        for pli in range(3):
            xd, yd = (xdec, ydec) if pli else (0, 0)
            pw, ph = (W_ + xd) >> xd, (H_ + yd) >> yd
            img = _deblock_content(rng, ph, pw, bd, lg)
            pad = 8
            full = np.pad(img, pad, mode="edge")
            pl = H.Plane.from_full(full, pad, pad, pw, ph, xd, yd)
            ty = "u8" if bd == 8 else "u16"
            pl.data = [RI.TInt(v, ty) for v in pl.data]
            # the callees' `T: Pixel` (inferred by rustc) resolve to the frame's pixel
            I.globals.vars["T"] = prim(bd)
            dp(fi, deb, pl, RI.TInt(pli, "usize"), fb, generics={"T": prim(bd)})
            res = np.array([int(v) for v in pl.data], np.int64).reshape(full.shape)
            res = res[pad:pad + ph, pad:pad + pw]
            cases.append((W_, H_, xdec, ydec, bd, pli, *levels, len(lgs)))
            planes_in.append(img.astype(np.uint16).reshape(-1))
            planes_out.append(res.astype(np.uint16).reshape(-1))
            print("  deblock %dx%d %d-bit dec %d%d plane %d levels %s: %d px changed" % (
                W_, H_, bd, xdec, ydec, pli, levels, int((res != img).sum())))
        lgs.append(lg.reshape(-1))
        sks.append(sk.reshape(-1))
    out["cases"] = np.array(cases, np.int32)
    out["px_in"] = np.concatenate(planes_in)
    out["px_out"] = np.concatenate(planes_out)
    out["lg"] = np.concatenate(lgs)
    out["skip"] = np.concatenate(sks)
    out["map_off"] = np.cumsum([0] + [len(v) for v in lgs]).astype(np.int64)


# ---------------------------------------------------------------- intra prediction
INTRA_MODE_NAMES = ["DC_PRED", "V_PRED", "H_PRED", "D45_PRED", "D135_PRED", "D117_PRED",
                    "D153_PRED", "D207_PRED", "D63_PRED", "SMOOTH_PRED", "SMOOTH_V_PRED",
                    "SMOOTH_H_PRED", "PAETH_PRED", "UV_CFL_PRED", "NEARESTMV", "NEAR0MV",
                    "NEAR1MV", "NEAR2MV", "GLOBALMV", "NEWMV"]


class PModeV(int):
    """A PredictionMode value (src/predict.rs:135-165 order); predict_intra
    runs the reference's method text (bound by intra_env)."""
    predict_fn = None
    pixel = None

    def is_intra(self):
        return int(self) < 14

    def predict_intra(self, *a):
        return PModeV.predict_fn(self, *a, generics={"T": PModeV.pixel})


class _PVariant:
    """PredictionVariant (src/predict.rs:168-184)."""
    NONE, LEFT, TOP, BOTH = 0, 1, 2, 3

    @staticmethod
    def new(x, y):
        x, y = int(x), int(y)
        return 0 if (x, y) == (0, 0) else 1 if y == 0 else 2 if x == 0 else 3


def intra_env(I):
    """Bind the reference's intra predictors: PredictionMode::predict_intra
    (src/predict.rs:202-241), native::predict_intra_inner (:538-597) and the
    Intra trait's default methods (:599-1034) per block size, and
    get_intra_edges (src/partition.rs:500-693)."""
    if getattr(I, "_intra", False):
        return
    I._intra = True
    pr = RI.Source(REF + "predict.rs")
    part = RI.Source(REF + "partition.rs")
    I.sources += [pr, part]
    ns = type("PredictionModeNS", (), {n: PModeV(i) for i, n in enumerate(INTRA_MODE_NAMES)})
    I.globals.vars["PredictionMode"] = ns
    I.globals.vars["PredictionVariant"] = _PVariant
    I.globals.vars["MAX_TX_SIZE"] = RI.TInt(64, "usize")  # src/context.rs:49
    I.globals.vars["MI_SIZE_LOG2"] = RI.TInt(2, "usize")
    I.globals.vars["size_of"] = lambda *a, **k: RI.TInt(1, "usize")
    I.globals.vars["AlignedArray"] = AlignedArray
    I.globals.vars["TileRect"] = RI.StructType("TileRect")
    for n in ("BlockOffset", "TileBlockOffset", "PlaneOffset"):
        I.globals.vars.setdefault(n, RI.StructType(n))
    trait = "pub trait Intra<T>: Dim"
    meths = ["pred_dc", "pred_dc_128", "pred_dc_left", "pred_dc_top", "pred_h", "pred_v",
             "pred_paeth", "pred_smooth", "pred_smooth_h", "pred_smooth_v", "pred_directional"]
    tfn = {m: I.make_fn(pr.fn(m, trait), I.globals) for m in meths}
    cache = {}

    def block_ns(w, h):
        if (w, h) not in cache:
            size = _NS(W=RI.TInt(w, "usize"), H=RI.TInt(h, "usize"))
            b = _NS(W=size.W, H=size.H)
            for m, f in tfn.items():
                setattr(b, m, lambda *a, _f=f, _s=size: _f(*a, bind={"Self": _s, "T": PModeV.pixel}))
            cache[(w, h)] = b
        return cache[(w, h)]
    inner = I.make_fn(pr.fn("predict_intra_inner", "pub(crate) mod native"), I.globals)

    def dispatch(mode, variant, dst, tx_size, bit_depth, ac, angle, edge_buf, cpu):
        # impl_intra!'s table (src/predict.rs:506-535): TX_WxH -> Block WxH
        b = block_ns(int(tx_size.width()), int(tx_size.height()))
        return inner(mode, variant, dst, bit_depth, ac, angle, edge_buf,
                     generics={"T": PModeV.pixel}, bind={"B": b})
    I.globals.vars["dispatch_predict_intra"] = dispatch
    for n in H.BLOCK_NAMES:  # `use BlockSize::*` in partition.rs
        I.globals.vars["BLOCK_" + n] = getattr(H.BlockSize, "BLOCK_" + n)
    I.globals.vars["TxSize"] = type("TxSizeNS", (), {
        "TX_%dX%d" % (1 << TX_W_LOG2[i], 1 << TX_H_LOG2[i]): TxSizeV(i) for i in range(19)})
    PModeV.predict_fn = I.make_fn(pr.fn("predict_intra", "impl PredictionMode"), I.globals)
    I.globals.vars["get_intra_edges"] = (lambda *a, _f=I.make_fn(part.fn("get_intra_edges"),
                                                                 I.globals):
                                         _f(*a, generics={"T": PModeV.pixel}))


# ---------------------------------------------------------------- lookahead
class _MapV:
    """BTreeMap<u64, V> as ContextInner uses it (get_mut / remove / insert /
    index)."""

    def __init__(self, d):
        self.d = d

    def get_mut(self, k):
        return self.d.get(int(RI.deref(k)))

    def remove(self, k):
        return self.d.pop(int(RI.deref(k)), None)

    def insert(self, k, v):
        self.d[int(RI.deref(k))] = v

    def index_any(self, k):
        return self.d[int(RI.deref(k))]


class _FrameTypeNS:
    KEY, INTER = 0, 1


def gen_lookahead(I, rng, out):
    """compute_lookahead_intra_costs (src/api/internal.rs:678-765) and
    compute_block_importances (:823-1077) as methods of a host ContextInner:
    three frames of a moving synthetic clip, output 0 = the current frame
    (KEY, referenced by 1 and 2), 1 references 0, 2 references 0 and 1 (two
    unique references: the propagation splits in half).  Recorded: every
    frame's intra costs, frame 1's block importances after frame 2
    propagated into it (pure f32 propagation) and frame 0's final values
    (after its log2)."""
    intra_env(I)
    api = RI.Source(REF + "api/internal.rs")
    I.sources.append(api)
    I.globals.vars["FrameType"] = _FrameTypeNS
    I.globals.vars["ArrayVec"] = type("ArrayVecNS", (), {"new": staticmethod(lambda: [])})
    I.globals.vars["IMPORTANCE_BLOCK_SIZE"] = RI.TInt(8, "usize")
    satd_ref = F(I, "get_satd_ref")
    intra_m = I.make_fn(api.fn("compute_lookahead_intra_costs"), I.globals)
    imp_m = I.make_fn(api.fn("compute_block_importances"), I.globals)
    for bd, W_, H_ in ((8, 64, 48), (10, 56, 40)):
        PModeV.pixel = prim(bd)
        I.globals.vars["T"] = prim(bd)
        I.globals.vars["get_satd"] = lambda *a, _g={"T": prim(bd)}: satd_ref(*a, generics=_g)
        w_imp, h_imp = W_ // 8, H_ // 8
        pad = 48
        planes, frames = [], []
        base = rng.integers(0, 1 << bd, (H_ + 2 * pad + 16, W_ + 2 * pad + 16))
        base = (np.cumsum(np.cumsum(base, 0), 1) // 97) % (1 << bd)  # smooth-ish texture
        for t in range(3):
            img = base[8 + t: 8 + t + H_, 8 + 2 * t: 8 + 2 * t + W_].copy()
            img = np.clip(img + rng.integers(-3, 4, img.shape), 0, (1 << bd) - 1)
            if t == 2:
                img[8:24, 16:40] = (1 << bd) - 1 - img[8:24, 16:40]  # an occlusion
            full = np.pad(img, pad, mode="edge")
            pl = H.Plane.from_full(full, pad, pad, W_, H_)
            ty = "u8" if bd == 8 else "u16"
            pl.data = [RI.TInt(int(v), ty) for v in pl.data]
            pl.clone = (lambda _p=pl: H.Plane(_p.cfg, list(_p.data)))
            planes.append(img)
            frames.append(RI.Struct("Frame", {"planes": [pl]}))
        fis = {}
        for t in range(3):
            mvs = rng.integers(-20, 21, (h_imp * 2, w_imp * 2, 2))
            mvs[..., 0] += -8 * t  # rows
            mvs[..., 1] += -16 * t
            lmv = [[[H.motion_vector(int(m[0]), int(m[1])) for m in row] for row in mvs],
                   [[H.motion_vector(int(m[0]) // 2, int(m[1]) // 2) for m in row] for row in mvs]]
            refs = {0: [0] * 7, 1: [0] * 7, 2: [0, 1, 0, 1, 0, 0, 0]}[t]
            rec = {0: RI.Struct("Ref", {"frame": frames[0], "output_frameno": RI.TInt(0, "u64")}),
                   1: RI.Struct("Ref", {"frame": frames[1], "output_frameno": RI.TInt(1, "u64")})}
            fis[t] = RI.Struct("FrameInvariants", {
                "invalid": False, "show_existing_frame": False,
                "input_frameno": RI.TInt(t, "u64"),
                "frame_type": _FrameTypeNS.KEY if t == 0 else _FrameTypeNS.INTER,
                "w_in_imp_b": RI.TInt(w_imp, "usize"), "h_in_imp_b": RI.TInt(h_imp, "usize"),
                "sequence": RI.Struct("Sequence", {"bit_depth": RI.TInt(bd, "usize")}),
                "cpu_feature_level": 0,
                "lookahead_intra_costs": [RI.TInt(0, "u32")] * (w_imp * h_imp),
                "block_importances": [np.float32(0)] * (w_imp * h_imp),
                "lookahead_mvs": lmv,
                "ref_frames": [RI.TInt(v, "u8") for v in refs],
                "rec_buffer": RI.Struct("RFS", {"frames": [rec.get(v) for v in range(8)]})})
        fq = _MapV({t: frames[t] for t in range(3)})
        ctx = RI.Struct("ContextInner", {
            "frame_invariants": _MapV(fis), "frame_q": fq,
            "config": RI.Struct("EncoderConfig", {"bit_depth": RI.TInt(bd, "usize")}),
            "output_frameno": RI.TInt(0, "u64")})
        ctx._f["get_rdo_lookahead_frames"] = lambda: RI.It(
            iter([(RI.TInt(t, "u64"), fis[t]) for t in range(3)]))
        for t in range(3):
            intra_m(ctx, RI.TInt(t, "u64"))
        f1_imp = []

        # capture frame 1's importances once frame 2 has propagated into it:
        # the loop visits 2 then 1; frame 1 is removed from the map when its
        # own turn comes, so snapshot at that moment
        orig_remove = ctx._f["frame_invariants"].remove

        def remove(k, _o=orig_remove):
            if int(RI.deref(k)) == 1:
                f1_imp.append([float(v) for v in fis[1]._f["block_importances"]])
            return _o(k)
        ctx._f["frame_invariants"].remove = remove
        imp_m(ctx)
        k = "la_bd%d_" % bd
        out[k + "frames"] = np.array(planes, np.uint16)
        out[k + "mvs"] = np.array([[[[int(m.row), int(m.col)] for m in row] for row in l]
                                   for l in fis[2]._f["lookahead_mvs"]], np.int16)
        out[k + "mvs1"] = np.array([[[int(m.row), int(m.col)] for m in row]
                                    for row in fis[1]._f["lookahead_mvs"][0]], np.int16)
        out[k + "intra"] = np.array([[int(v) for v in fis[t]._f["lookahead_intra_costs"]]
                                     for t in range(3)], np.uint32)
        out[k + "imp1"] = np.array(f1_imp[0], np.float32)
        out[k + "imp0"] = np.array([float(v) for v in fis[0]._f["block_importances"]], np.float32)
        print("lookahead bd%d: intra costs %s..., imp1 sum %.3f, imp0 max %.3f" % (
            bd, out[k + "intra"][0][:4], out[k + "imp1"].sum(), out[k + "imp0"].max()))


# ---------------------------------------------------------------- rate / set_quantizers
def gen_rate(I, rng, out):
    """bexp64 / blog64 / q57 (src/rate.rs) over a grid, and
    FrameInvariants::set_quantizers (src/encoder.rs:865-935) on a host
    FrameInvariants: the CDEF strengths of inter frames (f32 polynomials)
    and lambda / me_lambda, for log_target_q values around rav1e's range."""
    rate = RI.Source(REF + "rate.rs")
    enc = RI.Source(REF + "encoder.rs")
    I.sources += [rate]
    I.globals.vars["CDEF_SEC_STRENGTHS"] = RI.TInt(4, "u8")
    bexp, blog = F(I, "bexp64", "rate.rs"), F(I, "blog64", "rate.rs")
    q57 = F(I, "q57", "rate.rs")
    logs = [0, 1, 7, 100, 1 << 20, (1 << 57) - 1, 3 << 56, -(1 << 57), 123456789012345678,
            -987654321098765]
    logs += [int(v) for v in rng.integers(-(1 << 59), 1 << 59, 40)]
    out["bexp"] = np.array([(v, int(bexp(RI.TInt(v, "i64")))) for v in logs], np.int64)
    ws = [1, 2, 3, 36, 55, 129, 1000, 65535, 1 << 40] + [int(v) for v in
                                                         rng.integers(1, 1 << 62, 30)]
    out["blog"] = np.array([(v, int(blog(RI.TInt(v, "i64")))) for v in ws], np.int64)
    out["q57"] = np.array([(v, int(q57(RI.TInt(v, "i32")))) for v in range(-8, 30)], np.int64)
    sq = I.make_fn(enc.fn("set_quantizers", "impl<T: Pixel> FrameInvariants<T>"), I.globals)
    I.globals.vars["clamp"] = I.make_fn(RI.Source(REF + "util/mod.rs").fn("clamp"), I.globals)
    rows = []
    for bd in (8, 10, 12):
        qlo = int(blog(RI.TInt(4, "i64")))
        qhi = int(blog(RI.TInt(30000, "i64")))
        for lq in list(np.linspace(qlo, qhi, 24).astype(np.int64)) + \
                [int(v) for v in rng.integers(qlo, qhi, 16)]:
            lq = int(lq) - int(q57(RI.TInt(3, "i32")))  # log_target_q = blog64(q) - q57(QSCALE)
            fi = RI.Struct("FrameInvariants", {
                "base_q_idx": RI.TInt(0, "u8"), "dc_delta_q": [RI.TInt(0, "i8")] * 3,
                "ac_delta_q": [RI.TInt(0, "i8")] * 3, "lambda": 0.0, "me_lambda": 0.0,
                "dist_scale": [0.0] * 3, "intra_only": False,
                "cdef_y_strengths": [RI.TInt(0, "u8")] * 8,
                "cdef_uv_strengths": [RI.TInt(0, "u8")] * 8,
                "sequence": RI.Struct("Sequence", {"bit_depth": RI.TInt(bd, "usize")})})
            lam = float(rng.uniform(1, 4000))
            qps = RI.Struct("QuantizerParameters", {
                "log_base_q": RI.TInt(lq, "i64"), "log_target_q": RI.TInt(lq, "i64"),
                "dc_qi": [RI.TInt(100, "u8")] * 3, "ac_qi": [RI.TInt(100, "u8")] * 3,
                "lambda": lam, "dist_scale": [1.0, 1.0, 1.0]})
            sq(fi, qps)
            rows.append((bd, lq, int(fi._f["cdef_y_strengths"][0]),
                         int(fi._f["cdef_uv_strengths"][0])))
    out["cdef_strengths"] = np.array(rows, np.int64)
    print("rate: %d bexp, %d blog, %d set_quantizers" % (len(logs), len(ws), len(rows)))


# ---------------------------------------------------------------- sse_optimize
def gen_sse(I, rng, out):
    """sse_plane (src/deblock.rs:1337-1407) per plane and sse_optimize
    (:1418-1475) on frames with a padded (128-filled, Plane::new)
    reconstruction and source: the tallies and the chosen levels."""
    dsrc = RI.Source(REF + "deblock.rs")
    ctx = RI.Source(REF + "context.rs")
    I.sources.append(dsrc)
    I.release = True
    for n in ("BlockOffset", "PlaneBlockOffset"):
        I.globals.vars[n] = RI.StructType(n)
        I.define_impl(n, ctx.impl(n))
    I.globals.vars.update({
        "MI_SIZE_LOG2": RI.TInt(2, "usize"), "MI_SIZE": RI.TInt(4, "usize"),
        "BLOCK_TO_PLANE_SHIFT": RI.TInt(2, "usize"), "SUPERBLOCK_TO_BLOCK_SHIFT": RI.TInt(4, "usize"),
        "MAX_LOOP_FILTER": RI.TInt(63, "usize"), "PLANES": RI.TInt(3, "usize"),
        "INTRA_FRAME": _RefV(0), "NEARESTMV": RI.TInt(14, "usize"),
        "GLOBALMV": RI.TInt(18, "usize"), "GLOBAL_GLOBALMV": RI.TInt(26, "usize")})
    sp = F(I, "sse_plane", "deblock.rs")
    so = F(I, "sse_optimize", "deblock.rs")
    cases, recs, srcs, lgs, sks, tallies, levels_out = [], [], [], [], [], [], []
    shapes = [(64, 48, 1, 1, 8, 2), (72, 40, 0, 0, 10, 3), (56, 64, 1, 0, 12, 1),
              (80, 56, 1, 1, 10, 4), (48, 48, 1, 1, 8, 0), (64, 32, 0, 0, 8, 6),
              (96, 64, 1, 1, 12, 2), (40, 56, 1, 1, 10, 8)]
    for n, (W_, H_, xdec, ydec, bd, amp) in enumerate(shapes):
        cols, rows = (W_ + 3) // 4, (H_ + 3) // 4
        lg, sk, _ = _deblock_map(rng, cols, rows, 0 if n % 2 else 1)
        fb = FrameBlocksV(cols, rows)
        for y in range(rows):
            for x in range(cols):
                n4 = 1 << int(lg[y, x])
                if x % n4 == 0 and y % n4 == 0:
                    fb.place(x, y, n4, n4, sk[y, x], False)
        pad = 8
        ty = "u8" if bd == 8 else "u16"
        planes = {"rec": [], "src": []}
        for pli in range(3):
            xd, yd = (xdec, ydec) if pli else (0, 0)
            pw, ph = (W_ + xd) >> xd, (H_ + yd) >> yd
            yy, xx = np.mgrid[0:ph, 0:pw]
            src = xx * rng.uniform(0.3, 2) + yy * rng.uniform(0.3, 2) + 50 + rng.integers(-3, 4, (ph, pw))
            # the reconstruction: the source + a step per 4x4 + noise (amp 0: exact)
            step = np.kron(rng.integers(-amp, amp + 1, ((ph + 3) // 4, (pw + 3) // 4)),
                           np.ones((4, 4)))[:ph, :pw]
            rec = src + step + (rng.integers(-1, 2, (ph, pw)) if amp else 0)
            for name, img in (("src", src), ("rec", rec)):
                img = np.clip(img * (1 << (bd - 8)), 0, (1 << bd) - 1).astype(np.int64)
                full = np.full((ph + 2 * pad, pw + 2 * pad), 128, np.int64)
                full[pad:pad + ph, pad:pad + pw] = img
                pl = H.Plane.from_full(full, pad, pad, pw, ph, xd, yd)
                pl.data = [RI.TInt(v, ty) for v in pl.data]
                planes[name].append(pl)
                (recs if name == "rec" else srcs).append(img.astype(np.uint16).reshape(-1))
        fi = RI.Struct("FrameInvariants", {
            "width": RI.TInt(W_, "usize"), "height": RI.TInt(H_, "usize"),
            "sequence": RI.Struct("Sequence", {"bit_depth": RI.TInt(bd, "usize")})})
        I.globals.vars["T"] = prim(bd)
        tl = []
        for pli in range(3):
            v = [RI.TInt(0, "i64") for _ in range(65)]
            h = [RI.TInt(0, "i64") for _ in range(65)]
            sp(fi, planes["rec"][pli], planes["src"][pli], v, h, RI.TInt(pli, "usize"), fb,
               generics={"T": prim(bd)})
            tl.append([int(x) for x in v] + [int(x) for x in h])
        deb = RI.Struct("DeblockState", {"levels": [RI.TInt(0, "u8")] * 4})
        fs = RI.Struct("FrameState", {
            "rec": RI.Struct("Frame", {"planes": planes["rec"]}),
            "input": RI.Struct("Frame", {"planes": planes["src"]}), "deblock": deb})
        so(fi, fs, fb, generics={"T": prim(bd)})
        lv = [int(x) for x in fs._f["deblock"]._f["levels"]]
        cases.append((W_, H_, xdec, ydec, bd, len(lgs)))
        lgs.append(lg.reshape(-1))
        sks.append(sk.reshape(-1))
        tallies.append(tl)
        levels_out.append(lv)
        print("  sse %dx%d %d-bit dec %d%d amp %d: levels %s" % (W_, H_, bd, xdec, ydec, amp, lv))
    out["cases"] = np.array(cases, np.int32)
    out["rec"] = np.concatenate(recs)
    out["src"] = np.concatenate(srcs)
    out["lg"] = np.concatenate(lgs)
    out["skip"] = np.concatenate(sks)
    out["map_off"] = np.cumsum([0] + [len(v) for v in lgs]).astype(np.int64)
    out["tally"] = np.array(tallies, np.int64)  # [case][plane][v 65 | h 65]
    out["levels"] = np.array(levels_out, np.int32)


SECTIONS = {"mc": gen_mc, "dist": gen_dist, "rdo": gen_rdo, "me": gen_me, "quant": gen_quant,
            "tx": gen_tx, "ds": gen_ds, "cdef": gen_cdef, "deblock": gen_deblock,
            "lookahead": gen_lookahead, "rate": gen_rate, "sse": gen_sse}


def main(argv):
    names = argv or list(SECTIONS)
    os.makedirs(OUT, exist_ok=True)
    for n in names:
        I = make_interp()
        # the sections that predate cdef keep the seeds they were generated with
        old = sorted(set(SECTIONS) - {"cdef", "deblock", "lookahead", "rate", "sse"})
        rng = np.random.default_rng(0x5EED + (old.index(n) if n in old else
                                              100 + sorted(set(SECTIONS) - set(old)).index(n)))
        random.seed(1)
        out = {}
        t = time.time()
        SECTIONS[n](I, rng, out)
        np.savez_compressed(os.path.join(OUT, "ref_%s.npz" % n), **out)
        print("%s: %.1f s" % (n, time.time() - t))


if __name__ == "__main__":
    main(sys.argv[1:])
