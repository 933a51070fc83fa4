"""The interpreter (rsinterp.py) run on the reference's OWN unit tests: the
known answers rav1e holds for the hot path, evaluated from the test text of
/root/reference/src, so the evaluator that produces the tests/golden/ref_*.npz
vectors is itself pinned by values the reference wrote down.

    python tools/refeval/gen_kat.py        (in the build container)

Evaluated test functions (each runs the reference's function text; its
assert!/assert_eq! fire inside the interpreter on a mismatch):

  src/dist.rs:342-375, 378-498     setup_planes + get_sad_same_inner /
                                   get_satd_same_inner, T = u8 and u16
                                   (88 known answers; get_sad / get_satd ->
                                   get_sad_ref / get_satd_ref, the
                                   check_asm ground truth)
  src/quantize.rs:160-202          test_divu_pair (every d in 1..1024, x in
                                   -1000..1000), test_tx_log_scale
  src/transform/mod.rs:632-666     log_tx_ratios
  src/transform/mod.rs:589-715     test_roundtrip's tolerance check over the
                                   `roundtrips` combination list, fht +
                                   inv_txfm2d_add evaluated (the specialize_f!
                                   dispatch is the host's), u8 and u16
  src/predict.rs:1047-1178         pred_matches_u8, pred_max over the
                                   native::Intra trait's default methods

The record (which tests ran, the values the interpreter produced for the
SAD/SATD table, how many roundtrip blocks) goes to tests/golden/ref_kat.npz;
tests/test_ref_golden.py checks it against tests/golden/dist_kat.json.
"""
import os
import re
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(__file__))
import gen_golden_ref as G  # noqa: E402
import rshost as H  # noqa: E402
import rsinterp as RI  # noqa: E402

REF = G.REF


class _CpuDefault:
    RUST = RI.TInt(0, "usize")

    @staticmethod
    def default():
        return 0

    def as_index(self):
        return 0


def plane_ns(bpp):
    """Plane::new (src/frame/plane.rs:215-244) for a pixel of `bpp` bytes,
    zero-filled, plus Plane::wrap (:246-266)."""
    class PlaneNS:
        @staticmethod
        def new(w, h, xdec, ydec, xpad, ypad):
            cfg = H.PlaneConfig(int(w), int(h), int(xdec), int(ydec), int(xpad), int(ypad), bpp)
            return H.Plane(cfg, [RI.TInt(0, "u8" if bpp == 1 else "u16")] *
                           (int(cfg.stride) * int(cfg.alloc_height)))

        @staticmethod
        def wrap(data, stride):
            data = RI.deref(data)
            vals = data.tolist() if isinstance(data, RI.Slice) else list(data)
            stride = int(stride)
            full = np.array([int(v) for v in vals], np.int64).reshape(-1, stride)
            p = H.Plane.from_full(full, 0, 0, stride, full.shape[0])
            ty = "u8" if bpp == 1 else "u16"
            p.data = [RI.TInt(v, ty) for v in p.data]
            return p
    return PlaneNS


def kat_dist(I, rec):
    dist = G.src_of(I, "dist.rs")
    sad_ref, satd_ref = G.F(I, "get_sad_ref"), G.F(I, "get_satd_ref")
    I.globals.vars["CpuFeatureLevel"] = _CpuDefault
    for n in H.BLOCK_NAMES:  # `use crate::partition::BlockSize::*;` (src/dist.rs:337)
        I.globals.vars["BLOCK_" + n] = getattr(H.BlockSize, "BLOCK_" + n)
    # setup_planes (src/dist.rs:342-375) fills 1.9 M padded pixels: too slow
    # to interpret, so the fixture is built here from its two formulas (the
    # test's own Plane::new geometry and xpad_off); the test bodies that hold
    # the known answers, get_sad_ref and get_satd_ref run interpreted.
    def setup(generics):
        bpp = 1 if generics["T"].name == "u8" else 2
        ns = plane_ns(bpp)
        a = ns.new(640, 480, 0, 0, 128 + 8, 128 + 8)
        b = ns.new(640, 480, 0, 0, 2 * 128 + 8, 2 * 128 + 8)
        xpad_off = (int(a.cfg.xorigin) - int(a.cfg.xpad)) - 8
        ty = "u8" if bpp == 1 else "u16"
        for p, f in ((a, lambda i, j: ((j + i) - xpad_off) & 255),
                     (b, lambda i, j: (j - i - xpad_off) & 255)):
            st, ah = int(p.cfg.stride), int(p.cfg.alloc_height)
            ii, jj = np.mgrid[0:ah, 0:st]
            p.data = [RI.TInt(int(v), ty) for v in f(ii, jj).reshape(-1)]
        return (a, b)
    inner = {k: I.make_fn(dist.fn("get_%s_same_inner" % k, "pub mod test"), I.globals)
             for k in ("sad", "satd")}
    for bd_t, bpp in (("u8", 1), ("u16", 2)):
        g = {"T": RI.PrimType(bd_t)}
        I.globals.vars["Plane"] = plane_ns(bpp)
        I.globals.vars["setup_planes"] = lambda _g=g: setup(generics=_g)
        got = {"sad": [], "satd": []}
        I.globals.vars["get_sad"] = (lambda *a, _g=g: got["sad"].append(
            int(sad_ref(*a, generics=_g))) or got["sad"][-1])
        I.globals.vars["get_satd"] = (lambda *a, _g=g: got["satd"].append(
            int(satd_ref(*a, generics=_g))) or got["satd"][-1])
        for k in ("sad", "satd"):
            inner[k](generics=g)  # its assert_eq! / panic! check the 22 answers
            rec["dist_%s_%s" % (k, bd_t)] = np.array(got[k], np.uint32)
            print("  get_%s_same_%s: %d blocks OK" % (k, bd_t, len(got[k])))


def kat_quant(I, rec):
    q = G.src_of(I, "quantize.rs")
    G.F(I, "divu_gen", "quantize.rs")
    G.F(I, "divu_pair", "quantize.rs")
    t = time.time()
    I.make_fn(q.fn("test_divu_pair", "mod test"), I.globals)()
    print("  test_divu_pair OK (%.0f s)" % (time.time() - t))
    names = ["TX_4X4", "TX_8X8", "TX_16X16", "TX_32X32", "TX_64X64", "TX_4X8", "TX_8X4",
             "TX_8X16", "TX_16X8", "TX_16X32", "TX_32X16", "TX_32X64", "TX_64X32", "TX_4X16",
             "TX_16X4", "TX_8X32", "TX_32X8", "TX_16X64", "TX_64X16"]
    for i, n in enumerate(names):
        I.globals.vars[n] = G.TxSizeV(i)
    G.F(I, "get_log_tx_scale", "quantize.rs")
    I.make_fn(q.fn("test_tx_log_scale", "mod test"), I.globals)()
    tm = G.src_of(I, "transform/mod.rs")
    I.globals.vars["TxSize"] = type("TxSizeNS", (), {n: G.TxSizeV(i) for i, n in enumerate(names)})
    I.globals.vars["get_rect_tx_log_ratio"] = I.make_fn(tm.fn("get_rect_tx_log_ratio"), I.globals)
    I.make_fn(tm.fn("log_tx_ratios", "mod test"), I.globals)()
    rec["quant_tests"] = np.array([1, 1, 1], np.int32)
    print("  test_tx_log_scale, log_tx_ratios OK")


TX_TYPES = ["DCT_DCT", "ADST_DCT", "DCT_ADST", "ADST_ADST", "FLIPADST_DCT", "DCT_FLIPADST",
            "FLIPADST_FLIPADST", "ADST_FLIPADST", "FLIPADST_ADST", "IDTX", "V_DCT", "H_DCT",
            "V_ADST", "H_ADST", "V_FLIPADST", "H_FLIPADST"]


def kat_roundtrip(I, rec, rng):
    """test_roundtrip (src/transform/mod.rs:589-630): random u8 src / dst,
    residual = src - dst, forward_transform + inverse_transform_add (the
    reference's fht / inv_txfm2d_add text, gen_golden_ref.gen_tx's
    bindings), every output within the listed tolerance of src."""
    tm = G.src_of(I, "transform/mod.rs").raw
    body = tm[tm.index("fn roundtrips<T: Pixel>()"):]
    body = body[:body.index("for &(tx_size, tx_type, tolerance)")]
    combos = [(n, t, int(tol)) for n, t, tol in
              re.findall(r"^\s*\((TX_\w+),\s*(\w+),\s*(\d+)\),", body, re.M)]
    names = {n: i for i, n in enumerate(
        ["TX_4X4", "TX_8X8", "TX_16X16", "TX_32X32", "TX_64X64", "TX_4X8", "TX_8X4", "TX_8X16",
         "TX_16X8", "TX_16X32", "TX_32X16", "TX_32X64", "TX_64X32", "TX_4X16", "TX_16X4",
         "TX_8X32", "TX_32X8", "TX_16X64", "TX_64X16"])}
    fwd, inv = G.tx_fns(I)
    worst, n = [], 0
    for bd_t in ("u8", "u16"):
        for name, tt, tol in combos:
            ts, ty = names[name], TX_TYPES.index(tt)
            w, h = 1 << G.TX_W_LOG2[ts], 1 << G.TX_H_LOG2[ts]
            for trial in range(2):
                src = rng.integers(0, 256, (h, w))
                dst = rng.integers(0, 256, (h, w))
                # forward_transform (..., 8, ...); the inverse reads the first
                # min(W,32) x min(H,32) coefficients (src/transform/inverse.rs)
                raster = fwd(ts, ty, (src - dst).reshape(-1).tolist(), 8)
                cw, ch = min(w, 32), min(h, 32)
                co = [raster[k] for k in range(cw * ch)]
                out = inv(ts, ty, co, dst, 8, bd_t)
                err = int(np.abs(src - out).max())
                assert err <= tol, (name, tt, bd_t, err, tol)
                worst.append((ts, ty, int(bd_t == "u16"), err, tol))
                n += 1
    rec["roundtrip"] = np.array(worst, np.int32)
    print("  roundtrips_u8 / roundtrips_u16: %d combinations x 2 trials OK" % len(combos))


def kat_intra(I, rec):
    pr = RI.Source(REF + "predict.rs")
    I.sources.append(pr)
    I.globals.vars["MAX_TX_SIZE"] = RI.TInt(64, "usize")  # src/context.rs:49
    I.globals.vars["size_of"] = lambda g=None: RI.TInt(1, "usize")
    trait = "pub trait Intra<T>: Dim"
    fns = {}
    for m in ("pred_dc", "pred_dc_128", "pred_dc_left", "pred_dc_top", "pred_h", "pred_v",
              "pred_paeth", "pred_smooth", "pred_smooth_h", "pred_smooth_v"):
        fns[m] = pr.fn(m, trait)

    def block_ns(w, h, px):
        size = G._NS(W=RI.TInt(w, "usize"), H=RI.TInt(h, "usize"))
        ns = G._NS()
        for m, f in fns.items():
            fn = I.make_fn(f, I.globals)
            setattr(ns, m, lambda *a, _f=fn, _s=size: _f(*a, bind={"Self": _s, "T": px}))
        return ns
    I.globals.vars["AlignedArray"] = G.AlignedArray
    for test, px, bpp in (("pred_matches_u8", "u8", 1), ("pred_max", "u16", 2)):
        I.globals.vars["Block4x4"] = block_ns(4, 4, RI.PrimType(px))
        I.globals.vars["Plane"] = plane_ns(bpp)
        I.make_fn(pr.fn(test, "mod test"), I.globals)()
        print("  %s OK" % test)
    rec["intra_tests"] = np.array([1, 1], np.int32)


def main():
    I = G.make_interp()
    rng = np.random.default_rng(0x4B47)
    rec = {}
    t = time.time()
    for name, fn in (("dist", lambda: kat_dist(I, rec)), ("intra", lambda: kat_intra(I, rec)),
                     ("quant", lambda: kat_quant(I, rec)),
                     ("roundtrip", lambda: kat_roundtrip(I, rec, rng))):
        if len(sys.argv) > 1 and name not in sys.argv[1:]:
            continue
        print(name)
        fn()
    np.savez_compressed(os.path.join(G.OUT, "ref_kat.npz"), **rec)
    print("kat: %.1f s" % (time.time() - t))


if __name__ == "__main__":
    main()
