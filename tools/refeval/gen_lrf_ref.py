"""Golden vectors for loop restoration's self-guided filter, produced by
RUNNING the reference's own Rust function text (rsinterp.py) -- run in the
build container (needs /root/reference):

    python tools/refeval/gen_lrf_ref.py

Functions evaluated (src/lrf.rs): setup_integral_image (:483-580, with
VertPaddedIter / HorzPaddedIter :336-481), sgrproj_stripe_filter (:582-748)
and sgrproj_solve (:764-965) over native::sgrproj_box_ab_r1/_r2,
sgrproj_box_f_r0/_r1/_r2 (:156-302), sgrproj_sum_finish and
get_integral_square (:305-334); RestorationState::new (:1197-1343) for the
unit geometry.  Only the resulting numbers are written (tests/golden/
ref_lrf.npz); tests/test_lrf.py checks oracle/orc_lrf.c against them.
"""
import os
import re
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(__file__))
import gen_golden_ref as G  # noqa: E402
import rshost as H  # noqa: E402
import rsinterp as RI  # noqa: E402

OUT = os.path.join(G.ROOT, "tests", "golden", "ref_lrf.npz")
IIS = 264  # STRIPE_IMAGE_STRIDE = 256 + 6 + 2 (src/lrf.rs:87)
PAD = 8


def interp():
    I = G.make_interp()
    I.release = True  # u32 sums wrap (wrapping_add), release arithmetic
    I.sources.append(RI.Source(G.REF + "lrf.rs"))
    src = G.src_of(I, "lrf.rs")
    for n in ("VertPaddedIter", "HorzPaddedIter"):
        fns = []
        for m in re.finditer(r"\bimpl\b[^{;]*\b%s\s*(<[^>]*>)?\s*\{" % n, src.src):
            fns += RI.parse_impl_fns(RI.find_item(src.src, "impl", n, m.start()))
        I.globals.vars[n] = RI.StructType(n)
        I.define_impl(n, fns)
    return I


def u(v):
    return RI.TInt(int(v), "usize")


def plane(arr, bd):
    """A plane of (h + 2 PAD) x (w + 2 PAD) with the visible area at PAD."""
    h, w = arr.shape[0] - 2 * PAD, arr.shape[1] - 2 * PAD
    pl = H.Plane.from_full(arr, PAD, PAD, w, h)
    ty = "u8" if bd == 8 else "u16"
    pl.data = [RI.TInt(int(v), ty) for v in pl.data]
    return pl


def content(rng, h, w, bd):
    """Smooth ramps + texture + noise: the box variances span the strength
    tables' whole range (z from 0 past 255)."""
    yy, xx = np.mgrid[0:h, 0:w]
    a = rng.uniform(0, np.pi)
    img = (np.cos(a) * xx + np.sin(a) * yy) * rng.uniform(0.5, 6)
    img = img + rng.integers(-12, 13, (h, w)) * rng.uniform(0.2, 3)
    img = img + (xx > w // 2) * rng.integers(0, 60) + (1 << bd) // 4 / (1 << (bd - 8))
    img = img * (1 << (bd - 8))
    return np.clip(np.rint(img), 0, (1 << bd) - 1).astype(np.int64)


def main():
    I = interp()
    setup = G.F(I, "setup_integral_image", "lrf.rs")
    stripe = G.F(I, "sgrproj_stripe_filter", "lrf.rs")
    solve = G.F(I, "sgrproj_solve", "lrf.rs")
    rng = np.random.default_rng(20260518)
    cases, planes_cd, planes_db, planes_in, iis, sqs, filt, xqds = [], [], [], [], [], [], [], []
    Hh, Ww = 48, 56
    # (x0, y0, stripe_w, stripe_h, crop_w, crop_h): interior, left edge, the
    # crop (frame) edge on the right / bottom, odd heights, short stripes
    geo = [(8, 8, 24, 16, None, None), (0, 0, 20, 17, None, None), (30, 10, 26, 21, None, None),
           (16, 36, 16, 12, None, None), (0, 20, 32, 9, None, None), (40, 4, 12, 31, 14, 40),
           (4, 2, 28, 14, 30, 16)]
    n = 0
    for bd in (8, 10, 12):
        fi = G.Fi(bd)
        for (x0, y0, sw, sh, cw, ch) in geo:
            cw = Ww - x0 if cw is None else cw
            ch = Hh - y0 if ch is None else ch
            full_cd = np.full((Hh + 2 * PAD, Ww + 2 * PAD), 128, np.int64)
            full_cd[PAD:PAD + Hh, PAD:PAD + Ww] = content(rng, Hh, Ww, bd)
            full_db = full_cd.copy()
            full_db[PAD:PAD + Hh, PAD:PAD + Ww] = np.clip(
                full_cd[PAD:PAD + Hh, PAD:PAD + Ww] + rng.integers(-4, 5, (Hh, Ww)) * (1 << (bd - 8)),
                0, (1 << bd) - 1)
            full_in = full_cd.copy()
            full_in[PAD:PAD + Hh, PAD:PAD + Ww] = np.clip(
                full_cd[PAD:PAD + Hh, PAD:PAD + Ww] + rng.integers(-9, 10, (Hh, Ww)) * (1 << (bd - 8)),
                0, (1 << bd) - 1)
            cd, db, inp = plane(full_cd, bd), plane(full_db, bd), plane(full_in, bd)
            po = RI.Struct("PlaneOffset", {"x": RI.TInt(x0, "isize"), "y": RI.TInt(y0, "isize")})
            nrow = 4 + sh + (sh & 1) + 2
            buf = RI.Struct("IntegralImageBuffer", {
                "integral_image": [RI.TInt(0, "u32") for _ in range(IIS * (nrow + 1))],
                "sq_integral_image": [RI.TInt(0, "u32") for _ in range(IIS * (nrow + 1))]})
            g = {"T": RI.PrimType("u8" if bd == 8 else "u16")}
            setup(buf, u(IIS), u(cw), u(ch), u(sw), u(sh), cd.slice(po), db.slice(po), generics=g)
            ii = np.array([int(v) for v in buf._f["integral_image"]], np.uint32)[:IIS * nrow]
            sq = np.array([int(v) for v in buf._f["sq_integral_image"]], np.uint32)[:IIS * nrow]
            for k in range(2):
                s = int(rng.integers(0, 16))
                xq = [int(rng.integers(-96, 32)), int(rng.integers(-32, 96))]
                outp = plane(np.zeros_like(full_cd), bd)
                stripe(u(s), [RI.TInt(xq[0], "i8"), RI.TInt(xq[1], "i8")], fi, buf, u(IIS), u(sw),
                       u(sh), cd.slice(po), outp.slice(po), generics=g)
                o = np.array([int(v) for v in outp.data], np.int64).reshape(full_cd.shape)
                filt.append(o[PAD + y0:PAD + y0 + sh, PAD + x0:PAD + x0 + sw].ravel().tolist())
                # sgrproj_solve: its integral image is the unit's own
                # (cdeffed = deblocked, crop = the unit, rdo_loop_decision
                # :2065-2075)
                r2 = sgr_solve(I, setup, solve, fi, cd, inp, x0, y0, sw, sh, s, g)
                cases.append((bd, x0, y0, sw, sh, cw, ch, s, xq[0], xq[1]))
                xqds.append(r2)
            planes_cd.append(full_cd)
            planes_db.append(full_db)
            planes_in.append(full_in)
            iis.append(np.pad(ii, (0, IIS * 48 - ii.size)))
            sqs.append(np.pad(sq, (0, IIS * 48 - sq.size)))
            n += 1
            print("lrf case", n, bd, (x0, y0, sw, sh, cw, ch), flush=True)
    maxlen = max(len(f) for f in filt)
    np.savez_compressed(
        OUT, cases=np.array(cases, np.int32), cd=np.array(planes_cd, np.uint16),
        db=np.array(planes_db, np.uint16), inp=np.array(planes_in, np.uint16),
        ii=np.array(iis, np.uint32), sq=np.array(sqs, np.uint32),
        filt=np.array([f + [0] * (maxlen - len(f)) for f in filt], np.uint16),
        xqd=np.array(xqds, np.int32), pad=np.int32(PAD), iis=np.int32(IIS))
    print("wrote", OUT)


def sgr_solve(I, setup, solve, fi, cd, inp, x0, y0, w, h, s, g):
    po = RI.Struct("PlaneOffset", {"x": RI.TInt(x0, "isize"), "y": RI.TInt(y0, "isize")})
    SIS = 264  # SOLVE_IMAGE_STRIDE
    nrow = 4 + h + (h & 1) + 2
    buf = RI.Struct("IntegralImageBuffer", {
        "integral_image": [RI.TInt(0, "u32") for _ in range(SIS * (nrow + 1))],
        "sq_integral_image": [RI.TInt(0, "u32") for _ in range(SIS * (nrow + 1))]})
    setup(buf, u(SIS), u(w), u(h), u(w), u(h), cd.slice(po), cd.slice(po), generics=g)
    I.globals.vars["SOLVE_IMAGE_STRIDE"] = u(SIS)
    r = solve(u(s), fi, buf, inp.slice(po), cd.slice(po), u(w), u(h), generics=g)
    return [int(r[0]), int(r[1])]


if __name__ == "__main__":
    main()
