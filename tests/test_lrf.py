"""Loop restoration, self-guided filter (src/lrf.rs): the oracle's
restatement (oracle/orc_lrf.c) pinned by vectors from evaluating the
reference's own setup_integral_image, sgrproj_stripe_filter and
sgrproj_solve (tests/golden/ref_lrf.npz, made by
tools/refeval/gen_lrf_ref.py: every bit depth, stripes at the frame's left
and bottom / right crop edges, odd heights, deblocked rows outside the
stripe, all 16 parameter sets), plus the unit geometry of
RestorationState::new and the rate helpers against hand-derived values."""
import ctypes as C
import os

import numpy as np
import pytest

from tests import oracle_lib as O

GOLD = os.path.join(os.path.dirname(__file__), "golden", "ref_lrf.npz")


def _lib():
    L = O.lib()
    vp, sz, i32 = C.c_void_p, C.c_ssize_t, C.c_int
    L.orc_lrf_integral.argtypes = [vp, sz, vp, sz] + [i32] * 7 + [vp, vp, i32]
    L.orc_sgr_stripe_filter.argtypes = [i32, vp, i32, vp, vp, i32, i32, i32, vp, sz, vp, sz, i32]
    L.orc_sgr_solve.argtypes = [i32, i32, vp, vp, i32, vp, sz, vp, sz, i32, i32, i32, vp]
    L.orc_lrf_config.argtypes = [i32] * 8 + [vp]
    L.orc_symbol_bits.restype = C.c_uint32
    L.orc_symbol_bits.argtypes = [C.c_uint32, vp, i32]
    L.orc_lrf_rate.restype = C.c_uint32
    L.orc_lrf_rate.argtypes = [vp, vp, i32, vp]
    return L


def _cases():
    g = np.load(GOLD)
    pad = int(g["pad"])
    k = 0
    for n in range(len(g["cd"])):
        for _ in range(2):
            yield g, n, k, pad
            k += 1


def _px(a, bd):
    return np.ascontiguousarray(a.astype(np.uint8 if bd == 8 else np.uint16))


@pytest.mark.parametrize("part", ["integral", "filter", "solve"])
def test_sgrproj_vs_reference(part):
    L = _lib()
    iis = 264
    checked = 0
    for g, n, k, pad in _cases():
        bd, x0, y0, sw, sh, cw, ch, s, xq0, xq1 = (int(v) for v in g["cases"][k])
        hbd = int(bd > 8)
        cd, db, inp = (_px(g[a][n], bd) for a in ("cd", "db", "inp"))
        st = cd.shape[1]
        org = pad * st + pad  # the visible origin
        nrow = 4 + sh + (sh & 1) + 2
        ii = np.zeros(iis * nrow, np.uint32)
        sq = np.zeros(iis * nrow, np.uint32)
        L.orc_lrf_integral(O.ptr(cd, org), st, O.ptr(db, org), st, hbd, x0, y0, cw, ch, sw, sh,
                           O.ptr(ii), O.ptr(sq), iis)
        if part == "integral":
            if k % 2 == 0:  # one image per geometry
                np.testing.assert_array_equal(ii, g["ii"][n][:iis * nrow], err_msg=str(g["cases"][k]))
                np.testing.assert_array_equal(sq, g["sq"][n][:iis * nrow])
                checked += 1
            continue
        if part == "filter":
            out = np.zeros((sh, sw), cd.dtype)
            xqd = np.array([xq0, xq1], np.int8)
            o = org + y0 * st + x0
            L.orc_sgr_stripe_filter(s, O.ptr(xqd), bd, O.ptr(ii), O.ptr(sq), iis, sw, sh,
                                    O.ptr(cd, o), st, O.ptr(out), sw, hbd)
            np.testing.assert_array_equal(out.ravel(), g["filt"][k][:sw * sh],
                                          err_msg=str(g["cases"][k]))
            checked += 1
            continue
        # solve: the unit's own integral image (cdeffed = deblocked, the
        # crop = the unit), as rdo_loop_decision sets it up (:2065-2075)
        nrow2 = 4 + sh + (sh & 1) + 2
        ii2 = np.zeros(iis * nrow2, np.uint32)
        sq2 = np.zeros(iis * nrow2, np.uint32)
        L.orc_lrf_integral(O.ptr(cd, org), st, O.ptr(cd, org), st, hbd, x0, y0, sw, sh, sw, sh,
                           O.ptr(ii2), O.ptr(sq2), iis)
        xqd = np.zeros(2, np.int8)
        o = org + y0 * st + x0
        L.orc_sgr_solve(s, bd, O.ptr(ii2), O.ptr(sq2), iis, O.ptr(inp, o), st, O.ptr(cd, o), st, hbd,
                        sw, sh, O.ptr(xqd))
        assert [int(xqd[0]), int(xqd[1])] == [int(v) for v in g["xqd"][k]], g["cases"][k]
        checked += 1
    assert checked >= 21


def test_lrf_config_units():
    """RestorationState::new (src/lrf.rs:1197-1343) on the BASELINE shapes:
    base_q_idx <= 160 gives 64 x 64 luma units and, in 4:2:0, 32 x 32
    chroma ones (one superblock each); larger quantizers larger units."""
    L = _lib()
    out = np.zeros((3, 6), np.int32)
    L.orc_lrf_config(3840, 2160, 1, 1, 100, 1, 8, 34, O.ptr(out))
    assert out[0].tolist() == [64, 0, 0, 64, 60, 34]
    assert out[1].tolist() == [32, 0, 0, 32, 60, 34]
    L.orc_lrf_config(3840, 2160, 0, 0, 134, 1, 8, 34, O.ptr(out))
    assert out[1].tolist() == [64, 0, 0, 64, 60, 34]
    L.orc_lrf_config(1920, 1080, 1, 1, 180, 0, 0, 0, O.ptr(out))
    assert out[0][:3].tolist() == [128, 1, 1] and out[0][4:].tolist() == [15, 8]
    L.orc_lrf_config(1920, 1080, 1, 1, 220, 0, 0, 0, O.ptr(out))
    assert out[0][0] == 256


def test_lrf_rate_helpers():
    """symbol_bits at a fresh writer (rng 0x8000, cnt -9) over the default
    switchable-restore CDF: the three symbols' costs follow their
    probabilities (9413, 13168, 10187 of 32768) at OD_BITRES precision."""
    L = _lib()
    cdf = np.array([32768 - 9413, 32768 - 22581, 0, 0], np.uint16)
    bits = [L.orc_symbol_bits(s, O.ptr(cdf), 3) for s in range(3)]
    ideal = [-np.log2(p / 32768) * 8 for p in (9413, 13168, 10187)]
    for b, i in zip(bits, ideal):
        assert abs(b - i) <= 8, (bits, ideal)
    ref = np.array([-32, 31], np.int8)
    none = L.orc_lrf_rate(O.ptr(cdf), O.ptr(ref), -1, O.ptr(np.zeros(2, np.int8)))
    assert none == bits[0]
    # a set with both radii: the symbol, 4 bits of set, two subexp codes
    r = L.orc_lrf_rate(O.ptr(cdf), O.ptr(ref), 0, O.ptr(np.array([-32, 31], np.int8)))
    assert r > bits[2] + 4 * 8


@pytest.mark.gpu
def test_gpu_lrf_stripe_filter_vs_reference():
    """The device's loop-restoration filter code (lrf_filter_kernel's chunk
    body, through rv_lrf_stripe_filter) on every stripe of the
    reference-evaluated vectors: setup_integral_image's view and
    sgrproj_stripe_filter at 8/10/12 bits, edge crops, odd heights, all 16
    sets -- bit-exact against tests/golden/ref_lrf.npz, not through the
    oracle."""
    import rav1e_amd as R
    R.require_device(0)
    checked = 0
    for g, n, k, pad in _cases():
        bd, x0, y0, sw, sh, cw, ch, s, xq0, xq1 = (int(v) for v in g["cases"][k])
        cd, db = (_px(g[a][n], bd) for a in ("cd", "db"))
        # (cw, ch): what is left from (x0, y0) to the crop's edge; the
        # device entry takes the crop itself
        fw, fh = x0 + cw, y0 + ch
        pc = R.DevicePlane.from_full(cd, pad, pad, fw, fh, bit_depth=bd)
        pdb = R.DevicePlane.from_full(db, pad, pad, fw, fh, bit_depth=bd)
        out = R.lrf_stripe_filter(pc, pdb, x0, y0, sw, sh, fw, fh, s, (xq0, xq1), bd)
        np.testing.assert_array_equal(out.ravel().astype(np.uint16), g["filt"][k][:sw * sh],
                                      err_msg=str(g["cases"][k]))
        checked += 1
    assert checked >= 21
