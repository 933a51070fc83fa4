"""Pin the CPU oracle against the reference's own known answers.

CPU-only (`-m "not gpu"`).  Sources of truth:
  - SAD/SATD: the 88 KATs of src/dist.rs:379-460 (tests/golden/dist_kat.json);
  - transforms: vectors produced by the reference's own 1-D kernels
    (tools/refeval, tests/golden/tx*_golden.npz) and the reference's
    round-trip tolerances (src/transform/mod.rs:668-715);
  - plane padding: test_plane_pad (src/frame/plane.rs:709-753).
"""
import json
import os

import numpy as np
import pytest

from tests import oracle_lib as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def kat():
    with open(os.path.join(GOLD, "dist_kat.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("dtype", [np.uint8, np.uint16])
def test_sad_satd_kat(kat, dtype):
    (inp, ix, iy), (rec, rx, ry) = O.dist_kat_planes(dtype)
    for i, name in enumerate(kat["blocks"]):
        w, h = O.block_wh(name)
        sad = O.get_sad(inp, iy + 40, ix + 32, rec, ry + 40, rx + 32, w, h)
        assert sad == kat["sad"][i], name
        for emu in (0, 1):  # 8-bit-range data: generated kernels agree too
            satd = O.get_satd(inp, iy + 40, ix + 32, rec, ry + 40, rx + 32, w, h, emu)
            assert satd == kat["satd"][i], (name, emu)


def test_satd_i16_hazard_10bit():
    """The generated SATD kernels run i16 lanes for u16 pixels
    (build/kernel/gen/dist.rs:193,256): max-magnitude 10-bit residuals wrap."""
    a = np.zeros((8, 8), dtype=np.uint16)
    b = np.zeros((8, 8), dtype=np.uint16)
    a[:] = 1023
    ref = O.get_satd(a, 0, 0, b, 0, 0, 8, 8, 0)
    gen = O.get_satd(a, 0, 0, b, 0, 0, 8, 8, 1)
    assert ref == (1023 * 64 + 4) >> 3
    assert gen != ref


@pytest.fixture(scope="module")
def tx1d():
    return np.load(os.path.join(GOLD, "tx1d_golden.npz"))


def test_tx1d_golden(tx1d):
    keys = sorted({k.rsplit("_", 1)[0] for k in tx1d.files})
    assert len(keys) == 30
    for key in keys:
        tag, k, n = key.split("_")
        kind, n = int(k[1:]), int(n[1:])
        ins, outs, rngs = tx1d[key + "_in"], tx1d[key + "_out"], tx1d[key + "_range"]
        for v, want, r in zip(ins, outs, rngs):
            got = O.fwd_txfm1d(kind, v) if tag == "fwd" else O.inv_txfm1d(kind, v, int(r))
            assert got is not None, key
            np.testing.assert_array_equal(got, want, err_msg=key)


@pytest.fixture(scope="module")
def tx2d():
    return np.load(os.path.join(GOLD, "tx2d_golden.npz"))


def test_tx2d_golden(tx2d):
    keys = sorted({k.rsplit("_", 1)[0] for k in tx2d.files if k.endswith("_out")})
    assert len(keys) > 500
    for key in keys:
        tag, s, t, bd = key.split("_")
        s, t, bd = int(s[1:]), int(t[1:]), int(bd[2:])
        if tag == "fwd":
            got = O.fwd_txfm2d(tx2d[key + "_in"], s, t, bd)
        else:
            dst = tx2d[key + "_dst"].astype(np.uint8 if bd == 8 else np.uint16)
            got = O.inv_txfm2d_add(tx2d[key + "_coeffs"], dst, s, t, bd)
        assert got is not None, key
        np.testing.assert_array_equal(np.asarray(got).ravel(),
                                      tx2d[key + "_out"].ravel(), err_msg=key)


# src/transform/mod.rs:668-715 (TX_64X64 commented out in the reference)
ROUNDTRIPS = [
    ("4x4", "DCT_DCT", 0), ("4x4", "ADST_DCT", 0), ("4x4", "DCT_ADST", 0),
    ("4x4", "ADST_ADST", 0), ("4x4", "IDTX", 0), ("4x4", "V_DCT", 0),
    ("4x4", "H_DCT", 0), ("4x4", "V_ADST", 0), ("4x4", "H_ADST", 0),
    ("8x8", "DCT_DCT", 1), ("8x8", "ADST_DCT", 1), ("8x8", "DCT_ADST", 1),
    ("8x8", "ADST_ADST", 1), ("8x8", "IDTX", 0), ("8x8", "V_DCT", 0),
    ("8x8", "H_DCT", 0), ("8x8", "V_ADST", 0), ("8x8", "H_ADST", 1),
    ("16x16", "DCT_DCT", 1), ("16x16", "ADST_DCT", 1), ("16x16", "DCT_ADST", 1),
    ("16x16", "ADST_ADST", 1), ("16x16", "IDTX", 0), ("16x16", "V_DCT", 1),
    ("16x16", "H_DCT", 1), ("32x32", "DCT_DCT", 2), ("32x32", "IDTX", 0),
    ("4x8", "DCT_DCT", 1), ("8x4", "DCT_DCT", 1), ("4x16", "DCT_DCT", 1),
    ("16x4", "DCT_DCT", 1), ("8x16", "DCT_DCT", 1), ("16x8", "DCT_DCT", 1),
    ("8x32", "DCT_DCT", 2), ("32x8", "DCT_DCT", 2), ("16x32", "DCT_DCT", 2),
    ("32x16", "DCT_DCT", 2),
]


@pytest.mark.parametrize("dtype", [np.uint8, np.uint16])
def test_transform_roundtrip(dtype):
    """test_roundtrip (src/transform/mod.rs:589-630) on the oracle."""
    rng = np.random.default_rng(7)
    for size, ttype, tol in ROUNDTRIPS:
        s, t = O.TX_NAMES.index(size), O.TX_TYPES.index(ttype)
        w, h = 1 << O.TX_W_LOG2[s], 1 << O.TX_H_LOG2[s]
        for _ in range(8):
            src = rng.integers(0, 256, (h, w)).astype(dtype)
            dst = rng.integers(0, 256, (h, w)).astype(dtype)
            res = src.astype(np.int16) - dst.astype(np.int16)
            co = O.fwd_txfm2d(res, s, t, 8)
            # forward output is the full W*H raster; the inverse reads
            # min(W,32)*min(H,32) coefficients (no 64-wide sizes here)
            rec = O.inv_txfm2d_add(co, dst, s, t, 8)
            err = np.abs(src.astype(np.int32) - rec.astype(np.int32)).max()
            assert err <= tol, (size, ttype, err)


def test_plane_pad():
    """test_plane_pad, src/frame/plane.rs:709-753."""
    d = np.zeros((9, 8), dtype=np.uint8)
    d[3:7, 2:6] = [[1, 2, 3, 4], [8, 7, 6, 5], [9, 8, 7, 6], [2, 3, 4, 5]]
    O.lib().orc_plane_pad(O.ptr(d), 8, 9, 2, 3, 0, 0, 4, 4, 0)
    want = np.array([[1, 1, 1, 2, 3, 4, 4, 4]] * 4 + [[8, 8, 8, 7, 6, 5, 5, 5],
                    [9, 9, 9, 8, 7, 6, 6, 6]] + [[2, 2, 2, 3, 4, 5, 5, 5]] * 3, np.uint8)
    np.testing.assert_array_equal(d, want)


def test_plane_geometry():
    """Plane::new (src/frame/plane.rs:215-244) for the frame layouts used."""
    # 1080p luma: padding SB_SIZE + FRAME_MARGIN = 64 + 24 = 88 (frame/mod.rs:23,60)
    assert O.plane_geometry(1920, 1080, 88, 88, 0) == (2112, 1256, 96, 88)
    assert O.plane_geometry(960, 540, 44, 44, 0) == (1088, 628, 64, 44)
    assert O.plane_geometry(1920, 1080, 88, 88, 1) == (2112, 1256, 96, 88)


# ---- MC: independent numpy restatement of src/mc.rs:213-408 --------------
def _filters():
    import ctypes
    L = O.lib()
    L.orc_get_filter.restype = ctypes.POINTER(ctypes.c_int32)
    L.orc_get_filter.argtypes = [ctypes.c_int] * 3
    return lambda m, f, n: np.array(L.orc_get_filter(m, f, n)[:8], dtype=np.int64)


def _rs(v, b):
    return (v + ((1 << b) >> 1)) >> b


def _np_put(src, y, x, w, h, cf, rf, bd, emu=False):
    filt = _filters()
    s = src.astype(np.int64)
    ib = 2 if bd == 12 else 4
    xf, yf = filt(0, cf, w), filt(0, rf, h)
    mx = (1 << bd) - 1

    def fin(v):
        if emu and src.dtype == np.uint8:
            return np.where(v < 0, 0, v & 255)
        return np.clip(v, 0, mx)
    if cf == 0 and rf == 0:
        return s[y:y + h, x:x + w].astype(src.dtype)
    if cf == 0:
        acc = sum(yf[k] * s[y - 3 + k:y - 3 + k + h, x:x + w] for k in range(8))
        return fin(_rs(acc, 7)).astype(src.dtype)
    if rf == 0:
        acc = sum(xf[k] * s[y:y + h, x - 3 + k:x - 3 + k + w] for k in range(8))
        return fin(_rs(_rs(acc, 7 - ib), ib)).astype(src.dtype)
    mid = sum(xf[k] * s[y - 3:y + h + 4, x - 3 + k:x - 3 + k + w] for k in range(8))
    mid = _rs(mid, 7 - ib).astype(np.int16).astype(np.int64)
    acc = sum(yf[k] * mid[k:k + h] for k in range(8))
    return fin(_rs(acc, 7 + ib)).astype(src.dtype)


@pytest.mark.parametrize("bd", [8, 10])
def test_put_8tap_matches_numpy_restatement(bd):
    rng = np.random.default_rng(bd)
    dtype = np.uint8 if bd == 8 else np.uint16
    src = rng.integers(0, 1 << bd, (160, 160)).astype(dtype)
    for w, h in [(4, 4), (8, 8), (16, 8), (4, 16), (32, 32), (64, 64)]:
        for cf, rf in [(0, 0), (0, 6), (10, 0), (2, 14), (8, 8)]:
            got = O.put_8tap(src, 20, 24, w, h, cf, rf, bd=bd)
            np.testing.assert_array_equal(got, _np_put(src, 20, 24, w, h, cf, rf, bd))


def test_put_8tap_u8_wrap_quirk():
    """REGULAR frac 8 over [0,255,0,255,255,0,255,0] overshoots to 311: the
    reference clamps to 255, the generated u8 kernels wrap (311 & 255 = 55)."""
    src = np.zeros((16, 16), dtype=np.uint8)
    src[:, 0:8] = [0, 255, 0, 255, 255, 0, 255, 0]
    ref = O.put_8tap(src, 4, 3, 4, 4, 0, 0)  # sanity copy
    assert ref[0, 0] == 255
    clamp = O.put_8tap(src, 4, 3, 8, 4, 8, 0, emulate_gen=0)
    wrap = O.put_8tap(src, 4, 3, 8, 4, 8, 0, emulate_gen=1)
    assert clamp[0, 0] == 255 and wrap[0, 0] == 311 & 255
    np.testing.assert_array_equal(wrap, _np_put(src, 4, 3, 8, 4, 8, 0, 8, emu=True))


def test_prep_avg_roundtrip_equals_put_when_same():
    """avg(prep(a), prep(a)) == put(a): an identity implied by src/mc.rs:310-408
    for in-range data (both round the same sum)."""
    rng = np.random.default_rng(3)
    src = rng.integers(0, 256, (96, 96)).astype(np.uint8)
    for cf, rf in [(0, 0), (4, 0), (0, 12), (6, 10)]:
        t = O.prep_8tap(src, 16, 16, 16, 16, cf, rf)
        avg = O.mc_avg(t, t)
        put = O.put_8tap(src, 16, 16, 16, 16, cf, rf)
        assert np.abs(avg.astype(int) - put.astype(int)).max() <= 1


def test_cdef_dist_and_sse():
    rng = np.random.default_rng(5)
    a = rng.integers(0, 256, (8, 8)).astype(np.uint8)
    b = rng.integers(0, 256, (8, 8)).astype(np.uint8)
    m = O.cdef_moments(a, b)
    s, d = a.astype(np.int64), b.astype(np.int64)
    assert list(m) == [s.sum(), d.sum(), (s * s).sum(), (d * d).sum(), (s * d).sum()]
    svar = (s * s).sum() - ((s.sum() ** 2 + 32) >> 6)
    dvar = (d * d).sum() - ((d.sum() ** 2 + 32) >> 6)
    sse = ((s - d) ** 2).sum()
    boost = (4033 / 16384) * (svar + dvar + 16384) / np.sqrt(16265089 + svar * dvar)
    assert O.cdef_dist(m, 8) == int(sse * boost + 0.5)
    big_a = rng.integers(0, 256, (32, 32)).astype(np.uint8)
    big_b = rng.integers(0, 256, (32, 32)).astype(np.uint8)
    parts = O.sse_wxh(big_a, big_b, 32, 32, 1, 1)  # chroma 4:2:0 -> 4x4 blocks
    assert parts.size == 64
    diff = (big_a.astype(np.int64) - big_b) ** 2
    assert int(parts.sum()) == int(diff.sum())
    assert int(parts[0]) == int(diff[:4, :4].sum())


def test_tx_dist_oracle_matches_restatement():
    """orc_tx_dist vs a numpy restatement of src/encoder.rs:1210-1224 with
    get_log_tx_scale (src/quantize.rs:34-39), incl. the i32 wrapping square
    sign-extended to u64."""
    rng = np.random.default_rng(77)
    for tw, th in ((4, 4), (16, 16), (32, 32), (64, 64), (16, 64)):
        area = min(tw, 32) * min(th, 32)
        co = rng.integers(-60000, 60000, area).astype(np.int64)
        rc = rng.integers(-60000, 60000, area).astype(np.int64)
        e = ((co - rc + 2 ** 31) % 2 ** 32) - 2 ** 31
        sq = ((e * e + 2 ** 31) % 2 ** 32) - 2 ** 31          # i32 wrap
        d = sum(int(v) % 2 ** 64 for v in sq) % 2 ** 64  # `as u64` sign-extends
        bits = 2 * (3 - ((tw * th > 256) + (tw * th > 1024)))
        want = ((d + (1 << (bits - 1))) % 2 ** 64) >> bits
        assert O.tx_dist(co.astype(np.int32), rc.astype(np.int32), tw, th) == want


# ---- quantize / dequantize (src/quantize.rs) ---------------------------------
def test_divu_pair_reference_test():
    """test_divu_pair (src/quantize.rs:160-168): divu_pair(x, divu_gen(d)) ==
    x / d (Rust: truncating) for d in 1..1024, x in -1000..1000."""
    for d in range(1, 1024):
        g = O.divu_gen(d)
        for x in range(-1000, 1000):
            assert O.divu_pair(x, g) == int(x / d), (d, x)


def test_log_tx_scale_reference_test():
    """test_tx_log_scale (src/quantize.rs:176-202), TxSize enum order."""
    want = [0, 0, 0, 1, 2, 0, 0, 0, 0, 1, 1, 2, 2, 0, 0, 0, 0, 1, 1]
    assert [O.lib().orc_get_log_tx_scale(s) for s in range(19)] == want


def _py_quantize(coeffs, scan, n, lts, ac_q, dc_q, is_intra):
    """Independent restatement of QuantizationContext::update + quantize
    (src/quantize.rs:205-316) with exact integer division for divu_pair."""
    dc_off = dc_q * (109 if is_intra else 108) // 256
    off0 = ac_q * (98 if is_intra else 97) // 256
    off1 = ac_q * (109 if is_intra else 108) // 256
    off_eob = ac_q * (88 if is_intra else 44) // 256
    dz = (ac_q - off_eob + (1 << lts) - 1) >> lts
    div = lambda x, d: -((-x) // d) if x < 0 else x // d  # noqa: E731
    sg = lambda v: (v > 0) - (v < 0)  # noqa: E731
    eob = 1
    for i in range(n - 1, 0, -1):
        if abs(int(coeffs[scan[i]])) >= dz:
            eob = i
            break
    q = np.zeros(n, np.int64)
    c0 = int(coeffs[0]) << lts
    q[0] = div(c0 + sg(c0) * dc_off, dc_q)
    mode = 1
    for i in range(1, min(eob, n - 1) + 1):
        c = int(coeffs[scan[i]]) << lts
        l0 = div(c, ac_q)
        v = div(c + sg(c) * (off1 if l0 > 1 - mode else off0), ac_q)
        q[scan[i]] = v
        if mode and v == 0:
            mode = 0
        elif v > 1:
            mode = 1
    return q, eob


@pytest.mark.parametrize("tx_size,tx_type", [(3, 0), (4, 0), (1, 0), (0, 3), (2, 9), (9, 0), (12, 0)])
def test_quantize_matches_restatement(tx_size, tx_type):
    """orc_quantize / orc_dequantize vs the restatement above, on coefficient
    magnitudes around the deadzone and large ones, several qindices, 8/10/12
    bits, intra and inter.  Scan orders: tools/refeval/gen_quant_tables.py
    (checked against src/scan_order.rs)."""
    rng = np.random.default_rng(500 + 19 * tx_type + tx_size)
    n = O.lib().orc_coded_tx_area(tx_size)
    lts = O.lib().orc_get_log_tx_scale(tx_size)
    scan = _scan(tx_size, tx_type)
    for bd in (8, 10, 12):
        for qi in (1, 60, 100, 200, 255):
            dcq, acq = O.lib().orc_dc_q(qi, 0, bd), O.lib().orc_ac_q(qi, 0, bd)
            for is_intra in (False, True):
                c = rng.integers(-3 * acq, 3 * acq, n)
                c[rng.random(n) < 0.5] = 0
                c[: n // 8] *= 7
                q, eob = O.quantize(c, tx_size, tx_type, qi, bd, is_intra)
                want, weob = _py_quantize(c, scan, n, lts, acq, dcq, is_intra)
                assert eob == weob and (q == want).all(), (bd, qi, is_intra)
                r = O.dequantize(q, tx_size, qi, bd)
                off = (1 << lts) - 1
                quant = np.full(n, acq, np.int64)
                quant[0] = dcq
                wr = (q.astype(np.int64) * quant + ((q >> 31) & off)) >> lts
                assert (r == wr).all()


def _scan(tx_size, tx_type):
    """The scan as the oracle's generated table holds it (read back through
    quantize of one-hot inputs is circular, so parse the header)."""
    import re
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "oracle", "orc_quant_tables.h")).read()
    def arr(name):
        m = re.search(name + r"\[\d+\] = \{(.*?)\};", hdr, re.S)
        return [int(v) for v in re.findall(r"\d+", m.group(1))]
    scans, off = arr("ORC_SCANS"), arr("ORC_SCAN_OFF")
    n = O.lib().orc_coded_tx_area(tx_size)
    o = off[tx_size * 16 + tx_type]
    return scans[o:o + n]


# ---- estimate_rate (src/rdo.rs:204-216) -------------------------------------
def _rate_table():
    """RDO_RATE_TABLE as the generated header holds it: [8][19][50]."""
    import re
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "oracle", "orc_rate_table.h")).read()
    m = re.search(r"RV_RDO_RATE_TABLE\[\d+\] = \{(.*?)\};", hdr, re.S)
    v = [int(x) for x in re.findall(r"\d+", m.group(1))]
    assert len(v) == 8 * 19 * 50
    return np.array(v, dtype=np.int64).reshape(8, 19, 50)


def _py_estimate_rate(tab, qindex, ts, fd):
    """Restatement with Rust's i64 semantics: `/` truncates toward zero,
    `>>` is arithmetic, the product wraps."""
    down = min(fd // 2000, 48)
    up = min(down + 1, 49)
    x0, x1 = down * 2000, up * 2000
    y0, y1 = int(tab[qindex // 32, ts, down]), int(tab[qindex // 32, ts, up])
    num = (y1 - y0) << 8
    slope = abs(num) // (x1 - x0) * (1 if num >= 0 else -1)
    prod = ((fd - x0) * slope + (1 << 63)) % (1 << 64) - (1 << 63)
    return max(y0 + (prod >> 8), 0)


def test_estimate_rate_reference_test():
    """estimate_rate_test (src/rdo.rs:2148-2150): distortion 0 at qindex 0,
    TX_4X4 reads the table's first entry."""
    tab = _rate_table()
    assert O.estimate_rate(0, 0, 0) == int(tab[0, 0, 0])


def test_estimate_rate_matches_restatement():
    """The oracle against the Python restatement over every q bin and
    TxSize: bin edges, interiors, the clamp to the last bins and large
    distortions."""
    tab = _rate_table()
    rng = np.random.default_rng(77)
    fds = [0, 1, 1999, 2000, 2001, 49999, 96000, 97999, 98000, 99999, 100000, 10 ** 7, 2 ** 40]
    fds += [int(x) for x in rng.integers(0, 120000, 12)]
    for q in (0, 31, 32, 100, 255):
        for ts in range(19):
            for fd in fds:
                assert O.estimate_rate(q, ts, fd) == _py_estimate_rate(tab, q, ts, fd), (q, ts, fd)


# ---- lookahead intra costs (src/api/internal.rs:680-765) --------------------
def test_lookahead_intra_costs_known_answers():
    """DC_PRED at the block's own tile origin is pred_dc_128, so a constant
    plane v costs get_satd of a DC-only difference: 64 |v - base| after the
    8x8 Hadamard, (64 |v - base| + 4) >> 3 = 8 |v - base| per block; a plane
    at the base value costs nothing; a block costs get_satd against a flat
    block of the base value."""
    for bd, dt in ((8, np.uint8), (10, np.uint16), (12, np.uint16)):
        base = 128 << (bd - 8)
        for v in (0, base, base + 7, (1 << bd) - 1):
            full = np.full((40, 56), v, dtype=dt)
            got = O.lookahead_intra_costs(full, 4, 8, 40, 24, bd)
            assert got.shape == (3, 5)
            assert (got == 8 * abs(v - base)).all(), (bd, v)
    rng = np.random.default_rng(5)
    full = rng.integers(0, 256, (48, 64)).astype(np.uint8)
    got = O.lookahead_intra_costs(full, 8, 0, 60, 36, 8)  # partial last column / row
    flat = np.full((8, 8), 128, dtype=np.uint8)
    for by in range(5):
        for bx in range(8):
            want = O.get_satd(full, 8 + 8 * by, 8 * bx, flat, 0, 0, 8, 8)
            assert got[by, bx] == want, (by, bx)


# ---- importance propagation (src/api/internal.rs:823-1010) ------------------
def _py_propagate(org, oyo, oxo, ref, ryo, rxo, nbx, nby, mvs, intra, imp, n_unique, out):
    """Restatement in numpy float32 scalars (IEEE single, no fused ops)."""
    f32 = np.float32
    out = out.astype(np.float32).copy()
    for y in range(nby):
        for x in range(nbx):
            row, col = int(mvs[y, x, 0]), int(mvs[y, x, 1])
            rx, ry = x * 64 + col, y * 64 + row
            px_x, px_y = int(rx / 8), int(ry / 8)  # toward zero
            inter = f32(O.get_satd(org, oyo + 8 * y, oxo + 8 * x, ref, ryo + px_y, rxo + px_x, 8, 8))
            ic = f32(intra[y, x])
            with np.errstate(divide="ignore", invalid="ignore"):
                fr = f32(1) - inter / ic
            fr = f32(0) if np.isnan(fr) or fr < 0 else fr
            amount = (ic + imp[y, x]) * fr / f32(n_unique)
            tlx = (rx - (63 if rx < 0 else 0)) // 64 * 64 if rx >= 0 else -((-(rx - 63)) // 64) * 64
            tly = (ry - (63 if ry < 0 else 0)) // 64 * 64 if ry >= 0 else -((-(ry - 63)) // 64) * 64
            trx, bly = tlx + 64, tly + 64
            parts = ((tlx, tly, (trx - rx) * (bly - ry)), (trx, tly, (rx + 64 - trx) * (bly - ry)),
                     (tlx, bly, (trx - rx) * (ry + 64 - bly)), (trx, bly, (rx + 64 - trx) * (ry + 64 - bly)))
            for tx, ty, a in parts:
                bx, by = int(tx / 64), int(ty / 64)
                if 0 <= bx < nbx and 0 <= by < nby:
                    out[by, bx] = out[by, bx] + amount * (f32(a) / f32(4096))
    return out


@pytest.mark.parametrize("n_unique", [1, 2, 3])
def test_propagate_importances_matches_restatement(n_unique):
    """The oracle's f32 propagation against the numpy restatement, bit for
    bit: sub-pel and negative MVs (truncating division, floor to the block
    grid), zero intra costs (inf and NaN fractions), targets off the grid."""
    rng = np.random.default_rng(300 + n_unique)
    w, h, pad = 64, 48, 40
    nbx, nby = 8, 6
    org = rng.integers(0, 256, (h + 2 * pad, w + 2 * pad)).astype(np.uint8)
    ref = rng.integers(0, 256, (h + 2 * pad, w + 2 * pad)).astype(np.uint8)
    mvs = rng.integers(-256, 257, (nby, nbx, 2)).astype(np.int16)
    intra = rng.integers(0, 3000, (nby, nbx)).astype(np.uint32)
    intra[0, :3] = 0
    imp = (rng.random((nby, nbx)) * 500).astype(np.float32)
    out0 = (rng.random((nby, nbx)) * 100).astype(np.float32)
    got = O.propagate_importances(org, pad, pad, ref, pad, pad, w, h, mvs, intra, imp, n_unique,
                                  out0)
    want = _py_propagate(org, pad, pad, ref, pad, pad, nbx, nby, mvs, intra, imp, n_unique, out0)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


# ---- intra prediction: the reference's own known answers -------------------
def _kat_edge(bd=8, fill=None):
    """pred_matches_u8's edge_buf (src/predict.rs:1047-1056) mapped into the
    257-pixel layout: edge_buf[i] = (i + 32).saturating_sub(64); left =
    edge_buf[60..64] (bottom-to-top), top_left = edge_buf[64], above =
    edge_buf[65..69]."""
    e = np.zeros(257, dtype=np.uint16 if bd > 8 else np.uint8)
    if fill is not None:
        e[:] = fill
        return e
    eb = [max(i + 32 - 64, 0) for i in range(129)]
    e[124:128] = eb[60:64]
    e[128] = eb[64]
    e[129:133] = eb[65:69]
    return e


def test_intra_pred_matches_u8_kats():
    """src/predict.rs:1047-1107 (mode, PredictionVariant) -> expected 4x4."""
    e = _kat_edge()
    kats = [
        (0, 3, [32] * 16), (0, 2, [35] * 16), (0, 1, [30] * 16), (0, 0, [128] * 16),
        (1, 3, [33, 34, 35, 36] * 4),
        (2, 3, [31] * 4 + [30] * 4 + [29] * 4 + [28] * 4),
        (12, 3, [32, 34, 35, 36, 30, 32, 32, 36, 29, 32, 32, 32, 28, 28, 32, 32]),
        (9, 3, [32, 34, 35, 35, 30, 32, 33, 34, 29, 31, 32, 32, 29, 30, 32, 32]),
        (11, 3, [31, 33, 34, 35, 30, 33, 34, 35, 29, 32, 34, 34, 28, 31, 33, 34]),
        (10, 3, [33, 34, 35, 36, 31, 31, 32, 33, 30, 30, 30, 31, 29, 30, 30, 30]),
    ]
    for mode, variant, want in kats:
        got = O.predict_intra(mode, variant, 4, 4, e, 8)
        assert got.ravel().tolist() == want, (mode, variant, got.ravel().tolist())


def test_intra_pred_max_kats():
    """src/predict.rs:1109-1170: 12-bit maximum edges predict the maximum."""
    e = _kat_edge(12, 4095)
    for mode in (0, 2, 1, 12, 9, 11, 10):
        assert (O.predict_intra(mode, 3, 4, 4, e, 12) == 4095).all(), mode


def test_intra_directional_constant_edges():
    """A constant edge predicts the constant in every mode and size (the
    directional interpolation weights sum to 32, the smooth ones to 256)."""
    for bd, v in ((8, 77), (10, 901), (12, 3000)):
        e = _kat_edge(bd, v)
        for tx in (0, 1, 4, 5, 12, 17):
            w, h = 1 << O.TX_W_LOG2[tx], 1 << O.TX_H_LOG2[tx]
            for mode in range(13):
                assert (O.predict_intra(mode, 3, w, h, e, bd) == v).all(), (bd, tx, mode)
