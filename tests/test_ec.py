"""Entropy coder: the oracle (oracle/orc_ec.c) against vectors made by
evaluating the reference's own ec.rs / write_coeffs_lv_map text
(tools/refeval/gen_ec_ref.py -> tests/golden/ref_ec.npz), the reference's
own ec.rs unit tests (src/ec.rs:1010-1101) restated on the oracle's writer and
reader, and (-m gpu) the product's device tokenizer + host range coder
(rav1e_amd/csrc/rv_ec.hip) against both."""
import os

import numpy as np
import pytest

from tests import oracle_lib as O

GOLD = os.path.join(os.path.dirname(__file__), "golden", "ref_ec.npz")


@pytest.fixture(scope="module")
def ref():
    return np.load(GOLD)


def test_writer_streams_match_reference(ref):
    ops, by, idx = ref["ec_ops"], ref["ec_bytes"], ref["ec_index"]
    for o0, no, b0, nb in idx:
        got = O.ec_replay_ops(ops[o0:o0 + no])
        np.testing.assert_array_equal(got, by[b0:b0 + nb])


def _decode(buf, seq):
    """Decode seq (('b', f) / ('s', cdf)) with the restated test Reader."""
    L = O.ec_lib()
    import ctypes as C
    r = C.create_string_buffer(64)
    L.orc_ecr_init(r, buf.ctypes.data, buf.size)
    out = []
    for kind, arg in seq:
        if kind == "b":
            out.append(bool(L.orc_ecr_bool(r, arg)))
        else:
            a = np.array(arg, np.uint16)
            out.append(L.orc_ecr_symbol(r, a.ctypes.data, a.size))
    return out


def test_reference_unit_tests_booleans_cdf_mixed():
    # src/ec.rs:1012-1101 (booleans, cdf, mixed), on the oracle's writer + reader
    w = O.EcWriter()
    vals = [(False, 1), (True, 2), (False, 3), (True, 1), (True, 2), (False, 3)]
    for v, f in vals:
        w.bool(v, f)
    assert _decode(w.done(), [("b", f) for _, f in vals]) == [v for v, _ in vals]
    cdf = [7296, 3819, 1716, 0]
    w = O.EcWriter()
    syms = [0, 0, 0, 1, 1, 1, 2, 2, 2]
    L = O.ec_lib()
    for s in syms:
        a = np.array(cdf, np.uint16)
        L.orc_ecw_symbol_update  # symbol without update: write through a copy, discard it
        import ctypes as C
        L.orc_ecw_symbol.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_int]
        L.orc_ecw_symbol(w.buf, s, a.ctypes.data, 4)
    assert _decode(w.done(), [("s", cdf)] * len(syms)) == syms
    seq = [("s", 0), ("b", (True, 2)), ("s", 0), ("b", (True, 2)), ("s", 0), ("b", (True, 2)),
           ("s", 1), ("b", (True, 1)), ("s", 1), ("b", (False, 2)), ("s", 1), ("s", 2),
           ("s", 2), ("s", 2)]
    w = O.EcWriter()
    for k, a in seq:
        if k == "s":
            arr = np.array(cdf, np.uint16)
            L.orc_ecw_symbol(w.buf, a, arr.ctypes.data, 4)
        else:
            w.bool(*a)
    dec = _decode(w.done(), [("s", cdf) if k == "s" else ("b", a[1]) for k, a in seq])
    assert dec == [a if k == "s" else a[0] for k, a in seq]


def test_reader_round_trip_random_adaptive():
    """A long random stream of adaptive symbols: the restated reader,
    adapting the same CDFs, decodes every symbol back."""
    rng = np.random.default_rng(3)
    cdf_w = O.ec_default_cdf(2)
    cdf_r = cdf_w.copy()
    w = O.EcWriter()
    seq = []
    fams = [(0, 3, 65), (877, 5, 420), (2977, 5, 210), (399, 12, 4)]
    for _ in range(5000):
        off, e, cnt = fams[int(rng.integers(0, len(fams)))]
        o = off + int(rng.integers(0, cnt)) * e
        s = int(min(e - 2, rng.geometric(0.5) - 1))
        w.symbol_update(s, cdf_w, o, e)
        seq.append((o, e, s))
    buf = w.done()
    L = O.ec_lib()
    import ctypes as C
    r = C.create_string_buffer(64)
    L.orc_ecr_init(r, buf.ctypes.data, buf.size)
    L.orc_update_cdf.argtypes = [C.c_void_p, C.c_int, C.c_uint32]
    for o, e, s in seq:
        v = L.orc_ecr_symbol(r, cdf_r[o:].ctypes.data, e - 1)
        assert v == s
        L.orc_update_cdf(cdf_r[o:].ctypes.data, e, v)
    np.testing.assert_array_equal(cdf_r, cdf_w)


def test_coefficient_coding_matches_reference(ref):
    jobs, co = ref["lv_jobs"], ref["lv_coeffs"]
    by, tb_ref, ret_ref = ref["lv_bytes"], ref["lv_tile_bytes"], ref["lv_ret"]
    fin_ref, init = ref["lv_final_cdf"], ref["lv_init_cdf"]
    b0 = t0 = 0
    for ci, (cid, j0, nj, xdec, ydec, q, ntiles) in enumerate(ref["lv_cases"]):
        np.testing.assert_array_equal(init[ci], O.ec_default_cdf(int(q)))
        got, tb, ret, fin = O.ec_code_jobs(jobs[j0:j0 + nj], co, init[ci], int(xdec), int(ydec))
        np.testing.assert_array_equal(tb[:ntiles], tb_ref[t0:t0 + ntiles])
        nb = int(tb_ref[t0:t0 + ntiles].sum())
        np.testing.assert_array_equal(got, by[b0:b0 + nb])
        np.testing.assert_array_equal(ret, ret_ref[j0:j0 + nj])
        np.testing.assert_array_equal(fin, fin_ref[t0 + ntiles - 1])
        b0 += nb
        t0 += ntiles


# ------------------------------------------------------------- the product
def _rand_jobs(rng, xdec, ydec, sbw, sbh, ntiles, vis_w4=None, vis_h4=None, scale=6.0):
    """A coding-order job list like gen_ec_ref's (quadtree leaves 64..8 in
    z-order, skip leaves, superblock rows, tiles) with random coefficients."""
    from tests.test_ec_util import leaves, rand_coeffs
    vis_w4 = vis_w4 or sbw * 16
    vis_h4 = vis_h4 or sbh * 16
    jobs, co = [], []
    for _ in range(ntiles):
        jobs.append((3, 0, 0, 0, 0, 0, 0, 0, 0, 0))
        for sby in range(sbh):
            jobs.append((2, 0, 0, 0, 0, 0, 0, 0, 0, 0))
            for sbx in range(sbw):
                lv = []
                leaves(rng, sbx * 16, sby * 16, 6, 3, vis_w4, vis_h4, lv)
                for x4, y4, lg in lv:
                    if rng.random() < 0.3:
                        jobs.append((1, 0, x4, y4, 0, 0, 0, lg, lg, 0))
                        continue
                    intra = lg == 6 and rng.random() < 0.25
                    for p in range(3):
                        xd = xdec if p else 0
                        plg = lg - xd
                        tx = min(plg - 2, 4)
                        n_tx = 1
                        if p and xdec == 0 and lg == 6:
                            tx, n_tx = 3, 4
                        cw = min(4 << tx, 32)
                        for t in range(n_tx):
                            bx = x4 + (t % 2) * 8 if n_tx == 4 else x4
                            by = y4 + (t // 2) * 8 if n_tx == 4 else y4
                            c = rand_coeffs(rng, cw, scale if p == 0 else scale / 2)
                            jobs.append((0, p, bx, by, tx, 0, 0 if intra else 1, plg, plg,
                                         sum(len(x) for x in co)))
                            co.append(c)
    return np.array(jobs, np.int64), np.concatenate(co).astype(np.int32)


def test_host_range_coder_matches_oracle_writer():
    """rv_ec_code_tokens (the product's host coder, plain C++ in the HIP
    library) against the oracle's writer on random symbol / bit streams."""
    import rav1e_amd as R
    rng = np.random.default_rng(11)
    for q in range(4):
        tok, cdf_o = [], O.ec_default_cdf(q)
        w = O.EcWriter()
        fams = [(0, 3, 65), (877, 5, 420), (2977, 5, 210), (399, 12, 4), (195, 6, 4), (4045, 17, 16)]
        for _ in range(4000):
            if rng.random() < 0.2:
                b = int(rng.integers(0, 2))
                tok.append(0x80000000 | b)
                w.bit(b)
                continue
            off, e, cnt = fams[int(rng.integers(0, len(fams)))]
            if e == 17:
                e = 3  # inter_tx_cdf[..][..][..=2]
            o = off + int(rng.integers(0, cnt)) * (17 if off == 4045 else e)
            if cdf_o[o + e - 1] > 32:
                continue  # not a CDF of e - 1 symbols + its counter (update_cdf's rate would overflow)
            s = int(min(e - 2, rng.geometric(0.4) - 1))
            tok.append(o | (e << 13) | (s << 18))
            w.symbol_update(s, cdf_o, o, e)
        want = w.done()
        cdf_p = R.ec_default_cdf(q)
        got = R.ec_code_tokens(np.array(tok, np.uint32), cdf_p)
        np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal(cdf_p, cdf_o)


@pytest.mark.gpu
def test_gpu_coefficient_coding_matches_reference(ref):
    import rav1e_amd as R
    R.require_device()
    jobs, co = ref["lv_jobs"], ref["lv_coeffs"]
    by, tb_ref, fin_ref, init = ref["lv_bytes"], ref["lv_tile_bytes"], ref["lv_final_cdf"], \
        ref["lv_init_cdf"]
    b0 = t0 = 0
    for ci, (cid, j0, nj, xdec, ydec, q, ntiles) in enumerate(ref["lv_cases"]):
        got, tb, fin, _ = R.code_coefficients(jobs[j0:j0 + nj], co, init[ci], int(xdec), int(ydec))
        np.testing.assert_array_equal(tb, tb_ref[t0:t0 + ntiles])
        nb = int(tb_ref[t0:t0 + ntiles].sum())
        np.testing.assert_array_equal(got, by[b0:b0 + nb])
        np.testing.assert_array_equal(fin, fin_ref[t0 + ntiles - 1])
        b0 += nb
        t0 += ntiles


@pytest.mark.gpu
@pytest.mark.parametrize("xdec,ydec,sbw,sbh,ntiles,scale", [
    (1, 1, 6, 4, 3, 6.0), (0, 0, 4, 3, 2, 4.0), (1, 1, 3, 2, 1, 400.0), (1, 1, 8, 2, 2, 0.3)])
def test_gpu_coefficient_coding_matches_oracle(xdec, ydec, sbw, sbh, ntiles, scale):
    """Larger tiles (more superblocks, ragged edges, golomb-range and
    near-empty blocks) through the device tokenizer + host coder against the
    oracle's sequential write_coeffs_lv_map."""
    import rav1e_amd as R
    R.require_device()
    rng = np.random.default_rng(sbw * 7 + ntiles)
    jobs, co = _rand_jobs(rng, xdec, ydec, sbw, sbh, ntiles, vis_w4=sbw * 16 - 2,
                          vis_h4=sbh * 16 - 6, scale=scale)
    for q in (0, 3):
        init = O.ec_default_cdf(q)
        want, tbw, _, finw = O.ec_code_jobs(jobs, co, init, xdec, ydec, cap=1 << 26)
        got, tb, fin, _ = R.code_coefficients(jobs, co, init, xdec, ydec)
        np.testing.assert_array_equal(tb, tbw[:ntiles])
        np.testing.assert_array_equal(got, want)
        np.testing.assert_array_equal(fin, finw)


# --------------------------------------------------------------- the replay
@pytest.mark.gpu
@pytest.mark.parametrize("W,H,xdec,tiles,speed,q", [
    (640, 360, 1, (0, 0), 10, 100), (640, 360, 1, (0, 0), 10, 40), (640, 360, 1, (0, 0), 6, 60),
    (1920, 1080, 1, (8, 17), 10, 60), (512, 384, 0, (4, 3), 10, 50)])
def test_gpu_replay_entropy_matches_cpu(W, H, xdec, tiles, speed, q):
    """RV_REPLAY_ENTROPY (F8: device tokens + host range coder + the CDF chain
    per pyramid level) against the CPU replay's sequential
    write_coeffs_lv_map over the same committed frames, frame by frame:
    bytes, tiles and the hash of every tile's bytes, plus the result words."""
    import rav1e_amd as R
    from rav1e_amd import replay as RP
    R.require_device()
    n = 10
    flags = RP.RV_REPLAY_ENTROPY | (RP.RV_REPLAY_SPEED6 if speed == 6 else 0)
    g = RP.HipReplay(W, H, xdec, xdec, 8, 2, tile_size=tiles, n_inputs=n + 2, flags=flags,
                     quantizer=q)
    g.synth_inputs(0)
    c = O.CpuReplay(W, H, xdec, xdec, 8, 2, tile_size=tiles, n_inputs=n + 2, threads=8,
                    speed=speed, entropy=True, quantizer=q)
    for i in range(n + 2):
        c.set_input(i, g.get_input(i))
    g.frame()
    c.frame()
    nonzero = 0
    try:
        for f in range(n):
            g.frame()
            c.frame()
            np.testing.assert_array_equal(g.results(), c.results(), err_msg=f"frame {f}")
            gs, cs = g.entropy_stats(), c.entropy_stats()
            assert gs[:3] == cs[:3], (f, gs, cs)
            nonzero += gs[0] > 8
    finally:
        g.close()
        c.close()
    assert nonzero >= 2  # coefficients were coded, not only empty tiles
