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
