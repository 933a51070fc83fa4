"""EPZS predictor sets (get_subset_predictors, src/me.rs:82-174): the
oracle's restatement (oracle/orc_me.c orc_subset_predictors) against
vectors the reference's own function text produced
(tests/golden/ref_epzs.npz, tools/refeval/gen_epzs_ref.py).  The device
restatement (rav1e_amd/csrc/rv_epzs.h) is checked through the replays'
GPU-vs-CPU parity (tests/test_replay.py), whose CPU side this pins."""
import ctypes as C
import os

import numpy as np

from tests import oracle_lib as O

GOLD = os.path.join(os.path.dirname(__file__), "golden", "ref_epzs.npz")


def _mv_ptr(a):
    a = np.ascontiguousarray(a, dtype=np.int16)
    return a, a.ctypes.data_as(C.c_void_p)


def test_oracle_subset_predictors_vs_reference():
    g = np.load(GOLD)
    L = O.lib()
    f = L.orc_subset_predictors
    f.restype = C.c_int
    f.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int,
                  C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]
    toff = np.concatenate([[0], np.cumsum(g["tile_len"])])
    poff = np.concatenate([[0], np.cumsum(g["prev_len"])])
    checked = 0
    for i, (tx, ty, cols, rows, fc, fr, has_prev, bx, by, ncmv) in enumerate(g["case"]):
        tile, tp = _mv_ptr(g["tile"][toff[i]:toff[i + 1]])
        prev, pp = _mv_ptr(g["prev"][poff[i]:poff[i + 1]]) if has_prev else (None, None)
        cm, cp = _mv_ptr(g["cmv"][i])
        out = np.zeros((17, 2), np.int16)
        n = f(int(bx), int(by), cp, int(ncmv), tp, int(cols), int(cols), pp, int(fc), int(fc),
              int(fr), int(tx + bx), int(ty + by), out.ctypes.data_as(C.c_void_p))
        want = g["out"][i]
        assert n == want[0], (i, n, want[0])
        np.testing.assert_array_equal(out[:n].reshape(-1), want[1:1 + 2 * n], err_msg=str(i))
        checked += 1
    assert checked == len(g["case"])
