"""Block importances over the lookahead window (compute_block_importances,
src/api/internal.rs:823-1081, rdo_lookahead_frames: src/api/config.rs:158)
in the replay.  CPU side: the oracle's window (oracle/orc_replay.c
importance_frame) against a numpy restatement of the reference's loop over
the same per-frame lookahead data (intra costs, 8x8 lookahead MVs, inter
costs), the f32 log2 against the host's log2f.  GPU side
(tests/test_replay.py ..._importance_window): the HIP replay's importances
and words against the oracle's."""
import ctypes as C

import numpy as np
import pytest

from rav1e_amd import replay as RP
from tests import oracle_lib as O

B_MV = 64  # IMPORTANCE_BLOCK_SIZE * MV_UNITS_PER_PIXEL


def coded_of_display(d):
    if d == 0:
        return 0
    j = {0: 0, 2: 1, 1: 2, 3: 3}[d % 4]
    return 4 * ((d - (4, 2, 1, 3)[j]) // 4) + j + 1


def _tdiv(a, b):
    """i64 division as Rust's `/`: truncating toward zero."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


def _propagate(mv, inter, intra, imp, nu, into):
    """One (frame, reference) pass in the reference's order (:900-1045),
    f32 throughout."""
    h, w = intra.shape
    f32 = np.float32
    for y in range(h):
        for x in range(w):
            rx = x * B_MV + int(mv[y, x, 1])
            ry = y * B_MV + int(mv[y, x, 0])
            ic, ec = f32(intra[y, x]), f32(inter[y, x])
            with np.errstate(divide="ignore", invalid="ignore"):
                fr = f32(1) - ec / ic
            fr = f32(0) if not (fr > 0) else fr  # f32::max(NaN, 0) = 0
            amt = (ic + imp[y, x]) * fr / f32(nu)
            tlx = _tdiv(rx - (B_MV - 1 if rx < 0 else 0), B_MV) * B_MV
            tly = _tdiv(ry - (B_MV - 1 if ry < 0 else 0), B_MV) * B_MV
            trx, bly = tlx + B_MV, tly + B_MV
            for tx, ty, fx, fy in ((tlx, tly, trx - rx, bly - ry),
                                   (trx, tly, rx + B_MV - trx, bly - ry),
                                   (tlx, bly, trx - rx, ry + B_MV - bly),
                                   (trx, bly, rx + B_MV - trx, ry + B_MV - bly)):
                bx, by = _tdiv(tx, B_MV), _tdiv(ty, B_MV)
                if 0 <= bx < w and 0 <= by < h:
                    into[by, bx] = into[by, bx] + amt * (f32(fx * fy) / f32(B_MV * B_MV))


def test_log2f_restatement_matches_host():
    L = O.lib()
    L.orc_log2f_mismatches.restype = C.c_uint64
    L.orc_log2f_mismatches.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32]
    # every float in [1, 2) (the argument 1 + imp / intra starts at 1), then
    # a stride over the rest of the positive range
    assert L.orc_log2f_mismatches(0x3F800000, 0x40000000, 1) == 0
    assert L.orc_log2f_mismatches(1, 0x7F800000, 251) == 0


def test_oracle_importance_window_vs_numpy():
    w, h, n, W = 256, 192, 9, 4
    refs = 2
    fr = [RP.synth_frame(w, h, t, 1, 1, 8) for t in range(n + 8)]
    c = O.CpuReplay(w, h, 1, 1, 8, refs, n_inputs=len(fr), threads=O.cpu_share(),
                    imp_window=W, imp_limit=n)
    for i, f in enumerate(fr):
        c.set_input(i, f)
    L = c.L
    L.orc_replay_la_data.argtypes = [C.c_void_p, C.c_long] + [C.c_void_p] * 4
    hi, wi = c.imp_shape
    c.frame()  # the key frame
    checked = nonzero = 0
    for coded in range(1, n):
        c.frame()
        got = c.importances()
        last = min(coded + W, n - 1)
        data = {}
        for m in range(coded, last + 1):
            intra = np.zeros((hi, wi), np.uint32)
            mv8 = np.zeros((refs, hi, wi, 2), np.int16)
            inter = np.zeros((refs, hi, wi), np.uint32)
            rd = np.zeros(2, np.int32)
            assert L.orc_replay_la_data(c.h, m, intra.ctypes.data, mv8.ctypes.data,
                                        inter.ctypes.data, rd.ctypes.data) == 0, (coded, m)
            data[m] = (intra, mv8, inter, list(rd[:refs]))
        imp = {m: np.zeros((hi, wi), np.float32) for m in data}
        for m in range(last, coded, -1):
            intra, mv8, inter, rd = data[m]
            uniq = []
            for k, d in enumerate(rd):
                if d not in [rd[j] for j in uniq]:
                    uniq.append(k)
            for k in uniq:
                t = coded_of_display(rd[k])
                if t < coded:
                    continue
                _propagate(mv8[k], inter[k], intra, imp[m], len(uniq), imp[t])
        ic = data[coded][0].astype(np.float32)
        want = np.zeros((hi, wi), np.float32)
        nz = ic > 0
        L.orc_log2f.restype = C.c_float
        L.orc_log2f.argtypes = [C.c_float]
        arg = (np.float32(1) + imp[coded][nz] / ic[nz]).astype(np.float32)
        want[nz] = [L.orc_log2f(float(a)) for a in arg]
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32),
                                      err_msg="coded frame %d" % coded)
        nonzero += bool((got > 0).any())  # level-2 frames are not referenced: zero
        checked += 1
    assert checked == n - 1 and nonzero >= (n - 1) // 2


def test_importance_window_changes_the_decision_inputs_only():
    """W = 0 keeps the input importances (zero: bias 0.65); a window gives
    non-negative importances and codes every frame."""
    w, h, n = 192, 128, 6
    fr = [RP.synth_frame(w, h, t, 1, 1, 8) for t in range(n + 6)]
    a = O.CpuReplay(w, h, n_inputs=len(fr), threads=2)
    b = O.CpuReplay(w, h, n_inputs=len(fr), threads=2, imp_window=3)
    for i, f in enumerate(fr):
        a.set_input(i, f)
        b.set_input(i, f)
    for _ in range(n):
        a.frame()
        b.frame()
        assert (a.importances() == 0).all()
        assert (b.importances() >= 0).all()
    assert (b.importances() > 0).any()
    with pytest.raises(AssertionError):
        O.CpuReplay(w, h, group=(1, 0, 2, 2), n_inputs=4, imp_window=2)
