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


def _pos_to_lvl(pos, depth=2):
    """src/encoder.rs:555-564"""
    v = pos | (1 << depth)
    return depth - ((v & -v).bit_length() - 1)


def rav1e_propagation_refs(n_coded):
    """Per coded frame m >= 1: the displays compute_block_importances
    propagates frame m's importance into, in its order -- unique_indices:
    fi.ref_frames de-duplicated by DPB slot, in mv index order
    (src/api/internal.rs:875-882) -- derived from rav1e's own tables, not
    the replay's: InterConfig with reorder, multiref, pyramid_depth 2,
    group_input_len 4 (:40-95), a group's output order idx_in_group_output
    0..5 with get_level / get_show_existing_frame / get_order_hint /
    get_slot_idx (:104-166), FrameInvariants::new_inter_frame's ref_frames
    (src/encoder.rs:761-828: level 0 LAST = the previous P slot, LAST2 the
    one before; level > 0 all = the backward slot, ALTREF the forward one,
    LAST3 its own slot), and the key frame filling every slot
    (refresh_frame_flags ALL_REF_FRAMES_MASK, :658).  Slot contents follow
    refresh_frame_flags in coding order (SEF frames refresh nothing)."""
    depth, gil = 2, 4
    slots = [0] * 8  # the display each DPB slot holds after the key frame
    out, m, g = {}, 0, 0
    while m < n_coded - 1:
        for idx in range(6):
            if idx >= depth and bin(idx - depth + 1).count("1") == 1 and idx != depth:
                continue  # show_existing_frame
            level = idx if idx < depth else _pos_to_lvl(idx - depth + 1, depth)
            offset = gil >> idx if idx < depth else idx - depth + 1
            oh = gil * g + offset

            def slot_of(o):
                lv = _pos_to_lvl(o, depth)
                return (o >> depth) % 4 if lv == 0 else 3 + lv
            slot_idx = (oh >> depth) & 3 if level == 0 else 3 + level
            if level == 0:
                rf = [(slot_idx + 4 - 1) % 4] * 7
                rf[1] = (slot_idx + 4 - 2) % 4  # LAST2: second_ref_frame at idx 0
            else:
                rf = [slot_of(oh - (gil >> level))] * 7
                rf[6] = slot_of(oh + (gil >> level))  # ALTREF
                rf[2] = slot_idx  # LAST3: ref_in_previous_group
            uniq = []
            for sl in rf:
                if sl not in uniq:
                    uniq.append(sl)
            m += 1
            out[m] = (oh, [slots[sl] for sl in uniq])
            slots[slot_idx] = oh
        g += 1
    return out


def test_lookahead_references_follow_rav1e_slots():
    """The oracle's and the GPU library's lookahead references (the slots the
    propagation splits over) equal rav1e's, frame by frame over 10 GOPs."""
    import rav1e_amd as R
    L = O.lib()
    L.orc_replay_la_refs.argtypes = [C.c_long, C.c_int, C.c_void_p]
    want = rav1e_propagation_refs(41)
    for m, (disp, refs) in want.items():
        assert RP.frame_info(m)["display"] == disp
        for name, fn in (("oracle", L.orc_replay_la_refs), ("hip", R.lib().rv_replay_la_refs)):
            out = np.zeros(7, np.int32)
            assert fn(m, 2, out.ctypes.data) == 0
            n = int(out[0])
            got = [int(out[1 + int(out[4 + i])]) for i in range(n)]
            assert got == refs, (name, m, disp, got, refs)
    # the first GOP: two slots holding the key frame count twice
    assert want[1][1] == [0, 0] and want[2][1] == [0, 0, 4] and want[3][1] == [0, 0, 2]


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
    rv_refs = rav1e_propagation_refs(n)
    c.frame()  # the key frame
    checked = nonzero = 0
    for coded in range(1, n):
        c.frame()
        got = c.importances()
        last = min(coded + W, n - 1)
        data = {}
        for m in range(coded, last + 1):
            intra = np.zeros((hi, wi), np.uint32)
            mv8 = np.zeros((3, hi, wi, 2), np.int16)
            inter = np.zeros((3, hi, wi), np.uint32)
            rd = np.zeros(7, np.int32)
            assert L.orc_replay_la_data(c.h, m, intra.ctypes.data, mv8.ctypes.data,
                                        inter.ctypes.data, rd.ctypes.data) == 0, (coded, m)
            nr = int(rd[0])
            order = [int(rd[4 + i]) for i in range(nr)]
            # the oracle's lookahead references, in propagation order, are rav1e's
            assert [int(rd[1 + k]) for k in order] == rv_refs[m][1], (m, rd)
            data[m] = (intra, mv8, inter, [int(rd[1 + k]) for k in range(nr)], order)
        imp = {m: np.zeros((hi, wi), np.float32) for m in data}
        for m in range(last, coded, -1):
            intra, mv8, inter, rd, order = data[m]
            for k in order:
                t = coded_of_display(rd[k])
                if t < coded:
                    continue
                _propagate(mv8[k], inter[k], intra, imp[m], len(order), imp[t])
        ic = data[coded][0].astype(np.float32)
        want = np.zeros((hi, wi), np.float32)
        nz = ic > 0
        L.orc_log2f.restype = C.c_float
        L.orc_log2f.argtypes = [C.c_float]
        arg = (np.float32(1) + imp[coded][nz] / ic[nz]).astype(np.float32)
        want[nz] = [L.orc_log2f(float(a)) for a in arg]
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32),
                                      err_msg="coded frame %d" % coded)
        nonzero += bool((got > 0).any())
        checked += 1
    # level-2 frames are LAST3 of the next level-2 frame: only the window's
    # last frames (nothing after them yet) stay zero
    assert checked == n - 1 and nonzero >= n - 3


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
    # a tile group's window needs the other groups' lookahead parts first
    g = O.CpuReplay(w, h, group=(1, 0, 2, 2), n_inputs=len(fr), imp_window=2)
    for i, f in enumerate(fr):
        g.set_input(i, f)
    g.frame()  # the key frame
    with pytest.raises(AssertionError):
        g.frame()
    assert g.la_due()[:2] == (1, 3)
