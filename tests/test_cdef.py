"""CDEF (src/cdef.rs): the oracle's restatement (oracle/orc_cdef.c) pinned
by vectors from evaluating the reference's own cdef_find_dir,
cdef_filter_block and adjust_strength (tests/golden/ref_cdef.npz, made by
tools/refeval/gen_golden_ref.py cdef, release semantics: debug_assert! off,
i32 wrap-around), and the HIP frame filter (rv_cdef_find_dirs +
rv_cdef_filter_plane) against the oracle's cdef_filter_frame on random
frames: every bit depth, 4:2:0 / 4:2:2 / 4:4:4, sizes that are not
multiples of 64 (the padded copy's CDEF_VERY_LARGE ring and its 128-filled
remainder), skip blocks and per-superblock strength indices.  Frame sizes
are multiples of 8, as rav1e's reconstruction always is (Frame::new,
src/frame/mod.rs:58-59); the C ABI rejects others."""
import os

import numpy as np
import pytest

from tests import oracle_lib as O

GOLD = os.path.join(os.path.dirname(__file__), "golden", "ref_cdef.npz")


def _gold():
    return np.load(GOLD)


def test_find_dir_vs_reference():
    g = _gold()
    for img, cs, d, v in zip(g["dir_img"], g["dir_shift"], g["dir_dir"], g["dir_var"]):
        assert O.cdef_find_dir(img, int(cs)) == (int(d), int(v))


def test_filter_block_vs_reference():
    g = _gold()
    n = 0
    for (bd, xdec, ydec, pri, sec, dr, damping), src, want in zip(
            g["filt_cases"], g["filt_src"], g["filt_dst"]):
        src = np.ascontiguousarray(src)
        hbd = bd > 8
        out = np.zeros((8, 8), np.uint16 if hbd else np.uint8)
        O.lib().orc_cdef_filter_block(O.ptr(out), 8, int(hbd), O.ptr(src, 2 * 12 + 2), 12,
                                      int(pri), int(sec), int(dr), int(damping), int(bd),
                                      int(xdec), int(ydec))
        ys, xs = 8 >> ydec, 8 >> xdec
        assert (out[:ys, :xs] == want[:ys, :xs]).all(), (bd, xdec, ydec, pri, sec, dr)
        n += int((want[:ys, :xs] != src[2:2 + ys, 2:2 + xs]).any())
    assert n > 40  # most cases change something


def test_adjust_strength_vs_reference():
    g = _gold()
    for (s, v), want in zip(g["adj_cases"], g["adj_out"]):
        assert O.cdef_adjust_strength(int(s), int(v)) == int(want)


def _frame(rng, w, h, xdec, ydec, bd, skip_p=0.3):
    def plane(pw, ph):
        yy, xx = np.mgrid[0:ph, 0:pw]
        img = ((xx * 3 + yy * 5) % 97) * 2 + np.kron(
            rng.integers(0, 60, ((ph + 7) // 8, (pw + 7) // 8)), np.ones((8, 8)))[:ph, :pw]
        img = img + rng.integers(-4, 5, (ph, pw))
        img = img * (1 << (bd - 8)) + (1 << bd) // 4
        return np.clip(img, 0, (1 << bd) - 1).astype(np.uint16 if bd > 8 else np.uint8)
    cw, ch = (w + xdec) >> xdec, (h + ydec) >> ydec
    planes = [plane(w, h), plane(cw, ch), plane(cw, ch)]
    mi_w, mi_h = 2 * ((w + 7) // 8), 2 * ((h + 7) // 8)
    skip = (rng.random((mi_h // 2, mi_w // 2)) < skip_p).astype(np.uint8)
    skip = np.kron(skip, np.ones((2, 2), np.uint8))
    skip[0::2, 0::2] |= (rng.random((mi_h // 2, mi_w // 2)) < 0.1).astype(np.uint8)
    idx = rng.integers(0, 8, ((h + 63) // 64, (w + 63) // 64)).astype(np.uint8)
    return planes, skip, idx


# FrameInvariants::new's tables (src/encoder.rs:667-686)
Y_STR = [0 * 4 + 0, 1 * 4 + 0, 2 * 4 + 1, 3 * 4 + 1, 5 * 4 + 2, 7 * 4 + 3, 10 * 4 + 3, 13 * 4 + 3]


def test_oracle_frame_skip_and_zero_strength_are_identity():
    rng = np.random.default_rng(5)
    planes, skip, idx = _frame(rng, 72, 40, 1, 1, 8)
    out, _, _ = O.cdef_filter_frame(planes, 72, 40, 1, 1, np.ones_like(skip), idx, Y_STR,
                                    Y_STR)
    assert all((a == b).all() for a, b in zip(out, planes))
    out, _, _ = O.cdef_filter_frame(planes, 72, 40, 1, 1, skip, idx, [0] * 8, [0] * 8)
    assert all((a == b).all() for a, b in zip(out, planes))
    out, dirs, _ = O.cdef_filter_frame(planes, 72, 40, 1, 1, skip, idx, Y_STR, Y_STR)
    assert any((a != b).any() for a, b in zip(out, planes))
    assert dirs.max() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("bd,xdec,ydec,w,h", [(8, 1, 1, 200, 136), (8, 1, 1, 136, 80),
                                              (10, 1, 0, 136, 72), (12, 0, 0, 128, 96),
                                              (10, 1, 1, 264, 72), (8, 0, 0, 64, 64)])
def test_cdef_frame_vs_oracle(bd, xdec, ydec, w, h):
    import rav1e_amd as R
    R.require_device(0)
    rng = np.random.default_rng(3000 + bd + 7 * w + xdec + 3 * h)
    for trial in range(3):
        planes, skip, idx = _frame(rng, w, h, xdec, ydec, bd)
        ys = [int(v) for v in rng.integers(0, 64, 8)]
        us = [int(v) for v in rng.integers(0, 64, 8)]
        if trial == 0:
            ys, us = Y_STR, Y_STR
        damping = 3 + (trial == 2)
        want, wdir, wvar = O.cdef_filter_frame(planes, w, h, xdec, ydec, skip, idx, ys, us,
                                               damping, bd)
        src, dst = [], []
        for p, a in enumerate(planes):
            xd, yd = (0, 0) if p == 0 else (xdec, ydec)
            src.append(R.DevicePlane.from_array(a, xpad=16, ypad=16, xdec=xd, ydec=yd))
            dst.append(R.DevicePlane.from_array(np.zeros_like(a), xpad=8, ypad=8, xdec=xd,
                                                ydec=yd, pad=False))
        gdir, gvar = R.cdef_filter_frame(src, dst, w, h, skip, idx, ys, us, damping, bd)
        nz = skip.reshape(skip.shape[0] // 2, 2, skip.shape[1] // 2, 2).min(axis=(1, 3)) == 0
        assert (gdir[nz] == wdir[nz]).all() and (gvar[nz] == wvar[nz]).all(), trial
        for p in range(3):
            got = dst[p].download_visible()
            bad = np.argwhere(got != want[p])
            assert bad.size == 0, (trial, p, bad[:5])
        assert any((want[p] != planes[p]).any() for p in range(3))
