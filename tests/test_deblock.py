"""Deblocking filter (deblock_plane, src/deblock.rs:1174-1335): the oracle's
restatement (oracle/orc_deblock.c) and the HIP kernel (rv_deblock_plane)
against vectors made by evaluating the reference's own deblock_plane text
(tests/golden/ref_deblock.npz, tools/refeval/gen_golden_ref.py deblock: every
filter size 4/6/8/14, 8/10/12-bit, 4:2:0 / 4:2:2 / 4:4:4, 4x4 .. 64x64
blocks, skip blocks, per-plane levels incl. 0); the HIP kernel against the
oracle on larger random layouts; the oracle's own behaviour (a step edge
inside the filter's reach is smoothed, level 0 is a no-op, the fast levels
of deblock_filter_optimize)."""
import os

import numpy as np
import pytest

from tests import oracle_lib as O

GOLD = os.path.join(os.path.dirname(__file__), "golden", "ref_deblock.npz")
GOLD_SSE = os.path.join(os.path.dirname(__file__), "golden", "ref_sse.npz")


def _ref_cases():
    g = np.load(GOLD)
    off = 0
    for c in g["cases"]:
        W, H, xdec, ydec, bd, pli = (int(v) for v in c[:6])
        levels = [int(v) for v in c[6:10]]
        m = int(c[10])
        xd, yd = (xdec, ydec) if pli else (0, 0)
        pw, ph = (W + xd) >> xd, (H + yd) >> yd
        n = pw * ph
        cols, rows = (W + 3) // 4, (H + 3) // 4
        mo = g["map_off"]
        lg = g["lg"][mo[m]:mo[m + 1]].reshape(rows, cols)
        sk = g["skip"][mo[m]:mo[m + 1]].reshape(rows, cols)
        px = np.uint16 if bd > 8 else np.uint8
        img = g["px_in"][off:off + n].reshape(ph, pw).astype(px)
        want = g["px_out"][off:off + n].reshape(ph, pw).astype(px)
        off += n
        yield (W, H, xd, yd, bd, pli, levels, lg, sk, img, want)


def test_oracle_deblock_vs_reference():
    n = changed = 0
    for W, H, xd, yd, bd, pli, levels, lg, sk, img, want in _ref_cases():
        pad = 16
        full = np.pad(img, pad, mode="edge")
        got = O.deblock_plane(full.copy(), pad, pad, W, H, xd, yd, pli, lg, sk, levels, bd)
        got = got[pad:pad + img.shape[0], pad:pad + img.shape[1]]
        bad = np.argwhere(got != want)
        assert bad.size == 0, (W, H, bd, xd, yd, pli, levels, bad[:5])
        n += 1
        changed += int((want != img).any())
    assert n == 24 and changed >= 18


def _sse_cases():
    """sse_plane / sse_optimize vectors (tools/refeval/gen_golden_ref.py sse:
    the reference's text evaluated on 128-padded planes)"""
    g = np.load(GOLD_SSE)
    off = 0
    mo = g["map_off"]
    for i, c in enumerate(g["cases"]):
        W, H, xdec, ydec, bd, m = (int(v) for v in c)
        cols, rows = (W + 3) // 4, (H + 3) // 4
        lg = g["lg"][mo[m]:mo[m + 1]].reshape(rows, cols)
        sk = g["skip"][mo[m]:mo[m + 1]].reshape(rows, cols)
        px = np.uint16 if bd > 8 else np.uint8
        recs, srcs = [], []
        for pli in range(3):
            xd, yd = (xdec, ydec) if pli else (0, 0)
            pw, ph = (W + xd) >> xd, (H + yd) >> yd
            recs.append(g["rec"][off:off + pw * ph].reshape(ph, pw).astype(px))
            srcs.append(g["src"][off:off + pw * ph].reshape(ph, pw).astype(px))
            off += pw * ph
        yield (W, H, xdec, ydec, bd, lg, sk, recs, srcs, g["tally"][i], list(g["levels"][i]))


def test_oracle_sse_optimize_vs_reference():
    """sse_optimize (src/deblock.rs:1418-1475): every plane's tallies and
    the chosen levels equal the reference's, incl. the horizontal tally's
    row-wise taps (sse_h_edge, :1129-1171) reading the 128 padding."""
    n = nonzero = 0
    for W, H, xdec, ydec, bd, lg, sk, recs, srcs, tally, levels in _sse_cases():
        vs, hs = [], []
        for pli in range(3):
            xd, yd = (xdec, ydec) if pli else (0, 0)
            v, h = O.deblock_sse_plane(recs[pli], srcs[pli], W, H, xd, yd, pli, lg, sk, bd)
            assert (v == tally[pli][:65]).all(), (W, H, bd, pli, np.argwhere(v != tally[pli][:65]))
            assert (h == tally[pli][65:]).all(), (W, H, bd, pli, np.argwhere(h != tally[pli][65:]))
            vs.append(v)
            hs.append(h)
        assert O.deblock_sse_levels(vs, hs) == levels, (W, H, bd, levels)
        n += 1
        nonzero += any(levels)
    assert n == 8 and nonzero >= 5


def _layout(rng, mi_w, mi_h, min_lg=1):
    """A random quad-tree of square blocks 64x64 .. 8x8 over the 4x4 grid:
    lg (log2 width in 4x4 units) and skip per 4x4 block."""
    lg = np.zeros((mi_h, mi_w), np.uint8)
    skip = np.zeros((mi_h, mi_w), np.uint8)

    def place(x, y, l):
        if x >= mi_w or y >= mi_h:
            return
        if l > min_lg and rng.random() < 0.6:
            h = 1 << (l - 1)
            for dy in (0, h):
                for dx in (0, h):
                    place(x + dx, y + dy, l - 1)
            return
        n = 1 << l
        lg[y:y + n, x:x + n] = l
        skip[y:y + n, x:x + n] = rng.random() < 0.5
    for y in range(0, mi_h, 16):
        for x in range(0, mi_w, 16):
            place(x, y, 4)
    return lg, skip


def _blocky(rng, h, w, bd):
    """8x8-blocky content plus noise: every edge has something to filter."""
    base = rng.integers(0, 1 << bd, ((h + 7) // 8, (w + 7) // 8))
    img = np.kron(base, np.ones((8, 8), np.int64))[:h, :w]
    img = img // 4 + (1 << bd) * 3 // 8 + rng.integers(-2, 3, (h, w))
    return np.clip(img, 0, (1 << bd) - 1).astype(np.uint16 if bd > 8 else np.uint8)


def test_oracle_smooths_a_step_and_level_zero_is_identity():
    w, h = 64, 32
    img = np.zeros((h + 32, w + 32), np.uint8)
    img[:, : 16 + 32] = 100
    img[:, 16 + 32:] = 106
    lg = np.full((h // 4, w // 4), 2, np.uint8)  # 16x16 blocks: an edge at x = 32
    skip = np.zeros_like(lg)
    a = O.deblock_plane(img.copy(), 16, 16, w, h, 0, 0, 0, lg, skip, [0, 0, 0, 0])
    assert (a == img).all()
    b = O.deblock_plane(img.copy(), 16, 16, w, h, 0, 0, 0, lg, skip, [20, 20, 0, 0])
    row = b[20, 16 + 24:16 + 40].astype(int)
    assert (np.diff(row) >= 0).all() and np.abs(np.diff(row)).max() < 6
    # the fast levels (speed >= 8): 8-bit inter frame at ac_q 128
    assert O.deblock_fast_level(128, 8) == (128 * 6017 + 650707 + (1 << 17)) >> 18


@pytest.mark.gpu
@pytest.mark.parametrize("bd,xdec,ydec,w,h", [(8, 1, 1, 200, 136), (10, 1, 1, 136, 72),
                                              (12, 0, 0, 128, 96), (8, 0, 0, 256, 64)])
def test_deblock_plane_vs_oracle(bd, xdec, ydec, w, h):
    import rav1e_amd as R
    R.require_device(0)
    rng = np.random.default_rng(2000 + bd + 7 * w + xdec)
    mi_w, mi_h = (w + 3) // 4, (h + 3) // 4
    for trial in range(3):
        lg, skip = _layout(rng, mi_w, mi_h)
        levels = [int(v) for v in rng.integers(0, 64, 4)]
        if trial == 0:
            levels = [63, 63, 63, 63]
        for pli in range(3):
            pw = w if pli == 0 else (w + xdec) >> xdec
            ph = h if pli == 0 else (h + ydec) >> ydec
            xd, yd = (0, 0) if pli == 0 else (xdec, ydec)
            img = _blocky(rng, ph, pw, bd)
            dp = R.DevicePlane.from_array(img, xpad=88 >> xd, ypad=88 >> yd, xdec=xd, ydec=yd)
            full = dp.download_full()
            xo, yo = dp.desc.xorigin, dp.desc.yorigin
            R.deblock_plane(dp, pli, w, h, lg, skip, levels, bd)
            want = O.deblock_plane(full.copy(), yo, xo, w, h, xd, yd, pli, lg, skip, levels, bd)
            got = dp.download_full()
            bad = np.argwhere(got != want)
            assert bad.size == 0, (trial, pli, levels, bad[:5])
            if trial == 0:
                assert (got != full).any()  # something was filtered


@pytest.mark.gpu
def test_deblock_plane_vs_reference():
    import rav1e_amd as R
    R.require_device(0)
    for W, H, xd, yd, bd, pli, levels, lg, sk, img, want in _ref_cases():
        dp = R.DevicePlane.from_array(img, xpad=88 >> xd, ypad=88 >> yd, xdec=xd, ydec=yd)
        R.deblock_plane(dp, pli, W, H, lg, sk, levels, bd)
        got = dp.download_visible()
        bad = np.argwhere(got != want)
        assert bad.size == 0, (W, H, bd, xd, yd, pli, levels, bad[:5])


def _dev_planes(R, imgs, xdec, ydec):
    return [R.DevicePlane.from_array(im, xpad=88 >> (xdec if p else 0), ypad=88 >> (ydec if p else 0),
                                     xdec=xdec if p else 0, ydec=ydec if p else 0)
            for p, im in enumerate(imgs)]


@pytest.mark.gpu
def test_deblock_sse_vs_reference():
    """rv_deblock_sse: the tallies and levels of the reference's sse_plane /
    sse_optimize vectors.  The device planes' borders are replicated: the
    kernel must read 128 outside the width, as rav1e's fresh planes hold."""
    import rav1e_amd as R
    R.require_device(0)
    for W, H, xdec, ydec, bd, lg, sk, recs, srcs, tally, levels in _sse_cases():
        rec = _dev_planes(R, recs, xdec, ydec)
        src = _dev_planes(R, srcs, xdec, ydec)
        got_t, got_l = R.deblock_sse(rec, src, W, H, lg, sk, bd)
        assert (got_t.reshape(3, 130) == tally).all(), (W, H, bd, np.argwhere(got_t.reshape(3, 130) != tally)[:5])
        assert got_l == levels, (W, H, bd, got_l, levels)


@pytest.mark.gpu
@pytest.mark.parametrize("bd,xdec,ydec,w,h", [(8, 1, 1, 200, 136), (10, 1, 0, 136, 72),
                                              (12, 0, 0, 128, 96), (8, 1, 1, 320, 184)])
def test_deblock_sse_and_frame_vs_oracle(bd, xdec, ydec, w, h):
    """sse_optimize + deblock_filter_frame with the levels kept on the
    device, against the oracle, on blocky reconstructions of a smooth source."""
    import rav1e_amd as R
    R.require_device(0)
    rng = np.random.default_rng(4000 + bd + 5 * w + ydec)
    mi_w, mi_h = (w + 3) // 4, (h + 3) // 4
    for trial in range(3):
        lg, skip = _layout(rng, mi_w, mi_h, min_lg=0 if trial == 2 else 1)
        recs, srcs = [], []
        for pli in range(3):
            xd, yd = (xdec, ydec) if pli else (0, 0)
            pw, ph = (w + xd) >> xd, (h + yd) >> yd
            yy, xx = np.mgrid[0:ph, 0:pw]
            src = (xx * rng.uniform(0.2, 1.5) + yy * rng.uniform(0.2, 1.5) + 40) * (1 << (bd - 8))
            amp = (1 + 3 * trial) << (bd - 8)
            rec = src + np.kron(rng.integers(-amp, amp + 1, ((ph + 7) // 8, (pw + 7) // 8)),
                                np.ones((8, 8)))[:ph, :pw]
            dt = np.uint16 if bd > 8 else np.uint8
            srcs.append(np.clip(src, 0, (1 << bd) - 1).astype(dt))
            recs.append(np.clip(rec, 0, (1 << bd) - 1).astype(dt))
        vs, hs = [], []
        for pli in range(3):
            xd, yd = (xdec, ydec) if pli else (0, 0)
            v, hh = O.deblock_sse_plane(recs[pli], srcs[pli], w, h, xd, yd, pli, lg, skip, bd)
            vs.append(v)
            hs.append(hh)
        want_l = O.deblock_sse_levels(vs, hs)
        rec = _dev_planes(R, recs, xdec, ydec)
        src = _dev_planes(R, srcs, xdec, ydec)
        got_t, got_l = R.deblock_sse(rec, src, w, h, lg, skip, bd)
        assert (got_t[:, 0] == np.array(vs)).all() and (got_t[:, 1] == np.array(hs)).all(), trial
        assert got_l == want_l, (trial, got_l, want_l)
        R.deblock_frame(rec, w, h, lg, skip, got_l, bd)
        for pli in range(3):
            xd, yd = (xdec, ydec) if pli else (0, 0)
            full = np.pad(recs[pli], 16, mode="edge")
            if want_l[0] or want_l[1]:
                O.deblock_plane(full, 16, 16, w, h, xd, yd, pli, lg, skip, want_l, bd)
            want = full[16:16 + recs[pli].shape[0], 16:16 + recs[pli].shape[1]]
            got = rec[pli].download_visible()
            assert (got == want).all(), (trial, pli, want_l, np.argwhere(got != want)[:5])
        if trial == 2:
            assert any(want_l)
