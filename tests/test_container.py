"""The stream containers either side of the hot path (rv_container.hip):
the y4m reader (the input of rav1e's CLI, src/bin/decoder/y4m.rs over the
y4m crate, restated from the format's definition -- the crate is absent, so
parity is pinned by files this test writes byte for byte) and the IVF
writer (ivf/src/lib.rs:6-30, whose field layout the test reads back with
the reference's own read_header / read_packet order). Host code: no GPU."""
import os
import struct

import numpy as np
import pytest

import rav1e_amd as R


def _write_y4m(path, frames, w, h, cs, fps=(30000, 1001), extra=""):
    with open(path, "wb") as f:
        f.write(("YUV4MPEG2 W%d H%d F%d:%d Ip A1:1 C%s%s\n" % (w, h, fps[0], fps[1], cs, extra)).encode())
        for fr in frames:
            f.write(b"FRAME\n")
            f.write(fr.astype("<u2" if fr.dtype == np.uint16 else np.uint8).tobytes())


@pytest.mark.parametrize("cs,bd,xd,yd", [("420jpeg", 8, 1, 1), ("420", 8, 1, 1), ("420p10", 10, 1, 1),
                                         ("444", 8, 0, 0), ("422p12", 12, 1, 0)])
def test_y4m_reader_frames(tmp_path, cs, bd, xd, yd):
    w, h = 70, 34  # odd chroma sizes in 4:2:0 / 4:2:2
    cw, ch = (w + xd) >> xd, (h + yd) >> yd
    n = w * h + 2 * cw * ch
    rng = np.random.default_rng(7)
    dt = np.uint16 if bd > 8 else np.uint8
    frames = [rng.integers(0, 1 << bd, n).astype(dt) for _ in range(3)]
    p = str(tmp_path / "in.y4m")
    _write_y4m(p, frames, w, h, cs)
    with R.Y4mReader(p) as y:
        i = y.info
        assert (i.width, i.height, i.bit_depth, i.xdec, i.ydec, i.fps_num, i.fps_den) == (
            w, h, bd, xd, yd, 30000, 1001)
        for fr in frames:
            got = y.read_frame()
            assert got is not None and got.dtype == dt
            np.testing.assert_array_equal(got, fr)
        assert y.read_frame() is None


def test_y4m_header_errors(tmp_path):
    info = R.Y4mInfo()
    L = R.lib()
    assert L.rv_y4m_parse_header(b"YUV4MPEG2 W16 H8 F25:1 Cmono", R.C.byref(info)) != 0
    assert L.rv_y4m_parse_header(b"YUV4MPEG W16 H8", R.C.byref(info)) != 0
    assert L.rv_y4m_parse_header(b"YUV4MPEG2 H8 F25:1", R.C.byref(info)) != 0
    assert L.rv_y4m_parse_header(b"YUV4MPEG2 W16 H8 F25:1 XCOMMENT=1", R.C.byref(info)) == 0
    assert (info.width, info.height, info.bit_depth, info.xdec, info.ydec) == (16, 8, 8, 1, 1)
    # a truncated frame is an error, not the end of the stream
    p = str(tmp_path / "t.y4m")
    with open(p, "wb") as f:
        f.write(b"YUV4MPEG2 W16 H8 F25:1 C420\nFRAME\n" + bytes(100))
    with R.Y4mReader(p) as y, pytest.raises(R.Rav1eHipError):
        y.read_frame()


def test_ivf_writer_layout(tmp_path):
    p = str(tmp_path / "out.ivf")
    pkts = [(0, b"\x12\x00\x0a\x0b"), (1, b""), (7, bytes(range(200)))]
    with R.IvfWriter(p, 3840, 2160, 60, 1) as v:
        for pts, d in pkts:
            v.write_frame(pts, d)
    b = open(p, "rb").read()
    # read_header (ivf/src/lib.rs:42-70): signature, two u16, tag, w, h,
    # then the two u32 the writer stored as framerate num, den
    assert b[:4] == b"DKIF"
    v0, v1 = struct.unpack_from("<HH", b, 4)
    assert (v0, v1) == (0, 32)
    assert b[8:12] == b"AV01"
    assert struct.unpack_from("<HHIIII", b, 12) == (3840, 2160, 60, 1, 0, 0)
    off = 32
    for pts, d in pkts:  # read_packet (:77-84)
        n, t = struct.unpack_from("<IQ", b, off)
        assert (n, t) == (len(d), pts)
        assert b[off + 12:off + 12 + n] == d
        off += 12 + n
    assert off == len(b)
