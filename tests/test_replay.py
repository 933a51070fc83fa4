"""Replay driver: the HIP schedule (rv_replay_*) must reproduce the CPU
replay (oracle/orc_replay.c, the same schedule over the oracle's
restatements) word for word; CPU-only tests pin the CPU replay itself."""
import numpy as np
import pytest

from rav1e_amd import replay as RP
from tests import oracle_lib as O


def _frames(w, h, xdec, ydec, bd, n):
    return [RP.synth_frame(w, h, t, xdec, ydec, bd) for t in range(n)]


def test_synth_frames_deterministic_and_moving():
    a = RP.synth_frame(128, 64, 3)
    b = RP.synth_frame(128, 64, 3)
    c = RP.synth_frame(128, 64, 4)
    assert a.dtype == np.uint8 and a.size == 128 * 64 * 3 // 2
    np.testing.assert_array_equal(a, b)
    assert (a != c).mean() > 0.5
    t10 = RP.synth_frame(128, 64, 3, bd=10)
    assert t10.dtype == np.uint16 and t10.max() <= 1023
    assert np.array_equal(t10[: 128 * 64] >> 2, a[: 128 * 64])


def test_cpu_replay_thread_invariant():
    fr = _frames(192, 128, 1, 1, 8, 3)
    outs = []
    for threads in (1, 3):
        r = O.CpuReplay(192, 128, 1, 1, 8, 2, threads=threads)
        for s, f in enumerate(fr):
            r.set_frame(s, f)
        r.frame(2)
        outs.append(r.results())
    np.testing.assert_array_equal(outs[0], outs[1])
    w = outs[0]
    nsb = 3 * 2
    assert w[-1] == (192 // 8) * (128 // 8)  # importance blocks
    assert w[-2] > 0 and w[-3] > 0  # satd sum, recon checksum
    # the motion found at full res tracks the synthetic global motion
    # (1.25, 0.75) px/frame: reference slot 1 is frame t=1, slot 0 is t=0
    per = 8 * 2 + 2
    subs = [int(w[sb * per + 6]) for sb in range(nsb)]
    cols = [((s & 0xFFFF) ^ 0x8000) - 0x8000 for s in subs]
    assert np.median(cols) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,xdec,ydec,bd,refs,tile", [
    (256, 192, 1, 1, 8, 2, None),
    (320, 128, 0, 0, 8, 1, None),
    (256, 128, 1, 1, 10, 2, None),
    (192, 128, 1, 1, 12, 1, None),  # 12 bits: exhaustive full search, 12-bit RDO kernel
    (384, 192, 1, 1, 8, 2, (2, 0, 4, 3)),
])
@pytest.mark.parametrize("flags", [0, RP.RV_REPLAY_SIDE_RDO, RP.RV_REPLAY_SPLIT_RDO,
                                   RP.RV_REPLAY_EXHAUSTIVE_FS])
def test_gpu_replay_matches_cpu_replay(w, h, xdec, ydec, bd, refs, tile, flags):
    import rav1e_amd as R
    R.require_device(0)
    fr = _frames(w, h, xdec, ydec, bd, refs + 1)
    g = RP.HipReplay(w, h, xdec, ydec, bd, refs, tile=tile, flags=flags)
    c = O.CpuReplay(w, h, xdec, ydec, bd, refs, tile=tile, threads=4)
    for s, f in enumerate(fr):
        g.set_frame(s, f)
        c.set_frame(s, f)
    for scale in (1, 2, 4):
        g.frame(scale)
        c.frame(scale)
        gw, cw = g.results(), c.results()
        bad = np.nonzero(gw != cw)[0]
        assert bad.size == 0, (scale, bad[:10], gw[bad[:10]], cw[bad[:10]])
    assert len(g.stage_ms()) == 10


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["1080p", "2160p", "2160p10", "2160p444"])
def test_gpu_replay_full_size_gop(config):
    """One GOP (me_range_scale 4, 2, 1, 1) at the BASELINE shapes, GPU words
    equal to the CPU replay's frame by frame."""
    import bench
    import rav1e_amd as R
    R.require_device(0)
    w, h, xdec, ydec, bd = bench.CONFIGS[config]
    fr = _frames(w, h, xdec, ydec, bd, 3)
    g = RP.HipReplay(w, h, xdec, ydec, bd, 2)
    c = O.CpuReplay(w, h, xdec, ydec, bd, 2, threads=O.cpu_share())
    for s, f in enumerate(fr):
        g.set_frame(s, f)
        c.set_frame(s, f)
    for i, scale in enumerate(RP.GOP_SCALES):
        g.frame(scale)
        c.frame(scale)
        gw, cw = g.results(), c.results()
        bad = np.nonzero(gw != cw)[0]
        assert bad.size == 0, (config, i, scale, bad[:10], gw[bad[:10]], cw[bad[:10]])
    g.close()
    c.close()
