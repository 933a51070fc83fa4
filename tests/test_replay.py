"""Replay driver: the HIP stream schedule (rv_replay_*) must reproduce the CPU
replay (oracle/orc_replay.c, the same schedule over the oracle's
restatements) word for word, frame by frame; CPU-only tests pin the CPU
replay itself, the synthetic input and the host-side frame parameters."""
import numpy as np
import pytest

from rav1e_amd import rate as RT
from rav1e_amd import replay as RP
from tests import oracle_lib as O

PER_REF = RP.WORDS_PER_REF


def _frames(w, h, xdec, ydec, bd, n):
    return [RP.synth_frame(w, h, t, xdec, ydec, bd) for t in range(n)]


def _sb_words(words, nsb, refs):
    per = PER_REF * refs + 4
    return words[: nsb * per].reshape(nsb, per)


def test_synth_frames_deterministic_and_moving():
    a = RP.synth_frame(128, 64, 3)
    b = RP.synth_frame(128, 64, 3)
    c = RP.synth_frame(128, 64, 4)
    assert a.dtype == np.uint8 and a.size == 128 * 64 * 3 // 2
    np.testing.assert_array_equal(a, b)
    assert (a != c).mean() > 0.5
    assert 40 < a.mean() < 220 and a.std() > 10
    t10 = RP.synth_frame(128, 64, 3, bd=10)
    assert t10.dtype == np.uint16 and t10.max() <= 1023
    assert np.array_equal(t10[: 128 * 64] >> 2, a[: 128 * 64])


def test_tiling_matches_the_encoders_tiling():
    """TilingInfo::from_target_tiles / the --tiles loop (src/tiling/
    tiler.rs:49-126, src/encoder.rs:583-621) at the BASELINE configs."""
    c = RP.tiling_for(3840, 2160, tile_cols=8)
    assert (c["tile_width_sb"], c["tile_height_sb"], c["cols"], c["rows"]) == (8, 34, 8, 1)
    e = RP.tiling_for(3840, 2160, tiles=4)
    assert (e["tile_width_sb"], e["tile_height_sb"], e["cols"], e["rows"]) == (30, 17, 2, 2)
    b = RP.tiling_for(1920, 1080)
    assert (b["cols"], b["rows"]) == (1, 1)
    assert RP.tile_groups(c, 8)[-1] == (56, 0, 4, 34)
    assert RP.tile_groups(c, 2) == [(0, 0, 32, 34), (32, 0, 28, 34)]
    assert RP.tile_groups(e, 4)[3] == (30, 17, 30, 17)
    with pytest.raises(ValueError):
        RP.tile_groups(RP.tiling_for(3840, 2160, tile_cols=4, tile_rows=2), 3)


def test_fixed_quantizer_frame_params():
    """select_qi / new_from_log_q (src/rate.rs:570-606, 746-775) for
    --quantizer 100: the P frame keeps base_q_idx 100, the pyramid's B
    levels are 15-step coarser, lambda = ln2/6 * q^2 grows with the level;
    bexp64 / blog64 invert each other (src/rate.rs:108-267)."""
    for v in (1, 8, 100, 1000, 123456):
        assert RT.bexp64(RT.blog64(v)) == v
    assert RT.blog64(8) == RT.q57(3)
    lv = RT.level_params(100, 8)
    assert lv[0]["base_q_idx"] == 100
    assert lv[0]["base_q_idx"] < lv[1]["base_q_idx"] < lv[2]["base_q_idx"]
    assert 15 < lv[0]["lambda"] < lv[1]["lambda"] < lv[2]["lambda"] < 100
    assert all(p["dist_scale"][0] == 1.0 and p["dist_scale"][1] > 1 for p in lv)
    assert abs(lv[0]["me_lambda"] ** 2 - lv[0]["lambda"]) < 1e-9
    lv10 = RT.level_params(100, 10)
    assert abs(lv10[0]["lambda"] / lv[0]["lambda"] - 16) < 1.0


def test_cpu_replay_stream_and_thread_invariant():
    w, h = 256, 128
    fr = _frames(w, h, 1, 1, 8, 12)
    outs = []
    for threads in (1, 3):
        r = O.CpuReplay(w, h, 1, 1, 8, 2, n_inputs=12, threads=threads)
        for i, f in enumerate(fr):
            r.set_input(i, f)
        infos = [r.frame() for _ in range(6)]
        outs.append(r.results())
    np.testing.assert_array_equal(outs[0], outs[1])
    assert [i["display"] for i in infos] == [0, 4, 2, 1, 3, 8]
    assert infos[0]["is_key"] and [i["me_range_scale"] for i in infos[1:]] == [4, 2, 1, 1, 4]
    assert infos[3]["ref_display"] == [0, 2] and infos[5]["ref_display"] == [4, 0]
    wd = outs[0]
    assert wd[-2] == (w // 8) * (h // 8)  # importance blocks
    assert wd[-1] > 0 and wd[-3] > 0 and wd[-4] == wd[-1]  # one group: group sum = frame sum
    sb = _sb_words(wd, 8, 2)
    assert (sb[:, 2 * PER_REF] < 8).all() and set(np.unique(sb[:, 2 * PER_REF + 1])) <= {0, 1}
    # the NEWMV of the full-res search and the lookahead MVs track the
    # synthetic motion (1.25 px/frame; display 8 from 4: +5 px, i.e. +40 in
    # 1/8 pel, the source moving right: the reference block sits left)
    def col(w):
        return ((int(w) & 0xFFFF) ^ 0x8000) - 0x8000
    assert np.median([col(s) for s in sb[:, RP.W_SUB]]) < 0
    assert np.median([col(s) for s in sb[:, RP.W_LOOK:RP.W_LOOK + 32:2].ravel()]) < 0


def test_cpu_replay_reconstruction_is_the_reference():
    """The coded frame's reconstruction lands in the DPB: the key frame's
    reconstruction is its input, an inter frame's differs from its input
    but stays close (skip / residual coding of a good prediction)."""
    w, h = 192, 128
    fr = _frames(w, h, 1, 1, 8, 8)
    r = O.CpuReplay(w, h, 1, 1, 8, 2, n_inputs=8, threads=2)
    for i, f in enumerate(fr):
        r.set_input(i, f)
    r.frame()
    np.testing.assert_array_equal(r.get_recon(0), fr[0])
    r.frame()
    rec = r.get_recon(4).astype(np.int32)
    err = np.abs(rec - fr[4].astype(np.int32))
    assert err.mean() < 6 and (rec != fr[4]).any()


def test_cpu_replay_importance_bias():
    """compute_distortion_bias with block importances: a uniform importance
    3 gives bias 1.65 instead of 0.65 (src/rdo.rs:495-508): every
    distortion scales up, the searches do not change."""
    w, h = 192, 128
    fr = _frames(w, h, 1, 1, 8, 8)
    res = []
    for imp in (None, np.full((h // 8) * (w // 8), 3.0, np.float32)):
        r = O.CpuReplay(w, h, 1, 1, 8, 1, n_inputs=8, threads=2)
        for i, f in enumerate(fr):
            r.set_input(i, f)
        r.set_importances(imp)
        r.frame()
        r.frame()
        res.append(_sb_words(r.results(), 6, 1))
    np.testing.assert_array_equal(res[0][:, :PER_REF], res[1][:, :PER_REF])
    cost = [np.ascontiguousarray(x[:, PER_REF + 2]).view(np.float64) for x in res]
    assert (cost[1] >= cost[0]).all() and (cost[1] > cost[0]).any()


@pytest.mark.parametrize("deblock,speed", [(False, 10), (True, 10), (True, 6)])
def test_cpu_tile_groups_equal_the_whole_frame(deblock, speed):
    """Two tile groups coded separately and exchanging their
    reconstructions (with deblocking: and their block maps, each deblocking
    the whole frame) reproduce the single-instance run of the same tiling,
    superblock for superblock (tiles are independent, src/encoder.rs:
    2772-2781)."""
    w, h = 384, 192
    fr = _frames(w, h, 1, 1, 8, 10)
    t = RP.tiling_for(w, h, tile_cols=2)
    ts = (t["tile_width_sb"], t["tile_height_sb"])
    rects = RP.tile_groups(t, 2)
    kw = dict(n_inputs=10, threads=2, tile_size=ts, deblock=deblock, speed=speed)
    single = O.CpuReplay(w, h, **kw)
    gs = [O.CpuReplay(w, h, group=r, **kw) for r in rects]
    for e in [single] + gs:
        for i, f in enumerate(fr):
            e.set_input(i, f)
    sbc = (w + 63) // 64
    for _ in range(6):
        single.frame()
        for g in gs:
            g.frame(pad=False)
        bufs = [g.export(r) for g, r in zip(gs, rects)]
        for k, g in enumerate(gs):
            for j, r in enumerate(rects):
                if j != k:
                    g.import_(r, bufs[j])
            g.pad_recon()
        ws = single.results()
        nsb = ((w + 63) // 64) * ((h + 63) // 64)
        sw = _sb_words(ws, nsb, 2)
        for g, (x0, y0, gw_, gh_) in zip(gs, rects):
            wg = g.results()
            gsb = _sb_words(wg, gw_ * gh_, 2)
            for sb in range(gw_ * gh_):
                fsb = (y0 + sb // gw_) * sbc + x0 + sb % gw_
                np.testing.assert_array_equal(gsb[sb], sw[fsb])
            assert wg[-1] == ws[-1]  # every rank holds the whole reconstruction


def test_cpu_replay_deblock_changes_the_reference():
    """RV_REPLAY_DEBLOCK: the coded frame is deblocked before it becomes a
    reference (the fast levels are non-zero at quantizer 100), so its
    reconstruction -- and every later frame's words -- differ from the
    undeblocked run; the searches of the first inter frame do not."""
    w, h = 256, 128
    fr = _frames(w, h, 1, 1, 8, 8)
    outs, recs = [], []
    for db in (False, True):
        r = O.CpuReplay(w, h, 1, 1, 8, 2, n_inputs=8, threads=2, deblock=db)
        for i, f in enumerate(fr):
            r.set_input(i, f)
        r.frame()
        r.frame()
        outs.append(_sb_words(r.results(), 8, 2))
        recs.append(r.get_recon(4))
    np.testing.assert_array_equal(outs[0][:, :2 * PER_REF], outs[1][:, :2 * PER_REF])
    assert (recs[0] != recs[1]).any()


def test_cpu_replay_loop_restoration():
    """RV_REPLAY_LRF: every unit of the coded frame (one 64x64 superblock in
    luma, 32x32 in 4:2:0 chroma at the levels' quantizers) gets rav1e's
    rdo_loop_decision choice -- None or a self-guided set whose xqd lie in
    SGRPROJ_XQD_MIN .. MAX -- and lrf_filter_frame changes the reference
    after CDEF; the first frame's searches do not change."""
    w, h = 256, 192
    fr = _frames(w, h, 1, 1, 8, 8)
    outs, recs, units = [], [], []
    for lrf in (False, True):
        r = O.CpuReplay(w, h, 1, 1, 8, 2, n_inputs=8, threads=2, deblock=True, cdef=True, lrf=lrf,
                        tile_size=(2, 2))
        for i, f in enumerate(fr):
            r.set_input(i, f)
        r.frame()
        r.frame()
        outs.append(_sb_words(r.results(), 8, 2))
        recs.append(r.get_recon(4))
        if lrf:
            units = [r.lrf_units(p, n) for p, n in ((0, 4 * 3), (1, 4 * 3), (2, 4 * 3))]
    np.testing.assert_array_equal(outs[0][:, :2 * PER_REF], outs[1][:, :2 * PER_REF])
    y = units[0]
    assert (y[:, 0] >= -1).all() and (y[:, 0] < 16).all()
    on = y[y[:, 0] >= 0]
    assert len(on) > 0, "no unit chose a filter"
    assert (on[:, 1] >= -96).all() and (on[:, 1] <= 31).all()
    assert (on[:, 2] >= -32).all() and (on[:, 2] <= 95).all()
    assert (recs[0] != recs[1]).any()


def test_cpu_replay_speed10_edge_superblocks_must_split():
    """Speed 10 (minimum block 64x64): a superblock past the bottom edge is
    split as encode_partition_topdown's must_split does (src/encoder.rs:
    2407-2445) down to the largest blocks inside the frame; 232 = 3 x 64 +
    40: the upper 32x32s stay whole, the lower ones split to 16x16, those to
    8x8 (the rows 32..39 inside).  The other superblocks are single 64x64
    blocks; the level words cover only the bottom superblock row."""
    w, h = 256, 232
    fr = _frames(w, h, 1, 1, 8, 8)
    r = O.CpuReplay(w, h, 1, 1, 8, 2, n_inputs=8, threads=2)
    for i, f in enumerate(fr):
        r.set_input(i, f)
    r.frame()
    r.frame()
    wd = r.results()
    assert RP.level_rect(w, h) == (0, 3, 4, 1)
    sbw, lv, part, tail = RP.level_words(w, h, 2, wd, speed=10)
    want = 1 | (2 << 2) | (2 << 3) | sum(1 << (5 + 2 * 4 + i) for i in range(4))
    np.testing.assert_array_equal(part, [0] * 12 + [want] * 4)
    R = 2
    # the leaves' rd costs: the upper 32x32s, the 8x8s of rows 32..39
    l1 = lv[0].reshape(2, 8, 4 * R + 4)
    assert (l1[0, :, 4 * R + 2] != 0).all()
    l3 = lv[2].reshape(8, 32, 4 * R + 4)
    assert (l3[4, :, 4 * R + 2] != 0).all()
    r.close()


def test_cpu_replay_speed6_searches_the_deblocking_levels():
    """Below speed 8 deblock_filter_optimize searches the levels
    (sse_optimize, src/deblock.rs:1418-1475): per direction and plane, from
    the frame's source, instead of one fast level from the quantizer."""
    w, h = 256, 200
    fr = _frames(w, h, 1, 1, 8, 8)
    got = {}
    for sp in (6, 10):
        r = O.CpuReplay(w, h, 1, 1, 8, 2, n_inputs=8, threads=2, deblock=True, speed=sp)
        for i, f in enumerate(fr):
            r.set_input(i, f)
        got[sp] = []
        for _ in range(3):
            r.frame()
            got[sp].append(r.deblock_levels())
        r.close()
    assert all(len(set(lv)) == 1 for lv in got[10])           # the fast level everywhere
    assert any(len(set(lv)) > 1 for lv in got[6]) and got[6] != got[10]
    assert all(0 <= v <= 63 for lv in got[6] for v in lv)


def test_cpu_replay_cdef_changes_the_reference():
    """RV_REPLAY_CDEF: after deblocking, the coded frame is CDEF-filtered
    (set_quantizers' inter strengths are non-zero at quantizer 100) before
    it becomes a reference."""
    from rav1e_amd import rate as RT
    lv = RT.level_params(100, 8)
    assert all(d["cdef_y"] > 0 and d["cdef_uv"] >= 0 for d in lv)
    w, h = 256, 128
    fr = _frames(w, h, 1, 1, 8, 8)
    recs = []
    for cd in (False, True):
        r = O.CpuReplay(w, h, 1, 1, 8, 2, n_inputs=8, threads=2, deblock=True, cdef=cd)
        for i, f in enumerate(fr):
            r.set_input(i, f)
        r.frame()
        r.frame()
        recs.append(r.get_recon(4))
    assert (recs[0] != recs[1]).any()


def test_cdef_strengths_of_set_quantizers():
    """set_quantizers' inter CDEF polynomials (src/encoder.rs:882-912) at
    a few quantizers: in range, monotone in q for luma's primary."""
    from rav1e_amd import rate as RT
    prev = -1
    for qz in (20, 60, 100, 160, 255):
        for bd in (8, 10, 12):
            d = RT.level_params(qz, bd)[0]
            assert 0 <= d["cdef_y"] <= 63 and 0 <= d["cdef_uv"] <= 63
        y = RT.level_params(qz, 8)[0]["cdef_y"] >> 2
        assert y >= prev
        prev = y


def test_cpu_speed6_partition_and_levels():
    """Speed 6 (config D): thread-invariant words; the 64x64 words keep the
    speed-10 layout; every superblock's partition mask is a valid tree
    (a 32x32 split only under a 64x64 split, a 16x16 split only under its
    32x32's); the bottom superblock row of a 200-row frame (8 visible rows)
    must split down to its 8x8 blocks."""
    w, h = 256, 200
    fr = _frames(w, h, 1, 1, 8, 10)
    outs = []
    for threads in (1, 3):
        r = O.CpuReplay(w, h, 1, 1, 8, 2, n_inputs=10, threads=threads, speed=6, quantizer=60)
        for i, f in enumerate(fr):
            r.set_input(i, f)
        for _ in range(5):
            r.frame()
        outs.append(r.results())
    np.testing.assert_array_equal(outs[0], outs[1])
    wd = outs[0]
    assert wd.size == RP.result_words(w, h, 2, speed=6)
    sbw, lv, part, tail = RP.level_words(w, h, 2, wd)
    assert [x.shape[0] for x in lv] == [64, 256, 1024]
    for m in part.astype(np.int64):
        if not m & 1:
            assert m == 0
        for q in range(4):
            if not m & (2 << q):
                for t in range(4):  # the 16x16 blocks of quadrant q
                    assert not m & (1 << (5 + ((q >> 1) * 2 + (t >> 1)) * 4 + (q & 1) * 2 + (t & 1)))
    # y = 192: the 64x64, its 32x32 and its 16x16 blocks are past the edge
    for m in part[-4:].astype(np.int64):
        assert m & 1 and m & 2 and m & 4 and m & (1 << 5) and m & (1 << 6)
    assert (lv[2][:, 9] <= 1).all() and (lv[2][:, 8] < 14).all()
    assert tail[0] != 0  # some committed block codes coefficients at quantizer 60


def test_cpu_replay_intra_screening():
    """New smooth content the references do not hold: non-skip superblocks
    get the intra screening, some choose an intra mode (result word 1000 +
    16 luma + chroma), their reconstruction follows the new content; with
    RV_REPLAY_NO_INTRA the same frames stay inter."""
    w, h = 320, 256
    fr = intra_frames(w, h, 1, 1, 8, 10)
    res = {}
    for intra in (True, False):
        r = O.CpuReplay(w, h, 1, 1, 8, 2, n_inputs=10, threads=4, intra=intra)
        for i, f in enumerate(fr):
            r.set_input(i, f)
        r.frame()
        wins, words, recs = 0, [], []
        for _ in range(5):
            fi = r.frame()
            wins += r.intra_stats()[1]
            words.append(_sb_words(r.results(), 20, 2)[:, 2 * PER_REF].copy())
            recs.append((fi["display"], r.get_recon(fi["display"])))
        res[intra] = (wins, words, recs)
        r.close()
    wins, words, recs = res[True]
    assert wins > 0 and any((wd >= 1000).any() for wd in words)
    assert res[False][0] == 0 and all((wd < 1000).all() for wd in res[False][1])
    for wd in words:
        for v in wd[wd >= 1000]:
            assert (v - 1000) // 16 < 13 and (v - 1000) % 16 < 13
    # intra improves the new content's reconstruction
    e = [np.abs(a[1].astype(int) - fr[a[0]].astype(int)).sum() for a in recs]
    e0 = [np.abs(a[1].astype(int) - fr[a[0]].astype(int)).sum() for a in res[False][2]]
    assert sum(e) < sum(e0)


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,bd,tiling,seed", [(320, 256, 8, None, 7),
                                                (384, 256, 10, {"tile_cols": 2}, 7),
                                                (256, 192, 12, None, 14)])
def test_gpu_replay_intra_matches_cpu(w, h, bd, tiling, seed):
    """The intra pass (screening, intra RDO, the round-by-round fixed point)
    on content where intra wins: words and reconstructions equal the CPU
    replay's tile raster order."""
    _gpu_vs_cpu(w, h, 1, 1, bd, 2, 9, tiling, inputs=intra_frames(w, h, 1, 1, bd, 17, seed=seed),
                want_intra=True)


@pytest.mark.gpu
def test_gpu_replay_intra_reruns_1080p():
    """1080p with content that makes intra win: intra winners change their
    neighbours' MV stacks, so frames need MV <-> intra outer passes (runs
    beyond one per frame, rv_replay_counters [17]); every one stays within its
    round budget (tws + 2 ths - 2) and the words equal the CPU
    replay's raster-order coding."""
    w, h, frames = 1920, 1080, 6
    cnt = _gpu_vs_cpu(w, h, 1, 1, 8, 2, frames, {"tile_cols": 2},
                      inputs=intra_frames(w, h, 1, 1, 8, frames + 8, seed=11), want_intra=True,
                      quantizer=60)
    runs, nonkey = int(cnt[17]), frames - 1
    assert runs > nonkey, (runs, nonkey)  # some frame re-ran its MV rounds after the intra pass


@pytest.mark.gpu
def test_gpu_synth_equals_numpy_twin():
    import rav1e_amd as R
    R.require_device(0)
    for (w, h, xd, yd, bd) in [(200, 120, 1, 1, 8), (136, 72, 0, 0, 10), (64, 48, 1, 1, 12)]:
        g = RP.HipReplay(w, h, xd, yd, bd, 1, n_inputs=3)
        g.synth_inputs(5)
        for i in range(3):
            np.testing.assert_array_equal(g.get_input(i), RP.synth_frame(w, h, 5 + i, xd, yd, bd))
        g.close()


def intra_frames(w, h, xdec, ydec, bd, n, seed=7):
    """The synthetic clip with new smooth content appearing on odd frames
    (ramps, a flat patch, a diagonal edge) that the references do not hold:
    inter prediction fails there and intra candidates win."""
    rng = np.random.default_rng(seed)
    out = []
    mx = (1 << bd) - 1
    for t in range(n):
        f = RP.synth_frame(w, h, t, xdec, ydec, bd).copy()
        if t % 2 == 1:
            Y = f[: w * h].reshape(h, w)
            for k in range(max(1, (w * h) // (160 * 160))):
                bw, bh = int(rng.integers(64, 200)), int(rng.integers(64, 160))
                x0, y0 = int(rng.integers(0, max(1, w - bw))), int(rng.integers(0, max(1, h - bh)))
                yy, xx = np.mgrid[0:min(bh, h - y0), 0:min(bw, w - x0)]
                kind = (t + k) % 3
                if kind == 0:
                    v = 30 + xx * rng.uniform(0.3, 1.2) + yy * rng.uniform(0, 0.5)
                elif kind == 1:
                    v = np.full(xx.shape, rng.uniform(20, 230))
                else:
                    v = np.where(xx > yy, 60.0, 190.0) + (xx + yy) * 0.1
                Y[y0:y0 + yy.shape[0], x0:x0 + xx.shape[1]] = np.clip(v * (1 << (bd - 8)), 0, mx)
        out.append(f)
    return out


_LRF = RP.RV_REPLAY_DEBLOCK | RP.RV_REPLAY_CDEF | RP.RV_REPLAY_LRF


def _gpu_vs_cpu(w, h, xdec, ydec, bd, refs, frames, tiling=None, flags=0, imp=None, quantizer=100,
                inputs=None, want_intra=False, imp_window=0, ready=False):
    import rav1e_amd as R
    R.require_device(0)
    t = RP.tiling_for(w, h, **(tiling or {}))
    ts = (t["tile_width_sb"], t["tile_height_sb"])
    nin = frames + 8
    g = RP.HipReplay(w, h, xdec, ydec, bd, refs, tile_size=ts, n_inputs=nin, flags=flags,
                     quantizer=quantizer, imp_window=imp_window, imp_limit=frames)
    g.synth_inputs(0)
    if inputs is not None:
        for i in range(nin):
            g.set_input(i, inputs[i])
    if ready:  # the engine may run ahead of the window (results unchanged)
        g.set_inputs_ready(nin)
    c = O.CpuReplay(w, h, xdec, ydec, bd, refs, tile_size=ts, n_inputs=nin,
                    threads=O.cpu_share(), quantizer=quantizer,
                    speed=6 if flags & RP.RV_REPLAY_SPEED6 else 10,
                    deblock=bool(flags & RP.RV_REPLAY_DEBLOCK),
                    cdef=bool(flags & RP.RV_REPLAY_CDEF),
                    intra=not flags & RP.RV_REPLAY_NO_INTRA,
                    mvref_standin=bool(flags & RP.RV_REPLAY_MVREF_STANDIN),
                    imp_window=imp_window, imp_limit=frames, lrf=bool(flags & RP.RV_REPLAY_LRF))
    for i in range(nin):
        c.set_input(i, g.get_input(i))
    nsb = ((w + 63) // 64) * ((h + 63) // 64)
    if imp is not None:
        g.set_importances(imp)
        c.set_importances(imp)
    won = nz = 0
    for n in range(frames):
        gi, ci = g.frame(), c.frame()
        assert gi == ci
        gw, cw = g.results(), c.results()
        bad = np.nonzero(gw != cw)[0]
        assert bad.size == 0, (n, gi, bad[:10], gw[bad[:10]], cw[bad[:10]])
        if flags & RP.RV_REPLAY_LRF and not gi["is_key"]:
            for p in range(3):  # every unit's choice (set, xqd)
                gu, cu = g.lrf_units(p), c.lrf_units(p, nsb)
                bad = np.nonzero((gu != cu).any(axis=1))[0]
                assert bad.size == 0, ("frame %d plane %d units" % (n, p),
                                       [(int(i), gu[i].tolist(), cu[i].tolist()) for i in bad[:12]])
        if imp_window:
            gimp, cimp = g.importances(), c.importances()
            np.testing.assert_array_equal(gimp.view(np.uint32), cimp.view(np.uint32),
                                          err_msg="importances of frame %d" % n)
            nz += bool((cimp > 0).any())
        won += c.intra_stats()[1] if c.intra else 0
    np.testing.assert_array_equal(g.get_recon(gi["display"]), c.get_recon(ci["display"]))
    if want_intra:
        cnt = g.counters()
        assert won > 0 and cnt[12] == won, (won, cnt[11:14])
    if imp_window:
        assert nz >= 2, nz  # the referenced frames carry importances
    cnt = g.counters()
    g.close()
    c.close()
    return cnt


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,xdec,ydec,bd,refs,tiling,flags", [
    (256, 192, 1, 1, 8, 2, None, 0),
    (320, 128, 0, 0, 8, 1, None, 0),
    (256, 128, 1, 1, 10, 2, None, 0),
    (192, 128, 1, 1, 12, 1, None, 0),  # 12 bits: exhaustive full search, 12-bit RDO kernel
    (384, 192, 1, 1, 8, 2, {"tile_cols": 2}, 0),
    (384, 256, 0, 0, 8, 2, {"tiles": 4}, 0),
    (256, 192, 1, 1, 8, 2, None, RP.RV_REPLAY_EXHAUSTIVE_FS),
    (320, 200, 1, 1, 8, 2, {"tile_cols": 2}, RP.RV_REPLAY_MVREF_STANDIN),  # the A/B stand-in stacks
    # speed 10 must_split at the frame edges (bottom; right + bottom; 4:4:4)
    (256, 232, 1, 1, 8, 2, None, 0),
    (200, 136, 1, 1, 10, 2, None, 0),
    (320, 168, 0, 0, 8, 2, {"tile_cols": 2}, 0),
    (256, 200, 1, 1, 8, 2, None, RP.RV_REPLAY_SPEED6),      # speed 6: partition RDO
    (256, 136, 1, 1, 10, 2, None, RP.RV_REPLAY_SPEED6),
    (192, 128, 0, 0, 8, 2, {"tile_cols": 2}, RP.RV_REPLAY_SPEED6),
    # deblocking before the reference write-back
    (256, 200, 1, 1, 8, 2, None, RP.RV_REPLAY_DEBLOCK),
    (192, 136, 0, 0, 10, 2, None, RP.RV_REPLAY_DEBLOCK),
    (256, 200, 1, 1, 8, 2, None, RP.RV_REPLAY_DEBLOCK | RP.RV_REPLAY_SPEED6),
    (192, 128, 0, 0, 12, 1, None, RP.RV_REPLAY_DEBLOCK | RP.RV_REPLAY_SPEED6),
    # CDEF after deblocking (cdef_filter_frame, cdef_bits 0)
    (256, 200, 1, 1, 8, 2, None, RP.RV_REPLAY_DEBLOCK | RP.RV_REPLAY_CDEF),
    (192, 136, 0, 0, 10, 2, None, RP.RV_REPLAY_DEBLOCK | RP.RV_REPLAY_CDEF),
    (256, 136, 1, 0, 8, 2, None, RP.RV_REPLAY_DEBLOCK | RP.RV_REPLAY_CDEF),
    (256, 200, 1, 1, 8, 2, None, RP.RV_REPLAY_DEBLOCK | RP.RV_REPLAY_CDEF | RP.RV_REPLAY_SPEED6),
    (192, 128, 0, 0, 12, 1, None, RP.RV_REPLAY_DEBLOCK | RP.RV_REPLAY_CDEF | RP.RV_REPLAY_SPEED6),
    # loop restoration after CDEF: the units' choices and the restored frame
    (256, 200, 1, 1, 8, 2, None, _LRF),
    (192, 136, 0, 0, 10, 2, None, _LRF),
    (384, 192, 1, 1, 8, 2, {"tile_cols": 2}, _LRF),
    (192, 128, 1, 1, 12, 1, None, _LRF),
    (256, 200, 1, 1, 8, 2, None, _LRF | RP.RV_REPLAY_SPEED6),
])
def test_gpu_replay_matches_cpu_replay(w, h, xdec, ydec, bd, refs, tiling, flags):
    _gpu_vs_cpu(w, h, xdec, ydec, bd, refs, 10, tiling, flags)


@pytest.mark.gpu
@pytest.mark.parametrize("fix,passes", [("0", None), ("1", "1"), ("1", "2"), ("1", None)])
def test_gpu_lrf_decision_paths(monkeypatch, fix, passes):
    """rdo_loop_decision's units by each decision kernel: the one-wave
    serial lrf_decide_kernel (RAV1E_LRF_FIX=0) and the fixed point, whole
    (default) or capped after one or two parallel passes so that its serial
    rest decides the tile from the first unsettled superblock on
    (RAV1E_LRF_FIX_PASSES); 70 superblocks in one tile cross the state
    chain's 64-superblock batches. Every unit equals the CPU replay's."""
    monkeypatch.setenv("RAV1E_LRF_FIX", fix)
    if passes is None:
        monkeypatch.delenv("RAV1E_LRF_FIX_PASSES", raising=False)
    else:
        monkeypatch.setenv("RAV1E_LRF_FIX_PASSES", passes)
    _gpu_vs_cpu(640, 448, 1, 1, 8, 2, 4, None, _LRF)


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, RP.RV_REPLAY_SPEED6])
def test_gpu_replay_importance_bias_and_quantizer(flags):
    w, h = 256, 192
    rng = np.random.default_rng(3)
    imp = rng.random((h // 8) * (w // 8)).astype(np.float32) * 7
    _gpu_vs_cpu(w, h, 1, 1, 8, 2, 6, imp=imp, quantizer=60, flags=flags)


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,bd,refs,tiling,flags,window,ready", [
    (256, 192, 8, 2, None, 0, 4, False),
    (256, 192, 8, 2, None, 0, 4, True),
    (320, 136, 10, 2, {"tile_cols": 2}, 0, 6, False),
    (256, 200, 8, 1, None, 0, 3, True),
    (256, 200, 8, 2, None, RP.RV_REPLAY_SPEED6, 4, False),
    (192, 128, 12, 2, None, RP.RV_REPLAY_DEBLOCK | RP.RV_REPLAY_CDEF, 2, False),
])
def test_gpu_replay_importance_window(w, h, bd, refs, tiling, flags, window, ready):
    """compute_block_importances over the lookahead window on the GPU's
    lookahead engine (its own thread, stream and round ring, W frames
    ahead; with every input ready, as far ahead as its ring allows): every
    frame's importances and words equal the CPU replay's."""
    _gpu_vs_cpu(w, h, 1, 1, bd, refs, 11, tiling, flags, quantizer=60, imp_window=window,
                ready=ready)


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, RP.RV_REPLAY_DEBLOCK,
                                   RP.RV_REPLAY_DEBLOCK | RP.RV_REPLAY_SPEED6,
                                   RP.RV_REPLAY_DEBLOCK | RP.RV_REPLAY_CDEF, _LRF])
def test_gpu_tile_groups_exchange(flags):
    """Two GPU tile groups in one process, exchanging reconstructions (with
    deblocking: and block maps; with loop restoration: each group's units)
    through their device exchange buffers (the RCCL all-gather's layout),
    reproduce the CPU replay of the whole frame."""
    import ctypes as C

    import rav1e_amd as R
    R.require_device(0)
    w, h = 384, 192
    t = RP.tiling_for(w, h, tile_cols=2)
    ts = (t["tile_width_sb"], t["tile_height_sb"])
    rects = RP.tile_groups(t, 2)
    gs = [RP.HipReplay(w, h, group=r, tile_size=ts, n_inputs=14, flags=flags) for r in rects]
    for k, g in enumerate(gs):
        g.synth_inputs(0)
        g.set_groups(rects, k, None)
    c = O.CpuReplay(w, h, tile_size=ts, n_inputs=14, threads=4,
                    deblock=bool(flags & RP.RV_REPLAY_DEBLOCK),
                    cdef=bool(flags & RP.RV_REPLAY_CDEF), lrf=bool(flags & RP.RV_REPLAY_LRF),
                    speed=6 if flags & RP.RV_REPLAY_SPEED6 else 10)
    for i in range(14):
        c.set_input(i, RP.synth_frame(w, h, i))
    L = R.lib()
    bufs = [g.exchange_buffers() for g in gs]
    nb = bufs[0][2]
    sbc = (w + 63) // 64
    for n in range(7):
        for g in gs:
            g.frame()
        c.frame()
        R._check(L.rv_device_sync(), "sync")  # the packs ran on the replay streams
        for k in range(2):  # all-gather: group j's send -> slot j of every recv
            for j in range(2):
                R._check(L.rv_memcpy_d2d(C.c_void_p(bufs[k][1] + j * nb), C.c_void_p(bufs[j][0]),
                                         nb, None), "rv_memcpy_d2d")
        R._check(L.rv_device_sync(), "sync")
        for g in gs:
            g.import_()
        cw = c.results()
        sw = _sb_words(cw, ((w + 63) // 64) * ((h + 63) // 64), 2)
        for g, (x0, y0, gw_, gh_) in zip(gs, rects):
            wg = g.results()
            gsb = _sb_words(wg, gw_ * gh_, 2)
            for sb in range(gw_ * gh_):
                np.testing.assert_array_equal(gsb[sb], sw[(y0 + sb // gw_) * sbc + x0 + sb % gw_])
            assert wg[-1] == cw[-1]
            if flags & RP.RV_REPLAY_LRF and n:  # every group holds every unit after the import
                nsb = sbc * ((h + 63) // 64)
                for p in range(3):
                    np.testing.assert_array_equal(g.lrf_units(p), c.lrf_units(p, nsb), err_msg=f"frame {n} plane {p}")
    for g in gs:
        g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, RP.RV_REPLAY_DEBLOCK | RP.RV_REPLAY_CDEF])
def test_gpu_tile_groups_importance_window(flags):
    """Two GPU tile groups with an importance window: each group's engine
    computes its own blocks' lookahead part, the parts meet in an in-process
    hub (the RCCL all-gather's role), every group propagates over the whole
    frame -- words, reconstructions and importances equal the CPU replay of
    the whole frame with the same window."""
    import ctypes as C

    import rav1e_amd as R
    R.require_device(0)
    w, h, nin, W = 384, 192, 20, 3
    t = RP.tiling_for(w, h, tile_cols=2)
    ts = (t["tile_width_sb"], t["tile_height_sb"])
    rects = RP.tile_groups(t, 2)
    hub = RP.LaHub(2)
    gs = [RP.HipReplay(w, h, group=r, tile_size=ts, n_inputs=nin, flags=flags, imp_window=W)
          for r in rects]
    for k, g in enumerate(gs):
        g.synth_inputs(0)
        g.set_groups(rects, k, None)
        g.set_la_exchange(hub=hub)
        g.set_inputs_ready(nin)  # the groups code one after another here
    c = O.CpuReplay(w, h, tile_size=ts, n_inputs=nin, threads=4, imp_window=W,
                    deblock=bool(flags & RP.RV_REPLAY_DEBLOCK), cdef=bool(flags & RP.RV_REPLAY_CDEF))
    for i in range(nin):
        c.set_input(i, RP.synth_frame(w, h, i))
    L = R.lib()
    bufs = [g.exchange_buffers() for g in gs]
    nb = bufs[0][2]
    sbc = (w + 63) // 64
    try:
        for n in range(9):
            for g in gs:
                g.frame()
            c.frame()
            R._check(L.rv_device_sync(), "sync")
            for k in range(2):
                for j in range(2):
                    R._check(L.rv_memcpy_d2d(C.c_void_p(bufs[k][1] + j * nb),
                                             C.c_void_p(bufs[j][0]), nb, None), "rv_memcpy_d2d")
            R._check(L.rv_device_sync(), "sync")
            for g in gs:
                g.import_()
            cw = c.results()
            sw = _sb_words(cw, sbc * ((h + 63) // 64), 2)
            ci = c.importances()
            for g, (x0, y0, gw_, gh_) in zip(gs, rects):
                wg = g.results()
                gsb = _sb_words(wg, gw_ * gh_, 2)
                for sb in range(gw_ * gh_):
                    np.testing.assert_array_equal(gsb[sb],
                                                  sw[(y0 + sb // gw_) * sbc + x0 + sb % gw_],
                                                  err_msg=f"frame {n}")
                assert wg[-1] == cw[-1]
                np.testing.assert_array_equal(g.importances().view(np.uint32),
                                              ci.view(np.uint32), err_msg=f"frame {n}")
        assert (ci > 0).any()
    finally:
        for g in gs:
            g.close()
        hub.close()


@pytest.mark.gpu
def test_gpu_replay_one_rank_rccl_la_exchange():
    """The RCCL branch of the engine's part exchange (pack, ncclAllGather on
    the engine stream) with a 1-rank communicator: the same importances and
    words as the run without one."""
    import os

    import rav1e_amd as R
    R.require_device(0)
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    L = R.lib()
    idb = np.zeros(256, np.uint8)
    assert L.rv_comm_unique_id(idb.ctypes.data, idb.size) > 0, L.rv_last_error()
    comm = L.rv_comm_create(idb.ctypes.data, 1, 0)
    assert comm, L.rv_last_error()
    w, h, nin = 256, 192, 20
    a, b = (RP.HipReplay(w, h, n_inputs=nin, imp_window=4, imp_limit=12) for _ in range(2))
    a.synth_inputs(0)
    b.synth_inputs(0)
    a.set_groups([(0, 0, 4, 3)], 0, None)
    a.set_la_exchange(comm=comm)
    try:
        for n in range(12):
            ia, ib = a.frame(), b.frame()
            assert ia == ib
            np.testing.assert_array_equal(a.results(), b.results())
            np.testing.assert_array_equal(a.importances().view(np.uint32),
                                          b.importances().view(np.uint32))
    finally:
        a.close()
        b.close()
        L.rv_comm_destroy(comm)


@pytest.mark.gpu
@pytest.mark.parametrize("window,k", [(0, 3), (5, 3), (5, 5)])
def test_gpu_pipelined_replay_matches_cpu(window, k):
    """PipelinedReplay: three instances (levels 0 + 4g+1, level 1, 4g+3) on
    their own streams and host threads, ordered by device events only; the
    reconstructions of a free-running stretch equal the sequential CPU
    replay's."""
    import rav1e_amd as R
    R.require_device(0)
    w, h, nin = 256, 200, 24
    g = RP.HipReplay(w, h, n_inputs=nin, imp_window=window, imp_limit=21)
    g.synth_inputs(0)
    if window:
        g.set_inputs_ready(nin)
    c = O.CpuReplay(w, h, n_inputs=nin, threads=O.cpu_share(), imp_window=window, imp_limit=21)
    for i in range(nin):
        c.set_input(i, g.get_input(i))
    eng = RP.PipelinedReplay(g, instances=k)
    try:
        for n in range(21):
            gi, ci = eng.frame(), c.frame()
            assert gi == ci, (n, gi, ci)
        eng.drain()
        R._check(R.lib().rv_device_sync(), "sync")
        for d in range(9, 21):
            np.testing.assert_array_equal(g.get_recon(d), c.get_recon(d), err_msg=f"display {d}")
    finally:
        eng.close()
        g.close()
        c.close()


@pytest.mark.gpu
def test_gpu_pipelined_window_ring_wraps():
    """The lookahead engine's ring (W + 29 entries) wraps: W = 2 over 44
    coded frames, three instances, every input declared in place (the engine
    runs as far ahead as the ring allows, so entries are reused while the
    instances still hold frames), deblocking + CDEF on.  Every frame's words
    and importances equal the CPU replay's."""
    import rav1e_amd as R
    R.require_device(0)
    w, h, nin, W, n = 192, 128, 60, 2, 44
    flags = RP.RV_REPLAY_DEBLOCK | RP.RV_REPLAY_CDEF
    g = RP.HipReplay(w, h, n_inputs=nin, flags=flags, imp_window=W, imp_limit=n)
    g.synth_inputs(0)
    c = O.CpuReplay(w, h, n_inputs=nin, threads=O.cpu_share(), deblock=True, cdef=True,
                    imp_window=W, imp_limit=n)
    for i in range(nin):
        c.set_input(i, g.get_input(i))
    g.set_inputs_ready(nin)
    eng = RP.PipelinedReplay(g)
    imps = {}
    try:
        for k in range(n):
            eng.frame()
            c.frame()
            imps[k] = c.importances()
        eng.drain()
        R._check(R.lib().rv_device_sync(), "sync")
        # the DPB after 44 coded frames (displays 0 .. 42 and 44): its 12
        # slots hold displays 33 .. 42, 44 and 31
        for d in list(range(33, 43)) + [44, 31]:
            np.testing.assert_array_equal(g.get_recon(d), c.get_recon(d), err_msg=f"display {d}")
        # the importances of the last frame each coded (the CPU's last is the
        # stream's last frame; the GPU primary's last is frame 43, display 41)
        assert (c.importances() >= 0).all()
    finally:
        eng.close()
        g.close()
        c.close()
    assert any((v > 0).any() for v in imps.values())


@pytest.mark.gpu
@pytest.mark.parametrize("flags,window,ready,twin", [
    (0, 0, False, "l2"), (RP.RV_REPLAY_DEBLOCK | RP.RV_REPLAY_CDEF, 0, False, "l2"),
    (RP.RV_REPLAY_SPEED6, 0, False, "l2"), (0, 5, False, "l2"), (0, 5, True, "l2"),
    (0, 5, True, "l2b"), (RP.RV_REPLAY_DEBLOCK, 0, False, "l2b"), (0, 5, True, "alt")])
def test_gpu_paired_replay_matches_cpu(flags, window, ready, twin):
    """PairedReplay: the level-2 frames on a twin instance (shared DPB, own
    stream and host thread) give every frame's words and reconstruction of
    the sequential CPU replay -- checked frame by frame, then over a run
    with no host synchronisation between frames."""
    import rav1e_amd as R
    R.require_device(0)
    w, h, nin = 256, 200, 24
    speed = 6 if flags & RP.RV_REPLAY_SPEED6 else 10
    g = RP.HipReplay(w, h, n_inputs=nin, flags=flags, imp_window=window, imp_limit=21)
    g.synth_inputs(0)
    if ready:
        g.set_inputs_ready(nin)
    c = O.CpuReplay(w, h, n_inputs=nin, threads=O.cpu_share(), speed=speed,
                    deblock=bool(flags & RP.RV_REPLAY_DEBLOCK), cdef=bool(flags & RP.RV_REPLAY_CDEF),
                    imp_window=window, imp_limit=21)
    for i in range(nin):
        c.set_input(i, g.get_input(i))
    eng = RP.PairedReplay(g, twin_levels=twin)
    try:
        for n in range(11):  # frame by frame
            gi, ci = eng.frame(), c.frame()
            assert gi == ci, (n, gi, ci)
            eng.drain()
            inst = eng.p if not n or eng.on_primary(n - 1) else eng.t
            np.testing.assert_array_equal(inst.results(), c.results())
        for n in range(11, 21):  # free-running: the streams overlap
            eng.frame()
            c.frame()
        eng.drain()
        R._check(R.lib().rv_device_sync(), "sync")
        for d in range(9, 21):  # displays coded in the second part
            np.testing.assert_array_equal(g.get_recon(d), c.get_recon(d))
    finally:
        eng.close()
        g.close()
        c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, RP.RV_REPLAY_DEBLOCK | RP.RV_REPLAY_CDEF | RP.RV_REPLAY_SPEED6, _LRF])
def test_gpu_replay_one_rank_rccl_exchange(flags):
    """The RCCL branch of the tile-group exchange (rv_replay.hip: pack,
    ncclAllGather on the replay stream, import, loop filters, pad) with a
    1-rank communicator (rv_comm_unique_id / rv_comm_create): the words and
    every reconstruction equal the run without a communicator."""
    import os

    import rav1e_amd as R
    R.require_device(0)
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")  # bootstrap over loopback (no network)
    L = R.lib()
    idb = np.zeros(256, np.uint8)
    assert L.rv_comm_unique_id(idb.ctypes.data, idb.size) > 0, L.rv_last_error()
    comm = L.rv_comm_create(idb.ctypes.data, 1, 0)
    assert comm, L.rv_last_error()
    w, h = 384, 192
    t = RP.tiling_for(w, h, tile_cols=2)
    ts = (t["tile_width_sb"], t["tile_height_sb"])
    rects = RP.tile_groups(t, 1)
    a, b = (RP.HipReplay(w, h, group=rects[0], tile_size=ts, n_inputs=14, flags=flags)
            for _ in range(2))
    a.synth_inputs(0)
    b.synth_inputs(0)
    a.set_groups(rects, 0, comm)
    try:
        for n in range(7):
            ia, ib = a.frame(), b.frame()
            assert ia == ib
            np.testing.assert_array_equal(a.results(), b.results())
            np.testing.assert_array_equal(a.get_recon(ia["display"]), b.get_recon(ib["display"]))
            if flags & RP.RV_REPLAY_LRF and n:  # the units came through the all-gather
                for p in range(3):
                    np.testing.assert_array_equal(a.lrf_units(p), b.lrf_units(p))
    finally:
        a.close()
        b.close()
        L.rv_comm_destroy(comm)


@pytest.mark.gpu
@pytest.mark.parametrize("config,speed,filters", [("360p", 10, 0), ("1080p", 10, 0), ("2160p", 10, 0),
                                                  ("2160p10", 10, 0),
                                                  ("2160p10", 6, 0), ("2160p444", 10, 0),
                                                  ("1080p", 10, _LRF), ("2160p444", 10, _LRF)])
def test_gpu_replay_full_size_gop(config, speed, filters):
    """The key frame and one GOP (me_range_scale 4, 2, 1, 1) at the BASELINE
    shapes and tilings (config D also at its speed-6 schedule; two shapes
    with every loop filter, loop restoration's units compared per frame),
    GPU words equal to the CPU replay's frame by frame."""
    import bench
    w, h, xdec, ydec, bd, tk = bench.CONFIGS[config][:6]
    _gpu_vs_cpu(w, h, xdec, ydec, bd, 2, 5, tk, flags=(RP.RV_REPLAY_SPEED6 if speed == 6 else 0) | filters)
