"""N > 1 bench path on the CPU: world_size-2 gloo ranks code the tile groups
of ONE stream through bench.timed_run and rav1e_amd.ranks.TileParallel
(the loop bench.py times on the GPU), with the oracle's CpuReplay standing
in for the device engine and gloo for the RCCL all-gather.  Checks: every
rank's superblock words equal a single-process run of the whole frame with
the same tiling, every rank ends with the same (whole) reconstruction, and
the reported time is the max over ranks."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from rav1e_amd import replay as RP

W, H, REFS, NIN = 384, 192, 2, 16


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tiling():
    from rav1e_amd import replay as RP
    t = RP.tiling_for(W, H, tile_cols=2)
    return t, (t["tile_width_sb"], t["tile_height_sb"])


def _single_words(frames, deblock=False, window=0):
    from rav1e_amd import replay as RP
    from tests import oracle_lib as O
    _, ts = _tiling()
    c = O.CpuReplay(W, H, 1, 1, 8, REFS, tile_size=ts, n_inputs=NIN, threads=2,
                    deblock=deblock, imp_window=window)
    for i in range(NIN):
        c.set_input(i, RP.synth_frame(W, H, i))
    for _ in range(frames):
        c.frame()
    w, imp = c.results(), c.importances()
    c.close()
    return w, imp


def _rank_main(rank, world, port, q, deblock, window):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import bench
    from rav1e_amd import replay as RP
    from rav1e_amd.ranks import RankGroup, TileParallel, rank_info
    from tests import oracle_lib as O
    info = rank_info()
    g = RankGroup(info)
    t, ts = _tiling()
    rects = RP.tile_groups(t, world)
    c = O.CpuReplay(W, H, 1, 1, 8, REFS, group=rects[rank], tile_size=ts, n_inputs=NIN,
                    threads=2, deblock=deblock, imp_window=window)
    for i in range(NIN):
        c.set_input(i, RP.synth_frame(W, H, i))
    if rank == 1:  # make rank 1 the slow one: the reported time must be its
        import time
        orig = c.frame

        def slow(sb_limit=0, pad=True):
            time.sleep(0.05)
            return orig(sb_limit, pad)
        c.frame = slow
    eng = TileParallel(c, rects, rank, g)
    dt, words = bench.timed_run(eng, g, steps=4, warmup=2)
    q.put((rank, dt, words.tolist(), rects[rank], c.importances().tolist()))
    c.close()
    g.close()


@pytest.mark.parametrize("deblock,window", [(False, 0), (True, 0), (True, 3)])
def test_two_rank_gloo_tile_parallel_stream(deblock, window):
    """With deblock the exchange also carries the block maps and each rank
    deblocks the whole frame.  With an importance window each rank computes
    its group's lookahead part and the parts are all-gathered before every
    frame: the ranks code the one-process stream, importances included."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q, deblock, window))
             for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        rank, dt, words, rect, imp = q.get(timeout=240)
        res[rank] = (dt, np.array(words, dtype=np.uint64), rect, np.array(imp, np.float32))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # max over ranks: both report the slow rank's time (>= 4 sleeps)
    assert abs(res[0][0] - res[1][0]) < 1e-9 and res[0][0] >= 0.2
    single, simp = _single_words(6, deblock, window)
    per = RP.sb_words_per(REFS)
    sbc = (W + 63) // 64
    sw = single[: len(single) - 5].reshape(-1, per)
    for r in range(2):
        words, (x0, y0, gw, gh) = res[r][1], res[r][2]
        gsb = words[: gw * gh * per].reshape(-1, per)
        for sb in range(gw * gh):
            np.testing.assert_array_equal(gsb[sb], sw[(y0 + sb // gw) * sbc + x0 + sb % gw])
        assert words[-1] == single[-1]  # the whole reconstruction on every rank
        np.testing.assert_array_equal(res[r][3].view(np.uint32), simp.view(np.uint32))
    if window:
        assert (simp > 0).any()
    assert res[0][2] != res[1][2]
