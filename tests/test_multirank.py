"""N > 1 bench path on the CPU: world_size-2 gloo ranks, each running its own
tile stream through bench.timed_run (the same loop bench.py times on the
GPU), with the oracle's CpuReplay standing in for the device engine.
Checks: no data-path collective is needed (each rank's words equal a
single-process run of that rank's stream), ranks encode different content,
and the reported time is the max over ranks."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

W, H, REFS = 192, 128, 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _stream_words(offset, steps=3, warmup=1):
    from rav1e_amd import replay as RP
    from tests import oracle_lib as O
    c = O.CpuReplay(W, H, 1, 1, 8, REFS, threads=2)
    for s in range(REFS + 1):
        c.set_frame(s, RP.synth_frame(W, H, offset + s))
    for i in range(warmup + steps):
        c.frame(RP.GOP_SCALES[i % 4])
    w = c.results()
    c.close()
    return w


def _rank_main(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import bench
    from rav1e_amd import replay as RP
    from rav1e_amd.ranks import RankGroup, rank_info
    from tests import oracle_lib as O
    info = rank_info()
    g = RankGroup(info)
    c = O.CpuReplay(W, H, 1, 1, 8, REFS, threads=2)
    for s in range(REFS + 1):
        c.set_frame(s, RP.synth_frame(W, H, info.frame_offset + s))
    if rank == 1:  # make rank 1 the slow one: the reported time must be its
        import time
        orig = c.frame

        def slow(scale, sb_limit=0):
            time.sleep(0.05)
            orig(scale, sb_limit)
        c.frame = slow
    dt, words = bench.timed_run(c, g, steps=3, warmup=1)
    sums = g.gather_u64(int(np.bitwise_xor.reduce(words)))
    q.put((rank, dt, words.tolist(), sums))
    c.close()
    g.close()


def test_two_rank_gloo_tile_streams():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        rank, dt, words, sums = q.get(timeout=240)
        res[rank] = (dt, np.array(words, dtype=np.uint64), sums)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # max over ranks: both report the slow rank's time (>= 3 sleeps)
    assert abs(res[0][0] - res[1][0]) < 1e-9 and res[0][0] >= 0.15
    # each rank's result = a single-process run of its own stream
    for r in range(2):
        np.testing.assert_array_equal(res[r][1], _stream_words(1000 * r))
    # different content per rank, and the gather agrees on every rank
    assert not np.array_equal(res[0][1], res[1][1])
    assert res[0][2] == res[1][2]
