"""Debug: first GPU-vs-CPU word mismatch of the entropy replay case."""
import sys
sys.path.insert(0, ".")
import numpy as np
import rav1e_amd as R
from rav1e_amd import replay as RP
from tests import oracle_lib as O
W, H, xdec, tiles, speed, q = 640, 360, 1, (0, 0), 10, 100
for flags in (RP.RV_REPLAY_ENTROPY, 0):
    g = RP.HipReplay(W, H, xdec, xdec, 8, 2, tile_size=tiles, n_inputs=12, flags=flags, quantizer=q)
    g.synth_inputs(0)
    c = O.CpuReplay(W, H, xdec, xdec, 8, 2, tile_size=tiles, n_inputs=12, threads=8, speed=speed,
                    entropy=bool(flags), quantizer=q)
    for i in range(12):
        c.set_input(i, g.get_input(i))
    g.frame(); c.frame()
    for f in range(4):
        gi = g.frame(); c.frame()
        a, b = g.results(), c.results()
        bad = np.nonzero(a != b)[0]
        print("flags", flags, "frame", f, gi, "n words", len(a), "bad", bad[:8], a[bad[:8]], b[bad[:8]])
    print("counters", g.counters())
    g.close(); c.close()
