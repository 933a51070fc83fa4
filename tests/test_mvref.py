"""rav1e's MV reference stack (find_mvrefs / setup_mvref_list,
src/context.rs:2308-2965) in the oracle (oracle/orc_mvref.c) against
vectors made by evaluating the reference's own text
(tools/refeval/gen_mvref_ref.py -> tests/golden/ref_mvref.npz): random tile
grids of coded blocks (intra, single-reference, compound; 64x64 .. 8x8
leaves; ragged tile edges) and queries of every square size for the single
and the compound stacks -- weights, order, extra search, clamp and mode
context."""
import os

import numpy as np

from tests import oracle_lib as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_oracle_find_mvrefs_vs_reference():
    g = np.load(os.path.join(GOLD, "ref_mvref.npz"))
    grids, cells, query, entries = g["grids"], g["cells"], g["query"], g["entries"]
    off, grid_of = 0, {}
    for (case, tx, ty, cols, rows, fcols, frows, W, Hh, sb0, sb1) in grids:
        c = cells[off:off + W * Hh]
        off += W * Hh
        b = np.zeros(W * Hh, O.BLK)
        b["ref"] = c[:, 0:2]
        b["mv"][:, 0] = c[:, 2:4]
        b["mv"][:, 1] = c[:, 4:6]
        b["n4_w"], b["n4_h"], b["newmv"] = c[:, 6], c[:, 7], c[:, 8]
        grid_of[case] = (b.reshape(Hh, W), tx, ty, cols, rows, fcols, frows, (sb0, sb1))
    assert off == len(cells)
    kinds = set()
    for q, ent in zip(query, entries):
        case, bx, by, bw4, bh4, r0, r1, ctx, n = (int(v) for v in q)
        grid, tx, ty, cols, rows, fcols, frows, sbias = grid_of[case]
        got_ctx, st = O.find_mvrefs(grid, cols, rows, tx, ty, fcols, frows, bx, by, bw4, bh4,
                                    (r0, r1), sbias)
        assert (got_ctx, len(st)) == (ctx, n), (case, bx, by, bw4, r0, r1)
        want = ent[:n]
        np.testing.assert_array_equal(st["this_mv"], want[:, 0:2])
        np.testing.assert_array_equal(st["comp_mv"], want[:, 2:4])
        np.testing.assert_array_equal(st["weight"], want[:, 4])
        kinds.add((bw4, r1 != 8, min(n, 3)))
    # the vectors cover every size, single and compound, short and long stacks
    assert {(16, False, 2), (16, True, 2), (2, False, 1)} <= kinds
