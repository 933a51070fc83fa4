"""Reference-evaluated vectors for the MV reference stack
(tests/golden/ref_mvref.npz).

    python tools/refeval/gen_mvref_ref.py        (in the build container)

Runs the reference's own text through tools/refeval/rsinterp.py:

  src/context.rs    ContextWriter::find_mvrefs, setup_mvref_list,
                    scan_row_mbmi, scan_col_mbmi, scan_blk_mbmi,
                    add_ref_mv_candidate, add_extra_mv_candidate,
                    find_matching_mv, find_matching_mv_and_update_weight,
                    find_matching_comp_mv_and_update_weight, add_offset,
                    find_valid_row_offs, find_valid_col_offs (:2308-2965),
                    Block::is_inter (:1417)
  src/partition.rs  has_tr (:695-750)

The environment supplies: the tile's block grid (TileBlocks indexed by a
TileBlockOffset, cols / rows / x / y / frame_cols / frame_rows), Block
records (mode, ref_frames, mv, n4_w, n4_h), TileBlockOffset::with_offset,
BlockSize values, RefType values with to_index(), PredictionMode values in
the enum's order (src/predict.rs:135-165), FrameInvariants'
ref_frame_sign_bias, and the crate constants MVREF_ROW_COLS (3),
REF_CAT_LEVEL (640), MAX_REF_MV_STACK_SIZE (8), REFMV_OFFSET (4),
LOCAL_BLOCK_MASK (15).

Vectors (one case = a random tile grid of coded blocks + queries):
  grid:  per case, every 4x4 unit's block: ref0, ref1, mv0 (row, col),
         mv1, n4_w, n4_h, newmv (mode counts as a NEWMV one)
  query: case, bx, by, bw4, bh4, ref0, ref1 -> mode_context, len,
         and up to 9 (this_mv, comp_mv, weight) entries
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(__file__))
import gen_golden_ref as G  # noqa: E402
import rshost as H  # noqa: E402
import rsinterp as RI  # noqa: E402

REF = G.REF
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
OUT = os.path.join(ROOT, "tests", "golden", "ref_mvref.npz")

MODES = ["DC_PRED", "V_PRED", "H_PRED", "D45_PRED", "D135_PRED", "D117_PRED", "D153_PRED",
         "D207_PRED", "D63_PRED", "SMOOTH_PRED", "SMOOTH_V_PRED", "SMOOTH_H_PRED", "PAETH_PRED",
         "UV_CFL_PRED", "NEARESTMV", "NEAR0MV", "NEAR1MV", "NEAR2MV", "GLOBALMV", "NEWMV",
         "NEAREST_NEARESTMV", "NEAR_NEARMV", "NEAREST_NEWMV", "NEW_NEARESTMV", "NEAR_NEWMV",
         "NEW_NEARMV", "GLOBAL_GLOBALMV", "NEW_NEWMV"]
PM = {n: i for i, n in enumerate(MODES)}
NEWMV_MODES = {PM[n] for n in ("NEWMV", "NEW_NEWMV", "NEAREST_NEWMV", "NEW_NEARESTMV",
                               "NEAR_NEWMV", "NEW_NEARMV")}
REF_NAMES = ["INTRA_FRAME", "LAST_FRAME", "LAST2_FRAME", "LAST3_FRAME", "GOLDEN_FRAME",
             "BWDREF_FRAME", "ALTREF2_FRAME", "ALTREF_FRAME", "NONE_FRAME"]


class RefT(int):
    """A RefType value (src/partition.rs RefType)."""

    def __new__(cls, v):
        return int.__new__(cls, v)

    def to_index(self):
        return RI.TInt(int(self) - 1, "usize")


def usz(v):
    return RI.TInt(int(v), "usize")


def mv(row, col):
    return H.motion_vector(int(row), int(col))


def tile_bo(x, y):
    bo = RI.Struct("BlockOffset", {"x": usz(x), "y": usz(y)})
    return RI.Struct("TileBlockOffset", {
        "0": bo, "with_offset": lambda dx, dy: tile_bo(x + int(RI.deref(dx)), y + int(RI.deref(dy)))})


class Blocks:
    """TileBlocks over a case's grid (src/tiling/tile_blocks.rs)."""

    def __init__(self, grid, cols, rows, x, y, frame_cols, frame_rows):
        self.grid, self._cols, self._rows, self._x, self._y = grid, cols, rows, x, y
        self.frame_cols, self.frame_rows = usz(frame_cols), usz(frame_rows)

    def index_any(self, bo):
        b = bo._f["0"]
        return self.grid[int(b._f["y"])][int(b._f["x"])]

    def cols(self):
        return usz(self._cols)

    def rows(self):
        return usz(self._rows)

    def x(self):
        return usz(self._x)

    def y(self):
        return usz(self._y)


def make():
    I = G.make_interp()
    for extra in ("context.rs", "partition.rs"):
        I.sources.append(RI.Source(REF + extra))
    ctx = G.src_of(I, "context.rs")
    I.define_impl("ContextWriter", [ctx.fn(n, "impl<'a> ContextWriter<'a>") for n in (
        "find_mvrefs", "setup_mvref_list", "scan_row_mbmi", "scan_col_mbmi", "scan_blk_mbmi",
        "add_ref_mv_candidate", "add_extra_mv_candidate", "find_matching_mv",
        "find_matching_mv_and_update_weight", "find_matching_comp_mv_and_update_weight",
        "add_offset", "find_valid_row_offs", "find_valid_col_offs")])
    I.define_impl("Block", [ctx.fn("is_inter", "impl Block")])
    I.define_fn(G.src_of(I, "partition.rs").fn("has_tr"))
    env = I.globals.vars
    for i, n in enumerate(H.BLOCK_NAMES):
        env["BLOCK_" + n] = H.BlockSizeV(i)
    env["BlockSize"] = type("BlockSizeNS", (), {"BLOCK_" + n: H.BlockSizeV(i)
                                                for i, n in enumerate(H.BLOCK_NAMES)})
    env["PredictionMode"] = type("PredictionModeNS", (), dict(PM))
    for i, n in enumerate(REF_NAMES):
        env[n] = RefT(i)
    env.update({"MVREF_ROW_COLS": usz(3), "REF_CAT_LEVEL": RI.TInt(640, "u32"),
                "MAX_REF_MV_STACK_SIZE": usz(8), "REFMV_OFFSET": usz(4),
                "LOCAL_BLOCK_MASK": usz(15)})
    env["CandidateMV"] = RI.StructType("CandidateMV")
    env["BlockOffset"] = RI.StructType("BlockOffset")
    env["PlaneBlockOffset"] = lambda bo: RI.Struct("PlaneBlockOffset", {"0": bo})
    env["ContextWriter"] = RI.StructType("ContextWriter")
    env["Block"] = RI.StructType("Block")
    I.release = True
    return I


def call(I, obj, name, *args):
    return I.make_method(obj._name, name, obj, I.globals)(*args)


def rand_mv(rng, pool):
    if rng.random() < 0.7:
        return pool[int(rng.integers(0, len(pool)))]
    return (int(rng.integers(-300, 300)), int(rng.integers(-300, 300)))


def gen_case(rng, I, case, out):
    # tile size in 4x4 units (ragged right / bottom edges), origin in the frame
    sbw, sbh = int(rng.integers(1, 4)), int(rng.integers(1, 4))
    cols = sbw * 16 - (int(rng.integers(0, 4)) * 2 if rng.random() < 0.4 else 0)
    rows = sbh * 16 - (int(rng.integers(0, 4)) * 2 if rng.random() < 0.4 else 0)
    tx, ty = int(rng.integers(0, 3)) * 16, int(rng.integers(0, 3)) * 16
    fcols, fr = tx + cols + int(rng.integers(0, 2)) * 16, ty + rows + int(rng.integers(0, 2)) * 16
    pool = [(int(rng.integers(-200, 200)), int(rng.integers(-200, 200))) for _ in range(3)]
    W, Hh = sbw * 16, sbh * 16
    cells = [[None] * W for _ in range(Hh)]
    recs = np.zeros((Hh, W, 9), np.int32)

    def leaf(x, y, n4):
        r = rng.random()
        if r < 0.2:
            refs, mode = (0, 8), PM["DC_PRED"]
        elif r < 0.45:
            refs, mode = (1, 2), PM[MODES[20 + int(rng.integers(0, 8))]]
        else:
            refs = (1 + int(rng.integers(0, 2)), 8)
            mode = PM[MODES[14 + int(rng.integers(0, 6))]]
        m0, m1 = rand_mv(rng, pool), rand_mv(rng, pool)
        if refs[1] == 8:
            m1 = (0, 0)
        if refs[0] == 0:
            m0 = m1 = (0, 0)
        b = RI.Struct("Block", {
            "mode": mode, "ref_frames": [RefT(refs[0]), RefT(refs[1])],
            "mv": [mv(*m0), mv(*m1)], "n4_w": usz(n4), "n4_h": usz(n4)})
        for j in range(y, min(y + n4, Hh)):
            for i in range(x, min(x + n4, W)):
                cells[j][i] = b
                recs[j, i] = (refs[0], refs[1], m0[0], m0[1], m1[0], m1[1], n4, n4,
                              int(mode in NEWMV_MODES))

    def split(x, y, n4):
        if n4 > 2 and rng.random() < 0.45:
            h = n4 // 2
            for (dx, dy) in ((0, 0), (h, 0), (0, h), (h, h)):
                split(x + dx, y + dy, h)
        else:
            leaf(x, y, n4)
    for sy in range(sbh):
        for sx in range(sbw):
            split(sx * 16, sy * 16, 16)
    blocks = Blocks(cells, cols, rows, tx, ty, fcols, fr)
    sbias = [bool(rng.random() < 0.5) for _ in range(7)]
    fi = RI.Struct("FrameInvariants", {"ref_frame_sign_bias": sbias})
    cw = RI.Struct("ContextWriter", {"bc": RI.Struct("BlockContext", {"blocks": blocks})})
    out["grids"].append((case, tx, ty, cols, rows, fcols, fr, W, Hh, int(sbias[0]), int(sbias[1])))
    out["cells"].append(recs.reshape(-1, 9))
    nq = 0
    for _ in range(40):
        n4 = [16, 16, 16, 8, 4, 2][int(rng.integers(0, 6))]
        bx = int(rng.integers(0, max(1, cols // n4))) * n4
        by = int(rng.integers(0, max(1, rows // n4))) * n4
        if bx >= cols or by >= rows:
            continue
        kind = int(rng.integers(0, 3))
        rf = (1, 8) if kind == 0 else (2, 8) if kind == 1 else (1, 2)
        bs = H.BlockSizeV(H.BLOCK_NAMES.index("%dX%d" % (n4 * 4, n4 * 4)))
        stack = []
        ctxv = call(I, cw, "find_mvrefs", tile_bo(bx, by), [RefT(rf[0]), RefT(rf[1])], stack, bs,
                    fi, rf[1] != 8)
        ent = np.zeros((9, 5), np.int32)
        for i, c in enumerate(stack):
            ent[i] = (int(c.this_mv.row), int(c.this_mv.col), int(c.comp_mv.row),
                      int(c.comp_mv.col), int(c.weight))
        out["query"].append((case, bx, by, n4, n4, rf[0], rf[1], int(ctxv), len(stack)))
        out["entries"].append(ent)
        nq += 1
    return nq


def main():
    t0 = time.time()
    rng = np.random.default_rng(0x3F5)
    I = make()
    out = {"grids": [], "cells": [], "query": [], "entries": []}
    nq = 0
    for case in range(24):
        nq += gen_case(rng, I, case, out)
    np.savez_compressed(OUT, grids=np.array(out["grids"], np.int32),
                        cells=np.concatenate(out["cells"]).astype(np.int32),
                        query=np.array(out["query"], np.int32),
                        entries=np.array(out["entries"], np.int32))
    print("wrote %s: %d cases, %d queries in %.0f s" % (OUT, len(out["grids"]), nq, time.time() - t0))


if __name__ == "__main__":
    main()
