"""Reference-evaluated vectors for get_subset_predictors
(tests/golden/ref_epzs.npz).

    python tools/refeval/gen_epzs_ref.py        (in the build container)

Runs the reference's own text through tools/refeval/rsinterp.py:

  src/me.rs   get_subset_predictors (:82-174)
  src/mc.rs   impl ops::Add / ops::Div<i16> for MotionVector,
              MotionVector::quantize_to_fullpel / is_zero (:33-58)

The environment supplies: TileBlockOffset / BlockOffset / PlaneBlockOffset
values, ArrayVec as a Python list, the tile's motion field
(TileMotionVectors: [y][x], cols(), x(), y()) and the reference frame's
field (FrameMotionVectors: [y][x], .cols, .rows) over random MV grids.

Vectors (one case = a tile field, a frame field or none, the coarse MVs,
a block offset):
  case:  tile x, y (frame 4x4), cols, rows, frame cols, rows, has_prev,
         bx, by, ncmv
  tile:  the case's tile field (rows x cols, row / col), flattened
  prev:  the frame field (frame rows x cols) or nothing
  cmv:   up to 7 coarse MVs
  out:   n, then up to 17 (row, col)
"""
import os
import re
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(__file__))
import gen_golden_ref as G  # noqa: E402
import rshost as H  # noqa: E402
import rsinterp as RI  # noqa: E402

REF = G.REF
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
OUT = os.path.join(ROOT, "tests", "golden", "ref_epzs.npz")


def usz(v):
    return RI.TInt(int(v), "usize")


def mv(row, col):
    return H.motion_vector(int(row), int(col))


class _ArrayVec:
    @staticmethod
    def new():
        return []


class FrameField:
    """FrameMotionVectors over a (rows, cols, 2) array: [y][x], .cols, .rows."""

    def __init__(self, a):
        self.a = a
        self.cols, self.rows = usz(a.shape[1]), usz(a.shape[0])

    def index_row(self, i):
        return [mv(r, c) for r, c in self.a[i]]


class TileField:
    """TileMotionVectors over a (rows, cols, 2) array: [y][x], cols(), rows(),
    x(), y() (the tile's frame offset)."""

    def __init__(self, a, x, y):
        self.a, self._x, self._y = a, x, y

    def index_row(self, i):
        return [mv(r, c) for r, c in self.a[i]]

    def cols(self):
        return usz(self.a.shape[1])

    def rows(self):
        return usz(self.a.shape[0])

    def x(self):
        return usz(self._x)

    def y(self):
        return usz(self._y)


def make():
    I = G.make_interp()
    mc = G.src_of(I, "mc.rs")
    fns = []
    for m in re.finditer(r"\bimpl\b[^{;]*\bMotionVector\s*\{", mc.src):
        fns += RI.parse_impl_fns(RI.find_item(mc.src, "impl", "MotionVector", m.start()))
    I.define_impl("MotionVector", fns)
    G.F(I, "get_subset_predictors", "me.rs")
    env = I.globals.vars
    env["ArrayVec"] = _ArrayVec
    env["BlockOffset"] = RI.StructType("BlockOffset")
    env["PlaneBlockOffset"] = RI.StructType("PlaneBlockOffset")
    I.release = True
    return I


def rand_field(rng, rows, cols, pool):
    a = np.zeros((rows, cols, 2), np.int64)
    for y in range(rows):
        for x in range(cols):
            r = rng.random()
            if r < 0.3:
                continue  # zero: not pushed, but part of the mean
            v = pool[int(rng.integers(0, len(pool)))] if r < 0.8 else \
                (int(rng.integers(-900, 900)), int(rng.integers(-900, 900)))
            a[y, x] = v
    return a


def main():
    rng = np.random.default_rng(0xE925)
    I = make()
    gsp = I.globals.vars["get_subset_predictors"]
    cases, tiles, prevs, cmvs, outs = [], [], [], [], []
    t0 = time.time()
    for case in range(400):
        cols = int(rng.integers(1, 40))
        rows = int(rng.integers(1, 40))
        tx, ty = int(rng.integers(0, 3)) * 16, int(rng.integers(0, 3)) * 16
        fc, fr = tx + cols + int(rng.integers(0, 20)), ty + rows + int(rng.integers(0, 20))
        pool = [(int(rng.integers(-300, 300)), int(rng.integers(-300, 300))) for _ in range(4)]
        tile = rand_field(rng, rows, cols, pool)
        has_prev = rng.random() < 0.7
        prev = rand_field(rng, fr, fc, pool) if has_prev else None
        bx, by = int(rng.integers(0, cols)), int(rng.integers(0, rows))
        if rng.random() < 0.3:  # the edges
            bx = [0, cols - 1, cols - 2][int(rng.integers(0, 3))] if cols > 1 else 0
            by = [0, rows - 1][int(rng.integers(0, 2))]
        ncmv = int(rng.integers(0, 8))
        cm = [(int(rng.integers(-1200, 1200)), int(rng.integers(-1200, 1200))) for _ in range(ncmv)]
        tbo = RI.Struct("TileBlockOffset", {"0": RI.Struct("BlockOffset", {"x": usz(bx),
                                                                           "y": usz(by)})})
        fref = RI.Struct("ReferenceFrame", {"frame_mvs": [FrameField(prev)] * 2}) if has_prev else None
        res = gsp(tbo, [mv(*c) for c in cm], TileField(tile, tx, ty), fref, usz(1))
        o = np.zeros(35, np.int64)
        o[0] = len(res)
        for i, m in enumerate(res):
            o[1 + 2 * i] = int(m.row)
            o[2 + 2 * i] = int(m.col)
        cases.append((tx, ty, cols, rows, fc, fr, int(has_prev), bx, by, ncmv))
        tiles.append(tile.reshape(-1, 2))
        prevs.append(prev.reshape(-1, 2) if has_prev else np.zeros((0, 2), np.int64))
        c = np.zeros((7, 2), np.int64)
        if ncmv:
            c[:ncmv] = cm
        cmvs.append(c)
        outs.append(o)
    np.savez_compressed(
        OUT, case=np.array(cases, np.int32), tile=np.concatenate(tiles).astype(np.int16),
        tile_len=np.array([len(t) for t in tiles], np.int32),
        prev=np.concatenate(prevs).astype(np.int16),
        prev_len=np.array([len(p) for p in prevs], np.int32),
        cmv=np.array(cmvs, np.int16), out=np.array(outs, np.int32))
    print("wrote %s: %d cases in %.1f s" % (OUT, len(cases), time.time() - t0))


if __name__ == "__main__":
    main()
