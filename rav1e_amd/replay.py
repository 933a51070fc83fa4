"""Hot-path replay: synthetic input frames and the HIP replay driver
(rv_replay_* of include/rav1e_hip.h).  See DESIGN.md "Replay driver".

The replay codes a stream in the reorder pyramid's coding order: per frame
the accelerated stages of a speed-10 rav1e encode of one tile group (coarse
1/4-res full search, 1/2-res and full-res diamond + sub-pel search, every
RDO inter candidate skip / non-skip with rav1e's rd cost, the winners'
reconstruction -- the later frames' reference -- and the 8x8 importance
SATD), all frames resident in HBM.
"""
from __future__ import annotations

import ctypes as C

import os

import numpy as np

from . import RvReplayCfg, RvReplayFrameInfo, RvReplayLevelParams, _check, lib
from . import rate as _rate

DEFAULT_QUANTIZER = 100  # rav1e's default --quantizer (src/api/config.rs)

RV_REPLAY_EXHAUSTIVE_FS = 4  # F1 without successive elimination (same results)
RV_REPLAY_SPEED6 = 8  # the speed-6 schedule: partition RDO 64x64 .. 8x8 (config D)
RV_REPLAY_DEBLOCK = 16  # deblock every coded frame before it becomes a reference (1 group)
RV_REPLAY_CDEF = 32  # CDEF after deblocking (needs RV_REPLAY_DEBLOCK), cdef_bits 0
RV_REPLAY_LRF = 512  # loop restoration (self-guided) after CDEF (needs RV_REPLAY_CDEF, one group)
RV_REPLAY_NO_INTRA = 64  # no intra-mode screening of non-skip superblocks (default: on
#                          at speed 10 in 4:2:0)
RV_REPLAY_ENTROPY = 128  # F8: code every frame's coefficients (device tokens, host range coder)
RV_REPLAY_MVREF_STANDIN = 256  # speed 10: neighbour-NEWMV stacks instead of rav1e's (A/B only)
# HIP-event stages of a frame: F0, F1, F2, FL (lookahead), F3 full-pel, F3
# sub-pel, F4 single, F4 compound, F4 argmin, F6 commit, F6b intra, F5, F7,
# then the lookahead's own span, the speed-10 edge levels' own span and
# (RV_REPLAY_ENTROPY) F8's coefficient tokens
N_STAGES = 16

# GOP of the reference's reorder pyramid (src/api/internal.rs:61-95):
# group_input_len 4, levels 0,1,2,2 -> me_range_scale = 4 >> level
# (src/encoder.rs:838).
GOP_SCALES = (4, 2, 1, 1)

def _hash32(x: np.ndarray) -> np.ndarray:
    """lowbias32 on uint32 arrays (wrapping), = synth_hash in rv_frame.hip."""
    x = x.astype(np.uint32)
    x ^= x >> np.uint32(16)
    x *= np.uint32(0x7FEB352D)
    x ^= x >> np.uint32(15)
    x *= np.uint32(0x846CA68B)
    x ^= x >> np.uint32(16)
    return x


def _u32(v) -> np.ndarray:
    return np.asarray(v, dtype=np.int64).astype(np.uint32)


def _wave(q: np.ndarray, period: int) -> np.ndarray:
    h = period // 2
    return np.where(q < h, 256 * q * (h - q) // (h * h), -(256 * (q - h) * (period - q) // (h * h)))


def _lat(ix: np.ndarray, iy: np.ndarray) -> np.ndarray:
    k = _u32(ix) * np.uint32(0x9E3779B1) ^ _u32(iy) * np.uint32(0x85EBCA77) ^ np.uint32(0x5EED)
    return (_hash32(k) & np.uint32(511)).astype(np.int64) - 256


def synth_plane(w, h, t, xdec=0, ydec=0, pidx=0, bd=8) -> np.ndarray:
    """Plane pidx of synthetic frame t (integer form):
    bit-identical to rv_synth_frame (rv_frame.hip synth_kernel).  A 2-D wave
    times a value-noise texture on an 8-px lattice plus +-2 noise, moving
    (1.25, 0.75) luma px per frame, in luma-space quarter-pel coordinates."""
    with np.errstate(over="ignore"):
        x = np.arange(w, dtype=np.int64)[None, :]
        y = np.arange(h, dtype=np.int64)[:, None]
        X4 = ((4 * x) << xdec) - 5 * t + 64 * pidx
        Y4 = ((4 * y) << ydec) - 3 * t
        X4, Y4 = np.broadcast_arrays(X4, Y4)
        ix, fx, iy, fy = X4 >> 5, X4 & 31, Y4 >> 5, Y4 & 31
        v = ((_lat(ix, iy) * (32 - fx) + _lat(ix + 1, iy) * fx) * (32 - fy) +
             (_lat(ix, iy + 1) * (32 - fx) + _lat(ix + 1, iy + 1) * fx) * fy)
        ta, wa = (12, 30) if pidx else (24, 60)
        tex = (v * ta) >> 18
        wave = (_wave(X4 % 388, 388) * _wave(Y4 % 244, 244) * wa) >> 12
        xs, ys = np.broadcast_arrays(x, y)
        hs = _hash32(_u32(xs) * np.uint32(0x27D4EB2D) ^ _u32(ys) * np.uint32(0x165667B1) ^
                     _u32(t) * np.uint32(0x9E3779B9) ^ _u32(pidx) * np.uint32(0x85EBCA6B))
        noise = (hs % np.uint32(5)).astype(np.int64) - 2
        v8 = np.clip(128 + wave + tex + noise, 0, 255)
        if bd == 8:
            return v8.astype(np.uint8)
        lo = (_hash32(hs ^ np.uint32(0xABCD)) & np.uint32((1 << (bd - 8)) - 1)).astype(np.int64)
        return ((v8 << (bd - 8)) | lo).astype(np.uint16)


def synth_frame(w, h, t, xdec=1, ydec=1, bd=8) -> np.ndarray:
    """Planar Y, U, V of synthetic frame t, concatenated (= rv_synth_frame)."""
    cw, ch = (w + xdec) >> xdec, (h + ydec) >> ydec
    y = synth_plane(w, h, t, 0, 0, 0, bd)
    u = synth_plane(cw, ch, t, xdec, ydec, 1, bd)
    v = synth_plane(cw, ch, t, xdec, ydec, 2, bd)
    return np.concatenate([y.ravel(), u.ravel(), v.ravel()])


def frame_bytes(width, height, xdec=1, ydec=1, bit_depth=8) -> int:
    """Bytes of one planar Y, U, V picture (tightly packed)."""
    cw, ch = (width + xdec) >> xdec, (height + ydec) >> ydec
    return (width * height + 2 * cw * ch) * (2 if bit_depth > 8 else 1)


# ---- tiling (TilingInfo, src/tiling/tiler.rs:18-138) ---------------------
MAX_TILE_WIDTH, MAX_TILE_AREA = 4096, 4096 * 2304
MAX_TILE_COLS = MAX_TILE_ROWS = 64
MAX_TILE_RATE = 4096.0 * 2176.0 * 60.0 * 1.1


def tile_log2(blk_size: int, target: int) -> int:
    """TilingInfo::tile_log2 (src/tiling/tiler.rs:132-138)."""
    k = 0
    while (blk_size << k) < target:
        k += 1
    return k


def tiling_info(width, height, tile_cols_log2=0, tile_rows_log2=0, frame_rate=30.0,
                sb_size_log2=6) -> dict:
    """TilingInfo::from_target_tiles (src/tiling/tiler.rs:49-126)."""
    import math
    fw, fh = (width + 7) & ~7, (height + 7) & ~7

    def shift(v, n):  # align_power_of_two_and_shift
        return (v + (1 << n) - 1) >> n
    sb_cols, sb_rows = shift(fw, sb_size_log2), shift(fh, sb_size_log2)
    max_tile_width_sb = MAX_TILE_WIDTH >> sb_size_log2
    max_tile_area_sb = MAX_TILE_AREA >> (2 * sb_size_log2)
    min_cols_log2 = tile_log2(max_tile_width_sb, sb_cols)
    max_cols_log2 = tile_log2(1, min(sb_cols, MAX_TILE_COLS))
    max_rows_log2 = tile_log2(1, min(sb_rows, MAX_TILE_ROWS))
    min_tiles_log2 = max(min_cols_log2, tile_log2(max_tile_area_sb, sb_cols * sb_rows))
    rl = math.ceil(math.log2(math.ceil(fw * fh * frame_rate / MAX_TILE_RATE)))
    min_tiles_rl_log2 = max(min_tiles_log2, int(rl))
    cols_log2 = min(max(tile_cols_log2, min_cols_log2), max_cols_log2)
    tile_w = shift(sb_cols, cols_log2)
    min_rows_log2 = min_tiles_log2 - cols_log2 if min_tiles_log2 > cols_log2 else 0
    min_rows_rl = min_tiles_rl_log2 - cols_log2 if min_tiles_rl_log2 > cols_log2 else 0
    rows_log2 = min(max(tile_rows_log2, min_rows_log2, min_rows_rl), max_rows_log2)
    tile_h = shift(sb_rows, rows_log2)
    return {"tile_width_sb": tile_w, "tile_height_sb": tile_h,
            "cols": (sb_cols + tile_w - 1) // tile_w, "rows": (sb_rows + tile_h - 1) // tile_h,
            "tile_cols_log2": cols_log2, "tile_rows_log2": rows_log2,
            "max_tile_cols_log2": max_cols_log2, "max_tile_rows_log2": max_rows_log2,
            "sb_cols": sb_cols, "sb_rows": sb_rows}


def tiling_for(width, height, tile_cols=0, tile_rows=0, tiles=0) -> dict:
    """The encoder's tiling: --tile-cols / --tile-rows, or --tiles via the
    search loop of src/encoder.rs:583-621."""
    t = tiling_info(width, height, tile_log2(1, max(tile_cols, 1)), tile_log2(1, max(tile_rows, 1)))
    if tiles > 0:
        rl = cl = 0
        while rl < t["max_tile_rows_log2"] or cl < t["max_tile_cols_log2"]:
            t = tiling_info(width, height, cl, rl)
            if t["rows"] * t["cols"] >= tiles:
                break
            if (t["tile_height_sb"] >= t["tile_width_sb"] and
                    t["tile_rows_log2"] < t["max_tile_rows_log2"]) or cl >= t["max_tile_cols_log2"]:
                rl += 1
            else:
                cl += 1
    return t


def tile_groups(tiling: dict, world: int) -> list:
    """Split the tiles (raster order) into `world` contiguous groups, one per
    rank; every group must be a rectangle of whole tiles.  Rects are
    (tx0, ty0, tw, th) in superblocks."""
    cols, rows = tiling["cols"], tiling["rows"]
    tws, ths = tiling["tile_width_sb"], tiling["tile_height_sb"]
    sbc, sbr = tiling["sb_cols"], tiling["sb_rows"]
    n = cols * rows
    if world < 1 or world > n:
        raise ValueError(f"{world} ranks for {n} tiles")
    out = []
    for r in range(world):
        a, b = r * n // world, (r + 1) * n // world
        tiles = [(i % cols, i // cols) for i in range(a, b)]
        c0, c1 = min(t[0] for t in tiles), max(t[0] for t in tiles)
        r0, r1 = min(t[1] for t in tiles), max(t[1] for t in tiles)
        if len(tiles) != (c1 - c0 + 1) * (r1 - r0 + 1):
            raise ValueError(f"tiles {a}..{b - 1} of a {cols}x{rows} grid are not a rectangle")
        x0, y0 = c0 * tws, r0 * ths
        out.append((x0, y0, min((c1 + 1) * tws, sbc) - x0, min((r1 + 1) * ths, sbr) - y0))
    return out


# result words per superblock and reference (rv_replay_results): coarse
# (mv, cost), the four half-res quadrants (the encode's build_half_res_pmvs),
# full-pel, sub-pel, the 16 lookahead 16x16 blocks, the lookahead's four
# half-res quadrants; then per superblock winner, skip, cost, distortion
WORDS_PER_REF = 2 + 8 + 2 + 2 + 32 + 8
W_COARSE, W_HALF, W_FULL, W_SUB, W_LOOK, W_HALF_LA = 0, 2, 10, 12, 14, 46


def sb_words_per(n_refs):
    return WORDS_PER_REF * n_refs + 4


def level_rect(width, height, tile_w_sb=0, tile_h_sb=0, tile_x0=0, tile_y0=0, speed=10, xdec=1,
               ydec=1):
    """The group superblocks (x0, y0, w, h) the 32x32 .. 8x8 levels cover:
    speed 6 every one; speed 10 (4:2:0 / 4:4:4) the bounding rectangle of
    those past the frame's right or bottom edge (encode_partition_topdown's
    must_split, src/encoder.rs:2407-2445); None without levels."""
    sbc, sbr = (width + 63) // 64, (height + 63) // 64
    tw = tile_w_sb or (sbc - tile_x0)
    th = tile_h_sb or (sbr - tile_y0)
    if speed == 6:
        return (0, 0, tw, th)
    if xdec != ydec:
        return None
    edge = [(x, y) for y in range(th) for x in range(tw)
            if (tile_x0 + x + 1) * 64 > width or (tile_y0 + y + 1) * 64 > height]
    if not edge:
        return None
    xs, ys = [e[0] for e in edge], [e[1] for e in edge]
    return (min(xs), min(ys), max(xs) - min(xs) + 1, max(ys) - min(ys) + 1)


def result_words(width, height, n_refs, tile_w_sb=0, tile_h_sb=0, tile_x0=0, tile_y0=0,
                 speed=10, xdec=1, ydec=1):
    """Result words of a group (rv_replay_results): per superblock
    WORDS_PER_REF * R + 4; with levels (level_rect) 4 * R + 4 per 32x32,
    16x16 and 8x8 block of the rectangle and one partition mask per
    superblock; then 5 tail words."""
    sbc, sbr = (width + 63) // 64, (height + 63) // 64
    tw = tile_w_sb or (sbc - tile_x0)
    th = tile_h_sb or (sbr - tile_y0)
    n = tw * th * sb_words_per(n_refs)
    rect = level_rect(width, height, tile_w_sb, tile_h_sb, tile_x0, tile_y0, speed, xdec, ydec)
    if rect:
        n += sum(rect[2] * rect[3] * 4 ** l * (4 * n_refs + 4) for l in (1, 2, 3)) + tw * th
    return n + 5


def level_words(width, height, n_refs, words, tile_w_sb=0, tile_h_sb=0, tile_x0=0, tile_y0=0,
                speed=6, xdec=1, ydec=1):
    """Split result words with levels: (superblock words [nsb, 46R+4], [level
    1..3 words [n_l, 4R+4]] over level_rect, partition masks [nsb], tail
    [5])."""
    sbc, sbr = (width + 63) // 64, (height + 63) // 64
    tw = tile_w_sb or (sbc - tile_x0)
    th = tile_h_sb or (sbr - tile_y0)
    nsb = tw * th
    rect = level_rect(width, height, tile_w_sb, tile_h_sb, tile_x0, tile_y0, speed, xdec, ydec)
    o = nsb * sb_words_per(n_refs)
    sbw = words[:o].reshape(nsb, sb_words_per(n_refs))
    lv = []
    for l in (1, 2, 3):
        n = rect[2] * rect[3] * 4 ** l
        lv.append(words[o:o + n * (4 * n_refs + 4)].reshape(n, 4 * n_refs + 4))
        o += n * (4 * n_refs + 4)
    return sbw, lv, words[o:o + nsb], words[o + nsb:]


class HipReplay:
    """The GPU replay of one tile group (rv_replay_create ... rv_replay_destroy).

    group = (tx0, ty0, tw, th) superblocks (None: the whole frame);
    tile_size = (tile_width_sb, tile_height_sb) of the uniform tiling (0: one
    tile); n_inputs input frames live in HBM (display d reads d % n_inputs)."""

    def __init__(self, width, height, xdec=1, ydec=1, bit_depth=8, n_refs=2, group=None,
                 tile_size=(0, 0), n_inputs=8, stream=None, flags=0,
                 quantizer=DEFAULT_QUANTIZER, imp_window=0, imp_limit=0):
        cfg = RvReplayCfg()
        cfg.width, cfg.height, cfg.xdec, cfg.ydec = width, height, xdec, ydec
        cfg.bit_depth, cfg.n_refs, cfg.n_inputs, cfg.flags = bit_depth, n_refs, n_inputs, flags
        cfg.tile_w_sb, cfg.tile_h_sb = tile_size
        if group:
            cfg.tile_x0, cfg.tile_y0, cfg.tile_w, cfg.tile_h = group
        self.cfg = cfg
        self.geom = (width, height, xdec, ydec, bit_depth)
        self.h = lib().rv_replay_create(C.byref(cfg), stream)
        if not self.h:
            raise RuntimeError(f"rv_replay_create: {lib().rv_last_error().decode()}")
        self.speed = 6 if flags & RV_REPLAY_SPEED6 else 10
        self.n_words = result_words(width, height, n_refs, cfg.tile_w, cfg.tile_h,
                                    cfg.tile_x0, cfg.tile_y0, self.speed, xdec, ydec)
        self.levels = _rate.level_params(quantizer, bit_depth)
        for lv, d in enumerate(self.levels):
            p = RvReplayLevelParams.from_dict(d)
            _check(lib().rv_replay_set_level_params(self.h, lv, C.byref(p)),
                   "rv_replay_set_level_params")
        self.imp_window = imp_window
        if imp_window:
            _check(lib().rv_replay_set_imp_window(self.h, int(imp_window), int(imp_limit)),
                   "rv_replay_set_imp_window")
        self.imp_shape = ((height + 7) // 8, (width + 7) // 8)

    def twin(self, stream=None):
        """A second instance sharing this one's DPB and inputs
        (rv_replay_create_twin): it codes the level-2 frames concurrently
        with this instance's levels 0 / 1 (PairedReplay).  stream: its
        stream (the caller's, kept alive until the twin closes); None: its
        own."""
        t = HipReplay.__new__(HipReplay)
        t.cfg, t.geom, t.speed, t.n_words, t.levels = self.cfg, self.geom, self.speed, \
            self.n_words, self.levels
        t.imp_window, t.imp_shape = self.imp_window, self.imp_shape
        t.h = lib().rv_replay_create_twin(self.h, stream)
        if not t.h:
            raise RuntimeError(f"rv_replay_create_twin: {lib().rv_last_error().decode()}")
        t.primary = self  # the DPB's owner outlives the twin
        return t

    def seek(self, n: int):
        """The next frame() codes coding-order frame n (rv_replay_seek)."""
        _check(lib().rv_replay_seek(self.h, int(n)), "rv_replay_seek")

    @property
    def stream(self):
        return lib().rv_replay_stream(self.h)

    def _frame_array(self):
        w, h, xd, yd, bd = self.geom
        n = frame_bytes(w, h, xd, yd, bd) // (2 if bd > 8 else 1)
        return np.zeros(n, dtype=np.uint16 if bd > 8 else np.uint8)

    def synth_inputs(self, t0: int = 0):
        _check(lib().rv_replay_synth_inputs(self.h, t0), "rv_replay_synth_inputs")

    def set_input(self, idx: int, yuv: np.ndarray):
        yuv = np.ascontiguousarray(yuv)
        _check(lib().rv_replay_set_input(self.h, idx, yuv.ctypes.data), "rv_replay_set_input")

    def get_input(self, idx: int) -> np.ndarray:
        out = self._frame_array()
        _check(lib().rv_replay_get_input(self.h, idx, out.ctypes.data), "rv_replay_get_input")
        return out

    def lrf_units(self, plane: int) -> np.ndarray:
        """RV_REPLAY_LRF: the last frame's units of plane p, (set, xqd0,
        xqd1) per superblock (set -1: None)."""
        n = ((self.cfg.width + 63) // 64) * ((self.cfg.height + 63) // 64)
        out = np.zeros(3 * n, np.int8)
        _check(lib().rv_replay_lrf_units(self.h, plane, out.ctypes.data, out.size), "rv_replay_lrf_units")
        return out.reshape(n, 3)

    def get_recon(self, display: int) -> np.ndarray:
        out = self._frame_array()
        _check(lib().rv_replay_get_recon(self.h, display, out.ctypes.data), "rv_replay_get_recon")
        return out

    def set_inputs_ready(self, displays: int):
        """The inputs of displays < `displays` are in place: the lookahead
        engine may run ahead as far as its ring allows
        (rv_replay_set_inputs_ready)."""
        _check(lib().rv_replay_set_inputs_ready(self.h, int(displays)),
               "rv_replay_set_inputs_ready")

    def set_importances(self, imp):
        if imp is None:
            _check(lib().rv_replay_set_importances(self.h, None, 0), "rv_replay_set_importances")
            return
        imp = np.ascontiguousarray(imp, dtype=np.float32)
        _check(lib().rv_replay_set_importances(self.h, imp.ctypes.data, imp.size),
               "rv_replay_set_importances")

    def importances(self) -> np.ndarray:
        """The block importances the last coded frame's RDO used."""
        out = np.zeros(self.imp_shape, np.float32)
        _check(lib().rv_replay_get_importances(self.h, out.ctypes.data, out.size),
               "rv_replay_get_importances")
        return out

    def frame(self) -> dict:
        fi = RvReplayFrameInfo()
        _check(lib().rv_replay_frame(self.h, C.byref(fi)), "rv_replay_frame")
        return {"display": fi.display, "me_range_scale": fi.me_range_scale, "level": fi.level,
                "is_key": fi.is_key, "ref_display": list(fi.ref_display),
                "compound": fi.compound}

    def set_la_exchange(self, comm=None, hub=None):
        """A tile group's importance window: how the other groups' lookahead
        parts arrive (rv_replay_set_la_exchange) -- an RCCL communicator
        (handle) or an in-process LaHub."""
        _check(lib().rv_replay_set_la_exchange(self.h, comm, hub.h if hub else None),
               "rv_replay_set_la_exchange")

    def set_groups(self, rects, my_group, comm=None):
        arr = np.ascontiguousarray(np.asarray(rects, dtype=np.int32).ravel())
        _check(lib().rv_replay_set_groups(self.h, len(rects), arr.ctypes.data, my_group, comm),
               "rv_replay_set_groups")

    def exchange_buffers(self):
        """(send, recv, bytes_per_group): device pointers of the packed
        region of this group and of the gathered regions of all groups."""
        s, r, n = C.c_void_p(), C.c_void_p(), C.c_size_t()
        _check(lib().rv_replay_exchange_buffers(self.h, C.byref(s), C.byref(r), C.byref(n)),
               "rv_replay_exchange_buffers")
        return s.value, r.value, n.value

    def import_(self):
        _check(lib().rv_replay_import(self.h), "rv_replay_import")

    def results(self) -> np.ndarray:
        out = np.zeros(self.n_words, dtype=np.uint64)
        n = lib().rv_replay_results(self.h, out.ctypes.data, out.size)
        if n < 0:
            _check(n, "rv_replay_results")
        return out[:n]

    def entropy_stats(self):
        """RV_REPLAY_ENTROPY: [last frame's coefficient bytes, tiles, FNV-1a
        of its tiles' bytes, frames coded, bytes over every frame] (waits
        for the host coder)."""
        out = np.zeros(5, np.uint64)
        n = lib().rv_replay_entropy_stats(self.h, out.ctypes.data, 5)
        if n < 0:
            _check(n, "rv_replay_entropy_stats")
        return [int(v) for v in out]

    def set_timing(self, stride: int, block: int = 1):
        """Record the timing events on coded frames f with (f // block) %
        stride == 0 (rv_replay_set_timing)."""
        _check(lib().rv_replay_set_timing(self.h, stride, block), "rv_replay_set_timing")

    def stage_ms(self) -> np.ndarray:
        out = np.zeros(N_STAGES, dtype=np.float32)
        n = lib().rv_replay_stage_times(self.h, out.ctypes.data, N_STAGES)
        if n < 0:
            _check(n, "rv_replay_stage_times")
        return out[:n]

    def stage_ms_sum(self, last_frames: int) -> np.ndarray:
        out = np.zeros(N_STAGES, dtype=np.float32)
        n = lib().rv_replay_stage_times_sum(self.h, last_frames, out.ctypes.data, N_STAGES)
        if n < 0:
            _check(n, "rv_replay_stage_times_sum")
        return out  # stages past n (F8 without RV_REPLAY_ENTROPY) stay 0

    def set_kernel_probe(self, on: bool = True):
        """(Re)start the F3 sub-pel kernel probe (rv_replay_set_kernel_probe)."""
        _check(lib().rv_replay_set_kernel_probe(self.h, 1 if on else 0),
               "rv_replay_set_kernel_probe")

    def kernel_probe(self) -> np.ndarray:
        """[launches, summed ms (HIP event pairs), candidate evaluations,
        jobs, summed ms (device clock spans)] of the probed F3 sub-pel
        launches since the probe started, then [launches, event ms,
        device-clock ms, single / compound luma candidates, single / compound
        chroma transform blocks] of the F4 candidate-list launches."""
        out = np.zeros(12, np.float64)
        _check(lib().rv_replay_kernel_probe(self.h, out.ctypes.data, 12) - 12,
               "rv_replay_kernel_probe")
        return out

    def counters(self) -> np.ndarray:
        """[F3 full-pel evals, F3 sub-pel evals, frames, F4 single-reference
        candidates, F4 compound candidates of the 64x64 blocks, then (speed
        6) single / compound of the 32x32, 16x16 and 8x8 blocks, superblocks
        intra-screened, intra winners, intra rounds] over the last <= 64
        frames, then (speed 10, since creation) the MV-stack rounds, the
        superblocks they re-evaluated, the frames, and the round runs (1 +
        the MV / intra passes of each frame), the lookahead's EPZS rounds,
        the jobs they re-ran and the frames they belong to."""
        out = np.zeros(21, dtype=np.uint64)
        _check(lib().rv_replay_counters(self.h, out.ctypes.data, 21) - 21, "rv_replay_counters")
        return out

    def close(self):
        if self.h:
            lib().rv_replay_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def frame_info(n: int, n_refs: int = 2) -> dict:
    """Coding-order frame n of the reorder pyramid (rv_replay.hip
    frame_info): display, me_range_scale, pyramid level, key flag,
    reference displays, compound."""
    if n == 0:
        return {"display": 0, "me_range_scale": 0, "level": 0, "is_key": 1,
                "ref_display": [0, 0], "compound": 0}
    g, j = (n - 1) // 4, (n - 1) % 4
    rf = ((0, -4), (0, 4), (0, 2), (2, 4))[j]
    refs = [max(0, 4 * g + rf[k]) for k in range(n_refs)] + [0] * (2 - n_refs)
    return {"display": 4 * g + (4, 2, 1, 3)[j], "me_range_scale": (4, 2, 1, 1)[j],
            "level": (0, 1, 2, 2)[j], "is_key": 0, "ref_display": refs,
            "compound": int(n_refs == 2 and j in (1, 3))}


class PairedReplay:
    """One stream coded by two instances of the same tile group: `primary`
    codes the key frame, the pyramid's levels 0 / 1 (display 4g+4, 4g+2)
    and (twin_levels "l2b", the default) the level-2 frame 4g+1; its twin
    (rv_replay_create_twin: shared DPB and inputs) the level-2 frame 4g+3
    ("l2": both level-2 frames), which no frame references, on its own
    stream and host thread.  Device events order the two: a twin frame of
    group g after the primary's level-1 frame of g, the primary's level-0
    frame of g + 2 (its DPB slot is display 4g's) after the twin's group g.
    frame() / drain() / results() / counters() / close() follow HipReplay's
    interface for bench.timed_run.  The frames' results are the sequential
    ones (the orders only interleave independent frames)."""

    def __init__(self, primary: "HipReplay", twin_levels: str = None):
        import queue
        import threading
        # which frames of a group the twin codes: "l2" both level-2 frames
        # (4g+1, 4g+3), "l2b" only 4g+3 (the primary codes 4g+1 after 4g+2)
        # (2160p: "l2b" 187 vs 163-166 fps for "l2", r04j2 -- the compound
        # frames 4g+2 and 4g+3 carry the most MV-stack rounds, so "l2" left
        # the twin with the heavier half)
        self.twin_levels = twin_levels or os.environ.get("RAV1E_PAIRED_TWIN", "l2b")
        if self.twin_levels not in ("l2", "l2b", "alt"):
            raise ValueError(f"PairedReplay: twin_levels {self.twin_levels!r}")
        self.p = primary
        self.t = primary.twin()
        self.n = 0
        self.q = queue.Queue()
        self.err = None
        self._thr = threading
        self.ev_p = [lib().rv_event_create() for _ in range(8)]
        self.ev_t = [lib().rv_event_create() for _ in range(8)]
        self.ready_p, self.ready_t = {}, {}
        self.worker = threading.Thread(target=self._run, daemon=True)
        self.worker.start()

    def on_primary(self, f: int) -> bool:
        """Inter frame f (coded frame f + 1: group f // 4, frame j = f % 4
        of it) runs on the primary.  "alt": the twin codes 4g+3, and 4g+1
        of the odd groups."""
        g, j = f // 4, f % 4
        if j < 2:
            return True
        if j == 3:
            return False
        return self.twin_levels == "l2b" or (self.twin_levels == "alt" and g % 2 == 0)

    def _flag(self, d, g):
        if g not in d:
            d[g] = self._thr.Event()
        return d[g]

    def frame(self) -> dict:
        n = self.n
        self.n += 1
        if n == 0:
            return self.p.frame()
        g, j = (n - 1) // 4, (n - 1) % 4
        if not self.on_primary(n - 1):
            self.q.put(n)
            return frame_info(n, self.p.cfg.n_refs)
        if j == 0 and g >= 2:
            self._flag(self.ready_t, g - 2).wait()
            self._raise()
            _check(lib().rv_stream_wait_event(self.p.stream, self.ev_t[(g - 2) % 8]),
                   "rv_stream_wait_event")
        self.p.seek(n)  # its own counter has not seen the twin's frames
        info = self.p.frame()
        if j == 1:
            _check(lib().rv_event_record(self.ev_p[g % 8], self.p.stream), "rv_event_record")
            self._flag(self.ready_p, g).set()
        return info

    def _run(self):
        while True:
            n = self.q.get()
            if n is None:
                self.q.task_done()
                return
            g, j = (n - 1) // 4, (n - 1) % 4
            try:
                if self.err is None:
                    self._flag(self.ready_p, g).wait()
                    _check(lib().rv_stream_wait_event(self.t.stream, self.ev_p[g % 8]),
                           "rv_stream_wait_event")
                    self.t.seek(n)
                    self.t.frame()
                    if j == 3:
                        _check(lib().rv_event_record(self.ev_t[g % 8], self.t.stream),
                               "rv_event_record")
            except Exception as e:  # handed to the main thread by drain()
                self.err = e
            finally:
                if j == 3:
                    self._flag(self.ready_t, g).set()
                self.q.task_done()

    def _raise(self):
        if self.err is not None:
            e, self.err = self.err, None
            raise e

    def drain(self):
        """Every frame issued so far has been submitted to its stream."""
        self.q.join()
        self._raise()

    def results(self) -> np.ndarray:
        self.drain()
        return self.p.results()

    def set_timing(self, stride: int, block: int = 1):
        self.p.set_timing(stride, block)
        self.t.set_timing(stride, block)

    def entropy_stats(self):
        """Both instances' coefficient coding: [bytes of the primary's last
        frame, tiles, its hash, frames coded by both, bytes over every
        frame of both]."""
        self.drain()
        a, b = self.p.entropy_stats(), self.t.entropy_stats()
        return [a[0], a[1], a[2], a[3] + b[3], a[4] + b[4]]

    def counters(self) -> np.ndarray:
        """HipReplay.counters summed over both instances (their frames do not
        overlap); [2] = the frames of the window."""
        self.drain()
        a, b = self.p.counters(), self.t.counters()
        out = a + b
        out[2] = max(a[2], b[2])
        return out

    def stage_ms_sum(self, kp: int, kt: int) -> np.ndarray:
        """Stage times summed over the primary's last kp and the twin's last kt
        instrumented frames."""
        self.drain()
        s = np.zeros(N_STAGES, np.float32)
        if kp:
            s = s + self.p.stage_ms_sum(kp)
        if kt:
            s = s + self.t.stage_ms_sum(kt)
        return s

    def close(self):
        if self.t is not None:
            self.q.put(None)
            self.worker.join()
            self.t.close()  # before the primary: it borrows the DPB
            self.t = None
            for e in self.ev_p + self.ev_t:
                lib().rv_event_destroy(e)

    def __getattr__(self, name):  # get_input, get_recon, ... of the primary
        return getattr(self.p, name)


def _refs_of(n: int, n_refs: int) -> list:
    fi = frame_info(n, n_refs)
    return sorted(set(fi["ref_display"][:n_refs]))


def _coded_of_display(d: int) -> int:
    """frame_info's inverse (rv_replay.hip coded_of_display)."""
    if d == 0:
        return 0
    j = {0: 0, 2: 1, 1: 2, 3: 3}[d % 4]
    off = (4, 2, 1, 3)[j]
    return 4 * ((d - off) // 4) + j + 1


class PipelinedReplay:
    """One stream coded by three instances of the same tile group (shared
    DPB and inputs, rv_replay_create_twin), each on its own stream and host
    thread: `primary` the key frame, the level-0 frames (display 4g+4) and
    the level-2 frames 4g+1 (each after the next group's level-0 frame), a
    twin the level-1 frames (4g+2), a second twin the level-2 frames 4g+3.
    Every frame waits, through device events, for the frames on the other
    instances it depends on: the producers of its references, and the
    previous occupant of its DPB slot (display d - rv_replay_dpb_slots())
    with every frame that
    reads it.  The frames' results are the sequential ones."""

    def __init__(self, primary: "HipReplay", instances: int = None):
        import queue
        import threading
        # 3: level 0 + 4g+1 | level 1 | 4g+3; 5: the level-1 and the 4g+3
        # frames alternate between two instances each (even / odd groups)
        self.k = instances or int(os.environ.get("RAV1E_PIPE_INSTANCES", "3"))
        if self.k not in (3, 5):
            raise ValueError(f"PipelinedReplay: {self.k} instances (3 or 5)")
        self.p = primary
        # RAV1E_PIPE_HP (A/B): "1" the twins (the compound frames' instances)
        # on high-priority streams; "L1" the level-1 twin alone (the frames
        # every level-2 frame waits for)
        self.hp_streams = []
        hp = os.environ.get("RAV1E_PIPE_HP")
        self.inst = [primary]
        for i in range(self.k - 1):
            st = None
            if hp == "1" or (hp == "L1" and i == 0):
                st = lib().rv_stream_create_priority(-1)
                if not st:
                    raise RuntimeError(f"rv_stream_create_priority: {lib().rv_last_error().decode()}")
                self.hp_streams.append(st)
            self.inst.append(primary.twin(st))
        self.R = primary.cfg.n_refs
        self.slots = int(lib().rv_replay_dpb_slots())
        self.DEP_SPAN = self.slots + 8
        assert self.EV_RING >= 2 * self.DEP_SPAN, (self.EV_RING, self.DEP_SPAN)
        self.n = 0
        self.err = None
        self.ev = [lib().rv_event_create() for _ in range(self.EV_RING)]
        self.done = {}  # coded frame -> threading.Event (its event is recorded)
        self.lock = threading.Lock()
        self.cv = threading.Condition(self.lock)
        self.issued_set, self.issued_upto, self.pruned = set(), -1, -1
        self.held = None  # a 4g+1 frame waiting for the next level-0 frame
        self.qs = [queue.Queue() for _ in self.inst]
        self.workers = [threading.Thread(target=self._run, args=(i,), daemon=True)
                        for i in range(self.k)]
        for w in self.workers:
            w.start()

    # device events, one per coded frame in flight: frame n records
    # ev[n % EV_RING]; a frame waits for frames at most DEP_SPAN back (its
    # references, and its DPB slot's previous occupant: slots + 8 covers it)
    EV_RING = 128

    def instance_of(self, n: int) -> int:
        if n == 0:
            return 0
        g, j = (n - 1) // 4, (n - 1) % 4
        if self.k == 3:
            return (0, 1, 0, 2)[j]
        return (0, 1 + g % 2, 0, 3 + g % 2)[j]

    def on_primary(self, f: int) -> bool:
        return self.instance_of(f + 1) == 0

    def _flag(self, n):
        with self.lock:
            if n not in self.done:
                assert n > self.pruned, (n, self.pruned)
                self.done[n] = __import__("threading").Event()
            return self.done[n]

    def _mark_issued(self, n):
        """Frame n's stream waits are queued: advance issued_upto (every
        frame <= it has queued its waits) and drop the flags no frame can
        wait on any more (a frame waits on frames at most DEP_SPAN back, and
        every frame still to queue its waits is after issued_upto)."""
        with self.lock:
            self.issued_set.add(n)
            while self.issued_upto + 1 in self.issued_set:
                self.issued_upto += 1
                self.issued_set.discard(self.issued_upto)
            cut = self.issued_upto - self.DEP_SPAN
            if cut > self.pruned:
                for k in range(self.pruned + 1, cut):
                    self.done.pop(k, None)
                self.pruned = cut - 1
            self.cv.notify_all()

    def _before_record(self, n):
        """Frame n is about to re-record ev[n % EV_RING], the event of frame
        n - EV_RING: every frame that can wait on that one (within DEP_SPAN
        after it) must have queued its stream wait first.  Those frames
        precede n and wait only on frames before them, none queued behind n
        on this instance, so this never deadlocks (and in practice never
        blocks: the instances stay within a few frames of each other)."""
        need = n - self.EV_RING + self.DEP_SPAN
        with self.lock:
            while self.issued_upto < need:
                self.cv.wait()

    def _deps(self, n: int) -> list:
        """Coded frames on other instances that frame n waits for."""
        if n == 0:
            return []
        d = frame_info(n, self.R)["display"]
        deps = {_coded_of_display(r) for r in _refs_of(n, self.R)}
        prev = d - self.slots  # the DPB slot's previous occupant and its readers
        if prev >= 0:
            c = _coded_of_display(prev)
            deps.add(c)
            for k in range(c + 1, c + 17):
                if k < n and prev in _refs_of(k, self.R):
                    deps.add(k)
        me = self.instance_of(n)
        return sorted(k for k in deps if k < n and self.instance_of(k) != me)

    def frame(self) -> dict:
        n = self.n
        self.n += 1
        i = self.instance_of(n)
        j = (n - 1) % 4 if n else -1
        if n and j == 2:  # 4g+1: after the next group's level-0 frame
            self.held = n
        else:
            self.qs[i].put(n)
            if n and j == 0 and self.held is not None:
                self.qs[0].put(self.held)
                self.held = None
        self._raise()
        return frame_info(n, self.R)

    def _run(self, i):
        inst = self.inst[i]
        while True:
            n = self.qs[i].get()
            if n is None:
                self.qs[i].task_done()
                return
            try:
                if self.err is None:
                    deps = self._deps(n)
                    assert all(n - k <= self.DEP_SPAN for k in deps), (n, deps)
                    for k in deps:
                        self._flag(k).wait()
                        _check(lib().rv_stream_wait_event(inst.stream, self.ev[k % self.EV_RING]),
                               "rv_stream_wait_event")
                    self._mark_issued(n)
                    if n:
                        inst.seek(n)
                    inst.frame()
                    self._before_record(n)
                    _check(lib().rv_event_record(self.ev[n % self.EV_RING], inst.stream),
                           "rv_event_record")
            except Exception as e:  # handed to the main thread by drain()
                self.err = e
            finally:
                if n not in self.issued_set and n > self.issued_upto:
                    self._mark_issued(n)
                self._flag(n).set()
                self.qs[i].task_done()

    def _raise(self):
        if self.err is not None:
            e, self.err = self.err, None
            raise e

    def drain(self):
        if self.held is not None:  # the stream ends: the held frame goes now
            self.qs[0].put(self.held)
            self.held = None
        for q in self.qs:
            q.join()
        self._raise()

    def results(self) -> np.ndarray:
        self.drain()
        return self.p.results()

    def set_timing(self, stride: int, block: int = 1):
        for t in self.inst:
            t.set_timing(stride, block)

    def entropy_stats(self):
        self.drain()
        st = [t.entropy_stats() for t in self.inst]
        a = st[0]
        return [a[0], a[1], a[2], sum(x[3] for x in st), sum(x[4] for x in st)]

    def counters(self) -> np.ndarray:
        self.drain()
        cs = [t.counters() for t in self.inst]
        out = sum(cs[1:], cs[0].copy())
        out[2] = max(c[2] for c in cs)
        return out

    def set_kernel_probe(self, on: bool = True):
        self.drain()
        for t in self.inst:
            t.set_kernel_probe(on)

    def kernel_probe(self) -> np.ndarray:
        self.drain()
        return sum((t.kernel_probe() for t in self.inst), np.zeros(12))

    def stage_ms_sum_frames(self, frames) -> tuple:
        """Stage times summed over the instrumented inter frames `frames`
        (f: coded frame f + 1), each instance its own last ones; returns
        (sum, frames counted)."""
        self.drain()
        s = np.zeros(N_STAGES, np.float32)
        cnt = [0] * self.k
        for f in frames:
            cnt[self.instance_of(f + 1)] += 1
        for t, k in zip(self.inst, cnt):
            if k:
                s = s + t.stage_ms_sum(min(k, 64))
        return s, sum(min(k, 64) for k in cnt)

    def close(self):
        if self.workers:
            for q in self.qs:
                q.put(None)
            for w in self.workers:
                w.join()
            self.workers = []
            for t in self.inst[1:]:
                t.close()  # before the primary: they borrow the DPB
            for st in self.hp_streams:
                lib().rv_stream_destroy(st)
            self.hp_streams = []
            for e in self.ev:
                lib().rv_event_destroy(e)

    def __getattr__(self, name):
        return getattr(self.p, name)


class LaHub:
    """The in-process exchange of the lookahead engines' frame parts between
    the tile groups of one process (rv_la_hub_create): GPU tests and the
    bench's rank emulation."""

    def __init__(self, n_groups: int):
        self.h = lib().rv_la_hub_create(int(n_groups))
        if not self.h:
            raise RuntimeError(f"rv_la_hub_create: {lib().rv_last_error().decode()}")

    def close(self):
        if self.h:
            lib().rv_la_hub_destroy(self.h)
            self.h = None


class RcclComm:
    """An RCCL communicator over all ranks (rv_comm_*), bootstrapped through
    torch.distributed (gloo): rank 0's unique id is broadcast as bytes."""

    def __init__(self, group):
        import torch
        info = group.info
        idb = np.zeros(256, dtype=np.uint8)
        if info.rank == 0:
            n = lib().rv_comm_unique_id(idb.ctypes.data, idb.size)
            if n < 0:
                _check(n, "rv_comm_unique_id")
        t = torch.from_numpy(idb)
        group.dist.broadcast(t, src=0)
        idb = t.numpy().copy()
        self.h = lib().rv_comm_create(idb.ctypes.data, info.world, info.rank)
        if not self.h:
            raise RuntimeError(f"rv_comm_create: {lib().rv_last_error().decode()}")

    def close(self):
        if self.h:
            lib().rv_comm_destroy(self.h)
            self.h = None
