"""Hot-path replay: synthetic input frames and the HIP replay driver
(rv_replay_* of include/rav1e_hip.h).  See DESIGN.md "Replay driver".

The replay runs, per frame, the accelerated stages of a speed-10 rav1e
encode of one tile (coarse 1/4-res full search, 1/2-res and full-res
diamond + sub-pel search, RDO candidate MC / transforms / distortion,
8x8 importance SATD) with all frames resident in HBM.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import RvReplayCfg, _check, lib

RV_REPLAY_SIDE_RDO = 1  # include/rav1e_hip.h
RV_REPLAY_SPLIT_RDO = 2
RV_REPLAY_EXHAUSTIVE_FS = 4  # F1 without successive elimination (same results)

# GOP of the reference's reorder pyramid (src/api/internal.rs:61-95):
# group_input_len 4, levels 0,1,2,2 -> me_range_scale = 4 >> level
# (src/encoder.rs:838).
GOP_SCALES = (4, 2, 1, 1)

_LATTICE = 8


def _value_noise(xs: np.ndarray, ys: np.ndarray) -> np.ndarray:
    """Bilinear value noise on an 8-px lattice of seeded values (0x5EED)."""
    rng = np.random.default_rng(0x5EED)
    lat = rng.random((257, 257)) * 2.0 - 1.0
    gx, gy = xs / _LATTICE, ys / _LATTICE
    x0, y0 = np.floor(gx), np.floor(gy)
    fx, fy = gx - x0, gy - y0
    x0 = x0.astype(np.int64) % 256
    y0 = y0.astype(np.int64) % 256
    v00 = lat[y0, x0]
    v01 = lat[y0, x0 + 1]
    v10 = lat[y0 + 1, x0]
    v11 = lat[y0 + 1, x0 + 1]
    return (v00 * (1 - fx) + v01 * fx) * (1 - fy) + (v10 * (1 - fx) + v11 * fx) * fy


def synth_plane(w, h, t, scale_x=1, scale_y=1, amp=60.0, tex=24.0, phase=0.0, bd=8):
    x = np.arange(w, dtype=np.float64)[None, :] * scale_x
    y = np.arange(h, dtype=np.float64)[:, None] * scale_y
    xm, ym = x - 1.25 * t, y - 0.75 * t
    base = 128.0 + amp * np.sin(2 * np.pi * xm / 97.0 + phase) * np.cos(2 * np.pi * ym / 61.0)
    base = base + tex * _value_noise(np.broadcast_to(xm, (h, w)), np.broadcast_to(ym, (h, w)))
    rng = np.random.default_rng(0x5EED ^ (int(t) * 2654435761 + int(phase * 1000)))
    base = base + rng.integers(-2, 3, (h, w))
    y8 = np.clip(np.floor(base + 0.5), 0, 255).astype(np.int64)
    if bd == 8:
        return y8.astype(np.uint8)
    return (y8 * 4 + rng.integers(0, 4, (h, w))).astype(np.uint16)


def synth_frame(w, h, t, xdec=1, ydec=1, bd=8) -> np.ndarray:
    """Planar Y, U, V of synthetic frame t, concatenated."""
    cw, ch = (w + xdec) >> xdec, (h + ydec) >> ydec
    y = synth_plane(w, h, t, bd=bd)
    u = synth_plane(cw, ch, t, 1 << xdec, 1 << ydec, 30.0, 12.0, 1.3, bd)
    v = synth_plane(cw, ch, t, 1 << xdec, 1 << ydec, 30.0, 12.0, 2.6, bd)
    return np.concatenate([y.ravel(), u.ravel(), v.ravel()])


def result_words(width, height, n_refs, tile_w_sb=0, tile_h_sb=0, tile_x0=0, tile_y0=0):
    sbc, sbr = (width + 63) // 64, (height + 63) // 64
    tw = tile_w_sb or (sbc - tile_x0)
    th = tile_h_sb or (sbr - tile_y0)
    return tw * th * (8 * n_refs + 2) + 4


class HipReplay:
    """The GPU replay of one tile (rv_replay_create ... rv_replay_destroy)."""

    def __init__(self, width, height, xdec=1, ydec=1, bit_depth=8, n_refs=2, tile=None,
                 stream=None, flags=0):
        cfg = RvReplayCfg()
        cfg.width, cfg.height, cfg.xdec, cfg.ydec = width, height, xdec, ydec
        cfg.bit_depth, cfg.n_refs, cfg.rdo_candidates = bit_depth, n_refs, 2 * n_refs
        cfg.flags = flags
        if tile:
            cfg.tile_x0, cfg.tile_y0, cfg.tile_w, cfg.tile_h = tile
        self.cfg = cfg
        self.h = lib().rv_replay_create(C.byref(cfg), stream)
        if not self.h:
            raise RuntimeError(f"rv_replay_create: {lib().rv_last_error().decode()}")
        self.n_words = result_words(width, height, n_refs, cfg.tile_w, cfg.tile_h,
                                    cfg.tile_x0, cfg.tile_y0)

    def set_frame(self, slot: int, yuv: np.ndarray):
        yuv = np.ascontiguousarray(yuv)
        _check(lib().rv_replay_set_frame(self.h, slot, yuv.ctypes.data), "rv_replay_set_frame")

    def frame(self, me_range_scale: int):
        _check(lib().rv_replay_frame(self.h, me_range_scale), "rv_replay_frame")

    def results(self) -> np.ndarray:
        out = np.zeros(self.n_words, dtype=np.uint64)
        n = lib().rv_replay_results(self.h, out.ctypes.data, out.size)
        if n < 0:
            _check(n, "rv_replay_results")
        return out[:n]

    def set_timing(self, stride: int, block: int = 1):
        """Record the timing events on frames f with (f // block) % stride == 0
        (rv_replay_set_timing)."""
        _check(lib().rv_replay_set_timing(self.h, stride, block), "rv_replay_set_timing")

    def stage_ms(self) -> np.ndarray:
        out = np.zeros(10, dtype=np.float32)
        n = lib().rv_replay_stage_times(self.h, out.ctypes.data, 10)
        if n < 0:
            _check(n, "rv_replay_stage_times")
        return out[:n]

    def stage_ms_sum(self, last_frames: int) -> np.ndarray:
        out = np.zeros(10, dtype=np.float32)
        n = lib().rv_replay_stage_times_sum(self.h, last_frames, out.ctypes.data, 10)
        if n < 0:
            _check(n, "rv_replay_stage_times_sum")
        return out[:n]

    def counters(self) -> np.ndarray:
        """[F3 full-pel evals, F3 sub-pel evals, frames] over the last <= 64 frames."""
        out = np.zeros(3, dtype=np.uint64)
        _check(lib().rv_replay_counters(self.h, out.ctypes.data, 3) - 3, "rv_replay_counters")
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
