"""rav1e_amd -- MI355X (gfx950) encode hot path for rav1e, host side.

Python mirror of the reference's dispatch interface for the hot path
(geobacter-rs/rav1e): ``CpuFeatureLevel`` with a ``HIP`` level, the
``get_sad`` / ``get_satd`` / ``put_8tap`` / ``prep_8tap`` / ``mc_avg`` /
``forward_transform`` / ``inverse_transform_add`` / ``sse_wxh`` /
``cdef_dist_wxh`` entry points, plus the batched forms that are the
production path.  Everything runs through the C ABI of
``rav1e_amd/lib/librav1e_hip.so`` (``include/rav1e_hip.h``); there is no
CPU fallback: without the library this module raises on import of any
entry point, and the HIP level requires a gfx950 device.
"""
from __future__ import annotations

import ctypes as C
import enum
import os

import numpy as np

_ROOT = os.path.dirname(os.path.abspath(__file__))
# RAV1E_HIP_LIB: another in-tree build of the same library (A/B benchmarks)
LIB_PATH = os.environ.get("RAV1E_HIP_LIB") or os.path.join(_ROOT, "lib", "librav1e_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(_ROOT), "include", "rav1e_hip.h")

RV_OK, RV_EINVAL, RV_EHIP, RV_ENOTSUP = 0, -1, -2, -3


class Rav1eHipError(RuntimeError):
    pass


# ---- C structs (include/rav1e_hip.h) -----------------------------------
class RvPlane(C.Structure):
    _fields_ = [("data", C.c_void_p), ("stride", C.c_int32),
                ("alloc_height", C.c_int32), ("width", C.c_int32),
                ("height", C.c_int32), ("xorigin", C.c_int32),
                ("yorigin", C.c_int32), ("xdec", C.c_int32),
                ("ydec", C.c_int32), ("hbd", C.c_int32),
                ("bit_depth", C.c_int32)]


class RvMv(C.Structure):
    _fields_ = [("row", C.c_int16), ("col", C.c_int16)]


class RvFsResult(C.Structure):
    _fields_ = [("best_mv", RvMv), ("reserved", C.c_uint32), ("cost", C.c_uint64)]


# job layouts as numpy dtypes (arrays of these go to the device verbatim)
DIST_JOB = np.dtype([("org_x", "<i4"), ("org_y", "<i4"), ("ref_x", "<i4"), ("ref_y", "<i4")])
INTRA_JOB = np.dtype([("x", "<i4"), ("y", "<i4"), ("mode", "<i4"), ("variant", "<i4")])
MC_JOB = np.dtype([("src_x", "<i4"), ("src_y", "<i4"), ("dst_x", "<i4"), ("dst_y", "<i4"),
                   ("col_frac", "<i4"), ("row_frac", "<i4")])
MOTION_VECTOR = np.dtype([("row", "<i2"), ("col", "<i2")])  # rv_mv / MotionVector
TX_JOB = np.dtype([("src_x", "<i4"), ("src_y", "<i4"), ("pred_x", "<i4"), ("pred_y", "<i4")])
FS_JOB = np.dtype([("po_x", "<i4"), ("po_y", "<i4"), ("x_lo", "<i4"), ("x_hi", "<i4"),
                   ("y_lo", "<i4"), ("y_hi", "<i4"), ("pmv0_row", "<i2"), ("pmv0_col", "<i2"),
                   ("pmv1_row", "<i2"), ("pmv1_col", "<i2"), ("lambda_", "<u4"),
                   ("reserved", "<i4")])
DS_JOB = np.dtype([("po_x", "<i4"), ("po_y", "<i4"), ("mvx_min", "<i4"), ("mvx_max", "<i4"),
                   ("mvy_min", "<i4"), ("mvy_max", "<i4"), ("pmv0_row", "<i2"),
                   ("pmv0_col", "<i2"), ("pmv1_row", "<i2"), ("pmv1_col", "<i2"),
                   ("lambda_", "<u4"), ("n_pred", "<i4"), ("pred", "<i2", (17, 2))])
FS_RESULT = np.dtype([("mv_row", "<i2"), ("mv_col", "<i2"), ("reserved", "<u4"),
                      ("cost", "<u8")])
REPLAY_CFG_FIELDS = ["width", "height", "xdec", "ydec", "bit_depth", "tile_x0", "tile_y0",
                     "tile_w", "tile_h", "n_refs", "tile_w_sb", "tile_h_sb", "n_inputs", "flags"]


class RvReplayCfg(C.Structure):
    _fields_ = [(f, C.c_int32) for f in REPLAY_CFG_FIELDS]


class RvReplayLevelParams(C.Structure):
    _fields_ = [("base_q_idx", C.c_int32), ("dc_delta_q", C.c_int32 * 3),
                ("ac_delta_q", C.c_int32 * 3), ("cdef_strengths", C.c_int32), ("lambda_", C.c_double),
                ("me_lambda", C.c_double), ("dist_scale", C.c_double * 3)]

    @classmethod
    def from_dict(cls, d):
        p = cls()
        p.base_q_idx = d["base_q_idx"]
        for i in range(3):
            p.dc_delta_q[i], p.ac_delta_q[i] = d["dc_delta_q"][i], d["ac_delta_q"][i]
            p.dist_scale[i] = d["dist_scale"][i]
        p.lambda_, p.me_lambda = d["lambda"], d["me_lambda"]
        p.cdef_strengths = d.get("cdef_y", 0) | d.get("cdef_uv", 0) << 8
        return p


class RvReplayFrameInfo(C.Structure):
    _fields_ = [("display", C.c_int32), ("me_range_scale", C.c_int32), ("level", C.c_int32),
                ("is_key", C.c_int32), ("ref_display", C.c_int32 * 2), ("compound", C.c_int32)]


# ---- reference enums ----------------------------------------------------
class CpuFeatureLevel(enum.IntEnum):
    """src/cpu_features/x86.rs:13-19 plus the HIP level."""
    NATIVE = 0
    SSE2 = 1
    SSSE3 = 2
    AVX2 = 3
    HIP = 4

    @staticmethod
    def default() -> "CpuFeatureLevel":
        """CpuFeatureLevel::default() with RAV1E_CPU_TARGET (x86.rs:34-61)."""
        return CpuFeatureLevel(lib().rv_cpu_feature_level_default())

    def as_index(self) -> int:
        return int(self)


class BlockSize(enum.IntEnum):
    """src/partition.rs:116-140 (order = table index)."""
    BLOCK_4X4 = 0
    BLOCK_4X8 = 1
    BLOCK_8X4 = 2
    BLOCK_8X8 = 3
    BLOCK_8X16 = 4
    BLOCK_16X8 = 5
    BLOCK_16X16 = 6
    BLOCK_16X32 = 7
    BLOCK_32X16 = 8
    BLOCK_32X32 = 9
    BLOCK_32X64 = 10
    BLOCK_64X32 = 11
    BLOCK_64X64 = 12
    BLOCK_64X128 = 13
    BLOCK_128X64 = 14
    BLOCK_128X128 = 15
    BLOCK_4X16 = 16
    BLOCK_16X4 = 17
    BLOCK_8X32 = 18
    BLOCK_32X8 = 19
    BLOCK_16X64 = 20
    BLOCK_64X16 = 21

    def width(self) -> int:
        return int(self.name.split("_")[1].split("X")[0])

    def height(self) -> int:
        return int(self.name.split("X")[-1])

    @staticmethod
    def from_width_and_height(w: int, h: int) -> "BlockSize":
        return BlockSize[f"BLOCK_{w}X{h}"]


class TxSize(enum.IntEnum):
    """src/transform/mod.rs:225-247."""
    TX_4X4 = 0
    TX_8X8 = 1
    TX_16X16 = 2
    TX_32X32 = 3
    TX_64X64 = 4
    TX_4X8 = 5
    TX_8X4 = 6
    TX_8X16 = 7
    TX_16X8 = 8
    TX_16X32 = 9
    TX_32X16 = 10
    TX_32X64 = 11
    TX_64X32 = 12
    TX_4X16 = 13
    TX_16X4 = 14
    TX_8X32 = 15
    TX_32X8 = 16
    TX_16X64 = 17
    TX_64X16 = 18

    def width(self) -> int:
        return int(self.name.split("_")[1].split("X")[0])

    def height(self) -> int:
        return int(self.name.split("X")[-1])


class TxType(enum.IntEnum):
    """src/transform/mod.rs:123-140."""
    DCT_DCT = 0
    ADST_DCT = 1
    DCT_ADST = 2
    ADST_ADST = 3
    FLIPADST_DCT = 4
    DCT_FLIPADST = 5
    FLIPADST_FLIPADST = 6
    ADST_FLIPADST = 7
    FLIPADST_ADST = 8
    IDTX = 9
    V_DCT = 10
    H_DCT = 11
    V_ADST = 12
    H_ADST = 13
    V_FLIPADST = 14
    H_FLIPADST = 15


class FilterMode(enum.IntEnum):
    """src/mc.rs:58-66."""
    REGULAR = 0
    SMOOTH = 1
    SHARP = 2
    BILINEAR = 3


# ---- library loading ------------------------------------------------------
_lib = None


def _declare(L):
    vp, i32, sz = C.c_void_p, C.c_int, C.c_size_t
    P = C.POINTER(RvPlane)
    sig = {
        "rv_cpu_feature_level_default": (i32, []),
        "rv_cpu_feature_level_index": (i32, [i32]),
        "rv_device_count": (i32, []),
        "rv_set_device": (i32, [i32]),
        "rv_last_error": (C.c_char_p, []),
        "rv_version": (C.c_char_p, []),
        "rv_malloc": (vp, [sz]),
        "rv_free": (None, [vp]),
        "rv_host_alloc": (vp, [sz]),
        "rv_host_free": (None, [vp]),
        "rv_memcpy_h2d": (i32, [vp, vp, sz, vp]),
        "rv_memcpy_d2h": (i32, [vp, vp, sz, vp]),
        "rv_memcpy_d2d": (i32, [vp, vp, sz, vp]),
        "rv_memset": (i32, [vp, i32, sz, vp]),
        "rv_stream_create": (vp, []),
        "rv_stream_create_priority": (vp, [i32]),
        "rv_stream_destroy": (i32, [vp]),
        "rv_stream_sync": (i32, [vp]),
        "rv_device_sync": (i32, []),
        "rv_trace_marker": (i32, [vp]),
        "rv_event_create": (vp, []),
        "rv_event_destroy": (i32, [vp]),
        "rv_event_record": (i32, [vp, vp]),
        "rv_event_sync": (i32, [vp]),
        "rv_stream_wait_event": (i32, [vp, vp]),
        "rv_event_elapsed_ms": (C.c_float, [vp, vp]),
        "rv_plane_geometry": (sz, [P, i32, i32, i32, i32, i32, i32, i32]),
        "rv_plane_pad": (i32, [P, vp]),
        "rv_plane_downsample": (i32, [P, P, vp]),
        "rv_sad_batch": (i32, [P, P, vp, i32, i32, i32, vp, vp]),
        "rv_satd_batch": (i32, [P, P, vp, i32, i32, i32, vp, vp]),
        "rv_sse_batch": (i32, [P, P, vp, i32, i32, i32, vp, vp]),
        "rv_lookahead_intra_costs": (i32, [P, i32, vp, vp]),
        "rv_propagate_importances_scratch": (sz, [i32, i32]),
        "rv_propagate_importances": (i32, [P, P, vp, vp, vp, i32, vp, vp, sz, vp]),
        "rv_cdef_moments_batch": (i32, [P, P, vp, i32, i32, i32, vp, vp]),
        "rv_put_8tap_batch": (i32, [P, P, vp, i32, i32, i32, i32, i32, i32, vp]),
        "rv_predict_intra_batch": (i32, [P, vp, vp, i32, i32, i32, vp]),
        "rv_deblock_plane": (i32, [P, i32, i32, i32, vp, vp, i32, vp, i32, vp]),
        "rv_deblock_fast_level": (i32, [i32, i32, i32]),
        "rv_deblock_sse": (i32, [P, P, i32, i32, vp, vp, i32, vp, vp, i32, vp]),
        "rv_deblock_frame": (i32, [P, i32, i32, vp, vp, i32, vp, i32, vp]),
        "rv_cdef_find_dirs": (i32, [P, i32, i32, vp, i32, vp, vp, i32, vp]),
        "rv_lrf_stripe_filter": (i32, [P, P] + [i32] * 10 + [vp, vp]),
        "rv_y4m_parse_header": (i32, [C.c_char_p, vp]),
        "rv_y4m_open": (vp, [C.c_char_p]),
        "rv_y4m_get_info": (i32, [vp, vp]),
        "rv_y4m_frame_bytes": (sz, [vp]),
        "rv_y4m_read_frame": (i32, [vp, vp]),
        "rv_y4m_close": (None, [vp]),
        "rv_ivf_create": (vp, [C.c_char_p, i32, i32, i32, i32]),
        "rv_ivf_write_frame": (i32, [vp, C.c_uint64, vp, sz]),
        "rv_ivf_close": (i32, [vp]),
        "rv_cdef_filter_plane": (i32, [P, P, i32, i32, i32, vp, i32, vp, vp, vp, vp, vp, i32, i32,
                                       vp]),
        "rv_prep_8tap_batch": (i32, [vp, P, vp, i32, i32, i32, i32, i32, i32, vp]),
        "rv_mc_avg_batch": (i32, [P, vp, vp, vp, i32, i32, i32, i32, vp]),
        "rv_mc_dist_batch": (i32, [P, P, vp, i32, i32, i32, i32, i32, i32, i32, vp, vp]),
        "rv_fwd_txfm_batch": (i32, [vp, vp, i32, i32, i32, i32, vp]),
        "rv_diff_fwd_txfm_batch": (i32, [P, P, vp, i32, i32, i32, i32, vp, vp]),
        "rv_inv_txfm_add_batch": (i32, [vp, P, vp, i32, i32, i32, i32, vp]),
        "rv_quantize_batch": (i32, [vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp,
                                    vp]),
        "rv_dequantize_batch": (i32, [vp, i32, i32, i32, i32, i32, i32, vp, vp]),
        "rv_estimate_rate_batch": (i32, [vp, i32, i32, i32, vp, vp]),
        "rv_full_search_batch": (i32, [P, P, vp, i32, i32, i32, i32, i32, vp, vp]),
        "rv_full_search_sea_batch": (i32, [P, P, vp, vp, i32, i32, vp, vp]),
        "rv_plane_box_sums": (i32, [P, vp, vp]),
        "rv_replay_create": (vp, [C.POINTER(RvReplayCfg), vp]),
        "rv_replay_create_twin": (vp, [vp, vp]),
        "rv_replay_seek": (i32, [vp, C.c_long]),
        "rv_replay_stream": (vp, [vp]),
        "rv_replay_destroy": (None, [vp]),
        "rv_q_lookup": (i32, [i32, i32, i32]),
        "rv_replay_synth_inputs": (i32, [vp, i32]),
        "rv_replay_set_level_params": (i32, [vp, i32, C.POINTER(RvReplayLevelParams)]),
        "rv_replay_set_input": (i32, [vp, i32, vp]),
        "rv_replay_get_input": (i32, [vp, i32, vp]),
        "rv_replay_get_recon": (i32, [vp, i32, vp]),
        "rv_replay_set_importances": (i32, [vp, vp, i32]),
        "rv_replay_set_imp_window": (i32, [vp, i32, C.c_long]),
        "rv_replay_set_inputs_ready": (i32, [vp, C.c_long]),
        "rv_replay_get_importances": (i32, [vp, vp, i32]),
        "rv_replay_frame": (i32, [vp, C.POINTER(RvReplayFrameInfo)]),
        "rv_replay_set_groups": (i32, [vp, i32, vp, i32, vp]),
        "rv_replay_exchange_buffers": (i32, [vp, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                             C.POINTER(C.c_size_t)]),
        "rv_replay_import": (i32, [vp]),
        "rv_comm_unique_id": (i32, [vp, i32]),
        "rv_comm_create": (vp, [vp, i32, i32]),
        "rv_comm_destroy": (None, [vp]),
        "rv_replay_results": (i32, [vp, vp, i32]),
        "rv_replay_entropy_stats": (i32, [vp, vp, i32]),
        "rv_replay_stage_times": (i32, [vp, vp, i32]),
        "rv_replay_stage_times_sum": (i32, [vp, i32, vp, i32]),
        "rv_replay_counters": (i32, [vp, vp, i32]),
        "rv_replay_dpb_slots": (i32, []),
        "rv_replay_set_kernel_probe": (i32, [vp, i32]),
        "rv_replay_kernel_probe": (i32, [vp, vp, i32]),
        "rv_round_ring_slots": (i32, [C.c_uint32, vp, i32]),
        "rv_replay_lrf_units": (i32, [vp, i32, vp, i32]),
        "rv_replay_la_refs": (i32, [C.c_long, i32, vp]),
        "rv_la_hub_create": (vp, [i32]),
        "rv_la_hub_destroy": (None, [vp]),
        "rv_replay_set_la_exchange": (i32, [vp, vp, vp]),
        "rv_replay_set_timing": (i32, [vp, i32, i32]),
        "rv_diamond_search_batch": (i32, [P, P, vp, i32, i32, i32, i32, i32, i32, i32, vp, vp]),
        "rv_telescopic_subpel_batch": (i32, [P, P, vp, vp, i32, i32, i32, i32, i32, i32, vp, vp]),
        "rv_tx_dist_batch": (i32, [vp, i32, vp, i32, i32, vp, vp]),
        "rav1e_fwd_txfm_hip": (i32, [vp, vp, i32, i32, i32]),
        "rav1e_inv_txfm_add_hip": (i32, [vp, vp, C.c_ssize_t, i32, i32, i32]),
        "rv_ec_scratch_bytes": (C.c_size_t, [i32]),
        "rv_ec_tokenize": (i32, [vp, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, C.c_uint32, vp,
                                 vp]),
        "rv_ec_code_tokens": (C.c_long, [vp, C.c_size_t, vp, vp, C.c_size_t]),
        "rv_ec_cdf_total": (i32, []),
        "rv_ec_default_cdf": (i32, [i32, vp]),
        "rv_ec_reset_counts": (None, [vp]),
        "rv_sad_fn": (vp, [i32, i32, i32]),
        "rv_satd_fn": (vp, [i32, i32, i32]),
        "rv_put_fn_get": (vp, [i32, i32, i32]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args


def lib():
    """Load the HIP library; raises if it was not built (no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise Rav1eHipError(
                f"{LIB_PATH} missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
        L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        _declare(L)
        _lib = L
    return _lib


def _check(rc, what):
    if rc != RV_OK:
        raise Rav1eHipError(f"{what} failed ({rc}): {lib().rv_last_error().decode()}")


def require_device(device: int = 0):
    """Fail loudly unless a gfx950 device is visible."""
    L = lib()
    if L.rv_device_count() <= device:
        raise Rav1eHipError("no HIP device visible: the HIP level needs a gfx950 GPU")
    _check(L.rv_set_device(device), "rv_set_device")


# ---- device memory --------------------------------------------------------
class DeviceBuffer:
    """Device allocation owned by Python (rv_malloc / rv_free)."""

    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        self.ptr = lib().rv_malloc(max(1, self.nbytes))
        if not self.ptr:
            raise Rav1eHipError(f"rv_malloc({nbytes}): {lib().rv_last_error().decode()}")

    @classmethod
    def from_array(cls, a: np.ndarray) -> "DeviceBuffer":
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes)
        b.upload(a)
        return b

    def upload(self, a: np.ndarray, stream=None):
        a = np.ascontiguousarray(a)
        assert a.nbytes <= self.nbytes
        if a.nbytes:
            _check(lib().rv_memcpy_h2d(self.ptr, a.ctypes.data, a.nbytes, stream), "rv_memcpy_h2d")

    def download(self, dtype, count=None, stream=None) -> np.ndarray:
        dt = np.dtype(dtype)
        n = self.nbytes // dt.itemsize if count is None else int(count)
        out = np.empty(n, dtype=dt)
        if out.nbytes:
            _check(lib().rv_memcpy_d2h(out.ctypes.data, self.ptr, out.nbytes, stream),
                   "rv_memcpy_d2h")
        return out

    def zero(self, stream=None):
        _check(lib().rv_memset(self.ptr, 0, self.nbytes, stream), "rv_memset")
        _check(lib().rv_stream_sync(stream), "rv_stream_sync")

    def free(self):
        if self.ptr:
            lib().rv_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class DevicePlane:
    """A padded plane in HBM with the reference's PlaneConfig geometry
    (Plane::new, src/frame/plane.rs:215-244)."""

    def __init__(self, width, height, xdec=0, ydec=0, xpad=0, ypad=0, hbd=False,
                 bit_depth=None):
        self.desc = RvPlane()
        nbytes = lib().rv_plane_geometry(C.byref(self.desc), width, height, xdec, ydec,
                                         xpad, ypad, 1 if hbd else 0)
        if bit_depth is not None:
            self.desc.bit_depth = int(bit_depth)
        self.buf = DeviceBuffer(nbytes)
        self.desc.data = self.buf.ptr
        self.dtype = np.uint16 if hbd else np.uint8

    @classmethod
    def from_array(cls, a: np.ndarray, xpad=0, ypad=0, xdec=0, ydec=0, pad=True,
                   bit_depth=None):
        p = cls(a.shape[1], a.shape[0], xdec, ydec, xpad, ypad, a.dtype == np.uint16,
                bit_depth)
        p.upload_visible(a, pad=pad)
        return p

    @classmethod
    def from_full(cls, full: np.ndarray, xorigin, yorigin, width, height, bit_depth=None):
        """Wrap a whole padded allocation (stride = full.shape[1])."""
        p = cls.__new__(cls)
        p.desc = RvPlane()
        p.desc.stride, p.desc.alloc_height = full.shape[1], full.shape[0]
        p.desc.width, p.desc.height = width, height
        p.desc.xorigin, p.desc.yorigin = xorigin, yorigin
        p.desc.hbd = 1 if full.dtype == np.uint16 else 0
        p.desc.bit_depth = bit_depth if bit_depth is not None else (0 if p.desc.hbd else 8)
        p.buf = DeviceBuffer.from_array(full)
        p.desc.data = p.buf.ptr
        p.dtype = full.dtype
        return p

    @property
    def shape_full(self):
        return (self.desc.alloc_height, self.desc.stride)

    def upload_visible(self, a: np.ndarray, pad=True):
        full = np.zeros(self.shape_full, dtype=self.dtype)
        d = self.desc
        full[d.yorigin:d.yorigin + d.height, d.xorigin:d.xorigin + d.width] = a
        self.buf.upload(full)
        if pad:
            _check(lib().rv_plane_pad(C.byref(self.desc), None), "rv_plane_pad")
            _check(lib().rv_stream_sync(None), "rv_stream_sync")

    def download_full(self) -> np.ndarray:
        return self.buf.download(self.dtype).reshape(self.shape_full)

    def download_visible(self) -> np.ndarray:
        d = self.desc
        return self.download_full()[d.yorigin:d.yorigin + d.height,
                                    d.xorigin:d.xorigin + d.width].copy()


def _sync(stream=None):
    _check(lib().rv_stream_sync(stream), "rv_stream_sync")


# ---- batched entry points (production path) -------------------------------
def sad_batch(org: DevicePlane, ref: DevicePlane, jobs: np.ndarray, w: int, h: int,
              satd: bool = False) -> np.ndarray:
    jobs = np.ascontiguousarray(jobs, dtype=DIST_JOB)
    dj = DeviceBuffer.from_array(jobs)
    out = DeviceBuffer(4 * len(jobs))
    f = lib().rv_satd_batch if satd else lib().rv_sad_batch
    _check(f(C.byref(org.desc), C.byref(ref.desc), dj.ptr, len(jobs), w, h, out.ptr, None),
           "rv_satd_batch" if satd else "rv_sad_batch")
    _sync()
    return out.download(np.uint32)


def satd_batch(org, ref, jobs, w, h) -> np.ndarray:
    return sad_batch(org, ref, jobs, w, h, satd=True)


def lookahead_intra_costs(plane: DevicePlane, bit_depth: int = 8) -> np.ndarray:
    """compute_lookahead_intra_costs (src/api/internal.rs:680-765) of a luma
    plane: u32 [ceil(h / 8), ceil(w / 8)]."""
    nbx, nby = (plane.desc.width + 7) // 8, (plane.desc.height + 7) // 8
    out = DeviceBuffer(4 * nbx * nby)
    _check(lib().rv_lookahead_intra_costs(C.byref(plane.desc), int(bit_depth), out.ptr, None),
           "rv_lookahead_intra_costs")
    _sync()
    return out.download(np.uint32, nbx * nby).reshape(nby, nbx)


def propagate_importances(org: DevicePlane, ref: DevicePlane, mvs: np.ndarray,
                          intra_costs: np.ndarray, importances: np.ndarray, n_unique: int,
                          ref_importances: np.ndarray) -> np.ndarray:
    """compute_block_importances' propagation (src/api/internal.rs:823-1010)
    for one (frame, reference) pass: mvs [h_imp, w_imp] MOTION_VECTOR,
    intra_costs u32, importances f32 of the frame; returns the reference's
    f32 importances after the pass (ref_importances is the value before)."""
    nbx, nby = (org.desc.width + 7) // 8, (org.desc.height + 7) // 8
    mv = np.ascontiguousarray(mvs, dtype=MOTION_VECTOR).reshape(nby * nbx)
    dm = DeviceBuffer.from_array(mv)
    di = DeviceBuffer.from_array(np.ascontiguousarray(intra_costs, dtype=np.uint32).ravel())
    dp = DeviceBuffer.from_array(np.ascontiguousarray(importances, dtype=np.float32).ravel())
    dr = DeviceBuffer.from_array(np.ascontiguousarray(ref_importances, dtype=np.float32).ravel())
    nbytes = lib().rv_propagate_importances_scratch(nbx, nby)
    ds = DeviceBuffer(max(1, nbytes))
    _check(lib().rv_propagate_importances(C.byref(org.desc), C.byref(ref.desc), dm.ptr, di.ptr,
                                          dp.ptr, int(n_unique), dr.ptr, ds.ptr, nbytes, None),
           "rv_propagate_importances")
    _sync()
    return dr.download(np.float32, nbx * nby).reshape(nby, nbx)


def sse_batch(org, ref, jobs, w, h) -> np.ndarray:
    jobs = np.ascontiguousarray(jobs, dtype=DIST_JOB)
    bw = min(w, 8) >> org.desc.xdec
    bh = min(h, 8) >> org.desc.ydec
    nsub = (w // bw) * (h // bh)
    dj = DeviceBuffer.from_array(jobs)
    out = DeviceBuffer(8 * nsub * max(1, len(jobs)))
    _check(lib().rv_sse_batch(C.byref(org.desc), C.byref(ref.desc), dj.ptr, len(jobs), w, h,
                              out.ptr, None), "rv_sse_batch")
    _sync()
    return out.download(np.uint64, nsub * len(jobs)).reshape(len(jobs), nsub)


def cdef_moments_batch(org, ref, jobs, w, h) -> np.ndarray:
    jobs = np.ascontiguousarray(jobs, dtype=DIST_JOB)
    nsub = (w // 8) * (h // 8)
    dj = DeviceBuffer.from_array(jobs)
    out = DeviceBuffer(40 * nsub * max(1, len(jobs)))
    _check(lib().rv_cdef_moments_batch(C.byref(org.desc), C.byref(ref.desc), dj.ptr, len(jobs),
                                       w, h, out.ptr, None), "rv_cdef_moments_batch")
    _sync()
    return out.download(np.int64, 5 * nsub * len(jobs)).reshape(len(jobs), nsub, 5)


def put_8tap_batch(dst: DevicePlane, src: DevicePlane, jobs, w, h, mode_x=0, mode_y=0,
                   bit_depth=8):
    jobs = np.ascontiguousarray(jobs, dtype=MC_JOB)
    dj = DeviceBuffer.from_array(jobs)
    _check(lib().rv_put_8tap_batch(C.byref(dst.desc), C.byref(src.desc), dj.ptr, len(jobs), w, h,
                                   mode_x, mode_y, bit_depth, None), "rv_put_8tap_batch")
    _sync()


class PredictionMode(enum.IntEnum):
    """src/predict.rs:135-166 (the intra modes)."""
    DC_PRED = 0
    V_PRED = 1
    H_PRED = 2
    D45_PRED = 3
    D135_PRED = 4
    D117_PRED = 5
    D153_PRED = 6
    D207_PRED = 7
    D63_PRED = 8
    SMOOTH_PRED = 9
    SMOOTH_V_PRED = 10
    SMOOTH_H_PRED = 11
    PAETH_PRED = 12


# RAV1E_INTRA_MODES (src/predict.rs:32-46): the screening order
RAV1E_INTRA_MODES = [0, 2, 1, 9, 11, 10, 12, 3, 4, 5, 6, 7, 8]
EDGE_PX = 4 * 64 + 1  # edge_buf: 4 * MAX_TX_SIZE + 1


def predict_intra_batch(dst: DevicePlane, jobs, edges: np.ndarray, tx_size, bit_depth=8):
    """PredictionMode::predict_intra (no CfL) of every job into dst; edges
    (n, 257) in rav1e's edge_buf layout (src/predict.rs:545-551)."""
    jobs = np.ascontiguousarray(jobs, dtype=INTRA_JOB)
    edges = np.ascontiguousarray(edges, dtype=np.uint16 if bit_depth > 8 else np.uint8)
    if edges.shape != (len(jobs), EDGE_PX):
        raise Rav1eHipError("predict_intra_batch: edges must be (n_jobs, 257)")
    if not (0 <= jobs["mode"]).all() or not (jobs["mode"] <= 12).all():
        raise Rav1eHipError("predict_intra_batch: CfL / inter modes are not intra predictions here")
    dj = DeviceBuffer.from_array(jobs)
    de = DeviceBuffer.from_array(edges)
    _check(lib().rv_predict_intra_batch(C.byref(dst.desc), dj.ptr, de.ptr, len(jobs), tx_size,
                                        bit_depth, None), "rv_predict_intra_batch")
    _sync()


def deblock_plane(plane: DevicePlane, pli, width, height, lg: np.ndarray, skip: np.ndarray,
                  levels, bit_depth=8):
    """deblock_plane (src/deblock.rs:1174-1335) of plane pli of a width x
    height frame, in place.  lg / skip: (rows, cols) per luma 4x4 block
    (log2 of the square block's width in 4x4 units, skip flag); levels =
    [Y vertical, Y horizontal, U, V]."""
    lg = np.ascontiguousarray(lg, dtype=np.uint8)
    skip = np.ascontiguousarray(skip, dtype=np.uint8)
    if lg.shape != skip.shape or lg.shape[1] < (width + 3) // 4 or lg.shape[0] < (height + 3) // 4:
        raise Rav1eHipError("deblock_plane: lg / skip must cover the frame's 4x4 grid")
    if not (lg <= 4).all():
        raise Rav1eHipError("deblock_plane: block sizes 4x4 .. 64x64 (lg 0 .. 4)")
    dl, ds = DeviceBuffer.from_array(lg), DeviceBuffer.from_array(skip)
    lv = np.ascontiguousarray(np.asarray(levels, dtype=np.uint8))
    _check(lib().rv_deblock_plane(C.byref(plane.desc), pli, width, height, dl.ptr, ds.ptr,
                                  lg.shape[1], lv.ctypes.data, bit_depth, None), "rv_deblock_plane")
    _sync()


def _map_buffers(width, height, lg, skip, who):
    lg = np.ascontiguousarray(lg, dtype=np.uint8)
    skip = np.ascontiguousarray(skip, dtype=np.uint8)
    if lg.shape != skip.shape or lg.shape[1] < (width + 3) // 4 or lg.shape[0] < (height + 3) // 4:
        raise Rav1eHipError(who + ": lg / skip must cover the frame's 4x4 grid")
    if not (lg <= 4).all():
        raise Rav1eHipError(who + ": block sizes 4x4 .. 64x64 (lg 0 .. 4)")
    return lg, DeviceBuffer.from_array(lg), DeviceBuffer.from_array(skip)


def deblock_sse(rec, src, width, height, lg: np.ndarray, skip: np.ndarray, bit_depth=8):
    """sse_optimize (src/deblock.rs:1418-1475) of a frame: rec / src = three
    DevicePlanes each (Y U V).  Returns (tallies (3, 2, 65) int64: vertical,
    horizontal per plane; levels [Y vertical, Y horizontal, U, V])."""
    lg, dl, ds = _map_buffers(width, height, lg, skip, "deblock_sse")
    rp = (RvPlane * 3)(*(p.desc for p in rec))
    sp = (RvPlane * 3)(*(p.desc for p in src))
    dt = DeviceBuffer(3 * 130 * 8)
    dv = DeviceBuffer(4)
    _check(lib().rv_deblock_sse(rp, sp, width, height, dl.ptr, ds.ptr, lg.shape[1], dt.ptr, dv.ptr,
                                bit_depth, None), "rv_deblock_sse")
    _sync()
    return (dt.download(np.int64, 390).reshape(3, 2, 65),
            [int(v) for v in dv.download(np.uint8, 4)])


def deblock_frame(planes, width, height, lg: np.ndarray, skip: np.ndarray, levels, bit_depth=8):
    """deblock_filter_frame (src/deblock.rs:1410-1416) of three DevicePlanes
    with the levels passed through device memory (rv_deblock_frame)."""
    lg, dl, ds = _map_buffers(width, height, lg, skip, "deblock_frame")
    pp = (RvPlane * 3)(*(p.desc for p in planes))
    dv = DeviceBuffer.from_array(np.ascontiguousarray(np.asarray(levels, dtype=np.uint8)))
    _check(lib().rv_deblock_frame(pp, width, height, dl.ptr, ds.ptr, lg.shape[1], dv.ptr,
                                  bit_depth, None), "rv_deblock_frame")
    _sync()


def deblock_fast_level(ac_q, bit_depth, is_key=False):
    return int(lib().rv_deblock_fast_level(int(ac_q), bit_depth, 1 if is_key else 0))


def cdef_filter_frame(src, dst, width, height, skip: np.ndarray, cdef_index: np.ndarray,
                      y_strengths, uv_strengths, damping=3, bit_depth=8, stream=None):
    """cdef_filter_frame (src/cdef.rs:542-641) of a frame: src / dst = three
    DevicePlanes each (Y, U, V; distinct), skip per luma 4x4 block (rows,
    cols >= 2 * ceil(width / 8)), cdef_index per 64x64 superblock, the
    FrameInvariants strength tables and damping.  Returns (dir, var) per
    8x8 luma block (cdef_analyze_superblock)."""
    cols8, rows8 = (width + 7) // 8, (height + 7) // 8
    skip = np.ascontiguousarray(skip, dtype=np.uint8)
    cdef_index = np.ascontiguousarray(cdef_index, dtype=np.uint8)
    if skip.shape[1] < 2 * cols8 or skip.shape[0] < 2 * rows8:
        raise Rav1eHipError("cdef_filter_frame: skip must cover the frame's 8x8 grid")
    if cdef_index.shape[0] < (height + 63) // 64 or cdef_index.shape[1] != (width + 63) // 64:
        raise Rav1eHipError("cdef_filter_frame: cdef_index is per 64x64 superblock")
    if cdef_index.max(initial=0) > 7:
        raise Rav1eHipError("cdef_filter_frame: cdef_index above 7")
    ds, di = DeviceBuffer.from_array(skip), DeviceBuffer.from_array(cdef_index)
    dd, dv = DeviceBuffer(cols8 * rows8), DeviceBuffer(4 * cols8 * rows8)
    ys = np.ascontiguousarray(np.asarray(y_strengths, dtype=np.uint8))
    us = np.ascontiguousarray(np.asarray(uv_strengths, dtype=np.uint8))
    if ys.shape != (8,) or us.shape != (8,):
        raise Rav1eHipError("cdef_filter_frame: 8 strengths per table")
    _check(lib().rv_cdef_find_dirs(C.byref(src[0].desc), width, height, ds.ptr, skip.shape[1],
                                   dd.ptr, dv.ptr, bit_depth, stream), "rv_cdef_find_dirs")
    for pli in range(3):
        _check(lib().rv_cdef_filter_plane(C.byref(src[pli].desc), C.byref(dst[pli].desc), pli,
                                          width, height, ds.ptr, skip.shape[1], dd.ptr, dv.ptr,
                                          di.ptr, ys.ctypes.data, us.ctypes.data, damping,
                                          bit_depth, stream), "rv_cdef_filter_plane")
    _sync(stream)
    return (dd.download(np.uint8).reshape(rows8, cols8),
            dv.download(np.int32).reshape(rows8, cols8))


def lrf_stripe_filter(cd, db, x0, y0, sw, sh, cw, ch, set_, xqd, bit_depth=8, stream=None):
    """One stripe through the device's loop-restoration filter code
    (lrf_filter_frame's chunk body): setup_integral_image's view of the
    sw x sh stripe at (x0, y0) of a cw x ch crop of DevicePlanes cd (the
    CDEF output) / db (the deblocked frame, outside the stripe's rows), then
    sgrproj_stripe_filter (src/lrf.rs:677-760) with set `set_` and xqd.
    Returns the restored stripe (sh x sw)."""
    hbd = cd.desc.hbd
    out = DeviceBuffer(sw * sh * (2 if hbd else 1))
    _check(lib().rv_lrf_stripe_filter(C.byref(cd.desc), C.byref(db.desc), x0, y0, sw, sh, cw, ch,
                                      set_, int(xqd[0]), int(xqd[1]), bit_depth, out.ptr, stream),
           "rv_lrf_stripe_filter")
    _sync(stream)
    return out.download(np.uint16 if hbd else np.uint8).reshape(sh, sw)


# ---- stream containers: y4m input, IVF output (rv_container.hip) -----------
class Y4mInfo(C.Structure):
    _fields_ = [(n, C.c_int) for n in ("width", "height", "bit_depth", "xdec", "ydec", "fps_num",
                                       "fps_den")]


class Y4mReader:
    """A y4m stream (the input rav1e's CLI reads, src/bin/decoder/y4m.rs):
    `info` (width, height, bit depth, chroma decimation, frame rate) and
    read_frame() -> the frame's packed planar samples (Y, U, V; the layout
    HipReplay.set_input takes), or None at the end of the stream."""

    def __init__(self, path):
        self.h = lib().rv_y4m_open(os.fsencode(path))
        if not self.h:
            raise Rav1eHipError(f"rv_y4m_open failed: {lib().rv_last_error().decode()}")
        self.info = Y4mInfo()
        _check(lib().rv_y4m_get_info(self.h, C.byref(self.info)), "rv_y4m_get_info")
        self.nbytes = int(lib().rv_y4m_frame_bytes(self.h))

    def read_frame(self):
        hbd = self.info.bit_depth > 8
        out = np.empty(self.nbytes // (2 if hbd else 1), np.uint16 if hbd else np.uint8)
        rc = lib().rv_y4m_read_frame(self.h, out.ctypes.data)
        if rc == 1:
            return None
        _check(rc, "rv_y4m_read_frame")
        return out

    def close(self):
        if self.h:
            lib().rv_y4m_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class IvfWriter:
    """An IVF file (ivf/src/lib.rs write_ivf_header / write_ivf_frame)."""

    def __init__(self, path, width, height, fps_num=30, fps_den=1):
        self.h = lib().rv_ivf_create(os.fsencode(path), width, height, fps_num, fps_den)
        if not self.h:
            raise Rav1eHipError(f"rv_ivf_create failed: {lib().rv_last_error().decode()}")

    def write_frame(self, pts, data: bytes):
        buf = np.frombuffer(bytes(data), np.uint8)
        _check(lib().rv_ivf_write_frame(self.h, int(pts), buf.ctypes.data if len(buf) else None,
                                        len(buf)), "rv_ivf_write_frame")

    def close(self):
        if self.h:
            _check(lib().rv_ivf_close(self.h), "rv_ivf_close")
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


# ---- entropy coding (src/ec.rs, src/context.rs write_coeffs_lv_map) --------
EC_JOB = np.dtype({"names": ["kind", "plane", "bx", "by", "tx_size", "tx_type", "is_inter",
                             "bw_lg", "bh_lg", "tile", "coeffs"],
                   "formats": [np.int32] * 10 + [np.uint64],
                   "offsets": [4 * i for i in range(10)] + [40], "itemsize": 48})


def ec_default_cdf(qctx):
    """CDFContext::new's coefficient CDFs for q context qctx (flat u16)."""
    out = np.zeros(lib().rv_ec_cdf_total(), np.uint16)
    _check(lib().rv_ec_default_cdf(qctx, out.ctypes.data), "rv_ec_default_cdf")
    return out


def ec_code_tokens(tokens, cdf):
    """One tile's tokens through the host range coder; cdf adapts in place."""
    tokens = np.ascontiguousarray(tokens, np.uint32)
    out = np.zeros(tokens.size // 2 + 4096, np.uint8)  # > 2 bytes per token never happens
    c2 = cdf.copy()
    n = lib().rv_ec_code_tokens(tokens.ctypes.data, tokens.size, c2.ctypes.data, out.ctypes.data,
                                out.size)
    if n < 0:
        _check(int(n), "rv_ec_code_tokens")
    if n > out.size:
        out = np.zeros(n, np.uint8)
        c2 = cdf.copy()
        lib().rv_ec_code_tokens(tokens.ctypes.data, tokens.size, c2.ctypes.data, out.ctypes.data,
                                out.size)
    cdf[:] = c2
    return out[:n]


def code_coefficients(jobs, coeffs, cdf_init, xdec, ydec):
    """A coding-order job sequence (rows kind, plane, bx, by, tx_size, tx_type,
    is_inter, bw_lg, bh_lg, coeff_off; kind 3 starts a tile) through the
    device tokenizer and the host range coder: write_coeffs_lv_map of every
    transform block, reset_skip_context / reset_left_contexts between them.
    Returns (bytes of all tiles, bytes per tile, the last tile's final CDFs,
    tokens)."""
    jobs = np.asarray(jobs, np.int64)
    n = len(jobs)
    co = DeviceBuffer.from_array(np.ascontiguousarray(coeffs, np.int32))
    ej = np.zeros(n, EC_JOB)
    for k, f in enumerate(["kind", "plane", "bx", "by", "tx_size", "tx_type", "is_inter",
                           "bw_lg", "bh_lg"]):
        ej[f] = jobs[:, k]
    starts = np.nonzero(jobs[:, 0] == 3)[0]
    if len(starts) == 0 or starts[0] != 0:
        starts = np.concatenate([[0], starts])
    tile = np.cumsum(jobs[:, 0] == 3) - 1
    ej["tile"] = np.maximum(tile, 0)
    ej["coeffs"] = co.ptr + 4 * jobs[:, 9].astype(np.uint64)
    ntiles = len(starts)
    ext = np.where(jobs[:, 0] == 0, 1 << jobs[:, 4], np.where(jobs[:, 0] == 1, 1 << np.maximum(jobs[:, 7] - 2, 0), 0))
    mw = int(max(1, (jobs[:, 2] + ext).max()))
    mh = int(max(1, (jobs[:, 3] + ext).max()))
    dj = DeviceBuffer.from_array(ej)
    dmap = DeviceBuffer(ntiles * 3 * mw * mh)
    scr = DeviceBuffer(lib().rv_ec_scratch_bytes(n))
    doff = DeviceBuffer(4 * (n + 1))
    cap = int(64 * n + 8 * int(np.asarray(coeffs).size) + 1024)
    dtok = DeviceBuffer(4 * cap)
    dst = DeviceBuffer(8)
    _check(lib().rv_ec_tokenize(dj.ptr, n, xdec, ydec, ntiles, mw, mh, dmap.ptr, scr.ptr, doff.ptr,
                                dtok.ptr, cap, dst.ptr, None), "rv_ec_tokenize")
    _sync(None)
    status = dst.download(np.uint32)
    if status[1]:
        raise Rav1eHipError("code_coefficients: token buffer overflow")
    off = doff.download(np.uint32)[:n + 1]
    tok = dtok.download(np.uint32)[:int(status[0])]
    out, tb, cdf = [], [], None
    for t in range(ntiles):
        a = int(off[starts[t]])
        b = int(off[starts[t + 1]]) if t + 1 < ntiles else int(off[n])
        cdf = np.array(cdf_init, np.uint16)
        by = ec_code_tokens(tok[a:b], cdf)
        out.append(by)
        tb.append(len(by))
    return np.concatenate(out), np.array(tb, np.int32), cdf, tok


def prep_8tap_batch(src: DevicePlane, jobs, w, h, mode_x=0, mode_y=0, bit_depth=8):
    jobs = np.ascontiguousarray(jobs, dtype=MC_JOB)
    dj = DeviceBuffer.from_array(jobs)
    out = DeviceBuffer(2 * w * h * max(1, len(jobs)))
    _check(lib().rv_prep_8tap_batch(out.ptr, C.byref(src.desc), dj.ptr, len(jobs), w, h,
                                    mode_x, mode_y, bit_depth, None), "rv_prep_8tap_batch")
    _sync()
    return out.download(np.int16, w * h * len(jobs)).reshape(len(jobs), h, w)


def mc_avg_batch(dst: DevicePlane, tmp1: np.ndarray, tmp2: np.ndarray, jobs, w, h,
                 bit_depth=8):
    jobs = np.ascontiguousarray(jobs, dtype=MC_JOB)
    dj = DeviceBuffer.from_array(jobs)
    t1 = DeviceBuffer.from_array(np.ascontiguousarray(tmp1, dtype=np.int16))
    t2 = DeviceBuffer.from_array(np.ascontiguousarray(tmp2, dtype=np.int16))
    _check(lib().rv_mc_avg_batch(C.byref(dst.desc), t1.ptr, t2.ptr, dj.ptr, len(jobs), w, h,
                                 bit_depth, None), "rv_mc_avg_batch")
    _sync()


def mc_dist_batch(org: DevicePlane, ref: DevicePlane, jobs, w, h, mode_x=0, mode_y=0,
                  bit_depth=8, metric=0) -> np.ndarray:
    jobs = np.ascontiguousarray(jobs, dtype=MC_JOB)
    dj = DeviceBuffer.from_array(jobs)
    out = DeviceBuffer(4 * max(1, len(jobs)))
    _check(lib().rv_mc_dist_batch(C.byref(org.desc), C.byref(ref.desc), dj.ptr, len(jobs), w, h,
                                  mode_x, mode_y, bit_depth, metric, out.ptr, None),
           "rv_mc_dist_batch")
    _sync()
    return out.download(np.uint32, len(jobs))


def fwd_txfm_batch(residual: np.ndarray, tx_size, tx_type, bit_depth=8) -> np.ndarray:
    """residual: [n, H, W] int16 -> coeffs [n, H*W] int32 (W-stride raster)."""
    r = np.ascontiguousarray(residual, dtype=np.int16)
    n = r.shape[0]
    w, h = TxSize(tx_size).width(), TxSize(tx_size).height()
    dr = DeviceBuffer.from_array(r)
    out = DeviceBuffer(4 * w * h * max(1, n))
    _check(lib().rv_fwd_txfm_batch(dr.ptr, out.ptr, n, int(tx_size), int(tx_type), bit_depth,
                                   None), "rv_fwd_txfm_batch")
    _sync()
    return out.download(np.int32, w * h * n).reshape(n, w * h)


def diff_fwd_txfm_batch(src: DevicePlane, pred: DevicePlane, jobs, tx_size, tx_type,
                        bit_depth=8) -> np.ndarray:
    jobs = np.ascontiguousarray(jobs, dtype=TX_JOB)
    w, h = TxSize(tx_size).width(), TxSize(tx_size).height()
    dj = DeviceBuffer.from_array(jobs)
    out = DeviceBuffer(4 * w * h * max(1, len(jobs)))
    _check(lib().rv_diff_fwd_txfm_batch(C.byref(src.desc), C.byref(pred.desc), dj.ptr, len(jobs),
                                        int(tx_size), int(tx_type), bit_depth, out.ptr, None),
           "rv_diff_fwd_txfm_batch")
    _sync()
    return out.download(np.int32, w * h * len(jobs)).reshape(len(jobs), w * h)


def coded_tx_area(tx_size) -> int:
    """av1_get_coded_tx_size(tx_size).area() (src/context.rs:1949-1956)."""
    t = TxSize(tx_size)
    return min(t.width(), 32) * min(t.height(), 32)


def quantize_batch(coeffs: np.ndarray, tx_size, tx_type, qindex, bit_depth=8, is_intra=False,
                   dc_delta_q=0, ac_delta_q=0):
    """QuantizationContext::update + quantize + dequantize (src/quantize.rs:
    205-333) of coeffs [n, >= coded area] (the forward transform's raster):
    (qcoeffs [n, coded], rcoeffs [n, coded], eob [n])."""
    c = np.ascontiguousarray(coeffs, dtype=np.int32)
    n, stride = c.shape
    coded = coded_tx_area(tx_size)
    dc = DeviceBuffer.from_array(c)
    dq = DeviceBuffer(4 * coded * max(1, n))
    dr = DeviceBuffer(4 * coded * max(1, n))
    de = DeviceBuffer(4 * max(1, n))
    _check(lib().rv_quantize_batch(dc.ptr, stride, n, int(tx_size), int(tx_type), int(qindex),
                                   bit_depth, int(bool(is_intra)), dc_delta_q, ac_delta_q, dq.ptr,
                                   dr.ptr, de.ptr, None), "rv_quantize_batch")
    _sync()
    return (dq.download(np.int32, coded * n).reshape(n, coded),
            dr.download(np.int32, coded * n).reshape(n, coded), de.download(np.uint32, n))


def dequantize_batch(qcoeffs: np.ndarray, tx_size, qindex, bit_depth=8, dc_delta_q=0,
                     ac_delta_q=0):
    """dequantize (src/quantize.rs:319-333) of [n, coded area] levels."""
    q = np.ascontiguousarray(qcoeffs, dtype=np.int32)
    n = q.shape[0]
    coded = coded_tx_area(tx_size)
    if q.shape[1] != coded:
        raise Rav1eHipError("dequantize_batch: rows must hold the coded area")
    dq = DeviceBuffer.from_array(q)
    dr = DeviceBuffer(4 * coded * max(1, n))
    _check(lib().rv_dequantize_batch(dq.ptr, n, int(tx_size), int(qindex), bit_depth, dc_delta_q,
                                     ac_delta_q, dr.ptr, None), "rv_dequantize_batch")
    _sync()
    return dr.download(np.int32, coded * n).reshape(n, coded)


def estimate_rate_batch(tx_dist: np.ndarray, tx_size, qindex) -> np.ndarray:
    """estimate_rate (src/rdo.rs:204-216) of each block's tx-domain
    distortion (u64) at base qindex: the table-interpolated rate, u64."""
    d = np.ascontiguousarray(tx_dist, dtype=np.uint64).ravel()
    n = d.size
    dd = DeviceBuffer.from_array(d if n else np.zeros(1, np.uint64))
    dr = DeviceBuffer(8 * max(1, n))
    _check(lib().rv_estimate_rate_batch(dd.ptr, n, int(qindex), int(tx_size), dr.ptr, None),
           "rv_estimate_rate_batch")
    _sync()
    return dr.download(np.uint64, n)


def inv_txfm_add_batch(coeffs: np.ndarray, dst: DevicePlane, jobs, tx_size, tx_type,
                       bit_depth=8):
    """coeffs: [n, min(H,32)*min(W,32)] int32, added into dst in place."""
    jobs = np.ascontiguousarray(jobs, dtype=TX_JOB)
    dc = DeviceBuffer.from_array(np.ascontiguousarray(coeffs, dtype=np.int32))
    dj = DeviceBuffer.from_array(jobs)
    _check(lib().rv_inv_txfm_add_batch(dc.ptr, C.byref(dst.desc), dj.ptr, len(jobs),
                                       int(tx_size), int(tx_type), bit_depth, None),
           "rv_inv_txfm_add_batch")
    _sync()


def full_search_batch(org: DevicePlane, ref: DevicePlane, jobs, blk_w, blk_h, step=1,
                      allow_hp=False) -> np.ndarray:
    jobs = np.ascontiguousarray(jobs, dtype=FS_JOB)
    dj = DeviceBuffer.from_array(jobs)
    out = DeviceBuffer(16 * max(1, len(jobs)))
    _check(lib().rv_full_search_batch(C.byref(org.desc), C.byref(ref.desc), dj.ptr, len(jobs),
                                      blk_w, blk_h, step, 1 if allow_hp else 0, out.ptr, None),
           "rv_full_search_batch")
    _sync()
    return out.download(FS_RESULT, len(jobs))


def plane_box_sums(plane: DevicePlane) -> DeviceBuffer:
    """rv_plane_box_sums: paired 4-tall x 8-wide then paired 4x4 box sums over
    the whole allocation (u32 S48(x, y) | S48(x + 8, y) << 16, then S4(x, y) |
    S4(x + 4, y) << 16, each in the plane's stride x alloc_height layout)."""
    d = plane.desc
    out = DeviceBuffer(8 * d.stride * d.alloc_height)
    _check(lib().rv_plane_box_sums(C.byref(d), out.ptr, None), "rv_plane_box_sums")
    _sync()
    return out


def full_search_sea_batch(org: DevicePlane, ref: DevicePlane, jobs, allow_hp=False,
                          s8: "DeviceBuffer | None" = None) -> np.ndarray:
    """rv_full_search_sea_batch (16x16, step 1): same results as
    full_search_batch by successive elimination over ref's box sums."""
    jobs = np.ascontiguousarray(jobs, dtype=FS_JOB)
    if s8 is None:
        s8 = plane_box_sums(ref)
    dj = DeviceBuffer.from_array(jobs)
    out = DeviceBuffer(16 * max(1, len(jobs)))
    _check(lib().rv_full_search_sea_batch(C.byref(org.desc), C.byref(ref.desc), s8.ptr, dj.ptr,
                                          len(jobs), 1 if allow_hp else 0, out.ptr, None),
           "rv_full_search_sea_batch")
    _sync()
    return out.download(FS_RESULT, len(jobs))


def diamond_search_batch(org: DevicePlane, ref: DevicePlane, jobs, blk_w, blk_h,
                         subpixel=False, use_satd=False, allow_hp=False,
                         bit_depth=8) -> np.ndarray:
    """diamond_me_search (src/me.rs:693-785) for every job in one launch."""
    jobs = np.ascontiguousarray(jobs, dtype=DS_JOB)
    dj = DeviceBuffer.from_array(jobs)
    out = DeviceBuffer(16 * max(1, len(jobs)))
    _check(lib().rv_diamond_search_batch(C.byref(org.desc), C.byref(ref.desc), dj.ptr,
                                         len(jobs), blk_w, blk_h, int(subpixel), int(use_satd),
                                         int(allow_hp), bit_depth, out.ptr, None),
           "rv_diamond_search_batch")
    _sync()
    return out.download(FS_RESULT, len(jobs))


def telescopic_subpel_batch(org: DevicePlane, ref: DevicePlane, jobs, start, blk_w, blk_h,
                            use_satd=False, allow_hp=False, bit_depth=8) -> np.ndarray:
    """telescopic_subpel_search (src/me.rs:858-941); start = FS_RESULT records
    (the full-pel best_mv / lowest_cost each search refines)."""
    jobs = np.ascontiguousarray(jobs, dtype=DS_JOB)
    start = np.ascontiguousarray(start, dtype=FS_RESULT)
    assert len(start) == len(jobs)
    dj, ds = DeviceBuffer.from_array(jobs), DeviceBuffer.from_array(start)
    out = DeviceBuffer(16 * max(1, len(jobs)))
    _check(lib().rv_telescopic_subpel_batch(C.byref(org.desc), C.byref(ref.desc), dj.ptr, ds.ptr,
                                            len(jobs), blk_w, blk_h, int(use_satd), int(allow_hp),
                                            bit_depth, out.ptr, None),
           "rv_telescopic_subpel_batch")
    _sync()
    return out.download(FS_RESULT, len(jobs))


def tx_dist_batch(coeffs: np.ndarray, rcoeffs: np.ndarray, tx_size) -> np.ndarray:
    """Transform-domain distortion (src/encoder.rs:1210-1224): coeffs [n][W*H]
    rasters, rcoeffs [n][coded area]."""
    coeffs = np.ascontiguousarray(coeffs, dtype=np.int32)
    rcoeffs = np.ascontiguousarray(rcoeffs, dtype=np.int32)
    n = coeffs.shape[0]
    dc, dr = DeviceBuffer.from_array(coeffs), DeviceBuffer.from_array(rcoeffs)
    out = DeviceBuffer(8 * max(1, n))
    _check(lib().rv_tx_dist_batch(dc.ptr, coeffs.shape[1], dr.ptr, n, int(tx_size), out.ptr, None),
           "rv_tx_dist_batch")
    _sync()
    return out.download(np.uint64, n)


# ---- reference-shaped single-call entry points ----------------------------
class PlaneRegion:
    """A block position inside a DevicePlane (PlaneRegion,
    src/tiling/plane_region.rs:110-152)."""

    def __init__(self, plane: DevicePlane, x: int, y: int):
        self.plane, self.x, self.y = plane, x, y


def _require_hip(cpu):
    if CpuFeatureLevel(cpu) != CpuFeatureLevel.HIP:
        raise Rav1eHipError(f"{CpuFeatureLevel(cpu).name}: only the HIP level is built here")


def get_sad(org: PlaneRegion, ref: PlaneRegion, bsize: BlockSize, bit_depth: int,
            cpu=CpuFeatureLevel.HIP) -> int:
    """get_sad (src/dist.rs:48-111)."""
    _require_hip(cpu)
    bs = BlockSize(bsize)
    job = np.array([(org.x, org.y, ref.x, ref.y)], dtype=DIST_JOB)
    return int(sad_batch(org.plane, ref.plane, job, bs.width(), bs.height())[0])


def get_satd(org: PlaneRegion, ref: PlaneRegion, bsize: BlockSize, bit_depth: int,
             cpu=CpuFeatureLevel.HIP) -> int:
    """get_satd (src/dist.rs:121-193)."""
    _require_hip(cpu)
    bs = BlockSize(bsize)
    job = np.array([(org.x, org.y, ref.x, ref.y)], dtype=DIST_JOB)
    return int(satd_batch(org.plane, ref.plane, job, bs.width(), bs.height())[0])


def put_8tap(dst: PlaneRegion, src: PlaneRegion, width, height, col_frac, row_frac,
             mode_x=FilterMode.REGULAR, mode_y=FilterMode.REGULAR, bit_depth=8,
             cpu=CpuFeatureLevel.HIP):
    """put_8tap (src/mc.rs:410-519): src = the block's integer position."""
    _require_hip(cpu)
    job = np.array([(src.x, src.y, dst.x, dst.y, col_frac, row_frac)], dtype=MC_JOB)
    put_8tap_batch(dst.plane, src.plane, job, width, height, int(mode_x), int(mode_y), bit_depth)


def prep_8tap(src: PlaneRegion, width, height, col_frac, row_frac,
              mode_x=FilterMode.REGULAR, mode_y=FilterMode.REGULAR, bit_depth=8,
              cpu=CpuFeatureLevel.HIP) -> np.ndarray:
    """prep_8tap (src/mc.rs:520-616): returns the i16 tmp[h][w]."""
    _require_hip(cpu)
    job = np.array([(src.x, src.y, 0, 0, col_frac, row_frac)], dtype=MC_JOB)
    return prep_8tap_batch(src.plane, job, width, height, int(mode_x), int(mode_y), bit_depth)[0]


def mc_avg(dst: PlaneRegion, tmp1, tmp2, width, height, bit_depth=8, cpu=CpuFeatureLevel.HIP):
    """mc_avg (src/mc.rs:617-706)."""
    _require_hip(cpu)
    job = np.array([(0, 0, dst.x, dst.y, 0, 0)], dtype=MC_JOB)
    mc_avg_batch(dst.plane, np.asarray(tmp1)[None], np.asarray(tmp2)[None], job, width, height,
                 bit_depth)


def forward_transform(residual: np.ndarray, tx_size: TxSize, tx_type: TxType, bit_depth=8,
                      cpu=CpuFeatureLevel.HIP) -> np.ndarray:
    """forward_transform (src/transform/mod.rs:556-566)."""
    _require_hip(cpu)
    return fwd_txfm_batch(np.asarray(residual)[None], tx_size, tx_type, bit_depth)[0]


def inverse_transform_add(coeffs: np.ndarray, dst: PlaneRegion, tx_size: TxSize,
                          tx_type: TxType, bit_depth=8, cpu=CpuFeatureLevel.HIP):
    """inverse_transform_add (src/transform/mod.rs:568-580)."""
    _require_hip(cpu)
    job = np.array([(0, 0, dst.x, dst.y)], dtype=TX_JOB)
    inv_txfm_add_batch(np.asarray(coeffs)[None], dst.plane, job, tx_size, tx_type, bit_depth)


def sse_wxh(src1: PlaneRegion, src2: PlaneRegion, w, h, compute_bias=None) -> float:
    """sse_wxh (src/rdo.rs:286-335): integer partials on the device, the
    f64 bias (compute_bias(x, y) per importance sub-block) on the host."""
    job = np.array([(src1.x, src1.y, src2.x, src2.y)], dtype=DIST_JOB)
    parts = sse_batch(src1.plane, src2.plane, job, w, h)[0]
    if compute_bias is None:
        return int(parts.sum())
    bw = min(w, 8) >> src1.plane.desc.xdec
    bh = min(h, 8) >> src1.plane.desc.ydec
    sx = w // bw
    total = 0.0
    for k, v in enumerate(parts):
        total += float(int(v)) * compute_bias((k % sx) * bw, (k // sx) * bh)
    return total


def cdef_dist_from_moments(m, bit_depth: int) -> int:
    """f64 tail of cdef_dist_wxh_8x8 (src/rdo.rs:242-252), on the host."""
    import math
    cs = bit_depth - 8
    sum_s, sum_d, s2, d2, sd = (int(v) for v in m)
    svar = float(s2 - ((sum_s * sum_s + 32) >> 6))
    dvar = float(d2 - ((sum_d * sum_d + 32) >> 6))
    sse = float(d2 + s2 - 2 * sd)
    boost = (4033.0 / 16384.0) * (svar + dvar + float(16384 << (2 * cs))) / math.sqrt(
        float(16265089 << (4 * cs)) + svar * dvar)
    v = sse * boost + 0.5
    return int(v) if v > 0 else 0


def cdef_dist_wxh(src1: PlaneRegion, src2: PlaneRegion, w, h, bit_depth=8,
                  compute_bias=None) -> float:
    """cdef_dist_wxh (src/rdo.rs:256-283)."""
    job = np.array([(src1.x, src1.y, src2.x, src2.y)], dtype=DIST_JOB)
    mom = cdef_moments_batch(src1.plane, src2.plane, job, w, h)[0]
    sx = w // 8
    total = 0.0
    for k, m in enumerate(mom):
        d = cdef_dist_from_moments(m, bit_depth)
        total += d * (compute_bias((k % sx) * 8, (k // sx) * 8) if compute_bias else 1.0)
    return total


def exported_symbols_from_header(path: str = HEADER_PATH):
    """Every function name include/rav1e_hip.h declares (macros expanded)."""
    import re
    text = open(path).read()
    names = set(re.findall(r"^\s*(?:[\w\s\*]+?)\b(rv_\w+|rav1e_\w+)\s*\(", text, re.M))
    names = {n for n in names if not n.startswith("rv_dist_fn") and n not in ("rv_put_fn",)}
    sizes = re.findall(r"X\((\d+), (\d+)\)", text.split("#define RV_DIST_SIZES")[1].split(
        "/*")[0])
    for w, h in sizes:
        names |= {f"rav1e_sad{w}x{h}_hip", f"rav1e_sad{w}x{h}_hbd_hip",
                  f"rav1e_satd_{w}x{h}_hip", f"rav1e_satd_{w}x{h}_hbd_hip"}
    pairs = re.findall(r"X\((\w+), (\w+), \d, \d\)", text.split("#define RV_FILTER_PAIRS")[1]
                       .split("#define RV_DECL_MC")[0])
    for nx, ny in pairs:
        names |= {f"rav1e_put_8tap_{nx}_{ny}_hip", f"rav1e_put_8tap_{nx}_{ny}_16bpc_hip",
                  f"rav1e_prep_8tap_{nx}_{ny}_hip", f"rav1e_prep_8tap_{nx}_{ny}_16bpc_hip"}
    return sorted(n for n in names if "##" not in n and not n.endswith("_hip_") and
                  n not in ("rav1e_sad", "rav1e_satd_", "rav1e_put_8tap_",
                            "rav1e_prep_8tap_"))
