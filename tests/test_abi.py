"""CPU-side checks of the C ABI (no GPU needed, no compute calls):
the library loads, exports every symbol include/rav1e_hip.h declares,
plane geometry and the dispatch level follow the reference, and argument
validation rejects what the reference's safe wrappers assert on."""
import ctypes as C
import os
import subprocess
import sys

import numpy as np
import pytest

import rav1e_amd as R
from tests import oracle_lib as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    names = R.exported_symbols_from_header()
    assert len(names) > 200
    L = R.lib()
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    # the per-size asm-shaped entry points of SURVEY.md §8b are all there
    for w, h in [(4, 4), (128, 128), (64, 16), (16, 64)]:
        assert f"rav1e_sad{w}x{h}_hip" in names and f"rav1e_satd_{w}x{h}_hbd_hip" in names


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/bin/roc-obj-ls", R.LIB_PATH], capture_output=True,
                         text=True)
    if out.returncode != 0:
        pytest.skip("roc-obj-ls unavailable")
    assert "gfx950" in out.stdout


def test_geometry_matches_plane_new():
    for (w, h, pad, hbd) in [(1920, 1080, 88, 0), (960, 540, 44, 0), (480, 270, 22, 0),
                             (3840, 2160, 88, 1), (640, 480, 136, 0), (17, 9, 5, 1)]:
        p = R.RvPlane()
        nbytes = R.lib().rv_plane_geometry(C.byref(p), w, h, 0, 0, pad, pad, hbd)
        stride, alloc_h, xo, yo = O.plane_geometry(w, h, pad, pad, hbd)
        assert (p.stride, p.alloc_height, p.xorigin, p.yorigin) == (stride, alloc_h, xo, yo)
        assert nbytes == stride * alloc_h * (2 if hbd else 1)


def test_cpu_feature_level_env():
    code = ("import rav1e_amd as R; import sys; "
            "sys.stdout.write(str(int(R.CpuFeatureLevel.default())))")
    for env, want in [("hip", 4), ("avx2", 3), ("rust", 0), ("sse2", 1)]:
        r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True,
                           text=True, env=dict(os.environ, RAV1E_CPU_TARGET=env))
        assert r.stdout.strip() == str(want), r.stderr
    assert R.lib().rv_cpu_feature_level_index(4) == 4


def test_argument_validation_rejects_without_launch():
    L = R.lib()
    p = R.RvPlane()
    L.rv_plane_geometry(C.byref(p), 64, 64, 0, 0, 8, 8, 0)
    out = C.c_void_p(0)
    # odd / oversized blocks (BlockSize::from_width_and_height panics)
    assert L.rv_sad_batch(C.byref(p), C.byref(p), None, 1, 3, 4, out, None) == R.RV_EINVAL
    assert L.rv_satd_batch(C.byref(p), C.byref(p), None, 1, 256, 4, out, None) == R.RV_EINVAL
    # assert!(w & (MI_SIZE-1) == 0) in sse_wxh, w & 7 in cdef_dist_wxh
    assert L.rv_sse_batch(C.byref(p), C.byref(p), None, 1, 6, 8, out, None) == R.RV_EINVAL
    assert L.rv_cdef_moments_batch(C.byref(p), C.byref(p), None, 1, 12, 8, out, None) == R.RV_EINVAL
    # bad filter mode / bit depth
    assert L.rv_put_8tap_batch(C.byref(p), C.byref(p), None, 1, 8, 8, 4, 0, 8, None) == R.RV_EINVAL
    assert L.rv_put_8tap_batch(C.byref(p), C.byref(p), None, 1, 8, 8, 0, 0, 10, None) == R.RV_EINVAL
    # transforms the reference leaves unimplemented
    assert L.rv_fwd_txfm_batch(None, None, 1, 4, 1, 8, None) == R.RV_ENOTSUP  # ADST64
    assert L.rv_fwd_txfm_batch(None, None, 1, 0, 5, 8, None) == R.RV_ENOTSUP  # row FlipAdst
    assert L.rv_inv_txfm_add_batch(None, C.byref(p), None, 1, 0, 4, 8, None) == R.RV_ENOTSUP
    assert L.rv_fwd_txfm_batch(None, None, 1, 19, 0, 8, None) == R.RV_EINVAL
    assert b"unsupported" in L.rv_last_error() or b"bad" in L.rv_last_error()
    # n = 0 is a no-op
    assert L.rv_sad_batch(C.byref(p), C.byref(p), None, 0, 8, 8, out, None) == R.RV_OK


def test_python_mirror_enums_follow_reference_order():
    assert R.BlockSize.from_width_and_height(64, 16) == R.BlockSize.BLOCK_64X16 == 21
    assert R.TxSize.TX_64X16 == 18 and R.TxSize(4).width() == 64
    assert R.TxType.H_FLIPADST == 15 and R.FilterMode.BILINEAR == 3
    assert [b.name for b in R.BlockSize][:3] == ["BLOCK_4X4", "BLOCK_4X8", "BLOCK_8X4"]
    assert O.BLOCKS == [f"{b.width()}x{b.height()}" for b in R.BlockSize]


def test_hip_level_required():
    with pytest.raises(R.Rav1eHipError):
        R._require_hip(R.CpuFeatureLevel.AVX2)


def test_no_device_here_fails_loudly():
    if R.lib().rv_device_count() > 0:
        pytest.skip("a device is visible")
    with pytest.raises(R.Rav1eHipError):
        R.require_device(0)


def test_round_ring_slots_keep_live_checks_apart():
    """The MV-stack / lookahead round loop (rv_replay.hip run_rounds) keeps
    kRoundsAhead rounds queued beyond the last published count it read, so
    up to kRoundsAhead + 2 checks are in flight at once.  Their device count
    slots, the slot each zeroes for its successor and their host
    publication slots must stay apart (round 4 published every check into
    one host slot and a count could be read for the wrong check; the slot
    layout is RoundRing's own code, through rv_round_ring_slots)."""
    L = R.lib()
    out = (C.c_int32 * 6)()
    slots = []
    for q in range(0, 3 * 256):
        assert L.rv_round_ring_slots(q, out, 6) == 6
        slots.append(tuple(out[:3]))
    ahead, kcnt, kpub = out[3], out[4], out[5]
    live = ahead + 2
    assert live < min(kcnt, kpub)
    for q in range(len(slots) - live):
        cnt, nxt, pub = slots[q]
        assert nxt == slots[q + 1][0]  # check q zeroes check q + 1's slot
        assert nxt != cnt
        for k in range(1, live):
            assert slots[q + k][0] != cnt, (q, k)  # no later live check counts into q's slot
            assert slots[q + k][1] != cnt, (q, k)  # ... or zeroes it
            assert slots[q + k][2] != pub, (q, k)  # ... or publishes over q's count
    # the ring wraps (the sequence number is u32): q and q + kPub share a slot
    assert slots[0][2] == slots[kpub][2]
