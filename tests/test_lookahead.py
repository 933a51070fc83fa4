"""The lookahead (src/api/internal.rs): compute_lookahead_intra_costs
(:678-765) and compute_block_importances (:823-1077), the oracle's
restatements (oracle/orc_lookahead.c, orc_intra.c) and the HIP kernels
(rv_lookahead_intra_costs, rv_propagate_importances) against vectors made by
evaluating the reference's own methods on a host ContextInner
(tests/golden/ref_lookahead.npz, tools/refeval/gen_golden_ref.py lookahead):
three frames, output 0 (KEY) referenced by 1 and 2, 2 referencing 0 and 1 --
frame 1's f32 importances after frame 2's pass and frame 0's final values
(log2 step included: both sides use numpy's float32 log2)."""
import os

import numpy as np
import pytest

from tests import oracle_lib as O

GOLD = os.path.join(os.path.dirname(__file__), "golden", "ref_lookahead.npz")
PAD = 48


def _case(bd):
    g = np.load(GOLD)
    k = "la_bd%d_" % bd
    frames = g[k + "frames"].astype(np.uint8 if bd == 8 else np.uint16)
    return (frames, g[k + "mvs"], g[k + "mvs1"], g[k + "intra"], g[k + "imp1"], g[k + "imp0"])


def _sample(mvs_full):
    """lookahead_mvs[y * 2][x * 2] per importance block."""
    return np.ascontiguousarray(mvs_full[0::2, 0::2])


def _propagate_all(prop, frames, mvs, mvs1, intra):
    """compute_block_importances' loop over outputs 2, 1 (reverse), unique
    references in order: 2 -> 0, 2 -> 1 (halves), then 1 -> 0."""
    h_imp, w_imp = intra.shape[1:]
    z = np.zeros((h_imp, w_imp), np.float32)
    imp0 = prop(frames[2], frames[0], _sample(mvs[0]), intra[2], z, 2, z)
    imp1 = prop(frames[2], frames[1], _sample(mvs[1]), intra[2], z, 2, z)
    imp0 = prop(frames[1], frames[0], _sample(mvs1), intra[1], imp1, 1, imp0)
    ic = intra[0].reshape(h_imp, w_imp).astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        fin = np.where(ic > 0, np.log2(np.float32(1) + imp0 / ic), np.float32(0))
    return imp1, fin.astype(np.float32)


@pytest.mark.parametrize("bd", [8, 10])
def test_oracle_lookahead_vs_reference(bd):
    frames, mvs, mvs1, intra, imp1, imp0 = _case(bd)
    H, W = frames.shape[1:]
    full = [np.pad(f, PAD, mode="edge") for f in frames]
    for t in range(3):
        got = O.lookahead_intra_costs(full[t], PAD, PAD, W, H, bd).ravel()
        np.testing.assert_array_equal(got, intra[t])
    intra = intra.reshape(3, H // 8, W // 8)

    def prop(org, ref, mv, ic, imp, n, into):
        return O.propagate_importances(np.pad(org, PAD, mode="edge"), PAD, PAD,
                                       np.pad(ref, PAD, mode="edge"), PAD, PAD, W, H, mv, ic,
                                       imp, n, into).reshape(H // 8, W // 8)
    g1, g0 = _propagate_all(prop, frames, mvs, mvs1, intra)
    np.testing.assert_array_equal(g1.ravel().view(np.uint32), imp1.view(np.uint32))
    np.testing.assert_array_equal(g0.ravel().view(np.uint32), imp0.view(np.uint32))
    assert (imp1 > 0).any() and (imp0 > 0).any()


@pytest.mark.gpu
@pytest.mark.parametrize("bd", [8, 10])
def test_hip_lookahead_vs_reference(bd):
    import rav1e_amd as R
    R.require_device(0)
    frames, mvs, mvs1, intra, imp1, imp0 = _case(bd)
    H, W = frames.shape[1:]
    dev = [R.DevicePlane.from_array(f, xpad=PAD, ypad=PAD) for f in frames]
    for t in range(3):
        np.testing.assert_array_equal(R.lookahead_intra_costs(dev[t], bd).ravel(), intra[t])
    intra = intra.reshape(3, H // 8, W // 8)
    fl = list(frames)
    idx = {id(f): k for k, f in enumerate(fl)}

    def prop(org, ref, mv, ic, imp, n, into):
        mvs_ = np.zeros(mv.shape[:2], R.MOTION_VECTOR)
        mvs_["row"], mvs_["col"] = mv[..., 0], mv[..., 1]
        return R.propagate_importances(dev[idx[id(org)]], dev[idx[id(ref)]], mvs_, ic, imp, n,
                                       into).reshape(H // 8, W // 8)
    g1, g0 = _propagate_all(prop, fl, mvs, mvs1, intra)
    np.testing.assert_array_equal(g1.ravel().view(np.uint32), imp1.view(np.uint32))
    np.testing.assert_array_equal(g0.ravel().view(np.uint32), imp0.view(np.uint32))
