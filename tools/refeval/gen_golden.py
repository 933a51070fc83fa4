"""Generate tests/golden/ fixtures from the reference source.

Run in the build container (needs /root/reference):
    python tools/refeval/gen_golden.py

Outputs (data only, committed):
  tests/golden/tx1d_golden.npz  1-D transform vectors produced by the
                                reference's own kernels (translated by
                                rs2py.py): inputs and outputs.
  tests/golden/tx2d_golden.npz  2-D forward (fht) and inverse+add vectors:
                                the reference's 1-D kernels driven by a
                                restatement of FwdTxfm2D::fht
                                (src/transform/forward.rs:1804-1899) and
                                NativeInvTxfm2D::inv_txfm2d_add
                                (src/transform/inverse.rs:1939-2114).
  tests/golden/dist_kat.json    the 88 SAD/SATD known answers of
                                src/dist.rs:379-460 and the fixture recipe of
                                src/dist.rs:342-375.
"""
import json
import os
import random
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(__file__))
import rs2py  # noqa: E402

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
OUT = os.path.join(ROOT, "tests", "golden")

FWD = {(1, 4): "daala_fdct4", (1, 8): "daala_fdct8", (1, 16): "daala_fdct16",
       (1, 32): "daala_fdct32", (1, 64): "daala_fdct64",
       (2, 4): "daala_fdst_vii_4", (2, 8): "daala_fdst8", (2, 16): "daala_fdst16",
       (3, 4): "daala_fdst_vii_4", (3, 8): "daala_fdst8", (3, 16): "daala_fdst16",
       (0, 4): "fidentity4", (0, 8): "fidentity8", (0, 16): "fidentity16",
       (0, 32): "fidentity32"}
INV = {(1, 4): "av1_idct4", (1, 8): "av1_idct8", (1, 16): "av1_idct16",
       (1, 32): "av1_idct32", (1, 64): "av1_idct64",
       (2, 4): "av1_iadst4", (2, 8): "av1_iadst8", (2, 16): "av1_iadst16",
       (3, 4): "av1_iflipadst4", (3, 8): "av1_iflipadst8", (3, 16): "av1_iflipadst16",
       (0, 4): "av1_iidentity4", (0, 8): "av1_iidentity8", (0, 16): "av1_iidentity16",
       (0, 32): "av1_iidentity32"}
# 2-D inverse only reaches these through txfm_types (inverse.rs:1580-1608)
INV2D = {k: v for k, v in INV.items() if k[0] != 3}

TX_W_LOG2 = [2, 3, 4, 5, 6, 2, 3, 3, 4, 4, 5, 5, 6, 2, 4, 3, 5, 4, 6]
TX_H_LOG2 = [2, 3, 4, 5, 6, 3, 2, 4, 3, 5, 4, 6, 5, 4, 2, 5, 3, 6, 4]
TX_COL = [1, 2, 1, 2, 3, 1, 3, 2, 3, 0, 1, 0, 2, 0, 3, 0]
TX_ROW = [1, 1, 2, 2, 1, 3, 3, 3, 2, 0, 0, 1, 0, 2, 0, 3]
FWD_SHIFT = {  # forward.rs:22-40 by (w, h)
    (4, 4): [[3, 0, 0], [2, 0, 1], [0, 0, 3]],
    (32, 32): [[4, -2, 0], [2, 0, 0], [0, 0, 2]],
    (16, 32): [[4, -2, 0], [2, 0, 0], [0, 0, 2]],
    (32, 16): [[4, -2, 0], [2, 0, 0], [0, 0, 2]],
    (16, 64): [[4, -2, 0], [2, 0, 0], [0, 0, 2]],
    (64, 16): [[4, -2, 0], [2, 0, 0], [0, 0, 2]],
    (64, 64): [[4, -1, -2], [2, 0, -1], [0, 0, 1]],
    (32, 64): [[4, -1, -2], [2, 0, -1], [0, 0, 1]],
    (64, 32): [[4, -1, -2], [2, 0, -1], [0, 0, 1]],
}
DEFAULT_SHIFT = [[4, -1, 0], [2, 0, 1], [0, 0, 3]]
INV_SHIFT = [0, 1, 2, 2, 2, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2]


def rsa(v, bit):
    if bit > 0:
        return rs2py._chk((v + ((1 << bit) >> 1)) >> bit)
    if bit < 0:
        return rs2py._chk(v << -bit)
    return v


def fht(ns, residual, tx_size, tx_type, bd):
    """FwdTxfm2D::fht restated (forward.rs:1804-1899)."""
    w, h = 1 << TX_W_LOG2[tx_size], 1 << TX_H_LOG2[tx_size]
    ck, rk = TX_COL[tx_type], TX_ROW[tx_type]
    sh = FWD_SHIFT.get((w, h), DEFAULT_SHIFT)[(bd - 8) // 2]
    buf = [0] * (w * h)
    for c in range(w):
        col = []
        for r in range(h):
            rr = h - 1 - r if ck == 3 else r
            col.append(rsa(int(residual[rr * w + c]), -sh[0]))
        out = [0] * h
        ns[FWD[(ck, h)]](col, out)
        for r in range(h):
            buf[r * w + c] = rsa(out[r], -sh[1])
    coeffs = [0] * (w * h)
    for r in range(h):
        out = [0] * w
        ns[FWD[(rk, w)]](buf[r * w:(r + 1) * w], out)
        for c in range(w):
            coeffs[r * w + c] = rsa(out[c], -sh[2])
    return coeffs


def inv_add(ns, coeffs, dst, tx_size, tx_type, bd):
    """NativeInvTxfm2D::inv_txfm2d + add restated (inverse.rs:1939-2114)."""
    w, h = 1 << TX_W_LOG2[tx_size], 1 << TX_H_LOG2[tx_size]
    ck, rk = TX_COL[tx_type], TX_ROW[tx_type]
    rect = TX_W_LOG2[tx_size] - TX_H_LOG2[tx_size]
    cw, ch = min(w, 32), min(h, 32)
    rng = bd + 8
    buf = [0] * (w * h)
    for r in range(ch):
        tin = [0] * 64
        for c in range(cw):
            raw = int(coeffs[r * cw + c])
            v = rs2py.round_shift(rs2py._chk(raw * 2896), 12) if abs(rect) == 1 else raw
            tin[c] = rs2py.clamp_value(v, rng)
        out = [0] * w
        ns[INV2D[(rk, w)]](tin, out, rng)
        buf[r * w:(r + 1) * w] = out
    crange = max(bd + 6, 16)
    res = [list(map(int, row)) for row in dst]
    for c in range(w):
        tin = [0] * 64
        for r in range(h):
            tin[r] = rs2py.clamp_value(rs2py.round_shift(buf[r * w + c], INV_SHIFT[tx_size]), crange)
        out = [0] * h
        ns[INV2D[(ck, h)]](tin, out, crange)
        for r in range(h):
            v = rs2py.round_shift(out[r], 4)
            res[r][c] = max(0, min((1 << bd) - 1, res[r][c] + v))
    return res


def gen_1d(ns, rng):
    d = {}
    for table, tag in ((FWD, "fwd"), (INV, "inv")):
        for (kind, n), name in sorted(table.items()):
            ins, outs, ranges = [], [], []
            for t in range(24):
                if tag == "fwd":
                    amp = [1, 16, 255 << 4, 1023 << 4, 4095 << 2][t % 5]
                    r_ = 0
                else:
                    r_ = [16, 18, 20][t % 3]
                    amp = [64, 3000, (1 << 15) - 1, (1 << 17) - 1][t % 4]
                if t == 0:
                    v = [amp] * n
                elif t == 1:
                    v = [amp if k % 2 else -amp for k in range(n)]
                else:
                    v = [rng.randint(-amp, amp) for _ in range(n)]
                out = [0] * n
                if tag == "fwd":
                    ns[name](v, out)
                else:
                    ns[name](v, out, r_)
                ins.append(v)
                outs.append(out)
                ranges.append(r_)
            key = "%s_k%d_n%d" % (tag, kind, n)
            d[key + "_in"] = np.array(ins, dtype=np.int32)
            d[key + "_out"] = np.array(outs, dtype=np.int32)
            d[key + "_range"] = np.array(ranges, dtype=np.int32)
    return d


def fwd_ok(tx_size, tx_type):
    w, h = 1 << TX_W_LOG2[tx_size], 1 << TX_H_LOG2[tx_size]
    ck, rk = TX_COL[tx_type], TX_ROW[tx_type]
    return rk != 3 and (ck, h) in FWD and (rk, w) in FWD


def inv_ok(tx_size, tx_type):
    w, h = 1 << TX_W_LOG2[tx_size], 1 << TX_H_LOG2[tx_size]
    ck, rk = TX_COL[tx_type], TX_ROW[tx_type]
    return (ck, h) in INV2D and (rk, w) in INV2D


def gen_2d(ns, rng):
    d = {}
    index = []
    for tx_size in range(19):
        w, h = 1 << TX_W_LOG2[tx_size], 1 << TX_H_LOG2[tx_size]
        for tx_type in range(16):
            for bd in (8, 10):
                if fwd_ok(tx_size, tx_type):
                    amp = (1 << bd) - 1
                    res = [rng.randint(-amp, amp) for _ in range(w * h)]
                    co = fht(ns, res, tx_size, tx_type, bd)
                    key = "fwd_s%d_t%d_bd%d" % (tx_size, tx_type, bd)
                    d[key + "_in"] = np.array(res, dtype=np.int16)
                    d[key + "_out"] = np.array(co, dtype=np.int32)
                    index.append(key)
                if inv_ok(tx_size, tx_type):
                    cw, ch = min(w, 32), min(h, 32)
                    # sparse, quantised-looking coefficients plus a few large
                    co = [0] * (cw * ch)
                    for k in range(cw * ch):
                        if rng.random() < 0.3:
                            co[k] = rng.randint(-(1 << (bd + 3)), 1 << (bd + 3))
                    co[0] = rng.randint(-(1 << (bd + 6)), 1 << (bd + 6))
                    dst = [[rng.randint(0, (1 << bd) - 1) for _ in range(w)] for _ in range(h)]
                    out = inv_add(ns, co, dst, tx_size, tx_type, bd)
                    key = "inv_s%d_t%d_bd%d" % (tx_size, tx_type, bd)
                    d[key + "_coeffs"] = np.array(co, dtype=np.int32)
                    d[key + "_dst"] = np.array(dst, dtype=np.uint16)
                    d[key + "_out"] = np.array(out, dtype=np.uint16)
                    index.append(key)
    return d, index


DIST_KAT = {
    "source": "src/dist.rs:379-402 (SAD), :437-460 (SATD); fixture src/dist.rs:342-375",
    "fixture": {
        "input_plane": "Plane::new(640, 480, 0, 0, 136, 136); px[i][j] = ((j+i) - xpad_off) & 255",
        "rec_plane": "Plane::new(640, 480, 0, 0, 264, 264); px[i][j] = (j - i - xpad_off) & 255",
        "xpad_off": "(xorigin - xpad) - 8",
        "region": "Area::StartingAt { x: 32, y: 40 }",
        "bit_depth": 8,
    },
    "blocks": ["4x4", "4x8", "8x4", "8x8", "8x16", "16x8", "16x16", "16x32", "32x16",
               "32x32", "32x64", "64x32", "64x64", "64x128", "128x64", "128x128",
               "4x16", "16x4", "8x32", "32x8", "16x64", "64x16"],
    "sad": [1912, 4296, 3496, 7824, 16592, 14416, 31136, 60064, 59552, 120128, 186688,
            250176, 438912, 654272, 1016768, 1689792, 8680, 6664, 31056, 27600, 93344, 116384],
    "satd": [1408, 2016, 1816, 3984, 5136, 4864, 9984, 13824, 13760, 27952, 37168, 45104,
             84176, 127920, 173680, 321456, 3136, 2632, 7056, 6624, 18432, 21312],
}


def main():
    ns = rs2py.load()
    rng = random.Random(0x5EED)
    os.makedirs(OUT, exist_ok=True)
    np.savez_compressed(os.path.join(OUT, "tx1d_golden.npz"), **gen_1d(ns, rng))
    d2, index = gen_2d(ns, rng)
    np.savez_compressed(os.path.join(OUT, "tx2d_golden.npz"), **d2)
    with open(os.path.join(OUT, "dist_kat.json"), "w") as f:
        json.dump(DIST_KAT, f, indent=1)
    print("tx2d cases:", len(index))


if __name__ == "__main__":
    main()
