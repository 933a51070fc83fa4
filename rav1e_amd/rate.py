"""Fixed-quantizer frame parameters (rate control off): the qindices and
lambdas rav1e gives a frame of each pyramid level for `--quantizer q`
(RCState::select_qi, src/rate.rs:746-775; QuantizerParameters::
new_from_log_q, :570-606; FrameInvariants::set_quantizers and the lambda
scaling, src/encoder.rs:865-880).  Host-side integer restatement; the
replay receives the results (rv_replay_set_level_params)."""
from __future__ import annotations

import bisect
import math

import numpy as np

from . import lib

MASK64 = (1 << 64) - 1
QSCALE = 3
MINQ, MAXQ = 0, 255


def _i64(v: int) -> int:
    v &= MASK64
    return v - (1 << 64) if v >> 63 else v


def q57(v: int) -> int:
    return v << 57


# src/rate.rs:64-80: MQP_Q12 = 1.0 for every subtype; DQP_Q57 steps of
# 33810170 / 86043287 (a 15-quantizer-step change) per subtype
MQP_Q12 = [4096, 4096, 4096, 4096]
DQP_Q57 = [int(-(33_810_170.0 / 86_043_287.0) * float(1 << 57)), 0,
           int((33_810_170.0 / 86_043_287.0) * float(1 << 57)),
           int(2.0 * (33_810_170.0 / 86_043_287.0) * float(1 << 57))]
FRAME_SUBTYPE_I, FRAME_SUBTYPE_P = 0, 1

ATANH_LOG2 = [
    0x32B803473F7AD0F4, 0x2F2A71BD4E25E916, 0x2E68B244BB93BA06, 0x2E39FB9198CE62E4,
    0x2E2E683F68565C8F, 0x2E2B850BE2077FC1, 0x2E2ACC58FE7B78DB, 0x2E2A9E2DE52FD5F2,
    0x2E2A92A338D53EEC, 0x2E2A8FC08F5E19B6, 0x2E2A8F07E51A485E, 0x2E2A8ED9BA8AF388,
    0x2E2A8ECE2FE7384A, 0x2E2A8ECB4D3E4B1A, 0x2E2A8ECA94940FE8, 0x2E2A8ECA6669811D,
    0x2E2A8ECA5ADEDD6A, 0x2E2A8ECA57FC347E, 0x2E2A8ECA57438A43, 0x2E2A8ECA57155FB4,
    0x2E2A8ECA5709D510, 0x2E2A8ECA5706F267, 0x2E2A8ECA570639BD, 0x2E2A8ECA57060B92,
    0x2E2A8ECA57060008, 0x2E2A8ECA5705FD25, 0x2E2A8ECA5705FC6C, 0x2E2A8ECA5705FC3E,
    0x2E2A8ECA5705FC33, 0x2E2A8ECA5705FC30, 0x2E2A8ECA5705FC2F, 0x2E2A8ECA5705FC2F]


def bexp64(logq57: int) -> int:
    """Binary exponential, Q57 log in, Q0 out (src/rate.rs:108-200): the
    CORDIC iteration with repeated steps 4, 13 and 40."""
    ipart = logq57 >> 57
    if ipart < 0:
        return 0
    if ipart >= 63:
        return 0x7FFFFFFFFFFFFFFF
    z = logq57 - q57(ipart)
    if z != 0:
        z = _i64(z << 5)
        w = 0x26A3D0E401DD846D
        i = 0
        for rep in (3, 12):
            while True:
                mask = -1 if z < 0 else 0
                w = _i64(w + (((w >> (i + 1)) + mask) ^ mask))
                z = _i64(z - ((ATANH_LOG2[i] + mask) ^ mask))
                if i >= rep:
                    break
                z = _i64(z * 2)
                i += 1
        while i < 32:
            mask = -1 if z < 0 else 0
            w = _i64(w + (((w >> (i + 1)) + mask) ^ mask))
            z = _i64((z - ((ATANH_LOG2[i] + mask) ^ mask)) * 2)
            i += 1
        wlo = 0
        if ipart > 30:
            while True:
                mask = -1 if z < 0 else 0
                wlo += ((w >> i) + mask) ^ mask
                z = _i64(z - ((ATANH_LOG2[31] + mask) ^ mask))
                if i >= 39:
                    break
                z = _i64(z * 2)
                i += 1
            while i < 61:
                mask = -1 if z < 0 else 0
                wlo += ((w >> i) + mask) ^ mask
                z = _i64((z - ((ATANH_LOG2[31] + mask) ^ mask)) * 2)
                i += 1
            wlo = _i64(wlo) & 0xFFFFFFFF
            wlo = wlo - (1 << 32) if wlo >> 31 else wlo  # i32
        w = _i64((w << 1) + wlo)
    else:
        w = 1 << 62
    if ipart < 62:
        w = ((w >> (61 - ipart)) + 1) >> 1
    return w


def blog64(w: int) -> int:
    """Binary log, Q0 in, Q57 out (src/rate.rs:205-267)."""
    if w <= 0:
        return -1
    ipart = w.bit_length() - 1
    w = w >> (ipart - 61) if ipart > 61 else _i64(w << (61 - ipart))
    z = 0
    if w & (w - 1):
        x, y = _i64(w + (1 << 61)), _i64(w - (1 << 61))
        for lo, hi, ti in ((0, 4, None), (3, 13, None), (12, 32, None), (32, 40, 31), (39, 62, 31)):
            for i in range(lo, hi):
                mask = -1 if y < 0 else 0
                a = ATANH_LOG2[i if ti is None else ti]
                z = _i64(z + (((a >> i) + mask) ^ mask))
                u = x >> (i + 1)
                x = _i64(x - (((y >> (i + 1)) + mask) ^ mask))
                y = _i64(y - ((u + mask) ^ mask))
        z = (z + 8) >> 4
    return q57(ipart) + z


def q_lookup(ac: bool, qindex: int, bit_depth: int) -> int:
    v = lib().rv_q_lookup(1 if ac else 0, qindex, bit_depth)
    if v < 0:
        raise ValueError("rv_q_lookup: bad arguments")
    return v


def select_qi(quantizer: int, ac: bool, bit_depth: int) -> int:
    """select_qi (src/quantize.rs:64-86): the table entry nearest in the
    log domain."""
    tab = [q_lookup(ac, i, bit_depth) for i in range(256)]
    if quantizer < tab[MINQ]:
        return MINQ
    if quantizer >= tab[MAXQ]:
        return MAXQ
    qi = bisect.bisect_left(tab, quantizer)
    if tab[qi] == quantizer:  # binary_search hit (the ac tables are strictly ascending)
        return qi
    qthresh = tab[qi - 1] * tab[qi]
    return qi - 1 if quantizer * quantizer < qthresh else qi


def chroma_offset(log_target_q: int):
    """src/rate.rs:561-567"""
    x = max(log_target_q, 0)
    y = (x >> 2) + (x >> 6)
    return 0x19D5D9FD5010B37 - y, 0xA4D3C25E68DC58 - y


Q57_SQUARE_EXP_SCALE = (2.0 * math.log(2.0)) / float(1 << 57)


def frame_params(quantizer: int, bit_depth: int, fti: int) -> dict:
    """QuantizerParameters of frame subtype fti for a fixed quantizer, and
    the FrameInvariants values the RDO uses: base_q_idx, per-plane dc/ac
    deltas, lambda (scaled for the bit depth), me_lambda, dist_scale."""
    ac_quantizer = q_lookup(True, quantizer, bit_depth)
    dc_qi = select_qi(ac_quantizer, False, bit_depth)
    dc_quantizer = q_lookup(False, dc_qi, bit_depth)
    log_ac_q = blog64(ac_quantizer) - q57(QSCALE + bit_depth - 8)
    log_dc_q = blog64(dc_quantizer) - q57(QSCALE + bit_depth - 8)
    log_base_q = (log_ac_q + log_dc_q + 1) >> 1
    log_q = ((log_base_q + (1 << 11)) >> 12) * MQP_Q12[fti] + DQP_Q57[fti]
    scale = q57(QSCALE + bit_depth - 8)
    off_u, off_v = chroma_offset(log_q)
    logs = [log_q, log_q + off_u, log_q + off_v]
    quant = [bexp64(lq + scale) for lq in logs]
    lambdas = [(math.log(2.0) / 6.0) * math.exp(float(lq) * Q57_SQUARE_EXP_SCALE) for lq in logs]
    dc_qis = [max(select_qi(q, False, bit_depth), 1) for q in quant]
    ac_qis = [max(select_qi(q, True, bit_depth), 1) for q in quant]
    base = ac_qis[0]
    # FrameInvariants::set_quantizers: lambda scaled by 1 << 2 (bd - 8),
    # me_lambda = sqrt(lambda) (src/encoder.rs:865-880)
    lam = lambdas[0] * float(1 << (2 * (bit_depth - 8)))
    cdef_y, cdef_uv = cdef_strengths(log_q)
    return {"base_q_idx": base, "cdef_y": cdef_y, "cdef_uv": cdef_uv,
            "dc_delta_q": [d - base for d in dc_qis], "ac_delta_q": [a - base for a in ac_qis],
            "lambda": lam, "me_lambda": math.sqrt(lam),
            "dist_scale": [1.0, lambdas[0] / lambdas[1], lambdas[0] / lambdas[2]]}


def _f32_poly(q, a, b, c, neg_sq):
    """clamp-free ((+/-)q*q*a + q*b + c).round() in f32 arithmetic, left to
    right like the reference's expression (no fused multiply-add)."""
    f = np.float32
    sq = (f(-q) if neg_sq else q) * q * f(a)
    v = f(f(sq) + f(q * f(b))) + f(c)
    v = float(f(v))
    return int(math.floor(abs(v) + 0.5)) * (1 if v >= 0 else -1)  # f32::round: half away


def cdef_strengths(log_target_q: int):
    """FrameInvariants::set_quantizers' CDEF strengths of an inter frame
    (src/encoder.rs:882-912, the !intra_only branch): q = bexp64(
    log_target_q + q57(QSCALE)) as f32, libaom-trained polynomials,
    cdef_y_strengths[0] / cdef_uv_strengths[0] = f1 * CDEF_SEC_STRENGTHS + f2."""
    q = np.float32(bexp64(log_target_q + q57(QSCALE)))

    def cl(v, hi):
        return min(max(v, 0), hi)
    y1 = cl(_f32_poly(q, 0.0000023593946, 0.0068615186, 0.02709886, True), 15)
    y2 = cl(_f32_poly(q, 0.00000057629734, 0.0013993345, 0.03831067, True), 3)
    u1 = cl(_f32_poly(q, 0.0000007095069, 0.0034628846, 0.00887099, True), 15)
    u2 = cl(_f32_poly(q, 0.00000023874085, 0.00028223585, 0.05576307, False), 3)
    return y1 * 4 + y2, u1 * 4 + u2


def level_params(quantizer: int, bit_depth: int, levels: int = 3) -> list:
    """frame_params of the inter frames of each pyramid level (subtype P +
    level, FrameInvariants::get_frame_subtype, src/encoder.rs:857-863)."""
    return [frame_params(quantizer, bit_depth, FRAME_SUBTYPE_P + lv) for lv in range(levels)]
