"""Compare the C oracle's 1-D transforms with the translated reference.

Dev-time check (needs /root/reference).  Usage:
    python tools/refeval/check_oracle_1d.py
"""
import ctypes
import os
import random
import sys

sys.path.insert(0, os.path.dirname(__file__))
import rs2py  # noqa: E402

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "librav1e_oracle.so"))

FWD = {  # (kind, n) -> reference function name
    (1, 4): "daala_fdct4", (1, 8): "daala_fdct8", (1, 16): "daala_fdct16",
    (1, 32): "daala_fdct32", (1, 64): "daala_fdct64",
    (2, 4): "daala_fdst_vii_4", (2, 8): "daala_fdst8", (2, 16): "daala_fdst16",
    (0, 4): "fidentity4", (0, 8): "fidentity8", (0, 16): "fidentity16",
    (0, 32): "fidentity32",
}
INV = {
    (1, 4): "av1_idct4", (1, 8): "av1_idct8", (1, 16): "av1_idct16",
    (1, 32): "av1_idct32", (1, 64): "av1_idct64",
    (2, 4): "av1_iadst4", (2, 8): "av1_iadst8", (2, 16): "av1_iadst16",
    (3, 4): "av1_iflipadst4", (3, 8): "av1_iflipadst8", (3, 16): "av1_iflipadst16",
    (0, 4): "av1_iidentity4", (0, 8): "av1_iidentity8", (0, 16): "av1_iidentity16",
    (0, 32): "av1_iidentity32",
}


def c_call(fn, kind, n, vec, *extra):
    a = (ctypes.c_int32 * n)(*vec)
    b = (ctypes.c_int32 * n)()
    rc = fn(kind, n, a, b, *extra)
    assert rc == 0, (kind, n)
    return list(b)


def main():
    ns = rs2py.load()
    rng = random.Random(1)
    bad = 0
    for (kind, n), name in FWD.items():
        for trial in range(300):
            amp = rng.choice([1, 16, 255 << 4, 4095 << 2])
            v = [rng.randint(-amp, amp) for _ in range(n)]
            ref = [0] * n
            ns[name](v, ref)
            got = c_call(lib.orc_fwd_txfm1d, kind, n, v)
            if ref != got:
                bad += 1
                print("FWD mismatch", name, v, ref, got)
                break
    for (kind, n), name in INV.items():
        for trial in range(300):
            rng_bits = rng.choice([16, 18, 20])
            amp = rng.choice([100, 3000, (1 << 15) - 1, (1 << 17) - 1])
            v = [rng.randint(-amp, amp) for _ in range(n)]
            ref = [0] * n
            ns[name](v, ref, rng_bits)
            got = c_call(lib.orc_inv_txfm1d, kind, n, v, rng_bits)
            if ref != got:
                bad += 1
                print("INV mismatch", name, rng_bits)
                print(" in ", v)
                print(" ref", ref)
                print(" got", got)
                break
    print("mismatching kernels:", bad)
    return bad


if __name__ == "__main__":
    sys.exit(1 if main() else 0)
