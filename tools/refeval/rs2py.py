"""Evaluate the reference's own 1-D transform functions.

Fixture-generation tool (runs only in the build container, where
/root/reference exists).  It reads the Rust source of geobacter-rs/rav1e's
1-D transform kernels as TEXT, translates the (very regular) subset of Rust
they are written in into Python, and executes that translation to produce
golden input/output vectors.  Nothing from the reference is written into the
repository: only the generated numbers (tests/golden/*.json).

Translated functions:
  src/transform/forward.rs : daala_fdct4/8/16/32/64, daala_fdst_vii_4,
                             daala_fdst8, daala_fdst16, fidentity4..32 and
                             every helper they call (rotations/butterflies
                             are provided here as Python restatements of
                             forward.rs:100-324; the lifting sequences
                             themselves are the reference's own text).
  src/transform/inverse.rs : av1_idct4..64, av1_iadst4/8/16,
                             av1_iflipadst4/8/16, av1_iidentity4..32.

Semantics: Python ints wrapped to i32 in every helper (release-mode Rust
wrapping); inputs are sized so the reference's bare `+`/`-` never wrap.
"""
import re

I32_MIN, I32_MAX = -(1 << 31), (1 << 31) - 1


def _chk(v):
    """Wrap to i32: the reference is measured in release mode, where i32
    overflow wraps (the helpers below are where the reference multiplies)."""
    return ((v + (1 << 31)) & 0xFFFFFFFF) - (1 << 31)


# ---- helpers shared by the translated code -------------------------------
# forward.rs:114-130 (TxOperations for i32)
def tx_mul(x, m):
    return _chk((_chk(x * m[0]) + ((1 << m[1]) >> 1)) >> m[1])


def rshift1(x):
    return _chk((x + (1 if x < 0 else 0)) >> 1)


def add_avg(a, b):
    return _chk((a + b) >> 1)


def sub_avg(a, b):
    return _chk((a - b) >> 1)


def copy_fn(x):
    return x


def _add(a, b):
    return _chk(a + b)


def _sub(a, b):
    return _chk(a - b)


class _Pi4:  # forward.rs:164-174
    ADD = None
    SUB = None

    @classmethod
    def kernel(cls, p0, p1, m):
        t = cls.ADD(p1, p0)
        a, out0 = tx_mul(p0, m[0]), tx_mul(t, m[1])
        return out0, cls.SUB(a, out0)


class RotatePi4Add(_Pi4):
    ADD, SUB = staticmethod(_add), staticmethod(_sub)


class RotatePi4AddAvg(_Pi4):
    ADD, SUB = staticmethod(add_avg), staticmethod(_sub)


class RotatePi4Sub(_Pi4):
    ADD, SUB = staticmethod(_sub), staticmethod(_add)


class RotatePi4SubAvg(_Pi4):
    ADD, SUB = staticmethod(sub_avg), staticmethod(_add)


class _Rot:  # forward.rs:201-220
    ADD = SUB = SHIFT = None

    @classmethod
    def half_kernel(cls, p0, p1, m):
        t = cls.ADD(p1, p0[0])
        a, b, c = tx_mul(p0[1], m[0]), tx_mul(p1, m[1]), tx_mul(t, m[2])
        out0 = _add(b, c)
        return out0, cls.SUB(a, cls.SHIFT(c))

    @classmethod
    def kernel(cls, p0, p1, m):
        return cls.half_kernel((p0, p0), p1, m)


class RotateAdd(_Rot):
    ADD, SUB, SHIFT = staticmethod(_add), staticmethod(_sub), staticmethod(copy_fn)


class RotateAddAvg(_Rot):
    ADD, SUB, SHIFT = staticmethod(add_avg), staticmethod(_sub), staticmethod(copy_fn)


class RotateAddShift(_Rot):
    ADD, SUB, SHIFT = staticmethod(_add), staticmethod(_sub), staticmethod(rshift1)


class RotateSub(_Rot):
    ADD, SUB, SHIFT = staticmethod(_sub), staticmethod(_add), staticmethod(copy_fn)


class RotateSubAvg(_Rot):
    ADD, SUB, SHIFT = staticmethod(sub_avg), staticmethod(_add), staticmethod(copy_fn)


class RotateSubShift(_Rot):
    ADD, SUB, SHIFT = staticmethod(_sub), staticmethod(_add), staticmethod(rshift1)


class _Neg:  # forward.rs:222-232
    ADD = None

    @classmethod
    def kernel(cls, p0, p1, m):
        t = cls.ADD(p0, p1)
        a, b, c = tx_mul(p0, m[0]), tx_mul(p1, m[1]), tx_mul(t, m[2])
        return _sub(b, c), _sub(c, a)


class RotateNeg(_Neg):
    ADD = staticmethod(_sub)


class RotateNegAvg(_Neg):
    ADD = staticmethod(sub_avg)


# inverse.rs helpers (src/transform/mod.rs:476-496)
def half_btf(w0, in0, w1, in1, bit):
    r = _chk(_chk(w0 * in0) + _chk(w1 * in1))
    return r if bit == 0 else _chk((r + (1 << (bit - 1))) >> bit)


def clamp_value(v, bit):
    v = _chk(v)
    hi, lo = (1 << (bit - 1)) - 1, -(1 << (bit - 1))
    return max(lo, min(hi, v))


def round_shift(v, bit):
    # src/util/mod.rs:241-243: `value: i32` is already wrapped, and so is the add
    return _chk(_chk(_chk(v) + ((1 << bit) >> 1)) >> bit)


class View:
    """`&mut output[a..b]`"""

    def __init__(self, base, a, b):
        self.base, self.a, self.b = base, a, b

    def __getitem__(self, i):
        return self.base[self.a + i]

    def __setitem__(self, i, v):
        self.base[self.a + i] = v

    def __len__(self):
        return self.b - self.a


def rev(arr, a, b):
    vals = [arr[i] for i in range(a, b)]
    for k, v in enumerate(reversed(vals)):
        arr[a + k] = v


def store_coeffs(arr, *vals):
    for i, v in enumerate(vals):
        arr[i] = v


# ---- Rust -> Python translation ----------------------------------------
def _strip_comments(src):
    return re.sub(r"//[^\n]*", "", src)


def _match_close(s, i, open_ch, close_ch):
    depth = 0
    for k in range(i, len(s)):
        if s[k] == open_ch:
            depth += 1
        elif s[k] == close_ch:
            depth -= 1
            if depth == 0:
                return k
    raise ValueError("unbalanced")


def _find_fn(src, name):
    m = re.search(r"\bfn\s+" + re.escape(name) + r"\s*(<[^>]*>)?\s*\(", src)
    if not m:
        raise KeyError(name)
    p0 = m.end() - 1
    p1 = _match_close(src, p0, "(", ")")
    params = src[p0 + 1:p1]
    b0 = src.index("{", p1)
    b1 = _match_close(src, b0, "{", "}")
    return params, src[b0 + 1:b1]


def _split_top(s, sep):
    out, depth, cur = [], 0, []
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == sep and depth == 0:
            out.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
            # a bare `{ ... }` block statement ends at its closing brace
            if ch == "}" and depth == 0 and sep == ";" and "".join(cur).strip().startswith("{"):
                out.append("".join(cur))
                cur = []
    if "".join(cur).strip():
        out.append("".join(cur))
    return out


def _param_names(params):
    names = []
    for p in _split_top(params, ","):
        p = p.strip()
        if p:
            names.append(p.split(":")[0].strip().replace("mut ", ""))
    return names


_METHODS = ("tx_mul", "rshift1", "sub_avg", "add_avg")


def _expr(e):
    e = e.strip()
    # `&mut output[a..b]` -> View
    e = re.sub(r"&mut\s+(\w+)\[(\d+)\.\.(\d+)\]", r"View(\1, \2, \3)", e)
    e = e.replace("&mut ", "").replace("&", "")
    e = re.sub(r"\b(\w+)\.(" + "|".join(_METHODS) + r")\(\)", r"\2(\1)", e)
    e = re.sub(r"\b(\w+)\.(" + "|".join(_METHODS) + r")\(", r"\2(\1, ", e)
    e = re.sub(r"(\w+)::(kernel|half_kernel)\(", r"\1.\2(", e)
    e = e.replace("store_coeffs!(", "store_coeffs(")
    e = re.sub(r"\b(\w+)\.(\d+)\b", r"\1[\2]", e)
    e = re.sub(r"\bas\s+(usize|i32|isize)\b", "", e)
    return e


def _array_init(ty_expr):
    m = re.match(r"\[\s*(.+?)\s*;\s*(\d+)\s*\]$", ty_expr.strip())
    if not m:
        return None
    v = m.group(1)
    if "(T, T)" in v:
        return "[(0, 0)] * %s" % m.group(2)
    return "[0] * %s" % m.group(2)


def _stmts(body, ind):
    out = []
    for st in _split_top(body, ";"):
        st = st.strip()
        if not st:
            continue
        if st.startswith("assert") or st.startswith("debug_assert"):
            continue
        if st.startswith("{") and st.endswith("}"):
            out.extend(_stmts(st[1:-1], ind))
            continue
        m = re.match(r"let\s+(mut\s+)?(\w+)\s*=\s*\|([^|]*)\|\s*\{(.*)\}$", st, re.S)
        if m:  # closure
            args = ", ".join(a.split(":")[0].strip() for a in m.group(3).split(",") if a.strip())
            out.append(" " * ind + "def %s(%s):" % (m.group(2), args))
            out.extend(_stmts(m.group(4), ind + 4))
            continue
        m = re.match(r"(\w+)\[(\d*)\.\.(\d+)\]\.reverse\(\)$", st)
        if m:
            out.append(" " * ind + "rev(%s, %s, %s)" % (m.group(1), m.group(2) or 0, m.group(3)))
            continue
        m = re.match(r"output\[\.\.(\d+)\]\.copy_from_slice\(&input\[\.\.\d+\]\)$", st)
        if m:
            out.append(" " * ind + "for _k in range(%s): output[_k] = input[_k]" % m.group(1))
            continue
        m = re.match(r"output\[\.\.(\d+)\]\s*\.iter_mut\(\)\s*\.zip\(input\[\.\.\d+\]\.iter\(\)\)\s*"
                     r"\.for_each\(\|\(outp, inp\)\|\s*\*outp\s*=\s*(.*)\)$", st, re.S)
        if m:
            rhs = _expr(m.group(2).replace("* *inp", "* input[_k]").replace("*inp", "input[_k]"))
            out.append(" " * ind + "for _k in range(%s): output[_k] = _chk(%s)" % (m.group(1), rhs))
            continue
        m = re.match(r"let\s+(mut\s+)?(.+?)(\s*:\s*(\[[^=]+\]|\w+))?\s*=\s*(.*)$", st, re.S)
        if m:
            lhs, rhs = m.group(2).strip(), m.group(5)
            init = _array_init(rhs) if m.group(4) else None
            if init is None and rhs.strip().startswith("[") and ";" in rhs:
                init = _array_init(rhs)
            out.append(" " * ind + "%s = %s" % (lhs, init if init else _expr(rhs)))
            continue
        out.append(" " * ind + _expr(st))
    return out


def translate(src, name):
    params, body = _find_fn(src, name)
    lines = ["def %s(%s):" % (name, ", ".join(_param_names(params)))]
    body_lines = _stmts(body, 4)
    tail = body.rstrip()
    if body_lines and not (tail.endswith(";") or tail.endswith("}")):
        # a trailing expression without `;` is the function's value
        body_lines[-1] = "    return " + body_lines[-1].strip()
    lines.extend(body_lines or ["    pass"])
    return "\n".join(lines)


FWD_FUNCS = [
    "butterfly_add", "butterfly_sub", "butterfly_neg", "butterfly_add_asym",
    "butterfly_sub_asym", "butterfly_neg_asym",
    "daala_fdct_ii_2_asym", "daala_fdst_iv_2_asym", "daala_fdct_ii_4", "daala_fdct4",
    "daala_fdst_vii_4", "daala_fdct_ii_2", "daala_fdst_iv_2", "daala_fdct_ii_4_asym",
    "daala_fdst_iv_4_asym", "daala_fdct_ii_8", "daala_fdct8", "daala_fdst_iv_8",
    "daala_fdst8", "daala_fdst_iv_4", "daala_fdct_ii_8_asym", "daala_fdst_iv_8_asym",
    "daala_fdct_ii_16", "daala_fdct16", "daala_fdst_iv_16", "daala_fdst16",
    "daala_fdct_ii_16_asym", "daala_fdst_iv_16_asym", "daala_fdct_ii_32", "daala_fdct32",
    "daala_fdct_ii_32_asym", "daala_fdst_iv_32_asym", "daala_fdct64",
    "fidentity4", "fidentity8", "fidentity16", "fidentity32",
]
INV_FUNCS = [
    "av1_idct4", "av1_iflipadst4", "av1_iadst4", "av1_iidentity4", "av1_idct8",
    "av1_iflipadst8", "av1_iadst8", "av1_iidentity8", "av1_idct16", "av1_iflipadst16",
    "av1_iadst16", "av1_iidentity16", "av1_idct32", "av1_iidentity32", "av1_idct64",
]


def load(ref_root="/root/reference"):
    """Return a namespace with the translated reference functions."""
    ns = dict(globals())
    fwd = _strip_comments(open(ref_root + "/src/transform/forward.rs").read())
    inv = _strip_comments(open(ref_root + "/src/transform/inverse.rs").read())
    # constants used by the inverse kernels (inverse.rs:22-33, mod.rs:52-54)
    for name in ("COSPI_INV", "SINPI_INV"):
        m = re.search(r"static\s+" + name + r"\s*:[^=]*=\s*\[([^\]]*)\]", inv)
        ns[name] = [int(x) for x in m.group(1).replace("\n", " ").split(",") if x.strip()]
    ns["INV_COS_BIT"] = int(re.search(r"const INV_COS_BIT: usize = (\d+);", inv).group(1))
    mod = _strip_comments(open(ref_root + "/src/transform/mod.rs").read())
    for name in ("SQRT2", "INV_SQRT2", "SQRT2_BITS"):
        ns[name] = int(re.search(r"static " + name + r": \w+ = (\d+);", mod).group(1))
    code = []
    for f in FWD_FUNCS:
        code.append(translate(fwd, f))
    for f in INV_FUNCS:
        code.append(translate(inv, f))
    src = "\n\n".join(code)
    exec(compile(src, "<reference-translation>", "exec"), ns)
    ns["__translation__"] = src
    return ns
