"""Generate the entropy-coder tables (data only) for the device tokenizer, the
host range coder and the oracle, from the reference's own table text.

Run in the build container (needs /root/reference):
    python tools/refeval/gen_ec_tables.py

The default coefficient CDFs (src/token_cdfs.rs) and the inter transform-type
CDFs (src/entropymode.rs default_inter_ext_tx_cdf) are normative AV1 data; this
script reads their `static` initialisers as text, expands rav1e's `cdf!` /
`cdf_size!` macros (src/util/mod.rs:21-29: `cdf!(a, b, ..)` is
`[32768 - a, 32768 - b, .., 0, 0]`, the last entry being the adaptation
counter) and the `[x; n]` repeat form, and writes one flat u16 table per
coefficient q context (`CDFContext::new`, src/context.rs:793-850) with the
offset of every CDF family.  The small context tables of
write_coeffs_lv_map (src/context.rs:101-372: eob_to_pos_*, k_eob_*,
av1_nz_map_ctx_offset, av1_tx_ind, tx_set_index_inter, num_tx_set) are read
the same way.

Outputs:
  rav1e_amd/csrc/rv_ec_tables.h   device + host tables of the product
  oracle/orc_ec_tables.h          the same data for the CPU oracle
"""
import os
import re

REF = "/root/reference/src"
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))

# constants the initialisers name (src/context.rs:82, 240-242; src/entropymode.rs:21)
CONSTS = {"CDFMAX": 32768, "TX_TYPES": 16, "NUM_BASE_LEVELS": 2, "BR_CDF_SIZE": 4,
          "TX_SIZE_SQR_CONTEXTS": 4}


def strip_comments(s):
    s = re.sub(r"/\*.*?\*/", "", s, flags=re.S)
    return re.sub(r"//[^\n]*", "", s)


def static_text(src, name):
    m = re.search(r"static\s+" + name + r"\s*:", src)
    assert m, name
    i = src.index("=", m.end())
    # the initialiser: from '=' to the matching ';' at bracket depth 0
    depth, j = 0, i + 1
    while True:
        c = src[j]
        if c in "([{":
            depth += 1
        elif c in ")]}":
            depth -= 1
        elif c == ";" and depth == 0:
            break
        j += 1
    return src[i + 1:j]


class P:
    """Rust array literal -> nested Python lists (ints)."""

    def __init__(self, s):
        self.t = re.findall(r"[A-Za-z_][A-Za-z_0-9]*!?|\d+|[\[\](),;*+\-]", s)
        self.i = 0

    def peek(self):
        return self.t[self.i] if self.i < len(self.t) else None

    def eat(self, x):
        assert self.t[self.i] == x, (self.t[self.i - 5:self.i + 5], x)
        self.i += 1

    def value(self):
        if self.peek() == "[":
            self.eat("[")
            items = []
            if self.peek() == "]":
                self.eat("]")
                return items
            first = self.value()
            if self.peek() == ";":  # [x; n]
                self.eat(";")
                n = self.expr()
                self.eat("]")
                return [first if not isinstance(first, list) else _deep(first) for _ in range(n)]
            items.append(first)
            while self.peek() == ",":
                self.eat(",")
                if self.peek() == "]":
                    break
                items.append(self.value())
            self.eat("]")
            return items
        if self.peek() == "cdf!":
            self.eat("cdf!")
            self.eat("(")
            vals = [self.expr()]
            while self.peek() == ",":
                self.eat(",")
                if self.peek() == ")":
                    break
                vals.append(self.expr())
            self.eat(")")
            return [32768 - v for v in vals] + [0, 0]
        return self.expr()

    def expr(self):
        v = self.term()
        while self.peek() in ("+", "-"):
            op = self.t[self.i]
            self.i += 1
            w = self.term()
            v = v + w if op == "+" else v - w
        return v

    def term(self):
        v = self.atom()
        while self.peek() == "*":
            self.i += 1
            v *= self.atom()
        return v

    def atom(self):
        t = self.t[self.i]
        self.i += 1
        if t == "(":
            v = self.expr()
            self.eat(")")
            return v
        if t == "-":
            return -self.atom()
        if t == "cdf_size!":
            self.eat("(")
            v = self.expr()
            self.eat(")")
            return v + 1
        if t.isdigit():
            return int(t)
        if t in CONSTS:
            return CONSTS[t]
        if t.startswith("TX_CLASS_"):
            return {"TX_CLASS_2D": 0, "TX_CLASS_HORIZ": 1, "TX_CLASS_VERT": 2}[t]
        raise KeyError(t)


def _deep(v):
    return [_deep(x) for x in v] if isinstance(v, list) else v


def parse_static(src, name):
    return P(static_text(src, name)).value()


def flat(v):
    if isinstance(v, list):
        out = []
        for x in v:
            out += flat(x)
        return out
    return [v]


# (name, static, per-qctx?) in the flat-table order; every CDF keeps its
# counter slot, so a family of shape [..][n + 1] is stored as is
FAMILIES = [
    ("TXB_SKIP", "av1_default_txb_skip_cdfs", (5, 13), 3),
    ("EOB16", "av1_default_eob_multi16_cdfs", (2, 2), 6),
    ("EOB32", "av1_default_eob_multi32_cdfs", (2, 2), 7),
    ("EOB64", "av1_default_eob_multi64_cdfs", (2, 2), 8),
    ("EOB128", "av1_default_eob_multi128_cdfs", (2, 2), 9),
    ("EOB256", "av1_default_eob_multi256_cdfs", (2, 2), 10),
    ("EOB512", "av1_default_eob_multi512_cdfs", (2, 2), 11),
    ("EOB1024", "av1_default_eob_multi1024_cdfs", (2, 2), 12),
    ("EOB_EXTRA", "av1_default_eob_extra_cdfs", (5, 2, 9), 3),
    ("BASE_EOB", "av1_default_coeff_base_eob_multi_cdfs", (5, 2, 4), 4),
    ("BASE", "av1_default_coeff_base_multi_cdfs", (5, 2, 42), 5),
    ("BR", "av1_default_coeff_lps_multi_cdfs", (5, 2, 21), 5),
    ("DC_SIGN", "av1_default_dc_sign_cdfs", (2, 3), 3),
]


def main():
    tok = strip_comments(open(os.path.join(REF, "token_cdfs.rs")).read())
    em = strip_comments(open(os.path.join(REF, "entropymode.rs")).read())
    ctx = strip_comments(open(os.path.join(REF, "context.rs")).read())
    tables = [[] for _ in range(4)]
    offs = {}
    for name, st, shape, n in FAMILIES:
        v = parse_static(tok, st)
        assert len(v) == 4, name
        offs[name] = len(tables[0])
        for q in range(4):
            f = flat(v[q])
            total = n
            for d in shape:
                total *= d
            assert len(f) == total, (name, len(f), total)
            tables[q] += f
    # inter_tx_cdf [TX_SETS_INTER = 4][TX_SIZE_SQR_CONTEXTS = 4][17] (no q context)
    itx = parse_static(em, "default_inter_ext_tx_cdf")
    f = flat(itx)
    assert len(f) == 4 * 4 * 17, len(f)
    offs["INTER_TX"] = len(tables[0])
    for q in range(4):
        tables[q] += f
    total = len(tables[0])
    assert total < (1 << 13), total
    small = {
        "num_tx_set": ("uint8_t", parse_static(ctx, "num_tx_set")),
        "tx_set_index_inter": ("int8_t", parse_static(ctx, "tx_set_index_inter")),
        "av1_tx_ind": ("uint8_t", flat(parse_static(ctx, "av1_tx_ind"))),
        "eob_to_pos_small": ("uint8_t", parse_static(ctx, "eob_to_pos_small")),
        "eob_to_pos_large": ("uint8_t", parse_static(ctx, "eob_to_pos_large")),
        "k_eob_group_start": ("uint16_t", parse_static(ctx, "k_eob_group_start")),
        "k_eob_offset_bits": ("uint16_t", parse_static(ctx, "k_eob_offset_bits")),
        "av1_nz_map_ctx_offset": ("int8_t", flat(parse_static(ctx, "av1_nz_map_ctx_offset"))),
    }
    assert len(small["av1_nz_map_ctx_offset"][1]) == 19 * 25
    assert len(small["av1_tx_ind"][1]) == 9 * 16

    def emit(path, prefix, device):
        q = "__constant__ " if device else ""
        lines = ["/* Generated by tools/refeval/gen_ec_tables.py from the reference's table",
                 " * text: the default coefficient CDFs (src/token_cdfs.rs) per coefficient q",
                 " * context and default_inter_ext_tx_cdf (src/entropymode.rs:764-), in rav1e's",
                 " * stored form (32768 - cdf, terminal 0, adaptation counter), plus the",
                 " * context tables of write_coeffs_lv_map (src/context.rs:101-372).  Data only.",
                 " */",
                 "#pragma once", "#include <stdint.h>", ""]
        for name, _, shape, n in FAMILIES:
            lines.append("#define %s_EC_%s %d  /* [%s][%d] */" % (
                prefix, name, offs[name], "][".join(str(d) for d in shape), n))
        lines.append("#define %s_EC_INTER_TX %d  /* [4][4][17] */" % (prefix, offs["INTER_TX"]))
        lines.append("#define %s_EC_TOTAL %d" % (prefix, total))
        lines.append("")
        lines.append("static const uint16_t %s_EC_DEFAULT_CDF[4][%d] = {" % (prefix, total))
        for t in tables:
            lines.append("  {")
            for i in range(0, total, 16):
                lines.append("    " + ", ".join(str(v) for v in t[i:i + 16]) + ",")
            lines.append("  },")
        lines.append("};")
        for name, (ty, vals) in small.items():
            lines.append("static %s%s %s_%s[%d] = {%s};" % (
                q if device else "const ", ty, prefix, name, len(vals), ", ".join(str(v) for v in vals)))
        with open(path, "w") as fh:
            fh.write("\n".join(lines) + "\n")

    emit(os.path.join(ROOT, "rav1e_amd", "csrc", "rv_ec_tables.h"), "RV", True)
    emit(os.path.join(ROOT, "oracle", "orc_ec_tables.h"), "ORC", False)
    print("ec tables: %d u16 per q context" % total)


if __name__ == "__main__":
    main()
