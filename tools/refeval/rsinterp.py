"""A small interpreter for the subset of Rust that rav1e's hot-path
reference functions are written in.

Fixture-generation tool only: it runs in the build container, where
/root/reference exists, and reads the reference's Rust source as TEXT.  A
function is located by name (`load_fn`), parsed into an AST and evaluated
directly -- no translation step, so the statements that run are the
reference's own.  What the interpreter supplies is the *environment*: the
Rust integer semantics (typed wrapping on `as` casts, typed declarations and
typed operands; truncating `/` and `%`), iterator adaptors, slices and raw
pointers over Python lists, and host objects standing in for rav1e's frame
types (`tools/refeval/rshost.py`).  Nothing from the reference is written
into the repository; only the vectors it produces (tests/golden/*).

Supported: fn items (also nested, and generic), let with patterns and
types, if / if let / match / for / while / loop / break / continue / return,
closures, blocks as expressions, struct and tuple-struct literals, impl
blocks (methods and std::ops operator traits), arrays `[v; n]`, ranges,
method chains, `as` casts, turbofish, macros `assert!`/`debug_assert!`
(checked) and `cfg!` (false).
"""
import math

import numpy as np
import re

# ---------------------------------------------------------------- integers
INT_BITS = {"i8": 8, "i16": 16, "i32": 32, "i64": 64, "i128": 128, "isize": 64,
            "u8": 8, "u16": 16, "u32": 32, "u64": 64, "u128": 128, "usize": 64}
FLOATS = ("f32", "f64")


class TInt(int):
    """An integer carrying its Rust type (arithmetic wraps to it)."""

    def __new__(cls, v, ty):
        o = int.__new__(cls, v)
        o.ty = ty
        return o

    def __repr__(self):
        return "%d%s" % (int(self), self.ty)


def wrap(v, ty):
    """Rust `as` / release-mode wrapping to integer type `ty`."""
    if ty is None:
        return v
    if ty in FLOATS:
        return float(v)
    if ty == "bool":
        return bool(v)
    bits = INT_BITS[ty]
    if isinstance(v, (float, np.floating)):  # float -> int `as` saturates, NaN -> 0
        if v != v:
            v = 0
        else:
            v = int(v)  # truncates toward zero
            lo, hi = (0, (1 << bits) - 1) if ty[0] == "u" else (-(1 << (bits - 1)), (1 << (bits - 1)) - 1)
            return TInt(max(lo, min(hi, v)), ty)
    v = int(v) & ((1 << bits) - 1)
    if ty[0] == "i" and v >> (bits - 1):
        v -= 1 << bits
    return TInt(v, ty)


def ty_of(v):
    return getattr(v, "ty", None)


def tdiv(a, b):
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def trem(a, b):
    return a - b * tdiv(a, b)


# ---------------------------------------------------------------- tokenizer
_TOK = re.compile(r"""
 (?P<ws>\s+)|
 (?P<comment>//[^\n]*|/\*.*?\*/)|
 (?P<lifetime>'[A-Za-z_]\w*(?!'))|
 (?P<char>'(?:\\.|[^\\'])')|
 (?P<str>"(?:\\.|[^"\\])*")|
 (?P<num>(?:0x[0-9a-fA-F_]+|0b[01_]+|\d[\d_]*(?:\.\d[\d_]*|\.(?![.\w]))?(?:[eE][+-]?\d+)?)
        (?:_?(?:i8|i16|i32|i64|i128|isize|u8|u16|u32|u64|u128|usize|f32|f64))?)|
 (?P<id>[A-Za-z_]\w*)|
 (?P<punct>\.\.=|\.\.\.|<<=|>>=|::|->|=>|==|!=|<=|>=|&&|\|\||\+=|-=|\*=|/=|%=|\^=|&=|\|=|<<|>>|\.\.|
           [-+*/%^!&|=<>@.,;:\#?(){}\[\]$~])
""", re.S | re.X)


class Tok:
    __slots__ = ("kind", "text")

    def __init__(self, kind, text):
        self.kind, self.text = kind, text

    def __repr__(self):
        return "%s:%s" % (self.kind, self.text)


def tokenize(src):
    out, pos = [], 0
    while pos < len(src):
        m = _TOK.match(src, pos)
        if not m:
            raise SyntaxError("cannot tokenize at %r" % src[pos:pos + 40])
        pos = m.end()
        k = m.lastgroup
        if k in ("ws", "comment"):
            continue
        out.append(Tok(k, m.group(k)))
    out.append(Tok("eof", ""))
    return out


def parse_num(text):
    suf = None
    m = re.match(r"^(.*?)_?(i8|i16|i32|i64|i128|isize|u8|u16|u32|u64|u128|usize|f32|f64)$", text)
    if m and not (text.startswith("0x") and m.group(2)[0] == "f"):
        text, suf = m.group(1), m.group(2)
    body = text.replace("_", "")
    if body.startswith("0x"):
        v = int(body, 16)
    elif body.startswith("0b"):
        v = int(body, 2)
    elif "." in body or "e" in body or "E" in body or suf in FLOATS:
        return np.float32(body) if suf == "f32" else float(body)
    else:
        v = int(body)
    return wrap(v, suf) if suf else v


# ---------------------------------------------------------------- parser
class Parser:
    """Recursive descent over the token list; expressions are tuples."""

    def __init__(self, src):
        self.t = tokenize(src)
        self.i = 0

    # -- token helpers
    def peek(self, k=0):
        return self.t[self.i + k]

    def at(self, text, k=0):
        return self.t[self.i + k].text == text and self.t[self.i + k].kind in ("punct", "id")

    def next(self):
        tok = self.t[self.i]
        self.i += 1
        return tok

    def eat(self, text):
        if self.at(text):
            self.i += 1
            return True
        return False

    def expect(self, text):
        tok = self.next()
        if tok.text != text:
            ctx = " ".join(t.text for t in self.t[max(0, self.i - 12):self.i + 6])
            raise SyntaxError("expected %r got %r near: %s" % (text, tok.text, ctx))
        return tok

    def expect_gt(self):
        tok = self.peek()
        if tok.text == ">":
            self.i += 1
        elif tok.text in (">>", ">=", ">>="):
            tok.text = tok.text[1:]
        else:
            self.expect(">")

    def ident(self):
        tok = self.next()
        if tok.kind != "id":
            raise SyntaxError("expected identifier, got %r" % tok.text)
        return tok.text

    # -- attributes / visibility
    def skip_attrs(self):
        while self.at("#"):
            self.next()
            self.eat("!")
            self.skip_balanced("[", "]")

    def skip_balanced(self, o, c):
        self.expect(o)
        depth = 1
        while depth:
            tok = self.next()
            if tok.text == o:
                depth += 1
            elif tok.text == c:
                depth -= 1
            elif tok.kind == "eof":
                raise SyntaxError("unbalanced " + o)

    def skip_vis(self):
        if self.eat("pub"):
            if self.at("("):
                self.skip_balanced("(", ")")

    # -- types (parsed into a string-ish tuple; only the name matters)
    def parse_type(self):
        if self.eat("&"):
            if self.peek().kind == "lifetime":
                self.next()
            self.eat("mut")
            return ("ref", self.parse_type())
        if self.eat("*"):
            if not self.eat("const"):
                self.expect("mut")
            return ("ptr", self.parse_type())
        if self.at("["):
            self.next()
            el = self.parse_type()
            if self.eat(";"):
                n = self.parse_expr()
                self.expect("]")
                return ("array", el, n)
            self.expect("]")
            return ("slice", el)
        if self.at("("):
            self.next()
            items = []
            while not self.at(")"):
                items.append(self.parse_type())
                if not self.eat(","):
                    break
            self.expect(")")
            return ("tuple", items)
        if self.eat("impl") or self.eat("dyn"):
            return self.parse_bounds()
        if self.at("fn") or self.at("Fn") or self.at("FnMut"):
            self.next()
            self.skip_balanced("(", ")")
            if self.eat("->"):
                self.parse_type()
            return ("fn",)
        segs = []
        if self.eat("<"):  # <T as Trait>::X
            t = self.parse_type()
            if self.eat("as"):
                self.parse_type()
            self.expect_gt()
            segs.append(t)
        else:
            segs.append(self.ident())
        gens = []
        while True:
            if self.at("<"):
                self.next()
                gens = self.parse_generic_args()
            if self.at("::") and self.peek(1).kind == "id":
                self.next()
                segs.append(self.ident())
                continue
            break
        if isinstance(segs[0], str) and len(segs) == 1:
            return ("name", segs[0], gens)
        return ("path", segs, gens)

    def parse_bounds(self):
        t = self.parse_type()
        while self.eat("+"):
            if self.peek().kind == "lifetime":
                self.next()
            else:
                self.parse_type()
        return t

    def parse_generic_args(self):
        args = []
        while not self.at(">") and not self.at(">>") and not self.at(">=") and not self.at(">>="):
            if self.peek().kind == "lifetime":
                self.next()
            elif self.peek().kind == "num" or self.at("{"):
                self.parse_primary()
            else:
                t = self.parse_type()
                if self.eat("="):  # associated type binding
                    t = self.parse_type()
                elif self.at(":"):
                    self.next()
                    self.parse_bounds()
                args.append(t)
            if not self.eat(","):
                break
        self.expect_gt()
        return args

    def parse_generic_params(self):
        names = []
        if not self.eat("<"):
            return names
        while not self.at(">"):
            if self.peek().kind == "lifetime":
                self.next()
                if self.eat(":"):
                    while self.peek().kind == "lifetime" or self.at("+"):
                        self.next()
            else:
                self.eat("const")
                names.append(self.ident())
                if self.eat(":"):
                    self.parse_bounds()
                if self.eat("="):
                    self.parse_type()
            if not self.eat(","):
                break
        self.expect_gt()
        return names

    def skip_where(self):
        if self.eat("where"):
            while not self.at("{") and not self.at(";"):
                if self.peek().kind == "lifetime":
                    self.next()
                else:
                    self.parse_type()
                if self.eat(":"):
                    self.parse_bounds()
                self.eat(",")

    # -- items
    def parse_fn(self):
        self.skip_attrs()
        self.skip_vis()
        for kw in ("const", "unsafe", "extern"):
            if self.eat(kw):
                if kw == "extern" and self.peek().kind == "str":
                    self.next()
        self.expect("fn")
        name = self.ident()
        gens = self.parse_generic_params()
        self.expect("(")
        params = []
        while not self.at(")"):
            self.skip_attrs()
            if self.at("&") and (self.at("self", 1) or self.at("mut", 1)
                                 or self.peek(1).kind == "lifetime"):
                self.next()
                if self.peek().kind == "lifetime":
                    self.next()
                self.eat("mut")
                self.expect("self")
                params.append((("bind", "self", False), None))
            elif self.at("self") or (self.at("mut") and self.at("self", 1)):
                self.eat("mut")
                self.next()
                params.append((("bind", "self", False), None))
            else:
                pat = self.parse_pattern()
                self.expect(":")
                ty = self.parse_type()
                params.append((pat, ty))
            if not self.eat(","):
                break
        self.expect(")")
        ret = None
        if self.eat("->"):
            ret = self.parse_type()
        self.skip_where()
        body = self.parse_block()
        return ("fn", name, gens, params, ret, body)

    # -- patterns
    def parse_pattern(self):
        p = self.parse_pattern1()
        if self.at("|") and not self.no_or_pat:
            alts = [p]
            while self.eat("|"):
                alts.append(self.parse_pattern1())
            return ("or", alts)
        return p

    no_or_pat = False

    def parse_pattern1(self):
        if self.eat("&&"):  # `&&pat`: two reference levels
            self.eat("mut")
            return ("deref", ("deref", self.parse_pattern1()))
        if self.eat("&"):
            self.eat("mut")
            return ("deref", self.parse_pattern1())
        if self.at("("):
            self.next()
            items = []
            while not self.at(")"):
                items.append(self.parse_pattern())
                if not self.eat(","):
                    break
            self.expect(")")
            return items[0] if len(items) == 1 and not self.t[self.i - 2].text == "," else ("tuple", items)
        if self.at("["):
            self.next()
            items = []
            while not self.at("]"):
                items.append(self.parse_pattern())
                if not self.eat(","):
                    break
            self.expect("]")
            return ("tuple", items)
        if self.at("_"):
            self.next()
            return ("wild",)
        if self.at(".."):
            self.next()
            return ("rest",)
        if self.peek().kind in ("num", "char", "str") or self.at("-"):
            neg = self.eat("-")
            v = self.parse_primary()
            if neg:
                v = ("un", "-", v)
            if self.at("..=") or self.at(".."):
                incl = self.next().text == "..="
                hi = self.parse_primary()
                return ("range", v, hi, incl)
            return ("lit", v)
        if self.at("ref"):
            self.next()
        mut = self.eat("mut")
        name = self.ident()
        segs = [name]
        while self.at("::"):
            self.next()
            segs.append(self.ident())
        if self.at("("):
            self.next()
            items = []
            while not self.at(")"):
                items.append(self.parse_pattern())
                if not self.eat(","):
                    break
            self.expect(")")
            return ("tstruct", segs, items)
        if self.at("{"):
            self.next()
            fields = []
            while not self.at("}"):
                if self.eat(".."):
                    continue
                f = self.ident()
                if self.eat(":"):
                    fields.append((f, self.parse_pattern()))
                else:
                    fields.append((f, ("bind", f, False)))
                if not self.eat(","):
                    break
            self.expect("}")
            return ("struct", segs, fields)
        if len(segs) == 1 and not name[0].isupper():
            if self.eat("@"):
                return ("at", name, self.parse_pattern1())
            return ("bind", name, mut)
        return ("const", segs)

    # -- statements / blocks
    def parse_block(self):
        self.expect("{")
        stmts, tail = [], None
        while not self.at("}"):
            # `#[cfg(feature = "...")]` on a statement: the feature is off
            # (rav1e's default build); a braced statement is skipped unparsed
            cfg_off = False
            while self.at("#"):
                j = self.i
                self.skip_attrs()
                if any(x.text == "cfg" for x in self.t[j:self.i]) and \
                        any(x.text == "feature" for x in self.t[j:self.i]):
                    cfg_off = True
            if cfg_off and self.at("{"):
                self.skip_balanced("{", "}")
                continue
            if self.at("}"):
                break
            if self.eat(";"):
                continue
            if self.at("let"):
                self.next()
                pat = self.parse_pattern()
                ty = self.parse_type() if self.eat(":") else None
                init = self.parse_expr() if self.eat("=") else None
                els = None
                if self.eat("else"):
                    els = self.parse_block()
                self.expect(";")
                stmts.append(("let", pat, ty, init, els))
                continue
            if self.at("fn") or (self.at("const") and self.at("fn", 1)) or self.at("pub"):
                stmts.append(("item", self.parse_fn()))
                continue
            if self.at("use"):
                while not self.eat(";"):
                    self.next()
                continue
            if self.at("const") or self.at("static"):
                self.next()
                name = self.ident()
                self.expect(":")
                self.parse_type()
                self.expect("=")
                e = self.parse_expr()
                self.expect(";")
                stmts.append(("let", ("bind", name, False), None, e, None))
                continue
            if self.peek().text in ("if", "match", "for", "while", "loop", "unsafe", "{") \
                    and self.peek().kind in ("id", "punct"):
                e = self.parse_primary()
                if self.at(".") or self.at("?"):
                    e = self.parse_postfix(e)
            else:
                e = self.parse_expr(stmt=True)
            if self.eat(";"):
                stmts.append(("expr", e))
            elif self.at("}"):
                tail = e
            elif e[0] in ("if", "iflet", "match", "for", "while", "whilelet", "loop", "block",
                          "unsafe"):
                stmts.append(("expr", e))
            else:
                self.expect(";")
        self.expect("}")
        return ("block", stmts, tail)

    # -- expressions
    BIN = [
        ("||",), ("&&",), ("==", "!=", "<", ">", "<=", ">="), ("|",), ("^",), ("&",),
        ("<<", ">>"), ("+", "-"), ("*", "/", "%"),
    ]
    ASSIGN = ("=", "+=", "-=", "*=", "/=", "%=", "^=", "&=", "|=", "<<=", ">>=")

    def parse_expr(self, stmt=False, nostruct=False):
        saved = getattr(self, "_nostruct", False)
        self._nostruct = nostruct
        try:
            return self.parse_assign()
        finally:
            self._nostruct = saved

    def parse_assign(self):
        lhs = self.parse_range()
        if self.peek().kind == "punct" and self.peek().text in self.ASSIGN:
            op = self.next().text
            rhs = self.parse_assign()
            return ("assign", op, lhs, rhs)
        return lhs

    def parse_range(self):
        if self.at("..") or self.at("..="):
            incl = self.next().text == "..="
            hi = None
            if not self._range_end():
                hi = self.parse_bin(0)
            return ("range", None, hi, incl)
        lo = self.parse_bin(0)
        if self.at("..") or self.at("..="):
            incl = self.next().text == "..="
            hi = None
            if not self._range_end():
                hi = self.parse_bin(0)
            return ("range", lo, hi, incl)
        return lo

    def _range_end(self):
        tok = self.peek()
        return tok.text in (")", "]", "}", ",", ";") or (tok.text == "{" and self._nostruct)

    def parse_bin(self, lvl):
        if lvl == len(self.BIN):
            return self.parse_cast()
        lhs = self.parse_bin(lvl + 1)
        while self.peek().kind == "punct" and self.peek().text in self.BIN[lvl]:
            op = self.next().text
            rhs = self.parse_bin(lvl + 1)
            lhs = ("bin", op, lhs, rhs)
        return lhs

    def parse_cast(self):
        e = self.parse_unary()
        while self.at("as"):
            self.next()
            e = ("cast", e, self.parse_type())
        return e

    def parse_unary(self):
        if self.at("-"):
            self.next()
            return ("un", "-", self.parse_unary())
        if self.at("!"):
            self.next()
            return ("un", "!", self.parse_unary())
        if self.at("*"):
            self.next()
            return ("deref", self.parse_unary())
        if self.at("&") or self.at("&&"):
            dbl = self.next().text == "&&"
            mut = self.eat("mut")
            e = ("ref", mut, self.parse_unary())
            return ("ref", False, e) if dbl else e
        return self.parse_postfix(self.parse_primary())

    def parse_postfix(self, e):
        while True:
            if self.at("?"):
                self.next()
                e = ("try", e)
            elif self.at("("):
                e = ("call", e, self.parse_args("(", ")"))
            elif self.at("["):
                self.next()
                idx = self.parse_expr()
                self.expect("]")
                e = ("index", e, idx)
            elif self.at("."):
                self.next()
                tok = self.next()
                if tok.kind == "num":
                    if isinstance(parse_num(tok.text), float):  # t.0.1
                        a, b = tok.text.split(".")
                        e = ("field", ("field", e, a), b)
                    else:
                        e = ("field", e, tok.text)
                    continue
                name = tok.text
                gens = []
                if self.at("::"):
                    self.next()
                    self.expect("<")
                    gens = self.parse_generic_args()
                if self.at("("):
                    e = ("mcall", e, name, self.parse_args("(", ")"), gens)
                else:
                    e = ("field", e, name)
            else:
                return e

    def parse_args(self, o, c):
        self.expect(o)
        args = []
        while not self.at(c):
            args.append(self.parse_expr())
            if not self.eat(","):
                break
        self.expect(c)
        return args

    def parse_primary(self):
        tok = self.peek()
        if tok.kind == "num":
            self.next()
            return ("lit", parse_num(tok.text))
        if tok.kind == "str":
            self.next()
            return ("lit", tok.text[1:-1])
        if tok.kind == "char":
            self.next()
            return ("lit", tok.text[1:-1])
        if tok.kind == "lifetime":  # labelled loop
            self.next()
            self.expect(":")
            e = self.parse_primary()
            return e[:-1] + (tok.text,) if e[0] in ("for", "while", "loop") else e
        t = tok.text
        if t == "(":
            self.next()
            items, trailing = [], False
            while not self.at(")"):
                items.append(self.parse_expr())
                trailing = False
                if not self.eat(","):
                    break
                trailing = True
            self.expect(")")
            if len(items) == 1 and not trailing:
                return items[0]
            return ("tuple", items)
        if t == "[":
            self.next()
            if self.at("]"):
                self.next()
                return ("array", [])
            first = self.parse_expr()
            if self.eat(";"):
                n = self.parse_expr()
                self.expect("]")
                return ("arrrep", first, n)
            items = [first]
            while self.eat(","):
                if self.at("]"):
                    break
                items.append(self.parse_expr())
            self.expect("]")
            return ("array", items)
        if t == "{":
            return self.parse_block()
        if t == "unsafe":
            self.next()
            return self.parse_block()
        if t == "if":
            return self.parse_if()
        if t == "match":
            self.next()
            scrut = self.parse_expr(nostruct=True)
            self.expect("{")
            arms = []
            while not self.at("}"):
                self.skip_attrs()
                self.eat("|")
                pat = self.parse_pattern()
                guard = None
                if self.eat("if"):
                    guard = self.parse_expr()
                self.expect("=>")
                body = self.parse_block() if self.at("{") else self.parse_expr()
                arms.append((pat, guard, body))
                self.eat(",")
            self.expect("}")
            return ("match", scrut, arms)
        if t == "for":
            self.next()
            pat = self.parse_pattern()
            self.expect("in")
            it = self.parse_expr(nostruct=True)
            body = self.parse_block()
            return ("for", pat, it, body, None)
        if t == "while":
            self.next()
            if self.eat("let"):
                pat = self.parse_pattern()
                self.expect("=")
                e = self.parse_expr(nostruct=True)
                return ("whilelet", pat, e, self.parse_block(), None)
            cond = self.parse_expr(nostruct=True)
            return ("while", cond, self.parse_block(), None)
        if t == "loop":
            self.next()
            return ("loop", self.parse_block(), None)
        if t in ("break", "continue"):
            self.next()
            label = self.next().text if self.peek().kind == "lifetime" else None
            val = None
            if t == "break" and not self._range_end():
                val = self.parse_expr()
            return (t, val, label)
        if t == "return":
            self.next()
            val = None if self._range_end() else self.parse_expr()
            return ("return", val)
        if t in ("|", "||", "move"):
            return self.parse_closure()
        if t == "<":  # <T as Trait>::item
            self.next()
            ty = self.parse_type()
            if self.eat("as"):
                self.parse_type()
            self.expect_gt()
            segs = [("type", ty)]
            while self.eat("::"):
                segs.append(self.ident())
            return ("path", segs)
        if tok.kind == "id":
            return self.parse_path_expr()
        raise SyntaxError("unexpected token %r near: %s" % (
            t, " ".join(x.text for x in self.t[max(0, self.i - 8):self.i + 8])))

    def parse_if(self):
        self.expect("if")
        if self.eat("let"):
            pat = self.parse_pattern()
            self.expect("=")
            e = self.parse_expr(nostruct=True)
            then = self.parse_block()
            els = self._else()
            return ("iflet", pat, e, then, els)
        cond = self.parse_expr(nostruct=True)
        then = self.parse_block()
        return ("if", cond, then, self._else())

    def _else(self):
        if self.eat("else"):
            if self.at("if"):
                return self.parse_if()
            return self.parse_block()
        return None

    def parse_closure(self):
        self.eat("move")
        params = []
        if self.eat("||"):
            pass
        else:
            self.expect("|")
            saved, self.no_or_pat = self.no_or_pat, True
            while not self.at("|"):
                pat = self.parse_pattern()
                if self.eat(":"):
                    self.parse_type()
                params.append(pat)
                if not self.eat(","):
                    break
            self.no_or_pat = saved
            self.expect("|")
        if self.eat("->"):
            self.parse_type()
        body = self.parse_expr()
        return ("closure", params, body)

    def parse_path_expr(self):
        segs = [self.ident()]
        gens = []
        while self.at("::"):
            self.next()
            if self.at("<"):
                self.next()
                gens = self.parse_generic_args()
                continue
            segs.append(self.ident())
        if self.at("!") and not self.at("=", 1):  # macro
            self.next()
            o = self.peek().text
            c = {"(": ")", "[": "]", "{": "}"}[o]
            if segs[-1] in ("vec",) and o == "[":
                inner = self.parse_primary()
                return ("vec", inner)
            start = self.i
            self.skip_balanced(o, c)
            return ("macro", segs[-1], self.t[start + 1:self.i - 1])
        if self.at("{") and not self._nostruct and (segs[-1][0].isupper() or len(segs) > 1) \
                and segs[-1][0].isupper():
            self.next()
            fields, base = [], None
            while not self.at("}"):
                if self.eat(".."):
                    base = self.parse_expr()
                    break
                f = self.ident() if self.peek().kind == "id" else self.next().text
                if self.eat(":"):
                    fields.append((f, self.parse_expr()))
                else:
                    fields.append((f, ("path", [f])))
                if not self.eat(","):
                    break
            self.expect("}")
            return ("structlit", segs, fields, base)
        if gens:
            return ("path", segs, gens)
        return ("path", segs)


# ---------------------------------------------------------------- runtime values
class Ref:
    """`&mut place` for a scalar place (variable cell or container slot)."""
    __slots__ = ("get", "set")

    def __init__(self, get, set_):
        self.get, self.set = get, set_


def elem_ref(container, idx):
    return Ref(lambda: container[idx], lambda v: container.__setitem__(idx, v))


def deref(v):
    while isinstance(v, Ref):
        v = v.get()
    return v


class Ptr:
    """A raw pointer into a flat Python list."""
    __slots__ = ("base", "off")

    def __init__(self, base, off):
        self.base, self.off = base, off

    def add(self, n):
        return Ptr(self.base, self.off + int(n))

    def offset(self, n):
        return Ptr(self.base, self.off + int(n))

    def sub(self, n):
        return Ptr(self.base, self.off - int(n))

    def read(self):
        return self.base[self.off]


class Slice:
    """`&[T]` / `&mut [T]`: a view [start, end) over a flat Python list."""
    __slots__ = ("base", "start", "end")

    def __init__(self, base, start=0, end=None):
        if isinstance(base, Slice):
            start += base.start
            end = base.start + (end if end is not None else len(base))
            base = base.base
        self.base, self.start = base, start
        self.end = len(base) if end is None else end
        if self.end > len(base) or self.start > self.end or self.start < 0:
            raise IndexError("slice [%d..%d] of %d" % (self.start, self.end, len(base)))

    def __len__(self):
        return self.end - self.start

    def _idx(self, i):
        i = int(i)
        if not 0 <= i < self.end - self.start:
            raise IndexError("index %d out of %d" % (i, self.end - self.start))
        return self.start + i

    def __getitem__(self, i):
        return self.base[self._idx(i)]

    def __setitem__(self, i, v):
        self.base[self._idx(i)] = v

    def sub(self, lo, hi):
        lo = 0 if lo is None else int(lo)
        hi = len(self) if hi is None else int(hi)
        if hi > len(self) or lo > hi:
            raise IndexError("range %d..%d of %d" % (lo, hi, len(self)))
        return Slice(self.base, self.start + lo, self.start + hi)

    def tolist(self):
        return self.base[self.start:self.end]

    def __iter__(self):
        return iter(self.base[self.start:self.end])


def as_slice(v):
    if isinstance(v, Slice):
        return v
    if isinstance(v, list):
        return Slice(v)
    if hasattr(v, "as_slice"):
        return v.as_slice()
    raise TypeError("not a slice: %r" % (type(v),))


class RangeV:
    __slots__ = ("lo", "hi", "incl")

    def __init__(self, lo, hi, incl):
        self.lo, self.hi, self.incl = lo, hi, incl

    def __iter__(self):
        hi = self.hi + 1 if self.incl else self.hi
        ty = ty_of(self.lo) or ty_of(self.hi)
        for v in range(int(self.lo), int(hi)):
            yield TInt(v, ty) if ty else v


class Struct:
    """A struct / tuple-struct / enum-variant value."""

    def __init__(self, name, fields):
        self.__dict__["_name"] = name
        self.__dict__["_f"] = dict(fields)

    def __getattr__(self, k):
        try:
            return self._f[k]
        except KeyError:
            raise AttributeError("%s has no field %s" % (self._name, k))

    def __setattr__(self, k, v):
        self._f[k] = v

    def copy(self):
        return Struct(self._name, dict(self._f))

    def __eq__(self, o):
        return isinstance(o, Struct) and o._name == self._name and o._f == self._f

    def __hash__(self):
        return hash((self._name, tuple(sorted(self._f.items()))))

    def __repr__(self):
        return "%s%r" % (self._name, self._f)


class It:
    """Rust iterator adaptors over a Python iterator."""

    def __init__(self, g):
        self.g = iter(g)

    def __iter__(self):
        return self.g

    def __next__(self):
        return next(self.g)


class Closure:
    def __init__(self, params, body, env, interp):
        self.params, self.body, self.env, self.interp = params, body, env, interp

    def __call__(self, *args):
        env = Env(self.env)
        for p, a in zip(self.params, args):
            self.interp.bind(p, a, env)
        try:
            return self.interp.ev(self.body, env)
        except _Return as r:
            return r.v


class _Break(Exception):
    def __init__(self, v, label):
        self.v, self.label = v, label


class _Continue(Exception):
    def __init__(self, label):
        self.label = label


class _Return(Exception):
    def __init__(self, v):
        self.v = v


class Env:
    __slots__ = ("vars", "parent")

    def __init__(self, parent=None):
        self.vars, self.parent = {}, parent

    def lookup(self, name):
        e = self
        while e is not None:
            if name in e.vars:
                return e
            e = e.parent
        return None

    def get(self, name):
        e = self.lookup(name)
        if e is None:
            raise NameError(name)
        return e.vars[name]


def type_name(ty):
    """The leaf name of a parsed type (for casts / declarations)."""
    if ty is None:
        return None
    if ty[0] == "name":
        return ty[1]
    if ty[0] == "path":
        return ty[1][-1] if isinstance(ty[1][-1], str) else None
    return None


# ---------------------------------------------------------------- interpreter
class Interp:
    def __init__(self, host):
        """host: dict of names (host functions, types, constants)."""
        self.globals = Env()
        self.globals.vars.update(host)
        self.impls = {}  # struct name -> {method: fn}
        self.sources = []  # Source files searched for unknown names

    def resolve(self, name):
        """Load an unknown static/const or free fn `name` from self.sources."""
        for src in self.sources:
            try:
                src.load_static(self, name)
                return True
            except KeyError:
                pass
        for src in self.sources:
            try:
                self.define_fn(src.fn(name))
                return True
            except KeyError:
                pass
        return False

    # -- loading
    def define_fn(self, fn, env=None):
        (env or self.globals).vars[fn[1]] = self.make_fn(fn, env or self.globals)

    def make_fn(self, fn, env):
        _, name, gens, params, ret, body = fn
        interp = self

        def call(*args, **kw):
            fenv = Env(env)
            for g in gens:
                if g in kw.get("generics", {}):
                    fenv.vars[g] = kw["generics"][g]
            fenv.vars.update(kw.get("bind", {}))
            if len(args) != len(params):
                raise TypeError("%s takes %d args, got %d" % (name, len(params), len(args)))
            for (pat, ty), a in zip(params, args):
                if ty is not None and ty[0] == "ref" and pat[0] == "bind" and \
                        isinstance(deref(a), Struct):
                    fenv.vars[pat[1]] = deref(a)  # `&` / `&mut` parameter: the caller's value
                    continue
                tn = type_name(ty)
                a = deref(a) if (tn in INT_BITS or tn in FLOATS) else a
                if tn in INT_BITS and isinstance(a, int) and not isinstance(a, bool):
                    a = wrap(a, tn)
                interp.bind(pat, a, fenv)
            try:
                v = interp.ev(body, fenv)
            except _Return as r:
                v = r.v
            rn = type_name(ret)
            if rn in INT_BITS and isinstance(v, int) and not isinstance(v, bool):
                v = wrap(v, rn)
            return v
        call.__name__ = name
        call.rs_fn = fn
        return call

    def define_impl(self, struct_name, fns):
        tbl = self.impls.setdefault(struct_name, {})
        for fn in fns:
            tbl[fn[1]] = fn

    # -- patterns
    def bind(self, pat, v, env):
        if not self.match(pat, v, env):
            raise ValueError("refutable pattern %r failed on %r" % (pat, v))

    def match(self, pat, v, env):
        k = pat[0]
        if k == "bind":
            if isinstance(v, Struct) and pat[1] != "self":
                v = v.copy()
            env.vars[pat[1]] = v
            return True
        if k == "wild" or k == "rest":
            return True
        if k == "deref":
            return self.match(pat[1], deref(v), env)
        if k == "tuple":
            v = deref(v)
            vals = list(v) if not isinstance(v, Slice) else v.tolist()
            pats = pat[1]
            if any(p[0] == "rest" for p in pats):
                r = [i for i, p in enumerate(pats) if p[0] == "rest"][0]
                head, tail = pats[:r], pats[r + 1:]
                return all(self.match(p, x, env) for p, x in zip(head, vals)) and \
                    all(self.match(p, x, env) for p, x in zip(tail, vals[len(vals) - len(tail):]))
            if len(vals) != len(pats):
                return False
            return all(self.match(p, x, env) for p, x in zip(pats, vals))
        if k == "lit":
            return deref(v) == self.ev(pat[1], env)
        if k == "range":
            v = deref(v)
            lo, hi = self.ev(pat[1], env), self.ev(pat[2], env)
            return lo <= v <= hi if pat[3] else lo <= v < hi
        if k == "or":
            return any(self.match(p, v, env) for p in pat[1])
        if k == "at":
            env.vars[pat[1]] = v
            return self.match(pat[2], v, env)
        if k == "const":
            segs = pat[1]
            if segs == ["None"]:
                return deref(v) is None
            c = self.path_value(segs, env)
            return deref(v) == c
        if k == "tstruct":
            segs, items = pat[1], pat[2]
            v = deref(v)
            if segs[-1] == "Some":
                return v is not None and self.match(items[0], v, env)
            if segs[-1] in ("Ok", "Err"):
                if not (isinstance(v, tuple) and len(v) == 2 and v[0] == segs[-1]):
                    return False
                return self.match(items[0], v[1], env)
            if not isinstance(v, Struct) or v._name.split("::")[-1] != segs[-1]:
                return False
            return all(self.match(p, v._f[str(i)], env) for i, p in enumerate(items))
        if k == "struct":
            v = deref(v)
            if not isinstance(v, Struct):
                return False
            if v._name.split("::")[-1] != pat[1][-1]:
                return False
            return all(self.match(p, v._f[f], env) for f, p in pat[2])
        raise NotImplementedError("pattern " + k)

    # -- paths
    def path_value(self, segs, env):
        first = segs[0]
        if isinstance(first, tuple) and first[0] == "type":
            base = self.type_obj(first[1], env)
        else:
            e = env.lookup(first)
            if e is not None:
                base = e.vars[first]
            elif first in INT_BITS or first in FLOATS:
                base = PrimType(first)
            elif first in ("std", "core", "crate", "self", "super"):
                rest = segs[1:]
                while rest and rest[0] in ("mem", "cmp", "ptr", "num", "u64", "u32", "i32",
                                           "i64", "i16", "u16", "u8", "f64", "usize", "isize",
                                           "f32") and len(rest) > 1:
                    if rest[0] in INT_BITS or rest[0] in FLOATS:
                        return getattr(PrimType(rest[0]), rest[1])
                    if rest[0] == "cmp":
                        return getattr(_Cmp, rest[1])
                    rest = rest[1:]
                return self.path_value(rest, env)
            elif first == "cmp":
                return getattr(_Cmp, segs[1])
            elif self.resolve(first):
                base = self.globals.vars[first]
            else:
                raise NameError("unknown path %s" % "::".join(map(str, segs)))
        for s in segs[1:]:
            if isinstance(base, StructType) and s in self.impls.get(base.name, {}):
                base = self.make_method(base.name, s, None, env)
            else:
                base = getattr(base, s)
        return base

    def type_obj(self, ty, env):
        n = type_name(ty)
        if n in INT_BITS or n in FLOATS:
            return PrimType(n)
        if ty[0] == "path":
            return self.path_value(ty[1], env)
        return env.get(n)

    def make_method(self, sname, mname, recv, env):
        fn = self.impls[sname][mname]
        st = self.globals.vars.get(sname)
        f = self.make_fn(fn, self.globals)
        if recv is None:
            return lambda *a: f(*a, bind={"Self": st})
        return lambda *a: f(recv, *a, bind={"Self": st})

    # -- evaluation
    def ev(self, e, env):
        return getattr(self, "ev_" + e[0])(e, env)

    def ev_lit(self, e, env):
        return e[1]

    def ev_path(self, e, env):
        segs = e[1]
        if len(segs) == 1 and isinstance(segs[0], str):
            if segs[0] == "None":
                return None
            if segs[0] in ("true", "false"):
                return segs[0] == "true"
        return self.path_value(segs, env)

    def ev_block(self, e, env):
        benv = Env(env)
        for st in e[1]:
            if st[0] == "item":
                self.define_fn(st[1], benv)
        for st in e[1]:
            k = st[0]
            if k == "let":
                _, pat, ty, init, els = st
                if init is None:
                    self.bind(pat, None, benv)
                    continue
                v = self.ev(init, benv)
                tn = type_name(ty)
                if tn in INT_BITS and isinstance(v, int) and not isinstance(v, bool):
                    v = wrap(v, tn)
                elif tn in FLOATS and isinstance(v, (int, float)):
                    v = float(v)
                if els is not None:
                    if not self.match(pat, v, benv):
                        self.ev(els, benv)
                else:
                    self.bind(pat, v, benv)
            elif k == "expr":
                self.ev(st[1], benv)
        if e[2] is not None:
            return self.ev(e[2], benv)
        return None

    def ev_unsafe(self, e, env):
        return self.ev(e[1], env)

    def ev_tuple(self, e, env):
        return tuple(deref_scalar(self.ev(x, env)) for x in e[1])

    def ev_array(self, e, env):
        return [deref_scalar(self.ev(x, env)) for x in e[1]]

    def ev_vec(self, e, env):
        v = self.ev(e[1], env)
        return list(v) if isinstance(v, list) else v

    def ev_arrrep(self, e, env):
        v = deref_scalar(self.ev(e[1], env))
        n = int(self.ev(e[2], env))
        if isinstance(v, list):
            return [list(v) for _ in range(n)]
        if isinstance(v, Struct):
            return [v.copy() for _ in range(n)]
        return [v] * n

    def ev_range(self, e, env):
        lo = self.ev(e[1], env) if e[1] is not None else None
        hi = self.ev(e[2], env) if e[2] is not None else None
        return RangeV(deref(lo), deref(hi), e[3])

    def ev_un(self, e, env):
        v = deref(self.ev(e[2], env))
        if e[1] == "-":
            if isinstance(v, (float, np.floating)):
                return -v
            return wrap(-int(v), ty_of(v)) if ty_of(v) else -v
        if isinstance(v, bool):
            return not v
        t = ty_of(v)
        return wrap(~int(v), t) if t else ~v

    def ev_deref(self, e, env):
        v = self.ev(e[1], env)
        if isinstance(v, Ptr):
            return v.read()
        return deref(v)

    def ev_ref(self, e, env):
        inner = e[2]
        if e[1]:  # &mut place of a scalar -> Ref
            if inner[0] == "path" and len(inner[1]) == 1:
                name = inner[1][0]
                scope = env.lookup(name)
                v = scope.vars[name]
                if isinstance(v, (int, float, np.floating, Struct)) or v is None:
                    return Ref(lambda: scope.vars[name], lambda x: scope.vars.__setitem__(name, x))
                return v
            if inner[0] == "index":
                base = self.ev(inner[1], env)
                idx = self.ev(inner[2], env)
                if not isinstance(idx, RangeV):
                    v = index_get(base, idx)
                    if isinstance(v, (int, float, np.floating)):
                        return index_ref(base, idx)
                    return v
        return self.ev(inner, env)

    def ev_cast(self, e, env):
        v = deref(self.ev(e[1], env))
        tn = type_name(e[2])
        if tn in INT_BITS:
            if isinstance(v, bool):
                v = int(v)
            if not isinstance(v, (int, float, np.floating)):
                v = int(v)
            return wrap(v, tn)
        if tn == "f32":  # IEEE single: every later f32 operation rounds (numpy float32)
            return np.float32(v)
        if tn in FLOATS:
            return float(v)
        return v

    def ev_bin(self, e, env):
        op = e[1]
        if op == "&&":
            return bool(deref(self.ev(e[2], env))) and bool(deref(self.ev(e[3], env)))
        if op == "||":
            return bool(deref(self.ev(e[2], env))) or bool(deref(self.ev(e[3], env)))
        a = deref(self.ev(e[2], env))
        b = deref(self.ev(e[3], env))
        return self.binop(op, a, b)

    def binop(self, op, a, b):
        if isinstance(a, Struct):
            meth = {"*": "mul", "+": "add", "-": "sub", "/": "div"}.get(op)
            if meth and meth in self.impls.get(a._name, {}):
                return self.make_method(a._name, meth, a, None)(b)
            if op == "==":
                return a == b
            if op == "!=":
                return a != b
            raise TypeError("no operator %s for %s" % (op, a._name))
        if op in ("==", "!=", "<", ">", "<=", ">="):
            if a is None or b is None:
                return {"==": a is b, "!=": a is not b}[op]
            return {"==": a == b, "!=": a != b, "<": a < b, ">": a > b,
                    "<=": a <= b, ">=": a >= b}[op]
        if isinstance(a, (float, np.floating)) or isinstance(b, (float, np.floating)):
            return {"+": lambda: a + b, "-": lambda: a - b, "*": lambda: a * b,
                    "/": lambda: a / b, "%": lambda: math.fmod(a, b)}[op]()
        if isinstance(a, bool) and isinstance(b, bool) and op in ("&", "|", "^"):
            return {"&": a and b, "|": a or b, "^": a != b}[op]
        ta, tb = ty_of(a), ty_of(b)
        ty = ta if op in ("<<", ">>") else (ta or tb)
        x, y = int(a), int(b)
        if op == "+":
            r = x + y
        elif op == "-":
            r = x - y
        elif op == "*":
            r = x * y
        elif op == "/":
            r = tdiv(x, y)
        elif op == "%":
            r = trem(x, y)
        elif op == "<<":
            r = x << y
        elif op == ">>":
            r = x >> y
        elif op == "&":
            r = x & y
        elif op == "|":
            r = x | y
        elif op == "^":
            r = x ^ y
        else:
            raise NotImplementedError(op)
        if ty:
            return wrap(r, ty)
        return r

    def ev_assign(self, e, env):
        op, lhs, rhs = e[1], e[2], e[3]
        v = deref_scalar(self.ev(rhs, env))
        if op != "=":
            cur = deref(self.ev(lhs, env)) if lhs[0] != "deref" else self.ev(lhs, env)
            cur = deref(cur)
            if isinstance(cur, Struct) and op == "+=":
                meth = self.impls.get(cur._name, {}).get("add_assign")
                if meth:
                    self.make_method(cur._name, "add_assign", cur, env)(v)
                    return None
            v = self.binop(op[:-1], cur, deref(v))
        self.store(lhs, v, env)
        return None

    def store(self, lhs, v, env):
        k = lhs[0]
        if isinstance(v, Struct):
            v = v.copy()
        if k == "path":
            name = lhs[1][0]
            scope = env.lookup(name)
            old = scope.vars[name]
            if isinstance(old, Ref):
                old.set(v)
                return
            t = ty_of(old)
            if t and isinstance(v, int) and not isinstance(v, bool) and not ty_of(v):
                v = wrap(v, t)
            scope.vars[name] = v
        elif k == "deref":
            tgt = self.ev(lhs[1], env)
            if isinstance(tgt, Ref):
                old = tgt.get()
                t = ty_of(old)
                if t and isinstance(v, int) and not ty_of(v):
                    v = wrap(v, t)
                tgt.set(v)
            elif isinstance(tgt, Ptr):
                tgt.base[tgt.off] = v
            elif isinstance(tgt, Struct) and isinstance(v, Struct):
                tgt._f.clear()
                tgt._f.update(v._f)
            else:
                raise TypeError("cannot assign through %r" % (tgt,))
        elif k == "index":
            base = self.ev(lhs[1], env)
            idx = deref(self.ev(lhs[2], env))
            old = index_get(base, idx)
            t = ty_of(old)
            if t and isinstance(v, int) and not isinstance(v, bool) and not ty_of(v):
                v = wrap(v, t)
            index_set(base, idx, v)
        elif k == "field":
            obj = deref(self.ev(lhs[1], env))
            setattr(obj, lhs[2], v)
        else:
            raise NotImplementedError("store to " + k)

    def ev_index(self, e, env):
        base = self.ev(e[1], env)
        idx = self.ev(e[2], env)
        return index_get(base, deref(idx) if not isinstance(idx, RangeV) else idx)

    def ev_field(self, e, env):
        obj = deref(self.ev(e[1], env))
        name = e[2]
        if isinstance(obj, tuple):
            return obj[int(name)]
        return getattr(obj, name)

    def ev_if(self, e, env):
        if deref(self.ev(e[1], env)):
            return self.ev(e[2], env)
        if e[3] is not None:
            return self.ev(e[3], env)
        return None

    def ev_iflet(self, e, env):
        v = self.ev(e[2], env)
        ienv = Env(env)
        if self.match(e[1], v, ienv):
            return self.ev(e[3], ienv)
        if e[4] is not None:
            return self.ev(e[4], env)
        return None

    def ev_match(self, e, env):
        v = self.ev(e[1], env)
        for pat, guard, body in e[2]:
            menv = Env(env)
            if self.match(pat, v, menv) and (guard is None or deref(self.ev(guard, menv))):
                return self.ev(body, menv)
        raise ValueError("no match arm for %r" % (v,))

    def _loop(self, label, it, step):
        for x in it:
            try:
                step(x)
            except _Break as b:
                if b.label is None or b.label == label:
                    return b.v
                raise
            except _Continue as c:
                if c.label is None or c.label == label:
                    continue
                raise
        return None

    def ev_for(self, e, env):
        _, pat, ite, body, label = e
        v = self.ev(ite, env)
        if ite[0] == "ref" and ite[1] and isinstance(deref(v), (Slice, list)):
            # `for x in &mut slice`: IntoIterator for &mut [T] yields &mut T
            s = as_slice(deref(v))
            it = iter([elem_ref(s.base, s.start + i) for i in range(len(s))])
        elif ite[0] == "path" and isinstance(deref(v), list) and \
                any(isinstance(x, Struct) for x in deref(v)):
            # `for x in v` over a variable: an owned collection is moved (a
            # mutation of x is never observed) and a `&mut` one yields &mut
            # T (`for mut c in mv_stack { c.weight += .. }`), so the elements
            # bind by reference instead of as copies
            lst = deref(v)
            it = iter([elem_ref(lst, i) for i in range(len(lst))])
        else:
            it = to_iter(v)

        def step(x):
            lenv = Env(env)
            self.bind(pat, x, lenv)
            self.ev(body, lenv)
        return self._loop(label, it, step)

    def ev_while(self, e, env):
        _, cond, body, label = e

        def gen():
            while deref(self.ev(cond, env)):
                yield None
        return self._loop(label, gen(), lambda _: self.ev(body, env))

    def ev_whilelet(self, e, env):
        _, pat, ve, body, label = e

        def gen():
            while True:
                lenv = Env(env)
                if not self.match(pat, self.ev(ve, env), lenv):
                    return
                yield lenv
        return self._loop(label, gen(), lambda lenv: self.ev(body, lenv))

    def ev_loop(self, e, env):
        def gen():
            while True:
                yield None
        return self._loop(e[2], gen(), lambda _: self.ev(e[1], env))

    def ev_break(self, e, env):
        raise _Break(self.ev(e[1], env) if e[1] is not None else None, e[2])

    def ev_continue(self, e, env):
        raise _Continue(e[2])

    def ev_return(self, e, env):
        raise _Return(self.ev(e[1], env) if e[1] is not None else None)

    def ev_closure(self, e, env):
        return Closure(e[1], e[2], env, self)

    def ev_try(self, e, env):
        return self.ev(e[1], env)

    def ev_structlit(self, e, env):
        segs, fields, base = e[1], e[2], e[3]
        vals = {} if base is None else dict(deref(self.ev(base, env))._f)
        st = None
        try:
            st = self.path_value(segs, env)
        except (NameError, AttributeError):
            pass
        for f, x in fields:
            v = deref_scalar(self.ev(x, env))
            if isinstance(st, StructType) and st.field_types.get(f) in INT_BITS \
                    and isinstance(v, int):
                v = wrap(v, st.field_types[f])
            vals[f] = v
        name = st.name if isinstance(st, StructType) else "::".join(segs)
        return Struct(name, vals)

    def ev_macro(self, e, env):
        name, toks = e[1], e[2]
        if name == "cfg":
            return False
        if name in ("assert", "debug_assert", "assert_eq", "debug_assert_eq", "assert_ne",
                    "debug_assert_ne"):
            if name.startswith("debug_") and getattr(self, "release", False):
                return None  # a release build compiles debug_assert! out
            args = self._macro_args(toks)
            if name.endswith("_eq"):
                a, b = (_eq_norm(deref(self.ev(x, env))) for x in args[:2])
                if a != b:
                    raise AssertionError("%s: %r != %r" % (name, a, b))
            elif name.endswith("_ne"):
                a, b = (deref(self.ev(x, env)) for x in args[:2])
                if a == b:
                    raise AssertionError("%s: %r == %r" % (name, a, b))
            elif not deref(self.ev(args[0], env)):
                raise AssertionError("reference %s! failed" % name)
            return None
        if name in ("unreachable", "unimplemented", "panic", "todo"):
            raise RuntimeError("reference %s!() reached" % name)
        if name in ("eprintln", "println", "format"):
            return ""
        host = getattr(self, "macros", {}).get(name)
        if host is not None:  # a macro the generator supplies (its expansion restated)
            return host(self, self._macro_args(toks), env)
        raise NotImplementedError("macro %s!" % name)

    def _macro_args(self, toks):
        p = Parser("")
        p.t = list(toks) + [Tok("eof", "")]
        p.i = 0
        args = []
        while p.peek().kind != "eof":
            if p.peek().kind == "str":  # message
                break
            args.append(p.parse_expr())
            if not p.eat(","):
                break
        return args

    def ev_call(self, e, env):
        fe = e[1]
        args = [self.ev(a, env) for a in e[2]]
        args = [deref_scalar(a) for a in args]
        if fe[0] == "path":
            segs = fe[1]
            if segs == ["Some"]:
                return args[0]
            if segs in (["Ok"], ["Err"]):
                return (segs[0], args[0])
            f = self.path_value(segs, env)
            if len(fe) > 2 and hasattr(f, "rs_fn"):  # turbofish on a generic fn
                gens = [self.type_obj(g, env) for g in fe[2]]
                return f(*args, generics=dict(zip(f.rs_fn[2], gens)))
        else:
            f = self.ev(fe, env)
        if isinstance(f, StructType):  # tuple-struct constructor
            return Struct(f.name, {str(i): a for i, a in enumerate(args)})
        return f(*args)

    def ev_mcall(self, e, env):
        _, re_, name, ae, gens = e
        recv = self.ev(re_, env)
        args = [deref_scalar(self.ev(a, env)) for a in ae]
        r = deref(recv) if not isinstance(recv, Ptr) else recv
        if isinstance(r, Struct) and name in self.impls.get(r._name, {}):
            return self.make_method(r._name, name, r, env)(*args)
        if isinstance(r, Struct) and "next" in self.impls.get(r._name, {}) and \
                name not in ("unwrap", "expect", "unwrap_or", "is_some", "is_none", "clone"):
            # a struct with its own `impl Iterator` (src/lrf.rs VertPaddedIter):
            # the std adaptors run over its next() (Some(x) = x, None = None)
            nxt = self.make_method(r._name, "next", r, env)

            def items(nxt=nxt):
                while True:
                    o = deref(nxt())
                    if o is None:
                        return
                    yield o
            r = It(items())
        gty = type_name(gens[0]) if gens else None
        return call_method(r, name, args, gty, recv)


def deref_scalar(v):
    """Values of scalar places are copied (Rust `Copy`)."""
    if isinstance(v, Ref):
        x = v.get()
        if isinstance(x, (int, float, bool)) or x is None:
            return v  # keep the reference: callers may write through it
    return v


class _Cmp:
    @staticmethod
    def max(a, b):
        return b if b >= a else a

    @staticmethod
    def min(a, b):
        return a if a <= b else b


class PrimType:
    """`u8`, `i32`, ... used as a path base: `i32::cast_from(x)`."""

    def __init__(self, name):
        self.name = name

    def cast_from(self, v):
        return wrap(deref(v), self.name)

    def from_(self, v):
        return wrap(deref(v), self.name)

    @property
    def MAX(self):
        b = INT_BITS[self.name]
        return wrap((1 << b) - 1 if self.name[0] == "u" else (1 << (b - 1)) - 1, self.name)

    @property
    def MIN(self):
        b = INT_BITS[self.name]
        return wrap(0 if self.name[0] == "u" else -(1 << (b - 1)), self.name)

    def max_value(self):
        return self.MAX

    def min_value(self):
        return self.MIN

    def sqrt(self, v):
        return math.sqrt(v)

    def __getattr__(self, k):
        if k == "from":
            return self.from_
        raise AttributeError(k)


class StructType:
    """A struct type name usable as a path base / tuple constructor."""

    def __init__(self, name, field_types=None, **consts):
        self.name = name
        self.field_types = field_types or {}
        self.__dict__.update(consts)


def _eq_norm(v):
    """assert_eq! operands: slices, arrays and vectors compare element-wise
    (PartialEq of [T] against [T; N] / Vec<T>)."""
    if isinstance(v, Slice):
        v = v.tolist()
    if isinstance(v, (list, tuple)):
        return [_eq_norm(deref(x)) for x in v]
    return v


def to_iter(v):
    v = deref(v)
    if isinstance(v, It):
        return v
    if isinstance(v, (RangeV, list, tuple, Slice)):
        return iter(v)
    if hasattr(v, "__iter__"):
        return iter(v)
    raise TypeError("not iterable: %r" % (type(v),))


def index_get(base, idx):
    base = deref(base)
    if hasattr(base, "index_any"):  # host containers indexed by a struct (FrameBlocks[bo])
        return base.index_any(idx)
    if isinstance(idx, RangeV):
        if hasattr(base, "index_range"):
            return base.index_range(idx)
        s = as_slice(base)
        hi = idx.hi + 1 if (idx.incl and idx.hi is not None) else idx.hi
        return s.sub(idx.lo, hi)
    if hasattr(base, "index_row"):
        return base.index_row(int(idx))
    if isinstance(base, tuple):
        return base[int(idx)]
    return base[int(idx)]


def index_set(base, idx, v):
    base = deref(base)
    base[int(idx)] = v


def index_ref(base, idx):
    base = deref(base)
    if isinstance(base, Slice):
        return elem_ref(base.base, base.start + int(idx))
    return elem_ref(base, int(idx))


# ---------------------------------------------------------------- methods
def _int_method(v, name, args, gty):
    t = ty_of(v) or "i32"
    bits = INT_BITS.get(t, 32)
    if name == "abs":
        return wrap(abs(int(v)), ty_of(v)) if ty_of(v) else abs(v)
    if name == "cmp":  # Ord::cmp -> Ordering as -1 / 0 / 1
        o = int(deref(args[0]))
        return (int(v) > o) - (int(v) < o)
    if name == "min":
        return v if v <= args[0] else args[0]
    if name == "max":
        return v if v >= args[0] else args[0]
    if name == "clamp":
        return max(args[0], min(args[1], v))
    if name == "signum":
        r = (v > 0) - (v < 0)
        return wrap(r, ty_of(v)) if ty_of(v) else r
    if name == "leading_zeros":
        x = int(v) & ((1 << bits) - 1)
        return TInt(bits - x.bit_length(), "u32")
    if name == "trailing_zeros":
        x = int(v) & ((1 << bits) - 1)
        return TInt(bits if x == 0 else (x & -x).bit_length() - 1, "u32")
    if name == "count_ones":
        return TInt(bin(int(v) & ((1 << bits) - 1)).count("1"), "u32")
    if name == "pow":
        return wrap(int(v) ** int(args[0]), ty_of(v))
    if name in ("wrapping_add", "overflowing_add"):
        return wrap(int(v) + int(args[0]), t)
    if name == "wrapping_sub":
        return wrap(int(v) - int(args[0]), t)
    if name == "wrapping_mul":
        return wrap(int(v) * int(args[0]), t)
    if name == "saturating_sub":
        r = int(v) - int(args[0])
        lo = 0 if t[0] == "u" else -(1 << (bits - 1))
        return wrap(max(lo, r), t)
    if name == "saturating_add":
        r = int(v) + int(args[0])
        hi = (1 << bits) - 1 if t[0] == "u" else (1 << (bits - 1)) - 1
        return wrap(min(hi, r), t)
    if name == "is_power_of_two":
        return v > 0 and (int(v) & (int(v) - 1)) == 0
    if name == "align_power_of_two_and_shift":  # util/mod.rs:103-105
        n = int(args[0])
        return wrap((int(v) + (1 << n) - 1) >> n, "usize")
    if name == "align_power_of_two":
        n = int(args[0])
        return wrap((int(v) + (1 << n) - 1) & ~((1 << n) - 1), "usize")
    if name in ("as_", "into", "cast"):  # target type comes from context: untyped
        return wrap(v, gty) if gty in INT_BITS else int(v)
    if name in ("clone", "to_owned"):
        return v
    if name == "is_finite":
        return True
    if name == "ilog":  # ILog::ilog, src/util/mod.rs:227-229
        return TInt(bits - (bits - (int(v) & ((1 << bits) - 1)).bit_length()), "usize")
    if name == "round_shift":  # ISimd::round_shift, src/util/simd.rs:98-100 (one lane)
        n = int(args[0])
        return wrap((int(v) + ((1 << n) >> 1)) >> n, ty_of(v))
    if name == "store_to_slice":  # one-lane SIMD store
        as_slice(args[0])[0] = v
        return None
    raise NotImplementedError("int method " + name)


def _float_method(v, name, args, gty):
    if name == "sqrt":
        return math.sqrt(v)
    if name == "abs":
        return abs(v)
    if name in ("min", "max"):  # f32::min / max: a NaN operand yields the other one
        a = args[0]
        if math.isnan(v):
            return a
        if math.isnan(a):
            return v
        return (min if name == "min" else max)(v, a)
    if name == "log2":
        return np.log2(v) if isinstance(v, np.float32) else math.log2(v)
    if name == "is_finite":
        return math.isfinite(v)
    if name in ("floor", "ceil", "round"):
        return float({"floor": math.floor, "ceil": math.ceil,
                      "round": lambda x: math.floor(x + 0.5) if x >= 0 else -math.floor(-x + 0.5)}[name](v))
    if name == "powi":
        return v ** int(args[0])
    if name == "ln":
        return math.log(v)
    if name in ("as_", "clone", "into"):
        return v
    raise NotImplementedError("float method " + name)


def _iter_method(g, name, args, gty):
    if name in ("iter", "into_iter", "by_ref"):
        return It(g)
    if name == "zip":
        return It(zip(g, to_iter(args[0])))
    if name == "map":
        f = args[0]
        return It(f(x) for x in g)
    if name == "filter":
        f = args[0]
        return It(x for x in g if f(x))
    if name == "filter_map":
        f = args[0]
        return It(y for y in (f(x) for x in g) if y is not None)
    if name == "flat_map":
        f = args[0]
        return It(y for x in g for y in to_iter(f(x)))
    if name == "take":
        n = int(args[0])
        return It(x for _, x in zip(range(n), g))
    if name == "skip":
        n = int(args[0])

        def sk():
            for i, x in enumerate(g):
                if i >= n:
                    yield x
        return It(sk())
    if name == "step_by":
        n = int(args[0])
        return It(x for i, x in enumerate(g) if i % n == 0)
    if name == "enumerate":
        return It((TInt(i, "usize"), x) for i, x in enumerate(g))
    if name == "rev":
        return It(reversed(list(g)))
    if name in ("cloned", "copied"):
        return It(deref(x) for x in g)
    if name == "chain":
        def ch():
            yield from g
            yield from to_iter(args[0])
        return It(ch())
    if name == "sum":
        s = 0
        for x in g:
            s = s + deref(x)
        return wrap(s, gty) if gty in INT_BITS else s
    if name == "product":
        s = 1
        for x in g:
            s = s * deref(x)
        return s
    if name == "count":
        return TInt(sum(1 for _ in g), "usize")
    if name == "for_each":
        f = args[0]
        for x in g:
            f(x)
        return None
    if name == "fold":
        acc, f = args[0], args[1]
        for x in g:
            acc = f(acc, x)
        return acc
    if name in ("collect",):
        return [deref_scalar(x) for x in g]
    if name == "last":
        r = None
        for x in g:
            r = x
        return r
    if name == "next":
        return next(g, None)
    if name == "nth":
        for i, x in enumerate(g):
            if i == int(args[0]):
                return x
        return None
    if name in ("min", "max"):
        vals = [deref(x) for x in g]
        if not vals:
            return None
        return min(vals) if name == "min" else max(vals)
    if name in ("min_by_key", "max_by_key"):
        f = args[0]
        best, bk = None, None
        for x in g:
            k = f(x)
            if best is None or (k < bk if name == "min_by_key" else k >= bk):
                best, bk = x, k
        return best
    if name == "position":
        f = args[0]
        for i, x in enumerate(g):
            if f(x):
                return TInt(i, "usize")
        return None
    if name == "rposition":
        f = args[0]
        vals = list(g)
        for i in range(len(vals) - 1, -1, -1):
            if f(vals[i]):
                return TInt(i, "usize")
        return None
    if name == "any":
        f = args[0]
        return any(f(x) for x in g)
    if name == "all":
        f = args[0]
        return all(f(x) for x in g)
    if name == "find":
        f = args[0]
        for x in g:
            if f(x):
                return x
        return None
    raise NotImplementedError("iterator method " + name)


_OPT = ("map", "unwrap_or", "unwrap", "unwrap_or_else", "is_some", "is_none", "and_then",
        "expect", "unwrap_or_default")


def _some_method(v, name, args):
    """Option::Some(v) methods (Some(x) is represented by x itself)."""
    if name in ("map", "and_then"):
        return args[0](v)
    if name in ("unwrap_or", "unwrap", "unwrap_or_else", "expect", "unwrap_or_default"):
        return v
    return name == "is_some"


def call_method(r, name, args, gty, raw):
    if name in ("is_none", "is_some") and not isinstance(r, (It, RangeV)):  # Option<tuple> too
        return (r is None) == (name == "is_none")
    if name in _OPT and r is not None and not isinstance(r, (It, RangeV, tuple, list, Slice)) \
            and not (name == "unwrap" and not isinstance(r, (int, float, Struct))):
        if not (isinstance(r, int) and type(r) not in (int, TInt, bool) and hasattr(type(r), name)):
            return _some_method(r, name, args)
    if isinstance(r, Ptr):
        return getattr(r, name)(*args)
    if isinstance(r, bool):
        if name == "then":
            return args[0]() if r else None
        raise NotImplementedError("bool method " + name)
    if isinstance(r, int):
        if type(r) not in (int, TInt) and hasattr(type(r), name):  # host enums
            return getattr(r, name)(*args)
        return _int_method(r, name, args, gty)
    if isinstance(r, (float, np.floating)):
        return _float_method(r, name, args, gty)
    if r is None or isinstance(r, tuple) and len(r) == 2 and r[0] in ("Ok", "Err"):
        return _option_method(r, name, args)
    if isinstance(r, (list, Slice)):
        return _slice_method(r, name, args, gty, raw)
    if isinstance(r, tuple) and name in ("unwrap", "expect"):  # Some((a, b)) of max_by_key
        return r
    if isinstance(r, (It, RangeV, tuple)):
        if isinstance(r, RangeV) and name == "contains":
            x = deref(args[0])
            return r.lo <= x <= r.hi if r.incl else r.lo <= x < r.hi
        if isinstance(r, RangeV) and name == "len":
            return TInt(max(0, r.hi - r.lo + (1 if r.incl else 0)), "usize")
        return _iter_method(to_iter(r), name, args, gty)
    if isinstance(r, Struct):
        if name in ("clone", "to_owned"):
            return r.copy()
        if name in ("as_ref", "as_mut", "unwrap", "expect"):  # Some(x) / Arc<x> is x here
            return r
        if name in r._f and callable(r._f[name]):  # host-supplied method
            return r._f[name](*args)
        raise NotImplementedError("%s has no method %s" % (r._name, name))
    m = getattr(r, name, None)
    if m is None and hasattr(r, "as_slice"):  # Deref to a slice
        return _slice_method(r.as_slice(), name, args, gty, raw)
    if m is None:
        if name in ("unwrap", "clone", "as_ref", "as_mut", "as_const", "borrow", "as_u8",
                    "as_u16"):
            return r
        raise NotImplementedError("%r has no method %s" % (type(r).__name__, name))
    return m(*args)


def _option_method(r, name, args):
    if isinstance(r, tuple):  # Result
        ok = r[0] == "Ok"
        if name == "unwrap":
            if not ok:
                raise RuntimeError("unwrap on Err")
            return r[1]
        if name == "unwrap_or_else":
            return r[1] if ok else args[0](r[1])
        if name == "is_ok":
            return ok
        raise NotImplementedError("Result." + name)
    if name == "map":
        return None
    if name == "unwrap_or":
        return args[0]
    if name == "unwrap_or_else":
        return args[0]()
    if name == "is_some":
        return False
    if name == "is_none":
        return True
    raise NotImplementedError("Option(None)." + name)


class OptSome:
    pass


def _slice_method(r, name, args, gty, raw):
    if isinstance(r, list) and name == "push":
        r.append(args[0])
        return None
    if isinstance(r, list) and name == "extend":  # Vec / ArrayVec::extend
        r.extend(list(to_iter(deref(args[0]))))
        return None
    s = as_slice(r)
    if name == "len":
        return TInt(len(s), "usize")
    if name == "is_empty":
        return len(s) == 0
    if name in ("iter", "into_iter"):
        return It(iter(s.tolist()))
    if name == "iter_mut":
        return It(elem_ref(s.base, s.start + i) for i in range(len(s)))
    if name in ("chunks", "chunks_mut", "chunks_exact", "chunks_exact_mut"):
        n = int(args[0])
        stop = len(s) - (len(s) % n if "exact" in name else 0)
        return It(s.sub(i, min(i + n, len(s))) for i in range(0, stop, n))
    if name in ("split_at", "split_at_mut"):
        n = int(args[0])
        return (s.sub(0, n), s.sub(n, len(s)))
    if name == "copy_from_slice" or name == "clone_from_slice":
        src = as_slice(deref(args[0]))
        if len(src) != len(s):
            raise ValueError("copy_from_slice length mismatch")
        vals = src.tolist()
        for i, v in enumerate(vals):
            s.base[s.start + i] = v
        return None
    if name == "fill":
        for i in range(len(s)):
            s.base[s.start + i] = args[0]
        return None
    if name == "as_ptr" or name == "as_mut_ptr":
        return Ptr(s.base, s.start)
    if name == "swap":
        a, b = s.start + int(args[0]), s.start + int(args[1])
        s.base[a], s.base[b] = s.base[b], s.base[a]
        return None
    if name == "reverse":
        vals = s.tolist()[::-1]
        s.base[s.start:s.end] = vals
        return None
    if name == "get_unchecked" or name == "get_unchecked_mut":
        return s[args[0]]
    if name == "binary_search":
        x = deref(args[0])
        vals = s.tolist()
        lo, hi = 0, len(vals)
        while lo < hi:
            mid = (lo + hi) // 2
            if vals[mid] < x:
                lo = mid + 1
            else:
                hi = mid
        if lo < len(vals) and vals[lo] == x:
            return ("Ok", TInt(lo, "usize"))
        return ("Err", TInt(lo, "usize"))
    if name in ("to_vec", "to_owned", "clone"):
        return s.tolist()
    if name == "sort_by":  # stable, like slice::sort_by; the closure returns an Ordering
        import functools
        vals = s.tolist()
        vals.sort(key=functools.cmp_to_key(lambda a, b: int(args[0](a, b))))
        for i, x in enumerate(vals):
            s.base[s.start + i] = x
        return None
    if name == "first":
        return s[0] if len(s) else None
    if name == "last":
        return s[len(s) - 1] if len(s) else None
    if name == "contains":
        return deref(args[0]) in s.tolist()
    return _iter_method(iter(s.tolist()), name, args, gty)


# ---------------------------------------------------------------- source access
def _strip(src):
    return re.sub(r"//[^\n]*", "", src)


def find_item(src, kind, name, after=0):
    """Text span of `fn name` / `impl ... for name` / `static name` in src."""
    if kind == "fn":
        pat = r"\bfn\s+" + re.escape(name) + r"\b"
    elif kind == "impl":
        pat = r"\bimpl\b[^{;]*\b" + re.escape(name) + r"\b[^{;]*\{"
    else:
        pat = r"\b(?:static|const)\s+" + re.escape(name) + r"\s*:"
    m = re.compile(pat).search(src, after)
    if not m:
        raise KeyError("%s %s" % (kind, name))
    # back up over attributes / qualifiers on the same item
    start = m.start()
    if kind == "fn":
        line0 = src.rfind("\n", 0, start) + 1
        start = line0
    if kind == "static":
        end = src.index(";", src.index("=", m.end()))
        # the value may contain `;` inside `[x; n]` -> balance brackets
        eq = src.index("=", m.end())
        depth, k = 0, eq + 1
        while True:
            ch = src[k]
            if ch in "([{":
                depth += 1
            elif ch in ")]}":
                depth -= 1
            elif ch == ";" and depth == 0:
                end = k
                break
            k += 1
        return src[start:end + 1]
    b0 = src.index("{", m.end() - 1 if kind == "impl" else m.end())
    depth, k = 0, b0
    while True:
        ch = src[k]
        if ch == "{":
            depth += 1
        elif ch == "}":
            depth -= 1
            if depth == 0:
                break
        k += 1
    return src[start:k + 1]


def parse_fn_text(text):
    p = Parser(text)
    return p.parse_fn()


def parse_impl_fns(text):
    """fns of an `impl ... { ... }` block (associated types/consts skipped)."""
    body = text[text.index("{") + 1:text.rindex("}")]
    p = Parser(body)
    fns = []
    while p.peek().kind != "eof":
        p.skip_attrs()
        if p.at("type") or p.at("const") and not p.at("fn", 1):
            while not p.eat(";"):
                p.next()
            continue
        if p.peek().kind == "eof":
            break
        fns.append(p.parse_fn())
    return fns


def parse_static(text):
    """(name, value expression) of a static/const item."""
    p = Parser(text)
    p.skip_attrs()
    p.skip_vis()
    p.next()  # static / const
    name = p.ident()
    p.expect(":")
    ty = p.parse_type()
    p.expect("=")
    return name, ty, p.parse_expr()


def typed_value(v, ty):
    """Apply a declared type (e.g. of a static) to a literal value tree."""
    if ty is None:
        return v
    if ty[0] == "array" or ty[0] == "slice":
        return [typed_value(x, ty[1]) for x in v] if isinstance(v, list) else v
    if ty[0] == "ref":
        return typed_value(v, ty[1])
    if ty[0] == "tuple" and isinstance(v, tuple):
        return tuple(typed_value(x, t) for x, t in zip(v, ty[1]))
    tn = type_name(ty)
    if tn in INT_BITS and isinstance(v, int) and not isinstance(v, bool):
        return wrap(v, tn)
    return v


class Source:
    """A reference source file read as text (comments stripped)."""

    def __init__(self, path):
        self.path = path
        self.raw = open(path).read()
        self.src = _strip(self.raw)

    def fn(self, name, after_text=None):
        after = self.src.index(after_text) if after_text else 0
        return parse_fn_text(find_item(self.src, "fn", name, after))

    def impl(self, name, after_text=None):
        after = self.src.index(after_text) if after_text else 0
        return parse_impl_fns(find_item(self.src, "impl", name, after))

    def static(self, name):
        return parse_static(find_item(self.src, "static", name))

    def load_static(self, interp, name):
        """Evaluate a static/const item into interp's globals (typed)."""
        n, ty, e = self.static(name)
        interp.globals.vars[n] = typed_value(interp.ev(e, interp.globals), ty)
        return interp.globals.vars[n]

    def line_of(self, name):
        m = re.search(r"\bfn\s+" + re.escape(name) + r"\b", self.raw)
        return self.raw[:m.start()].count("\n") + 1
