"""nGQL expression / GO-sentence front end (host side).

The reference parses nGQL with bison (src/parser/parser.yy) and ships WHERE / YIELD expressions
between graphd and storaged in the binary Expression encoding (src/common/filter/Expressions.cpp:
93-116, per-kind encoders :159-199, :450-507, :572-605, :697-711, :779-792, :1002-1021,
:1155-1176, :1249-1268). This module restates the grammar subset the GO path uses
(parser.yy:331-583 expressions, :585-785 GO clauses) and produces that exact encoding, so callers
can hand `Expression.encode()` bytes to the C-ABI (include/nebula_gn.h) the same way graphd hands
`filter` bytes to StorageService.getBound.
"""
from __future__ import annotations

import re
import struct
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

# Expression::Kind (src/common/filter/Expressions.h:386-407)
K_PRIMARY, K_FUNC, K_UNARY, K_CAST, K_ARITH, K_REL, K_LOGIC = 1, 2, 3, 4, 5, 6, 7
K_SRC_PROP, K_EDGE_RANK, K_EDGE_DST, K_EDGE_SRC, K_EDGE_TYPE, K_ALIAS = 8, 9, 10, 11, 12, 13
K_VAR_PROP, K_DST_PROP, K_INPUT_PROP, K_UUID = 14, 15, 16, 17

UNARY_OPS = {"+": 0, "-": 1, "!": 2}                       # UnaryExpression::Operator
ARITH_OPS = {"+": 0, "-": 1, "*": 2, "/": 3, "%": 4, "^": 5}
REL_OPS = {"<": 0, "<=": 1, ">": 2, ">=": 3, "==": 4, "!=": 5, "CONTAINS": 6}
LOGIC_OPS = {"&&": 0, "||": 1, "XOR": 2}
CAST_TYPES = {"int": 0, "string": 1, "double": 2, "bool": 3, "timestamp": 4}   # ColumnType


def _s16(s: str) -> bytes:
    b = s.encode()
    return struct.pack("<H", len(b)) + b


class Expr:
    def encode(self) -> bytes:
        raise NotImplementedError

    def props(self):
        """(kind, alias, prop) of every property reference, in traversal order."""
        return []

    def to_string(self) -> str:
        """Expression::toString (Expressions.cpp): the column name of an un-aliased YIELD column
        (GoExecutor::getResultColumnNames, GoExecutor.cpp:976-987)."""
        raise NotImplementedError


@dataclass
class Prim(Expr):
    value: object
    kind = K_PRIMARY

    def encode(self):
        v = self.value
        if isinstance(v, bool):
            return bytes([K_PRIMARY, 2, 1 if v else 0])
        if isinstance(v, int):
            return bytes([K_PRIMARY, 0]) + struct.pack("<q", v)
        if isinstance(v, float):
            return bytes([K_PRIMARY, 1]) + struct.pack("<d", v)
        return bytes([K_PRIMARY, 3]) + _s16(v)

    def to_string(self):
        v = self.value
        if isinstance(v, bool):
            return "true" if v else "false"
        if isinstance(v, int):
            return str(v)
        if isinstance(v, float):
            return "%.15f" % v
        return v


@dataclass
class Prop(Expr):
    """Alias.prop and relatives: $^.tag.p, $$.tag.p, $-.p, $var.p, e._dst/_src/_rank/_type."""
    kind: int
    ref: str
    alias: str
    prop: str

    def encode(self):
        return bytes([self.kind]) + _s16(self.ref) + _s16(self.alias) + _s16(self.prop)

    def props(self):
        return [(self.kind, self.alias, self.prop)]

    def to_string(self):                                          # Expressions.cpp:118-137
        out = self.ref
        if self.ref not in ("", "$"):
            out += "."
        out += self.alias
        if self.alias:
            out += "."
        return out + self.prop


@dataclass
class Func(Expr):
    name: str
    args: List[Expr]
    kind = K_FUNC

    def encode(self):
        out = bytes([K_FUNC]) + _s16(self.name) + struct.pack("<H", len(self.args))
        return out + b"".join(a.encode() for a in self.args)

    def props(self):
        return [p for a in self.args for p in a.props()]

    def to_string(self):
        return self.name + "(" + ",".join(a.to_string() for a in self.args) + ")"


@dataclass
class Unary(Expr):
    op: int
    operand: Expr
    kind = K_UNARY

    def encode(self):
        return bytes([K_UNARY, self.op]) + self.operand.encode()

    def props(self):
        return self.operand.props()

    def to_string(self):
        return "+-!"[self.op] + "(" + self.operand.to_string() + ")"


@dataclass
class Cast(Expr):
    ctype: int
    operand: Expr
    kind = K_CAST

    def encode(self):
        return bytes([K_CAST, self.ctype]) + self.operand.encode()

    def props(self):
        return self.operand.props()

    def to_string(self):
        return "(" + ("int", "string", "double", "bool", "timestamp")[self.ctype % 5] + ")" + self.operand.to_string()


@dataclass
class Binary(Expr):
    kind: int
    op: int
    left: Expr
    right: Expr

    def encode(self):
        return bytes([self.kind, self.op]) + self.left.encode() + self.right.encode()

    def props(self):
        return self.left.props() + self.right.props()

    def to_string(self):
        names = {K_ARITH: ("+", "-", "*", "/", "%", "^"), K_REL: ("<", "<=", ">", ">=", "==", "!=", " CONTAINS "),
                 K_LOGIC: ("&&", "||", "XOR")}[self.kind]
        o = names[self.op] if self.op < len(names) else "?"
        return "(" + self.left.to_string() + o + self.right.to_string() + ")"


# ------------------------------------------------------------------------------ std::hash
def std_hash_bytes(data: bytes, seed: int = 0xC70F6907) -> int:
    """libstdc++ std::_Hash_bytes (64-bit) — std::hash<std::string> used for NBA vids
    (src/graph/test/TraverseTestBase.h:125) and the hash() function (FunctionManager.cpp:439-465)."""
    mask = (1 << 64) - 1
    mul = (0xC6A4A793 << 32) + 0x5BD1E995

    def shift_mix(v):
        return v ^ (v >> 47)

    n = len(data)
    aligned = n & ~7
    h = (seed ^ (n * mul)) & mask
    for i in range(0, aligned, 8):
        d = int.from_bytes(data[i:i + 8], "little")
        d = (shift_mix((d * mul) & mask) * mul) & mask
        h ^= d
        h = (h * mul) & mask
    if n & 7:
        d = 0
        for b in reversed(data[aligned:]):
            d = (d << 8) + b
        h ^= d
        h = (h * mul) & mask
    h = (shift_mix(h) * mul) & mask
    h = shift_mix(h)
    return h


def to_i64(u: int) -> int:
    u &= (1 << 64) - 1
    return u - (1 << 64) if u >= (1 << 63) else u


def nebula_hash(s: str) -> int:
    return to_i64(std_hash_bytes(s.encode()))


# ------------------------------------------------------------------------------ lexer
_TOKEN = re.compile(r"""
    (?P<ws>\s+)
  | (?P<double>(?:\d+\.\d*|\.\d+)(?:[eE][-+]?\d+)?|\d+[eE][-+]?\d+)
  | (?P<hex>0[xX][0-9a-fA-F]+)
  | (?P<int>\d+)
  | (?P<str>"(?:[^"\\]|\\.)*"|'(?:[^'\\]|\\.)*')
  | (?P<ref>\$\^|\$\$|\$-)
  | (?P<var>\$[A-Za-z_][A-Za-z0-9_]*)
  | (?P<op><=|>=|==|!=|&&|\|\||->|[<>+\-*/%^!(),.@:])
  | (?P<name>[A-Za-z_][A-Za-z0-9_]*)
""", re.X)

KEYWORDS = {"GO", "STEPS", "TO", "FROM", "OVER", "REVERSELY", "BIDIRECT", "WHERE", "YIELD",
            "DISTINCT", "AS", "AND", "OR", "XOR", "NOT", "CONTAINS", "TRUE", "FALSE", "UUID",
            "INT", "DOUBLE", "STRING", "BOOL", "TIMESTAMP"}


@dataclass
class Tok:
    kind: str
    text: str


def tokenize(src: str) -> List[Tok]:
    out, pos = [], 0
    while pos < len(src):
        m = _TOKEN.match(src, pos)
        if not m:
            raise SyntaxError(f"bad token at {src[pos:pos + 20]!r}")
        pos = m.end()
        k = m.lastgroup
        if k == "ws":
            continue
        t = m.group(k)
        if k == "name" and t.upper() in KEYWORDS:
            out.append(Tok("kw", t.upper()))
        else:
            out.append(Tok(k, t))
    out.append(Tok("eof", ""))
    return out


def _unescape(s: str) -> str:
    body = s[1:-1]
    return re.sub(r"\\(.)", lambda m: {"n": "\n", "t": "\t", "r": "\r"}.get(m.group(1), m.group(1)), body)


class Parser:
    def __init__(self, src: str):
        self.toks = tokenize(src)
        self.i = 0

    # helpers
    def peek(self, k=0) -> Tok:
        return self.toks[min(self.i + k, len(self.toks) - 1)]

    def take(self) -> Tok:
        t = self.toks[self.i]
        self.i += 1
        return t

    def accept(self, kind, text=None) -> Optional[Tok]:
        t = self.peek()
        if t.kind == kind and (text is None or t.text == text):
            return self.take()
        return None

    def expect(self, kind, text=None) -> Tok:
        t = self.accept(kind, text)
        if t is None:
            raise SyntaxError(f"expected {text or kind}, got {self.peek().text!r}")
        return t

    def is_op(self, text):
        t = self.peek()
        return t.kind == "op" and t.text == text

    def is_kw(self, text):
        t = self.peek()
        return t.kind == "kw" and t.text == text

    def label(self) -> str:
        t = self.peek()
        if t.kind == "name" or (t.kind == "kw" and t.text not in ("AND", "OR", "XOR", "NOT", "CONTAINS")):
            self.take()
            return t.text if t.kind == "name" else t.text.lower()
        raise SyntaxError(f"expected a name, got {t.text!r}")

    # expression := logic_xor                                   parser.yy:574-583
    def expression(self) -> Expr:
        e = self.logic_or()
        while self.is_kw("XOR"):
            self.take()
            e = Binary(K_LOGIC, LOGIC_OPS["XOR"], e, self.logic_or())
        return e

    def logic_or(self):
        e = self.logic_and()
        while self.is_op("||") or self.is_kw("OR"):
            self.take()
            e = Binary(K_LOGIC, LOGIC_OPS["||"], e, self.logic_and())
        return e

    def logic_and(self):
        e = self.equality()
        while self.is_op("&&") or self.is_kw("AND"):
            self.take()
            e = Binary(K_LOGIC, LOGIC_OPS["&&"], e, self.equality())
        return e

    def equality(self):
        e = self.relational()
        while self.is_op("==") or self.is_op("!="):
            op = self.take().text
            e = Binary(K_REL, REL_OPS[op], e, self.relational())
        return e

    def relational(self):
        e = self.additive()
        while True:
            t = self.peek()
            if t.kind == "op" and t.text in ("<", ">", "<=", ">="):
                self.take()
                e = Binary(K_REL, REL_OPS[t.text], e, self.additive())
            elif t.kind == "kw" and t.text == "CONTAINS":
                self.take()
                e = Binary(K_REL, REL_OPS["CONTAINS"], e, self.additive())
            else:
                return e

    def additive(self):
        e = self.multiplicative()
        while self.is_op("+") or self.is_op("-"):
            op = self.take().text
            e = Binary(K_ARITH, ARITH_OPS[op], e, self.multiplicative())
        return e

    def multiplicative(self):
        e = self.arith_xor()
        while self.is_op("*") or self.is_op("/") or self.is_op("%"):
            op = self.take().text
            e = Binary(K_ARITH, ARITH_OPS[op], e, self.arith_xor())
        return e

    def arith_xor(self):
        e = self.unary()
        while self.is_op("^"):
            self.take()
            e = Binary(K_ARITH, ARITH_OPS["^"], e, self.unary())
        return e

    def unary(self):                                              # parser.yy:471-485
        if self.is_op("+"):
            self.take()
            return Unary(UNARY_OPS["+"], self.unary())
        if self.is_op("!") or self.is_kw("NOT"):
            self.take()
            return Unary(UNARY_OPS["!"], self.unary())
        if self.is_op("(") and self.peek(1).kind == "kw" and self.peek(1).text.lower() in CAST_TYPES \
                and self.peek(2).kind == "op" and self.peek(2).text == ")":
            self.take()
            ct = CAST_TYPES[self.take().text.lower()]
            self.take()
            return Cast(ct, self.unary())
        return self.primary()

    def primary(self):                                            # parser.yy:331-344
        if self.is_op("-"):
            self.take()
            t = self.peek()
            if t.kind in ("int", "hex"):
                self.take()
                return Prim(-int(t.text, 0))
            return Unary(UNARY_OPS["-"], self.base())
        return self.base()

    def base(self):                                               # parser.yy:346-382
        t = self.peek()
        if t.kind in ("int", "hex"):
            self.take()
            v = int(t.text, 0)
            if v > (1 << 63) - 1:
                raise SyntaxError("integer out of range")
            return Prim(v)
        if t.kind == "double":
            self.take()
            return Prim(float(t.text))
        if t.kind == "str":
            self.take()
            return Prim(_unescape(t.text))
        if t.kind == "kw" and t.text in ("TRUE", "FALSE"):
            self.take()
            return Prim(t.text == "TRUE")
        if t.kind == "ref":
            self.take()
            if t.text == "$-":
                if self.accept("op", "."):
                    if self.accept("op", "*"):
                        return Prop(K_INPUT_PROP, "$-", "", "*")
                    return Prop(K_INPUT_PROP, "$-", "", self.label())
                return Prop(K_INPUT_PROP, "$-", "", "id")
            self.expect("op", ".")
            tag = self.label()
            self.expect("op", ".")
            prop = self.label()
            return Prop(K_SRC_PROP if t.text == "$^" else K_DST_PROP, t.text, tag, prop)
        if t.kind == "var":
            self.take()
            name = t.text[1:]
            if self.accept("op", "."):
                if self.accept("op", "*"):
                    return Prop(K_VAR_PROP, "$", name, "*")
                return Prop(K_VAR_PROP, "$", name, self.label())
            return Prop(K_VAR_PROP, "$", name, "id")
        if self.is_op("("):
            self.take()
            e = self.expression()
            self.expect("op", ")")
            return e
        if t.kind == "kw" and t.text == "UUID":
            raise SyntaxError("uuid() needs the storage UUID service and is not supported")
        if t.kind in ("name", "kw"):
            name = self.label()
            if self.is_op("("):                                   # function call
                self.take()
                args = []
                if not self.is_op(")"):
                    args.append(self.expression())
                    while self.accept("op", ","):
                        args.append(self.expression())
                self.expect("op", ")")
                return Func(name, args)
            if self.is_op("."):                                   # alias_ref_expression
                self.take()
                prop = self.label()
                special = {"_type": K_EDGE_TYPE, "_src": K_EDGE_SRC, "_dst": K_EDGE_DST, "_rank": K_EDGE_RANK}
                if prop in special:
                    return Prop(special[prop], "", name, prop)
                return Prop(K_ALIAS, "", name, prop)
            return Prim(name)                                     # bare name_label -> string
        raise SyntaxError(f"unexpected token {t.text!r}")


def parse_expr(src: str) -> Expr:
    p = Parser(src)
    e = p.expression()
    p.expect("eof")
    return e


def eval_const(e: Expr) -> object:
    """Evaluate a constant FROM-list item the way GoExecutor::prepareFrom does (integers, hash())."""
    if isinstance(e, Prim):
        return e.value
    if isinstance(e, Func) and e.name == "hash" and len(e.args) == 1:
        v = eval_const(e.args[0])
        if isinstance(v, str):
            return nebula_hash(v)
        if isinstance(v, bool):
            return int(v)
        if isinstance(v, int):
            return v                       # std::hash<int64_t> is the identity in libstdc++
        raise ValueError("hash() of a double is not supported in FROM")
    if isinstance(e, Unary) and e.op == UNARY_OPS["-"]:
        return -eval_const(e.operand)
    raise ValueError("FROM accepts integer literals and hash(...) only")


# ------------------------------------------------------------------------------ GO sentence
FORWARD, REVERSELY, BIDIRECT = 0, 1, 2


@dataclass
class YieldCol:
    expr: Expr
    alias: str = ""


@dataclass
class GoSentence:
    """Parsed `GO [M TO] N STEPS FROM ... OVER ... [WHERE ...] [YIELD [DISTINCT] ...]`."""
    record_from: int = 1
    record_to: int = 1
    vids: List[int] = field(default_factory=list)
    over: List[Tuple[str, str]] = field(default_factory=list)     # (edge name, alias or "")
    over_all: bool = False
    direction: int = FORWARD
    where: Optional[Expr] = None
    distinct: bool = False
    yields: List[YieldCol] = field(default_factory=list)
    # FROM $-.col / $var.col (GoExecutor fromType_, GoExecutor.cpp:149-180): 0 literal vids, 1 $-, 2 $var
    from_type: int = 0
    from_var: str = ""
    from_col: str = ""

    def column_names(self, edge_names: Sequence[str] = ()) -> List[str]:
        """getResultColumnNames (GoExecutor.cpp:976-987): alias, else the expression text. OVER *
        without YIELD yields `<edge>._dst' per edge of the space (`edge_names', schema order)."""
        if not self.yields and self.over_all:
            return [n + "._dst" for n in edge_names]
        return [y.alias if y.alias else y.expr.to_string() for y in self.yields]


def parse_go(src: str) -> GoSentence:
    p = Parser(src)
    s = GoSentence()
    p.expect("kw", "GO")
    # step_clause (parser.yy:610-625)
    if p.peek().kind == "int":
        a = int(p.take().text)
        if p.accept("kw", "TO"):
            b = int(p.expect("int").text)
            if a > b:
                raise SyntaxError("Invalid step range")
            s.record_from, s.record_to = a, b
        else:
            s.record_from = s.record_to = a
        p.expect("kw", "STEPS")
    # from_clause (:626-656)
    p.expect("kw", "FROM")
    t = p.peek()
    if t.kind == "ref" and t.text == "$-" or t.kind == "var":      # from_clause: input_ref / var_ref
        p.take()
        p.expect("op", ".")
        col = "*" if p.accept("op", "*") else p.label()
        s.from_type, s.from_var, s.from_col = (1, "", col) if t.kind == "ref" else (2, t.text[1:], col)
    while s.from_type == 0:
        if p.peek().kind in ("ref", "var"):
            raise SyntaxError("FROM accepts vids, $-.col or $var.col")
        e = p.primary() if p.is_op("-") or p.is_op("+") else p.base()
        if isinstance(e, Unary) and e.op == UNARY_OPS["+"]:
            e = e.operand
        v = eval_const(e)
        if isinstance(v, bool) or not isinstance(v, int):
            raise SyntaxError("Vertex ID should be of type integer")
        s.vids.append(v)
        if not p.accept("op", ","):
            break
    # over_clause (:681-733)
    p.expect("kw", "OVER")
    if p.accept("op", "*"):
        s.over_all = True
    else:
        while True:
            name = p.label()
            alias = ""
            if p.accept("kw", "AS"):
                alias = p.label()
            s.over.append((name, alias))
            if not p.accept("op", ","):
                break
    if p.accept("kw", "REVERSELY"):
        s.direction = REVERSELY
    elif p.accept("kw", "BIDIRECT"):
        s.direction = BIDIRECT
    if p.accept("kw", "WHERE"):
        s.where = p.expression()
    if p.accept("kw", "YIELD"):
        if p.accept("kw", "DISTINCT"):
            s.distinct = True
        while True:
            e = p.expression()
            alias = ""
            if p.accept("kw", "AS"):
                alias = p.label()
            s.yields.append(YieldCol(e, alias))
            if not p.accept("op", ","):
                break
    else:                                                         # parser.yy:592-604
        for name, _ in s.over:
            s.yields.append(YieldCol(Prop(K_EDGE_DST, "", name, "_dst")))
    p.expect("eof")
    return s
