"""Pipes and variables around GO: `GO ... | GO FROM $-.col ...` and `$v = GO ...; GO FROM $v.col ...`.

Host-side restatement of the graphd pieces that chain GO sentences (the traversal itself runs in the
library, include/nebula_gn.h ngx_go with input_* set):
  - PipeExecutor (src/graph/PipeExecutor.cpp:21-130): the left sentence's InterimResult feeds the
    right one; `A | (B | C)` nests (parser.yy:1298-1314);
  - AssignmentExecutor / VariableHolder: `$v = <sentence>` keeps the result under the name;
    SequentialSentences (parser.yy:2054-2070) run `;`-separated sentences in order, the last one's
    result is the response;
  - GoExecutor::setupInterimResult (GoExecutor.cpp:990-1068): the interim schema takes each
    column's calculateExprType, or for UNKNOWN the variant type of the first record;
  - YieldClauseWrapper::prepare (TraverseExecutor.cpp:344-392): `$-.*` / `$v.*` in YIELD expands to
    every input column.
Only GO sentences are traversal sentences here (the other executors are outside the GO path).
`backend` is an Engine (the product) or the oracle's Oracle: both take `go(space, s, input=...)`.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

from . import ngql

T_UNKNOWN, T_BOOL, T_INT, T_VID, T_FLOAT, T_DOUBLE, T_STRING, T_TIMESTAMP = 0, 1, 2, 3, 4, 5, 6, 21
_KIND_TYPE = {"bool": T_BOOL, "int": T_INT, "id": T_INT, "timestamp": T_INT, "float": T_DOUBLE,
              "double": T_DOUBLE, "str": T_STRING}


@dataclass
class Interim:
    """InterimResult (src/graph/InterimResult.h): column names, schema types, rows of typed cells
    ((kind, value) pairs as GoResult.rows holds them)."""
    names: List[str]
    types: List[int] = field(default_factory=list)
    rows: List[tuple] = field(default_factory=list)

    @staticmethod
    def from_result(names: Sequence[str], col_types: Sequence[int], rows: Sequence[tuple]) -> "Interim":
        if not rows:
            return Interim(list(names))
        types = []
        for i, t in enumerate(col_types):
            if t == T_UNKNOWN:                                    # GoExecutor.cpp:1008-1026
                kind, v = rows[0][i]
                t = T_BOOL if kind == "empty" and v is not None else _KIND_TYPE.get(kind, T_UNKNOWN)
            types.append(t)
        return Interim(list(names), types, list(rows))


class PipelineError(Exception):
    pass


def _split(text: str, sep: str) -> List[str]:
    """Split at `sep' outside quotes and parentheses; a `|' of `||' is not a pipe."""
    out, depth, quote, cur, i = [], 0, None, [], 0
    while i < len(text):
        ch = text[i]
        if quote:
            cur.append(ch)
            if ch == "\\" and i + 1 < len(text):
                cur.append(text[i + 1])
                i += 1
            elif ch == quote:
                quote = None
        elif ch in "\"'":
            quote = ch
            cur.append(ch)
        elif ch == "(":
            depth += 1
            cur.append(ch)
        elif ch == ")":
            depth -= 1
            cur.append(ch)
        elif ch == sep and depth == 0 and not (sep == "|" and (text[i + 1:i + 2] == "|" or text[i - 1:i] == "|")):
            out.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
        i += 1
    out.append("".join(cur))
    return out


def _unwrap(text: str) -> str:
    """`( piped )' -> `piped' when the parentheses enclose the whole sentence."""
    t = text.strip()
    while t.startswith("(") and t.endswith(")"):
        depth = 0
        for i, ch in enumerate(t):
            depth += ch == "("
            depth -= ch == ")"
            if depth == 0 and i < len(t) - 1:
                return t
        t = t[1:-1].strip()
    return t


def expand_input_star(s: ngql.GoSentence, names: Optional[Sequence[str]], var: str = "") -> None:
    """YieldClauseWrapper::needAllPropsFromInput / needAllPropsFromVar: `$-.*` / `$v.*` -> one
    column per input column."""
    cols = []
    for y in s.yields:
        e = y.expr
        if isinstance(e, ngql.Prop) and e.prop == "*" and e.kind in (ngql.K_INPUT_PROP, ngql.K_VAR_PROP):
            if names is None:
                raise PipelineError("Inputs nullptr." if e.kind == ngql.K_INPUT_PROP else
                                    "Variable `%s' not defined." % e.alias)
            for n in names:
                cols.append(ngql.YieldCol(ngql.Prop(e.kind, e.ref, e.alias, n)))
            continue
        cols.append(y)
    s.yields = cols


@dataclass
class Outcome:
    ok: bool
    error: str = ""
    names: List[str] = field(default_factory=list)
    col_types: List[int] = field(default_factory=list)
    rows: List[tuple] = field(default_factory=list)


class Pipeline:
    """Runs nGQL text made of GO sentences, pipes, parentheses, `$v = ...' and `;'."""

    def __init__(self, backend, space: int, edge_names: Sequence[str] = (), **go_kw):
        self.backend = backend
        self.space = space
        self.edge_names = list(edge_names)
        self.go_kw = go_kw
        self.variables: Dict[str, Interim] = {}

    def _go(self, text: str, inp: Optional[Interim]) -> Outcome:
        try:
            s = ngql.parse_go(text)
        except (SyntaxError, ValueError) as e:
            return Outcome(False, "SyntaxError: %s" % e)
        feed = None
        if s.from_type == 1:
            feed = inp if inp is not None else Interim([])
        elif s.from_type == 2:
            if s.from_var not in self.variables:
                return Outcome(False, "Variable `%s' not defined" % s.from_var)
            feed = self.variables[s.from_var]
        # `$v.*` reads the variable; `$-.*` the pipe input
        star_var = next((e.alias for y in s.yields for e in [y.expr]
                         if isinstance(e, ngql.Prop) and e.kind == ngql.K_VAR_PROP and e.prop == "*"), None)
        try:
            if star_var is not None:
                v = self.variables.get(star_var)
                expand_input_star(s, v.names if v else None, star_var)
            expand_input_star(s, inp.names if inp is not None else None)
        except PipelineError as e:
            return Outcome(False, str(e))
        names = s.column_names(self.edge_names)
        r = self.backend.go(self.space, s, input=feed, **self.go_kw)
        if not r.ok:
            return Outcome(False, r.error, names)
        return Outcome(True, "", names, list(r.col_types), list(r.rows))

    def _yield_constant(self, text: str) -> Outcome:
        """A YIELD sentence with no input (YieldExecutor::executeConstant, YieldExecutor.cpp:343-379):
        one row of its constant expressions (integer literals, hash(...), their negation, and string /
        bool / double literals), typed as Collector::getSchema types the values; it is the left side
        of `YIELD <vid> AS id | GO FROM $-.id ...` (GoTest.cpp:3083-3088)."""
        p = ngql.Parser(text)
        p.expect("kw", "YIELD")
        names, row = [], []
        while True:
            e = p.expression()
            alias = p.label() if p.accept("kw", "AS") else ""
            try:
                v = ngql.eval_const(e)
            except ValueError:
                if not isinstance(e, ngql.Prim):
                    raise PipelineError("only constant YIELD sentences run in this path: " + text[:40])
                v = e.value
            names.append(alias or e.to_string())
            if isinstance(v, bool):
                row.append(("bool", v))
            elif isinstance(v, int):
                row.append(("int", v))
            elif isinstance(v, float):
                row.append(("double", v))
            else:
                row.append(("str", v))
            if not p.accept("op", ","):
                break
        p.expect("eof")
        types = [_KIND_TYPE[k] for k, _ in row]
        return Outcome(True, "", names, types, [tuple(row)])

    def _piped(self, text: str, inp: Optional[Interim]) -> Outcome:
        parts = _split(text, "|")
        cur = inp
        out = None
        for i, part in enumerate(parts):
            body = _unwrap(part)
            if len(_split(body, "|")) > 1:
                out = self._piped(body, cur)                      # ( set_sentence ) as a traverse sentence
            elif body.upper().startswith("YIELD") and cur is None:
                out = self._yield_constant(body)
            else:
                if not body.upper().startswith("GO"):
                    raise PipelineError("only GO sentences run in this path: " + body[:40])
                out = self._go(body, cur)
            if not out.ok:
                return out
            if i + 1 < len(parts):
                cur = Interim.from_result(out.names, out.col_types, out.rows)
        return out

    def run(self, text: str) -> Outcome:
        out = Outcome(True)
        for stmt in _split(text, ";"):
            stmt = stmt.strip()
            if not stmt:
                continue
            var = None
            if stmt.startswith("$"):
                head, eq, rest = stmt.partition("=")
                if eq and head.strip()[1:].isidentifier():
                    var, stmt = head.strip()[1:], rest.strip()
            out = self._piped(stmt, None)
            if not out.ok:
                return out
            if var is not None:
                self.variables[var] = Interim.from_result(out.names, out.col_types, out.rows)
        return out


def run(backend, space: int, text: str, edge_names: Sequence[str] = (), **go_kw) -> Outcome:
    return Pipeline(backend, space, edge_names, **go_kw).run(text)
