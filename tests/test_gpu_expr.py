"""Device expression evaluation pinned to the reference's ExpressionTest answers.

Every case of tests/golden/expr_cases.json (src/common/filter/test/ExpressionTest.cpp, the same fixture
test_oracle_expr.py pins the oracle with) is run on device 0 as a YIELD column and as a WHERE filter of
a GO over a one-edge space, through the JIT kernels and through the interpreter, with the filter pushed
to storage and kept in graphd, and compared with the oracle: value BITS for doubles (not a tolerance),
the column type, the filtered row set, and the error outcome of the FAILED cases.

Math functions: abs/floor/ceil/round/sqrt are correctly rounded on the device; the other libm calls of
the fixture take literal arguments and are evaluated at compile time with the host libm, so they are
glibc's values exactly; the same functions of a row value are refused (NGX_E_UNSUPPORTED) unless the
flag device_libm accepts the device libm (test_libm_of_row_values_*).
"""
import math
import struct

import pytest

from nebula_amd import engine, kvfmt, ngql
from nebula_amd.kvfmt import DOUBLE, INT, STRING
from oracle import oracle
from tests import fixtures
from tests.test_oracle_expr import CASES

pytestmark = pytest.mark.gpu

SPACE, ETYPE, TAG = 7, 11, 21


def one_edge() -> fixtures.Dataset:
    """One part; vertices 1 and 2 with tag t(name, x); one edge 1 -e-> 2 with e(a INT, b DOUBLE, s STRING)
    stored out and in, and 64 edges 3 -e-> 100..163 whose b values sweep doubles for the libm checks."""
    schemas = [fixtures.SchemaDef(False, TAG, "t", [("name", STRING), ("x", INT)]),
               fixtures.SchemaDef(True, ETYPE, "e", [("a", INT), ("b", DOUBLE), ("s", STRING)])]
    b = kvfmt.KVBatch()
    for v, name in ((1, "one"), (2, "two"), (3, "three")):
        b.put(kvfmt.vertex_key(1, v, TAG), kvfmt.encode_row([STRING, INT], [name, v * 10]))

    def edge(src, dst, vals):
        row = kvfmt.encode_row([INT, DOUBLE, STRING], vals)
        b.put(kvfmt.edge_key(1, src, ETYPE, 0, dst), row)
        b.put(kvfmt.edge_key(1, dst, -ETYPE, 0, src), row)

    edge(1, 2, [16, 3.14, "Hello"])
    for k in range(64):
        # awkward doubles: near multiples of pi/4, tiny, huge, negative, integral
        x = (k - 32) * 0.7853981633974483 * (1 + 1e-15 * k) + (1e-300 if k % 7 == 0 else 0.0)
        if k % 9 == 0:
            x = 10.0 ** (k // 4 - 8)
        edge(3, 100 + k, [k - 32, x, WORDS[k % len(WORDS)] + ("%02d" % k if k % 3 else "")])
    for k, num in enumerate(NUMBERS):                 # strings that parse as numbers (casts)
        edge(4, 300 + k, [k, float(k), num])
    for k in range(8):                                # longer than a device builder buffer
        edge(5, 400 + k, [k, 0.0, ("Long Name " * (4 + k))[: 40 + 8 * k]])
    edge(200, 3, [1, 1.0, "  Root "])                 # GO 1 TO 2 STEPS FROM 200: two record hops
    edge(6, 500, [0, 0.0, "1.7976931348623157e308"])   # strtod beyond the exact fast path
    return fixtures.Dataset(space=SPACE, num_parts=1, schemas=schemas, batch=b)


WORDS = ["Hello", " hello ", "  ", "", "MiXeD Case", "abc", "  lead", "trail  ", "a b c", "ZZ top"]
NUMBERS = ["0", "42", "-17", "+8", "  12", "\t-5", "9223372036854775807", "-9223372036854775808",
           "3.25", "-0.5", ".75", "1e3", "2.5E-3", "  7.0", "123456789012", "-0", "0.1", "1.5e10"]


@pytest.fixture(scope="module")
def env():
    ds = one_edge()
    o = oracle.Oracle()
    o.set_flags(threads=2)
    ds.load_oracle(o)
    e = engine.Engine(0)
    ds.load_engine(e)
    yield ds, o, e
    e.close()
    o.close()


def _bits(rows):
    """Cells with doubles as their IEEE bits, so -0.0 / 0.0 and last-place differences count."""
    out = []
    for r in rows:
        t = []
        for kind, v in r:
            if kind in ("float", "double"):
                t.append((kind, struct.pack("<d", float(v)).hex()))
            else:
                t.append((kind, v))
        out.append(tuple(t))
    return sorted(out, key=repr)


def _run(e, ds, s, pushdown):
    try:
        return e.go(ds.space, s, pushdown=pushdown), None
    except engine.EngineError as x:
        return None, x


# functions the device refuses (NGX_E_UNSUPPORTED) in the fixture: none
REFUSED_FUNCS = set()


def _refusal_expected(case):
    return any(f + "(" in case["expr"] for f in REFUSED_FUNCS)


def _sentence(expr, where):
    s = ngql.parse_go("GO FROM 1 OVER e YIELD e._dst")
    if where:
        s.where = expr
    else:
        s.yields = [ngql.YieldCol(expr, "v")]
    return s


def _check_all(env, where, jit, pushdown):
    ds, o, e = env
    e.set_flag("jit", jit)
    bad, refused = [], []
    try:
        for case in CASES:
            s = _sentence(ngql.parse_expr(case["expr"]), where)
            ref = o.go(ds.space, s, pushdown=pushdown)
            got, exc = _run(e, ds, s, pushdown)
            if exc is not None:
                if exc.code == engine.E_UNSUPPORTED and _refusal_expected(case):
                    refused.append(case["line"])
                    continue
                bad.append((case["line"], case["expr"], "raised", exc.code, str(exc)))
                continue
            if got.ok != ref.ok:
                bad.append((case["line"], case["expr"], "ok", got.ok, ref.ok, got.error, ref.error))
            elif ref.ok and (_bits(got.rows) != _bits(ref.rows) or got.col_types != ref.col_types):
                bad.append((case["line"], case["expr"], "rows", got.rows, ref.rows, got.col_types, ref.col_types))
            elif case["op"] == "FAILED" and not where and ref.ok:
                bad.append((case["line"], case["expr"], "oracle did not fail"))
    finally:
        e.set_flag("jit", 1)
    assert not bad, bad[:10]
    return refused


@pytest.mark.parametrize("jit", [1, 0], ids=["jit", "vm"])
def test_expression_cases_as_yield(env, jit):
    _check_all(env, where=False, jit=jit, pushdown=True)


@pytest.mark.parametrize("pushdown", [True, False], ids=["pushed", "graphd"])
@pytest.mark.parametrize("jit", [1, 0], ids=["jit", "vm"])
def test_expression_cases_as_where(env, jit, pushdown):
    _check_all(env, where=True, jit=jit, pushdown=pushdown)


EXACT_OF_ROWS = ["abs(e.b)", "floor(e.b)", "ceil(e.b)", "round(e.b)", "sqrt(abs(e.b))", "sqrt(e.a)",
                 "abs(e.a)", "floor(e.a / 3)", "round(e.b * 2.5)"]
INEXACT_OF_ROWS = ["sin(e.b)", "cos(e.b)", "tan(e.b)", "exp(e.b / 50)", "log(abs(e.b))", "pow(e.b, 2)",
                   "hypot(e.b, e.a)", "cbrt(e.b)", "atan(e.b)", "exp2(e.a)", "log10(abs(e.b))"]


@pytest.mark.parametrize("jit", [1, 0], ids=["jit", "vm"])
def test_libm_exact_functions_of_row_values(env, jit):
    """Correctly rounded functions of row values run on the device and equal glibc bit for bit."""
    ds, o, e = env
    e.set_flag("jit", jit)
    try:
        for f in EXACT_OF_ROWS:
            s = ngql.parse_go(f"GO FROM 3 OVER e YIELD e._dst, {f} AS v")
            ref, got = o.go(ds.space, s), e.go(ds.space, s)
            assert ref.ok and got.ok and len(ref.rows) == 64
            assert _bits(got.rows) == _bits(ref.rows), f
    finally:
        e.set_flag("jit", 1)


def test_libm_of_row_values_refused_by_default(env):
    ds, o, e = env
    assert e.get_flag("device_libm") == 0
    for f in INEXACT_OF_ROWS:
        for q in (f"GO FROM 3 OVER e YIELD {f} AS v", f"GO FROM 3 OVER e WHERE {f} > 0.5 YIELD e._dst"):
            with pytest.raises(engine.EngineError) as x:
                e.go(ds.space, ngql.parse_go(q))
            assert x.value.code == engine.E_UNSUPPORTED, (q, x.value)
    # literal arguments fold on the host: accepted, and glibc's value
    s = ngql.parse_go("GO FROM 3 OVER e YIELD e._dst, sin(0.5) + e.b AS v")
    assert _bits(e.go(ds.space, s).rows) == _bits(o.go(ds.space, s).rows)


def test_libm_of_row_values_with_device_libm(env):
    """device_libm=1: the device libm within 2 ulp of glibc (and equal type/row set)."""
    ds, o, e = env
    e.set_flag("device_libm", 1)
    try:
        for f in INEXACT_OF_ROWS:
            s = ngql.parse_go(f"GO FROM 3 OVER e YIELD e._dst, {f} AS v")
            ref, got = o.go(ds.space, s), e.go(ds.space, s)
            assert ref.ok and got.ok and got.col_types == ref.col_types
            for (gd, gv), (rd, rv) in zip(sorted(got.rows, key=repr), sorted(ref.rows, key=repr)):
                assert gd == rd
                a, b = float(gv[1]), float(rv[1])
                if math.isnan(b) or math.isinf(b):
                    assert repr(a) == repr(b), (f, a, b)
                else:
                    assert abs(a - b) <= 2 * math.ulp(b), (f, a, b)
    finally:
        e.set_flag("device_libm", 0)


STRING_YIELDS = [
    "lower(e.s)", "upper(e.s)", "trim(e.s)", "ltrim(e.s)", "rtrim(e.s)", "left(e.s, 3)", "left(e.s, e.a % 7)",
    "right(e.s, 4)", "right(e.s, e.a)", "lpad(e.s, 12, \"*-\")", "rpad(e.s, 9, \"ab\")", "lpad(e.s, 2, 5)",
    "substr(e.s, 2, 3)", "substr(e.s, -3, 2)", "substr(e.s, e.a, 2)", "e.s + \"!\"", "\"<\" + upper(e.s) + \">\"",
    "(string)e.a", "(string)e.a + e.s", "trim(lower(e.s))", "length(rpad(e.s, 20, \"xyz\"))",
    "lower($^.t.name) + \"/\" + upper($$.t.name)", "(string)(e.a > 0)", "hash(lower(e.s))",
    "(string)(e.a * 1.0)", "(string)floor(e.b)", "(string)(e.a * 0.0)", "(string)(e.a * 1e14)",
    "(string)e.b", "(string)(e.b / 3)", "(string)(e.b * 1e300)", "(string)(e.a / 7.0) + \"|\" + (string)e.b",
]


@pytest.mark.parametrize("jit", [1, 0], ids=["jit", "vm"])
def test_string_functions_of_row_values(env, jit):
    """The string functions over every edge's string (views and builders; four builder columns in one
    YIELD, so the result string arena holds several strings per row), against the oracle."""
    ds, o, e = env
    e.set_flag("jit", jit)
    try:
        for i in range(0, len(STRING_YIELDS), 4):
            cols = ", ".join(f"{x} AS c{j}" for j, x in enumerate(STRING_YIELDS[i:i + 4]))
            s = ngql.parse_go(f"GO FROM 3 OVER e YIELD e._dst, {cols}")
            ref = o.go(ds.space, s)
            got = e.go(ds.space, s)
            assert got.ok == ref.ok, (cols, got.error, ref.error)
            if not ref.ok:                   # lpad(e.s, 2, 5): the pad is read (bad_get) once it is needed
                continue
            assert _bits(got.rows) == _bits(ref.rows), cols
            assert got.col_types == ref.col_types
            cgot = e.go(ds.space, s, columnar=True)
            assert _bits(cgot.rows) == _bits(ref.rows), cols
    finally:
        e.set_flag("jit", 1)


@pytest.mark.parametrize("q", [
    "GO FROM 3 OVER e WHERE lower(e.s) CONTAINS \"hel\" YIELD e._dst, e.s",
    "GO FROM 3 OVER e WHERE trim(e.s) == \"\" YIELD e._dst",
    "GO FROM 3 OVER e WHERE e.s + \"x\" > \"Z\" YIELD e._dst, lpad(e.s, 6, \"0\")",
    "GO FROM 3 OVER e WHERE substr(upper(e.s), 1, 1) == \"A\" || left(e.s, 1) == \" \" YIELD e._dst",
    "GO FROM 3 OVER e YIELD DISTINCT lower(trim(e.s)) AS w",
    "GO 1 TO 2 STEPS FROM 200 OVER e YIELD e._dst, upper(e.s) + (string)e.a AS u",
    "GO FROM 4 OVER e YIELD e._dst, (int)e.s AS i",
    "GO FROM 4 OVER e WHERE (int)e.s > 5 YIELD e._dst",
    "GO FROM 4 OVER e YIELD e._dst, (double)e.s AS d",
])
@pytest.mark.parametrize("jit", [1, 0], ids=["jit", "vm"])
def test_string_queries(env, q, jit):
    """Filters over built strings (pushed and in graphd), DISTINCT over built strings, two record hops
    (two string arenas), and the string -> int / double casts (strtoll / strtod: a FAILED outcome
    where the reference's folly::to throws) against the oracle."""
    ds, o, e = env
    e.set_flag("jit", jit)
    try:
        s = ngql.parse_go(q)
        for pushdown in (True, False):
            ref = o.go(ds.space, s, pushdown=pushdown)
            got, exc = _run(e, ds, s, pushdown)
            assert exc is None, (q, exc)
            assert got.ok == ref.ok, (q, got.error, ref.error)
            if ref.ok:
                assert _bits(got.rows) == _bits(ref.rows), q
    finally:
        e.set_flag("jit", 1)


def test_strings_longer_than_a_builder_buffer_are_refused(env):
    """A built string longer than kStrBuildBytes is a host-only construct (NGX_E_UNSUPPORTED, the caller
    runs its CPU path), never a truncated answer; views of the same strings stay on the device."""
    ds, o, e = env
    for q in ("GO FROM 5 OVER e YIELD upper(e.s)", "GO FROM 5 OVER e YIELD e.s + e.s",
              "GO FROM 5 OVER e WHERE lower(e.s) != \"\" YIELD e._dst",
              "GO FROM 6 OVER e YIELD (double)e.s"):         # 1.79e308: strtod's big-number rounding
        with pytest.raises(engine.EngineError) as x:
            e.go(ds.space, ngql.parse_go(q))
        assert x.value.code == engine.E_UNSUPPORTED, q
    s = ngql.parse_go("GO FROM 5 OVER e YIELD e._dst, trim(e.s), substr(e.s, 5, 30), right(e.s, 50)")
    assert _bits(e.go(ds.space, s).rows) == _bits(o.go(ds.space, s).rows)
