"""Pipes and variables through the oracle (FROM $-.col / $var.col: VertexBackTracker, getRoots,
rowsOfVids; src/graph/GoExecutor.cpp:471-509, :675-718, :1317-1330) against the reference GoTest
answers (tests/golden/gotest_cases.py PIPE_CASES), with filter pushdown on and off; column names
(getResultColumnNames) from the host pipeline checked against the oracle's Expression::toString."""
import pytest

from nebula_amd import ngql, pipeline
from oracle import oracle
from tests import fixtures
from tests.golden.gotest_cases import PIPE_CASES


@pytest.fixture(scope="module")
def nba():
    ds = fixtures.nba()
    o = oracle.Oracle()
    ds.load_oracle(o)
    return ds, o


def check(out, case):
    if case.get("error"):
        assert not out.ok
        return
    assert out.ok, out.error
    got = fixtures.normalize_cells(out.rows)
    if case.get("empty"):
        assert got == []
        return
    assert sorted(got, key=repr) == fixtures.nba_expected(case["rows"])
    if "names" in case:
        assert out.names == case["names"]


@pytest.mark.parametrize("pushdown", [True, False])
@pytest.mark.parametrize("case", PIPE_CASES, ids=[f"L{c['line']}" for c in PIPE_CASES])
def test_pipe_known_answers(nba, case, pushdown):
    ds, o = nba
    out = pipeline.run(o, ds.space, fixtures.nba_query(case["query"]), ["serve", "like", "teammate"], pushdown=pushdown)
    check(out, case)


@pytest.mark.parametrize("case", PIPE_CASES, ids=[f"L{c['line']}" for c in PIPE_CASES])
def test_column_names_match_oracle(nba, case):
    """Each GO's column names (Expression::toString of un-aliased YIELD columns) as the oracle's
    restated GoExecutor reports them."""
    ds, o = nba
    names = []

    class Spy:
        def go(self, space, s, input=None, **kw):
            r = o.go(space, s, input=input, **kw)
            if r.ok and r.column_names:
                names.append((s.column_names(["serve", "like", "teammate"]), r.column_names))
            return r

    pipeline.run(Spy(), ds.space, fixtures.nba_query(case["query"]), ["serve", "like", "teammate"])
    for mine, theirs in names:
        assert mine == theirs


def test_expression_to_string_matches_oracle():
    for src in ["$-.name", "$var.x", "$^.player.name", "$$.team.name", "like._dst", "e.p0 + 3 * 2",
                "udf_is_in($-.id, 1, 123)", "(int)$-.x", "!($-.a == 1) && e.b > 2.5", "-e.p0", "\"abc\" != $-.s",
                "true XOR false", "e.s CONTAINS \"x\""]:
        e = ngql.parse_expr(src)
        assert e.to_string() == oracle.expr_to_string(e.encode()), src


def test_split_pipes_and_or():
    assert pipeline._split("GO FROM 1 OVER e WHERE a || b | GO FROM $-.x OVER e", "|") == \
        ["GO FROM 1 OVER e WHERE a || b ", " GO FROM $-.x OVER e"]
    assert pipeline._split("A | (B | C)", "|") == ["A ", " (B | C)"]
    assert pipeline._split("A WHERE s == \"x|y\" | B", "|") == ["A WHERE s == \"x|y\" ", " B"]
    assert pipeline._unwrap(" ( B | C ) ") == "B | C"
    assert pipeline._unwrap("(a) + (b)") == "(a) + (b)"


def test_interim_types_from_first_record():
    """setupInterimResult: UNKNOWN columns take the first record's variant type."""
    it = pipeline.Interim.from_result(["a", "b", "c"], [0, 3, 0], [(("int", 1), ("id", 2), ("str", "x"))])
    assert it.types == [pipeline.T_INT, pipeline.T_VID, pipeline.T_STRING]
    assert pipeline.Interim.from_result(["a"], [0], []).types == []
