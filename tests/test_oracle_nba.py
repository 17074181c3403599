"""Oracle pin: the restated GoExecutor against the reference GoTest answers on the NBA fixture
(src/graph/test/GoTest.cpp, tests/golden/gotest_cases.py). GoTest runs every case with
filter_pushdown on and off (GoTest.cpp:20-31, :3111); so does this test."""
import pytest

from nebula_amd import ngql
from oracle import oracle
from tests import fixtures
from tests.golden.gotest_cases import CASES


@pytest.fixture(scope="module")
def nba():
    ds = fixtures.nba()
    o = oracle.Oracle()
    ds.load_oracle(o)
    return ds, o


@pytest.mark.parametrize("pushdown", [True, False])
@pytest.mark.parametrize("case", CASES, ids=[f"L{c['line']}" for c in CASES])
def test_gotest_known_answers(nba, case, pushdown):
    ds, o = nba
    s = ngql.parse_go(fixtures.nba_query(case["query"]))
    r = o.go(ds.space, s, pushdown=pushdown)
    if case.get("error"):                # E_EXECUTION_ERROR in the reference
        assert not r.ok
        return
    assert r.ok, r.error
    if case.get("ok_only"):                # NStepQueryHangAndOOM: the 40-step walk must succeed
        return
    got = fixtures.normalize_cells(r.rows)
    if case.get("empty"):
        assert got == []
        return
    assert got == fixtures.nba_expected(case["rows"])


@pytest.mark.parametrize("case", [c for c in CASES if "pushdown" in c], ids=lambda c: f"L{c['line']}")
def test_filter_pushdown_rewrite_strings(case):
    """TEST_FILTER_PUSHDOWN_REWRITE (GoTest.cpp:1580-1596): rewrite result and its toString."""
    s = ngql.parse_go(fixtures.nba_query(case["query"]))
    pushed = oracle.expr_pushdown(s.where.encode())
    if case["pushdown"] is None:
        assert pushed == b""
    else:
        assert pushed != b""
        assert oracle.expr_to_string(pushed) == fixtures.nba_query(case["pushdown"])
