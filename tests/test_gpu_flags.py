"""Storaged / graphd flags at the boundary.

* FLAGS_enable_reservoir_sampling (QueryBaseProcessor.cpp:13): storage keeps a random sample of each
  vertex's edges (QueryBoundProcessor::processEdgeSampling, QueryBoundProcessor.cpp:83-164, chosen at
  :213). A random sample has no bit-exact device counterpart, so with the flag set both entry points
  return NGX_E_UNSUPPORTED before any work and the shims run the reference's CPU path (INTEGRATION.md
  §1-2); with it cleared the same requests answer as the oracle does.
"""
import pytest

from nebula_amd import engine, ngql
from oracle import oracle
from tests import fixtures

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nba():
    ds = fixtures.nba()
    o = oracle.Oracle()
    ds.load_oracle(o)
    e = engine.Engine(0)
    ds.load_engine(e)
    yield ds, o, e
    e.close()
    o.close()


@pytest.fixture(scope="module")
def qb():
    ds = fixtures.querybound()
    o = oracle.Oracle()
    ds.load_oracle(o)
    e = engine.Engine(0)
    ds.load_engine(e)
    yield ds, o, e
    e.close()
    o.close()


GO = "GO 2 STEPS FROM {P:Tim Duncan} OVER like WHERE like.likeness > 80 YIELD like._dst, like.likeness"


def test_reservoir_sampling_refuses_go(nba):
    ds, o, e = nba
    s = ngql.parse_go(fixtures.nba_query(GO))
    assert e.get_flag("enable_reservoir_sampling") == 0
    e.set_flag("enable_reservoir_sampling", 1)
    try:
        assert e.get_flag("enable_reservoir_sampling") == 1
        with pytest.raises(engine.EngineError) as x:
            e.go(ds.space, s)
        assert x.value.code == engine.E_UNSUPPORTED
        assert "reservoir" in str(x.value)
    finally:
        e.set_flag("enable_reservoir_sampling", 0)
    ref, got = o.go(ds.space, s), e.go(ds.space, s)
    assert ref.ok and got.ok and got.rows
    assert sorted(fixtures.normalize_cells(got.rows), key=repr) == sorted(fixtures.normalize_cells(ref.rows), key=repr)


def test_reservoir_sampling_refuses_get_neighbors(qb):
    ds, o, e = qb
    parts, cols = fixtures.querybound_request([101])
    e.set_flag("enable_reservoir_sampling", 1)
    try:
        with pytest.raises(engine.EngineError) as x:
            e.get_neighbors(0, parts, [101], cols)
        assert x.value.code == engine.E_UNSUPPORTED
    finally:
        e.set_flag("enable_reservoir_sampling", 0)
    got, ref = e.get_neighbors(0, parts, [101], cols), o.get_neighbors(0, parts, [101], cols)
    assert got.failed_codes == [] and got.total_edges == ref.total_edges > 0


def test_trace_go_logs_every_step(nba, capfd):
    """graphd's FLAGS_trace_go (GoExecutor.cpp:559-569, 834-836): with trace_go set the library logs one
    line per step (frontier, scanned edges, next frontier, time) and the total row count on stderr."""
    ds, o, e = nba
    s = ngql.parse_go(fixtures.nba_query("GO 3 STEPS FROM {P:Tim Duncan} OVER like YIELD like._dst"))
    e.set_flag("trace_go", 1)
    try:
        got = e.go(ds.space, s)
    finally:
        e.set_flag("trace_go", 0)
    err = capfd.readouterr().err
    steps = [ln for ln in err.splitlines() if "trace_go" in ln and "Step:" in ln]
    assert [ln.split("Step:")[1].split()[0] for ln in steps] == ["1", "2", "3"]
    assert f"Total rows:{len(got.rows)}" in err
    for ln, edges in zip(steps, got.hop_edges):
        assert f"scanned edges {edges}," in ln
    e.go(ds.space, s)
    assert "trace_go" not in capfd.readouterr().err


def _rows(r):
    return sorted(fixtures.normalize_cells(r.rows), key=repr)


def test_query_over_string_arena_limit_then_normal_queries(nba):
    """A GO whose built strings exceed the device string arena (flag str_arena_max, 8 GiB by default)
    fails with NGX_E_UNSUPPORTED after the row reservation counters were handed out (its final launch
    never runs). The next queries on the same context must start from clean counters: each equals the
    oracle (a stale counter set made blocks allocate past the outputs)."""
    ds, o, e = nba
    built = ngql.parse_go(fixtures.nba_query(
        "GO 2 STEPS FROM {P:Tim Duncan}, {P:Tony Parker} OVER like YIELD (string)like.likeness AS s, like._dst"))
    plain = ngql.parse_go(fixtures.nba_query(GO))
    for _ in range(3):
        e.set_flag("str_arena_max", 64)
        try:
            with pytest.raises(engine.EngineError) as x:
                e.go(ds.space, built)
            assert x.value.code == engine.E_UNSUPPORTED and "string arena" in str(x.value)
        finally:
            e.set_flag("str_arena_max", 0)
        for s in (plain, built):
            ref, got = o.go(ds.space, s), e.go(ds.space, s)
            assert ref.ok and got.ok and got.rows
            assert _rows(got) == _rows(ref)


def test_dyn_hops_over_type_without_edges_after_rows():
    """Device-driven hops (flag dyn_hops) over an edge type that has no edges: no final launch runs, so
    the row count must be this query's 0, not the count of the query before it."""
    ds = fixtures.nba()
    ds.schemas.append(fixtures.SchemaDef(True, 99, "vacant", [("w", fixtures.INT)]))
    o = oracle.Oracle()
    ds.load_oracle(o)
    with engine.Engine(0) as e:
        ds.load_engine(e)
        e.set_flag("dyn_hops", 1)
        full = ngql.parse_go(fixtures.nba_query("GO 2 STEPS FROM {P:Tim Duncan} OVER like YIELD like._dst"))
        empty = ngql.parse_go(fixtures.nba_query("GO 2 STEPS FROM {P:Tim Duncan} OVER vacant YIELD vacant._dst"))
        for _ in range(2):
            got = e.go(ds.space, full)
            assert got.ok and _rows(got) == _rows(o.go(ds.space, full)) and got.rows
            got = e.go(ds.space, empty)
            assert got.ok and got.rows == [] and o.go(ds.space, empty).rows == []
            dev = e.go(ds.space, empty, on_device=True)
            assert dev.ok and dev.nrows == 0
    o.close()
