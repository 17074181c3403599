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
