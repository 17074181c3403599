"""Storage-side semantics on the device against the oracle: max_edge_returned_per_vertex, edge and tag
TTL, per-part E_PART_NOT_FOUND.

* QueryBoundTest MaxEdgesReturenedTest (src/storage/test/QueryBoundTest.cpp:602-627) and TTLTest
  (:695-720) through ngx_get_neighbors, plus a cap counted after a filter and a partly expired TTL.
* GO with the storaged flag max_edge_returned_per_vertex set (every hop's request is capped: first N
  emitted edges per (vertex, type) in key order, counted after the pushed filter, .inl:501-606).
* GO over a space whose edge type and tag carry TTL (ttl_col / ttl_duration): expired edges are skipped
  on every hop (storage builds a RowReader whenever TTL info exists, .inl:519-536), expired tag rows
  are absent ($^ / $$ props take defaults in graphd, src-tag filters fail in storage).
"""
import pytest

from nebula_amd import datagen, engine, ngql
from oracle import oracle
from tests import fixtures

pytestmark = pytest.mark.gpu


def _alias_rel(alias, prop, op, value):
    return ngql.Binary(ngql.K_REL, ngql.REL_OPS[op], ngql.Prop(ngql.K_ALIAS, "", alias, prop), ngql.Prim(value))


def _edges(res, parts, cols):
    vids = [x for _, vs in parts for x in vs]
    out = []
    for i in range(res.total_edges):
        t = int(res.edge_type[i])
        vals = tuple(res.edge_cells[i][c][1] for c, (own, cid, name) in enumerate(cols)
                     if own == engine.EDGE and cid == t and name != "_dst")
        out.append((vids[res.edge_vertex[i]], t, int(res.edge_dst[i]), vals))
    return sorted(out, key=repr)


def _oracle_edges(resp):
    out = []
    for v in resp.vertices:
        for ed in v["edges"]:
            for x in ed["edges"]:
                out.append((v["vid"], ed["type"], x["dst"], tuple(x["values"] or ())))
    return sorted(out, key=repr)


# ----------------------------------------------------------------------------- GetNeighbors
@pytest.fixture(scope="module")
def qb():
    ds = fixtures.querybound()
    e = engine.Engine(0)
    ds.load_engine(e)
    yield ds, e
    e.close()


@pytest.mark.parametrize("cap,filt", [(5, None), (3, ("col_0", ">=", 10003)), (1, ("col_0", "<", 10006)), (7, None)])
def test_querybound_max_edges(qb, cap, filt):
    """MaxEdgesReturenedTest: 5 of the 7 out-edges per vertex; with a filter the cap counts passing edges,
    in key order (rank LE bytes, then dst LE bytes)."""
    ds, e = qb
    o = oracle.Oracle()
    ds.load_oracle(o)
    o.set_flags(max_edges=cap)
    parts, cols = fixtures.querybound_request([101])
    f = _alias_rel("101", *filt).encode() if filt else b""
    ref = o.get_neighbors(0, parts, [101], cols, f)
    got = e.get_neighbors(0, parts, [101], cols, f, max_edges_per_vertex=cap)
    assert got.failed_codes == [] and ref.failed_codes == []
    assert got.total_edges == ref.total_edges
    assert _edges(got, parts, cols) == _oracle_edges(ref)
    per_vertex = {}
    for i in range(got.total_edges):
        per_vertex[int(got.edge_vertex[i])] = per_vertex.get(int(got.edge_vertex[i]), 0) + 1
    assert max(per_vertex.values()) <= cap
    if filt is None:
        assert got.total_edges == 30 * min(cap, 7)


def _ttl_space():
    ds = fixtures.querybound()
    ds.schemas = [s for s in ds.schemas if (s.is_edge and s.sid == 101) or (not s.is_edge and s.sid == 3001)]
    for s in ds.schemas:
        if s.is_edge:
            s.ttl_col, s.ttl_dur = "col_0", 200
        else:
            s.ttl_col, s.ttl_dur = "tag_3001_col_0", 100
    return ds


@pytest.mark.parametrize("now", [1_700_000_000, 10_205, 3_115, 1])
def test_querybound_ttl(now):
    """TTLTest (mockSchemaWithTTLMan: edge 101 ttl_col col_0, tag 3001 TTL'd too): at a real clock every
    edge expired (no vertices, no failed codes); at smaller clocks a part of the edges (col_0 = dst + 0 ..)
    and of the tag rows (tag_3001_col_0 = vid + 3001) survive."""
    ds = _ttl_space()
    o = oracle.Oracle()
    ds.load_oracle(o)
    o.set_flags(now_sec=now)
    parts, _ = fixtures.querybound_request([101])
    cols = [(3, 101, "col_10"), (3, 101, "col_0"), (1, 3001, "tag_3001_col_0")]
    ref = o.get_neighbors(0, parts, [101], cols)
    with engine.Engine(0) as e:
        ds.load_engine(e)
        got = e.get_neighbors(0, parts, [101], cols, now_sec=now)
    assert got.failed_codes == [] and ref.failed_codes == []
    assert got.total_edges == ref.total_edges
    assert _edges(got, parts, cols) == _oracle_edges(ref)
    if now == 1_700_000_000:
        assert got.total_edges == 0 and ref.vertices == []
    # tag columns of the vertices that returned edges: expired tag rows are absent
    vids = [x for _, vs in parts for x in vs]
    want = {}
    for v in ref.vertices:
        for t in v["tags"]:
            want[v["vid"]] = t["values"][0]
    have = {}
    for vi in set(int(i) for i in got.edge_vertex):
        if got.vertex_has_tag[vi * len(cols) + 2]:
            have[vids[vi]] = got.vertex_cells[vi][2][1]
    assert have == want


def test_get_neighbors_part_not_found():
    """Parts this shard does not hold (outside 1..num_parts here) fail with E_PART_NOT_FOUND (-14) per part,
    the other parts answer normally (QueryBaseProcessor.inl:835-851)."""
    ds = fixtures.RmatDataset(10)
    o = oracle.Oracle()
    ds.load_oracle(o)
    with engine.Engine(0) as e:
        ds.load_engine(e)
        vids = [int(v) for v in datagen.sample_vids(5, 1 << 10, 40)]
        byp = {}
        for v in vids:
            byp.setdefault(v % 100 + 1, []).append(v)
        parts = sorted(byp.items()) + [(101, [7, 8]), (0, [9])]
        cols = [(3, 1, "_dst"), (3, 1, "p0")]
        ref = o.get_neighbors(ds.space, parts, [1], cols)
        before = e.stats()
        got = e.get_neighbors(ds.space, parts, [1], cols)
        ok = e.get_neighbors(ds.space, parts[:3], [1], cols)
        after = e.stats()
    assert sorted(got.failed_codes) == sorted(ref.failed_codes) == [(-14, 0), (-14, 101)]
    assert got.total_edges == ref.total_edges > 0
    assert _edges(got, parts, cols) == _oracle_edges(ref)
    # onFinished (BaseProcessor.h:51-60): latency_in_us, get_bound qps / error_qps / latency
    assert got.latency_in_us > 0 and ok.latency_in_us > 0 and not ok.failed_codes
    d = {k: after[k] - before.get(k, 0) for k in after}
    assert d["storage_get_bound_qps"] == 1 and d["storage_get_bound_error_qps"] == 1
    assert d["storage_get_bound_latency_us_count"] == 2
    assert d["storage_get_bound_latency_us_sum"] == got.latency_in_us + ok.latency_in_us


# ----------------------------------------------------------------------------- GO
GO_QUERIES = [
    ("GO 2 STEPS FROM {S} OVER e YIELD e._dst, e._rank, e.p0", True),
    ("GO 3 STEPS FROM {S} OVER e WHERE e.p0 < 50 YIELD e._dst, e.p0, e.p1", True),
    ("GO 3 STEPS FROM {S} OVER e WHERE e.p0 < 50 YIELD e._dst, e.p0, e.p1", False),
    ("GO 2 STEPS FROM {S} OVER e REVERSELY WHERE e.p0 > 20 YIELD e._dst, e.p0", True),
    ("GO 1 TO 3 STEPS FROM {S} OVER e BIDIRECT WHERE e.p0 % 3 == 1 YIELD e._dst, e._src, $^.vt.name", True),
    ("GO 2 STEPS FROM {S} OVER e WHERE $^.vt.v0 > 300 && e.p0 < 70 YIELD $$.vt.v0, $^.vt.name, e.p0", True),
]


@pytest.fixture(scope="module")
def rmat_ttl():
    """RMAT scale 12 (in-edges, tag vt) with TTL on e (ttl_col p0, 950 s) and on vt (ttl_col v0, 500 s):
    at now = 1000 the edges with p0 < 50 and the tags with v0 < 500 are expired."""
    ds = fixtures.RmatDataset(12, with_in=True, with_tag=True)
    for s in ds.schemas:
        if s.is_edge:
            s.ttl_col, s.ttl_dur = "p0", 950
        else:
            s.ttl_col, s.ttl_dur = "v0", 500
    o = oracle.Oracle()
    o.set_flags(threads=8)
    ds.load_oracle(o)
    e = engine.Engine(0)
    ds.load_engine(e)
    yield ds, o, e
    e.close()


@pytest.mark.parametrize("mode", ["jit", "vm"])
@pytest.mark.parametrize("now", [1000, 1040, 1])
@pytest.mark.parametrize("qi", range(len(GO_QUERIES)))
def test_go_ttl(rmat_ttl, qi, now, mode):
    ds, o, e = rmat_ttl
    e.set_flag("jit", 1 if mode == "jit" else 0)
    text, push = GO_QUERIES[qi]
    s = ngql.parse_go(text.replace("{S}", ", ".join(str(int(v)) for v in datagen.sample_vids(70 + qi, 1 << 12, 40))))
    o.set_flags(threads=8, now_sec=now)
    ref = o.go(ds.space, s, pushdown=push)
    got = e.go(ds.space, s, pushdown=push, now_sec=now)
    assert got.ok == ref.ok, (got.error, ref.error)
    assert fixtures.normalize_cells(got.rows) == fixtures.normalize_cells(ref.rows)
    if now == 1:
        assert got.rows                                   # nothing expired


@pytest.fixture(scope="module")
def rmat_plain():
    ds = fixtures.RmatDataset(12, with_in=True, with_tag=True)
    o = oracle.Oracle()
    ds.load_oracle(o)
    e = engine.Engine(0)
    ds.load_engine(e)
    yield ds, o, e
    e.set_flag("max_edge_returned_per_vertex", 0)
    e.close()


@pytest.mark.parametrize("mode", ["jit", "vm"])
@pytest.mark.parametrize("cap", [1, 3, 17])
@pytest.mark.parametrize("qi", range(len(GO_QUERIES)))
def test_go_max_edges(rmat_plain, qi, cap, mode):
    """Every hop's storage request capped (FLAGS_max_edge_returned_per_vertex): the frontier, the final
    rows and the pushed-filter counting all follow the reference; RMAT hubs exceed every cap."""
    ds, o, e = rmat_plain
    e.set_flag("jit", 1 if mode == "jit" else 0)
    e.set_flag("max_edge_returned_per_vertex", cap)
    try:
        text, push = GO_QUERIES[qi]
        s = ngql.parse_go(text.replace("{S}", ", ".join(str(int(v)) for v in datagen.sample_vids(90 + qi, 1 << 12, 40))))
        o.set_flags(threads=8, max_edges=cap)
        ref = o.go(ds.space, s, pushdown=push)
        got = e.go(ds.space, s, pushdown=push)
        assert got.ok == ref.ok, (got.error, ref.error)
        assert fixtures.normalize_cells(got.rows) == fixtures.normalize_cells(ref.rows)
        assert got.rows
    finally:
        e.set_flag("max_edge_returned_per_vertex", 0)
        o.set_flags(threads=8)
