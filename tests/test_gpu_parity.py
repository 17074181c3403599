"""GPU parity: libnebula_gn (HIP, through the C ABI) against the oracle and the reference's own
known answers.

* GoTest (src/graph/test/GoTest.cpp) on the NBA fixture, filter pushdown on and off: device rows ==
  transcribed expected rows == oracle rows.
* QueryBoundTest (src/storage/test/QueryBoundTest.cpp) requests through ngx_get_neighbors ==
  oracle QueryBoundProcessor responses (edges, key props, latest-version rows, tag props,
  failed codes).
* RMAT (configs C2 shape at small scale) GO queries covering multi-hop, M TO N, REVERSELY,
  BIDIRECT, $^/$$ props, compound WHERE, arithmetic YIELD and DISTINCT: device == oracle, exact.
Results are compared sorted (verifyResult, src/graph/test/TestBase.h:188-233); integers and
doubles bit-exact.
"""

import numpy as np
import pytest

from nebula_amd import datagen, engine, ngql
from oracle import oracle
from tests import fixtures
from tests.golden.gotest_cases import CASES

pytestmark = pytest.mark.gpu


def _engine(mode):
    """An engine on device 0 running the final hop through per-query hipRTC kernels ("jit") or the
    precompiled bytecode interpreter ("vm")."""
    e = engine.Engine(0)
    e.set_flag("jit", 1 if mode.startswith("jit") else 0)
    return e


def _load(ds, e, mode):
    """Commit the dataset to the engine; "-narrow" modes store integer columns at their narrowest width
    (flag narrow_columns = 1, the default, read at commit: int8/int16 columns sign-extended on load), the
    others at 8 bytes. The module fixtures run the generated kernels on narrow columns (the product
    default) and the interpreter on 8-byte columns, so both widths and both evaluators are covered."""
    e.set_flag("narrow_columns", 1 if mode.endswith("-narrow") else 0)
    ds.load_engine(e)


def _check_jit(e, mode):
    if mode.startswith("jit"):
        assert e.get_flag("jit_failed") == 0, e.jit_note()
        assert e.jit_note() == ""


@pytest.fixture(scope="module", params=["jit-narrow", "vm"])
def nba(request):
    ds = fixtures.nba()
    o = oracle.Oracle()
    ds.load_oracle(o)
    e = _engine(request.param)
    _load(ds, e, request.param)
    yield ds, o, e
    _check_jit(e, request.param)
    e.close()


@pytest.mark.parametrize("pushdown", [True, False])
@pytest.mark.parametrize("case", CASES, ids=[f"L{c['line']}" for c in CASES])
def test_gotest_nba(nba, case, pushdown):
    ds, o, e = nba
    s = ngql.parse_go(fixtures.nba_query(case["query"]))
    r = e.go(ds.space, s, pushdown=pushdown)
    ref = o.go(ds.space, s, pushdown=pushdown)
    if case.get("error"):                # E_EXECUTION_ERROR in the reference: both refuse the query
        assert not ref.ok and not r.ok
        return
    assert r.ok, r.error
    got = fixtures.normalize_cells(r.rows)
    assert ref.ok
    assert got == fixtures.normalize_cells(ref.rows)
    if ref.rows:                         # the reference sets column types only from result rows
        assert r.col_types == ref.col_types
    if case.get("empty"):
        assert got == []
    elif not case.get("ok_only"):
        assert got == fixtures.nba_expected(case["rows"])


# ----------------------------------------------------------------------------- QueryBoundTest
@pytest.fixture(scope="module")
def qb():
    ds = fixtures.querybound()
    o = oracle.Oracle()
    ds.load_oracle(o)
    e = _engine("vm")
    ds.load_engine(e)
    yield o, e
    e.close()


def _oracle_edges(resp):
    out = []
    for v in resp.vertices:
        for ed in v["edges"]:
            for x in ed["edges"]:
                out.append((v["vid"], ed["type"], x["dst"], tuple(x["values"] or ())))
    return sorted(out, key=repr)


def _plain(cell):
    kind, v = cell
    return v


def _engine_edges(res, parts, cols):
    vids = [x for _, vs in parts for x in vs]
    out = []
    for i in range(res.total_edges):
        t = int(res.edge_type[i])
        vals = tuple(_plain(res.edge_cells[i][c]) for c, (own, cid, name) in enumerate(cols)
                     if own == engine.EDGE and cid == t and name != "_dst")
        out.append((vids[res.edge_vertex[i]], t, int(res.edge_dst[i]), vals))
    return sorted(out, key=repr)


def _oracle_tags(resp):
    out = {}
    for v in resp.vertices:
        for t in v["tags"]:
            names = [c[0] for c in resp.vertex_schema[t["tag_id"]]]
            for n, val in zip(names, t["values"]):
                out[(v["vid"], t["tag_id"], n)] = val
    return out


def _engine_tags(res, parts, cols):
    vids = [x for _, vs in parts for x in vs]
    with_edges = set(int(i) for i in res.edge_vertex)
    out = {}
    for vi in with_edges:
        for c, (own, cid, name) in enumerate(cols):
            if own == engine.SOURCE and res.vertex_has_tag[vi * len(cols) + c]:
                out[(vids[vi], cid, name)] = _plain(res.vertex_cells[vi][c])
    return out


def _qb_compare(o, e, et, filt=b"", cols=None):
    parts, default_cols = fixtures.querybound_request(et)
    cols = cols if cols is not None else default_cols
    ref = o.get_neighbors(0, parts, et, cols, filt)
    got = e.get_neighbors(0, parts, et, cols, filt)
    assert sorted(got.failed_codes) == sorted(ref.failed_codes)
    assert got.total_edges == ref.total_edges
    assert _engine_edges(got, parts, cols) == _oracle_edges(ref)
    assert _engine_tags(got, parts, cols) == _oracle_tags(ref)
    return got


def _alias_rel(alias, prop, op, value):
    return ngql.Binary(ngql.K_REL, ngql.REL_OPS[op], ngql.Prop(ngql.K_ALIAS, "", alias, prop), ngql.Prim(value))


def _src_rel(tag, prop, op, value):
    return ngql.Binary(ngql.K_REL, ngql.REL_OPS[op], ngql.Prop(ngql.K_SRC_PROP, "$^", tag, prop), ngql.Prim(value))


@pytest.mark.parametrize("et", [[101], [-101], [101, 102, 103], [-102, 103]])
def test_querybound_plain(qb, et):
    r = _qb_compare(*qb, et)
    assert r.total_edges == 30 * len(et) * 6 or r.total_edges > 0


def test_querybound_edge_filter(qb):
    _qb_compare(*qb, [101], _alias_rel("101", "col_0", ">=", 10007).encode())
    _qb_compare(*qb, [101], _alias_rel("101", "col_10", "==", "string_col_10_1").encode(), cols=[(3, 101, "col_10")])


def test_querybound_tag_filters(qb):
    _qb_compare(*qb, [101], _src_rel("3001", "tag_3001_col_0", ">=", 20 + 3001).encode())
    f = ngql.Binary(ngql.K_LOGIC, 0, _src_rel("3001", "tag_3001_col_0", ">=", 3021),
                    _alias_rel("101", "col_0", ">=", 10007)).encode()
    _qb_compare(*qb, [101], f)


def test_querybound_invalid_filter(qb):
    f = ngql.Prop(ngql.K_INPUT_PROP, "$-", "", "tag_3001_col_0").encode()
    r = _qb_compare(*qb, [101], f)
    assert len(r.failed_codes) == 3 and all(c == -31 for c, _ in r.failed_codes)


def test_querybound_other_type_alias_skips(qb):
    # alias of a type that is not this edge's: storage getter error -> edge skipped (.inl:556-564)
    f = ngql.Binary(ngql.K_LOGIC, 1, _alias_rel("102", "col_0", ">", 0), _alias_rel("101", "col_0", ">", 0)).encode()
    _qb_compare(*qb, [101, 102], f)


# ----------------------------------------------------------------------------- RMAT
RMAT_QUERIES = [
    "GO 3 STEPS FROM {S} OVER e WHERE e.p0 < 50 YIELD e._dst, e._rank, e.p0, e.p1",
    "GO FROM {S} OVER e",
    "GO 2 STEPS FROM {S} OVER e YIELD e._src, e._dst, e._type",
    "GO 2 STEPS FROM {S} OVER e REVERSELY WHERE e.p1 > 500000 YIELD e._src, e._dst, e.p1",
    "GO 1 TO 3 STEPS FROM {S} OVER e WHERE e.p0 % 7 == 3 YIELD e._dst, e.p0",
    "GO 2 STEPS FROM {S} OVER e BIDIRECT WHERE e.p0 > 90 YIELD e._dst, e.p0 * 2 + 1",
    "GO 2 STEPS FROM {S} OVER e WHERE $^.vt.v0 > 100 && e.p0 % 3 == 0 YIELD $^.vt.name, $$.vt.v0, e.p0 + e.p1",
    "GO FROM {S} OVER e WHERE (e.p0 * 1.5 > 30.0) || udf_is_in(e.p0, 1, 2, 3) YIELD e.p0 / 3.0, e.p1 % 7",
    "GO 3 STEPS FROM {S} OVER e YIELD DISTINCT e._dst",
    "GO 2 STEPS FROM {S} OVER e WHERE $$.vt.name CONTAINS \"7\" YIELD $$.vt.name, e._dst",
    "GO FROM {S} OVER e WHERE e.p0 >= 10 XOR e.p1 < 100000 YIELD e._dst, abs(e.p0 - 50), e.p1 > 5 && true",
]


@pytest.fixture(scope="module", params=["jit-narrow", "vm"])
def rmat(request):
    ds = fixtures.RmatDataset(12, with_in=True, with_tag=True)
    o = oracle.Oracle()
    o.set_flags(threads=8)
    ds.load_oracle(o)
    e = _engine(request.param)
    _load(ds, e, request.param)
    yield ds, o, e
    _check_jit(e, request.param)
    e.close()


@pytest.mark.parametrize("pushdown", [True, False])
@pytest.mark.parametrize("qi", range(len(RMAT_QUERIES)))
def test_rmat_go(rmat, qi, pushdown):
    ds, o, e = rmat
    seeds = datagen.sample_vids(1000 + qi, 1 << ds.scale, 40)
    q = RMAT_QUERIES[qi].replace("{S}", ", ".join(str(int(v)) for v in seeds))
    s = ngql.parse_go(q)
    ref = o.go(ds.space, s, pushdown=pushdown)
    got = e.go(ds.space, s, pushdown=pushdown)
    assert got.ok == ref.ok, (got.error, ref.error)
    if not ref.ok:
        return
    if ref.rows:
        assert got.col_types == ref.col_types
    a, b = fixtures.normalize_cells(got.rows), fixtures.normalize_cells(ref.rows)
    assert len(a) == len(b)
    assert a == b
    # TEPS numerator: edges scanned per hop agree with the restated storage scan
    assert got.hop_edges[:len(ref.hop_scanned)] == ref.hop_scanned[:len(got.hop_edges)]


def test_rmat_device_results(rmat):
    """result_on_device leaves the rows in HBM: same row count and hop statistics as the host path."""
    ds, o, e = rmat
    seeds = datagen.sample_vids(77, 1 << ds.scale, 40)
    s = ngql.parse_go(RMAT_QUERIES[0].replace("{S}", ", ".join(str(int(v)) for v in seeds)))
    host = e.go(ds.space, s)
    dev = e.go(ds.space, s, on_device=True)
    assert dev.ok and dev.nrows == len(host.rows) and dev.hop_edges == host.hop_edges


def test_rmat_empty_and_missing_seeds(rmat):
    ds, o, e = rmat
    for q in ["GO FROM -5 OVER e", "GO 3 STEPS FROM 99999999 OVER e YIELD e._dst"]:
        s = ngql.parse_go(q)
        got = e.go(ds.space, s)
        assert got.ok and got.rows == []


# (query, the oracle's Status text, the device's failure class): graphd's evaluation of WHERE / YIELD
# fails the query (GoExecutor.cpp:1277-1294); the device reports the class of the failure, not
# Expressions.cpp's text, so the kind is pinned on both sides
# (the WHERE of case 2 runs in graphd only with pushdown off: pushed, a storage filter error skips the
# edge instead, QueryBaseProcessor.inl:586-602)
ERROR_CASES = [
    ("GO FROM 1, 2, 3 OVER e YIELD e.p1 * 9223372036854775807", True, "Out of range", "failed to evaluate"),
    ("GO FROM 1, 2, 3 OVER e YIELD e.p1 / (e.p0 - e.p0)", True, "Division by zero", "failed to evaluate"),
    ("GO FROM 1, 2, 3 OVER e WHERE e.p1 % (e.p0 - e.p0) > 1 YIELD e._dst", False, "Division by zero", "failed to evaluate"),
    ("GO 2 STEPS FROM 1, 2, 3 OVER e YIELD -9223372036854775807 - 1 - e.p0 - 1", True, "Out of range", "failed to evaluate"),
]


@pytest.mark.parametrize("case", range(len(ERROR_CASES)))
def test_rmat_query_error_matches(rmat, case):
    ds, o, e = rmat
    q, push, ref_text, dev_text = ERROR_CASES[case]
    s = ngql.parse_go(q)
    ref = o.go(ds.space, s, pushdown=push)
    got = e.go(ds.space, s, pushdown=push)
    assert not ref.ok and ref_text in ref.error, ref.error
    assert not got.ok and got.code == engine.E_QUERY and dev_text in got.error, (got.code, got.error)
    # the same query on the host path that the device refuses nothing of: a good query still runs after it
    ok = e.go(ds.space, ngql.parse_go("GO FROM 1, 2, 3 OVER e YIELD e.p1"))
    assert ok.ok


def test_rmat_device_results_values(rmat):
    """result_on_device leaves the rows in HBM, columnar: the arrays copied back hold the same rows as
    the host result (compared sorted: GO rows come in chunk-completion order, as the reference's come
    in response order), typed int columns carry no per-row type array, strings carry lengths."""
    ds, o, e = rmat
    seeds = datagen.sample_vids(78, 1 << ds.scale, 60)
    q = ("GO 2 STEPS FROM " + ", ".join(str(int(v)) for v in seeds) +
         " OVER e WHERE e.p0 < 50 YIELD e._dst, e._rank, e.p0, e.p1, $^.vt.name")
    s = ngql.parse_go(q)
    host = e.go(ds.space, s)
    dev = e.go(ds.space, s, on_device=True, fetch=True)
    assert host.ok and dev.ok and dev.nrows == len(host.rows) > 0
    for c in range(4):
        x, ln, t = dev.dev_cols[c]
        assert ln is None and t is None
    x, ln, t = dev.dev_cols[4]
    assert ln is not None and t is None
    got = sorted(zip(dev.src.tolist(), dev.dst.tolist(), dev.rank.tolist(),
                     *[dev.dev_cols[c][0].tolist() for c in range(4)], dev.dev_cols[4][1].tolist()))
    ref = sorted(zip(host.src.tolist(), host.dst.tolist(), host.rank.tolist(),
                     *[[r[c][1] for r in host.rows] for c in range(4)],
                     [len(r[4][1].encode()) for r in host.rows]))
    assert got == ref


# --------------------------------------------------------------------------- larger RMAT (C2 shape)
@pytest.fixture(scope="module", params=["jit", "vm"])
def rmat16(request):
    ds = fixtures.RmatDataset(16, threads=8)
    o = oracle.Oracle()
    o.set_flags(threads=8)
    ds.load_oracle(o)
    e = _engine(request.param)
    _load(ds, e, request.param)
    yield ds, o, e
    _check_jit(e, request.param)
    e.close()


@pytest.mark.parametrize("sel", [10, 50, 90])
def test_rmat16_bench_query(rmat16, sel):
    """The bench query (BASELINE configs[1] shape) at scale 16: GO 3 STEPS from 200 vids WHERE
    e.p0 < sel: rows and per-hop scanned edges equal the oracle's; hubs span many 2048-edge chunks."""
    ds, o, e = rmat16
    seeds = datagen.rmat_seeds(16, 200, 16, 42, 7 + sel, threads=8)
    q = (f"GO 3 STEPS FROM {', '.join(str(int(v)) for v in seeds)} OVER e WHERE e.p0 < {sel} "
         "YIELD e._dst, e._rank, e.p0, e.p1")
    s = ngql.parse_go(q)
    ref = o.go(ds.space, s)
    got = e.go(ds.space, s)
    assert ref.ok and got.ok, (got.error, ref.error)
    assert got.hop_edges == ref.hop_scanned
    assert fixtures.normalize_cells(got.rows) == fixtures.normalize_cells(ref.rows)


@pytest.mark.parametrize("lane_rows,wg", [(4, 1024), (8, 1024), (16, 1024), (0, 256)])
def test_compaction_lane_rows(rmat16, rmat, lane_rows, wg):
    """The next-frontier compaction at each rows-per-lane width (flag compact_lane_rows, default 4) and
    in 256-thread workgroups (flag compact_wg; a pipelined batch's default, 16 rows per lane):
    the bench query at scale 16 (one edge type) and a BIDIRECT query at
    scale 12 with in-edges (two slots per frontier row) give the oracle's rows and per-hop scans."""
    cases = [(rmat16, datagen.rmat_seeds(16, 300, 16, 42, 99, threads=8),
              "GO 3 STEPS FROM {S} OVER e WHERE e.p0 < 50 YIELD e._dst, e._rank, e.p0, e.p1"),
             (rmat, datagen.sample_vids(99, 1 << 12, 40),
              "GO 3 STEPS FROM {S} OVER e BIDIRECT WHERE e.p0 > 60 YIELD e._dst, e.p1")]
    for (ds, o, e), seeds, text in cases:
        q = text.replace("{S}", ", ".join(str(int(v)) for v in seeds))
        s = ngql.parse_go(q)
        e.set_flag("compact_lane_rows", lane_rows)
        e.set_flag("compact_wg", wg)
        try:
            got = e.go(ds.space, s, columnar=True, rows=False, digest_fn=oracle.digest_columns)
        finally:
            e.set_flag("compact_lane_rows", 0)
            e.set_flag("compact_wg", 0)
        # the oracle's sorted row digests, once per (graph, query) over the widths and modes
        key = (id(o), q)
        if key not in _LANE_REFS:
            _LANE_REFS[key] = o.go(ds.space, s, digest=True)
        ref = _LANE_REFS[key]
        assert ref.ok and got.ok, (got.error, ref.error)
        assert got.hop_edges == ref.hop_scanned
        assert got.nrows == ref.nrows and ref.nrows > 0
        assert np.array_equal(got.digests, ref.digests)


_LANE_REFS = {}


# --------------------------------------------------------------------------- C4: power law + supernodes
PL_QUERIES = [
    "GO 2 STEPS FROM {S} OVER pl REVERSELY YIELD pl._dst, pl.w, pl.score",
    "GO 2 STEPS FROM {S} OVER pl REVERSELY WHERE pl.w < 30 && pl.score > 0.25 YIELD pl._dst, pl._src, pl.score",
    "GO 2 STEPS FROM {S} OVER pl WHERE pl.score * 100.0 > pl.w YIELD pl._dst, pl.w + 1",
    "GO 1 TO 2 STEPS FROM {S} OVER pl BIDIRECT WHERE pl.w == 7 YIELD pl._dst, pl._src, pl.w",
]


@pytest.fixture(scope="module", params=["jit", "vm"])
def plaw(request):
    ds = fixtures.powerlaw_dataset(50000, superdeg=30000, threads=8)
    o = oracle.Oracle()
    o.set_flags(threads=8)
    ds.load_oracle(o)
    e = _engine(request.param)
    _load(ds, e, request.param)
    yield ds, o, e
    _check_jit(e, request.param)
    e.close()


@pytest.mark.parametrize("qi", range(len(PL_QUERIES)))
def test_powerlaw_supernodes(plaw, qi):
    """C4 shape: seeds include the supernodes (in-degree 30000 = 15 chunks of 2048 edges each), so
    one frontier entry spans many workgroups; REVERSELY has no pushdown (GoExecutor.cpp:528-533)."""
    ds, o, e = plaw
    seeds = [0, 7919, 15838, 23757] + [int(v) for v in datagen.sample_vids(300 + qi, ds.n, 20)]
    q = PL_QUERIES[qi].replace("{S}", ", ".join(str(v) for v in seeds))
    s = ngql.parse_go(q)
    ref = o.go(ds.space, s)
    got = e.go(ds.space, s)
    assert ref.ok and got.ok, (got.error, ref.error)
    assert got.hop_edges[:len(ref.hop_scanned)] == ref.hop_scanned[:len(got.hop_edges)]
    assert fixtures.normalize_cells(got.rows) == fixtures.normalize_cells(ref.rows)


# --------------------------------------------------------------------------- C5: SNB-like, strings
SNB_QUERIES = [
    "GO 4 STEPS FROM {S} OVER knows WHERE knows.creationDate > 1400000000 && $^.person.gender == \"female\" "
    "YIELD knows._dst, knows.weight, $^.person.firstName, $$.person.age",
    "GO 2 STEPS FROM {S} OVER knows, likes WHERE likes.creationDate > 1300000000 || knows.weight > 5.0 "
    "YIELD knows._dst, likes._dst, likes.creationDate, knows.weight",
    "GO 1 STEPS FROM {S} OVER likes WHERE $$.post.lang == \"en\" && $$.post.length > 40 "
    "YIELD likes._dst, $$.post.content, $$.post.lang",
    "GO 2 STEPS FROM {S} OVER hasCreator, likes REVERSELY WHERE likes.creationDate > 1400000000 "
    "YIELD hasCreator._dst, likes._dst, likes.creationDate",
    "GO 3 STEPS FROM {S} OVER * WHERE $^.person.firstName CONTAINS \"a\" YIELD knows._dst, likes._dst, hasCreator._dst",
]


@pytest.fixture(scope="module", params=["jit", "vm"])
def snb(request):
    ds = fixtures.snb_dataset(5000, threads=8)
    o = oracle.Oracle()
    o.set_flags(threads=8)
    ds.load_oracle(o)
    e = _engine(request.param)
    _load(ds, e, request.param)
    yield ds, o, e
    _check_jit(e, request.param)
    e.close()


@pytest.mark.parametrize("pushdown", [True, False])
@pytest.mark.parametrize("qi", range(len(SNB_QUERIES)))
def test_snb_compound(snb, qi, pushdown):
    """C5 shape: multi-edge-type schema with string + int props, a batch of person seeds, compound
    WHERE over edge, $^ and $$ props, multi-column YIELD (strings returned through the columnar
    result)."""
    ds, o, e = snb
    seeds = [int(v) for v in datagen.sample_vids(500 + qi, ds.np, 400)]
    q = SNB_QUERIES[qi].replace("{S}", ", ".join(str(v) for v in seeds))
    s = ngql.parse_go(q)
    ref = o.go(ds.space, s, pushdown=pushdown)
    got = e.go(ds.space, s, pushdown=pushdown)
    assert got.ok == ref.ok, (got.error, ref.error)
    if not ref.ok:
        return
    assert got.col_types == ref.col_types
    assert fixtures.normalize_cells(got.rows) == fixtures.normalize_cells(ref.rows)


@pytest.mark.parametrize("compact", [True, False])
def test_rmat_device_digest_matches_oracle_rows(rmat, compact):
    """ngx_go_result_digest (the device reduction that pins C3's rows by value) over a device-resident
    result equals the oracle restatement's row hash of the oracle's own rows; with a narrowed / constant
    column layout (compact) and at 8 bytes."""
    ds, o, e = rmat
    seeds = datagen.sample_vids(4242, 1 << ds.scale, 60)
    for where in ("", " WHERE e.p0 < 50", " WHERE e.p0 >= 50"):
        q = f"GO 3 STEPS FROM {', '.join(str(int(v)) for v in seeds)} OVER e{where} YIELD e._src, e._dst, e._rank, e.p0, e.p1"
        s = ngql.parse_go(q)
        ref = o.go(ds.space, s)
        got = e.go(ds.space, s, on_device=True, compact=compact, device_digest=True)
        assert ref.ok and got.ok and got.nrows == len(ref.rows) > 0
        cols = [np.array([int(r[k][1]) for r in ref.rows], dtype=np.int64) for k in range(5)]
        # the device hashes the row's src vid, then every YIELD column (here e._src again)
        assert got.device_digest == oracle.row_digest([cols[0]] + cols)
