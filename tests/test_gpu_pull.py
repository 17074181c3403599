"""Direction-optimizing ("pull") intermediate hops against the oracle.

The pull expansion (kernels.h launchPull) computes a hop's next frontier from the in-edges of every
row of the shard (the mirror slot -t of each OVER type t, verified at commit to be the exact transpose)
instead of storing a mark per frontier edge. The frontier must be the same set of dsts
(GoExecutor::getDstIdsFromRespWithBackTrack, src/graph/GoExecutor.cpp:675-718), so every query here
runs with pull forced on every intermediate hop (pull_factor 1), with pull off (pull_factor 0) and at
the default threshold, and all three must equal the oracle, hop statistics included.

Cases: RMAT (C2 shape, scale 12 and 16), the power-law graph with supernodes (long in-lists go
through the segment queue drained across workgroups), the SNB-like multi-type schema (several mirror
pairs per hop, BIDIRECT / REVERSELY / OVER *), the NBA fixture (GoTest answers), spaces whose in-edges
are NOT the transpose of their out-edges (one in-edge missing or misdirected: pull must not be used),
and enough queries in a row to wrap the one-byte mark epoch several times.
"""
import numpy as np
import pytest

from nebula_amd import datagen, engine, ngql
from oracle import oracle
from tests import fixtures
from tests.golden.gotest_cases import CASES

pytestmark = pytest.mark.gpu

FACTORS = [1, 0, 200]


def _run(e, o, space, q, factor, pushdown=True, mirrored=True):
    s = ngql.parse_go(q)
    e.set_flag("pull_factor", factor)
    before = e.get_flag("pull_hops")
    got = e.go(space, s, pushdown=pushdown)
    pulled = e.get_flag("pull_hops") - before
    ref = o.go(space, s, pushdown=pushdown)
    assert got.ok == ref.ok, (got.error, ref.error)
    if ref.ok:
        assert got.hop_edges[:len(ref.hop_scanned)] == ref.hop_scanned[:len(got.hop_edges)]
        assert fixtures.normalize_cells(got.rows) == fixtures.normalize_cells(ref.rows)
    if factor == 0:
        assert pulled == 0
    if mirrored and factor == 1 and ref.ok and any(100 * h >= e.info(space).vertices for h in got.hop_edges[:-1]):
        assert pulled > 0                # pull_factor 1: every intermediate hop with E >= V / 100 pulls
    return pulled


@pytest.fixture(scope="module", params=["dyn", "host"])
def rmat12(request):
    """dyn: device-driven hops (the kernels pass |F| and E along, pull-or-push decided on the device);
    host: the host reads every hop's totals and launches exact grids."""
    ds = fixtures.RmatDataset(12, with_in=True, with_tag=True)
    o = oracle.Oracle()
    o.set_flags(threads=8)
    ds.load_oracle(o)
    e = engine.Engine(0)
    e.set_flag("dyn_hops", 1 if request.param == "dyn" else 0)
    ds.load_engine(e)
    yield ds, o, e
    e.close()


RMAT_Q = [
    "GO 3 STEPS FROM {S} OVER e WHERE e.p0 < 50 YIELD e._dst, e._rank, e.p0, e.p1",
    "GO 3 STEPS FROM {S} OVER e REVERSELY YIELD e._dst, e.p1",
    "GO 2 STEPS FROM {S} OVER e BIDIRECT WHERE e.p0 > 90 YIELD e._dst, e.p0",
    "GO 1 TO 4 STEPS FROM {S} OVER e WHERE e.p0 % 11 == 3 YIELD e._src, e._dst",
    "GO 4 STEPS FROM {S} OVER e YIELD DISTINCT e._dst",
]


@pytest.mark.parametrize("factor", FACTORS)
@pytest.mark.parametrize("qi", range(len(RMAT_Q)))
def test_pull_rmat12(rmat12, qi, factor):
    ds, o, e = rmat12
    seeds = datagen.sample_vids(900 + qi, 1 << ds.scale, 30)
    q = RMAT_Q[qi].replace("{S}", ", ".join(str(int(v)) for v in seeds))
    _run(e, o, ds.space, q, factor)


def test_pull_rmat16_bench_query():
    """The bench query at scale 16, 200 seeds: pull forced and off give the oracle's rows."""
    ds = fixtures.RmatDataset(16, threads=8, with_in=True)
    o = oracle.Oracle()
    o.set_flags(threads=8)
    ds.load_oracle(o)
    with engine.Engine(0) as e:
        ds.load_engine(e)
        seeds = datagen.rmat_seeds(16, 200, 16, 42, 5, threads=8)
        q = (f"GO 3 STEPS FROM {', '.join(str(int(v)) for v in seeds)} OVER e WHERE e.p0 < 50 "
             "YIELD e._dst, e._rank, e.p0, e.p1")
        assert _run(e, o, ds.space, q, 1) == 2
        _run(e, o, ds.space, q, 0)
        assert _run(e, o, ds.space, q, 200) >= 1      # hop 2 of the bench query pulls by default


@pytest.fixture(scope="module")
def plaw():
    ds = fixtures.powerlaw_dataset(50000, superdeg=30000, threads=8)
    o = oracle.Oracle()
    o.set_flags(threads=8)
    ds.load_oracle(o)
    e = engine.Engine(0)
    ds.load_engine(e)
    yield ds, o, e
    e.close()


PL_Q = [
    "GO 2 STEPS FROM {S} OVER pl REVERSELY YIELD pl._dst, pl.w",
    "GO 3 STEPS FROM {S} OVER pl WHERE pl.w < 30 YIELD pl._dst, pl.score",
    "GO 3 STEPS FROM {S} OVER pl BIDIRECT WHERE pl.w == 7 YIELD pl._dst, pl._src",
]


@pytest.mark.parametrize("factor", FACTORS)
@pytest.mark.parametrize("qi", range(len(PL_Q)))
def test_pull_powerlaw_supernodes(plaw, qi, factor):
    """In-degree 30000 supernodes: their in-lists (and any long list unresolved after the per-row
    probes) are split into 1024-edge segments taken by whichever workgroups are free."""
    ds, o, e = plaw
    for seeds in ([11, 12, 13], [0, 7919] + [int(v) for v in datagen.sample_vids(40 + qi, ds.n, 10)]):
        q = PL_Q[qi].replace("{S}", ", ".join(str(v) for v in seeds))
        _run(e, o, ds.space, q, factor)


@pytest.fixture(scope="module")
def snb():
    ds = fixtures.snb_dataset(3000, threads=8)
    o = oracle.Oracle()
    o.set_flags(threads=8)
    ds.load_oracle(o)
    e = engine.Engine(0)
    ds.load_engine(e)
    yield ds, o, e
    e.close()


SNB_Q = [
    "GO 4 STEPS FROM {S} OVER knows WHERE knows.creationDate > 1400000000 YIELD knows._dst, $$.person.age",
    "GO 3 STEPS FROM {S} OVER knows, likes YIELD knows._dst, likes._dst",
    "GO 3 STEPS FROM {S} OVER knows BIDIRECT YIELD knows._dst",
    "GO 2 STEPS FROM {S} OVER * REVERSELY YIELD knows._dst, likes._dst, hasCreator._dst",
]


@pytest.mark.parametrize("factor", FACTORS)
@pytest.mark.parametrize("qi", range(len(SNB_Q)))
def test_pull_snb_multitype(snb, qi, factor):
    ds, o, e = snb
    seeds = [int(v) for v in datagen.sample_vids(700 + qi, ds.np, 200)]
    _run(e, o, ds.space, SNB_Q[qi].replace("{S}", ", ".join(str(v) for v in seeds)), factor)


@pytest.fixture(scope="module")
def nba():
    ds = fixtures.nba()
    o = oracle.Oracle()
    ds.load_oracle(o)
    e = engine.Engine(0)
    ds.load_engine(e)
    yield ds, o, e
    e.close()


MULTI = [c for c in CASES if "STEPS" in c["query"] and not c.get("error")]


@pytest.mark.parametrize("case", MULTI, ids=[f"L{c['line']}" for c in MULTI])
def test_pull_gotest_nba(nba, case):
    """GoTest multi-step answers with every intermediate hop pulled."""
    ds, o, e = nba
    q = fixtures.nba_query(case["query"])
    _run(e, o, ds.space, q, 1)
    e.set_flag("pull_factor", 1)
    r = e.go(ds.space, ngql.parse_go(q))
    got = fixtures.normalize_cells(r.rows)
    if case.get("ok_only"):                  # compared with the oracle by _run
        assert r.ok
        return
    assert got == ([] if case.get("empty") else fixtures.nba_expected(case["rows"]))


def _skewed_space(variant):
    """200 vertices with out-edges e(w INT); the in-edges (-e) are the exact transpose except as the
    variant says: "drop" omits one in-edge, "wrong" points one in-edge at another source."""
    import random
    from nebula_amd import kvfmt
    rnd = random.Random(7)
    b = kvfmt.KVBatch()
    edges = sorted({(rnd.randrange(200), rnd.randrange(200)) for _ in range(1500)})
    nparts = 5
    for i, (src, dst) in enumerate(edges):
        row = kvfmt.encode_row([kvfmt.INT], [i])
        b.put(kvfmt.edge_key(src % nparts + 1, src, 1, 0, dst), row)
        if variant == "drop" and i == 100:
            continue
        isrc = (src + 1) % 200 if variant == "wrong" and i == 100 else src
        b.put(kvfmt.edge_key(dst % nparts + 1, dst, -1, 0, isrc), row)
    return fixtures.Dataset(3, nparts, [fixtures.SchemaDef(True, 1, "e", [("w", kvfmt.INT)])], b)


@pytest.mark.parametrize("variant", ["drop", "wrong", "exact"])
def test_pull_needs_exact_mirror(variant):
    """Pull is used only when the in-slot is the exact transpose of the out-slot (checked at commit);
    otherwise every hop pushes and the rows still equal the oracle's."""
    ds = _skewed_space(variant)
    o = oracle.Oracle()
    ds.load_oracle(o)
    with engine.Engine(0) as e:
        ds.load_engine(e)
        q = "GO 3 STEPS FROM 1, 2, 3, 50 OVER e YIELD e._dst, e.w"
        pulled = _run(e, o, ds.space, q, 1, mirrored=variant == "exact")
        assert (pulled > 0) == (variant == "exact")
        _run(e, o, ds.space, "GO 3 STEPS FROM 1, 2, 3, 50 OVER e REVERSELY YIELD e._dst, e.w", 1,
             mirrored=variant == "exact")


def test_pull_epoch_wrap(rmat12):
    """140 pulled queries in a row: the one-byte mark epoch wraps (marks cleared, the frontier
    re-marked) several times without losing a frontier."""
    ds, o, e = rmat12
    seeds = datagen.sample_vids(4242, 1 << ds.scale, 8)
    q = "GO 4 STEPS FROM " + ", ".join(str(int(v)) for v in seeds) + " OVER e YIELD e._dst"
    s = ngql.parse_go(q)
    ref = fixtures.normalize_cells(o.go(ds.space, s).rows)
    e.set_flag("pull_factor", 1)
    for i in range(140):
        got = e.go(ds.space, s)
        assert got.ok and fixtures.normalize_cells(got.rows) == ref, i


DENSE_Q = RMAT_Q + [
    "GO 3 STEPS FROM {S} OVER e WHERE $^.vt.v0 > 100 YIELD e._src, e._dst, $^.vt.name, $$.vt.v0",
    "GO 2 STEPS FROM {S} OVER e REVERSELY WHERE e.p0 < 60 YIELD e._src, e._dst, e.p1",
    "GO 3 STEPS FROM {S} OVER e WHERE e.p1 % (e.p0 - e.p0) > 1 YIELD e._dst",          # fails (division by zero)
]


@pytest.fixture(scope="module")
def rmat12_host():
    ds = fixtures.RmatDataset(12, with_in=True, with_tag=True)
    o = oracle.Oracle()
    o.set_flags(threads=8)
    ds.load_oracle(o)
    e = engine.Engine(0)
    ds.load_engine(e)
    yield ds, o, e
    e.close()
    o.close()


@pytest.mark.parametrize("dense,close_total", [(1, 1), (1, 0), (0, 1)])
def test_dense_final_hop(rmat12_host, dense, close_total):
    """The final hop over every CSR position of its slot, reading the frontier from the pull's marks
    (flag dense_final; no next-frontier list, no entry arrays), on and off: rows, hop statistics and
    errors equal the oracle's, for typed cells, $^ / $$ props and src rows, REVERSELY, and a device-resident
    compact YIELD-only result (the bench's layout) compared by row digest. close_total 1: the hop's
    frontier total (the statistics) summed by the final hop's close (flag dense_close_total), 0: its own launch."""
    ds, o, e = rmat12_host
    e.set_flag("dense_final", dense)
    e.set_flag("dense_close_total", close_total)
    e.set_flag("pull_factor", 1)
    before = e.get_flag("dense_finals")
    try:
        for qi, q in enumerate(DENSE_Q):
            seeds = datagen.sample_vids(1700 + qi, 1 << ds.scale, 30)
            text = q.replace("{S}", ", ".join(str(int(v)) for v in seeds))
            s = ngql.parse_go(text)
            got, ref = e.go(ds.space, s), o.go(ds.space, s)
            assert got.ok == ref.ok, (text, got.error, ref.error)
            if not ref.ok:
                continue
            assert got.hop_edges == ref.hop_scanned, text
            assert fixtures.normalize_cells(got.rows) == fixtures.normalize_cells(ref.rows), text
        # the bench's placement
        seeds = datagen.sample_vids(1799, 1 << ds.scale, 60)
        s = ngql.parse_go(f"GO 3 STEPS FROM {', '.join(str(int(v)) for v in seeds)} OVER e WHERE e.p0 < 50 "
                          "YIELD e._dst, e._rank, e.p0, e.p1")
        ref = o.go(ds.space, s)
        cols = [np.array([int(r[c][1]) for r in ref.rows], dtype=np.int64) for c in range(4)]
        want = oracle.row_digest([np.zeros(len(ref.rows), np.int64)] + cols)
        prep = e.prepare_go(ds.space, s, on_device=True, compact=True, yield_only=True)
        r = e.go(ds.space, prep, rows=False, device_digest=True)
        assert r.ok and r.hop_edges == ref.hop_scanned and tuple(r.device_digest) == tuple(want)
        assert r.hop_frontier == ref.hop_frontier, (r.hop_frontier, ref.hop_frontier)
        got = e.go_batch([prep] * 6, digests=True)
        assert all(g[0] == 0 and tuple(g[3]) == tuple(want) for g in got)
    finally:
        e.set_flag("dense_final", 1)
        e.set_flag("dense_close_total", 1)
        e.set_flag("pull_factor", 200)
    used = e.get_flag("dense_finals") - before
    assert (used > 0) if dense else (used == 0)
