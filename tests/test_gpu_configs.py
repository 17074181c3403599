"""BASELINE.json configs at their stated sizes, HIP path (C ABI, device 0) against the oracle.

* C1  NBA fixture (TraverseTestBase), GO 2 STEPS OVER like / serve WHERE ... YIELD ...
* C2  RMAT scale 22, edge factor 16, 100 parts, e(p0 INT, p1 INT) with in-edges stored (bench.py's
      graph), the bench query `GO 3 STEPS ... WHERE e.p0 < 50 YIELD e._dst, e._rank, e.p0, e.p1`: the
      bench step itself (1000 seeds) row-for-row against the oracle with pull default / forced / off;
      another 1000-seed batch through size-independent properties.
* C4  power law with 4 supernodes of in-degree ~1e6 (one frontier entry spans ~470 chunks of 2048
      edges), GO 1/2 STEPS REVERSELY.
* C5  LDBC-SNB-like (knows / likes / hasCreator, string + int props), a 10k-vid batch, GO 4 STEPS,
      compound WHERE, multi-column YIELD.
(C3, 8 shards, is rehearsed in tests/test_multishard.py at world 8 over the host exchange.)

Large results are compared as sorted 128-bit digests of each row's serialized cells (the oracle's
ColumnValue bytes; oracle.digest_columns builds the same bytes from the device's host_columnar
arrays), so a difference in any row, value, type or multiplicity fails.
"""
import numpy as np
import pytest

from nebula_amd import datagen, engine, ngql
from oracle import oracle
from tests import fixtures

pytestmark = pytest.mark.gpu

C2_QUERY = "GO 3 STEPS FROM {S} OVER e WHERE e.p0 < {K} YIELD e._dst, e._rank, e.p0, e.p1"


def _digest_go(e, space, s, pushdown=True):
    r = e.go(space, s, pushdown=pushdown, columnar=True, rows=False, digest_fn=oracle.digest_columns)
    assert r.ok, r.error
    return r


def _same_digests(got, ref):
    assert ref.ok, ref.error
    assert got.nrows == ref.nrows
    assert got.col_types == ref.col_types or ref.nrows == 0
    assert np.array_equal(got.digests, ref.digests)


def _seed_list(vids):
    return ", ".join(str(int(v)) for v in vids)


# ----------------------------------------------------------------------------------------- C1
C1_QUERIES = [
    "GO 2 STEPS FROM {P:Tim Duncan}, {P:Tony Parker}, {P:LeBron James} OVER like WHERE like.likeness > 80 "
    "YIELD like._dst, like.likeness, $^.player.name, $$.player.age",
    "GO 2 STEPS FROM {P:Tim Duncan}, {P:Kobe Bryant}, {P:Dwyane Wade} OVER like, serve "
    "WHERE $^.player.age >= 30 YIELD like._dst, serve._dst, serve.start_year, like.likeness, $$.team.name",
    "GO 2 STEPS FROM {P:Manu Ginobili} OVER serve, like REVERSELY WHERE $^.player.age > 30 "
    "YIELD serve._dst, like._dst, $^.player.name",
]


@pytest.mark.parametrize("mode", ["jit", "vm"])
@pytest.mark.parametrize("pushdown", [True, False])
@pytest.mark.parametrize("qi", range(len(C1_QUERIES)))
def test_c1_nba_go2(qi, pushdown, mode):
    ds = fixtures.nba()
    o = oracle.Oracle()
    ds.load_oracle(o)
    with engine.Engine(0) as e:
        e.set_flag("jit", 1 if mode == "jit" else 0)
        ds.load_engine(e)
        s = ngql.parse_go(fixtures.nba_query(C1_QUERIES[qi]))
        ref = o.go(ds.space, s, pushdown=pushdown)
        got = e.go(ds.space, s, pushdown=pushdown)
        assert got.ok == ref.ok, (got.error, ref.error)
        assert ref.rows
        assert fixtures.normalize_cells(got.rows) == fixtures.normalize_cells(ref.rows)
        assert got.col_types == ref.col_types


# ----------------------------------------------------------------------------------------- C2
@pytest.fixture(scope="module")
def c2(rmat22):
    ds, o = rmat22
    e = engine.Engine(0)
    ds.load_engine(e)
    info = e.info(ds.space)
    assert info.vertices > 2_000_000 and info.edges > 60_000_000          # scale 22, ef 16, collapsed
    yield ds, o, e
    e.close()


@pytest.fixture(scope="module")
def c2_ref(c2):
    """bench.py's first timed plan (1000 seeds, sample seed 42) and the oracle's result of it (row digests),
    computed once for the tests below"""
    ds, o, e = c2
    seeds = datagen.rmat_seeds(22, 1000, 16, 42, 42, threads=16)
    s = ngql.parse_go(C2_QUERY.replace("{S}", _seed_list(seeds)).replace("{K}", "50"))
    return s, o.go(ds.space, s, digest=True)


@pytest.mark.timeout(600)
def test_c2_bench_step_vs_oracle(c2, c2_ref):
    """The exact step bench.py times (its first plan: 1000 seeds, sample seed 42), on the graph bench.py
    builds (in-edges stored, so hop 2 may pull), row for row against the oracle: sorted 128-bit row
    digests and every hop's scanned edges, with pull at its default factor (hop 2 pulls: the hops a
    factor of 1 would pull too), off (factor 0), and once on the interpreter kernels."""
    ds, o, e = c2
    s, ref = c2_ref
    assert ref.ok and ref.nrows > 20_000_000 and sum(ref.hop_scanned) > 60_000_000
    default = e.get_flag("pull_factor")
    pulls = {}
    try:
        for factor, jit in ((default, 1), (0, 1), (default, 0)):
            e.set_flag("pull_factor", factor)
            e.set_flag("jit", jit)
            before = e.get_flag("pull_hops")
            got = _digest_go(e, ds.space, s)
            pulls[(factor, jit)] = e.get_flag("pull_hops") - before
            assert got.hop_edges == ref.hop_scanned, (factor, jit)
            _same_digests(got, ref)
    finally:
        e.set_flag("pull_factor", default)
        e.set_flag("jit", 1)
    assert pulls[(0, 1)] == 0 and pulls[(default, 1)] >= 1
    # the bench's own result placement: rows in HBM with compact integer arrays (compact_results), the
    # YIELD columns only (yield_only: no src row array), fetched and widened, digest for digest equal to
    # the oracle's rows; and with the row arrays (bench.py --row-arrays)
    for yield_only in (True, False):
        got = e.go(ds.space, s, on_device=True, fetch=True, compact=True, yield_only=yield_only)
        assert got.ok and got.hop_edges == ref.hop_scanned
        key_w, col_w = got.dev_widths
        # src / dst vids < 2^31, p0 < 100; every rank 0: a constant column (width 0, no bytes per row)
        assert col_w == [4, 0, 1, 8] and key_w[1:] == [4, 0]
        assert yield_only or got.src is not None
        assert got.dev_consts[1][1] == 0
        cols = [np.ascontiguousarray(x) for x, _, _ in got.dev_cols]
        assert all(ln is None and t is None for _, ln, t in got.dev_cols)
        digests = oracle.digest_columns(got.col_types, got.nrows, [c.ctypes.data for c in cols], [None] * 4, [None] * 4)
        assert got.nrows == ref.nrows and np.array_equal(digests, ref.digests)
        del cols, got


@pytest.mark.timeout(300)
def test_c2_bench_batch_pinned(c2, c2_ref):
    """The timed path itself at C2 (What's weak #2): bench.py's own timed plans — its
    sentence(i) seeds (rmat_seeds(..., 42, 42 + i)), 20 of them, compact YIELD-only device results — run
    through ngx_go_batch (four lanes, two front streams, two final streams, deferred frees, per-lane rows)
    with digests. Four small queries go first, so lanes 1 to 3 hold small scratch and grow in the middle
    of the batch when their first C2 query arrives. Every query's code, rows, edges and row digest equal
    the same plan through ngx_go; plan 0's rows, fetched, equal the oracle's (sorted 128-bit row digests)
    and their row digest is the batch's."""
    ds, o, e = c2
    q = C2_QUERY.replace("{K}", "50")
    sents = [ngql.parse_go(q.replace("{S}", _seed_list(datagen.rmat_seeds(22, 1000, 16, 42, 42 + i, threads=16))))
             for i in range(20)]
    small = [ngql.parse_go(q.replace("{S}", _seed_list(datagen.rmat_seeds(22, 3, 16, 42, 900 + i, threads=16))))
             for i in range(4)]
    preps = [e.prepare_go(ds.space, s, on_device=True, compact=True, yield_only=True) for s in small + sents]
    e.set_flag("release_lanes", 1)                  # lanes 1 to 3 start empty: they grow inside the batch
    assert e.get_flag("batch_lanes") == 4
    before = e.get_flag("batch_overlaps")
    got = e.go_batch(preps, digests=True)
    assert e.get_flag("batch_overlaps") - before >= len(preps) - 2
    # the same batch with 4 reservation groups (64 K-row blocks filling up faster per group, more closes in
    # flight per lane) and with one final stream: r06 found a lane's next final hop racing the lane's last
    # close on two final streams (C2, 4 groups)
    e.set_flag("resv_groups", 4)
    try:
        got4 = e.go_batch(preps, digests=True)
    finally:
        e.set_flag("resv_groups", 8)
    e.set_flag("batch_finals", 1)
    try:
        got1 = e.go_batch(preps, digests=True)
    finally:
        e.set_flag("batch_finals", 2)
    for i, p in enumerate(preps):
        alone = e.go(ds.space, p, rows=False, device_digest=True)
        assert alone.ok
        for g in (got, got4, got1):
            code, nrows, edges, dig = g[i]
            assert code == 0 and (nrows, edges) == (alone.nrows, sum(alone.hop_edges)), i
            assert tuple(dig) == tuple(alone.device_digest), i
    # plan 0 against the oracle: its fetched rows' 128-bit digests, and the batch digest of those rows
    _, ref = c2_ref                                 # the same plan as sents[0] (seed sample 42 + 0)
    assert ref.ok and ref.nrows == got[4][1] and sum(ref.hop_scanned) == got[4][2]
    r = e.go(ds.space, sents[0], on_device=True, fetch=True, compact=True, yield_only=True)
    assert r.ok
    cols = [np.ascontiguousarray(x) for x, _, _ in r.dev_cols]
    digests = oracle.digest_columns(r.col_types, r.nrows, [c.ctypes.data for c in cols], [None] * 4, [None] * 4)
    assert np.array_equal(digests, ref.digests)
    assert oracle.row_digest([np.zeros(r.nrows, np.int64)] + cols) == tuple(got[4][3])
    del cols, r, digests


@pytest.mark.timeout(600)
def test_c2_full_batch_properties(c2):
    """The bench step through properties that hold at any size, beside the oracle check above:
      * without WHERE every scanned edge of the last hop is a row;
      * WHERE p0 < 50 and WHERE p0 >= 50 partition those rows (filter linearity), and the rows of
        `p0 < 50` are exactly the p0 < 50 rows of the unfiltered result (p0 values counted)."""
    ds, o, e = c2
    seeds = _seed_list(datagen.rmat_seeds(22, 1000, 16, 42, 43, threads=16))
    q50 = ngql.parse_go(C2_QUERY.replace("{S}", seeds).replace("{K}", "50"))
    lt = e.go(ds.space, q50, on_device=True)
    everything = e.go(ds.space, ngql.parse_go(
        f"GO 3 STEPS FROM {seeds} OVER e YIELD e._dst, e._rank, e.p0, e.p1"), on_device=True, fetch=True)
    ge = e.go(ds.space, ngql.parse_go(
        f"GO 3 STEPS FROM {seeds} OVER e WHERE e.p0 >= 50 YIELD e._dst"), on_device=True)
    assert lt.ok and everything.ok and ge.ok
    assert lt.nrows > 20_000_000
    assert everything.nrows == everything.hop_edges[-1] == lt.hop_edges[-1]
    assert lt.nrows + ge.nrows == everything.nrows
    p0 = everything.dev_cols[2][0]
    assert int(np.count_nonzero(p0 < 50)) == lt.nrows


# ----------------------------------------------------------------------------------------- C4
@pytest.fixture(scope="module")
def c4():
    ds = fixtures.powerlaw_dataset(8_000_000, ef=2, nsuper=4, superdeg=1_000_000, threads=16)
    o = oracle.Oracle()
    o.set_flags(threads=16)
    ds.load_oracle(o, threads=16)
    e = engine.Engine(0)
    ds.load_engine(e)
    ds.rows.free()
    yield ds, o, e
    e.close()
    o.close()


SUPERNODES = [0, 7919, 15838, 23757]          # datagen.cpp ngd_powerlaw: (j / superdeg) * 7919 % n

C4_QUERIES = [
    "GO 1 STEPS FROM {S} OVER pl REVERSELY YIELD pl._dst, pl.w, pl.score",
    "GO 2 STEPS FROM {S} OVER pl REVERSELY WHERE pl.w == 7 YIELD pl._dst, pl._src, pl.score",
    "GO 2 STEPS FROM {S} OVER pl REVERSELY WHERE pl.w < 3 && pl.score > 0.5 YIELD pl._dst, pl.w * 2 + 1",
]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("qi", range(len(C4_QUERIES)))
def test_c4_supernodes_reversely(c4, qi):
    """Supernode seeds: in-degree ~0.94e6 each, so a single frontier entry covers ~460 workgroup chunks
    (edge-balanced expansion); REVERSELY has no pushdown, graphd evaluates WHERE (GoExecutor.cpp:528-533).
    Generated and interpreter kernels."""
    ds, o, e = c4
    s = ngql.parse_go(C4_QUERIES[qi].replace("{S}", _seed_list(SUPERNODES)))
    ref = o.go(ds.space, s, digest=True)
    for mode in (1, 0):
        e.set_flag("jit", mode)
        got = _digest_go(e, ds.space, s)
        assert got.hop_edges == ref.hop_scanned
        assert got.hop_edges[0] > 3_600_000                  # ~4 x 0.94e6 in-edges in hop 1
        _same_digests(got, ref)
        assert got.nrows > 0
    e.set_flag("jit", 1)


# ----------------------------------------------------------------------------------------- C5
@pytest.fixture(scope="module")
def c5():
    ds = fixtures.snb_dataset(50_000, knows_deg=20, likes_deg=10, threads=16)
    o = oracle.Oracle()
    o.set_flags(threads=16)
    ds.load_oracle(o, threads=16)
    e = engine.Engine(0)
    ds.load_engine(e)
    yield ds, o, e
    e.close()
    o.close()


C5_QUERIES = [
    "GO 4 STEPS FROM {S} OVER knows WHERE knows.creationDate > 1400000000 && $^.person.gender == \"female\" "
    "YIELD knows._dst, knows.weight, $^.person.firstName, $$.person.age",
    "GO 4 STEPS FROM {S} OVER knows, likes WHERE $^.person.age < 40 && $^.person.gender == \"male\" "
    "YIELD knows._dst, likes._dst, likes.creationDate, knows.weight, $^.person.firstName",
    "GO 4 STEPS FROM {S} OVER likes, hasCreator WHERE $$.post.lang == \"en\" || $$.person.age > 60 "
    "YIELD likes._dst, hasCreator._dst, $$.post.content, $$.post.length, $$.person.firstName",
]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("pushdown", [True, False])
@pytest.mark.parametrize("qi", range(len(C5_QUERIES)))
def test_c5_snb_10k_batch(c5, qi, pushdown):
    """A 10 000-person seed batch, GO 4 STEPS, compound WHERE over edge / $^ / $$ props, string and int
    YIELD columns (strings delivered as host pointers in the columnar result). Generated and
    interpreter kernels."""
    ds, o, e = c5
    seeds = datagen.sample_vids(9000 + qi, ds.np, 10_000)
    s = ngql.parse_go(C5_QUERIES[qi].replace("{S}", _seed_list(seeds)))
    ref = o.go(ds.space, s, pushdown=pushdown, digest=True)
    for mode in (1, 0):
        e.set_flag("jit", mode)
        got = _digest_go(e, ds.space, s, pushdown=pushdown)
        assert got.hop_edges == ref.hop_scanned
        assert got.hop_frontier[0] == 10_000
        _same_digests(got, ref)
        assert got.nrows > 0
    e.set_flag("jit", 1)
