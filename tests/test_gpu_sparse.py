"""Sparse intermediate hops against the oracle.

A push hop whose scanned edges are few next to the shard's rows (E * sparse_factor <= V) builds the next
frontier in the expansion itself (kernels.h SparseArgs, k_expand_sparse): one atomicOr per edge on the
frontier bitmap dedups the destinations, and each workgroup reserves its new rows' frontier places and
edge offsets with one atomic, so the hop costs O(E) instead of a compaction sweep over every row of the
shard (GoExecutor::getDstIdsFromResp keeps a hop's dsts as a set, src/graph/GoExecutor.cpp:675-718).

Every query runs with sparse forced on every push hop (sparse_factor -1), off (0) and at the default,
each combined with pull off and forced, and all must equal the oracle, per-hop scanned edges included.
The bitmap's clean state (all zero before a sparse hop, kept by compactions that write it as zeros)
is exercised by running the cases back to back in one engine, sparse and pulled hops interleaved.
"""
import numpy as np
import pytest

from nebula_amd import datagen, engine, ngql
from oracle import oracle
from tests import fixtures
from tests.golden.gotest_cases import CASES
from tests.test_gpu_pull import PL_Q, RMAT_Q, SNB_Q

pytestmark = pytest.mark.gpu

SPARSE = [-1, 0, 16]
PULL = [0, 1, 200]


def _run(e, o, space, q, sparse, pull, digest=False):
    """digest: compare the sorted 128-bit row digests (large results) instead of the typed cells"""
    s = ngql.parse_go(q)
    e.set_flag("sparse_factor", sparse)
    e.set_flag("pull_factor", pull)
    before = e.get_flag("sparse_hops")
    if digest:
        got = e.go(space, s, columnar=True, rows=False, digest_fn=oracle.digest_columns)
    else:
        got = e.go(space, s)
    used = e.get_flag("sparse_hops") - before
    ref = o.go(space, s, digest=digest)
    assert got.ok == ref.ok, (got.error, ref.error)
    if ref.ok:
        assert got.hop_edges[:len(ref.hop_scanned)] == ref.hop_scanned[:len(got.hop_edges)]
        if digest:
            assert got.nrows == ref.nrows and np.array_equal(got.digests, ref.digests)
        else:
            assert fixtures.normalize_cells(got.rows) == fixtures.normalize_cells(ref.rows)
    if sparse == 0:
        assert used == 0
    if sparse < 0 and pull == 0 and ref.ok and any(h > 0 for h in got.hop_edges[:-1]):
        assert used > 0                       # forced: every push hop with edges is sparse
    return used


@pytest.fixture(scope="module")
def rmat12():
    ds = fixtures.RmatDataset(12, with_in=True, with_tag=True)
    o = oracle.Oracle()
    o.set_flags(threads=8)
    ds.load_oracle(o)
    e = engine.Engine(0)
    ds.load_engine(e)
    yield ds, o, e
    e.close()
    o.close()


@pytest.mark.parametrize("pull", PULL)
@pytest.mark.parametrize("sparse", SPARSE)
@pytest.mark.parametrize("qi", range(len(RMAT_Q)))
def test_sparse_rmat12(rmat12, qi, sparse, pull):
    ds, o, e = rmat12
    for k, n in ((0, 30), (1, 3)):
        seeds = datagen.sample_vids(900 + 10 * qi + k, 1 << ds.scale, n)
        _run(e, o, ds.space, RMAT_Q[qi].replace("{S}", ", ".join(str(int(v)) for v in seeds)), sparse, pull)


def test_sparse_rmat16_bench_query_uses_it_by_default():
    """The bench query at scale 16 (V = 65 K rows): hop 1 of 20 seeds scans few edges, so it is sparse at
    the default factor; hop 2 pulls from the bitmap the sparse hop wrote."""
    ds = fixtures.RmatDataset(16, threads=8, with_in=True)
    o = oracle.Oracle()
    o.set_flags(threads=8)
    ds.load_oracle(o)
    with engine.Engine(0) as e:
        ds.load_engine(e)
        for i in range(4):
            seeds = datagen.rmat_seeds(16, 20, 16, 42, 5 + i, threads=8)
            q = (f"GO 3 STEPS FROM {', '.join(str(int(v)) for v in seeds)} OVER e WHERE e.p0 < 50 "
                 "YIELD e._dst, e._rank, e.p0, e.p1")
            assert _run(e, o, ds.space, q, 16, 200, digest=True) >= 1
            _run(e, o, ds.space, q, 0, 200, digest=True)
    o.close()


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
    o.close()


@pytest.mark.parametrize("sparse", SPARSE)
@pytest.mark.parametrize("qi", range(len(PL_Q)))
def test_sparse_powerlaw_supernodes(plaw, qi, sparse):
    """Supernode destinations: thousands of edges of one hop hit the same bitmap word."""
    ds, o, e = plaw
    for seeds in ([11, 12, 13], [0, 7919] + [int(v) for v in datagen.sample_vids(40 + qi, ds.n, 10)]):
        _run(e, o, ds.space, PL_Q[qi].replace("{S}", ", ".join(str(v) for v in seeds)), sparse, 0)


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
    o.close()


@pytest.mark.parametrize("pull", [0, 1])
@pytest.mark.parametrize("sparse", SPARSE)
@pytest.mark.parametrize("qi", range(len(SNB_Q)))
def test_sparse_snb_multitype(snb, qi, sparse, pull):
    """Several edge-type slots per hop: a new row's entries (one per slot) take consecutive places."""
    ds, o, e = snb
    seeds = [int(v) for v in datagen.sample_vids(700 + qi, ds.np, 200)]
    _run(e, o, ds.space, SNB_Q[qi].replace("{S}", ", ".join(str(v) for v in seeds)), sparse, pull)


MULTI = [c for c in CASES if "STEPS" in c["query"] and not c.get("error")]


def test_sparse_gotest_nba():
    """GoTest multi-step answers with every push hop sparse."""
    ds = fixtures.nba()
    o = oracle.Oracle()
    ds.load_oracle(o)
    with engine.Engine(0) as e:
        ds.load_engine(e)
        for case in MULTI:
            q = fixtures.nba_query(case["query"])
            _run(e, o, ds.space, q, -1, 0)
            if not case.get("ok_only"):
                r = e.go(ds.space, ngql.parse_go(q))
                assert fixtures.normalize_cells(r.rows) == ([] if case.get("empty") else fixtures.nba_expected(case["rows"]))
    o.close()


def test_sparse_bitmap_clean_state_across_spaces():
    """the frontier bitmap's zero state is keyed on the allocation and the words a
    compaction zeroed, not on the pointer alone. A GO 2 STEPS in the larger space leaves its sparse hop's
    bits set over its rows; a GO 3 STEPS in the smaller space clears only its own words, then its hop-2
    compaction writes them as zeros and marks the bitmap clean; the larger space's next sparse hop must
    still clear the words past the smaller space's rows, or its dedup sees stale bits and drops rows."""
    big = fixtures.RmatDataset(13, with_in=True)
    small = fixtures.GenDataset(datagen.RMAT_SPACE + 7, 100, datagen.rmat(10, 16, 43, 100, True, False),
                                datagen.rmat_schemas(False))
    o = oracle.Oracle()
    o.set_flags(threads=8)
    big.load_oracle(o)
    small.load_oracle(o)
    with engine.Engine(0) as e:
        big.load_engine(e)
        small.load_engine(e)
        e.set_flag("pull_factor", 0)
        e.set_flag("sparse_factor", 16)
        sb = datagen.sample_vids(11, 1 << 13, 4)
        ss = datagen.sample_vids(12, 1 << 10, 30)
        qb = f"GO 2 STEPS FROM {', '.join(str(int(v)) for v in sb)} OVER e YIELD e._src, e._dst, e.p0"
        qs = f"GO 3 STEPS FROM {', '.join(str(int(v)) for v in ss)} OVER e YIELD e._dst, e.p1"
        for space, q in [(big.space, qb), (small.space, qs), (big.space, qb), (small.space, qs), (big.space, qb)]:
            s = ngql.parse_go(q)
            got, ref = e.go(space, s), o.go(space, s)
            assert got.ok and ref.ok
            assert got.hop_edges == ref.hop_scanned
            assert fixtures.normalize_cells(got.rows) == fixtures.normalize_cells(ref.rows)
        assert e.get_flag("sparse_hops") >= 3
    o.close()
