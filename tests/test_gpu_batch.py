"""ngx_go_batch (the native loop over prepared GO plans) against the same plans run one ngx_go at a time
and against the oracle, with the batch pipeline on and off.

With "batch_pipeline" on, consecutive device-resident plans overlap: a query whose final hop is enqueued
yields before it waits for its row count, and the next one prepares and enqueues its first hops (seed,
sparse and pulled hops, program uploads) behind it on the stream (engine.cpp GoPipe). Every query's code,
row count, per-hop scanned edges (summed) and the value digest of its device-resident rows
(ngx_go_result_digest) must be what the query has alone — mixes of pipelinable plans with DISTINCT, host
results, failing queries, empty frontiers and changing programs, in orders that put each kind before
and after the others.
"""
import random

import numpy as np
import pytest

from nebula_amd import datagen, engine, ngql
from oracle import oracle
from tests import fixtures
from tests.test_gpu_pull import RMAT_Q

pytestmark = pytest.mark.gpu

EXTRA_Q = [
    "GO FROM {S} OVER e YIELD e._dst, e.p0",                               # one hop
    "GO 2 STEPS FROM {S} OVER e WHERE e.p1 % (e.p0 - e.p0) > 1 YIELD e._dst",   # fails (division by zero)
    "GO 3 STEPS FROM 4398046511104 OVER e YIELD e._dst",                     # no such vertex: no rows
    "GO 3 STEPS FROM {S} OVER e WHERE e.p0 < 50 YIELD e._src, e._dst, e._rank, e.p0, e.p1",
]


@pytest.fixture(scope="module")
def rmat():
    ds = fixtures.RmatDataset(12, with_in=True, with_tag=True)
    o = oracle.Oracle()
    o.set_flags(threads=8)
    ds.load_oracle(o)
    e = engine.Engine(0)
    ds.load_engine(e)
    yield ds, o, e
    e.close()
    o.close()


def _queries(ds, n_seed_sets=2):
    out = []
    for qi, q in enumerate(RMAT_Q + EXTRA_Q):
        for k in range(n_seed_sets):
            seeds = datagen.sample_vids(5100 + 10 * qi + k, 1 << ds.scale, (25, 3)[k % 2])
            out.append(q.replace("{S}", ", ".join(str(int(v)) for v in seeds)))
    return out


def _prepare(e, ds, q, mode):
    s = ngql.parse_go(q)
    if mode == "compact":
        return e.prepare_go(ds.space, s, on_device=True, compact=True)
    if mode == "lean":                      # the bench's plans: compact YIELD columns only
        return e.prepare_go(ds.space, s, on_device=True, compact=True, yield_only=True)
    if mode == "device":
        return e.prepare_go(ds.space, s, on_device=True)
    return e.prepare_go(ds.space, s)


def _alone(e, ds, prep):
    """(code, rows, edges, digest) of one prepared plan through ngx_go"""
    on_dev = bool(prep.plan.result_on_device)
    r = e.go(ds.space, prep, rows=False)
    dig = (0, 0, 0)
    if r.ok and on_dev:
        r2 = e.go(ds.space, prep, rows=False, device_digest=True)
        dig = r2.device_digest
    return r.code, r.nrows, int(sum(r.hop_edges)) if r.ok else None, dig


@pytest.mark.parametrize("pipeline", [1, 0])
def test_batch_equals_one_at_a_time(rmat, pipeline):
    ds, o, e = rmat
    rng = random.Random(77)
    qs = _queries(ds)
    modes = ["lean", "compact", "device", "host"]
    items = [(q, m) for q in qs for m in modes]
    rng.shuffle(items)
    # runs of pipelinable plans (the bench's shape) between the mixed ones
    items = [(q, "compact") for q in qs[:6]] + items + [(q, "compact") for q in qs[-6:]]
    preps = [_prepare(e, ds, q, m) for q, m in items]
    want = [_alone(e, ds, p) for p in preps]
    e.set_flag("batch_pipeline", pipeline)
    before = e.get_flag("batch_overlaps")
    got = e.go_batch(preps, digests=True)
    overlaps = e.get_flag("batch_overlaps") - before
    e.set_flag("batch_pipeline", 1)
    for (q, m), w, g in zip(items, want, got):
        code, rows, edges, dig = g
        assert code == w[0], (q, m, g, w)
        if code == 0:
            assert (rows, edges) == (w[1], w[2]), (q, m)
            # DISTINCT keeps one row of each group, whichever: its src (hashed with the row) is not fixed
            if "DISTINCT" not in q:
                assert tuple(dig) == tuple(w[3]), (q, m)
    if pipeline:
        assert overlaps >= 10
    else:
        assert overlaps == 0


def test_batch_rows_equal_oracle(rmat):
    """A pipelined run of the bench's query shape: every query's digest equals the oracle's rows."""
    ds, o, e = rmat
    preps, refs = [], []
    for k in range(12):
        seeds = datagen.sample_vids(6200 + k, 1 << ds.scale, 40)
        w = (" WHERE e.p0 < 50", "", " WHERE e.p0 >= 50")[k % 3]
        # odd k: the bench's plans (yield_only, no e._src: no src row array, the key hashes as 0)
        ys = "e._dst, e._rank, e.p0, e.p1" if k % 2 else "e._src, e._dst, e._rank, e.p0, e.p1"
        q = f"GO 3 STEPS FROM {', '.join(str(int(v)) for v in seeds)} OVER e{w} YIELD {ys}"
        s = ngql.parse_go(q)
        ref = o.go(ds.space, s)
        assert ref.ok
        cols = [np.array([int(r[c][1]) for r in ref.rows], dtype=np.int64) for c in range(len(s.yields))]
        if k % 2:
            refs.append((len(ref.rows), int(sum(ref.hop_scanned)),
                         oracle.row_digest([np.zeros(len(ref.rows), np.int64)] + cols)))
            preps.append(e.prepare_go(ds.space, s, on_device=True, compact=True, yield_only=True))
        else:
            refs.append((len(ref.rows), int(sum(ref.hop_scanned)), oracle.row_digest([cols[0]] + cols)))
            preps.append(e.prepare_go(ds.space, s, on_device=True, compact=True))
    before = e.get_flag("batch_overlaps")
    got = e.go_batch(preps, digests=True)
    assert e.get_flag("batch_overlaps") - before == len(preps) - 1
    for (code, rows, edges, dig), (nrows, scanned, rdig) in zip(got, refs):
        assert code == 0
        assert (rows, edges) == (nrows, scanned)
        assert tuple(dig) == tuple(rdig)


def test_batch_last_result_stays_on_device(rmat):
    """The last query's rows are in HBM after the batch, as ngx_go leaves them: a following ngx_go of the
    same plan returns the same digest, and the context keeps working after a pipelined batch whose last
    query failed."""
    ds, o, e = rmat
    seeds = datagen.sample_vids(31, 1 << ds.scale, 30)
    q = f"GO 3 STEPS FROM {', '.join(str(int(v)) for v in seeds)} OVER e YIELD e._dst, e.p1"
    bad = f"GO 2 STEPS FROM {', '.join(str(int(v)) for v in seeds)} OVER e YIELD e.p1 / (e.p0 - e.p0)"
    p = e.prepare_go(ds.space, ngql.parse_go(q), on_device=True, compact=True)
    pb = e.prepare_go(ds.space, ngql.parse_go(bad), on_device=True, compact=True)
    got = e.go_batch([p, p, pb], digests=True)
    assert [g[0] for g in got] == [0, 0, engine.E_QUERY]
    alone = e.go(ds.space, p, rows=False, device_digest=True)
    assert alone.ok and tuple(got[0][3]) == tuple(got[1][3]) == alone.device_digest
    assert e.go_batch([]) == []


@pytest.mark.parametrize("lanes,close_stream,fronts", [(2, 0, 2), (3, 0, 2), (4, 0, 2), (3, 0, 1), (3, 1, 1), (2, 1, 1),
                                                        (3, 1, 2), (8, 0, 2)])
def test_batch_lanes(rmat, lanes, close_stream, fronts):
    """Deeper pipelines (flag batch_lanes: up to lanes - 1 queries wait for their row counts while the next
    one runs its hops on its own lane and its own result rows), consecutive queries' hops on two front
    streams (flag batch_fronts) or one, with each overlapped final hop's close on the close stream beside
    the next final hop (flag batch_close_stream) or behind it: every query's code, row
    count, scanned edges and row digest are what it has alone, over mixed plans."""
    ds, o, e = rmat
    rng = random.Random(91 + lanes)
    qs = _queries(ds)
    items = [(q, rng.choice(["lean", "compact", "device", "host"])) for q in qs]
    items = [(q, "lean") for q in qs[:8]] + items + [(q, "compact") for q in qs[-8:]]
    preps = [_prepare(e, ds, q, m) for q, m in items]
    want = [_alone(e, ds, p) for p in preps]
    assert e.get_flag("batch_lanes") == 4 and e.get_flag("batch_close_stream") == 1
    assert e.get_flag("batch_fronts") == 2
    e.set_flag("batch_lanes", lanes)
    e.set_flag("batch_close_stream", close_stream)
    e.set_flag("batch_fronts", fronts)
    e.set_flag("batch_finals", 1)                   # one final stream: the close stream is used when asked
    try:
        before = e.get_flag("batch_overlaps")
        got = e.go_batch(preps, digests=True)
        overlaps = e.get_flag("batch_overlaps") - before
        plain = e.go_batch(preps[:12])                  # no digests: nothing read back between the queries
    finally:
        e.set_flag("batch_lanes", 4)
        e.set_flag("batch_close_stream", 1)
        e.set_flag("batch_fronts", 2)
        e.set_flag("batch_finals", 2)
    for (q, m), w, g in list(zip(items, want, got)) + list(zip(items[:12], want[:12], plain)):
        assert g[0] == w[0], (q, m, g, w)
        if g[0] == 0:
            assert (g[1], g[2]) == (w[1], w[2]), (q, m)
            if len(g) > 3 and "DISTINCT" not in q:
                assert tuple(g[3]) == tuple(w[3]), (q, m)
    assert overlaps >= 10
    with pytest.raises(Exception):
        e.set_flag("batch_lanes", 9)


def _digest_fixed(q, mode):
    """A DISTINCT result keeps one row of each group, whichever came first (GoExecutor.cpp:1298-1305): the
    YIELD columns are fixed, the src vid of the row kept is not, and the device digest hashes it (DISTINCT
    plans keep the src row array: yield_only does not apply to them). Their rows are compared as cells."""
    return "DISTINCT" not in q


@pytest.mark.parametrize("groups", [16, 4, 1, 64])
def test_resv_groups(rmat, groups):
    """The final hop's rows reserved over another number of groups (flag resv_groups; 8 = a group per XCD
    by default): every plan's code, rows, edges and row digest as with 8, one at a time and in a pipelined
    batch. (Round 5 saw a digest differ at 16 groups: it was a DISTINCT plan whose digest hashes the src of
    whichever row of a group DISTINCT keeps, which the row placement decides, not a misplaced row.)"""
    ds, o, e = rmat
    qs = _queries(ds)
    items = [(q, m) for q in qs for m in ("lean", "compact")]
    preps = [_prepare(e, ds, q, m) for q, m in items]
    want = [_alone(e, ds, p) for p in preps]
    e.set_flag("resv_groups", groups)
    try:
        assert e.get_flag("resv_groups") == groups
        alone = [_alone(e, ds, p) for p in preps]
        got = e.go_batch(preps, digests=True)
    finally:
        e.set_flag("resv_groups", 8)
    for (q, m), w, a, g in zip(items, want, alone, got):
        assert a[:3] == w[:3] and g[0] == w[0], (q, m)
        if w[0] == 0:
            assert (g[1], g[2]) == (w[1], w[2]), (q, m)
            if _digest_fixed(q, m):
                assert a[3] == w[3] and tuple(g[3]) == tuple(w[3]), (q, m)
    # DISTINCT: the YIELD cells (host rows) are the oracle's under either group count
    for q in {q for q, _ in items if not _digest_fixed(q, "")}:
        s = ngql.parse_go(q)
        ref = o.go(ds.space, s)
        for gr in (groups, 8):
            e.set_flag("resv_groups", gr)
            got = e.go(ds.space, s)
            assert got.ok and ref.ok
            assert fixtures.normalize_cells(got.rows) == fixtures.normalize_cells(ref.rows), (q, gr)


def test_resv_groups_switch(rmat):
    """8 -> 16 -> 8 -> 3 groups on one context, a batch after each switch (the counters are reallocated,
    the block table keeps entries of other geometries, tagged by launch): the bench's query shape equals
    the oracle's rows every time."""
    ds, o, e = rmat
    preps, refs = [], []
    for k in range(4):
        seeds = datagen.sample_vids(7300 + k, 1 << ds.scale, 40)
        q = f"GO 3 STEPS FROM {', '.join(str(int(v)) for v in seeds)} OVER e WHERE e.p0 < 50 YIELD e._dst, e._rank, e.p0, e.p1"
        s = ngql.parse_go(q)
        ref = o.go(ds.space, s)
        assert ref.ok
        cols = [np.array([int(r[c][1]) for r in ref.rows], dtype=np.int64) for c in range(len(s.yields))]
        refs.append((len(ref.rows), int(sum(ref.hop_scanned)), oracle.row_digest([np.zeros(len(ref.rows), np.int64)] + cols)))
        preps.append(e.prepare_go(ds.space, s, on_device=True, compact=True, yield_only=True))
    try:
        for groups in (8, 16, 8, 3, 8):
            e.set_flag("resv_groups", groups)
            got = e.go_batch(preps + preps, digests=True)
            for (code, rows, edges, dig), ref in zip(got, refs + refs):
                assert code == 0 and (rows, edges, tuple(dig)) == (ref[0], ref[1], tuple(ref[2])), groups
            r = e.go(ds.space, preps[0], rows=False, device_digest=True)
            assert r.ok and (r.nrows, tuple(r.device_digest)) == (refs[0][0], tuple(refs[0][2])), groups
    finally:
        e.set_flag("resv_groups", 8)


def test_release_parked_lanes(rmat):
    """the parked lanes' scratch and result rows are freed on request (flag release_lanes, or
    batch_release_lanes after every batch), and later batches give the same outcomes."""
    ds, o, e = rmat
    qs = _queries(ds)[:8]
    preps = [_prepare(e, ds, q, "lean") for q in qs]
    first = e.go_batch(preps, digests=True)
    before = e.get_flag("released_lane_bytes")
    e.set_flag("release_lanes", 1)
    assert e.get_flag("released_lane_bytes") > before
    assert e.go_batch(preps, digests=True) == first
    e.set_flag("batch_release_lanes", 1)
    try:
        mid = e.get_flag("released_lane_bytes")
        assert e.go_batch(preps, digests=True) == first
        assert e.get_flag("released_lane_bytes") > mid
        assert e.go_batch(preps, digests=True) == first
    finally:
        e.set_flag("batch_release_lanes", 0)


def test_batch_bad_plan_reports_every_query():
    """a batch that fails before any query runs (a null plan) reports the error for every
    query; the Python wrapper raises instead of returning zero-filled successes."""
    import ctypes
    with engine.Engine(0) as e:
        codes = (ctypes.c_int32 * 2)()
        arr = (ctypes.c_void_p * 2)(None, None)
        rc = e.L.ngx_go_batch(e.h, ctypes.cast(arr, ctypes.c_void_p), 2, codes, None, None, None)
        assert rc != 0 and list(codes) == [rc, rc]


@pytest.mark.parametrize("lanes,fronts", [(3, 2), (4, 2), (3, 1)])
def test_batch_two_final_streams(rmat, lanes, fronts):
    """Flag batch_finals 2 (the default): consecutive queries' final hops on two final streams (each close after its own
    final hop on that stream), so two final hops of different lanes may run at once: every query's code,
    rows, scanned edges and digest are what it has alone."""
    ds, o, e = rmat
    rng = random.Random(191 + lanes)
    qs = _queries(ds)
    items = [(q, rng.choice(["lean", "compact", "device", "host"])) for q in qs]
    items = [(q, "lean") for q in qs[:8]] + items + [(q, "compact") for q in qs[-8:]]
    preps = [_prepare(e, ds, q, m) for q, m in items]
    want = [_alone(e, ds, p) for p in preps]
    e.set_flag("batch_finals", 2)
    e.set_flag("batch_lanes", lanes)
    e.set_flag("batch_fronts", fronts)
    try:
        before = e.get_flag("batch_overlaps")
        got = e.go_batch(preps, digests=True)
        overlaps = e.get_flag("batch_overlaps") - before
        plain = e.go_batch(preps[:12])
    finally:
        e.set_flag("batch_finals", 2)
        e.set_flag("batch_lanes", 4)
        e.set_flag("batch_fronts", 2)
    for (q, m), w, g in list(zip(items, want, got)) + list(zip(items[:12], want[:12], plain)):
        assert g[0] == w[0], (q, m, g, w)
        if g[0] == 0:
            assert (g[1], g[2]) == (w[1], w[2]), (q, m)
            if len(g) > 3 and "DISTINCT" not in q:
                assert tuple(g[3]) == tuple(w[3]), (q, m)
    assert overlaps >= 10
