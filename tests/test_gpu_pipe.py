"""Pipes and variables on the device path (ngx_go with input_*: GoExecutor fromType_ kPipe /
kVariable, src/graph/GoExecutor.cpp:471-509, :675-718, :1317-1330): the reference GoTest answers on
the NBA fixture (JIT and interpreter kernels, pushdown on and off), then RMAT pipes against the
oracle's back-tracker restatement — one walk from all vids (1 step, no `$-' reads), one walk per
vid (multi-step), one walk per input row (`$-' in WHERE / YIELD), DISTINCT over the union, and the
errors of setupStarts."""
import pytest

from nebula_amd import datagen, engine, ngql, pipeline
from oracle import oracle
from tests import fixtures
from tests.golden.gotest_cases import PIPE_CASES
from tests.test_oracle_pipe import check

pytestmark = pytest.mark.gpu
EDGES = ["serve", "like", "teammate"]


@pytest.fixture(scope="module", params=["jit", "vm"])
def nba(request):
    ds = fixtures.nba()
    e = engine.Engine(0)
    e.set_flag("jit", 1 if request.param == "jit" else 0)
    ds.load_engine(e)
    yield ds, e
    e.close()


@pytest.mark.parametrize("pushdown", [True, False])
@pytest.mark.parametrize("case", PIPE_CASES, ids=[f"L{c['line']}" for c in PIPE_CASES])
def test_pipe_known_answers_device(nba, case, pushdown):
    ds, e = nba
    out = pipeline.run(e, ds.space, fixtures.nba_query(case["query"]), EDGES, pushdown=pushdown)
    check(out, case)


@pytest.fixture(scope="module")
def rmat():
    ds = fixtures.RmatDataset(11, with_in=True, with_tag=True)
    o = oracle.Oracle()
    o.set_flags(threads=8)
    ds.load_oracle(o)
    e = engine.Engine(0)
    ds.load_engine(e)
    yield ds, o, e
    e.close()


RMAT_PIPES = [
    # one walk from all distinct vids (1 step, no input reads); duplicate vids repeat rows
    "GO 2 STEPS FROM {S} OVER e YIELD e._dst AS id | GO FROM $-.id OVER e YIELD e._dst, e.p0",
    "GO FROM {S} OVER e YIELD e._dst AS id | GO FROM $-.id OVER e REVERSELY WHERE e.p1 > 300000 YIELD e._src, e.p1",
    # one walk per vid (multi-step, M TO N)
    "GO FROM {S} OVER e YIELD e._dst AS id | GO 2 STEPS FROM $-.id OVER e YIELD e._dst, e.p1 % 5",
    "GO FROM {S} OVER e YIELD e._dst AS id | GO 1 TO 3 STEPS FROM $-.id OVER e WHERE e.p0 < 20 YIELD e._dst",
    # one walk per input row: $- in WHERE and YIELD (ints, strings, doubles, bools)
    "GO FROM {S} OVER e YIELD e._dst AS id, e.p0 AS w, $$.vt.name AS nm | "
    "GO FROM $-.id OVER e WHERE e.p0 > $-.w YIELD $-.w, $-.nm, e.p0 - $-.w, $$.vt.v0",
    "GO FROM {S} OVER e YIELD e._dst AS id, e.p0 * 0.5 AS h, e.p1 > 500000 AS big | "
    "GO 2 STEPS FROM $-.id OVER e WHERE $-.big || e.p0 < 10 YIELD $-.h + e.p0, $-.big, e._dst",
    "GO FROM {S} OVER e YIELD e._src AS s, e._dst AS d | GO FROM $-.d OVER e BIDIRECT YIELD $-.s, $-.d, e._dst",
    # DISTINCT over the union of walks
    "GO FROM {S} OVER e YIELD e._dst AS id, e.p0 % 3 AS k | GO FROM $-.id OVER e YIELD DISTINCT $-.k, e.p1 % 4",
    "GO FROM {S} OVER e YIELD e._dst AS id | GO 2 STEPS FROM $-.id OVER e YIELD DISTINCT e._dst",
    # variables
    "$v = GO FROM {S} OVER e YIELD e._dst AS id, e.p0 AS w; GO FROM $v.id OVER e WHERE e.p0 < $v.w YIELD $v.*, e.p0",
    # a bool of an UNKNOWN-typed column: unset in the response, kept in the interim result and as a
    # DISTINCT key (true and false rows stay apart)
    "GO FROM {S} OVER e YIELD e._dst AS id, !(e.p0 > 50) AS b | GO FROM $-.id OVER e WHERE $-.b YIELD DISTINCT $-.b, e.p1 % 3",
    "GO FROM {S} OVER e YIELD e._dst AS id | GO 2 STEPS FROM $-.id OVER e YIELD DISTINCT !(e.p0 > 50), e.p1 % 2",
]


@pytest.mark.parametrize("qi", range(len(RMAT_PIPES)))
def test_rmat_pipes_vs_oracle(rmat, qi):
    ds, o, e = rmat
    seeds = datagen.sample_vids(900 + qi, 1 << ds.scale, 6)
    q = RMAT_PIPES[qi].replace("{S}", ", ".join(str(int(v)) for v in seeds))
    ref = pipeline.run(o, ds.space, q)
    got = pipeline.run(e, ds.space, q)
    assert ref.ok and got.ok, (got.error, ref.error)
    assert got.names == ref.names
    assert len(got.rows) == len(ref.rows) > 0
    assert sorted(fixtures.normalize_cells(got.rows), key=repr) == sorted(fixtures.normalize_cells(ref.rows), key=repr)
    if "DISTINCT" in q:
        assert len(set(map(tuple, fixtures.normalize_cells(got.rows)))) == len(got.rows)


def test_pipe_errors_match_oracle(rmat):
    ds, o, e = rmat
    inp = pipeline.Interim(["id", "id"], [pipeline.T_VID, pipeline.T_INT], [(("id", 1), ("int", 2))])
    cases = [
        ("GO FROM $-.id OVER e", inp),                                               # Duplicate column
        ("GO FROM $-.nope OVER e", pipeline.Interim(["id"], [3], [(("id", 1),)])),   # Column not found
        ("GO FROM $-.s OVER e", pipeline.Interim(["s"], [6], [(("str", "x"),)])),    # not a VID / INT column
        ("GO FROM $-.* OVER e", pipeline.Interim(["id"], [3], [(("id", 1),)])),
        ("GO FROM 1 OVER e YIELD $-.id", None),
        ("GO FROM $-.id OVER e YIELD $v.id", pipeline.Interim(["id"], [3], [(("id", 1),)])),
        ("GO FROM $-.id OVER e YIELD $-.zz", pipeline.Interim(["id"], [3], [(("id", 5),)])),
    ]
    for q, i in cases:
        s = ngql.parse_go(q)
        ref = o.go(ds.space, s, input=i)
        got = e.go(ds.space, s, input=i)
        assert not ref.ok and not got.ok, q
        assert got.error == ref.error, q


def test_pipe_empty_input_keeps_types(rmat):
    ds, o, e = rmat
    s = ngql.parse_go("GO FROM $-.id OVER e YIELD $-.id, e.p0")
    got = e.go(ds.space, s, input=pipeline.Interim(["id"]))
    ref = o.go(ds.space, s, input=pipeline.Interim(["id"]))
    assert got.ok and ref.ok and got.rows == ref.rows == []
    # no data: `$-.id' is UNKNOWN (calculateExprType, TraverseExecutor.cpp:150-158); the reference's
    # onEmptyInputs response carries no rows, so the oracle reports no types at all
    assert got.col_types == [0, 2]


@pytest.mark.parametrize("q", [
    "GO 2 STEPS FROM $-.id OVER e WHERE e.p0 < 3 YIELD e._dst, e.p1 % 5",
    "GO 1 TO 3 STEPS FROM $-.id OVER e REVERSELY WHERE e.p0 < 2 YIELD e._dst, e._src",
    "GO 3 STEPS FROM $-.id OVER e BIDIRECT YIELD DISTINCT e._dst",
    # reading the input: (frontier row, input row) entries, $-.x from the device input table
    "GO 2 STEPS FROM $-.id OVER e WHERE e.p0 < $-.w / 20 YIELD $-.w, $-.nm, e._dst, e.p0 + $-.w",
    "GO FROM $-.id OVER e WHERE $-.w > 90 || e.p0 == 3 YIELD DISTINCT $-.nm, e.p0 % 4",
    "GO 1 TO 2 STEPS FROM $-.id OVER e REVERSELY WHERE e.p0 < 2 YIELD upper($-.nm) + \"/\" + (string)$-.w, e._dst",
])
def test_multi_root_walk_in_batches(rmat, q):
    """A sentence from an input walks from 64 distinct input vids at a time (root sets over the frontier
    rows, GoExecutor's back tracker as bitmasks), not once per vid or per input row: the input here has
    179 distinct vids (3 walks), 234 rows and duplicates; the rows equal the oracle's back-tracker result.
    Sentences that read $-.x evaluate it per (frontier row, input row) entry on the device."""
    ds, o, e = rmat
    seeds = ", ".join(str(int(v)) for v in datagen.sample_vids(4242, 1 << ds.scale, 20))
    first = f"GO FROM {seeds} OVER e YIELD e._dst AS id, e.p0 AS w, $$.vt.name AS nm"
    full = f"{first} | {q}"
    ids = {r[0][1] for r in pipeline.run(o, ds.space, first).rows}
    assert len(ids) > 128
    before = e.get_flag("pipe_walks")
    ref = pipeline.run(o, ds.space, full)
    got = pipeline.run(e, ds.space, full)
    walks = e.get_flag("pipe_walks") - before
    assert ref.ok and got.ok, (got.error, ref.error)
    assert sorted(fixtures.normalize_cells(got.rows), key=repr) == sorted(fixtures.normalize_cells(ref.rows), key=repr)
    assert len(got.rows) > 0
    assert walks == (len(ids) + 63) // 64
