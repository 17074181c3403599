"""GPU parity of the QueryResponse payload: the RowWriter rows the device encodes for
GetNeighbors (IdAndProp.props per edge, TagData.data per vertex tag) and the response schemas, byte
for byte against the oracle's restated QueryBoundProcessor (src/storage/query/QueryBoundProcessor.cpp
:18-261, RowWriter src/dataman/RowWriter.cpp:48-263).

Cases: the QueryBoundTest request (QueryBoundTest.cpp:97-127), a wide request (>= 16 response columns:
block offsets), and a typed space whose rows cover every field type, old schema versions (missing
fields -> defaults), empty values (no RowReader: props not collected, Skip padding, key props landing
in earlier fields) and columns of several edge types.
"""
import pytest

from nebula_amd import engine, kvfmt
from nebula_amd.kvfmt import BOOL, DOUBLE, FLOAT, INT, STRING, TIMESTAMP, VID
from oracle import oracle
from tests import fixtures

pytestmark = pytest.mark.gpu


def _oracle_payload(resp, parts):
    vids = [x for _, vs in parts for x in vs]
    edges = sorted((v["vid"], ed["type"], x["dst"], x["raw"] or b"")
                   for v in resp.vertices for ed in v["edges"] for x in ed["edges"])
    tags = sorted((v["vid"], t["tag_id"], t["raw"]) for v in resp.vertices for t in v["tags"])
    return edges, tags, set(v["vid"] for v in resp.vertices)


def _engine_payload(res, parts, with_edges):
    vids = [x for _, vs in parts for x in vs]
    edges = sorted((vids[int(res.edge_vertex[i])], int(res.edge_type[i]), int(res.edge_dst[i]), res.edge_props[i])
                   for i in range(res.total_edges))
    # the processor answers only vertices that kept an edge (QueryBoundProcessor.cpp:219-231)
    tags = sorted((vids[vi], t, raw) for vi, t, raw in res.tag_rows if vids[vi] in with_edges)
    return edges, tags


def _compare(o, e, space, parts, et, cols, filt=b""):
    ref = o.get_neighbors(space, parts, et, cols, filt)
    got = e.get_neighbors(space, parts, et, cols, filt, encode_rows=True)
    assert sorted(got.failed_codes) == sorted(ref.failed_codes)
    ref_edges, ref_tags, with_edges = _oracle_payload(ref, parts)
    got_edges, got_tags = _engine_payload(got, parts, with_edges)
    assert len(got_edges) == len(ref_edges) > 0
    assert got_edges == ref_edges
    assert got_tags == ref_tags
    assert got.edge_schema == {k: [tuple(c) for c in v] for k, v in ref.edge_schema.items()}
    assert got.vertex_schema == {k: [tuple(c) for c in v] for k, v in ref.vertex_schema.items()}
    return got


@pytest.fixture(scope="module")
def qb():
    ds = fixtures.querybound()
    o = oracle.Oracle()
    ds.load_oracle(o)
    e = engine.Engine(0)
    e.set_flag("jit", 0)
    ds.load_engine(e)
    yield o, e
    e.close()


@pytest.mark.parametrize("et", [[101], [-101], [101, 102, 103], [-102, 103]])
def test_querybound_rows(qb, et):
    parts, cols = fixtures.querybound_request(et)
    _compare(*qb, 0, parts, et, cols)


def test_querybound_wide_rows(qb):
    """20 props + _src/_rank/_type: 22 response columns, one block offset per row."""
    parts, _ = fixtures.querybound_request([101])
    cols = [(1, 3001, f"tag_3001_col_{i}") for i in range(6)] + [(3, 101, "_src"), (3, 101, "_dst")]
    cols += [(3, 101, f"col_{i}") for i in range(20)] + [(3, 101, "_rank"), (3, 101, "_type")]
    r = _compare(*qb, 0, parts, [101], cols)
    assert all(len(p) > 0 for p in r.edge_props)


def test_querybound_only_structure(qb):
    """Only `_dst` of a type: no edge schema, IdAndProp.props unset (empty)."""
    parts, _ = fixtures.querybound_request([101])
    cols = [(3, 101, "_dst"), (3, 102, "_dst"), (3, 102, "col_1")]
    r = _compare(*qb, 0, parts, [101, 102], cols)
    assert 101 not in r.edge_schema and 102 in r.edge_schema


# ----------------------------------------------------------------------------- every field type
TYPED_V0 = [("i", INT), ("s", STRING)]
TYPED_V1 = TYPED_V0 + [("f", FLOAT), ("d", DOUBLE), ("b", BOOL), ("ts", TIMESTAMP), ("v", VID)]
TAG = [("name", STRING), ("ok", BOOL), ("w", FLOAT), ("n", INT)]


def _typed():
    """Space 7, 3 parts: tag 11, edges 21 / 22 (two schema versions each); edge rows of version 0 and
    1, a few empty values, negative and large ints, float/double extremes."""
    schemas = [fixtures.SchemaDef(False, 11, "t", TAG)]
    for et in (21, 22):
        schemas.append(fixtures.SchemaDef(True, et, f"e{et}", TYPED_V0, 0))
        schemas.append(fixtures.SchemaDef(True, et, f"e{et}", TYPED_V1, 1))
    b = kvfmt.KVBatch()
    nparts = 3
    vids = list(range(1, 31))
    for v in vids:
        part = v % nparts + 1
        if v % 4:
            b.put(kvfmt.vertex_key(part, v, 11), kvfmt.encode_row([t for _, t in TAG],
                                                                  [f"v{v}" * (v % 3), v % 2 == 0, v / 7.0, -v * 1000003]))
        for k in range(6):
            dst = (v * 7 + k * 13) % 40 + 1
            for et in (21, 22):
                rank = (k - 2) * 1_000_000_007
                key = kvfmt.edge_key(part, v, et, rank, dst)
                if (v + k) % 5 == 0:
                    val = b""                                               # empty value: no RowReader
                elif (v + k + et) % 3 == 0:
                    val = kvfmt.encode_row([t for _, t in TYPED_V0], [v * k - 50, "x" * k], ver=0)
                else:
                    val = kvfmt.encode_row([t for _, t in TYPED_V1],
                                           [-(v << 40) + k, f"s{v}_{k}", 1.5 / (k + 1), -2.0 ** (v % 60) / 3,
                                            (v + k) % 2 == 1, 1_600_000_000 + v * k, v * 1000 + k], ver=1)
                b.put(key, val)
                b.put(kvfmt.edge_key(dst % nparts + 1, dst, -et, rank, v), val)
    return fixtures.Dataset(7, nparts, schemas, b)


@pytest.fixture(scope="module")
def typed():
    ds = _typed()
    o = oracle.Oracle()
    ds.load_oracle(o)
    e = engine.Engine(0)
    e.set_flag("jit", 0)
    ds.load_engine(e)
    parts = {}
    for v in range(1, 41):
        parts.setdefault(v % 3 + 1, []).append(v)
    yield o, e, sorted(parts.items())
    e.close()


TYPED_COLS = [
    # key props after value props: with an empty value they land in the earlier fields
    [(3, 21, "i"), (3, 21, "_rank"), (3, 21, "s"), (3, 21, "f"), (3, 21, "_type"), (3, 21, "d"), (3, 21, "b"),
     (3, 21, "ts"), (3, 21, "v"), (3, 21, "_src"), (3, 21, "_dst")],
    [(1, 11, "name"), (1, 11, "ok"), (1, 11, "w"), (1, 11, "n"), (3, 21, "_dst"), (3, 21, "s"), (3, 22, "_dst"),
     (3, 22, "d"), (3, 22, "_rank"), (3, 22, "ts")],
    [(3, -21, "_src"), (3, -21, "f"), (3, -21, "v"), (3, 22, "b"), (3, 22, "i")],
]


@pytest.mark.parametrize("ci", range(len(TYPED_COLS)))
def test_typed_rows(typed, ci):
    o, e, parts = typed
    cols = TYPED_COLS[ci]
    et = sorted(set(c[1] for c in cols if c[0] == 3))
    _compare(o, e, 7, parts, et, cols)
