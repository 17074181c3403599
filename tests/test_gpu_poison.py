"""Every word a kernel reads was written by a kernel of the same query.

The engine flag poison_buffers fills every device scratch buffer allocated from then on with 0xA5
bytes (engine.cpp DBuf). Without it a fresh process's allocations are often zero and later ones hold
an earlier query's values, which can hide a kernel reading a word nothing wrote: the wire-row encoder
(k_encode_rows) did fault once on exactly that. With the poison:

* the GetNeighbors wire rows (encode_rows, RowWriter format) of the RowReaderTest codec dataset equal
  the oracle's, on the generated and on the interpreter kernels; before the encoder runs the library
  checks on the host that every type, flag and cell word it will read holds a written value;
* GO queries (multi-hop, pull and push hops, M TO N, DISTINCT, result_on_device with compact
  results, GetNeighbors over the RMAT graph) on a fresh engine equal the oracle.

The flag is process-wide; each test turns it off again before it ends.
"""
import pytest

from nebula_amd import datagen, engine, ngql
from oracle import oracle
from tests import fixtures
from tests.test_gpu_codec import COLS, _dataset
from tests.test_gpu_response import TYPED_COLS, _compare, _typed

pytestmark = pytest.mark.gpu


class _Poisoned:
    def __init__(self, **flags):
        self.flags = flags

    def __enter__(self):
        self.e = engine.Engine(0)
        self.e.set_flag("poison_buffers", 1)
        for k, v in self.flags.items():
            self.e.set_flag(k, v)
        return self.e

    def __exit__(self, *exc):
        try:
            self.e.set_flag("poison_buffers", 0)
        finally:
            self.e.close()


def _raw_rows(ref):
    raw = {}
    for v in ref.vertices:
        for ed in v["edges"]:
            for x in ed["edges"]:
                raw[x["dst"]] = x["raw"] or b""
    return raw


@pytest.mark.parametrize("jit", [1, 0])
def test_encoded_rows_with_poisoned_scratch(jit):
    ds = _dataset()
    o = oracle.Oracle()
    ds.load_oracle(o)
    ref = o.get_neighbors(1, [(1, [1])], [1], COLS)
    with _Poisoned(jit=jit) as e:
        assert e.get_flag("poison_buffers") == 1
        ds.load_engine(e)
        for _ in range(2):                       # fresh buffers, then the same buffers reused
            got = e.get_neighbors(1, [(1, [1])], [1], COLS, encode_rows=True)
            assert got.failed_codes == []
            assert {int(got.edge_dst[i]): got.edge_props[i] for i in range(got.total_edges)} == _raw_rows(ref)
            assert got.edge_schema == {k: [tuple(c) for c in v] for k, v in ref.edge_schema.items()}
    o.close()


POISON_GO = [
    "GO 3 STEPS FROM {S} OVER e WHERE e.p0 < 50 YIELD e._dst, e._rank, e.p0, e.p1",
    "GO 2 STEPS FROM {S} OVER e YIELD e._src, e._dst, e._type",
    "GO 1 TO 3 STEPS FROM {S} OVER e WHERE e.p0 % 7 == 3 YIELD e._dst, e.p0",
    "GO 2 STEPS FROM {S} OVER e BIDIRECT WHERE e.p0 > 90 YIELD e._dst, e.p0 * 2 + 1",
    "GO 2 STEPS FROM {S} OVER e WHERE $^.vt.v0 > 100 && e.p0 % 3 == 0 YIELD $^.vt.name, $$.vt.v0, e.p0 + e.p1",
    "GO 3 STEPS FROM {S} OVER e YIELD DISTINCT e._dst",
]


@pytest.fixture(scope="module")
def rmat_ref():
    ds = fixtures.RmatDataset(12, with_in=True, with_tag=True)
    o = oracle.Oracle()
    o.set_flags(threads=8)
    ds.load_oracle(o)
    yield ds, o
    o.close()


@pytest.mark.parametrize("jit", [1, 0])
def test_go_with_poisoned_scratch(rmat_ref, jit):
    ds, o = rmat_ref
    with _Poisoned(jit=jit) as e:
        ds.load_engine(e)
        for qi, text in enumerate(POISON_GO):
            seeds = datagen.sample_vids(500 + qi, 1 << ds.scale, 40)
            s = ngql.parse_go(text.replace("{S}", ", ".join(str(int(v)) for v in seeds)))
            for pull in (0, 1):                 # default direction choice, then every eligible hop pulled
                e.set_flag("pull_factor", 200 if pull == 0 else 1)
                ref = o.go(ds.space, s)
                got = e.go(ds.space, s)
                assert got.ok == ref.ok, (text, got.error, ref.error)
                assert fixtures.normalize_cells(got.rows) == fixtures.normalize_cells(ref.rows), text
                assert got.hop_edges[:len(ref.hop_scanned)] == ref.hop_scanned[:len(got.hop_edges)]
        # device-resident compact results: the row count and the rows' key arrays, widened
        seeds = datagen.sample_vids(77, 1 << ds.scale, 40)
        s = ngql.parse_go(POISON_GO[0].replace("{S}", ", ".join(str(int(v)) for v in seeds)))
        host = e.go(ds.space, s)
        dev = e.go(ds.space, s, on_device=True)
        assert dev.ok and dev.nrows == len(host.rows) and dev.hop_edges == host.hop_edges


@pytest.mark.parametrize("jit", [1, 0])
def test_response_payloads_with_poisoned_scratch(jit):
    """The QueryResponse payload cases of test_gpu_response (every field type, two schema versions,
    empty values, several edge types, tag rows, >= 16 columns) on a poisoned engine, each request twice."""
    ds = _typed()
    o = oracle.Oracle()
    ds.load_oracle(o)
    parts = {}
    for v in range(1, 41):
        parts.setdefault(v % 3 + 1, []).append(v)
    parts = sorted(parts.items())
    with _Poisoned(jit=jit) as e:
        ds.load_engine(e)
        for cols in TYPED_COLS:
            et = sorted(set(c[1] for c in cols if c[0] == 3))
            for _ in range(2):
                _compare(o, e, 7, parts, et, cols)
    o.close()
    qds = fixtures.querybound()
    qo = oracle.Oracle()
    qds.load_oracle(qo)
    with _Poisoned(jit=jit) as e:
        qds.load_engine(e)
        qparts, _ = fixtures.querybound_request([101])
        cols = [(1, 3001, f"tag_3001_col_{i}") for i in range(6)] + [(3, 101, "_src"), (3, 101, "_dst")]
        cols += [(3, 101, f"col_{i}") for i in range(20)] + [(3, 101, "_rank"), (3, 101, "_type")]
        _compare(qo, e, 0, qparts, [101], cols)
        for et in ([101], [-101], [101, 102, 103], [-102, 103]):
            p2, c2 = fixtures.querybound_request(et)
            _compare(qo, e, 0, p2, et, c2)
    qo.close()
