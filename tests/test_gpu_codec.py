"""The reference's codec byte vectors through the product path: rows assembled byte by byte as in
RowReaderTest (src/dataman/test/RowReaderTest.cpp:14-151) are loaded as edge values with
reference-format keys (NebulaKeyUtils), exported to device columns by the library's RowReader
(exporter.cpp) and read back through ngx_get_neighbors, against the literal values of the test and
against the oracle. The device-encoded response rows (encode_rows, RowWriter format) must equal the
oracle's.
"""
import pytest

from nebula_amd import engine, kvfmt
from oracle import oracle
from tests import fixtures
from tests.test_codec_vectors import ENCODED_TYPES, ENCODED_VALUES, encoded_data_row

pytestmark = pytest.mark.gpu

NAMES = ["bool_col1", "str_col1", "int_col1", "int_col2", "vid_col", "str_col2", "bool_col2", "float_col",
         "double_col", "timestamp_col"]
FIELDS = list(zip(NAMES, ENCODED_TYPES))


def _dataset():
    b = kvfmt.KVBatch()
    # 1 -> 2: the encodedData row (schema version 0)
    b.put(kvfmt.edge_key(1, 1, 1, 0, 2), encoded_data_row())
    # 1 -> 3: headerInfo data2, a version-0xFF01 header with no field bytes (every read fails -> defaults)
    b.put(kvfmt.edge_key(1, 1, 1, 0, 3), b"\x40\x01\xff")
    # 1 -> 4: a version with no schema (bad row: skipped by the storage scan)
    b.put(kvfmt.edge_key(1, 1, 1, 0, 4), b"\x40\x02\xff")
    # 1 -> 5: empty value (no RowReader: only key props)
    b.put(kvfmt.edge_key(1, 1, 1, 0, 5), b"")
    schemas = [fixtures.SchemaDef(True, 1, "enc", FIELDS, 0), fixtures.SchemaDef(True, 1, "enc", FIELDS, 0xFF01)]
    return fixtures.Dataset(1, 1, schemas, b)


COLS = [(3, 1, "_dst")] + [(3, 1, n) for n in NAMES]


@pytest.fixture(scope="module")
def loaded():
    ds = _dataset()
    o = oracle.Oracle()
    ds.load_oracle(o)
    e = engine.Engine(0)
    ds.load_engine(e)
    yield o, e
    e.close()


def test_encoded_data_row_values(loaded):
    o, e = loaded
    got = e.get_neighbors(1, [(1, [1])], [1], COLS)
    ref = o.get_neighbors(1, [(1, [1])], [1], COLS)
    assert got.failed_codes == [] and ref.failed_codes == []
    assert got.total_edges == ref.total_edges
    by_dst = {int(got.edge_dst[i]): [v for _, v in got.edge_cells[i][1:]] for i in range(got.total_edges)}
    row = by_dst[2]
    assert row[:7] == ENCODED_VALUES[:7]
    assert row[7] == ENCODED_VALUES[7] and row[8] == ENCODED_VALUES[8] and row[9] == ENCODED_VALUES[9]
    # the no-data version-0xFF01 row reads every field as its type default
    assert by_dst[3] == [False, "", 0, 0, 0, "", False, 0.0, 0.0, 0]
    ref_rows = {}
    for v in ref.vertices:
        for ed in v["edges"]:
            for x in ed["edges"]:
                ref_rows[x["dst"]] = list(x["values"] or ())
    assert sorted(by_dst) == sorted(ref_rows)
    for d, vals in ref_rows.items():
        assert by_dst[d] == vals, d


def test_encoded_rows_match_oracle(loaded):
    o, e = loaded
    got = e.get_neighbors(1, [(1, [1])], [1], COLS, encode_rows=True)
    ref = o.get_neighbors(1, [(1, [1])], [1], COLS)
    raw = {}
    for v in ref.vertices:
        for ed in v["edges"]:
            for x in ed["edges"]:
                raw[x["dst"]] = x["raw"] or b""
    assert {int(got.edge_dst[i]): got.edge_props[i] for i in range(got.total_edges)} == raw
    assert got.edge_schema == {k: [tuple(c) for c in v] for k, v in ref.edge_schema.items()}
