"""Oracle pin: the restated QueryBoundProcessor against the reference QueryBoundTest expectations
(src/storage/test/QueryBoundTest.cpp:129-206 checkResponse, :296-720 cases)."""
import pytest

from nebula_amd import ngql
from oracle import oracle
from tests import fixtures

E_INVALID_FILTER = -31


@pytest.fixture(scope="module")
def qb():
    ds = fixtures.querybound()
    o = oracle.Oracle()
    ds.load_oracle(o)
    return o


def check_response(resp, vertex_num, edge_fields, dst_from, edge_num):
    """checkResponse (QueryBoundTest.cpp:129-206)."""
    assert resp.failed_codes == []
    assert len(resp.vertices) == vertex_num
    total = 0
    for v in resp.vertices:
        vid = v["vid"]
        size = sum(len(resp.vertex_schema[t["tag_id"]]) for t in v["tags"])
        assert size == 3
        tags = {t["tag_id"]: t for t in v["tags"]}

        def tagval(tag, name):
            cols = [c[0] for c in resp.vertex_schema[tag]]
            return tags[tag]["values"][cols.index(name)]

        assert tagval(3001, "tag_3001_col_0") == vid + 3001
        assert tagval(3003, "tag_3003_col_2") == vid + 3003 + 2
        assert tagval(3005, "tag_3005_col_4") == "tag_string_col_4"
        for ed in v["edges"]:
            assert ed["type"] in resp.edge_schema
            row_num = 0
            for e in ed["edges"]:
                dst = e["dst"]
                assert dst == dst_from + row_num
                vals = e["values"]
                assert len(vals) + 1 == edge_fields
                assert vals[0] == 0                                   # _rank
                for i in range(1, 6):
                    assert vals[i] == (i - 1) * 2 + dst              # col_0, col_2 ... col_8
                for i in range(6, 11):
                    assert vals[i] == f"string_col_{(i - 6 + 5) * 2}_2"   # latest version wins
                row_num += 1
            assert row_num == edge_num
            total += row_num
    assert total == resp.total_edges


def alias_rel(alias, prop, op, value):
    """`<alias>.<prop> <op> value` for the test's numeric edge names (AdHocSchemaManager "101" <-> 101)."""
    return ngql.Binary(ngql.K_REL, ngql.REL_OPS[op], ngql.Prop(ngql.K_ALIAS, "", alias, prop), ngql.Prim(value))


def run(o, et, filt=b"", cols=None, max_edges=2**31 - 1):
    parts, default_cols = fixtures.querybound_request(et)
    o.set_flags(max_edges=max_edges)
    r = o.get_neighbors(0, parts, et, cols if cols is not None else default_cols, filt)
    o.set_flags()
    return r


def test_out_bound_simple(qb):
    check_response(run(qb, [101]), 30, 12, 10001, 7)


def test_in_bound_simple(qb):
    check_response(run(qb, [-101]), 30, 12, 20001, 5)


def test_only_edge_filter(qb):
    f = alias_rel("101", "col_0", ">=", 10007).encode()
    check_response(run(qb, [101], f), 30, 12, 10007, 1)
    f2 = alias_rel("101", "col_10", "==", "string_col_10_1").encode()
    r = run(qb, [101], f2, cols=[(3, 101, "col_10")])
    assert r.failed_codes == [] and r.vertices == []


def test_only_tag_filter(qb):
    f = ngql.Binary(ngql.K_REL, ngql.REL_OPS[">="], ngql.Prop(ngql.K_SRC_PROP, "$^", "3001", "tag_3001_col_0"),
                    ngql.Prim(20 + 3001)).encode()
    check_response(run(qb, [101], f), 10, 12, 10001, 7)


def test_tag_and_edge_filter(qb):
    left = ngql.Binary(ngql.K_REL, ngql.REL_OPS[">="], ngql.Prop(ngql.K_SRC_PROP, "$^", "3001", "tag_3001_col_0"),
                       ngql.Prim(20 + 3001))
    f = ngql.Binary(ngql.K_LOGIC, 0, left, alias_rel("101", "col_0", ">=", 10007)).encode()
    check_response(run(qb, [101], f), 10, 12, 10007, 1)


def test_invalid_filter(qb):
    f = ngql.Prop(ngql.K_INPUT_PROP, "$-", "", "tag_3001_col_0").encode()
    r = run(qb, [101], f)
    assert len(r.failed_codes) == 3
    assert all(c == E_INVALID_FILTER for c, _ in r.failed_codes)


def test_multi_edge_query(qb):
    check_response(run(qb, [101, 102, 103]), 30, 12, 10001, 7)


def test_max_edges_returned(qb):
    check_response(run(qb, [101], max_edges=5), 30, 12, 10001, 5)


def test_gen_buckets():
    # QueryBoundTest.cpp:445-499 (30 vertices)
    assert oracle.gen_buckets(30, 3, 10) == [3] * 10
    assert oracle.gen_buckets(30, 3, 9) == [4, 4, 4] + [3] * 6
    assert oracle.gen_buckets(30, 4, 40) == [5, 5] + [4] * 5
    assert oracle.gen_buckets(30, 40, 40) == [30]


def test_ttl():
    """TTLTest (QueryBoundTest.cpp:695-720) with mockSchemaWithTTLMan (TestUtils.h:116-125)."""
    ds = fixtures.querybound()
    ds.schemas = [s for s in ds.schemas if (s.is_edge and s.sid == 101) or (not s.is_edge and s.sid == 3001)]
    for s in ds.schemas:
        if s.is_edge:
            s.ttl_col, s.ttl_dur = "col_0", 200
    o = oracle.Oracle()
    ds.load_oracle(o)
    o.set_flags(now_sec=1_700_000_000)
    parts, _ = fixtures.querybound_request([101])
    r = o.get_neighbors(0, parts, [101], [(3, 101, "col_10")])
    assert r.failed_codes == [] and r.vertices == []
