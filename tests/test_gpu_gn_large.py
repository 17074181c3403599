"""A GetNeighbors response large enough that the library types its cells on several host threads
(per-thread string arenas rebased into one strings block): 2000 vertices x 40 out-edges with a
string and an int prop, every vertex requested, against the oracle's QueryBoundProcessor."""
import random

import pytest

from nebula_amd import engine, kvfmt, ngql
from oracle import oracle
from tests import fixtures

pytestmark = pytest.mark.gpu


def _space():
    rnd = random.Random(11)
    b = kvfmt.KVBatch()
    nparts = 7
    for v in range(2000):
        for j in range(40):
            dst = rnd.randrange(2000)
            s = "s%d-%s" % (v, "x" * rnd.randrange(0, 30))
            row = kvfmt.encode_row([kvfmt.STRING, kvfmt.INT], [s, v * 100 + j])
            b.put(kvfmt.edge_key(v % nparts + 1, v, 5, j, dst), row)
    return fixtures.Dataset(4, nparts, [fixtures.SchemaDef(True, 5, "big", [("s", kvfmt.STRING), ("i", kvfmt.INT)])], b)


def test_large_response_cells():
    ds = _space()
    o = oracle.Oracle()
    ds.load_oracle(o)
    parts = {}
    for v in range(2000):
        parts.setdefault(v % 7 + 1, []).append(v)
    parts = sorted(parts.items())
    cols = [(engine.EDGE, 5, "_dst"), (engine.EDGE, 5, "s"), (engine.EDGE, 5, "i")]
    filt = ngql.Binary(ngql.K_REL, ngql.REL_OPS[">"], ngql.Prop(ngql.K_ALIAS, "", "big", "i"), ngql.Prim(1000)).encode()
    with engine.Engine(0) as e:
        ds.load_engine(e)
        for f in (b"", filt):
            got = e.get_neighbors(4, parts, [5], cols, f)
            ref = o.get_neighbors(4, parts, [5], cols, f)
            assert got.failed_codes == ref.failed_codes == []
            assert got.total_edges == ref.total_edges > 60000
            vids = [x for _, vs in parts for x in vs]
            mine = sorted((vids[int(got.edge_vertex[i])], int(got.edge_dst[i]), got.edge_cells[i][1][1], got.edge_cells[i][2][1])
                          for i in range(got.total_edges))
            theirs = sorted((v["vid"], x["dst"], x["values"][0], x["values"][1])
                            for v in ref.vertices for ed in v["edges"] for x in ed["edges"])
            assert mine == theirs
