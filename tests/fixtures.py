"""Test fixtures: reference-format datasets (schemas + KV rows) and loaders for the oracle and the
product. A `Dataset` is the same bytes for both sides."""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field
from typing import Dict, List, Tuple

from nebula_amd import kvfmt, ngql
from nebula_amd.kvfmt import BOOL, DOUBLE, FLOAT, INT, STRING, TIMESTAMP, VID

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@dataclass
class SchemaDef:
    is_edge: bool
    sid: int
    name: str
    fields: List[Tuple[str, int]]
    ver: int = 0
    ttl_col: str = ""
    ttl_dur: int = 0


@dataclass
class Dataset:
    space: int
    num_parts: int
    schemas: List[SchemaDef]
    batch: kvfmt.KVBatch
    extra_parts: List[int] = field(default_factory=list)   # parts outside 1..num_parts (test-only layouts)
    names: Dict[str, int] = field(default_factory=dict)

    def load_oracle(self, orc):
        orc.add_space(self.space, self.num_parts)
        for p in self.extra_parts:
            orc.add_part(self.space, p)
        for s in self.schemas:
            orc.add_schema(self.space, s.is_edge, s.sid, s.name, s.fields, s.ver, s.ttl_col, s.ttl_dur)
        orc.put_batch(self.space, self.batch)
        orc.finalize()
        return orc

    def load_engine(self, eng):
        eng.add_space(self.space, self.num_parts)
        for s in self.schemas:
            eng.add_schema(self.space, s.is_edge, s.sid, s.name, s.fields, s.ver, s.ttl_col, s.ttl_dur)
        eng.load_batch(self.space, self.batch)
        eng.commit(self.space)
        return eng


class GenDataset:
    """A generated space (datagen Rows + schemas) loadable into the oracle and the engine."""

    def __init__(self, space, num_parts, rows, schemas):
        self.space, self.num_parts, self.rows = space, num_parts, rows
        self.schemas = [SchemaDef(e, i, n, f) for e, i, n, f in schemas]

    def load_oracle(self, orc, threads=8):
        orc.add_space(self.space, self.num_parts)
        for s in self.schemas:
            orc.add_schema(self.space, s.is_edge, s.sid, s.name, s.fields, s.ver, s.ttl_col, s.ttl_dur)
        orc.put_kv(self.space, *self.rows.arrays())
        orc.finalize(threads)
        return orc

    def load_engine(self, eng):
        eng.add_space(self.space, self.num_parts)
        for s in self.schemas:
            eng.add_schema(self.space, s.is_edge, s.sid, s.name, s.fields, s.ver, s.ttl_col, s.ttl_dur)
        eng.load_kv(self.space, *self.rows.arrays())
        eng.commit(self.space)
        return eng


class RmatDataset(GenDataset):
    """RMAT space of bench.py (datagen.rmat): edge `e`(p0 INT, p1 INT), optional tag `vt`."""

    def __init__(self, scale, ef=16, seed=42, num_parts=100, with_in=False, with_tag=False, threads=0):
        from nebula_amd import datagen
        super().__init__(datagen.RMAT_SPACE, num_parts,
                         datagen.rmat(scale, ef, seed, num_parts, with_in, with_tag, threads=threads),
                         datagen.rmat_schemas(with_tag))
        self.scale = scale


def powerlaw_dataset(n, ef=8, nsuper=4, superdeg=20000, seed=42, num_parts=100, threads=0):
    """C4 shape: power-law graph with `nsuper` supernodes of in-degree `superdeg` (out + in rows)."""
    from nebula_amd import datagen
    rows = datagen.powerlaw(n, ef, 2.0, nsuper, superdeg, seed, num_parts, datagen.PL_EDGE, threads=threads)
    ds = GenDataset(datagen.PL_SPACE, num_parts, rows, datagen.powerlaw_schemas())
    ds.n = n
    return ds


def snb_dataset(np_, knows_deg=20, likes_deg=10, seed=42, num_parts=100, threads=0):
    """C5 shape: LDBC-SNB-like persons/posts with knows/likes/hasCreator (string + int props)."""
    from nebula_amd import datagen
    rows = datagen.snb(np_, knows_deg, 0, likes_deg, seed, num_parts, threads=threads)
    ds = GenDataset(datagen.SNB_SPACE, num_parts, rows, datagen.snb_schemas())
    ds.np = np_
    return ds


# ----------------------------------------------------------------------------- NBA (GoTest)
def nba() -> Dataset:
    """TraverseTestBase's NBA space: partition_num=1, player/team tags, serve/like/teammate edges.
    Every edge is written out (src, +type) and in (dst, -type) with the same row, as
    InsertEdgeExecutor does (src/graph/InsertEdgeExecutor.cpp:207-226)."""
    d = json.load(open(os.path.join(GOLDEN, "nba.json")))
    tags, edges = d["tag_ids"], d["edge_types"]
    schemas = [
        SchemaDef(False, tags["player"], "player", [("name", STRING), ("age", INT)]),
        SchemaDef(False, tags["team"], "team", [("name", STRING)]),
        SchemaDef(True, edges["serve"], "serve", [("start_year", INT), ("end_year", INT)]),
        SchemaDef(True, edges["like"], "like", [("likeness", INT)]),
        SchemaDef(True, edges["teammate"], "teammate", [("start_year", INT), ("end_year", INT)]),
        SchemaDef(False, tags["bachelor"], "bachelor", [("name", STRING), ("speciality", STRING)]),
    ]
    nparts = d["space_parts"]
    b = kvfmt.KVBatch()
    vid = ngql.nebula_hash

    def part(v):
        return (v % (1 << 64)) % nparts + 1

    for name, age in d["players"]:
        v = vid(name)
        b.put(kvfmt.vertex_key(part(v), v, tags["player"]), kvfmt.encode_row([STRING, INT], [name, age]))
    for name in d["teams"]:
        v = vid(name)
        b.put(kvfmt.vertex_key(part(v), v, tags["team"]), kvfmt.encode_row([STRING], [name]))

    def edge(etype, src, dst, rank, types, vals):
        row = kvfmt.encode_row(types, vals)
        b.put(kvfmt.edge_key(part(src), src, etype, rank, dst), row)
        b.put(kvfmt.edge_key(part(dst), dst, -etype, rank, src), row)

    for p, t, rank, s, e in d["serve"]:
        edge(edges["serve"], vid(p), vid(t), rank, [INT, INT], [s, e])
    for p, o, likeness in d["like"]:
        edge(edges["like"], vid(p), vid(o), 0, [INT], [likeness])
    for p, o, s, e in d["teammate"]:
        edge(edges["teammate"], vid(p), vid(o), 0, [INT, INT], [s, e])
    return Dataset(space=1, num_parts=nparts, schemas=schemas, batch=b)


def nba_query(q: str) -> str:
    """Replace {P:name} / {T:name} with vids."""
    import re
    return re.sub(r"\{[PT]:([^}]+)\}", lambda m: str(ngql.nebula_hash(m.group(1))), q)


def nba_expected(rows):
    out = []
    for r in rows:
        t = []
        for c in r:
            if isinstance(c, str) and c[:2] in ("P:", "T:"):
                t.append(ngql.nebula_hash(c[2:]))
            else:
                t.append(c)
        out.append(tuple(t))
    return sorted(out, key=repr)


def normalize_cells(rows):
    """ColumnValue -> comparable python values, as TestBase::convert does (ints from integer / id /
    timestamp / bool, strings, floats)."""
    out = []
    for r in rows:
        t = []
        for kind, v in r:
            if kind in ("int", "id", "timestamp"):
                t.append(int(v))
            elif kind == "bool":
                t.append(int(v))
            elif kind in ("float", "double"):
                t.append(float(v))
            elif kind == "str":
                t.append(v)
            else:
                t.append((kind, v))
        out.append(tuple(t))
    return sorted(out, key=repr)


# ----------------------------------------------------------------------------- QueryBoundTest
def querybound() -> Dataset:
    """mockData of src/storage/test/QueryBoundTest.cpp:24-95 with mockSchemaMan
    (src/storage/test/TestUtils.h:105-114): parts 0..2, vids partId*10..+9, tags 3001-3009
    (3 int + 3 string), edges 101-109 (10 int + 10 string), 7 out-edges and 5 in-edges per type,
    3 versions per edge, rows written without a schema (RowWriter(nullptr))."""
    schemas = []
    for tag in range(3001, 3010):
        f = [(f"tag_{tag}_col_{i}", INT) for i in range(3)] + [(f"tag_{tag}_col_{i}", STRING) for i in range(3, 6)]
        schemas.append(SchemaDef(False, tag, str(tag), f))
    for et in range(101, 110):
        f = [(f"col_{i}", INT) for i in range(10)] + [(f"col_{i}", STRING) for i in range(10, 20)]
        schemas.append(SchemaDef(True, et, str(et), f))
    b = kvfmt.KVBatch()
    int_max = 2**31 - 1
    for part in range(3):
        for vid in range(part * 10, (part + 1) * 10):
            for tag in range(3001, 3010):
                w = kvfmt.RowWriter(None)
                for i in range(3):
                    w.int(vid + tag + i)
                for i in range(3, 6):
                    w.string(f"tag_string_col_{i}")
                b.put(kvfmt.vertex_key(part, vid, tag, 0), w.encode())
            for dst in range(10001, 10008):
                for version in range(3):
                    for et in range(101, 110):
                        w = kvfmt.RowWriter(None)
                        for i in range(10):
                            w.int(int_max if version == 1 else dst + i)
                        for i in range(10, 20):
                            w.string(f"string_col_{i}_{version}")
                        b.put(kvfmt.edge_key(part, vid, et, 0, dst, int_max - version), w.encode())
            for src in range(20001, 20006):
                for version in range(3):
                    for et in range(101, 110):
                        w = kvfmt.RowWriter(None)
                        for i in range(10):
                            w.int(src + i)
                        for i in range(10, 20):
                            w.string(f"string_col_{i}_{version}")
                        b.put(kvfmt.edge_key(part, vid, -et, 0, src, int_max - version), w.encode())
    return Dataset(space=0, num_parts=0, schemas=schemas, batch=b, extra_parts=[0, 1, 2])


def querybound_request(edge_types):
    """buildRequest (QueryBoundTest.cpp:97-127): all 30 vids by part, tag cols, _dst/_rank, col_0..col_18 even."""
    parts = [(p, list(range(p * 10, (p + 1) * 10))) for p in range(3)]
    cols = []
    for i in range(3):
        cols.append((1, 3001 + i * 2, f"tag_{3001 + i * 2}_col_{i * 2}"))
    for e in edge_types:
        cols.append((3, e, "_dst"))
        cols.append((3, e, "_rank"))
    for i in range(10):
        for e in edge_types:
            cols.append((3, e, f"col_{i * 2}"))
    return parts, cols
