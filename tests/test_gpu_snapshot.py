"""Shard ingest and restart on the device:

* ngx_load_snapshot_rows: the NBA space fed as per-part raft snapshot streams — encodeKV records
  (src/kvstore/LogEncoder.cpp:16-27) of prefix(part) in key order, as
  SnapshotManagerImpl::accessAllRowsInSnapshot produces them (src/kvstore/SnapshotManagerImpl.cpp:15-53),
  cut into batches at arbitrary record boundaries, with system commit / part keys
  (NebulaKeyUtils.cpp:48-67) mixed in as a whole-space stream would carry — answers the GoTest
  queries exactly as the oracle does;
* ngx_save_snapshot / ngx_open_snapshot: a committed shard written to a file and opened in a fresh
  context answers every query exactly as the original (RMAT with tag props, SNB with strings), and a
  damaged, truncated, foreign-space or foreign-schema file is refused without touching the space.
"""
import os
import struct

import pytest

from nebula_amd import datagen, engine, kvfmt, ngql
from oracle import oracle
from tests import fixtures
from tests.golden.gotest_cases import CASES

pytestmark = pytest.mark.gpu


def _system_keys(part):
    commit = struct.pack("<iI", (part << 8) | 4, 1)        # systemCommitKey: kSystem, kSystemCommit
    partk = struct.pack("<iI", (part << 8) | 4, 2)         # systemPartKey
    return [(commit, struct.pack("<qq", 1234, 5)), (partk, b"")]


def _streams(ds):
    """Per part: the encodeKV records of its data keys in bytewise key order, plus system keys."""
    by_part = {}
    for k, v in zip(ds.batch.keys, ds.batch.vals):
        part = struct.unpack_from("<i", k, 0)[0] >> 8
        by_part.setdefault(part, []).append((k, v))
    out = {}
    for part, kvs in by_part.items():
        recs = [kvfmt.encode_kv(k, v) for k, v in sorted(kvs)]
        recs += [kvfmt.encode_kv(k, v) for k, v in _system_keys(part)]
        out[part] = recs
    return out


def _load_streamed(ds, e, batch_records=7):
    e.add_space(ds.space, ds.num_parts)
    for s in ds.schemas:
        e.add_schema(ds.space, s.is_edge, s.sid, s.name, s.fields, s.ver, s.ttl_col, s.ttl_dur)
    for part, recs in sorted(_streams(ds).items()):
        for i in range(0, len(recs), batch_records):
            e.load_snapshot_rows(ds.space, b"".join(recs[i:i + batch_records]))
    e.commit(ds.space)


def _rows(r):
    assert r.ok, r.error
    return fixtures.normalize_cells(r.rows)


@pytest.fixture(scope="module")
def nba_streamed():
    ds = fixtures.nba()
    o = oracle.Oracle()
    ds.load_oracle(o)
    e = engine.Engine(0)
    _load_streamed(ds, e)
    yield ds, o, e
    e.close()


@pytest.mark.parametrize("case", CASES[:40], ids=[f"L{c['line']}" for c in CASES[:40]])
def test_snapshot_stream_gotest(nba_streamed, case):
    ds, o, e = nba_streamed
    s = ngql.parse_go(fixtures.nba_query(case["query"]))
    got, ref = e.go(ds.space, s), o.go(ds.space, s)
    assert got.ok == ref.ok
    if not ref.ok:
        return
    assert _rows(got) == fixtures.normalize_cells(ref.rows)
    assert _rows(got) == ([] if case.get("empty") else fixtures.nba_expected(case["rows"]))


def test_snapshot_stream_truncated_record_stages_nothing():
    ds = fixtures.nba()
    with engine.Engine(0) as e:
        e.add_space(ds.space, ds.num_parts)
        for s in ds.schemas:
            e.add_schema(ds.space, s.is_edge, s.sid, s.name, s.fields, s.ver, s.ttl_col, s.ttl_dur)
        recs = next(iter(_streams(ds).values()))
        good = b"".join(recs[:5])
        with pytest.raises(engine.EngineError) as ei:
            e.load_snapshot_rows(ds.space, good + recs[5][:-1])
        assert ei.value.code == engine.E_BAD_ARGUMENT
        e.commit(ds.space)
        assert e.info(ds.space).edges == 0 and e.info(ds.space).vertices == 0


RMAT_Q = [
    "GO 3 STEPS FROM {S} OVER e WHERE e.p0 < 50 YIELD e._dst, e._rank, e.p0, e.p1",
    "GO 2 STEPS FROM {S} OVER e REVERSELY WHERE $^.vt.v0 > 100 YIELD $^.vt.name, $$.vt.v0, e.p1",
]


def _register(ds, e):
    e.add_space(ds.space, ds.num_parts)
    for s in ds.schemas:
        e.add_schema(ds.space, s.is_edge, s.sid, s.name, s.fields, s.ver, s.ttl_col, s.ttl_dur)


def test_snapshot_file_roundtrip_rmat(tmp_path):
    ds = fixtures.RmatDataset(12, with_in=True, with_tag=True)
    o = oracle.Oracle()
    ds.load_oracle(o)
    path = str(tmp_path / "shard0.ngxsnap")
    seeds = ", ".join(str(int(v)) for v in datagen.sample_vids(31, 1 << ds.scale, 30))
    qs = [ngql.parse_go(q.replace("{S}", seeds)) for q in RMAT_Q]
    with engine.Engine(0) as e:
        ds.load_engine(e)
        first = [_rows(e.go(ds.space, s)) for s in qs]
        info = e.info(ds.space)
        e.save_snapshot(ds.space, path, "ckpt-2026-10-17")
    assert os.path.getsize(path) > 128
    with engine.Engine(0) as e2:
        _register(ds, e2)
        with pytest.raises(engine.EngineError) as ei:
            e2.go(ds.space, qs[0], raise_on_error=True)
        assert e2.open_snapshot(ds.space, path) == "ckpt-2026-10-17"
        i2 = e2.info(ds.space)
        assert (i2.vertices, i2.edges, i2.slots, i2.tags) == (info.vertices, info.edges, info.slots, info.tags)
        for s, want in zip(qs, first):
            assert _rows(e2.go(ds.space, s)) == want == fixtures.normalize_cells(o.go(ds.space, s).rows)


def test_snapshot_file_roundtrip_snb_strings(tmp_path):
    ds = fixtures.snb_dataset(1500, threads=8)
    o = oracle.Oracle()
    o.set_flags(threads=8)
    ds.load_oracle(o)
    path = str(tmp_path / "snb.ngxsnap")
    seeds = ", ".join(str(int(v)) for v in datagen.sample_vids(5, ds.np, 100))
    q = ngql.parse_go(f"GO 2 STEPS FROM {seeds} OVER knows, likes WHERE $$.post.lang == \"en\" || knows.weight > 5.0 "
                      "YIELD knows._dst, likes._dst, $$.post.content, $^.person.firstName")
    with engine.Engine(0) as e:
        ds.load_engine(e)
        e.save_snapshot(ds.space, path, "")
    with engine.Engine(0) as e2:
        _register(ds, e2)
        assert e2.open_snapshot(ds.space, path) == ""
        assert _rows(e2.go(ds.space, q)) == fixtures.normalize_cells(o.go(ds.space, q).rows)


def test_snapshot_file_refused(tmp_path):
    ds = fixtures.nba()
    path = str(tmp_path / "nba.ngxsnap")
    q = ngql.parse_go(fixtures.nba_query("GO FROM {P:Tim Duncan} OVER like YIELD like._dst"))
    with engine.Engine(0) as e:
        ds.load_engine(e)
        want = _rows(e.go(ds.space, q))
        e.save_snapshot(ds.space, path, "t")
        with pytest.raises(engine.EngineError):
            e.save_snapshot(ds.space, str(tmp_path / "x"), "t" * 64)      # tag too long
    raw = open(path, "rb").read()
    bad = {}
    flipped = bytearray(raw)
    flipped[len(raw) // 2] ^= 0x40
    bad["flipped"] = bytes(flipped)
    bad["truncated"] = raw[:len(raw) - 9]
    bad["header"] = b"XXXXXXXX" + raw[8:]
    for name, blob in bad.items():
        p = str(tmp_path / f"{name}.ngxsnap")
        open(p, "wb").write(blob)
        with engine.Engine(0) as e:
            ds.load_engine(e)
            with pytest.raises(engine.EngineError) as ei:
                e.open_snapshot(ds.space, p)
            assert ei.value.code == engine.E_SNAPSHOT, name
            assert _rows(e.go(ds.space, q)) == want                     # space untouched
    with engine.Engine(0) as e:
        # another schema set: one more field on `like`
        e.add_space(ds.space, ds.num_parts)
        for s in ds.schemas:
            f = s.fields + [("extra", kvfmt.INT)] if s.name == "like" else s.fields
            e.add_schema(ds.space, s.is_edge, s.sid, s.name, f, s.ver, s.ttl_col, s.ttl_dur)
        with pytest.raises(engine.EngineError) as ei:
            e.open_snapshot(ds.space, path)
        assert ei.value.code == engine.E_SNAPSHOT
    with engine.Engine(0) as e:
        e.add_space(ds.space + 1, ds.num_parts)                          # another space id
        with pytest.raises(engine.EngineError) as ei:
            e.open_snapshot(ds.space + 1, path)
        assert ei.value.code == engine.E_SNAPSHOT
        with pytest.raises(engine.EngineError):
            e.open_snapshot(ds.space + 1, str(tmp_path / "missing.ngxsnap"))
