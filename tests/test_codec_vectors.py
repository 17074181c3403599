"""Codec byte vectors of the reference's own unit tests, pinned on the oracle's RowReader and on the
Python-side writers (kvfmt) the fixtures are built with.

* RowReaderTest.headerInfo / encodedData (src/dataman/test/RowReaderTest.cpp:14-272): header bytes
  -> schema version, and a hand-assembled 10-column row -> field values;
* RowWriterTest.withSchema / skip / offsetsCreation (src/dataman/test/RowWriterTest.cpp:133-290):
  written rows read back with the same schema, skipped fields as type defaults, block offsets
  every 16 fields;
* NebulaKeyUtilsTest.SimpleTest (src/common/utils/test/NebulaKeyUtilsTest.cpp:13-42): 24-byte
  vertex keys and 40-byte edge keys with their fields at the offsets of NebulaKeyUtils.h:189-212.

The device side of the same row bytes (exporter RowReader -> columns -> GetNeighbors) is pinned in
tests/test_gpu_codec.py.
"""
import struct

import pytest

from nebula_amd import kvfmt
from nebula_amd.kvfmt import BOOL, DOUBLE, FLOAT, INT, STRING, TIMESTAMP, VID
from oracle import oracle

STR1 = "Hello World!"
STR2 = "Welcome to the future!"
PI_F = struct.unpack("<f", struct.pack("<f", 3.1415926))[0]
E = 2.71828182845904523536028747135266249775724709369995

# RowReaderTest.encodedData schema (RowReaderTest.cpp:79-104)
ENCODED_TYPES = [BOOL, STRING, INT, INT, VID, STRING, BOOL, FLOAT, DOUBLE, TIMESTAMP]


def encoded_data_row() -> bytes:
    """The row RowReaderTest.cpp:106-151 assembles byte by byte."""
    b = bytearray(b"\x00")                            # header: version 0, 1-byte offsets, no blocks
    b += b"\x01"                                     # col 0 bool
    b += kvfmt.varint(len(STR1)) + STR1.encode()     # col 1 string
    b += kvfmt.varint(100)                           # col 2 int
    b += kvfmt.varint(0xFFFFFFFFFFFFFFFF)            # col 3 int (-1 as uint64)
    b += struct.pack("<q", 0x8877665544332211 - (1 << 64))   # col 4 vid, raw 8 bytes
    b += kvfmt.varint(len(STR2)) + STR2.encode()     # col 5 string
    b += b"\x00"                                     # col 6 bool
    b += struct.pack("<f", 3.1415926)                # col 7 float
    b += struct.pack("<d", E)                        # col 8 double
    b += kvfmt.varint(1551331827)                    # col 9 timestamp
    return bytes(b)


ENCODED_VALUES = [True, STR1, 100, -1, 0x8877665544332211 - (1 << 64), STR2, False, PI_F, E, 1551331827]


@pytest.mark.parametrize("row,ver", [
    (b"\x00", 0),                                    # simplest row
    (b"\x40\x01\xff", 0x00FF01),                     # 2 version bytes
    (b"\x60\x01\xff\xff\x40\xf0", 0x00FFFF01),       # 3 version bytes + block offsets
    (b"\x01\xff\x40\x08\xf0", 0),                    # no version, 2-byte offsets
])
def test_header_schema_version(row, ver):
    assert oracle.row_schema_ver(row) == ver


def test_encoded_data_reader():
    got = oracle.row_read(ENCODED_TYPES, encoded_data_row())
    assert got[:7] == ENCODED_VALUES[:7]
    assert got[7] == pytest.approx(PI_F, rel=0, abs=0)   # float read widened to double exactly
    assert got[8] == E
    assert got[9] == 1551331827


def test_encoded_data_writers_produce_the_reference_bytes():
    """The same values written with a schema give the test's hand-assembled bytes, from both the
    fixture writer (kvfmt) and the oracle's RowWriter restatement."""
    want = encoded_data_row()
    w = kvfmt.RowWriter(ENCODED_TYPES)
    w.bool(True).string(STR1).int(100).int(-1).int(0x8877665544332211 - (1 << 64)).string(STR2)
    w.bool(False).float(3.1415926).double(E).int(1551331827)
    assert w.encode() == want
    vals = [(2, True), (3, STR1), (0, 100), (0, -1), (0, 0x8877665544332211 - (1 << 64)), (3, STR2),
            (2, False), (4, 3.1415926), (1, E), (0, 1551331827)]
    assert oracle.row_write(ENCODED_TYPES, vals) == want


def test_row_writer_with_schema():
    """RowWriterTest.withSchema (RowWriterTest.cpp:153-217): a double into a FLOAT column, an int
    into a VID column."""
    types = [INT, INT, STRING, STRING, BOOL, FLOAT, VID, TIMESTAMP]
    vals = [(0, 1), (0, 2), (3, "Hello"), (3, "World"), (2, True), (1, 3.1415926), (0, 1234567), (0, 1551331827)]
    row = oracle.row_write(types, vals)
    got = oracle.row_read(types, row)
    assert got[:5] == [1, 2, "Hello", "World", True]
    assert got[5] == struct.unpack("<f", struct.pack("<f", 3.1415926))[0]
    assert got[6:] == [1234567, 1551331827]
    w = kvfmt.RowWriter(types)
    w.int(1).int(2).string("Hello").string("World").bool(True).double(3.1415926).int(1234567).int(1551331827)
    assert w.encode() == row


def test_row_writer_skip():
    """RowWriterTest.skip (RowWriterTest.cpp:220-290): skipped and implicitly skipped fields read
    back as the type defaults."""
    types = [INT, FLOAT, INT, STRING, STRING, BOOL, VID, DOUBLE, TIMESTAMP]
    vals = [(6, 1), (1, 3.14), (6, 1), (3, "Hello"), (6, 1), (2, True)]
    got = oracle.row_read(types, oracle.row_write(types, vals))
    assert got[0] == 0
    assert got[1] == struct.unpack("<f", struct.pack("<f", 3.14))[0]
    assert got[2:] == [0, "Hello", "", True, 0, 0.0, 0]


def test_row_writer_offsets_creation():
    """RowWriterTest.offsetsCreation (RowWriterTest.cpp:133-150): 33 int fields -> block offsets at
    fields 16 and 32 (two stored offsets after the header)."""
    types = [INT] * 33
    row = oracle.row_write(types, [(0, i) for i in range(33)], with_schema=False)
    w = kvfmt.RowWriter()
    for i in range(33):
        w.int(i)
    assert w.encode() == row
    # every value < 128 is a 1-byte varint: the data is 33 bytes, so offsets are 1 byte wide
    assert row[0] == 0x00
    assert row[1:3] == bytes([16, 32])
    assert len(row) == 3 + 33
    assert oracle.row_read(types, row) == list(range(33))


def test_key_layout():
    """NebulaKeyUtilsTest.SimpleTest: part 15, src 1001, dst 2001, tag 1001, type 101, rank 10,
    versions 20 (NebulaKeyUtilsTest.cpp:14-20); field offsets NebulaKeyUtils.h:189-212."""
    vk = kvfmt.vertex_key(15, 1001, 1001, 20)
    assert len(vk) == 24                                  # isVertex: kVertexLen
    item, vid, tag, ver = struct.unpack("<iqiq", vk)
    assert item & 0xFF == 1 and item >> 8 == 15           # kData type byte + part
    assert (vid, tag, ver) == (1001, 1001, 20)
    ek = kvfmt.edge_key(15, 1001, 101, 10, 2001, 20)
    assert len(ek) == 40                                  # isEdge: kEdgeLen
    item, src, et, rank, dst, ver = struct.unpack("<iqiqqq", ek)
    assert item >> 8 == 15 and (src, rank, dst, ver) == (1001, 10, 2001, 20)
    assert et == 101 | 0x40000000                         # edge type tagged on disk
    assert (et & ~0x40000000 if et > 0 else et) == 101    # getEdgeType read-back
    nk = kvfmt.edge_key(15, 2001, -101, 10, 1001, 20)     # in-edge: the negative type round-trips
    et = struct.unpack_from("<i", nk, 12)[0]
    assert (et & ~0x40000000 if et > 0 else et) == -101


def test_varint_extremes():
    """folly varint (RowReader.inl:62-68): LEB128 of the uint64 bit pattern, 10 bytes for -1."""
    assert kvfmt.varint(0) == b"\x00"
    assert kvfmt.varint(127) == b"\x7f"
    assert kvfmt.varint(128) == b"\x80\x01"
    assert kvfmt.varint(-1) == b"\xff" * 9 + b"\x01"
    for v in (0, 1, 127, 128, 2 ** 31, 2 ** 63 - 1, -2 ** 63, -1):
        row = oracle.row_write([INT], [(0, v)])
        assert oracle.row_read([INT], row) == [v]


def test_encode_kv_layout():
    """LogEncoderTest.KVTest (src/kvstore/test/LogEncoderTest.cpp:117-122): the raft snapshot record
    ngx_load_snapshot_rows ingests."""
    rec = kvfmt.encode_kv(b"KV_key", b"KV_val")
    assert rec == struct.pack("<II", 6, 6) + b"KV_keyKV_val"
    assert kvfmt.decode_kv(rec) == (b"KV_key", b"KV_val")
