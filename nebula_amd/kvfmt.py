"""Reference-format KV rows, written from Python (host side; small fixtures and tests).

Restates the byte layouts the storage path reads:
* keys — src/common/utils/NebulaKeyUtils.cpp:12-45 (24-byte vertex keys, 40-byte edge keys,
  edge type stored as `type | 0x40000000`);
* rows — src/dataman/RowWriter.cpp:39-263 / RowWriter.inl (header byte, little-endian schema
  version, block offsets every 16 fields, LEB128 varints for INT/TIMESTAMP/string lengths,
  raw little-endian VID/FLOAT/DOUBLE, one byte BOOL).
Large synthetic graphs are generated natively (nebula_amd/csrc/datagen.cpp); this module serves the
reference test fixtures (QueryBoundTest mock data, the NBA dataset).
"""
from __future__ import annotations

import struct
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

BOOL, INT, VID, FLOAT, DOUBLE, STRING, TIMESTAMP = 1, 2, 3, 4, 5, 6, 21     # SupportedType


def edge_key(part: int, src: int, etype: int, rank: int, dst: int, ver: int = 0) -> bytes:
    item = (part << 8) | 1
    et = (etype | 0x40000000) & 0xFFFFFFFF
    return struct.pack("<iqIqqq", item, src, et, rank, dst, ver)


def vertex_key(part: int, vid: int, tag: int, ver: int = 0) -> bytes:
    item = (part << 8) | 1
    return struct.pack("<iqiq", item, vid, tag & ~0x40000000, ver)


def encode_kv(key: bytes, val: bytes) -> bytes:
    """One record of a raft snapshot stream / WAL batch: u32 key size, u32 value size, key, value
    (kvstore::encodeKV, src/kvstore/LogEncoder.cpp:16-27)."""
    return struct.pack("<II", len(key), len(val)) + key + val


def decode_kv(rec: bytes) -> Tuple[bytes, bytes]:
    """kvstore::decodeKV (src/kvstore/LogEncoder.cpp:29-36)."""
    ks, vs = struct.unpack_from("<II", rec, 0)
    return rec[8:8 + ks], rec[8 + ks:8 + ks + vs]


def varint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _occupied(v: int) -> int:
    n = 0
    while True:
        n += 1
        v >>= 8
        if not v:
            return n


class RowWriter:
    """RowWriter with a schema (list of types) or without one (types follow the written values)."""

    def __init__(self, types: Optional[Sequence[int]] = None, ver: int = 0):
        self.types = list(types) if types is not None else None
        self.ver = ver
        self.cord = bytearray()
        self.col = 0
        self.blocks: List[int] = []

    def _type(self, stream_type):
        if self.types is None or self.col >= len(self.types):
            return stream_type
        return self.types[self.col]

    def _done(self):
        self.col += 1
        if self.col % 16 == 0:
            self.blocks.append(len(self.cord))

    def int(self, v: int):
        t = self._type(INT)
        if t in (INT, TIMESTAMP):
            self.cord += varint(v)
        elif t == VID:
            self.cord += struct.pack("<q", v)
        else:
            self.cord += varint(0)
        self._done()
        return self

    def double(self, v: float):
        t = self._type(DOUBLE)
        self.cord += struct.pack("<f", v) if t == FLOAT else struct.pack("<d", v if t == DOUBLE else 0.0)
        self._done()
        return self

    def float(self, v: float):
        t = self._type(FLOAT)
        self.cord += struct.pack("<d", v) if t == DOUBLE else struct.pack("<f", v if t == FLOAT else 0.0)
        self._done()
        return self

    def bool(self, v: bool):
        t = self._type(BOOL)
        self.cord += bytes([1 if (v and t == BOOL) else 0])
        self._done()
        return self

    def string(self, s: str):
        t = self._type(STRING)
        b = s.encode() if isinstance(s, str) else bytes(s)
        if t == STRING:
            self.cord += varint(len(b)) + b
        else:
            self.cord += varint(0)
        self._done()
        return self

    def value(self, v, t: Optional[int] = None):
        """Write a Python value, choosing the stream type from the schema column (or the value)."""
        t = t if t is not None else (self.types[self.col] if self.types and self.col < len(self.types) else None)
        if isinstance(v, bool) or t == BOOL:
            return self.bool(bool(v))
        if isinstance(v, str) or t == STRING:
            return self.string(v)
        if isinstance(v, float) and t == FLOAT:
            return self.float(v)
        if isinstance(v, float) or t in (DOUBLE,):
            return self.double(float(v))
        return self.int(int(v))

    def encode(self) -> bytes:
        if self.types is not None:
            # Skip(numFields - colNum) padding, with the reference's block-offset bookkeeping
            for i in range(self.col, len(self.types)):
                t = self.types[i]
                if t == BOOL:
                    self.cord += b"\x00"
                elif t in (INT, TIMESTAMP, STRING):
                    self.cord += varint(0)
                elif t == FLOAT:
                    self.cord += struct.pack("<f", 0.0)
                elif t == DOUBLE:
                    self.cord += struct.pack("<d", 0.0)
                elif t == VID:
                    self.cord += struct.pack("<Q", 0)
                if i != 0 and i % 16 == 0:
                    self.blocks.append(len(self.cord))
            self.col = max(self.col, len(self.types))
        ob = _occupied(len(self.cord))
        header = ob - 1
        out = bytearray()
        if self.ver > 0:
            vb = _occupied(self.ver)
            out.append(header | (vb << 5))
            out += self.ver.to_bytes(8, "little")[:vb]
        else:
            out.append(header)
        for off in self.blocks:
            out += off.to_bytes(8, "little")[:ob]
        return bytes(out + self.cord)


def encode_row(types: Sequence[int], values: Sequence, ver: int = 0) -> bytes:
    w = RowWriter(types, ver)
    for t, v in zip(types, values):
        w.value(v, t)
    return w.encode()


class KVBatch:
    """A batch of (key, value) rows as contiguous byte arrays + offsets (the C-ABI input form)."""

    def __init__(self):
        self.keys: List[bytes] = []
        self.vals: List[bytes] = []

    def put(self, k: bytes, v: bytes):
        self.keys.append(k)
        self.vals.append(v)

    def __len__(self):
        return len(self.keys)

    def arrays(self):
        kb = b"".join(self.keys)
        vb = b"".join(self.vals)
        ko = np.zeros(len(self.keys) + 1, dtype=np.uint64)
        vo = np.zeros(len(self.vals) + 1, dtype=np.uint64)
        ko[1:] = np.cumsum([len(k) for k in self.keys], dtype=np.uint64)
        vo[1:] = np.cumsum([len(v) for v in self.vals], dtype=np.uint64)
        return (np.frombuffer(kb, dtype=np.uint8) if kb else np.zeros(1, np.uint8), ko,
                np.frombuffer(vb, dtype=np.uint8) if vb else np.zeros(1, np.uint8), vo)
