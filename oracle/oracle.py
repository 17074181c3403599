"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/liborc.so, the C++ CPU restatement of the reference GetNeighbors
processor and GoExecutor (see oracle/orc_core.h). Imported only by tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg, never by nebula_amd/.
"""
from __future__ import annotations

import ctypes
import os
import struct
import subprocess
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liborc.so")

SOURCE, DEST, EDGE = 1, 2, 3


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, u64p = ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)
        L.orc_engine_new.restype = vp
        L.orc_engine_free.argtypes = [vp]
        L.orc_buf_free.argtypes = [vp]
        L.orc_set_flags.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32]
        L.orc_set_graph_threads.argtypes = [vp, ctypes.c_int32]
        L.orc_add_space.argtypes = [vp, ctypes.c_int32, ctypes.c_int32]
        L.orc_add_part.argtypes = [vp, ctypes.c_int32, ctypes.c_int32]
        L.orc_add_schema.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_char_p,
                                     ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(ctypes.c_char_p),
                                     ctypes.POINTER(ctypes.c_int32), ctypes.c_char_p, ctypes.c_int64]
        L.orc_put_kv.argtypes = [vp, ctypes.c_int32, ctypes.c_uint64, vp, vp, vp, vp]
        L.orc_finalize.argtypes = [vp, ctypes.c_int32]
        L.orc_kv_size.argtypes = [vp, ctypes.c_int32]
        L.orc_kv_size.restype = ctypes.c_uint64
        for fn in ("orc_get_neighbors",):
            getattr(L, fn).argtypes = [vp, ctypes.c_char_p, ctypes.c_uint64, u64p]
            getattr(L, fn).restype = vp
        L.orc_go.argtypes = [vp, ctypes.c_int32, ctypes.c_char_p, ctypes.c_uint64, u64p]
        L.orc_go.restype = vp
        for fn in ("orc_expr_eval", "orc_expr_roundtrip", "orc_expr_pushdown", "orc_expr_to_string"):
            getattr(L, fn).argtypes = [ctypes.c_char_p, ctypes.c_uint64, u64p]
            getattr(L, fn).restype = vp
        L.orc_std_hash_string.argtypes = [ctypes.c_char_p, ctypes.c_uint64]
        L.orc_std_hash_string.restype = ctypes.c_int64
        L.orc_row_write.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32), ctypes.c_char_p,
                                    ctypes.c_uint64, ctypes.c_int32, u64p]
        L.orc_row_write.restype = vp
        L.orc_row_read.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32), ctypes.c_char_p,
                                   ctypes.c_uint64, u64p]
        L.orc_row_read.restype = vp
        L.orc_row_schema_ver.argtypes = [ctypes.c_char_p, ctypes.c_uint64]
        L.orc_row_schema_ver.restype = ctypes.c_int32
        L.orc_hop_digest.argtypes = [ctypes.c_uint64, vp, vp, vp, vp, vp, vp, ctypes.c_int64, ctypes.c_int32, u64p]
        L.orc_row_digest.argtypes = [ctypes.c_uint64, ctypes.c_int32, ctypes.POINTER(vp), u64p]
        L.orc_digest_columns.argtypes = [ctypes.c_int32, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.orc_gen_buckets.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)]
        L.orc_gen_buckets.restype = ctypes.c_int32
        _lib = L
    return _lib


def _take(ptr, n) -> bytes:
    if not ptr:
        return b""
    data = ctypes.string_at(ptr, n)
    lib().orc_buf_free(ptr)
    return data


def _call(fn, *args) -> bytes:
    n = ctypes.c_uint64(0)
    p = fn(*args, ctypes.byref(n))
    return _take(p, n.value)


class _Rd:
    def __init__(self, b: bytes):
        self.b, self.p = b, 0

    def get(self, fmt):
        v = struct.unpack_from("<" + fmt, self.b, self.p)
        self.p += struct.calcsize("<" + fmt)
        return v[0] if len(v) == 1 else v

    def str(self) -> bytes:
        n = self.get("I")
        s = self.b[self.p:self.p + n]
        self.p += n
        return s

    def variant(self):
        w = self.get("B")
        if w == 0:
            return self.get("q")
        if w == 1:
            return self.get("d")
        if w == 2:
            return bool(self.get("B"))
        if w == 3:
            return self.str().decode("utf-8", "surrogateescape")
        if w == 0xFF:
            return ERR
        raise ValueError(f"bad variant tag {w}")


class _Err:
    def __repr__(self):
        return "<ERR>"


ERR = _Err()


def _s(s: str) -> bytes:
    b = s.encode() if isinstance(s, str) else s
    return struct.pack("<I", len(b)) + b


# ---------------------------------------------------------------------------- expressions

def go_request(s, pushdown=True, rows=True, digest=False, input=None) -> bytes:
    """The orc_go request blob of a parsed GoSentence (also fed to the sanitizer driver, tools/san)."""
    b = struct.pack("<IIi", s.record_from, s.record_to, len(s.vids)) + struct.pack(f"<{len(s.vids)}q", *s.vids)
    b += struct.pack("<i", len(s.over))
    for n, a in s.over:
        b += _s(n) + _s(a)
    b += struct.pack("<Bi", 1 if s.over_all else 0, s.direction)
    b += struct.pack("<B", 1 if s.where is not None else 0) + _s(s.where.encode() if s.where is not None else b"")
    b += struct.pack("<Bi", 1 if s.distinct else 0, len(s.yields))
    for y in s.yields:
        b += _s(y.expr.encode()) + _s(y.alias)
    b += struct.pack("<BB", 1 if pushdown else 0, 2 if digest else (0 if rows else 1))
    ft = getattr(s, "from_type", 0)
    b += struct.pack("<B", ft) + _s(getattr(s, "from_var", "")) + _s(getattr(s, "from_col", ""))
    names = input.names if (ft and input is not None) else []
    types = input.types if (ft and input is not None) else []
    rws = input.rows if (ft and input is not None) else []
    b += struct.pack("<i", len(names))
    for i, n in enumerate(names):
        b += _s(n) + struct.pack("<i", types[i] if i < len(types) else 0)
    b += struct.pack("<q", len(rws))
    for row in rws:
        for kind, v in row:
            if kind == "str":
                b += struct.pack("<B", 3) + _s(v.encode("utf-8", "surrogateescape"))
            elif kind in ("float", "double"):
                b += struct.pack("<Bd", 1, v)
            elif kind == "bool" or (kind == "empty" and v is not None):
                b += struct.pack("<BB", 2, 1 if v else 0)
            else:
                b += struct.pack("<Bq", 0, int(v))
    return b


def expr_eval(enc: bytes):
    """Evaluate a constant encoded expression. Returns ('ok', value) | ('err', msg) | ('prep', msg)."""
    r = _Rd(_call(lib().orc_expr_eval, enc, len(enc)))
    tag = r.get("B")
    if tag == 1:
        return ("ok", r.variant())
    return ("err" if tag == 0 else "prep", r.str().decode())


def expr_roundtrip(enc: bytes) -> bytes:
    return _call(lib().orc_expr_roundtrip, enc, len(enc))


def expr_pushdown(enc: bytes) -> bytes:
    return _call(lib().orc_expr_pushdown, enc, len(enc))


def expr_to_string(enc: bytes) -> str:
    return _call(lib().orc_expr_to_string, enc, len(enc)).decode()


def std_hash(s: str) -> int:
    b = s.encode()
    return lib().orc_std_hash_string(b, len(b))


def row_read(types: Sequence[int], row: bytes, ver: int = 0):
    arr = (ctypes.c_int32 * len(types))(*types)
    r = _Rd(_call(lib().orc_row_read, ver, len(types), arr, row, len(row)))
    return _decode_row(r)[1]


def row_write(types: Sequence[int], values: Sequence[Tuple[int, object]], ver: int = 0, with_schema=True) -> bytes:
    """values: (tag, v) with tag 0 int64, 1 double, 2 bool, 3 string, 4 float, 5 uint64, 6 skip(n)."""
    blob = b""
    for t, v in values:
        blob += bytes([t])
        blob += {0: lambda x: struct.pack("<q", x), 1: lambda x: struct.pack("<d", x),
                 2: lambda x: struct.pack("<B", 1 if x else 0), 3: lambda x: _s(x),
                 4: lambda x: struct.pack("<f", x), 5: lambda x: struct.pack("<Q", x),
                 6: lambda x: struct.pack("<q", x)}[t](v)
    arr = (ctypes.c_int32 * max(1, len(types)))(*types)
    return _call(lib().orc_row_write, ver, len(types), arr, blob, len(blob), 1 if with_schema else 0)


def row_schema_ver(row: bytes) -> int:
    return lib().orc_row_schema_ver(row, len(row))


def gen_buckets(n: int, min_per_bucket: int, max_handlers: int) -> List[int]:
    out = (ctypes.c_int32 * max(1, max_handlers))()
    k = lib().orc_gen_buckets(n, min_per_bucket, max_handlers, out)
    return list(out[:k])


def sort_digests(raw: np.ndarray) -> np.ndarray:
    """16-byte row digests -> (n, 2) uint64 array in sorted row order (a multiset fingerprint)."""
    d = np.ascontiguousarray(raw).view(np.uint64).reshape(-1, 2)
    order = np.lexsort((d[:, 1], d[:, 0]))
    return d[order]


def digest_columns(col_types: Sequence[int], nrows: int, x_ptrs, len_ptrs, t_ptrs) -> np.ndarray:
    """Sorted digests of rows given column-wise (pointers of a host_columnar device result)."""
    n = len(col_types)
    ct = (ctypes.c_int32 * max(1, n))(*col_types)
    X = (ctypes.c_void_p * max(1, n))(*x_ptrs)
    L_ = (ctypes.c_void_p * max(1, n))(*len_ptrs)
    T = (ctypes.c_void_p * max(1, n))(*t_ptrs)
    out = np.zeros(16 * max(nrows, 1), dtype=np.uint8)
    if nrows:
        lib().orc_digest_columns(n, ct, nrows, X, L_, T, out.ctypes.data)
    return sort_digests(out[:16 * nrows])


def _decode_row(r: _Rd):
    raw = r.str()
    n = r.get("i")
    if n < 0:
        return raw, None
    return raw, [r.variant() for _ in range(n)]


# ---------------------------------------------------------------------------- engine
@dataclass
class NeighborsResponse:
    failed_codes: List[Tuple[int, int]]
    vertex_schema: Dict[int, List[Tuple[str, int]]]
    edge_schema: Dict[int, List[Tuple[str, int]]]
    vertices: List[dict]
    total_edges: int


@dataclass
class GoResult:
    ok: bool
    error: str
    col_types: List[int]
    rows: List[tuple]
    hop_frontier: List[int] = field(default_factory=list)
    hop_scanned: List[int] = field(default_factory=list)
    seconds: float = 0.0                 # wall time of the restated GoExecutor run (no serialisation)
    nrows: int = 0
    digests: Optional[np.ndarray] = None  # digest=True: sorted 16-byte row digests
    column_names: List[str] = field(default_factory=list)   # getResultColumnNames


def _cell(r: _Rd):
    t = r.get("B")
    if t == 0:
        return ("empty", None)
    if t == 1:
        return ("bool", bool(r.get("B")))
    if t in (2, 3, 21):
        return ({2: "int", 3: "id", 21: "timestamp"}[t], r.get("q"))
    if t in (4, 5):
        return ({4: "float", 5: "double"}[t], r.get("d"))
    if t == 6:
        return ("str", r.str().decode("utf-8", "surrogateescape"))
    if t == 0xFE:
        return ("type_error", None)
    if t == 0xFD:                        # a bool of an UNKNOWN column: unset in the response
        return ("empty", bool(r.get("B")))
    raise ValueError(t)


class Oracle:
    def __init__(self):
        self.L = lib()
        self.h = ctypes.c_void_p(self.L.orc_engine_new())

    def close(self):
        if self.h:
            self.L.orc_engine_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_flags(self, max_handlers=10, min_vertices=3, max_edges=2**31 - 1, now_sec=0, threads=1, graph_threads=1):
        """threads: the reader-pool threads that run a request's buckets; graph_threads (test harness, not a
        reference flag): threads of the final evaluation of GO (rows in the sequential order)."""
        self.L.orc_set_flags(self.h, max_handlers, min_vertices, max_edges, now_sec, threads)
        self.L.orc_set_graph_threads(self.h, graph_threads)

    def add_space(self, space: int, num_parts: int):
        self.L.orc_add_space(self.h, space, num_parts)

    def add_part(self, space: int, part: int):
        self.L.orc_add_part(self.h, space, part)

    def add_schema(self, space, is_edge, sid, name, fields: Sequence[Tuple[str, int]], ver=0, ttl_col="", ttl_dur=0):
        names = (ctypes.c_char_p * max(1, len(fields)))(*[f[0].encode() for f in fields])
        types = (ctypes.c_int32 * max(1, len(fields)))(*[f[1] for f in fields])
        self.L.orc_add_schema(self.h, space, 1 if is_edge else 0, sid, name.encode(), ver, len(fields), names, types,
                              ttl_col.encode(), ttl_dur)

    def put_kv(self, space: int, keys, koff, vals, voff):
        n = len(koff) - 1
        keys, koff, vals, voff = (np.ascontiguousarray(a) for a in (keys, koff, vals, voff))
        self.L.orc_put_kv(self.h, space, n, keys.ctypes.data, koff.ctypes.data, vals.ctypes.data, voff.ctypes.data)

    def put_batch(self, space: int, batch):
        self.put_kv(space, *batch.arrays())

    def finalize(self, threads=1):
        self.L.orc_finalize(self.h, threads)

    def kv_size(self, space):
        return self.L.orc_kv_size(self.h, space)

    def get_neighbors(self, space, parts: Sequence[Tuple[int, Sequence[int]]], edge_types: Optional[Sequence[int]],
                      return_columns: Sequence[Tuple[int, int, str]], filter_bytes: bytes = b"",
                      only_vertex_props=False) -> NeighborsResponse:
        b = struct.pack("<ii", space, len(parts))
        for p, vids in parts:
            b += struct.pack("<ii", p, len(vids)) + struct.pack(f"<{len(vids)}q", *vids)
        et = list(edge_types or [])
        b += struct.pack("<Bi", 1 if edge_types is not None else 0, len(et)) + struct.pack(f"<{len(et)}i", *et)
        b += _s(filter_bytes)
        b += struct.pack("<i", len(return_columns))
        for owner, i, name in return_columns:
            b += struct.pack("<ii", owner, i) + _s(name)
        b += struct.pack("<B", 1 if only_vertex_props else 0)
        t0 = time.perf_counter()
        n = ctypes.c_uint64(0)
        p = self.L.orc_get_neighbors(self.h, b, len(b), ctypes.byref(n))
        self.last_seconds = time.perf_counter() - t0     # processor + response encoding, no Python decode
        r = _Rd(_take(p, n.value))
        failed = [r.get("ii") for _ in range(r.get("i"))]

        def schemas():
            out = {}
            for _ in range(r.get("i")):
                k = r.get("i")
                out[k] = [(r.str().decode(), r.get("i")) for _ in range(r.get("i"))]
            return out

        vs, es = schemas(), schemas()
        verts = []
        for _ in range(r.get("i")):
            vid = r.get("q")
            tags = []
            for _ in range(r.get("i")):
                tid = r.get("i")
                raw, vals = _decode_row(r)
                tags.append({"tag_id": tid, "raw": raw, "values": vals})
            edata = []
            for _ in range(r.get("i")):
                et = r.get("i")
                edges = []
                for _ in range(r.get("i")):
                    dst = r.get("q")
                    has = r.get("B")
                    raw, vals = _decode_row(r) if has else (None, None)
                    edges.append({"dst": dst, "raw": raw, "values": vals})
                edata.append({"type": et, "edges": edges})
            verts.append({"vid": vid, "tags": tags, "edges": edata})
        return NeighborsResponse(failed, vs, es, verts, r.get("i"))

    def go(self, space: int, s, pushdown=True, rows=True, digest=False, input=None) -> GoResult:
        """Run a parsed nebula_amd.ngql.GoSentence through the restated GoExecutor. digest=True
        returns the rows as sorted 128-bit digests of their serialized cells (digest_columns())."""
        b = go_request(s, pushdown, rows, digest, input)
        r = _Rd(_call(self.L.orc_go, self.h, space, b, len(b)))
        ok = r.get("B") == 1
        err = r.str().decode()
        ncol = r.get("i")
        types = [r.get("i") for _ in range(ncol)]
        nrows = r.get("q")
        dig = None
        if digest:
            dig = sort_digests(np.frombuffer(r.b, dtype=np.uint8, count=16 * nrows, offset=r.p))
            r.p += 16 * nrows
        out = [tuple(_cell(r) for _ in range(ncol)) for _ in range(nrows)] if rows and not digest else []
        hops = r.get("i")
        fr, sc = [], []
        for _ in range(hops):
            fr.append(r.get("q"))
            sc.append(r.get("q"))
        secs = r.get("d")
        names_out = [r.str().decode() for _ in range(r.get("i"))]
        return GoResult(ok, err, types, out, fr, sc, secs, nrows, dig, names_out)


def hop_digest(rows, vid, off, dst, p0, p1, rank=0, threads=1):
    """Expected (sum, xor, rows) row-hash digests of a record hop's result rows (src, dst, rank, p0, p1)
    over the out-edges of frontier rows `rows` of a generated CSR shard, for no filter, p0 < 50 and
    p0 >= 50 (orc_digest.cpp; compared with ngx_go_result_digest of the device result)."""
    import numpy as np
    rows = np.ascontiguousarray(rows, dtype=np.int64)
    vid = np.ascontiguousarray(vid, dtype=np.int64)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    dst = np.ascontiguousarray(dst, dtype=np.int64)
    p0 = np.ascontiguousarray(p0, dtype=np.int8)
    p1 = np.ascontiguousarray(p1, dtype=np.int64)
    out = (ctypes.c_uint64 * 9)()
    lib().orc_hop_digest(len(rows), rows.ctypes.data, vid.ctypes.data, off.ctypes.data, dst.ctypes.data,
                         p0.ctypes.data, p1.ctypes.data, int(rank), int(threads), out)
    return {"all": tuple(out[0:3]), "lt": tuple(out[3:6]), "ge": tuple(out[6:9])}


def row_digest(cols):
    """(sum, xor, rows) of the row hashes of equal-length int64 columns (the first is the src vid)."""
    import numpy as np
    cols = [np.ascontiguousarray(c, dtype=np.int64) for c in cols]
    ptrs = (ctypes.c_void_p * len(cols))(*[c.ctypes.data for c in cols])
    out = (ctypes.c_uint64 * 3)()
    lib().orc_row_digest(len(cols[0]) if cols else 0, len(cols), ptrs, out)
    return tuple(out)
