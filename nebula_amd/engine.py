"""Host-side mirror of the reference's GetNeighbors / GO interface over libnebula_gn.so.

`Engine` is one shard (one GPU). Its methods follow the reference call surface for the path:
  add_space / add_schema   meta::SchemaManager (src/meta/SchemaManager.h:18-56)
  load_kv / commit         the KV rows of the space's parts (NebulaKeyUtils keys + RowWriter values)
                           -> per-part CSR + columnar props in HBM
  get_neighbors            StorageClient::getNeighbors -> QueryBoundProcessor
                           (src/storage/client/StorageClient.cpp:121-157, QueryBoundProcessor.cpp)
  go                       GoExecutor (src/graph/GoExecutor.cpp) for `GO [M TO] N STEPS FROM ...
                           OVER ... [REVERSELY|BIDIRECT] [WHERE ...] YIELD [DISTINCT] ...`
There is no CPU fallback: a missing library raises at import of the first Engine.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np

from . import ngql

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libnebula_gn.so")

NGX_OK = 0
E_BAD_ARGUMENT = -1001
E_UNSUPPORTED = -1002
E_QUERY = -1003
E_DEVICE = -1004
E_NOT_LOADED = -1005
E_SNAPSHOT = -1006

SOURCE, DEST, EDGE = 1, 2, 3


class EngineError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


# ----------------------------------------------------------------------------- C structs
c_i32, c_i64, c_u32, c_u64, c_dbl = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_double
P = ctypes.POINTER


class Config(ctypes.Structure):
    _fields_ = [("device", c_i32), ("rank", c_i32), ("world", c_i32), ("nccl_unique_id", ctypes.c_void_p),
                ("exchange", ctypes.c_void_p), ("exchange_user", ctypes.c_void_p)]


class KVBatchC(ctypes.Structure):
    _fields_ = [("n", c_u64), ("keys", ctypes.c_void_p), ("key_off", ctypes.c_void_p), ("vals", ctypes.c_void_p),
                ("val_off", ctypes.c_void_p)]


class GraphInfo(ctypes.Structure):
    _fields_ = [("vertices", c_u64), ("edges", c_u64), ("device_bytes", c_u64), ("slots", c_i32), ("tags", c_i32)]


class CellV(ctypes.Union):
    _fields_ = [("i", c_i64), ("d", c_dbl), ("str_off", c_u64)]


class Cell(ctypes.Structure):
    _fields_ = [("kind", c_i32), ("str_len", c_i32), ("v", CellV)]


class PropDef(ctypes.Structure):
    _fields_ = [("owner", c_i32), ("id", c_i32), ("name", ctypes.c_char_p)]


class GnRequest(ctypes.Structure):
    _fields_ = [("space", c_i32), ("nparts", c_i32), ("parts", P(c_i32)), ("part_nvids", P(c_u32)),
                ("vids", P(c_i64)), ("nedge_types", c_i32), ("edge_types", P(c_i32)), ("filter", ctypes.c_char_p),
                ("filter_len", c_u32), ("ncols", c_i32), ("cols", P(PropDef)), ("max_edges_per_vertex", c_i32),
                ("now_sec", c_i64), ("encode_rows", c_i32)]


class SchemaDefC(ctypes.Structure):
    _fields_ = [("is_edge", c_i32), ("id", c_i32), ("ncols", c_i32), ("names", P(ctypes.c_char_p)),
                ("types", P(c_i32))]


class GnResult(ctypes.Structure):
    _fields_ = [("code", c_i32), ("nfailed", c_i32), ("failed_codes", P(c_i32)), ("nedges", c_u64),
                ("edge_vertex", P(c_u32)), ("edge_type", P(c_i32)), ("edge_dst", P(c_i64)), ("ncols", c_i32),
                ("edge_cells", P(Cell)), ("nvertices", c_u32), ("vertex_cells", P(Cell)),
                ("vertex_has_tag", P(ctypes.c_uint8)), ("strings", ctypes.c_void_p), ("strings_len", c_u64),
                ("edge_props", ctypes.c_void_p), ("edge_props_off", P(c_u64)), ("nschemas", c_i32),
                ("schemas", P(SchemaDefC)), ("ntag_rows", c_u32), ("tag_row_vertex", P(c_u32)),
                ("tag_row_tag", P(c_i32)), ("tag_props", ctypes.c_void_p), ("tag_props_off", P(c_u64)),
                ("latency_in_us", c_i64)]


class GoPlan(ctypes.Structure):
    _fields_ = [("space", c_i32), ("record_from", c_u32), ("record_to", c_u32), ("nstarts", c_u64),
                ("starts", P(c_i64)), ("nover", c_i32), ("over_names", P(ctypes.c_char_p)),
                ("over_aliases", P(ctypes.c_char_p)), ("over_all", c_i32), ("direction", c_i32),
                ("where", ctypes.c_char_p), ("where_len", c_u32), ("nyields", c_i32),
                ("yields", P(ctypes.c_char_p)), ("yield_lens", P(c_u32)), ("distinct", c_i32),
                ("filter_pushdown", c_i32), ("now_sec", c_i64), ("result_on_device", c_i32),
                ("host_columnar", c_i32), ("input_vid_col", ctypes.c_char_p), ("input_var", ctypes.c_char_p),
                ("input_ncols", c_i32), ("input_names", P(ctypes.c_char_p)), ("input_types", P(c_i32)),
                ("input_nrows", c_u64), ("input_cells", P(Cell)), ("input_strings", ctypes.c_char_p),
                ("yield_only", c_i32), ("compact_results", c_i32)]


_CELL_KIND = {"empty": 0, "bool": 1, "int": 2, "id": 3, "float": 4, "double": 5, "str": 6, "timestamp": 21}


def _input_arrays(inp):
    """An Interim (nebula_amd.pipeline) as the plan's input_* arrays; the tuple keeps them alive."""
    nc, nr = len(inp.names), len(inp.rows)
    names = (ctypes.c_char_p * max(1, nc))(*[n.encode() for n in inp.names])
    types = (c_i32 * max(1, nc))(*(list(inp.types) + [0] * (nc - len(inp.types))))
    cells = (Cell * max(1, nr * nc))()
    strings = bytearray()
    for r, row in enumerate(inp.rows):
        for c, (kind, v) in enumerate(row):
            cl = cells[r * nc + c]
            cl.kind = _CELL_KIND[kind] if not (kind == "empty" and v is not None) else 1
            if kind == "str":
                b = v.encode("utf-8", "surrogateescape")
                cl.v.str_off = len(strings)
                cl.str_len = len(b)
                strings += b
            elif kind in ("float", "double"):
                cl.v.d = v
            elif v is not None:                                   # ints, bools (an unset bool too)
                cl.v.i = int(v)
    return names, types, cells, bytes(strings) + b"\0", nc, nr


class CsrSlotC(ctypes.Structure):
    _fields_ = [("etype", c_i32), ("off", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("rank", ctypes.c_void_p),
                ("ncols", c_i32), ("cols", ctypes.c_void_p)]


class CsrShardC(ctypes.Structure):
    _fields_ = [("nvertices", c_u64), ("vpart", ctypes.c_void_p), ("vid", ctypes.c_void_p), ("nslots", c_i32),
                ("slots", P(CsrSlotC))]


class GoResultC(ctypes.Structure):
    _fields_ = [("code", c_i32), ("ncols", c_i32), ("col_types", P(c_i32)), ("nrows", c_u64), ("cells", P(Cell)),
                ("row_src", P(c_i64)), ("row_dst", P(c_i64)), ("row_rank", P(c_i64)), ("row_type", P(c_i32)),
                ("strings", ctypes.c_void_p), ("strings_len", c_u64), ("nhops", c_i32),
                ("hop_frontier", P(c_u64)), ("hop_edges", P(c_u64)), ("hop_next", P(c_u64)),
                ("device_ms", c_dbl), ("dev_src", ctypes.c_void_p), ("dev_dst", ctypes.c_void_p),
                ("dev_rank", ctypes.c_void_p), ("dev_type", ctypes.c_void_p), ("dev_cols", ctypes.c_void_p),
                ("dev_type_const", ctypes.c_int32), ("host_cols", ctypes.c_void_p),
                ("hop_exchange_bytes", P(c_u64)), ("host_prep_ms", c_dbl), ("host_tail_ms", c_dbl),
                ("dev_key_w", c_i32 * 3), ("dev_col_w", P(c_i32)),
                ("dev_key_const", c_i64 * 3), ("dev_col_const", P(c_i64))]


class Stat(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("value", c_i64)]


class KernelStat(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("launches", c_u32), ("total_ms", c_dbl), ("algo_bytes", c_u64)]


# every symbol include/nebula_gn.h declares: (name, restype, argtypes)
SIGNATURES = {
    "ngx_open": (c_i32, [P(Config), P(ctypes.c_void_p)]),
    "ngx_close": (None, [ctypes.c_void_p]),
    "ngx_last_error": (ctypes.c_char_p, [ctypes.c_void_p]),
    "ngx_build_info": (ctypes.c_char_p, []),
    "ngx_get_unique_id": (c_i32, [ctypes.c_void_p]),
    "ngx_add_space": (c_i32, [ctypes.c_void_p, c_i32, c_i32]),
    "ngx_add_schema": (c_i32, [ctypes.c_void_p, c_i32, c_i32, c_i32, ctypes.c_char_p, c_i64, c_i32,
                               P(ctypes.c_char_p), P(c_i32), ctypes.c_char_p, c_i64]),
    "ngx_load_kv": (c_i32, [ctypes.c_void_p, c_i32, P(KVBatchC)]),
    "ngx_load_csr": (c_i32, [ctypes.c_void_p, c_i32, P(CsrShardC)]),
    "ngx_commit": (c_i32, [ctypes.c_void_p, c_i32]),
    "ngx_graph_info_get": (c_i32, [ctypes.c_void_p, c_i32, P(GraphInfo)]),
    "ngx_get_neighbors": (c_i32, [ctypes.c_void_p, P(GnRequest), P(P(GnResult))]),
    "ngx_gn_result_free": (None, [P(GnResult)]),
    "ngx_go": (c_i32, [ctypes.c_void_p, P(GoPlan), P(P(GoResultC))]),
    "ngx_go_result_free": (None, [P(GoResultC)]),
    "ngx_go_batch": (c_i32, [ctypes.c_void_p, ctypes.c_void_p, c_i32, P(c_i32), P(c_u64), P(c_u64), P(c_u64)]),
    "ngx_set_profiling": (c_i32, [ctypes.c_void_p, c_i32]),
    "ngx_synchronize": (c_i32, [ctypes.c_void_p]),
    "ngx_go_result_digest": (c_i32, [ctypes.c_void_p, P(GoResultC), P(c_u64)]),
    "ngx_stats": (c_i32, [ctypes.c_void_p, P(P(Stat)), P(c_i32)]),
    "ngx_kernel_stats": (c_i32, [ctypes.c_void_p, P(P(KernelStat)), P(c_i32)]),
    "ngx_set_flag": (c_i32, [ctypes.c_void_p, ctypes.c_char_p, c_i64]),
    "ngx_get_flag": (c_i32, [ctypes.c_void_p, ctypes.c_char_p, P(c_i64)]),
    "ngx_jit_note": (ctypes.c_char_p, [ctypes.c_void_p]),
    "ngx_hash_string": (c_i64, [ctypes.c_char_p, c_u64]),
    "ngx_device_to_host": (c_i32, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, c_u64]),
    "ngx_load_snapshot_rows": (c_i32, [ctypes.c_void_p, c_i32, ctypes.c_void_p, c_u64]),
    "ngx_save_snapshot": (c_i32, [ctypes.c_void_p, c_i32, ctypes.c_char_p, ctypes.c_char_p]),
    "ngx_open_snapshot": (c_i32, [ctypes.c_void_p, c_i32, ctypes.c_char_p, ctypes.c_char_p]),
}


class DevColumn(ctypes.Structure):
    _fields_ = [("x", ctypes.c_void_p), ("len", ctypes.c_void_p), ("type", ctypes.c_void_p)]

_lib = None


def lib():
    """Load libnebula_gn.so. Raises if it is not built: there is no other implementation."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise EngineError(E_DEVICE, f"{LIB_PATH} is missing; build it with `make -C nebula_amd/csrc`")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


XCHG_ALLGATHER, XCHG_ALLTOALL = 0, 1
ExchangeFn = ctypes.CFUNCTYPE(c_i32, ctypes.c_void_p, c_i32, ctypes.c_void_p, ctypes.c_void_p, c_u64)


def dist_exchange(group=None):
    """Host collective for ngx_config.exchange over torch.distributed (gloo): lets world > 1 shards
    share one GPU (multi-shard tests) where RCCL needs one GPU per rank. Semantics: nebula_gn.h."""
    import torch
    import torch.distributed as dist

    def fn(user, op, send, recv, nbytes):
        try:
            w, me = dist.get_world_size(group), dist.get_rank(group)
            n_send = nbytes if op == XCHG_ALLGATHER else nbytes * w
            sb = torch.frombuffer(bytearray(ctypes.string_at(send, n_send)), dtype=torch.uint8) if n_send else \
                torch.zeros(0, dtype=torch.uint8)
            got = [torch.empty(n_send, dtype=torch.uint8) for _ in range(w)]
            dist.all_gather(got, sb, group=group)     # gloo has no all_to_all: gather and pick blocks
            if op == XCHG_ALLTOALL:
                got = [g[me * nbytes:(me + 1) * nbytes] for g in got]
            out = torch.cat(got).numpy()
            if out.size:
                ctypes.memmove(recv, out.ctypes.data, out.size)
            return 0
        except Exception:                          # never raise through the C ABI
            return 1

    return ExchangeFn(fn)


def unique_id() -> bytes:
    buf = ctypes.create_string_buffer(128)
    rc = lib().ngx_get_unique_id(buf)
    if rc:
        raise EngineError(rc, "ncclGetUniqueId failed")
    return buf.raw


# ----------------------------------------------------------------------------- results
def _cells(cells, n, ncols, strings: bytes):
    out = []
    kinds = {0: "empty", 1: "bool", 2: "int", 3: "id", 4: "float", 5: "double", 6: "str", 21: "timestamp"}
    for r in range(n):
        row = []
        for c in range(ncols):
            cl = cells[r * ncols + c]
            k = kinds.get(cl.kind, str(cl.kind))
            if cl.kind == 0:
                row.append(("empty", bool(cl.v.i) if cl.str_len == 1 else None))
            elif cl.kind == 1:
                row.append(("bool", bool(cl.v.i)))
            elif cl.kind in (4, 5):
                row.append((k, cl.v.d))
            elif cl.kind == 6:
                o = cl.v.str_off
                row.append(("str", strings[o:o + cl.str_len].decode("utf-8", "surrogateescape")))
            else:
                row.append((k, cl.v.i))
        out.append(tuple(row))
    return out


@dataclass
class GoResult:
    ok: bool
    error: str
    code: int
    col_types: List[int]
    rows: List[tuple]
    src: np.ndarray = None
    dst: np.ndarray = None
    rank: np.ndarray = None
    etype: np.ndarray = None
    hop_frontier: List[int] = field(default_factory=list)
    hop_edges: List[int] = field(default_factory=list)
    hop_next: List[int] = field(default_factory=list)
    hop_xchg: List[int] = field(default_factory=list)     # world > 1: frontier bytes sent per hop
    device_ms: float = 0.0
    nrows: int = 0
    # on_device + fetch: the HBM result copied back as arrays (x, len or None, type or None) per column
    dev_cols: List[tuple] = field(default_factory=list)
    # on_device: ([src, dst, rank] widths, per-column widths) in bytes; 8 unless compact
    dev_widths: Optional[tuple] = None
    dev_consts: Optional[tuple] = None       # (key values, column values) of width-0 (constant) columns
    digests: object = None               # columnar + digest_fn: whatever digest_fn returned
    device_digest: Optional[tuple] = None  # on_device + device_digest: (sum, xor, rows) of the row hashes
    host_prep_ms: float = 0.0            # library host time before the first launch / after the device
    host_tail_ms: float = 0.0


@dataclass
class NeighborsResult:
    code: int
    failed_codes: List[Tuple[int, int]]
    total_edges: int
    edge_vertex: np.ndarray
    edge_type: np.ndarray
    edge_dst: np.ndarray
    edge_cells: List[tuple]
    vertex_cells: List[tuple]
    vertex_has_tag: np.ndarray
    # encode_rows: the QueryResponse payload (RowWriter rows, schemas)
    edge_props: Optional[List[bytes]] = None           # IdAndProp.props per returned edge
    edge_schema: Optional[dict] = None                 # signed type -> [(name, type)]
    vertex_schema: Optional[dict] = None               # tag id -> [(name, type)]
    tag_rows: Optional[List[Tuple[int, int, bytes]]] = None   # (request vid index, tag id, TagData.data)
    latency_in_us: int = 0                             # ResponseCommon.latency_in_us


def _arr(ptr, n, dtype):
    if n == 0 or not ptr:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dtype, copy=True)


# ----------------------------------------------------------------------------- engine
class PreparedGo:
    """A GO sentence encoded once for ngx_go (ngx_go_plan and the arrays it points into); reusable across
    calls while the sentence object it came from is not changed (Engine.prepare_go)."""

    def __init__(self, plan, keep):
        self.plan = plan
        self._keep = keep


class Engine:
    def __init__(self, device: int = 0, rank: int = 0, world: int = 1, nccl_id: Optional[bytes] = None,
                 exchange=None):
        """world > 1: one shard per rank over RCCL (nccl_id from unique_id() on rank 0), or over a host
        collective `exchange` (dist_exchange()) when the ranks share a GPU."""
        self.L = lib()
        self._uid = ctypes.create_string_buffer(nccl_id, 128) if nccl_id else None
        self._xchg = exchange                      # keep the ctypes callback alive with the context
        cfg = Config(device, rank, world, ctypes.cast(self._uid, ctypes.c_void_p) if self._uid else None,
                     ctypes.cast(exchange, ctypes.c_void_p) if exchange else None, None)
        h = ctypes.c_void_p()
        rc = self.L.ngx_open(ctypes.byref(cfg), ctypes.byref(h))
        if rc:
            raise EngineError(rc, "ngx_open failed (no HIP device or RCCL init failed)")
        self.h = h
        self.rank, self.world = rank, world

    def close(self):
        if getattr(self, "h", None):
            self.L.ngx_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc: int, what: str):
        if rc:
            raise EngineError(rc, f"{what}: {self.L.ngx_last_error(self.h).decode()}")

    # ---- schema + data
    def add_space(self, space: int, num_parts: int):
        self._check(self.L.ngx_add_space(self.h, space, num_parts), "add_space")

    def add_schema(self, space, is_edge, sid, name, fields: Sequence[Tuple[str, int]], ver=0, ttl_col="", ttl_dur=0):
        names = (ctypes.c_char_p * max(1, len(fields)))(*[f[0].encode() for f in fields])
        types = (c_i32 * max(1, len(fields)))(*[f[1] for f in fields])
        self._check(self.L.ngx_add_schema(self.h, space, 1 if is_edge else 0, sid, name.encode(), ver, len(fields),
                                          names, types, ttl_col.encode(), ttl_dur), "add_schema")

    def load_kv(self, space: int, keys, koff, vals, voff):
        keys, vals = np.ascontiguousarray(keys, dtype=np.uint8), np.ascontiguousarray(vals, dtype=np.uint8)
        koff, voff = np.ascontiguousarray(koff, dtype=np.uint64), np.ascontiguousarray(voff, dtype=np.uint64)
        b = KVBatchC(len(koff) - 1, keys.ctypes.data, koff.ctypes.data, vals.ctypes.data, voff.ctypes.data)
        self._check(self.L.ngx_load_kv(self.h, space, ctypes.byref(b)), "load_kv")

    def load_csr(self, space: int, vpart, vid, slots):
        """ngx_load_csr: this shard's vertex table (sorted by (part, vid)) and per slot (etype, off, dst,
        [column arrays of the latest schema's fields]) as int64 / uint64 arrays (datagen.Csr.slots)."""
        vpart = np.ascontiguousarray(vpart, dtype=np.int32)
        vid = np.ascontiguousarray(vid, dtype=np.int64)
        keep = [vpart, vid]
        cs = (CsrSlotC * max(1, len(slots)))()
        for k, (etype, off, dst, cols) in enumerate(slots):
            off = np.ascontiguousarray(off, dtype=np.uint64)
            dst = np.ascontiguousarray(dst, dtype=np.int64)
            cols = [np.ascontiguousarray(c, dtype=np.int64) for c in cols]
            ptrs = (ctypes.c_void_p * max(1, len(cols)))(*[c.ctypes.data for c in cols])
            keep += [off, dst, cols, ptrs]
            cs[k] = CsrSlotC(int(etype), off.ctypes.data, dst.ctypes.data, None, len(cols),
                             ctypes.cast(ptrs, ctypes.c_void_p))
        sh = CsrShardC(len(vid), vpart.ctypes.data, vid.ctypes.data, len(slots), cs)
        self._check(self.L.ngx_load_csr(self.h, space, ctypes.byref(sh)), "load_csr")
        del keep

    def load_batch(self, space: int, batch):
        self.load_kv(space, *batch.arrays())

    def load_snapshot_rows(self, space: int, rows: bytes):
        """Stage a part's snapshot stream: encodeKV records (kvfmt.encode_kv), as SnapshotManagerImpl
        streams them (src/kvstore/SnapshotManagerImpl.cpp:15-53)."""
        buf = ctypes.create_string_buffer(bytes(rows), len(rows)) if rows else None
        self._check(self.L.ngx_load_snapshot_rows(self.h, space, buf, len(rows)), "load_snapshot_rows")

    def save_snapshot(self, space: int, path: str, tag: str = ""):
        self._check(self.L.ngx_save_snapshot(self.h, space, path.encode(), tag.encode()), "save_snapshot")

    def open_snapshot(self, space: int, path: str) -> str:
        """Load a device snapshot file saved by save_snapshot; returns its checkpoint tag."""
        tag = ctypes.create_string_buffer(64)
        self._check(self.L.ngx_open_snapshot(self.h, space, path.encode(), tag), "open_snapshot")
        return tag.value.decode()

    def commit(self, space: int):
        self._check(self.L.ngx_commit(self.h, space), "commit")

    def info(self, space: int) -> GraphInfo:
        gi = GraphInfo()
        self._check(self.L.ngx_graph_info_get(self.h, space, ctypes.byref(gi)), "graph_info")
        return gi

    # ---- GetNeighbors
    def get_neighbors(self, space, parts: Sequence[Tuple[int, Sequence[int]]], edge_types: Optional[Sequence[int]],
                      return_columns: Sequence[Tuple[int, int, str]], filter_bytes: bytes = b"",
                      max_edges_per_vertex: int = 2**31 - 1, now_sec: int = 0,
                      encode_rows: bool = False, decode: bool = True) -> NeighborsResult:
        """decode=False: counts and failed codes only (no Python cells; the bench's latency loop)."""
        pid = np.array([p for p, _ in parts], dtype=np.int32)
        nv = np.array([len(v) for _, v in parts], dtype=np.uint32)
        vids = np.array([x for _, v in parts for x in v], dtype=np.int64)
        et = np.array(list(edge_types or []), dtype=np.int32)
        cols = (PropDef * max(1, len(return_columns)))(*[PropDef(o, i, n.encode()) for o, i, n in return_columns])
        req = GnRequest(space, len(parts), pid.ctypes.data_as(P(c_i32)), nv.ctypes.data_as(P(c_u32)),
                        vids.ctypes.data_as(P(c_i64)), len(et), et.ctypes.data_as(P(c_i32)), filter_bytes,
                        len(filter_bytes), len(return_columns), cols, max_edges_per_vertex, now_sec,
                        1 if encode_rows else 0)
        out = P(GnResult)()
        rc = self.L.ngx_get_neighbors(self.h, ctypes.byref(req), ctypes.byref(out))
        try:
            r = out.contents
            if rc and rc not in (NGX_OK,) and r.nfailed == 0:
                raise EngineError(rc, self.L.ngx_last_error(self.h).decode())
            failed = [(r.failed_codes[2 * i], r.failed_codes[2 * i + 1]) for i in range(r.nfailed)]
            if not decode:
                return NeighborsResult(code=r.code, failed_codes=failed, total_edges=r.nedges, edge_vertex=None,
                                       edge_type=None, edge_dst=None, edge_cells=[], vertex_cells=[],
                                       vertex_has_tag=None, latency_in_us=r.latency_in_us)
            strings = ctypes.string_at(r.strings, r.strings_len) if r.strings_len else b""
            nc = r.ncols
            enc = {}
            if encode_rows:
                off = _arr(r.edge_props_off, r.nedges + 1, np.uint64)
                blob = ctypes.string_at(r.edge_props, int(off[-1])) if r.nedges and off[-1] else b""
                enc["edge_props"] = [blob[int(off[i]):int(off[i + 1])] for i in range(r.nedges)]
                es, vs = {}, {}
                for k in range(r.nschemas):
                    sd = r.schemas[k]
                    cols_ = [(sd.names[j].decode(), sd.types[j]) for j in range(sd.ncols)]
                    (es if sd.is_edge else vs)[sd.id] = cols_
                enc["edge_schema"], enc["vertex_schema"] = es, vs
                toff = _arr(r.tag_props_off, r.ntag_rows + 1, np.uint64)
                tblob = ctypes.string_at(r.tag_props, int(toff[-1])) if r.ntag_rows and toff[-1] else b""
                enc["tag_rows"] = [(int(r.tag_row_vertex[k]), int(r.tag_row_tag[k]), tblob[int(toff[k]):int(toff[k + 1])])
                                   for k in range(r.ntag_rows)]
            return NeighborsResult(
                code=r.code, failed_codes=failed, total_edges=r.nedges,
                edge_vertex=_arr(r.edge_vertex, r.nedges, np.uint32), edge_type=_arr(r.edge_type, r.nedges, np.int32),
                edge_dst=_arr(r.edge_dst, r.nedges, np.int64),
                edge_cells=_cells(r.edge_cells, r.nedges, nc, strings),
                vertex_cells=_cells(r.vertex_cells, r.nvertices, nc, strings),
                vertex_has_tag=_arr(r.vertex_has_tag, r.nvertices * nc, np.uint8),
                latency_in_us=r.latency_in_us, **enc)
        finally:
            self.L.ngx_gn_result_free(out)

    # ---- GO
    def go(self, space: int, s: Union[str, ngql.GoSentence], pushdown: bool = True, now_sec: int = 0,
           raise_on_error: bool = False, rows: bool = True, on_device: bool = False, fetch: bool = False,
           columnar: bool = False, digest_fn=None, arrays: bool = True, input=None,
           yield_only: bool = False, compact: bool = False, device_digest: bool = False) -> GoResult:
        """Run one GO. rows=False skips decoding cells into Python tuples; on_device=True leaves the
        result rows in HBM (GoResult.nrows and the statistics only); with fetch=True the HBM arrays
        (src/dst/rank/type and the columnar YIELD columns) are copied back into the result.
        columnar=True asks for host_columnar results: no cells; with rows=True they are rebuilt here
        from the columns (ColumnValue typing by col_types) so they compare with the cell path.
        digest_fn(col_types, nrows, x_ptrs, len_ptrs, type_ptrs) is called on the host columns
        before the result is freed (tests: large-result comparison). FROM $-.col / $var.col reads
        `input' (a nebula_amd.pipeline.Interim; None: no input, no rows). yield_only (with on_device):
        only the YIELD columns are materialised; src / dst / rank arrays only where a column aliases them.
        device_digest (with on_device): GoResult.device_digest = (sum, xor, rows) of the row hashes, computed
        on the device (ngx_go_result_digest; oracle.row_digest restates it).
        compact (with on_device): integer result arrays at the widths of the stored columns they copy
        (ngx_go_plan.compact_results); fetch widens them back to int64 (GoResult.dev_widths keeps them)."""
        if isinstance(s, PreparedGo):                       # its own pushdown / result-placement flags
            plan, keep = s.plan, s
            on_device, columnar = bool(plan.result_on_device), bool(plan.host_columnar)
        else:
            if isinstance(s, str):
                s = ngql.parse_go(s)
            keep = self.prepare_go(space, s, pushdown=pushdown, now_sec=now_sec, on_device=on_device,
                                   columnar=columnar, yield_only=yield_only, input=input, compact=compact)
            plan = keep.plan
        out = P(GoResultC)()
        rc = self.L.ngx_go(self.h, ctypes.byref(plan), ctypes.byref(out))
        try:
            r = out.contents
            err = self.L.ngx_last_error(self.h).decode() if rc else ""
            if rc and (raise_on_error or rc in (E_DEVICE, E_UNSUPPORTED)):
                raise EngineError(rc, err)
            strings = ctypes.string_at(r.strings, r.strings_len) if r.strings_len else b""
            n = r.nrows
            if on_device:
                # pointer slices (one C loop each) rather than an element access per index: this path
                # runs once per bench step
                nh, nc = r.nhops, r.ncols
                xb = r.hop_exchange_bytes
                res = GoResult(ok=rc == 0, error=err, code=rc, col_types=r.col_types[:nc] if nc else [],
                               rows=[], nrows=n, host_prep_ms=r.host_prep_ms, host_tail_ms=r.host_tail_ms,
                               hop_frontier=r.hop_frontier[:nh] if nh else [],
                               hop_edges=r.hop_edges[:nh] if nh else [],
                               hop_next=r.hop_next[:nh] if nh else [],
                               hop_xchg=xb[:nh] if xb and nh else [],
                               device_ms=r.device_ms)
                if rc == 0 and r.dev_col_w:
                    # width 0: a constant column (value in dev_key_const / dev_col_const, no array)
                    res.dev_widths = (r.dev_key_w[:3], r.dev_col_w[:nc] if nc else [])
                    res.dev_consts = (r.dev_key_const[:3], r.dev_col_const[:nc] if nc and r.dev_col_const else [0] * nc)
                if device_digest and rc == 0:
                    d3 = (c_u64 * 3)()
                    drc = self.L.ngx_go_result_digest(self.h, out, d3)
                    if drc:
                        raise EngineError(drc, self.L.ngx_last_error(self.h).decode())
                    res.device_digest = (int(d3[0]), int(d3[1]), int(d3[2]))
                if fetch and rc == 0:
                    kw = res.dev_widths[0] if res.dev_widths else [8, 8, 8]
                    cw = res.dev_widths[1] if res.dev_widths else [8] * r.ncols
                    kc, cc = res.dev_consts if res.dev_widths else ([0, 0, 0], [0] * r.ncols)

                    def key(ptr, k):
                        if kw[k] == 0:
                            return np.full(n, kc[k], np.int64)
                        return self._d2h_int(ptr, n, kw[k]) if ptr else None
                    res.src = key(r.dev_src, 0)
                    res.dst = key(r.dev_dst, 1)
                    res.rank = key(r.dev_rank, 2)
                    res.etype = (self._d2h(r.dev_type, n, np.int32) if r.dev_type
                                 else np.full(n, r.dev_type_const, np.int32))   # one OVER type: no column
                    cols = ctypes.cast(r.dev_cols, P(DevColumn)) if r.dev_cols else None
                    for c in range(r.ncols):
                        dc = cols[c]
                        res.dev_cols.append((np.full(n, cc[c], np.int64) if cw[c] == 0 else self._d2h_int(dc.x, n, cw[c]),
                                             self._d2h(dc.len, n, np.uint32) if dc.len else None,
                                             self._d2h(dc.type, n, np.uint8) if dc.type else None))
                return res
            if columnar:
                if not arrays:                             # delivery only (bench): no Python copies
                    return GoResult(ok=rc == 0, error=err, code=rc, col_types=[r.col_types[i] for i in range(r.ncols)],
                                    rows=[], nrows=r.nrows, hop_edges=[r.hop_edges[i] for i in range(r.nhops)],
                                    device_ms=r.device_ms, host_prep_ms=r.host_prep_ms, host_tail_ms=r.host_tail_ms)
                return self._columnar(r, rc, err, rows, digest_fn)
            res = GoResult(
                ok=rc == 0, error=err, code=rc, col_types=[r.col_types[i] for i in range(r.ncols)],
                rows=_cells(r.cells, n, r.ncols, strings) if rows else [],
                src=_arr(r.row_src, n, np.int64), dst=_arr(r.row_dst, n, np.int64),
                rank=_arr(r.row_rank, n, np.int64), etype=_arr(r.row_type, n, np.int32),
                hop_frontier=[r.hop_frontier[i] for i in range(r.nhops)],
                hop_edges=[r.hop_edges[i] for i in range(r.nhops)],
                hop_next=[r.hop_next[i] for i in range(r.nhops)],
                               hop_xchg=[r.hop_exchange_bytes[i] for i in range(r.nhops)] if r.hop_exchange_bytes else [],
                               device_ms=r.device_ms, nrows=n)
            return res
        finally:
            self.L.ngx_go_result_free(out)

    def go_batch(self, prepared: Sequence["PreparedGo"], digests: bool = False):
        """Run prepared GO plans back to back in one native call (ngx_go_batch): per query (code, result
        rows, edges scanned over all hops), plus with `digests` the device-resident result's digest
        (sum, xor, count as ngx_go_result_digest; zeros for a failed query)."""
        n = len(prepared)
        arr = (ctypes.POINTER(GoPlan) * max(n, 1))(*[ctypes.pointer(p.plan) for p in prepared])
        codes, rows, edges = (c_i32 * max(n, 1))(), (c_u64 * max(n, 1))(), (c_u64 * max(n, 1))()
        dg = (c_u64 * max(3 * n, 1))() if digests else None
        rc = self.L.ngx_go_batch(self.h, ctypes.cast(arr, ctypes.c_void_p), n, codes, rows, edges, dg)
        if rc != 0 and all(codes[i] == 0 for i in range(n)):
            raise EngineError(rc, "go_batch: " + self.L.ngx_last_error(self.h).decode())
        out = [(int(codes[i]), int(rows[i]), int(edges[i])) for i in range(n)]
        if digests:
            out = [o + ((int(dg[3 * i]), int(dg[3 * i + 1]), int(dg[3 * i + 2])),) for i, o in enumerate(out)]
        return out

    def prepare_go(self, space: int, s, pushdown: bool = True, now_sec: int = 0, on_device: bool = False,
                   columnar: bool = False, yield_only: bool = False, input=None, compact: bool = False) -> PreparedGo:
        """Encode a GO sentence (expressions in Expression::encode bytes, vids as int64) into the C plan
        once; go() accepts the result in place of the sentence (the bench's timed loop)."""
        if isinstance(s, str):
            s = ngql.parse_go(s)
        starts = np.array(s.vids, dtype=np.int64)
        names = (ctypes.c_char_p * max(1, len(s.over)))(*[n.encode() for n, _ in s.over])
        aliases = (ctypes.c_char_p * max(1, len(s.over)))(*[(a or "").encode() for _, a in s.over])
        where = s.where.encode() if s.where is not None else b""
        yb = [y.expr.encode() for y in s.yields]
        yarr = (ctypes.c_char_p * max(1, len(yb)))(*yb)
        ylen = (c_u32 * max(1, len(yb)))(*[len(y) for y in yb])
        plan = GoPlan(space, s.record_from, s.record_to, len(starts), starts.ctypes.data_as(P(c_i64)), len(s.over),
                      names, aliases, 1 if s.over_all else 0, s.direction, where if where else None, len(where),
                      len(yb), yarr, ylen, 1 if s.distinct else 0, 1 if pushdown else 0, now_sec,
                      1 if on_device else 0, 1 if columnar else 0)
        plan.yield_only = 1 if yield_only else 0
        plan.compact_results = 1 if compact else 0
        keep = [starts, names, aliases, where, yb, yarr, ylen]
        if s.from_type:
            from .pipeline import Interim
            inp = _input_arrays(input if input is not None else Interim([]))
            names_a, types_a, cells_a, strings_a, nc, nr = inp
            fcol = s.from_col.encode()
            fvar = s.from_var.encode() if s.from_type == 2 else None
            plan.input_vid_col = fcol
            plan.input_var = fvar
            plan.input_ncols, plan.input_nrows = nc, nr
            plan.input_names, plan.input_types, plan.input_cells = names_a, types_a, cells_a
            plan.input_strings = strings_a
            keep += [inp, fcol, fvar]
        return PreparedGo(plan, keep)

    def _columnar(self, r, rc, err, rows, digest_fn=None):
        n = r.nrows
        types = [r.col_types[i] for i in range(r.ncols)]
        res = GoResult(ok=rc == 0, error=err, code=rc, col_types=types, rows=[], nrows=n,
                       hop_frontier=[r.hop_frontier[i] for i in range(r.nhops)],
                       hop_edges=[r.hop_edges[i] for i in range(r.nhops)],
                       hop_next=[r.hop_next[i] for i in range(r.nhops)],
                               hop_xchg=[r.hop_exchange_bytes[i] for i in range(r.nhops)] if r.hop_exchange_bytes else [],
                               device_ms=r.device_ms)
        if rc != 0:
            return res
        res.src, res.dst, res.rank = _arr(r.row_src, n, np.int64), _arr(r.row_dst, n, np.int64), \
            _arr(r.row_rank, n, np.int64)
        res.etype = _arr(r.row_type, n, np.int32) if r.row_type else np.full(n, r.dev_type_const, np.int32)
        cols = ctypes.cast(r.host_cols, P(DevColumn)) if r.host_cols else None
        if digest_fn is not None:
            res.digests = digest_fn(types, n, [cols[c].x for c in range(r.ncols)],
                                    [cols[c].len for c in range(r.ncols)], [cols[c].type for c in range(r.ncols)])
            if not rows:
                return res
        for c in range(r.ncols):
            dc = cols[c]
            x = _arr(ctypes.cast(dc.x, P(c_i64)), n, np.int64)
            ln = _arr(ctypes.cast(dc.len, P(c_u32)), n, np.uint32) if dc.len else None
            t = _arr(ctypes.cast(dc.type, P(ctypes.c_uint8)), n, np.uint8) if dc.type else None
            res.dev_cols.append((x, ln, t))
        if rows:
            static = {1: 3, 2: 1, 3: 1, 21: 1, 4: 2, 5: 2, 6: 4}         # SupportedType -> V_* of its rows
            kinds = {1: "bool", 2: "int", 3: "id", 21: "timestamp", 4: "float", 5: "double", 6: "str"}
            out = []
            for i in range(n):
                row = []
                for c, (x, ln, t) in enumerate(res.dev_cols):
                    vt = int(t[i]) if t is not None else static.get(types[c], 0)
                    v = int(x[i])
                    if vt == 4:
                        row.append(("str", ctypes.string_at(v, int(ln[i])).decode("utf-8", "surrogateescape")
                                    if ln[i] else ""))
                    elif vt == 2:
                        row.append((kinds.get(types[c], "double"), float(np.int64(v).view(np.float64))))
                    elif vt == 3:
                        row.append(("bool", bool(v)) if types[c] == 1 else ("empty", bool(v)))
                    elif vt == 1:
                        row.append((kinds.get(types[c], "int"), v))
                    else:
                        row.append(("empty", None))
                out.append(tuple(row))
            res.rows = out
        return res

    def _d2h(self, ptr, n, dtype):
        out = np.zeros(n, dtype=dtype)
        if n and ptr:
            self._check(self.L.ngx_device_to_host(self.h, out.ctypes.data, ptr, out.nbytes), "device_to_host")
        return out

    def _d2h_int(self, ptr, n, width):
        """A device array of n signed integers at `width` bytes each, widened to int64."""
        dt = {1: np.int8, 2: np.int16, 4: np.int32}.get(int(width), np.int64)
        return self._d2h(ptr, n, dt).astype(np.int64, copy=False)

    # ---- flags
    def set_flag(self, name: str, value: int):
        self._check(self.L.ngx_set_flag(self.h, name.encode(), int(value)), "set_flag")

    def get_flag(self, name: str) -> int:
        v = c_i64()
        self._check(self.L.ngx_get_flag(self.h, name.encode(), ctypes.byref(v)), "get_flag")
        return v.value

    def jit_note(self) -> str:
        return self.L.ngx_jit_note(self.h).decode()

    # ---- measurement
    def set_profiling(self, on: bool):
        self._check(self.L.ngx_set_profiling(self.h, 1 if on else 0), "set_profiling")

    def stats(self) -> Dict[str, int]:
        """Service counters (storage_get_bound_qps / _error_qps / _latency_us_*), as ngx_stats names them."""
        p = P(Stat)()
        n = c_i32()
        self._check(self.L.ngx_stats(self.h, ctypes.byref(p), ctypes.byref(n)), "stats")
        return {p[i].name.decode(): p[i].value for i in range(n.value)}

    def kernel_stats(self) -> Dict[str, Tuple[int, float, int]]:
        p = P(KernelStat)()
        n = c_i32()
        self._check(self.L.ngx_kernel_stats(self.h, ctypes.byref(p), ctypes.byref(n)), "kernel_stats")
        return {p[i].name.decode(): (p[i].launches, p[i].total_ms, p[i].algo_bytes) for i in range(n.value)}


def build_info() -> dict:
    """ngx_build_info() parsed, plus whether its source digest matches the sources in this tree."""
    import hashlib
    import glob
    raw = lib().ngx_build_info().decode()
    info = dict(kv.split("=", 1) for kv in raw.replace(" built=", " built=").split(" ") if "=" in kv)
    csrc = os.path.join(HERE, "csrc")
    srcs = sorted(glob.glob(os.path.join(csrc, "*.cpp")) + glob.glob(os.path.join(csrc, "*.h")) +
                  glob.glob(os.path.join(csrc, "*.hip")) +
                  [os.path.join(csrc, "../../include/nebula_gn.h"), os.path.join(csrc, "exports.map"),
                   os.path.join(csrc, "Makefile")], key=lambda p: os.path.relpath(p, csrc))
    h = hashlib.sha256()
    for p in srcs:
        with open(p, "rb") as f:
            h.update(f.read())
    info["tree_sha"] = h.hexdigest()[:16]
    info["matches_tree"] = info.get("src_sha") == info["tree_sha"]
    info["raw"] = raw
    return info


def hash_string(s: str) -> int:
    b = s.encode()
    return lib().ngx_hash_string(b, len(b))
