"""Synthetic graphs in the reference KV format (ctypes over libngx_datagen.so, csrc/datagen.cpp).

`Rows` owns the generated key/value arrays; `arrays()` hands zero-copy numpy views to
Engine.load_kv / Oracle.put_kv. Graph shapes follow BASELINE.json configs C2-C5.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libngx_datagen.so")

# RMAT space layout used by bench.py and the RMAT parity tests
RMAT_SPACE, RMAT_EDGE, RMAT_TAG = 1, 1, 10
RMAT_EDGE_NAME, RMAT_TAG_NAME = "e", "vt"
RMAT_EDGE_FIELDS = [("p0", 2), ("p1", 2)]
RMAT_TAG_FIELDS = [("v0", 2), ("name", 6)]
GRAPH500 = (0.57, 0.19, 0.19)


class _Rows(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint64), ("keys", ctypes.c_void_p), ("key_off", ctypes.c_void_p),
                ("vals", ctypes.c_void_p), ("val_off", ctypes.c_void_p)]


class _Csr(ctypes.Structure):
    _fields_ = [("nv", ctypes.c_uint64), ("vpart", ctypes.c_void_p), ("vid", ctypes.c_void_p), ("nslots", ctypes.c_int32),
                ("etype", ctypes.c_int32 * 2), ("ne", ctypes.c_uint64 * 2), ("off", ctypes.c_void_p * 2),
                ("dst", ctypes.c_void_p * 2), ("p0", ctypes.c_void_p * 2), ("p1", ctypes.c_void_p * 2)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing; build with `make -C nebula_amd/csrc`")
        L = ctypes.CDLL(LIB_PATH)
        i32, i64, u64, dbl = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double
        R = ctypes.POINTER(_Rows)
        L.ngd_rmat.argtypes = [i32, i32, dbl, dbl, dbl, u64, i32, i32, i32, i32, i32, i32, i32, i32, R]
        L.ngd_rmat.restype = i32
        L.ngd_powerlaw.argtypes = [i64, i32, dbl, i32, i64, u64, i32, i32, i32, i32, i32, R]
        L.ngd_powerlaw.restype = i32
        L.ngd_snb.argtypes = [i64, i32, i64, i32, u64, i32, i32, i32, i32, i32, i32, i32, i32, i32, R]
        L.ngd_snb.restype = i32
        L.ngd_free.argtypes = [R]
        L.ngd_sample_vids.argtypes = [u64, u64, u64, ctypes.c_void_p]
        L.ngd_rmat_seeds.argtypes = [i32, i32, dbl, dbl, dbl, u64, u64, u64, i32, ctypes.c_void_p]
        L.ngd_rmat_seeds.restype = i32
        C_ = ctypes.POINTER(_Csr)
        L.ngd_rmat_csr.argtypes = [i32, i32, dbl, dbl, dbl, u64, i32, i32, i32, i32, i32, i32, C_]
        L.ngd_rmat_csr.restype = i32
        L.ngd_csr_free.argtypes = [C_]
        L.ngd_rmat_csr_sample.argtypes = [i32, i32, dbl, dbl, dbl, u64, i32, i32, i32, i32, i32, i32, ctypes.c_char_p]
        L.ngd_rmat_csr_sample.restype = i32
        L.ngd_rmat_csr_build.argtypes = [i32, u64, i32, i32, i32, i32, i32, i32, i32, ctypes.c_char_p, C_]
        L.ngd_rmat_csr_build.restype = i32
        _lib = L
    return _lib


class Rows:
    def __init__(self):
        self.r = _Rows()

    @property
    def n(self) -> int:
        return self.r.n

    def arrays(self):
        n = self.r.n
        ko = np.ctypeslib.as_array(ctypes.cast(self.r.key_off, ctypes.POINTER(ctypes.c_uint64)), shape=(n + 1,))
        vo = np.ctypeslib.as_array(ctypes.cast(self.r.val_off, ctypes.POINTER(ctypes.c_uint64)), shape=(n + 1,))
        kb, vb = int(ko[-1]), int(vo[-1])
        keys = np.ctypeslib.as_array(ctypes.cast(self.r.keys, ctypes.POINTER(ctypes.c_uint8)), shape=(max(kb, 1),))
        vals = np.ctypeslib.as_array(ctypes.cast(self.r.vals, ctypes.POINTER(ctypes.c_uint8)), shape=(max(vb, 1),))
        return keys, ko, vals, vo

    def free(self):
        if self.r.keys:
            lib().ngd_free(ctypes.byref(self.r))

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def _threads(threads):
    return threads or min(16, os.cpu_count() or 1)


def rmat(scale: int, ef: int = 16, seed: int = 42, num_parts: int = 100, with_in: bool = False,
         with_tag: bool = False, rank: int = 0, world: int = 1, threads: int = 0, abc=GRAPH500) -> Rows:
    r = Rows()
    rc = lib().ngd_rmat(scale, ef, abc[0], abc[1], abc[2], seed, num_parts, RMAT_EDGE, int(with_in), int(with_tag),
                        RMAT_TAG, rank, world, _threads(threads), ctypes.byref(r.r))
    if rc:
        raise ValueError("bad rmat parameters")
    return r


class Csr:
    """One shard of the RMAT graph as CSR arrays (ngd_rmat_csr): `vpart`/`vid` (the vertex table sorted by
    (part, vid)) and per slot `slots[s] = (etype, off, dst, [p0, p1])` as zero-copy numpy views; the
    input of Engine.load_csr (ngx_load_csr)."""

    def __init__(self):
        self.c = _Csr()

    def _view(self, ptr, n, ct, dt):
        return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ct)), shape=(max(n, 1),))[:n].view(dt)

    @property
    def nv(self) -> int:
        return self.c.nv

    @property
    def vpart(self):
        return self._view(self.c.vpart, self.c.nv, ctypes.c_int32, np.int32)

    @property
    def vid(self):
        return self._view(self.c.vid, self.c.nv, ctypes.c_int64, np.int64)

    @property
    def slots(self):
        out = []
        for s in range(self.c.nslots):
            ne = self.c.ne[s]
            out.append((self.c.etype[s], self._view(self.c.off[s], self.c.nv + 1, ctypes.c_uint64, np.uint64),
                        self._view(self.c.dst[s], ne, ctypes.c_int64, np.int64),
                        [self._view(self.c.p0[s], ne, ctypes.c_int64, np.int64),
                         self._view(self.c.p1[s], ne, ctypes.c_int64, np.int64)]))
        return out

    def free(self):
        if self.c.vid:
            lib().ngd_csr_free(ctypes.byref(self.c))

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def rmat_csr(scale: int, ef: int = 16, seed: int = 42, num_parts: int = 100, with_in: bool = False,
             rank: int = 0, world: int = 1, threads: int = 0, abc=GRAPH500) -> Csr:
    """The graph of rmat() (same edges, props; no tags) as this shard's CSR, without KV rows."""
    c = Csr()
    rc = lib().ngd_rmat_csr(scale, ef, abc[0], abc[1], abc[2], seed, num_parts, RMAT_EDGE, int(with_in), rank, world,
                            _threads(threads), ctypes.byref(c.c))
    if rc:
        raise ValueError("bad rmat_csr parameters")
    return c


def rmat_csr_sample(scale: int, prefix: str, producer: int, producers: int, world: int, ef: int = 16, seed: int = 42,
                    num_parts: int = 100, with_in: bool = False, threads: int = 0, abc=GRAPH500):
    """Producer `producer` of `producers` samples its share of the rmat() edge stream and writes every
    shard's keys to files under `prefix` (then all producers meet; then rmat_csr_build per shard)."""
    rc = lib().ngd_rmat_csr_sample(scale, ef, abc[0], abc[1], abc[2], seed, num_parts, int(with_in), world, producer,
                                   producers, _threads(threads), prefix.encode())
    if rc:
        raise ValueError(f"rmat_csr_sample failed ({rc})")


def rmat_csr_build(scale: int, prefix: str, rank: int, world: int, producers: int, seed: int = 42,
                   num_parts: int = 100, with_in: bool = False, threads: int = 0) -> Csr:
    """This shard's CSR from every producer's files (removed as read): equal to rmat_csr(…, rank, world)."""
    c = Csr()
    rc = lib().ngd_rmat_csr_build(scale, seed, num_parts, RMAT_EDGE, int(with_in), rank, world, producers,
                                  _threads(threads), prefix.encode(), ctypes.byref(c.c))
    if rc:
        raise ValueError(f"rmat_csr_build failed ({rc})")
    return c


def powerlaw(n: int, ef: int = 8, alpha: float = 2.0, nsuper: int = 4, superdeg: int = 1_000_000, seed: int = 42,
             num_parts: int = 100, etype: int = 1, rank: int = 0, world: int = 1, threads: int = 0) -> Rows:
    r = Rows()
    rc = lib().ngd_powerlaw(n, ef, alpha, nsuper, superdeg, seed, num_parts, etype, rank, world, _threads(threads),
                            ctypes.byref(r.r))
    if rc:
        raise ValueError("bad powerlaw parameters")
    return r


@dataclass
class SnbIds:
    person: int = 21
    post: int = 22
    knows: int = 31
    likes: int = 32
    has_creator: int = 33


def snb(np_: int, knows_deg: int = 20, nposts: int = 0, likes_deg: int = 10, seed: int = 42, num_parts: int = 100,
        ids: SnbIds = SnbIds(), rank: int = 0, world: int = 1, threads: int = 0) -> Rows:
    r = Rows()
    nposts = nposts or 2 * np_
    rc = lib().ngd_snb(np_, knows_deg, nposts, likes_deg, seed, num_parts, ids.person, ids.post, ids.knows, ids.likes,
                       ids.has_creator, rank, world, _threads(threads), ctypes.byref(r.r))
    if rc:
        raise ValueError("bad snb parameters")
    return r


def sample_vids(seed: int, rng: int, k: int) -> np.ndarray:
    out = np.zeros(k, dtype=np.int64)
    lib().ngd_sample_vids(seed, rng, k, out.ctypes.data)
    return out


def rmat_seeds(scale: int, k: int, ef: int = 16, seed: int = 42, sample_seed: int = 42, threads: int = 0,
               abc=GRAPH500) -> np.ndarray:
    """k vids sampled uniformly from the RMAT vertices that have out-edges."""
    out = np.zeros(k, dtype=np.int64)
    rc = lib().ngd_rmat_seeds(scale, ef, abc[0], abc[1], abc[2], seed, sample_seed, k, _threads(threads),
                              out.ctypes.data)
    if rc:
        raise ValueError("could not sample seeds")
    return out


def rmat_schemas(with_tag: bool = False):
    """(is_edge, id, name, fields) of the RMAT space."""
    s = [(True, RMAT_EDGE, RMAT_EDGE_NAME, RMAT_EDGE_FIELDS)]
    if with_tag:
        s.append((False, RMAT_TAG, RMAT_TAG_NAME, RMAT_TAG_FIELDS))
    return s


# power-law space (C4): one edge type with an INT and a DOUBLE prop, no tags
PL_SPACE, PL_EDGE, PL_EDGE_NAME = 2, 1, "pl"
PL_EDGE_FIELDS = [("w", 2), ("score", 5)]


def powerlaw_schemas():
    return [(True, PL_EDGE, PL_EDGE_NAME, PL_EDGE_FIELDS)]


# LDBC-SNB-like space (C5)
SNB_SPACE = 3


def snb_schemas(ids: SnbIds = SnbIds()):
    """(is_edge, id, name, fields) of the SNB-like space, field order as ngd_snb writes the rows."""
    return [
        (False, ids.person, "person", [("firstName", 6), ("age", 2), ("gender", 6)]),
        (False, ids.post, "post", [("content", 6), ("length", 2), ("lang", 6)]),
        (True, ids.knows, "knows", [("creationDate", 2), ("weight", 5)]),
        (True, ids.likes, "likes", [("creationDate", 2)]),
        (True, ids.has_creator, "hasCreator", [("creationDate", 2)]),
    ]
