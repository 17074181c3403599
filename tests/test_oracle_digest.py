"""The order-independent row digest (oracle/orc_digest.cpp) that pins C3's 1 G result rows by value
(tests/test_gpu_c3.py): hop_digest over a CSR equals row_digest over the same rows listed explicitly,
equals a pure-Python restatement of the hash, is independent of row order, and splits additively over
the p0 filters (CPU only)."""
import numpy as np

from oracle import oracle

M = (1 << 64) - 1


def _mix(z):
    z = ((z ^ (z >> 30)) * 0xbf58476d1ce4e5b9) & M
    z = ((z ^ (z >> 27)) * 0x94d049bb133111eb) & M
    return z ^ (z >> 31)


def _py_digest(rows):
    s = x = 0
    for r in rows:
        h = 0x9E3779B97F4A7C15
        for v in r:
            h = _mix(h ^ (int(v) & M))
        s, x = (s + h) & M, x ^ h
    return (s, x, len(rows))


def test_hop_digest_matches_rows():
    rng = np.random.default_rng(5)
    nv = 300
    deg = rng.integers(0, 9, nv)
    off = np.concatenate(([0], np.cumsum(deg))).astype(np.uint64)
    ne = int(off[-1])
    vid = rng.integers(-(1 << 40), 1 << 40, nv)
    dst = rng.integers(-(1 << 62), 1 << 62, ne)
    p0 = rng.integers(0, 100, ne).astype(np.int8)
    p1 = rng.integers(-(1 << 63), (1 << 63) - 1, ne, dtype=np.int64)
    rows = rng.choice(nv, 120, replace=False)
    got = oracle.hop_digest(rows, vid, off, dst, p0, p1, rank=0, threads=3)
    tuples = [(vid[r], dst[e], 0, p0[e], p1[e]) for r in rows for e in range(int(off[r]), int(off[r + 1]))]
    assert got["all"] == _py_digest(tuples)
    lt = [t for t in tuples if t[3] < 50]
    ge = [t for t in tuples if t[3] >= 50]
    assert got["lt"] == _py_digest(lt) and got["ge"] == _py_digest(ge)
    assert (got["lt"][0] + got["ge"][0]) & M == got["all"][0] and got["lt"][1] ^ got["ge"][1] == got["all"][1]
    cols = [np.array([t[k] for t in tuples], dtype=np.int64) for k in range(5)]
    assert oracle.row_digest(cols) == got["all"]
    perm = rng.permutation(len(tuples))
    assert oracle.row_digest([c[perm] for c in cols]) == got["all"]
    # one changed value changes the digest
    cols[4][7] ^= 1
    assert oracle.row_digest(cols) != got["all"]
