"""ngd_rmat_csr (the C3 test's shard builder) against ngd_rmat's KV rows (the bench's input): the same
shard, built here from the reference-format keys and RowWriter values the way the exporter reads them
(NebulaKeyUtils key layout, RocksDB bytewise order within a (part, src, type) prefix, identical keys
collapsed, the vertex table = every key's source sorted by (part, vid)). CPU only."""
import numpy as np
import pytest

from nebula_amd import datagen


def _varints(buf, off, n):
    out = np.zeros((n, 2), np.int64)
    for i in range(n):
        p = int(off[i]) + 1                              # header byte (RowWriter.cpp:49-75)
        for f in range(2):
            v, sh = 0, 0
            while True:
                b = int(buf[p]); p += 1
                v |= (b & 0x7F) << sh
                sh += 7
                if b < 0x80:
                    break
            out[i, f] = np.int64(np.uint64(v))
    return out


def _from_rows(rows):
    keys, ko, vals, vo = rows.arrays()
    n = rows.n
    assert np.all(np.diff(ko) == 40)
    k = keys[:int(ko[-1])].reshape(n, 40)
    part = k[:, 0:4].copy().view("<i4").ravel() >> 8
    src = k[:, 4:12].copy().view("<i8").ravel()
    t = k[:, 12:16].copy().view("<i4").ravel()
    et = np.where(t > 0, t & ~0x40000000, t)
    rk = k[:, 16:24].copy().view("<i8").ravel()
    dst = k[:, 24:32].copy().view("<i8").ravel()
    assert np.all(rk == 0)
    props = _varints(vals, vo, n)
    # bytewise key order within (part, src, type): rank LE bytes (all 0), then dst LE bytes
    dkey = dst.astype(np.uint64).byteswap()
    order = np.lexsort((dkey, et, src, part))
    part, src, et, dst, props = part[order], src[order], et[order], dst[order], props[order]
    keep = np.ones(n, bool)
    keep[1:] = (part[1:] != part[:-1]) | (src[1:] != src[:-1]) | (et[1:] != et[:-1]) | (dst[1:] != dst[:-1])
    part, src, et, dst, props = part[keep], src[keep], et[keep], dst[keep], props[keep]
    vt = np.unique(np.stack([part.astype(np.int64), src]).T, axis=0)   # sorted by (part, vid)
    slots = {}
    for s in np.unique(et):
        m = et == s
        row = np.searchsorted(vt[:, 0] * (1 << 40) + vt[:, 1], part[m].astype(np.int64) * (1 << 40) + src[m])
        off = np.zeros(len(vt) + 1, np.uint64)
        np.add.at(off, row + 1, 1)
        slots[int(s)] = (np.cumsum(off).astype(np.uint64), dst[m], props[m, 0], props[m, 1])
    return vt, slots


@pytest.mark.parametrize("rank,world,with_in", [(0, 1, True), (1, 3, True), (2, 3, False)])
def test_rmat_csr_equals_kv_rows(rank, world, with_in):
    rows = datagen.rmat(12, 16, 42, 10, with_in, False, rank=rank, world=world, threads=4)
    vt, slots = _from_rows(rows)
    rows.free()
    c = datagen.rmat_csr(12, 16, 42, 10, with_in, rank=rank, world=world, threads=3)
    assert c.nv == len(vt)
    assert np.array_equal(c.vpart, vt[:, 0].astype(np.int32)) and np.array_equal(c.vid, vt[:, 1])
    got = c.slots
    assert sorted(s[0] for s in got) == sorted(slots)
    for etype, off, dst, (p0, p1) in got:
        eoff, edst, ep0, ep1 = slots[etype]
        assert np.array_equal(off, eoff)
        assert np.array_equal(dst, edst)
        assert np.array_equal(p0, ep0) and np.array_equal(p1, ep1)
    c.free()


def test_rmat_csr_split_sampling_equals_one_process(tmp_path):
    """The C3 test's split generation: 3 producers sample a third each and write every shard's keys;
    each of 3 shards builds from the files exactly the shard ngd_rmat_csr builds alone."""
    world = 3
    prefix = str(tmp_path / "k")
    for q in range(world):
        datagen.rmat_csr_sample(11, prefix, q, world, world, num_parts=10, with_in=True, threads=2)
    for r in range(world):
        a = datagen.rmat_csr_build(11, prefix, r, world, world, num_parts=10, with_in=True, threads=2)
        b = datagen.rmat_csr(11, 16, 42, 10, True, rank=r, world=world, threads=2)
        assert a.nv == b.nv and np.array_equal(a.vid, b.vid) and np.array_equal(a.vpart, b.vpart)
        for sa, sb in zip(a.slots, b.slots):
            assert sa[0] == sb[0]
            assert np.array_equal(sa[1], sb[1]) and np.array_equal(sa[2], sb[2])
            assert all(np.array_equal(x, y) for x, y in zip(sa[3], sb[3]))
    assert not list(tmp_path.iterdir())                  # the builders removed every file
