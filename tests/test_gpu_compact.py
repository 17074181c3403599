"""Compact device results (ngx_go_plan.compact_results) against the 8-byte device results and the oracle.

With compact_results the final hop writes the src / dst / rank row arrays and every YIELD column that
copies one stored integer column (of the only OVER type, present in every row) at the width the
snapshot stores that column at; every other column stays 8 bytes. Widened back to int64 the rows
must equal the 8-byte result's rows value for value (sorted: GO rows land in chunk order), on the
generated kernels and on the interpreter, over M TO N record hops, several OVER types, tag and
computed columns, and the queries whose compact flag is ignored (DISTINCT) — and the rows must be the
oracle's (the reference path, GoExecutor.cpp:1082-1335: the integers a row carries, whatever bytes
hold them in HBM).
"""
import numpy as np
import pytest

from nebula_amd import datagen, engine, ngql
from oracle import oracle
from tests import fixtures

pytestmark = pytest.mark.gpu

QUERIES = [
    # (query, expected key widths, expected column widths); None: not checked. Every rank of the RMAT
    # graph is 0, so the rank is a constant column (width 0, ngx_go_result.dev_key_const): no bytes
    ("GO 3 STEPS FROM {S} OVER e WHERE e.p0 < 50 YIELD e._dst, e._rank, e.p0, e.p1",
     [2, 2, 0], [2, 0, 1, 8]),
    ("GO 1 TO 3 STEPS FROM {S} OVER e WHERE e.p0 % 7 == 1 YIELD e._src, e._dst, e.p0, e.p0 + 1, e.p1 % 1000",
     [2, 2, 0], [2, 2, 1, 8, 8]),
    ("GO 2 STEPS FROM {S} OVER e REVERSELY YIELD e._dst, e.p1, e.p0, $^.vt.v0, $^.vt.name",
     [2, 2, 0], [2, 8, 1, 8, 8]),
    ("GO 2 STEPS FROM {S} OVER e BIDIRECT WHERE e.p0 > 80 YIELD e._dst, e.p0, e._rank",
     [2, 2, 0], [2, 8, 0]),                 # two slots: aliased keys compact, e.p0 at 8 bytes
    ("GO 2 STEPS FROM {S} OVER e YIELD DISTINCT e._dst, e.p0",
     [8, 8, 8], [8, 8]),
    ("GO 3 STEPS FROM {S} OVER e WHERE $$.vt.v0 > 10 YIELD e.p0, $$.vt.v0, e._dst",
     [2, 2, 0], [1, 8, 2]),
]


@pytest.fixture(scope="module")
def rmat12():
    ds = fixtures.RmatDataset(12, with_in=True, with_tag=True)
    o = oracle.Oracle()
    o.set_flags(threads=8)
    ds.load_oracle(o)
    e = engine.Engine(0)
    ds.load_engine(e)
    yield ds, o, e
    e.close()
    o.close()


def _digests(r):
    cols = [np.ascontiguousarray(x) for x, _, _ in r.dev_cols]
    lens = [ln.ctypes.data if ln is not None else None for _, ln, _ in r.dev_cols]
    types = [t.ctypes.data if t is not None else None for _, _, t in r.dev_cols]
    return oracle.digest_columns(r.col_types, r.nrows, [c.ctypes.data for c in cols], lens, types)


@pytest.mark.parametrize("jit", [1, 0])
@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_compact_equals_wide(rmat12, qi, jit):
    ds, o, e = rmat12
    q, key_w, col_w = QUERIES[qi]
    seeds = datagen.sample_vids(700 + qi, 1 << ds.scale, 40)
    s = ngql.parse_go(q.replace("{S}", ", ".join(str(int(v)) for v in seeds)))
    e.set_flag("jit", jit)
    try:
        wide = e.go(ds.space, s, on_device=True, fetch=True)
        comp = e.go(ds.space, s, on_device=True, fetch=True, compact=True)
    finally:
        e.set_flag("jit", 1)
    assert wide.ok and comp.ok, (wide.error, comp.error)
    assert wide.dev_widths == ([8, 8, 8], [8] * len(wide.col_types))
    assert comp.nrows == wide.nrows > 0 and comp.hop_edges == wide.hop_edges
    if key_w is not None:
        assert comp.dev_widths[0] == key_w
    if col_w is not None:
        assert comp.dev_widths[1] == col_w
    if comp.dev_widths[0][2] == 0:                  # a constant rank: its value, and no array behind it
        assert comp.dev_consts[0][2] == 0
    # rows land in chunk completion order (final_kernels.h, !ORDERED): compare the sorted rows over the
    # row arrays and every column without per-row lengths / types (strings are pointers into arenas)
    def table(r):
        arrs = []
        # DISTINCT keeps one row of each group, whichever wins the device hash: only its YIELD values match
        for name in (() if s.distinct else ("src", "dst", "rank", "etype")):
            a = getattr(r, name)
            if a is not None:
                arrs.append(a)
        arrs += [x for x, ln, t in r.dev_cols if ln is None and t is None]
        m = np.stack(arrs, axis=1)
        return m[np.lexsort(m.T[::-1])]
    for name in ("src", "dst", "rank"):
        assert (getattr(wide, name) is None) == (getattr(comp, name) is None), name
    for (x8, l8, t8), (xc, lc, tc) in zip(wide.dev_cols, comp.dev_cols):
        assert (l8 is None) == (lc is None) and (t8 is None) == (tc is None)
    assert np.array_equal(table(wide), table(comp))
    if not s.distinct:
        # the compact rows are the oracle's rows (string columns compare through their digests)
        ref = o.go(ds.space, s, digest=True)
        assert ref.ok and ref.nrows == comp.nrows
        if all(t is None and ln is None for _, ln, t in comp.dev_cols):
            assert np.array_equal(_digests(comp), ref.digests)
