"""yield_only (ngx_go_plan): a result_on_device GO writes its YIELD columns and only the row arrays
a YIELD column aliases (e._src / e._dst / e._rank of the OVER type). The columns must equal those of
the full run (which also writes every row array), for the generated and the interpreter kernels."""
import numpy as np
import pytest

from nebula_amd import datagen, engine, ngql
from tests import fixtures

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["jit", "vm"])
def rmat(request):
    ds = fixtures.RmatDataset(12, with_in=True, with_tag=True)
    e = engine.Engine(0)
    e.set_flag("jit", 1 if request.param == "jit" else 0)
    e.set_flag("jit_async", 0)
    ds.load_engine(e)
    yield ds, e
    e.close()


QUERIES = [
    ("GO 3 STEPS FROM {S} OVER e WHERE e.p0 < 50 YIELD e._dst, e._rank, e.p0, e.p1", (False, True, True)),
    ("GO 2 STEPS FROM {S} OVER e YIELD e.p0 * 2, $$.vt.name", (False, False, False)),
    ("GO 1 TO 3 STEPS FROM {S} OVER e REVERSELY YIELD e._src, e.p1", (True, False, False)),
    ("GO 2 STEPS FROM {S} OVER e BIDIRECT WHERE e.p0 > 80 YIELD e._dst, e._type", (False, True, False)),
]


@pytest.mark.parametrize("qi", range(len(QUERIES)))
def test_yield_only_columns_equal(rmat, qi):
    ds, e = rmat
    q, kept = QUERIES[qi]
    seeds = datagen.sample_vids(70 + qi, 1 << ds.scale, 50)
    s = ngql.parse_go(q.replace("{S}", ", ".join(str(int(v)) for v in seeds)))
    full = e.go(ds.space, s, on_device=True, fetch=True)
    lean = e.go(ds.space, s, on_device=True, fetch=True, yield_only=True)
    assert full.ok and lean.ok, (full.error, lean.error)
    assert full.nrows == lean.nrows > 0
    assert (lean.src is not None, lean.dst is not None, lean.rank is not None) == kept
    # final-hop chunks may claim output ranges in any order: compare the rows as sorted tuples of
    # every column (value bits, lengths, types) plus the row arrays the lean run kept
    def table(r):
        cols = []
        for x, ln, t in r.dev_cols:
            cols.append(x)
            if ln is not None:
                cols.append(ln.astype(np.int64))
            if t is not None:
                cols.append(t.astype(np.int64))
        for keep, arr in zip(kept, (r.src, r.dst, r.rank)):
            if keep:
                cols.append(arr)
        m = np.stack(cols, axis=1)
        return m[np.lexsort(m.T[::-1])]
    assert np.array_equal(table(full), table(lean))
