"""Print where the bench query's result columns live (GPU box): the dst row array and each YIELD
column's device pointer and width, to check that e._dst / e._rank alias the row arrays (no second
store per row). python tools/probe_alias.py [scale]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    from nebula_amd import datagen, engine, ngql
    from tests import fixtures
    ds = fixtures.RmatDataset(scale, with_in=True)
    with engine.Engine(0) as e:
        ds.load_engine(e)
        seeds = datagen.rmat_seeds(scale, 100, 16, 42, 1)
        s = ngql.parse_go("GO 3 STEPS FROM " + ", ".join(str(int(v)) for v in seeds) +
                          " OVER e WHERE e.p0 < 50 YIELD e._dst, e._rank, e.p0, e.p1")
        for yo in (True, False):
            prep = e.prepare_go(ds.space, s, on_device=True, compact=True, yield_only=yo)
            out = ctypes.POINTER(engine.GoResultC)()
            rc = e.L.ngx_go(e.h, ctypes.byref(prep.plan), ctypes.byref(out))
            r = out.contents
            cols = ctypes.cast(r.dev_cols, ctypes.POINTER(engine.DevColumn))
            print(f"yield_only={yo} rc={rc} rows={r.nrows} src={r.dev_src} dst={r.dev_dst} rank={r.dev_rank} "
                  f"key_w={list(r.dev_key_w[:3])} col_w={list(r.dev_col_w[:r.ncols])}")
            for c in range(r.ncols):
                print(f"  col {c}: x={cols[c].x} len={cols[c].len} t={cols[c].type}")
            e.L.ngx_go_result_free(out)


if __name__ == "__main__":
    main()
