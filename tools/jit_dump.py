"""Write the hipRTC source of the bench query's final-hop kernel (NGX_JIT_DUMP) for offline ISA study:
python tools/jit_dump.py OUT.hip [scale]. Runs on a GPU box (the engine needs a device)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out = sys.argv[1]
    scale = int(sys.argv[2]) if len(sys.argv) > 2 else 14
    os.environ["NGX_JIT_DUMP"] = out
    from nebula_amd import datagen, engine, ngql
    from tests import fixtures
    ds = fixtures.RmatDataset(scale)
    with engine.Engine(0) as e:
        ds.load_engine(e)
        seeds = datagen.rmat_seeds(scale, 100, 16, 42, 1)
        s = ngql.parse_go("GO 3 STEPS FROM " + ", ".join(str(int(v)) for v in seeds) +
                          " OVER e WHERE e.p0 < 50 YIELD e._dst, e._rank, e.p0, e.p1")
        # the bench's timed plan: compact, YIELD-only device results
        p = e.prepare_go(ds.space, s, on_device=True, yield_only=True, compact=True)
        r = e.go(ds.space, p, rows=False)
        print("ok", r.ok, "jit", e.get_flag("jit_compiled"), e.jit_note(), "dense", e.get_flag("dense_finals"))


if __name__ == "__main__":
    main()
