"""Host timeline of one GetNeighbors request (bench.py's: 1000 RMAT seeds by part, _dst/p0/p1, filter
e.p0 < 50): NGX_HOST_TRACE=1 prints the library's marks; the Python call is timed around them."""
import os
import sys
import time

os.environ["NGX_HOST_TRACE"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nebula_amd import datagen, engine, ngql  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 20
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from tests import fixtures  # noqa: E402
ds = fixtures.RmatDataset(scale, threads=16)
e = engine.Engine(0)
e.set_flag("jit_async", 0)
ds.load_engine(e)
seeds = [int(v) for v in datagen.rmat_seeds(scale, 1000, 16, 42, 42, threads=16)]
by = {}
for v in seeds:
    by.setdefault(v % 100 + 1, []).append(v)
parts = sorted(by.items())
cols = [(engine.EDGE, 1, "_dst"), (engine.EDGE, 1, "p0"), (engine.EDGE, 1, "p1")]
filt = ngql.Binary(ngql.K_REL, ngql.REL_OPS["<"], ngql.Prop(ngql.K_ALIAS, "", "e", "p0"), ngql.Prim(50)).encode()
for i in range(8):
    t = time.perf_counter()
    r = e.get_neighbors(datagen.RMAT_SPACE, parts, [1], cols, filt, decode=False)
    print("python call %.1f us, %d edges" % ((time.perf_counter() - t) * 1e6, r.total_edges), file=sys.stderr, flush=True)
