"""Debug: the pull test's failing query in host / dyn modes and several pull factors (GPU)."""
import sys
sys.path.insert(0, ".")
from nebula_amd import datagen, engine, ngql
from oracle import oracle
from tests import fixtures

ds = fixtures.RmatDataset(12, with_in=True, with_tag=True)
o = oracle.Oracle()
o.set_flags(threads=8)
ds.load_oracle(o)
for qi in range(2):
    seeds = datagen.sample_vids(900 + qi, 1 << 12, 30)
    q = "GO 3 STEPS FROM {S} OVER e WHERE e.p0 < 50 YIELD e._dst, e._rank, e.p0, e.p1".replace(
        "{S}", ", ".join(str(int(v)) for v in seeds))
    s = ngql.parse_go(q)
    ref = o.go(ds.space, s)
    print("oracle", ref.hop_scanned, flush=True)
    for dyn in (0, 1):
        e = engine.Engine(0)
        e.set_flag("dyn_hops", dyn)
        ds.load_engine(e)
        for factor in (0, 1, 0, 200, 0, 0):
            e.set_flag("pull_factor", factor)
            got = e.go(ds.space, s)
            print(f"q{qi} dyn={dyn} factor={factor}", got.hop_edges, got.hop_next, "OK" if got.hop_edges == ref.hop_scanned else "BAD", flush=True)
        e.close()
