"""Attribution of the C2 final hop's HBM bytes by result column (What's weak #3).

Runs the bench query's hop structure with different YIELD lists over the same 1000 seeds — each a
device-resident, compact, YIELD-only result like bench.py's timed step — `--reps` times each, in a fixed
order, so that one rocprofv3 --pmc pass per counter set gives every variant's final-hop bytes
(tools/wprobe_summary.py pairs the ngx_jit_final dispatches with the variants in this order):

  all   YIELD e._dst, e._rank, e.p0, e.p1   (the bench's: dst 4 B + p0 1 B + p1 8 B per row)
  dst   YIELD e._dst                        (4 B per row)
  p0    YIELD e.p0                          (1 B per row)
  p1    YIELD e.p1                          (8 B per row)
  none  YIELD e._rank                       (a constant column: no bytes per row)

Usage (GPU box): python tools/wprobe.py [--reps 3] > gpurun_out/wprobe.json
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

VARIANTS = [("all", "e._dst, e._rank, e.p0, e.p1"), ("dst", "e._dst"), ("p0", "e.p0"), ("p1", "e.p1"),
            ("none", "e._rank")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--scale", type=int, default=22)
    ap.add_argument("--flag", action="append", default=[])
    args = ap.parse_args()
    from nebula_amd import datagen, engine, ngql
    t0 = time.time()
    c = datagen.rmat_csr(args.scale, 16, 42, 100, with_in=True, threads=16)
    eng = engine.Engine(0)
    for f in args.flag:
        n, _, v = f.partition("=")
        eng.set_flag(n, int(v))
    eng.add_space(datagen.RMAT_SPACE, 100)
    for is_edge, sid, name, fields in datagen.rmat_schemas():
        eng.add_schema(datagen.RMAT_SPACE, is_edge, sid, name, fields)
    eng.load_csr(datagen.RMAT_SPACE, c.vpart, c.vid, c.slots)
    eng.commit(datagen.RMAT_SPACE)
    c.free()
    print(f"[wprobe] loaded in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    seeds = datagen.rmat_seeds(args.scale, 1000, 16, 42, 42, threads=16)
    sl = ", ".join(str(int(v)) for v in seeds)
    out = {"order": [], "variants": {}}
    preps = {}
    for name, ys in VARIANTS:
        s = ngql.parse_go(f"GO 3 STEPS FROM {sl} OVER e WHERE e.p0 < 50 YIELD {ys}")
        preps[name] = eng.prepare_go(datagen.RMAT_SPACE, s, on_device=True, yield_only=True, compact=True)
        r = eng.go(datagen.RMAT_SPACE, preps[name], rows=False)      # JIT compile outside the probed order
        assert r.ok, r.error
    for name, _ in VARIANTS:
        for _ in range(args.reps):
            r = eng.go(datagen.RMAT_SPACE, preps[name], rows=False)
            assert r.ok, r.error
            out["order"].append(name)
            out["variants"][name] = {"rows": r.nrows, "final_edges": r.hop_edges[-1],
                                     "widths": list(r.dev_widths[1]) if getattr(r, "dev_widths", None) else None}
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
