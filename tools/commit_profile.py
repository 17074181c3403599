"""Where the C2 snapshot build's time goes (What's weak #9): bench.py's load path — RMAT rows
in the reference KV format (datagen.rmat), ngx_load_kv, ngx_commit — with the commit's phases timed by
the library (NGX_HOST_TRACE=1: export, tables, destinations, upload, mirrors), beside the columnar load
(datagen.rmat_csr + ngx_load_csr + ngx_commit) of the same graph.

Usage (GPU box): NGX_HOST_TRACE=1 python tools/commit_profile.py [scale] 2> commit_trace.txt
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    from nebula_amd import datagen, engine
    out = {"scale": scale, "threads": int(os.environ.get("OMP_NUM_THREADS", "16"))}
    t = time.time()
    rows = datagen.rmat(scale, 16, 42, 100, with_in=True, with_tag=False, threads=16)
    out["generate_kv_s"] = time.time() - t
    out["kv_rows"] = rows.n
    e = engine.Engine(0)
    e.add_space(datagen.RMAT_SPACE, 100)
    for is_edge, sid, name, fields in datagen.rmat_schemas():
        e.add_schema(datagen.RMAT_SPACE, is_edge, sid, name, fields)
    t = time.time()
    e.load_kv(datagen.RMAT_SPACE, *rows.arrays())
    out["load_kv_s"] = time.time() - t
    rows.free()
    t = time.time()
    e.commit(datagen.RMAT_SPACE)
    out["commit_kv_s"] = time.time() - t
    e.close()
    t = time.time()
    c = datagen.rmat_csr(scale, 16, 42, 100, with_in=True, threads=16)
    out["generate_csr_s"] = time.time() - t
    e = engine.Engine(0)
    e.add_space(datagen.RMAT_SPACE, 100)
    for is_edge, sid, name, fields in datagen.rmat_schemas():
        e.add_schema(datagen.RMAT_SPACE, is_edge, sid, name, fields)
    t = time.time()
    e.load_csr(datagen.RMAT_SPACE, c.vpart, c.vid, c.slots)
    out["load_csr_s"] = time.time() - t
    c.free()
    t = time.time()
    e.commit(datagen.RMAT_SPACE)
    out["commit_csr_s"] = time.time() - t
    e.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
