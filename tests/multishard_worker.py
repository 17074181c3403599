"""One shard of a world-N GO run (tests/test_multishard.py starts N of these as child processes).

Every rank loads the same generated rows; ngx_load_kv keeps the parts with part % world == rank
(Nebula's pickHosts placement, CreateSpaceProcessor.cpp:107-120), ngx_commit all-gathers the vertex
tables, and each hop's frontier marks are exchanged through `engine.dist_exchange()` (gloo) — the
host collective of ngx_config.exchange — so N shards can share one GPU. The rank writes its rows
(normalized cells) and per-hop scanned-edge counts as JSON; the parent merges them as graphd would.

Usage: python tests/multishard_worker.py RANK WORLD PORT OUT.json SCALE QUERIES.json [jit|vm]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rank, world, port = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    out, scale, qfile = sys.argv[4], int(sys.argv[5]), sys.argv[6]
    mode = sys.argv[7] if len(sys.argv) > 7 else "jit"
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    from nebula_amd import engine, ngql
    from tests import fixtures

    queries = json.load(open(qfile))
    ds = fixtures.RmatDataset(scale, with_in=True, with_tag=True)
    e = engine.Engine(0, rank, world, exchange=engine.dist_exchange())
    e.set_flag("jit", 1 if mode == "jit" else 0)
    ds.load_engine(e)
    res = []
    for q in queries:
        r = e.go(ds.space, ngql.parse_go(q["text"]), pushdown=q.get("pushdown", True))
        res.append({"ok": r.ok, "error": r.error, "col_types": list(r.col_types) if r.ok else [],
                    "rows": [list(t) for t in fixtures.normalize_cells(r.rows)] if r.ok else [],
                    "hop_edges": list(r.hop_edges), "jit_failed": e.get_flag("jit_failed")})
    e.close()
    with open(out, "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
