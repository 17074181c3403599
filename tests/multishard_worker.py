"""One shard of a world-N GO run (tests/test_multishard.py starts N of these as child processes).

The rank materialises only its own parts (datagen's sharded generator; ngx_load_kv would drop the
others anyway: part % world == rank, Nebula's pickHosts placement, CreateSpaceProcessor.cpp:107-120),
ngx_commit all-gathers the vertex tables, and each hop's frontier marks are exchanged through
`engine.dist_exchange()` (gloo) — the host collective of ngx_config.exchange — so N shards can share
one GPU. Per query the rank writes its status, per-hop scanned edges and exchange bytes as JSON and
its rows as sorted 128-bit digests (oracle.digest_columns, the test checker) in a .npy file; the
parent merges them as graphd merges storage responses.

Usage: python tests/multishard_worker.py RANK WORLD PORT OUT.json SCALE QUERIES.json [jit|vm] [full|plain|csr]
       [snap:DIR | snapmix:DIR]
(full: in-edges + tag `vt`, the multi-shard parity graph; plain: out-edges only; csr: in-edges, no tag,
bulk-loaded with ngx_load_csr from datagen.rmat_csr instead of KV rows)
"""
import datetime
import json
import os
import sys
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rank, world, port = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    out, scale, qfile = sys.argv[4], int(sys.argv[5]), sys.argv[6]
    mode = sys.argv[7] if len(sys.argv) > 7 else "jit"
    layout = sys.argv[8] if len(sys.argv) > 8 else "full"
    full = layout == "full"
    csr = layout == "csr"
    import numpy as np
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=300))
    from nebula_amd import datagen, engine, ngql, pipeline
    from oracle import oracle

    queries = json.load(open(qfile))
    snap = sys.argv[9] if len(sys.argv) > 9 else ""

    def fresh():
        x = engine.Engine(0, rank, world, exchange=engine.dist_exchange())
        x.set_flag("jit", 1 if mode == "jit" else 0)
        x.add_space(datagen.RMAT_SPACE, 100)
        for is_edge, sid, name, fields in datagen.rmat_schemas(full):
            x.add_schema(datagen.RMAT_SPACE, is_edge, sid, name, fields)
        return x

    def committed(seed):
        x = fresh()
        if csr:                                          # in-edges, no tags, bulk-loaded (ngx_load_csr)
            c = datagen.rmat_csr(scale, 16, seed, 100, True, rank=rank, world=world, threads=4)
            x.load_csr(datagen.RMAT_SPACE, c.vpart, c.vid, c.slots)
            c.free()
        else:
            rows = datagen.rmat(scale, 16, seed, 100, full, full, rank=rank, world=world, threads=4)
            x.load_kv(datagen.RMAT_SPACE, *rows.arrays())
            rows.free()
        x.commit(datagen.RMAT_SPACE)
        return x

    t0 = time.time()
    e = committed(42)
    print(f"[rank {rank}] committed in {(time.time() - t0) * 1e3:.0f} ms", file=sys.stderr, flush=True)
    if snap:
        # snap:DIR  every shard saves its snapshot, and a fresh context per shard opens it (collective:
        #           the shards check they hold snapshots of one commit); the queries run on those
        # snapmix:DIR  shard 1 opens a snapshot of another commit: every shard's open must fail
        kind, d = snap.split(":", 1)
        e.save_snapshot(datagen.RMAT_SPACE, os.path.join(d, f"a{rank}.snap"), "a")
        e.close()
        if kind == "snapmix":
            other = committed(43)
            other.save_snapshot(datagen.RMAT_SPACE, os.path.join(d, f"b{rank}.snap"), "b")
            other.close()
        e = fresh()
        path = os.path.join(d, f"{'b' if kind == 'snapmix' and rank == 1 else 'a'}{rank}.snap")
        try:
            e.open_snapshot(datagen.RMAT_SPACE, path)
            opened = ""
        except engine.EngineError as x:
            opened = str(x)
        if kind == "snapmix":
            with open(out, "w") as f:
                json.dump({"open_error": opened}, f)
            e.close()
            dist.barrier()
            dist.destroy_process_group()
            return
        assert not opened, opened
    res = []
    default_pf = e.get_flag("pull_factor")

    class Sharded:
        """graphd over the shards: every shard runs the sentence on the whole input (multi-root walks
        exchange root sets per hop), the responses are concatenated in rank order (GoExecutor merges
        storage responses, GoExecutor.cpp:580-606) and DISTINCT applies to the merged rows."""

        def go(self, space, s, **kw):
            r = e.go(space, s, **kw)
            mine = (r.ok, r.error, list(r.col_types) if r.ok else [], [tuple(x) for x in r.rows] if r.ok else [])
            parts = [None] * world
            dist.all_gather_object(parts, mine)
            bad = [p for p in parts if not p[0]]
            rows = [x for p in parts for x in p[3]]
            if s.distinct:
                seen, uniq = set(), []
                for x in rows:
                    if x not in seen:
                        seen.add(x)
                        uniq.append(x)
                rows = uniq
            return types.SimpleNamespace(ok=not bad, error=bad[0][1] if bad else "", rows=rows,
                                         col_types=next((p[2] for p in parts if p[3]), parts[0][2]))

    for i, q in enumerate(queries):
        if q.get("batch"):
            # ngx_go_batch over prepared device-resident plans (compact YIELD columns): each plan alone
            # (ngx_go + device digest) and then all of them pipelined, on every shard
            e.set_flag("pull_factor", q.get("pull_factor", default_pf))
            e.set_flag("xchg_lists", q.get("xchg_lists", -1))
            e.set_flag("dst_props", q.get("dst_props", -1))
            e.set_flag("dense_world_dev", q.get("dense_world_dev", 1))
            preps = [e.prepare_go(datagen.RMAT_SPACE, ngql.parse_go(t), on_device=True, compact=True, yield_only=True)
                     for t in q["batch"]]
            alone = []
            for p in preps:
                r = e.go(datagen.RMAT_SPACE, p, rows=False, device_digest=True)
                alone.append([r.code, r.nrows, int(sum(r.hop_edges)) if r.ok else 0,
                              list(r.device_digest) if r.ok else [0, 0, 0]])
            ov = e.get_flag("batch_overlaps")
            t0 = time.time()
            got = e.go_batch(preps, digests=True)
            print(f"[rank {rank}] batch {i}: {len(preps)} plans in {(time.time() - t0) * 1e3:.0f} ms",
                  file=sys.stderr, flush=True)
            np.save(f"{out}.{i}.npy", np.zeros((0, 2), np.uint64))
            res.append({"batch": True, "alone": alone, "got": [[g[0], g[1], g[2], list(g[3])] for g in got],
                        "overlaps": e.get_flag("batch_overlaps") - ov})
            continue
        if q.get("pipe"):
            walks = e.get_flag("pipe_walks")
            t0 = time.time()
            o = pipeline.run(Sharded(), datagen.RMAT_SPACE, q["text"])
            print(f"[rank {rank}] pipe {i}: {(time.time() - t0) * 1e3:.0f} ms", file=sys.stderr, flush=True)
            np.save(f"{out}.{i}.npy", np.zeros((0, 2), np.uint64))
            res.append({"ok": o.ok, "error": o.error, "rows": [list(map(list, x)) for x in o.rows],
                        "pipe_walks": e.get_flag("pipe_walks") - walks})
            continue
        pf = q.get("pull_factor", default_pf)
        e.set_flag("pull_factor", pf[rank] if isinstance(pf, list) else pf)     # a list: per rank
        e.set_flag("xchg_lists", q.get("xchg_lists", -1))
        e.set_flag("dst_props", q.get("dst_props", -1))
        e.set_flag("dense_world_dev", q.get("dense_world_dev", 1))
        pulls = e.get_flag("pull_hops")
        lists = e.get_flag("xchg_list_hops")
        fetches = e.get_flag("dst_fetches")
        denses = e.get_flag("dense_finals")
        r = e.go(datagen.RMAT_SPACE, ngql.parse_go(q["text"]), pushdown=q.get("pushdown", True), columnar=True,
                 rows=False, digest_fn=oracle.digest_columns)
        np.save(f"{out}.{i}.npy", r.digests if r.ok else np.zeros((0, 2), np.uint64))
        res.append({"ok": r.ok, "error": r.error, "col_types": list(r.col_types) if r.ok else [], "nrows": r.nrows,
                    "hop_edges": list(r.hop_edges), "hop_xchg": list(r.hop_xchg),
                    "jit_failed": e.get_flag("jit_failed"), "pull_hops": e.get_flag("pull_hops") - pulls,
                    "list_hops": e.get_flag("xchg_list_hops") - lists,
                    "dst_fetches": e.get_flag("dst_fetches") - fetches,
                    "dense_finals": e.get_flag("dense_finals") - denses})
    e.close()
    with open(out, "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
