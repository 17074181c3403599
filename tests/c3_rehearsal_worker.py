"""One rank of the C3 run on one GPU (tests/test_gpu_c3.py and scripts/c3_rehearsal.sh start WORLD of
these as child processes on device 0).

BASELINE C3 is `GO 3 STEPS … WHERE e.p0 < 50` from 1000 seeds on RMAT scale 26 (100 parts) over 8 GPUs.
`bench.py --gpus 8` runs it with RCCL; this runs the same engine path with every rank on device 0 and
the frontier exchange over the host collective (gloo, ngx_config.exchange), on C3's graph with the
bench's layout (every out-edge also stored as its in-edge, so pull hops run at world 8 over the
all-gathered frontier bitmap). The shard is bulk-loaded (ngx_load_csr from datagen.rmat_csr: the
graph of datagen.rmat without building 2.1 G KV rows on one box). No oracle holds this size, so the
result is checked through properties that hold at any size:

  * per hop, the scanned edges summed over the shards equal Σ out-degree of that hop's frontier,
    computed independently with numpy from the generator's out-edges (a host BFS, frontiers
    all-gathered over gloo);
  * without WHERE every scanned edge of the last hop is a row;
  * `WHERE e.p0 < 50` and `WHERE e.p0 >= 50` partition those rows;
  * every rank takes the same pull decisions (the parent checks that at least one hop pulled);
  * the rows themselves: an order-independent digest (sum and XOR of a 64-bit hash of every row's
    (src, dst, rank, p0, p1)) of the device result, computed on the device (ngx_go_result_digest), equals
    the digest of the rows the generator's edges give (oracle.hop_digest over the out-edges of the last
    hop's frontier rows, filtered by p0), per filter; the parent compares the sums over the shards.

Usage: python tests/c3_rehearsal_worker.py RANK WORLD PORT OUT.json SCALE [out|in] [pull_factor]
"""
import datetime
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

QUERY = "GO 3 STEPS FROM {S} OVER e{W} YIELD e._dst, e._rank, e.p0, e.p1"


def log(rank, *a):
    print(f"[rank {rank}]", *a, file=sys.stderr, flush=True)


def main():
    rank, world, port, out, scale = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], int(sys.argv[5])
    with_in = (sys.argv[6] if len(sys.argv) > 6 else "in") == "in"
    pull_factor = int(sys.argv[7]) if len(sys.argv) > 7 else -1
    import numpy as np
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=1800))
    from nebula_amd import datagen, engine, ngql
    from oracle import oracle

    threads = max(1, int(os.environ.get("NGX_HOST_THREADS", "2")))
    res = {"rank": rank}
    t0 = time.time()
    # every rank samples 1/world of the edge stream and hands each shard its keys through files in
    # NGX_C3_KEYS (tmpfs), then builds its own shard from them: the generation is not repeated per rank
    prefix = os.path.join(os.environ["NGX_C3_KEYS"], "k")
    datagen.rmat_csr_sample(scale, prefix, rank, world, world, with_in=with_in, threads=threads)
    dist.barrier()
    c = datagen.rmat_csr_build(scale, prefix, rank, world, world, with_in=with_in, threads=threads)
    res["gen_s"] = time.time() - t0
    # the shard's distinct out-edges for the host BFS (independent of the engine): vid -> out-list
    etype, off, dst, props = next(s for s in c.slots if s[0] == datagen.RMAT_EDGE)
    vid = c.vid.copy()
    off = off.copy()
    odst = dst.copy()
    op0 = props[0].astype(np.int8)                   # p0 in 0..99
    op1 = props[1].copy()
    log(rank, f"generated {c.nv} vertex rows, {[len(s[2]) for s in c.slots]} edges per slot in {res['gen_s']:.1f}s")

    e = engine.Engine(0, rank, world, exchange=engine.dist_exchange())
    if pull_factor >= 0:
        e.set_flag("pull_factor", pull_factor)
    e.add_space(datagen.RMAT_SPACE, 100)
    for is_edge, sid, name, fields in datagen.rmat_schemas():
        e.add_schema(datagen.RMAT_SPACE, is_edge, sid, name, fields)
    t0 = time.time()
    e.load_csr(datagen.RMAT_SPACE, c.vpart, c.vid, c.slots)
    c.free()
    t1 = time.time()
    e.commit(datagen.RMAT_SPACE)
    info = e.info(datagen.RMAT_SPACE)
    res.update({"load_s": t1 - t0, "commit_s": time.time() - t1, "vertices": info.vertices, "edges": info.edges,
                "device_gib": info.device_bytes / 2**30})
    log(rank, f"load {t1 - t0:.1f}s commit {res['commit_s']:.1f}s: {info.vertices} vertices, {info.edges} edges, "
              f"{info.device_bytes / 2**30:.2f} GiB")

    seeds = datagen.rmat_seeds(scale, 1000, 16, 42, 42, threads=threads)
    S = ", ".join(str(int(v)) for v in seeds)
    for name, w in (("lt", " WHERE e.p0 < 50"), ("ge", " WHERE e.p0 >= 50"), ("all", "")):
        pulls = e.get_flag("pull_hops")
        t = time.time()
        r = e.go(datagen.RMAT_SPACE, ngql.parse_go(QUERY.replace("{S}", S).replace("{W}", w)), on_device=True,
                 compact=True, device_digest=True)
        res[name] = {"ok": r.ok, "error": r.error, "nrows": r.nrows, "hop_edges": list(r.hop_edges),
                     "hop_xchg": list(r.hop_xchg), "pull_hops": e.get_flag("pull_hops") - pulls,
                     "ms": (time.time() - t) * 1e3,
                     "digest": [str(x) for x in r.device_digest] if r.device_digest else None}
        log(rank, name, res[name])
    e.close()

    # host BFS over the generator's out-edges: hop h scans Σ out-degree of F_h; F_{h+1} = their dsts
    t0 = time.time()
    order = np.argsort(vid, kind="stable")
    svid = vid[order]
    frontier = np.sort(seeds.astype(np.int64))       # hop 1 scans a repeated seed again (no dedup)
    bfs = []
    for h in range(3):
        pos = np.searchsorted(svid, frontier)
        pos = np.minimum(pos, max(len(svid) - 1, 0))
        hit = (svid[pos] == frontier) if len(svid) else np.zeros(len(frontier), bool)
        rows = order[pos[hit]]
        lo, hi = off[rows].astype(np.int64), off[rows + 1].astype(np.int64)
        bfs.append(int((hi - lo).sum()))
        if h == 2:
            # the last hop's rows: every out-edge of this shard's frontier rows, hashed as the device
            # hashes its result rows (src, dst, rank 0, p0, p1), per filter
            dg = oracle.hop_digest(rows, vid, off, odst, op0, op1, 0, threads)
            res["host_digest"] = {k: [str(x) for x in v] for k, v in dg.items()}
            break
        lens = hi - lo
        nz = lens > 0
        lo, lens = lo[nz], lens[nz]
        idx = np.repeat(lo - np.concatenate(([0], np.cumsum(lens)[:-1])), lens) + np.arange(int(lens.sum()))
        mine = np.unique(odst[idx])
        parts = [None] * world
        dist.all_gather_object(parts, mine)
        frontier = np.unique(np.concatenate(parts))
        log(rank, f"host BFS hop {h + 1}: {bfs[-1]} edges, next frontier {len(frontier)}")
    res["bfs_hop_edges"] = bfs
    res["bfs_s"] = time.time() - t0
    with open(out, "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
