"""One rank of the C3 rehearsal (scripts/c3_rehearsal.sh starts WORLD of these on one GPU).

BASELINE C3 is `GO 3 STEPS … WHERE e.p0 < 50` from 1000 seeds on RMAT scale 26 over 8 GPUs. The
8-GPU run uses RCCL; this rehearsal runs the same engine path with every rank on device 0 and the
frontier exchange over the host collective (gloo, ngx_config.exchange), at the C3 graph size, and
checks the result through properties that hold at any size (no oracle at this size):

  * per hop, the scanned edges summed over the shards equal Σ out-degree of that hop's frontier,
    computed independently from the generator's rows with numpy (a host BFS over the distinct
    (src, dst) pairs each shard generated, frontiers all-gathered over gloo);
  * without WHERE every scanned edge of the last hop is a row;
  * `WHERE e.p0 < 50` and `WHERE e.p0 >= 50` partition those rows.

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
    with_in = (sys.argv[6] if len(sys.argv) > 6 else "out") == "in"
    pull_factor = int(sys.argv[7]) if len(sys.argv) > 7 else -1
    import numpy as np
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=1800))
    from nebula_amd import datagen, engine, ngql

    threads = max(1, int(os.environ.get("OMP_NUM_THREADS", "16")) // world)
    t0 = time.time()
    rows = datagen.rmat(scale, 16, 42, 100, with_in, False, rank=rank, world=world, threads=threads)
    log(rank, f"generated {rows.n} rows in {time.time() - t0:.1f}s")
    # the distinct out-edges (src, dst) of this shard, independent of the engine (keys: item(4) src(8)
    # type(4) rank(8) dst(8) version(8); every generated key is an edge key here)
    keys, ko, _, _ = rows.arrays()
    k = keys[:int(ko[-1])].reshape(-1, 40)
    etype = k[:, 12:16].copy().view(np.int32).ravel()
    src_le = k[:, 4:12].copy().view("<i8").ravel()            # vids as the exporter reads them (native LE)
    dst_le = k[:, 24:32].copy().view("<i8").ravel()
    outm = etype == (datagen.RMAT_EDGE | 0x40000000)           # kvfmt.edge_key: the type carries the edge bit
    pairs = np.unique((src_le[outm].astype(np.uint64) << np.uint64(32)) | dst_le[outm].astype(np.uint64))
    del k, etype, src_le, dst_le, outm
    psrc = (pairs >> np.uint64(32)).astype(np.int64)
    pdst = (pairs & np.uint64(0xFFFFFFFF)).astype(np.int64)
    del pairs
    log(rank, f"{len(psrc)} distinct out-edges")

    e = engine.Engine(0, rank, world, exchange=engine.dist_exchange())
    if pull_factor >= 0:
        e.set_flag("pull_factor", pull_factor)
    e.add_space(datagen.RMAT_SPACE, 100)
    for is_edge, sid, name, fields in datagen.rmat_schemas():
        e.add_schema(datagen.RMAT_SPACE, is_edge, sid, name, fields)
    t0 = time.time()
    e.load_kv(datagen.RMAT_SPACE, *rows.arrays())
    rows.free()
    t1 = time.time()
    e.commit(datagen.RMAT_SPACE)
    info = e.info(datagen.RMAT_SPACE)
    log(rank, f"load {t1 - t0:.1f}s commit {time.time() - t1:.1f}s: {info.vertices} vertices, {info.edges} edges, "
              f"{info.device_bytes / 2**30:.2f} GiB")

    seeds = datagen.rmat_seeds(scale, 1000, 16, 42, 42, threads=threads)
    S = ", ".join(str(int(v)) for v in seeds)
    res = {"rank": rank, "load_s": t1 - t0, "vertices": info.vertices, "edges": info.edges,
           "device_gib": info.device_bytes / 2**30}
    for name, w in (("lt", " WHERE e.p0 < 50"), ("ge", " WHERE e.p0 >= 50"), ("all", "")):
        pulls = e.get_flag("pull_hops")
        t = time.time()
        r = e.go(datagen.RMAT_SPACE, ngql.parse_go(QUERY.replace("{S}", S).replace("{W}", w)), on_device=True)
        res[name] = {"ok": r.ok, "error": r.error, "nrows": r.nrows, "hop_edges": list(r.hop_edges),
                     "hop_xchg": list(r.hop_xchg), "pull_hops": e.get_flag("pull_hops") - pulls,
                     "ms": (time.time() - t) * 1e3}
        log(rank, name, res[name])
    e.close()

    # host BFS over the generator's edges: hop h scans Σ out-degree of F_h; F_{h+1} = their dsts
    frontier = np.sort(seeds.astype(np.int64))       # hop 1 scans a repeated seed again (no dedup)
    order = np.argsort(psrc, kind="stable")
    psrc, pdst = psrc[order], pdst[order]
    bfs = []
    for h in range(3):
        lo = np.searchsorted(psrc, frontier, "left")
        hi = np.searchsorted(psrc, frontier, "right")
        bfs.append(int((hi - lo).sum()))
        if h == 2:
            break
        lens = hi - lo
        nz = lens > 0
        lo, lens = lo[nz], lens[nz]
        idx = np.repeat(lo - np.concatenate(([0], np.cumsum(lens)[:-1])), lens) + np.arange(int(lens.sum()))
        mine = np.unique(pdst[idx])
        parts = [None] * world
        dist.all_gather_object(parts, mine)
        frontier = np.unique(np.concatenate(parts))
        log(rank, f"host BFS hop {h + 1}: {bfs[-1]} edges, next frontier {len(frontier)}")
    res["bfs_hop_edges"] = bfs
    with open(out, "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
