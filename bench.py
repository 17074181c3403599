"""Benchmark: traversed edges/sec of `GO 3 STEPS FROM <1k vids> OVER e WHERE e.p0 < 50 YIELD e._dst,
e._rank, e.p0, e.p1` on an RMAT graph (BASELINE.json configs[1]: scale 22, edge factor 16, 100 parts;
weak scaling: scale 22 + log2(N) over N GPUs, parts hashed to GPUs as part % N).

One step = one GO query through libnebula_gn (seeds on host -> result rows and cells on host),
with a fresh 1k-seed sample per step. Traversed edges = sum over hops of the edges scanned
(SURVEY.md §8d). The JSON line also carries the HBM roofline of the dominant kernel (HIP events on
the engine stream) and a CPU baseline (the oracle restatement on a bounded sample, rank 0, N=1).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]; N > 1 under torch.distributed.run.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md)
METRIC = "traversed edges/sec for GO 3 STEPS WHERE on RMAT; % HBM roofline"
QUERY = "GO 3 STEPS FROM {S} OVER e WHERE e.p0 < 50 YIELD e._dst, e._rank, e.p0, e.p1"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--scale", type=int, default=0, help="RMAT scale (default 22 + log2(N))")
    p.add_argument("--ef", type=int, default=16)
    p.add_argument("--seeds", type=int, default=1000)
    p.add_argument("--parts", type=int, default=100)
    p.add_argument("--cpu-budget", type=float, default=10.0, help="target seconds of oracle work (0: skip)")
    p.add_argument("--threads", type=int, default=16, help="host threads for datagen / oracle")
    p.add_argument("--host-exchange", action="store_true",
                   help="rehearsal of the N > 1 path on one GPU: every rank on device 0, frontier exchange "
                        "through the host collective (gloo) instead of RCCL")
    p.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"),
                   help="PMC-derived HBM bytes per launch of the dominant kernel (from profiles/)")
    return p.parse_args()


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    scale = args.scale or 22 + int(round(math.log2(world)))

    import numpy as np
    import torch
    import torch.distributed as dist
    from nebula_amd import datagen, engine, ngql

    device = 0 if args.host_exchange else local
    torch.cuda.set_device(device)
    uid, xchg = None, None
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        if args.host_exchange:
            xchg = engine.dist_exchange()
        else:
            obj = [engine.unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            uid = obj[0]

    t0 = time.time()
    rows = datagen.rmat(scale, args.ef, 42, args.parts, with_in=False, with_tag=False, rank=rank, world=world,
                        threads=args.threads)
    log(f"[rank {rank}] generated {rows.n} rows of RMAT scale {scale} in {time.time() - t0:.1f}s")
    eng = engine.Engine(device, rank, world, uid, exchange=xchg)
    eng.add_space(datagen.RMAT_SPACE, args.parts)
    for is_edge, sid, name, fields in datagen.rmat_schemas():
        eng.add_schema(datagen.RMAT_SPACE, is_edge, sid, name, fields)
    t0 = time.time()
    eng.load_kv(datagen.RMAT_SPACE, *rows.arrays())
    eng.commit(datagen.RMAT_SPACE)
    info = eng.info(datagen.RMAT_SPACE)
    log(f"[rank {rank}] snapshot: {info.vertices} vertices, {info.edges} edges, "
        f"{info.device_bytes / 2**30:.2f} GiB in HBM, load+commit {time.time() - t0:.1f}s")
    keep_rows = rank == 0 and world == 1 and args.cpu_budget > 0
    if not keep_rows:
        rows.free()

    def sentence(step, k):
        seeds = datagen.rmat_seeds(scale, k, args.ef, 42, 42 + step, threads=args.threads)
        return ngql.parse_go(QUERY.replace("{S}", ", ".join(str(int(v)) for v in seeds)))

    plans = [sentence(i, args.seeds) for i in range(args.warmup + args.steps)]

    def step(s, on_device=True):
        r = eng.go(datagen.RMAT_SPACE, s, rows=False, on_device=on_device)
        if not r.ok:
            raise RuntimeError(r.error)
        return r

    def barrier():
        if world > 1:
            dist.barrier()

    for i in range(args.warmup):
        step(plans[i])
    log(f"[rank {rank}] warmup done")
    eng.set_profiling(True)
    barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    edges = 0
    result_rows = 0
    dev_ms = 0.0
    hop_edges = None
    for i in range(args.steps):
        r = step(plans[args.warmup + i])
        edges += sum(r.hop_edges)
        result_rows += r.nrows
        dev_ms += r.device_ms
        hop_edges = r.hop_edges
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t_start
    stats = eng.kernel_stats()
    eng.set_profiling(False)
    # the same steps with the result rows and typed cells delivered to host memory (reported only)
    host_steps = min(2, args.steps)
    barrier()
    t_h = time.perf_counter()
    for i in range(host_steps):
        step(plans[args.warmup + i], on_device=False)
    barrier()
    host_ms = (time.perf_counter() - t_h) * 1e3 / max(host_steps, 1)
    jit = {"compiled": eng.get_flag("jit_compiled"), "failed": eng.get_flag("jit_failed"),
           "compile_ms": eng.get_flag("jit_compile_us") / 1e3, "vgprs": eng.get_flag("jit_vgprs"),
           "scratch_bytes": eng.get_flag("jit_scratch"), "note": eng.jit_note()}

    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0])
        e = torch.tensor([edges, result_rows], dtype=torch.int64)
        dist.all_reduce(e, op=dist.ReduceOp.SUM)
        edges, result_rows = int(e[0]), int(e[1])

    # dominant kernel roofline (algorithmic bytes / HIP-event time)
    dom = max(stats.items(), key=lambda kv: kv[1][1]) if stats else None
    roof = None
    if dom:
        name, (launches, ms, algo) = dom
        achieved = algo / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
        traffic = None
        if os.path.exists(args.traffic):
            try:
                tj = json.load(open(args.traffic))
                if tj.get("kernel_class") == name:
                    traffic = tj.get("bytes_per_launch")
            except Exception:
                traffic = None
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": name,
                "launches": launches, "avg_launch_us": round(ms * 1e3 / max(launches, 1), 2),
                "algo_bytes_per_launch": algo // max(launches, 1)}
    all_ms = sum(v[1] for v in stats.values())
    all_bytes = sum(v[2] for v in stats.values())

    cpu = None
    if keep_rows:
        cpu = cpu_baseline(rows, scale, args)
        rows.free()

    if rank == 0:
        tepss = edges / elapsed
        out = {
            "metric": METRIC, "value": round(tepss, 1), "unit": "edges/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3 / args.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int64",
            "data": "synthetic RMAT (Graph500 .57/.19/.19/.05, splitmix64 seed 42), reference KV format",
            "config": {"workload": f"C2: RMAT scale-{scale} ef{args.ef}, 1 edge type e(p0 int, p1 int), "
                                   f"{args.parts} parts, GO 3 STEPS from {args.seeds} vids WHERE e.p0 < 50",
                       "scale": scale, "edge_factor": args.ef, "parts": args.parts, "seeds": args.seeds,
                       "query": QUERY.replace("{S}", f"<{args.seeds} vids>"),
                       "parallelism": f"{world} shard(s), part % {world}, "
                                      + ("host (gloo) exchange, all shards on GPU 0 (rehearsal)" if args.host_exchange
                                         else "RCCL bitmap all-to-all per hop")},
            "roofline": roof,
            "cpu_baseline": cpu,
            "edges_per_step": edges // args.steps,
            "rows_per_step": result_rows // args.steps,
            "hop_edges_last_step": hop_edges,
            "device_ms_per_step": round(dev_ms / args.steps, 3),
            "ms_per_step_host_rows": round(host_ms, 3),
            "timed_region": "seeds on host -> result rows + YIELD cells in HBM (result_on_device); "
                            "ms_per_step_host_rows adds D2H and host cell conversion",
            "jit": jit,
            "path_roofline": {"algo_bytes": all_bytes, "kernel_ms": round(all_ms, 3),
                              "frac": round(all_bytes / (all_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if all_ms else None},
            "kernels": {k: {"launches": v[0], "ms": round(v[1], 3), "algo_bytes": v[2]} for k, v in stats.items()},
        }
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(rows, scale, args):
    """The oracle (C++ restatement of storaged + GoExecutor) on the same graph and query shape, with a
    seed count doubled from 4 until one run takes >= cpu_budget/2 seconds."""
    from nebula_amd import datagen, ngql
    from oracle import oracle
    t0 = time.time()
    o = oracle.Oracle()
    o.set_flags(threads=args.threads)
    o.add_space(datagen.RMAT_SPACE, args.parts)
    for is_edge, sid, name, fields in datagen.rmat_schemas():
        o.add_schema(datagen.RMAT_SPACE, is_edge, sid, name, fields)
    o.put_kv(datagen.RMAT_SPACE, *rows.arrays())
    o.finalize(args.threads)
    log(f"oracle loaded in {time.time() - t0:.1f}s")
    k, best = 4, None
    while True:
        seeds = datagen.rmat_seeds(scale, k, args.ef, 42, 42, threads=args.threads)
        s = ngql.parse_go(QUERY.replace("{S}", ", ".join(str(int(v)) for v in seeds)))
        r = o.go(datagen.RMAT_SPACE, s, rows=False)
        edges = sum(r.hop_scanned)
        best = (k, edges, r.seconds)
        log(f"oracle: {k} seeds, {edges} edges, {r.seconds:.2f}s")
        if r.seconds >= args.cpu_budget / 2 or k >= args.seeds:
            break
        k *= 2
    k, edges, sec = best
    o.close()
    return {"value": round(edges / sec, 1), "unit": "edges/s", "cores": args.threads, "kind": "port",
            "sample": f"same graph and query, first {k} of the seed sample, {edges} edges traversed in "
                      f"{sec:.2f}s (oracle C++ restatement, {args.threads} threads)"}


if __name__ == "__main__":
    main()
