"""Benchmark: traversed edges/sec of `GO 3 STEPS FROM <1k vids> OVER e WHERE e.p0 < 50 YIELD e._dst,
e._rank, e.p0, e.p1` on an RMAT graph (BASELINE.json metric).

Workload by GPU count (one process per GPU, parts hashed to GPUs as part % N, Nebula's pickHosts):
  N = 1  configs[1] (C2): RMAT scale 22, edge factor 16, 100 parts
  N = 8  configs[2] (C3): RMAT scale 26, edge factor 16, 100 parts, per-hop frontier exchange (RCCL:
         bitmap all-to-all after a push hop, bitmap all-gather before a pull hop)
  N = 2, 4: scale 22 + log2(N) (weak scaling between the two anchors); --scale overrides.

One step = one GO query through libnebula_gn (seeds on host -> result rows and YIELD columns in HBM),
with a fresh 1k-seed sample per step. Traversed edges = sum over hops of the edges scanned
(SURVEY.md §8d), summed over ranks. The JSON line also carries the HBM roofline of the dominant
kernel (HIP events on the engine stream), the per-hop frontier exchange (N > 1), the host-delivery
cost of the rows, and a CPU baseline (rank 0, N = 1): the oracle restatement of the reference path
on the same graph, all host cores for GO end to end plus one thread for storage-only GetNeighbors.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]; N > 1 under torch.distributed.run.
"""
import argparse
import datetime
import json
import math
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md)
METRIC = "traversed edges/sec for GO 3 STEPS WHERE on RMAT; % HBM roofline"
QUERY = "GO 3 STEPS FROM {S} OVER e WHERE e.p0 < 50 YIELD e._dst, e._rank, e.p0, e.p1"
NOT_HBM = ("exchange",)        # kernel classes whose bytes are not HBM traffic (xGMI, reported apart)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # 100 queries per timed batch (a graphd's stream of sessions): the pipeline's fill and drain (the first
    # query's hops and the last one's final hop run alone) are ~1 step's time per batch, 10% at 10 steps
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--scale", type=int, default=0, help="RMAT scale (default: 22 at N=1, 26 at N=8, else 22+log2 N)")
    p.add_argument("--ef", type=int, default=16)
    p.add_argument("--seeds", type=int, default=1000)
    p.add_argument("--parts", type=int, default=100)
    p.add_argument("--cpu-budget", type=float, default=20.0, help="target seconds of oracle GO work (0: skip)")
    p.add_argument("--threads", type=int, default=16, help="host threads for datagen / oracle")
    p.add_argument("--out-only", action="store_true", help="store out-edges only (no -e in-edge slot)")
    p.add_argument("--row-arrays", action="store_true",
                   help="timed step also writes the src / dst / rank row arrays (GetNeighbors' edge keys) beside "
                        "the YIELD columns. Default off: GO's result is its YIELD columns (GoExecutor.cpp:1288-1297 "
                        "builds each record from the yields only); with them the C2 final hop measured 289 vs 250 us")
    p.add_argument("--no-compact", action="store_true",
                   help="timed step writes every result value at 8 bytes (default: compact_results, integer "
                        "arrays at the widths of the stored columns they copy)")
    p.add_argument("--host-exchange", action="store_true",
                   help="rehearsal of the N > 1 path on one GPU: every rank on device 0, frontier exchange "
                        "through the host collective (gloo) instead of RCCL")
    p.add_argument("--host-loop", choices=["native", "python"], default="native",
                   help="timed steps driven by one native loop over the prepared plans (ngx_go_batch, as a C++ "
                        "graphd would) or by a Python call per step")
    p.add_argument("--flag", action="append", default=[], metavar="NAME=VALUE",
                   help="engine flag (ngx_set_flag) set before the run, e.g. dyn_hops=1; repeatable")
    p.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"),
                   help="PMC-derived HBM bytes per launch of the dominant kernel (from profiles/)")
    return p.parse_args()


def default_scale(world):
    if world == 8:
        return 26
    return 22 + int(round(math.log2(world)))


def cpu_info():
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    return model, os.cpu_count() or 1, usable


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    scale = args.scale or default_scale(world)

    import numpy as np
    import torch
    import torch.distributed as dist
    from nebula_amd import datagen, engine, ngql

    device = 0 if args.host_exchange else local
    torch.cuda.set_device(device)
    uid, xchg = None, None
    if world > 1:
        # bounded collectives: a dead rank ends the others instead of hanging the node
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=600))
        if args.host_exchange:
            xchg = engine.dist_exchange()
        else:
            obj = [engine.unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            uid = obj[0]

    build = engine.build_info()
    if rank == 0:
        log(f"[rank 0] libnebula_gn {build['raw']} (sources in tree: {build['tree_sha']}, "
            f"match={build['matches_tree']})")
    t0 = time.time()
    # every out-edge also stored as its in-edge (-e), as InsertEdgeExecutor writes them,
    # at every N: the in-edge slot is what the pull hops read (world > 1: against the all-gathered
    # frontier bitmap), so N = 1 and N = 8 run the same direction-optimizing algorithm
    with_in = not args.out_only
    rows = datagen.rmat(scale, args.ef, 42, args.parts, with_in=with_in, with_tag=False, rank=rank, world=world,
                        threads=args.threads)
    log(f"[rank {rank}] generated {rows.n} rows of RMAT scale {scale} in {time.time() - t0:.1f}s")
    eng = engine.Engine(device, rank, world, uid, exchange=xchg)
    for f in args.flag:
        name, _, val = f.partition("=")
        eng.set_flag(name, int(val))
    eng.add_space(datagen.RMAT_SPACE, args.parts)
    for is_edge, sid, name, fields in datagen.rmat_schemas():
        eng.add_schema(datagen.RMAT_SPACE, is_edge, sid, name, fields)
    t0 = time.time()
    eng.load_kv(datagen.RMAT_SPACE, *rows.arrays())
    # the library staged its own copy: the generator's rows go before the export doubles the footprint
    # (C3: ~20 GB of rows per rank), unless the CPU baseline reads them
    keep_rows = rank == 0 and world == 1 and args.cpu_budget > 0
    if not keep_rows:
        rows.free()
    eng.commit(datagen.RMAT_SPACE)
    info = eng.info(datagen.RMAT_SPACE)
    log(f"[rank {rank}] snapshot: {info.vertices} vertices, {info.edges} edges, "
        f"{info.device_bytes / 2**30:.2f} GiB in HBM, load+commit {time.time() - t0:.1f}s")

    def sentence(step, k):
        seeds = datagen.rmat_seeds(scale, k, args.ef, 42, 42 + step, threads=args.threads)
        return ngql.parse_go(QUERY.replace("{S}", ", ".join(str(int(v)) for v in seeds)))

    plans = [sentence(i, args.seeds) for i in range(args.warmup + args.steps)]
    # the timed steps' sentences encoded once into C plans (a C++ host keeps its prepared plan the same way)
    prepared = {}

    def step(s, on_device=True, columnar=False, rows_=False):
        key = (id(s), on_device, columnar)
        if key not in prepared:
            prepared[key] = eng.prepare_go(datagen.RMAT_SPACE, s, on_device=on_device, columnar=columnar,
                                           yield_only=on_device and not args.row_arrays,
                                           compact=on_device and not args.no_compact)
        r = eng.go(datagen.RMAT_SPACE, prepared[key], rows=rows_, arrays=False)
        if not r.ok:
            raise RuntimeError(r.error)
        return r

    def barrier():
        if world > 1:
            dist.barrier()

    for s_ in plans:                                        # encoded before the timed region
        prepared[(id(s_), True, False)] = eng.prepare_go(datagen.RMAT_SPACE, s_, on_device=True,
                                                         yield_only=not args.row_arrays, compact=not args.no_compact)
    if args.host_loop == "native" and args.warmup:
        # warmed through the timed loop's own path (the batch, its streams and coroutine stacks)
        for code, _, _ in eng.go_batch([prepared[(id(plans[i]), True, False)] for i in range(args.warmup)]):
            if code:
                raise RuntimeError(f"GO failed in warmup ({code}): {eng.L.ngx_last_error(eng.h).decode()}")
    else:
        for i in range(args.warmup):
            step(plans[i])
    log(f"[rank {rank}] warmup done")
    barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    edges = 0
    result_rows = 0
    dev_ms = 0.0
    hop_edges = None
    hop_xchg = None
    final_8d = final_edges = final_rows = 0
    p1_width = None
    prep_ms = tail_ms = 0.0
    timed = [prepared[(id(plans[args.warmup + i]), True, False)] for i in range(args.steps)]
    overlaps = eng.get_flag("batch_overlaps")
    if args.host_loop == "native":
        # the K steps in one native loop over the prepared plans (ngx_go_batch: each is one ngx_go; the
        # next query's host work and first hops enqueued while this one's final hop runs)
        for code, nrows, e in eng.go_batch(timed):
            if code:
                raise RuntimeError(f"GO failed in the timed loop ({code}): {eng.L.ngx_last_error(eng.h).decode()}")
            edges += e
            result_rows += nrows
    else:
        for i in range(args.steps):
            r = step(plans[args.warmup + i])
            edges += sum(r.hop_edges)
            result_rows += r.nrows
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t_start
    overlaps = eng.get_flag("batch_overlaps") - overlaps
    # the same steps again with per-kernel HIP events (their records would perturb the timed loop), one
    # Python call each: per-step statistics
    eng.set_profiling(True)
    for i in range(args.steps):
        r = step(plans[args.warmup + i])
        dev_ms += r.device_ms                            # device time: HIP events, profiled pass only
        prep_ms += r.host_prep_ms
        tail_ms += r.host_tail_ms
        hop_edges = r.hop_edges
        hop_xchg = r.hop_xchg
        final_8d += 24 * r.hop_edges[-1] + 40 * r.nrows
        final_edges += r.hop_edges[-1]
        final_rows += r.nrows
        if r.dev_widths and len(r.dev_widths[1]) >= 4:
            p1_width = r.dev_widths[1][3]               # YIELD e._dst, e._rank, e.p0, e.p1: p1's width
    stats = eng.kernel_stats()
    eng.set_profiling(False)

    # GetNeighbors, the storage boundary (QueryBoundProcessor, the final-hop request GoExecutor sends):
    # one step's 1000 seeds grouped by part, return columns _dst, p0, p1, pushed filter e.p0 < 50, rows
    # and typed cells delivered to host memory (reported beside `value`)
    gn_stats = None
    if world == 1:
        seeds0 = [int(v) for v in datagen.rmat_seeds(scale, args.seeds, args.ef, 42, 42, threads=args.threads)]
        by_part = {}
        for v in seeds0:
            by_part.setdefault(v % args.parts + 1, []).append(v)
        gparts = sorted(by_part.items())
        gcols = [(engine.EDGE, 1, "_dst"), (engine.EDGE, 1, "p0"), (engine.EDGE, 1, "p1")]
        gfilt = ngql.Binary(ngql.K_REL, ngql.REL_OPS["<"], ngql.Prop(ngql.K_ALIAS, "", "e", "p0"), ngql.Prim(50)).encode()
        for _ in range(3):
            eng.get_neighbors(datagen.RMAT_SPACE, gparts, [1], gcols, gfilt, decode=False)
        reps = 20
        t_g = time.perf_counter()
        for _ in range(reps):
            gr = eng.get_neighbors(datagen.RMAT_SPACE, gparts, [1], gcols, gfilt, decode=False)
        g_ms = (time.perf_counter() - t_g) * 1e3 / reps
        gn_stats = {"request": "1000 vids by part, return _dst/p0/p1, filter e.p0 < 50, cells to host",
                    "ms_per_request": round(g_ms, 3), "edges_returned": gr.total_edges,
                    "returned_edges_per_s": round(gr.total_edges / (g_ms / 1e3), 1)}

    # the same steps with the rows delivered to host memory (reported, never `value`): columnar arrays
    # in page-locked staging (host_columnar), and typed cells (ColumnValue) built on host threads
    host_steps = min(2, args.steps)
    step(plans[0], on_device=False, columnar=True)          # sizes the page-locked staging once
    barrier()
    t_h = time.perf_counter()
    col_tail = col_dev = 0.0
    col_bytes = 0
    for i in range(host_steps):
        r = step(plans[args.warmup + i], on_device=False, columnar=True)
        col_tail += r.host_tail_ms
        col_dev += r.device_ms
        col_bytes = r.nrows * 40
    barrier()
    host_col_ms = (time.perf_counter() - t_h) * 1e3 / max(host_steps, 1)
    col_tail /= max(host_steps, 1)
    col_dev /= max(host_steps, 1)
    t_h = time.perf_counter()
    step(plans[args.warmup], on_device=False)
    barrier()
    host_cell_ms = (time.perf_counter() - t_h) * 1e3
    jit = {"compiled": eng.get_flag("jit_compiled"), "failed": eng.get_flag("jit_failed"),
           "compile_ms": eng.get_flag("jit_compile_us") / 1e3, "vgprs": eng.get_flag("jit_vgprs"),
           "scratch_bytes": eng.get_flag("jit_scratch"), "note": eng.jit_note()}

    xchg_ms = stats.get("exchange", (0, 0.0, 0))[1]
    xchg_bytes = stats.get("exchange", (0, 0.0, 0))[2]
    if world > 1:
        t = torch.tensor([elapsed, xchg_ms], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, xchg_ms_max = float(t[0]), float(t[1])
        e = torch.tensor([edges, result_rows, xchg_bytes], dtype=torch.int64)
        dist.all_reduce(e, op=dist.ReduceOp.SUM)
        edges, result_rows, xchg_bytes_all = int(e[0]), int(e[1]), int(e[2])

    # dominant kernel roofline. `frac` = the bytes the kernel must move on this layout (a
    # fraction <= 1 of the bytes the kernel actually moves) / its HIP-event launch time / 8 TB/s. For the
    # final hop that is the library's stored-width count (dst 4 B + p0 1 B per scanned edge, rank a
    # constant column: 0 B; 13 B written per row: dst 4, p0 1, p1 8 — 17 with --row-arrays' src) plus the YIELD-only column p1 read at whole 128-B lines:
    # a line of 128 / w values is fetched when any of its edges passes, 1 - (1 - f)^(128 / w) of the
    # lines at pass fraction f (random at C2: every line). SURVEY.md §8d's figure (every field 8 B) is
    # kept beside it as frac_8d, a TEPS-equivalent credit, not a bandwidth.
    hbm = {k: v for k, v in stats.items() if k not in NOT_HBM}
    dom = max(hbm.items(), key=lambda kv: kv[1][1]) if hbm else None
    roof = None
    final_fix = 0
    if dom:
        name, (launches, ms, algo) = dom
        traffic = None
        # the committed PMC bytes were measured on the N = 1 C2 step: other workloads report none
        if os.path.exists(args.traffic) and world == 1 and scale == 22:
            try:
                tj = json.load(open(args.traffic))
                # and on the same result layout (compact_results and the row arrays change the final hop's
                # writes)
                if tj.get("kernel_class") == name and bool(tj.get("compact", False)) == (not args.no_compact) \
                        and bool(tj.get("yield_only", False)) == (not args.row_arrays):
                    traffic = tj.get("bytes_per_launch")
            except Exception:
                traffic = None
        avg_s = ms * 1e-3 / max(launches, 1)
        stored = algo // max(launches, 1)             # the library's count: fields at their stored widths
        must, algo8, line_note = stored, stored, None
        if name == "final" and final_8d and launches:
            # the profiled pass re-runs the timed steps: one final launch per step
            algo8 = final_8d // args.steps
            e_last = max(final_edges // args.steps, 1)
            rows_last = final_rows // args.steps
            f = min(1.0, rows_last / e_last)
            w = p1_width or 8
            lines = 1.0 - (1.0 - f) ** (128 // w)
            p1_bytes = int(e_last * w * lines)
            must = stored + p1_bytes
            line_note = {"p1_width": w, "pass_fraction": round(f, 4), "p1_lines_read": round(lines, 6),
                         "p1_line_bytes": p1_bytes}
            final_fix = (must - stored) * launches
        gbs = lambda b: b / avg_s / 1e9 if avg_s > 0 else 0.0
        achieved = gbs(must)
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": name,
                "launches": launches, "avg_launch_us": round(ms * 1e3 / max(launches, 1), 2),
                "algo_bytes_per_launch": must,
                "bytes_model": "bytes the final hop must move: scanned-edge reads at stored widths (dst, filter "
                               "column p0; constant rank 0 B) + result rows at written widths + the YIELD-only "
                               "column p1 at whole 128-B lines",
                "p1_lines": line_note,
                # the HBM bytes the PMC counters measured per launch over this launch time: the kernel's
                # real memory throughput
                "frac_counter": round(traffic / avg_s / 1e9 / HBM_PEAK_GBS, 4) if traffic and avg_s > 0 else None,
                "traffic_over_must": round(traffic / must, 3) if traffic and must else None,
                # the same launch credited per SURVEY.md §8d (24 B / scanned edge + 40 B / row, every field
                # 8 B): a TEPS-equivalent credit, above the bytes the kernel moves with narrow columns
                "frac_8d": round(gbs(algo8) / HBM_PEAK_GBS, 4), "algo_bytes_8d": algo8,
                # stored widths without the p1 lines (the library's own per-kernel count)
                "stored_width": {"algo_bytes_per_launch": stored,
                                 "frac": round(gbs(stored) / HBM_PEAK_GBS, 4) if avg_s > 0 else None,
                                 "compact_results": not args.no_compact}}
    all_ms = sum(v[1] for v in hbm.values())
    all_bytes_stored = sum(v[2] for v in hbm.values())
    all_bytes = all_bytes_stored + final_fix

    cpu = None
    if keep_rows:
        cpu = cpu_baseline(rows, scale, args, edges // max(args.steps, 1))
        rows.free()

    if rank == 0:
        tepss = edges / elapsed
        workload = ("C3" if world == 8 and scale == 26 else "C2" if world == 1 and scale == 22 else "weak-scaling")
        out = {
            "metric": METRIC, "value": round(tepss, 1), "unit": "edges/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed * 1e3 / args.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int64",
            "data": "synthetic RMAT (Graph500 .57/.19/.19/.05, splitmix64 seed 42), reference KV format",
            "config": {"workload": f"{workload}: RMAT scale-{scale} ef{args.ef}, 1 edge type e(p0 int, p1 int), "
                                   f"{args.parts} parts over {world} GPU(s), GO 3 STEPS from {args.seeds} vids "
                                   "WHERE e.p0 < 50",
                       "scale": scale, "edge_factor": args.ef, "parts": args.parts, "seeds": args.seeds,
                       "query": QUERY.replace("{S}", f"<{args.seeds} vids>"),
                       "scale_rule": "N=1: 22 (C2), N=8: 26 (C3), else 22+log2(N)",
                       "edge_layout": "out-edges + in-edges (-e)" if with_in else "out-edges",
                       "parallelism": f"{world} shard(s), part % {world}, "
                                      + ("host (gloo) exchange, all shards on GPU 0 (rehearsal)" if args.host_exchange
                                         else "RCCL bitmap all-to-all per hop"),
                       **({"engine_flags": args.flag} if args.flag else {})},
            "roofline": roof,
            "cpu_baseline": cpu,
            "edges_per_step": edges // args.steps,
            "rows_per_step": result_rows // args.steps,
            "hop_edges_last_step": hop_edges,
            "device_ms_per_step": round(dev_ms / args.steps, 3),
            "device_ms_note": "first launch to last result write, HIP events, measured in the profiled re-run of the steps",
            "host_ms_per_step": {"library_prep": round(prep_ms / args.steps, 3), "library_tail": round(tail_ms / args.steps, 3),
                                 "note": "inside ngx_go: before the first launch (plan, programs, seeds) / after the "
                                         "device finished; the rest of ms_per_step - device_ms is the Python caller"},
            "host_loop": args.host_loop,
            "batch_overlaps": overlaps,
            "timed_region": ("seeds on host -> the YIELD columns of every result row in HBM (result_on_device; "
                             + ("and the src / dst / rank row arrays" if args.row_arrays else
                                "yield_only: the YIELD columns are the result, as GoExecutor's records; e._dst / "
                                "e._rank alias the dst / rank row arrays, no src array") + ")"),
            "get_neighbors": gn_stats,
            "host_delivery": {"ms_per_step_columnar": round(host_col_ms, 3), "ms_per_step_cells": round(host_cell_ms, 3),
                              "columnar_library_tail_ms": round(col_tail, 3), "columnar_device_ms": round(col_dev, 3),
                              "columnar_row_bytes": col_bytes,
                              "note": "same query with the rows copied to host memory: columnar arrays in "
                                      "page-locked staging (host_columnar), or typed ColumnValue cells"},
            "jit": jit,
            # every kernel's library byte count (stored widths; a pulled hop credited with what the pull
            # reads: 9 B per row, not its scanned edges), the final hop as in `roofline`
            "path_roofline": {"algo_bytes": all_bytes, "algo_bytes_stored_width": all_bytes_stored,
                              "kernel_ms": round(all_ms, 3),
                              "frac": round(all_bytes / (all_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if all_ms else None,
                              # the whole step: every kernel's algorithmic bytes over the wall time per step
                              "frac_wall": round(all_bytes / max(args.steps, 1) / (elapsed / args.steps)
                                                 / 1e9 / HBM_PEAK_GBS, 4) if elapsed > 0 else None},
            "kernels": {k: {"launches": v[0], "ms": round(v[1], 3), "algo_bytes": v[2]} for k, v in stats.items()},
            "build": {"library": build["raw"], "sources_sha": build["tree_sha"], "matches_tree": build["matches_tree"]},
        }
        if world > 1:
            out["exchange"] = {"bytes_per_step_all_ranks": xchg_bytes_all // args.steps,
                               "rank0_bytes_per_hop_last_step": hop_xchg,
                               "ms_per_step_max_rank": round(xchg_ms_max / args.steps, 3),
                               "note": "per-hop bitmap all-to-all of next-frontier rows (RCCL send/recv over xGMI); "
                                       "HIP-event time includes pack + merge kernels"}
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(rows, scale, args, gpu_edges_per_step):
    """The oracle (C++ restatement of storaged + GoExecutor, the reference CPU path) on this host, same
    graph: (1) GO end to end (the bench query) on all threads, seeds added until it traverses >= 10% of
    one GPU step's edges and runs >= cpu_budget/2 s; (2) storage only, one thread: a GetNeighbors request
    returning one edge prop, as the reference's GetNeighborsBenchmark (GetNeighborsBenchmark.cpp:390-402)."""
    from nebula_amd import datagen, ngql
    from oracle import oracle
    model, nproc, usable = cpu_info()
    # every core this process may use: the affinity set, capped by the host share the launcher grants
    # (OMP_NUM_THREADS; 16 per GPU on the MI355X boxes, whose nproc counts the whole machine)
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = max(1, min(usable, share) if share > 0 else usable)
    t0 = time.time()
    o = oracle.Oracle()
    # 4 buckets per thread (max_handlers_per_req): the reader pool balances RMAT's hub-heavy vertices
    # (genBuckets cuts the request's vertex list into equal counts, not equal edges)
    o.set_flags(threads=threads, max_handlers=4 * threads, graph_threads=threads)
    o.add_space(datagen.RMAT_SPACE, args.parts)
    for is_edge, sid, name, fields in datagen.rmat_schemas():
        o.add_schema(datagen.RMAT_SPACE, is_edge, sid, name, fields)
    o.put_kv(datagen.RMAT_SPACE, *rows.arrays())
    o.finalize(threads)
    log(f"oracle loaded in {time.time() - t0:.1f}s")
    k, best = 1, None
    while True:
        seeds = datagen.rmat_seeds(scale, k, args.ef, 42, 42, threads=args.threads)
        s = ngql.parse_go(QUERY.replace("{S}", ", ".join(str(int(v)) for v in seeds)))
        r = o.go(datagen.RMAT_SPACE, s, rows=False)
        edges = sum(r.hop_scanned)
        best = (k, edges, r.seconds)
        log(f"oracle GO: {k} seeds, {edges} edges, {r.seconds:.2f}s")
        if (edges >= 0.1 * gpu_edges_per_step and r.seconds >= args.cpu_budget / 2) or k >= args.seeds \
                or r.seconds >= args.cpu_budget:
            break
        k *= 2
    k, edges, sec = best
    # the reference's own shape of the same work: graphd's final evaluation on one thread
    # (processFinalResult), storage on all of them; a quarter of the sample keeps the run short
    o.set_flags(threads=threads, max_handlers=4 * threads, graph_threads=1)
    k1 = max(1, k // 4)
    seeds = datagen.rmat_seeds(scale, k1, args.ef, 42, 42, threads=args.threads)
    r1 = o.go(datagen.RMAT_SPACE, ngql.parse_go(QUERY.replace("{S}", ", ".join(str(int(v)) for v in seeds))),
              rows=False)
    serial = round(sum(r1.hop_scanned) / r1.seconds, 1)
    log(f"oracle GO, one graphd thread: {k1} seeds, {sum(r1.hop_scanned)} edges, {r1.seconds:.2f}s")
    # storage-only, one thread: GetNeighbors over a sample of vertices, `_dst` + one prop, no filter
    o.set_flags(threads=1, max_handlers=1)
    vids = datagen.rmat_seeds(scale, 50000, args.ef, 42, 4343, threads=args.threads)
    parts = {}
    for v in vids:
        parts.setdefault(int(v) % args.parts + 1, []).append(int(v))
    parts = sorted(parts.items())
    gn = {}
    for label, cols in (("one_prop", [(3, 1, "_dst"), (3, 1, "p0")]), ("dst_only", [(3, 1, "_dst")])):
        resp = o.get_neighbors(datagen.RMAT_SPACE, parts, [1], cols)
        gn[label] = round(resp.total_edges / o.last_seconds, 1)
        gn["edges"] = resp.total_edges
    o.close()
    return {"value": round(edges / sec, 1), "unit": "edges/s", "cores": threads, "kind": "port",
            "per_thread": round(edges / sec / threads, 1),
            "sample": f"same graph and query, first {k} seed(s) of the seed sample: {edges} edges traversed "
                      f"({100.0 * edges / max(gpu_edges_per_step, 1):.0f}% of one GPU step) in {sec:.2f}s, "
                      f"oracle C++ restatement on {threads} threads (storage scan and final evaluation alike)",
            "graphd_one_thread": {"value": serial, "seeds": k1,
                                  "note": "the reference's shape: storage on all threads, graphd's "
                                          "processFinalResult on one"},
            "cpu_model": model, "nproc": nproc, "usable_cpus": usable,
            "threads_note": "cores = the process's CPU share (OMP_NUM_THREADS, 16 per GPU on these boxes; nproc counts "
                            "the whole machine), capped by its affinity set",
            "storage_get_neighbors_1thread": {
                "edges_per_s_one_prop": gn["one_prop"], "edges_per_s_dst_only": gn["dst_only"],
                "edges": gn["edges"],
                "reference_published": "1.51e6 edges/s one prop, 5.28e6 _dst only, 1 thread, Xeon E5-2690 v2 "
                                       "(GetNeighborsBenchmark.cpp:390-403)"},
            "note": "value parallelises graphd's final evaluation too (rows kept in order), which the "
                    "reference runs on one thread (GoExecutor.cpp:1082-1335): a more generous baseline "
                    "than the reference's own shape (graphd_one_thread)"}


if __name__ == "__main__":
    main()
