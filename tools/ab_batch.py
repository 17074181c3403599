"""In-process A/B of engine flags on bench.py's timed loop (C2 graph loaded once, through ngx_load_csr).

bench.py pays ~50 s of KV load + commit per run, and two runs on the same box differ by a few percent;
this tool builds the C2 shard once and times bench.py's exact timed step — `go_batch` over the same 20
prepared plans (seeds rmat_seeds(22, 1000, 16, 42, 42 + i)), after a 5-plan warmup batch — alternately
per variant, R rounds, and prints the median and spread of ms per step for each variant.

Usage (GPU box): python tools/ab_batch.py [--rounds 8] [--steps 20] VARIANT ...
  VARIANT = "base" or comma-separated NAME=VALUE engine flags, e.g. "batch_finals=2,batch_lanes=4";
  "env:NAME=VALUE" items set an environment variable for the variant (e.g. env:NGX_JIT_WAVES=8, read when
  a generated kernel is compiled)
With --final, each round also runs the 20 plans one at a time with HIP-event profiling and reports the
final hop's average launch time per variant.
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

QUERY = "GO 3 STEPS FROM {S} OVER e WHERE e.p0 < 50 YIELD e._dst, e._rank, e.p0, e.p1"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--scale", type=int, default=22)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--final", action="store_true")
    ap.add_argument("--prewarm", type=int, default=0, help="untimed batches of the timed plans before round 0")
    ap.add_argument("--sleep-ms", type=float, default=0, help="idle host time before each timed batch")
    ap.add_argument("--busy-ms", type=float, default=0, help="unrelated device work (buffer fills) before round 0")
    ap.add_argument("--prewarm-warm", type=int, default=0, help="untimed batches of the warm-up plans only before round 0")
    ap.add_argument("--spin-ms", type=float, default=0, help="host busy loop (no GPU work) before each timed batch")
    ap.add_argument("--commit-flag", action="append", default=[], help="NAME=VALUE engine flag set before the load")
    args = ap.parse_args()
    import torch
    from nebula_amd import datagen, engine, ngql
    torch.cuda.set_device(0)
    t0 = time.time()
    c = datagen.rmat_csr(args.scale, 16, 42, 100, with_in=True, threads=args.threads)
    eng = engine.Engine(0)
    for kv in args.commit_flag:
        n, _, val = kv.partition("=")
        eng.set_flag(n, int(val))
    eng.add_space(datagen.RMAT_SPACE, 100)
    for is_edge, sid, name, fields in datagen.rmat_schemas():
        eng.add_schema(datagen.RMAT_SPACE, is_edge, sid, name, fields)
    eng.load_csr(datagen.RMAT_SPACE, c.vpart, c.vid, c.slots)
    eng.commit(datagen.RMAT_SPACE)
    c.free()
    info = eng.info(datagen.RMAT_SPACE)
    print(f"[ab] C2 shard loaded in {time.time() - t0:.1f}s: {info.vertices} vertices, {info.edges} edges, "
          f"{info.device_bytes / 2**30:.3f} GiB in HBM", flush=True)

    def plan(i):
        seeds = datagen.rmat_seeds(args.scale, 1000, 16, 42, 42 + i, threads=args.threads)
        s = ngql.parse_go(QUERY.replace("{S}", ", ".join(str(int(v)) for v in seeds)))
        return eng.prepare_go(datagen.RMAT_SPACE, s, on_device=True, yield_only=True, compact=True)

    preps = [plan(i) for i in range(args.warmup + args.steps)]
    warm, timed = preps[:args.warmup], preps[args.warmup:]
    edges = None
    parsed = []
    for v in args.variants:
        flags, envs = [], []
        if v != "base":
            for kv in v.split(","):
                n, _, val = kv.partition("=")
                if n.startswith("env:"):
                    envs.append((n[4:], val))
                else:
                    flags.append((n, int(val)))
        parsed.append((v, (flags, envs)))
    defaults = {n: eng.get_flag(n) for _, (fl, _) in parsed for n, _ in fl}
    res = {v: [] for v, _ in parsed}
    fin = {v: [] for v, _ in parsed}
    if args.busy_ms:
        buf = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < args.busy_ms:
            buf.fill_(1)
            torch.cuda.synchronize()
        del buf
    for _ in range(args.prewarm_warm):
        eng.go_batch(warm)
    for _ in range(args.prewarm):
        eng.go_batch(warm)
        eng.go_batch(timed)
    torch.cuda.synchronize()
    for r in range(args.rounds):
        for v, (flags, envs) in (parsed if r % 2 == 0 else parsed[::-1]):
            saved = {n: os.environ.get(n) for n, _ in envs}
            for n, val in envs:
                os.environ[n] = val
            for n, val in flags:
                eng.set_flag(n, val)
            if args.sleep_ms:
                time.sleep(args.sleep_ms / 1e3)
            for code, _, _ in eng.go_batch(warm):
                assert code == 0
            torch.cuda.synchronize()
            if args.spin_ms:
                t_s = time.perf_counter()
                while (time.perf_counter() - t_s) * 1e3 < args.spin_ms:
                    pass
            a0 = eng.get_flag("dbuf_allocs")
            print(f"[ab] timed batch {v} round {r} begins", file=sys.stderr, flush=True)
            t = time.perf_counter()
            out = eng.go_batch(timed)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            grown = eng.get_flag("dbuf_allocs") - a0
            if grown:
                print(f"[ab] {v}: {grown} device buffer allocations inside the timed batch", flush=True)
            assert all(o[0] == 0 for o in out), out
            e = sum(o[2] for o in out)
            assert edges is None or e == edges
            edges = e
            res[v].append(dt * 1e3 / args.steps)
            if args.final:
                eng.set_profiling(True)
                s0 = eng.kernel_stats().get("final", (0, 0.0, 0))
                for p in timed:
                    assert eng.go(datagen.RMAT_SPACE, p, rows=False).ok
                s1 = eng.kernel_stats().get("final", (0, 0.0, 0))
                eng.set_profiling(False)
                if s1[0] > s0[0]:
                    fin[v].append((s1[1] - s0[1]) * 1e3 / (s1[0] - s0[0]))
            for n, _ in flags:
                eng.set_flag(n, defaults[n])
            for n, old in saved.items():
                if old is None:
                    os.environ.pop(n, None)
                else:
                    os.environ[n] = old
        print(f"[ab] round {r}: " + "  ".join(f"{v} {res[v][-1]:.4f}" for v, _ in parsed), flush=True)
    for v, _ in parsed:
        x = res[v]
        med = statistics.median(x)
        fx = f"  final {statistics.median(fin[v]):.1f} us" if fin[v] else ""
        print(f"[ab] {v:40s} median {med:.4f} ms/step  min {min(x):.4f}  max {max(x):.4f}  "
              f"TEPS {edges / args.steps / (med * 1e-3):.4g}{fx}", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
