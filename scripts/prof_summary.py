"""Summarise a scripts/profile.sh run (rocprofv3 CSVs under gpurun_out/prof/<tag>) into profiles/.

Writes profiles/<tag>_kernel_stats.csv (the rocprofv3 --stats table as produced), and
profiles/<tag>_summary.md + profiles/<tag>_traffic.json with, per kernel, the average duration from
the kernel trace and the average FETCH_SIZE / WRITE_SIZE per launch from the two PMC passes.

HBM bytes (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of wide coalesced
streaming reads on gfx950, so the corrected read figure is 2 x FETCH_SIZE (an upper bound for
narrower access widths, which are uncalibrated); WRITE_SIZE is exact for 16-B-per-lane stores.
Both counters are in KB (1024 B).

Usage: python scripts/prof_summary.py <tag> [--dominant KERNEL_SUBSTRING]
"""
import argparse
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name, kid=None):
    n = name.split("(")[0].replace("void ", "").strip()
    # generated kernels share one name across query shapes (each its own module): keep the modules apart
    # (r05's traffic averaged the timed step's module with the host-delivery step's 8-byte one: 1.31x
    # "write amplification" that no timed launch had)
    if kid is not None and n.startswith("ngx_jit_"):
        n += f"#{kid}"
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--dominant", default="", help="kernel name substring whose traffic bench.py reads")
    ap.add_argument("--kernel-class", default="final",
                    help="bench.py's name for the dominant kernel (its roofline.kernel); written as kernel_class")
    args = ap.parse_args()
    src = os.path.join(ROOT, "gpurun_out", "prof", args.tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(dst, f"{args.tag}_kernel_stats.csv"))
    trace = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))):
        trace[short(r["Kernel_Name"], r.get("Kernel_Id"))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    pmc = {}
    for kind in ("fetch", "write"):
        d = collections.defaultdict(list)
        f = os.path.join(src, kind, "run_counter_collection.csv")
        if os.path.exists(f):
            for r in csv.DictReader(open(f)):
                d[short(r["Kernel_Name"], r.get("Kernel_Id"))].append(float(r["Counter_Value"]))
        pmc[kind] = d
    rows = []
    for k, durs in sorted(trace.items(), key=lambda kv: -sum(kv[1])):
        fe = pmc["fetch"].get(k)
        wr = pmc["write"].get(k)
        fetch_b = 2 * 1024 * sum(fe) / len(fe) if fe else None
        write_b = 1024 * sum(wr) / len(wr) if wr else None
        rows.append({"kernel": k, "launches": len(durs), "avg_us": sum(durs) / len(durs) / 1e3,
                     "total_ms": sum(durs) / 1e6, "fetch_bytes_x2": fetch_b, "write_bytes": write_b})
    bench = None
    bj = os.path.join(src, "bench_trace.json")
    if os.path.exists(bj):
        for line in open(bj):
            if line.startswith("{"):
                bench = json.loads(line)
    with open(os.path.join(dst, f"{args.tag}_summary.md"), "w") as f:
        f.write(f"# rocprofv3 summary `{args.tag}`\n\n")
        f.write("Command: `bash scripts/profile.sh` (kernel trace + stats pass, then separate `--pmc FETCH_SIZE` and "
                "`--pmc WRITE_SIZE` passes of the same bench command).\n\n")
        if bench:
            f.write(f"bench line of the trace pass: value {bench['value']:.4g} {bench['unit']}, "
                    f"ms_per_step {bench['ms_per_step']}, roofline {json.dumps(bench.get('roofline'))}\n\n")
        f.write("| kernel | launches | avg us | total ms | HBM read B/launch (2x FETCH_SIZE) | HBM write B/launch (WRITE_SIZE) |\n")
        f.write("|---|---|---|---|---|---|\n")
        for r in rows:
            fb = f"{r['fetch_bytes_x2']:.4g}" if r["fetch_bytes_x2"] is not None else "-"
            wb = f"{r['write_bytes']:.4g}" if r["write_bytes"] is not None else "-"
            f.write(f"| `{r['kernel'][:90]}` | {r['launches']} | {r['avg_us']:.2f} | {r['total_ms']:.3f} | {fb} | {wb} |\n")
    traffic = {"tag": args.tag, "kernels": rows}
    if args.dominant:
        dom = [r for r in rows if args.dominant in r["kernel"]]
        if dom:
            d = max(dom, key=lambda r: (r["launches"], r["total_ms"]))     # the timed step's module
            traffic["kernel_class"] = args.kernel_class
            # the result layout the profiled bench ran with (bench.py uses the bytes only for the same one)
            traffic["compact"] = bool(bench and ((bench.get("roofline") or {}).get("stored_width") or {}).get("compact_results"))
            # ... and whether it wrote the YIELD columns only (bench.py's default since r05; --row-arrays not)
            traffic["yield_only"] = bool(bench and "yield_only" in (bench.get("timed_region") or ""))
            traffic["kernel_name"] = d["kernel"]
            if d["fetch_bytes_x2"] is not None and d["write_bytes"] is not None:
                traffic["bytes_per_launch"] = d["fetch_bytes_x2"] + d["write_bytes"]
    # SQ pass (profile.sh SQPASS=1): per-launch wave counters; WAVE_CYCLES / WAIT_* / ACTIVE_INST count
    # quad-cycles (MI355X_MICROARCH.md), WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES
    sqf = os.path.join(src, "sq", "run_counter_collection.csv")
    if os.path.exists(sqf):
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(sqf)):
            acc[short(r["Kernel_Name"], r.get("Kernel_Id"))][r["Counter_Name"]].append(float(r["Counter_Value"]))
        sq = {}
        for k, d in acc.items():
            per = {c: sum(v) / len(v) for c, v in d.items()}
            wc = per.get("SQ_WAVE_CYCLES") or 0.0
            if wc:
                per["frac_wait_any"] = per.get("SQ_WAIT_ANY", 0.0) / wc
                per["frac_wait_inst_any"] = per.get("SQ_WAIT_INST_ANY", 0.0) / wc
                per["frac_active_inst_any"] = per.get("SQ_ACTIVE_INST_ANY", 0.0) / wc
            durs = trace.get(k)
            if wc and durs:
                # average resident waves = wave cycles (4 per quad-cycle) / kernel cycles at 2.4 GHz
                per["avg_resident_waves_at_2p4ghz"] = 4 * wc / (sum(durs) / len(durs) * 2.4)
            sq[k] = per
        traffic["sq_per_launch"] = sq
        with open(os.path.join(dst, f"{args.tag}_summary.md"), "a") as f:
            f.write("\nSQ counters per launch (separate --pmc pass; quad-cycle units):\n\n")
            f.write("| kernel | waves | wave quad-cycles | wait_any | wait_inst_any | active_inst_any | VMEM rd / wr instr | resident waves @2.4 GHz |\n")
            f.write("|---|---|---|---|---|---|---|---|\n")
            for k, per in sorted(sq.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
                if not per.get("SQ_WAVE_CYCLES"):
                    continue
                f.write(f"| `{k[:60]}` | {per.get('SQ_WAVES', 0):.0f} | {per['SQ_WAVE_CYCLES']:.4g} | "
                        f"{per['frac_wait_any']:.2f} | {per['frac_wait_inst_any']:.2f} | {per['frac_active_inst_any']:.2f} | "
                        f"{per.get('SQ_INSTS_VMEM_RD', 0):.3g} / {per.get('SQ_INSTS_VMEM_WR', 0):.3g} | "
                        f"{per.get('avg_resident_waves_at_2p4ghz', 0):.0f} |\n")
    json.dump(traffic, open(os.path.join(dst, f"{args.tag}_traffic.json"), "w"), indent=1)
    if "bytes_per_launch" in traffic:        # the file bench.py reads by default
        json.dump(traffic, open(os.path.join(dst, "traffic.json"), "w"), indent=1)
    print(open(os.path.join(dst, f"{args.tag}_summary.md")).read())


if __name__ == "__main__":
    sys.exit(main())
