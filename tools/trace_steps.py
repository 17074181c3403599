"""Per-launch view of a rocprofv3 kernel trace (scripts/trace.sh): the kernels of the last timed step in
launch order with their durations and the gaps between them, and per-kernel averages.

Usage: python tools/trace_steps.py gpurun_out/prof/<tag>/trace/run_kernel_trace.csv [--first-kernel SUBSTR]
"""
import argparse
import collections
import csv


def short(n):
    return n.split("(")[0].replace("void ", "").strip()[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--first-kernel", default="k_seed_frontier", help="kernel that starts a step")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    avg = collections.defaultdict(list)
    for r in rows:
        avg[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    starts = [i for i, r in enumerate(rows) if a.first_kernel in r["Kernel_Name"]]
    if len(starts) >= 2:
        lo, hi = starts[-2], starts[-1]
        print("step (launch order): kernel, us, gap before (us)")
        prev = None
        for r in rows[lo:hi]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            gap = (s - prev) / 1e3 if prev else 0.0
            print(f"  {short(r['Kernel_Name']):60s} {(e - s) / 1e3:9.2f} {gap:9.2f}")
            prev = e
        print(f"  step span {(int(rows[hi - 1]['End_Timestamp']) - int(rows[lo]['Start_Timestamp'])) / 1e3:.1f} us")
    print("per kernel: launches, avg us, total ms")
    for k, v in sorted(avg.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {k:60s} {len(v):6d} {sum(v) / len(v):9.2f} {sum(v) / 1e3:9.3f}")


if __name__ == "__main__":
    main()
