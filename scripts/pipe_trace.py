"""Merge a pipelined batch's host marks (NGX_PIPE_TRACE=1, '[ngx pipe] <ns> q<i> <what>' on stderr, CLOCK_MONOTONIC)
with the rocprofv3 kernel trace of the same run (Start/End_Timestamp, same clock on Linux): one timeline in
microseconds from the batch's first mark, host lines prefixed 'H', kernel lines 'K q<queue>'.

Usage: python scripts/pipe_trace.py <dir with bench.err and trace/> [--batch N] [--us MAX]
"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--batch", type=int, default=-1, help="which dumped batch (default: the last)")
    ap.add_argument("--us", type=float, default=2500.0)
    args = ap.parse_args()
    batches, cur = [], []
    for line in open(os.path.join(args.dir, "bench.err")):
        if not line.startswith("[ngx pipe]"):
            continue
        parts = line.split(None, 4)
        if parts[2] == "clocks":
            if cur:
                batches.append(cur)
            cur = []
            continue
        cur.append((int(parts[2]), "H", parts[3] + " " + parts[4].strip() if len(parts) > 4 else parts[3]))
    if cur:
        batches.append(cur)
    marks = batches[args.batch]
    t0 = marks[0][0]
    t1 = marks[-1][0]
    f = glob.glob(os.path.join(args.dir, "trace", "**", "*kernel_trace.csv"), recursive=True)[0]
    ev = list(marks)
    for r in csv.DictReader(open(f)):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e < t0 or s > t1:
            continue
        ev.append((s, "K", f"q{r['Queue_Id']} {r['Kernel_Name'][:40]} ({(e - s) / 1e3:.1f} us, ends {(e - t0) / 1e3:.1f})"))
    ev.sort()
    for t, kind, what in ev:
        us = (t - t0) / 1e3
        if us > args.us:
            break
        print(f"{us:9.1f} {kind} {what}")


if __name__ == "__main__":
    main()
