"""Summarise a tools/calib.sh run (gpurun_out/calib/<tag>) into profiles/<tag>_hbm_calibration.json.

Per pattern of tools/hbm_calib.hip: the HIP-event bandwidth, and counter / known bytes for FETCH_SIZE
(read patterns) and WRITE_SIZE (write patterns), both counters read in KiB as rocprofv3 reports them.
A ratio of 0.5 means the counter shows half the bytes moved (the microarch guide's 16-B read case).
The read ratio of the final hop's own widths is what scripts/prof_summary.py scales FETCH_SIZE by.

Usage: python3 tools/calib_summary.py <tag>
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(path):
    d = collections.defaultdict(list)
    if os.path.exists(path):
        for r in csv.DictReader(open(path)):
            d[r["Kernel_Name"].split("(")[0].replace("void ", "").strip()].append(float(r["Counter_Value"]))
    return d


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r04"
    src = os.path.join(ROOT, "gpurun_out", "calib", tag)
    ev = json.load(open(os.path.join(src, "events.json")))
    fetch = counters(os.path.join(src, "fetch", "run_counter_collection.csv"))
    write = counters(os.path.join(src, "write", "run_counter_collection.csv"))
    out = []
    for p in ev["patterns"]:
        k = p["kernel"]
        if p["dir"] == "mix":
            row = dict(p)
            f, w = fetch.get(k), write.get(k)
            row["fetch_bytes"] = sum(f) / len(f) * 1024 if f else None
            row["write_bytes"] = sum(w) / len(w) * 1024 if w else None
            row["fetch_over_known_read"] = round(row["fetch_bytes"] / p["known_read_bytes"], 4) if f else None
            row["write_over_known_write"] = round(row["write_bytes"] / p["known_write_bytes"], 4) if w else None
            out.append(row)
            continue
        c = fetch.get(k) if p["dir"] == "read" else write.get(k)
        kb = sum(c) / len(c) if c else None
        row = dict(p)
        row["counter"] = "FETCH_SIZE" if p["dir"] == "read" else "WRITE_SIZE"
        row["counter_bytes"] = kb * 1024 if kb is not None else None
        row["counter_over_known"] = round(kb * 1024 / p["known_bytes"], 4) if kb is not None else None
        out.append(row)
    res = {"tag": tag, "buffer_bytes": ev["buffer_bytes"], "tool": "tools/hbm_calib.hip via tools/calib.sh",
           "note": "counter_over_known: the PMC counter (KiB x 1024) over the bytes the pattern moves once "
                   "(for the half gather: every 128-B line of the buffer is touched)", "patterns": out}
    dst = os.path.join(ROOT, "profiles", f"{tag}_hbm_calibration.json")
    json.dump(res, open(dst, "w"), indent=1)
    for r in out:
        if r["dir"] == "mix":
            print(f"{r['kernel']:24s} mix {r['best_ms'] * 1e3:8.1f} us {r['GBps']:8.1f} GB/s  FETCH/read = "
                  f"{r['fetch_over_known_read']}  WRITE/write = {r['write_over_known_write']}")
            continue
        print(f"{r['kernel']:24s} {r['dir']:5s} w{r['width']:<2d} {r['GBps']:8.1f} GB/s  "
              f"{r['counter']} / known = {r['counter_over_known']}")
    print("->", dst)


if __name__ == "__main__":
    main()
