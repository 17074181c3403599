"""Per-variant final-hop bytes from tools/wprobe.sh's rocprofv3 passes (see tools/wprobe.py).

Usage: python tools/wprobe_summary.py gpurun_out/wprobe/<tag>
Prints, per YIELD variant, the rows, the must-write bytes (rows x written widths), and per launch of
ngx_jit_final: 2 x FETCH_SIZE, WRITE_SIZE (KB counters, x 1024), the write requests and the share of them
that are 64-B requests (TCC_EA0_WRREQ / TCC_EA0_WRREQ_64B), and the durations of the trace pass.
"""
import collections
import csv
import glob
import json
import os
import sys

WIDTH = {"all": 13, "dst": 4, "p0": 1, "p1": 8, "none": 0}


def finals(path, counter=None):
    f = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return []
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(f[0])):
        if "ngx_jit_final" not in r["Kernel_Name"]:
            continue
        per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    return [per[k] for k in sorted(per)]


def main():
    d = sys.argv[1]
    meta = json.loads([ln for ln in open(os.path.join(d, "wprobe.json")) if ln.startswith("{")][-1])
    order = meta["order"]
    n = len(order)
    fetch = finals(os.path.join(d, "fetch"))[-n:]
    write = finals(os.path.join(d, "write"))[-n:]
    wreq = finals(os.path.join(d, "wreq"))[-n:]
    tr = glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True)
    durs = []
    if tr:
        rows = sorted(csv.DictReader(open(tr[0])), key=lambda r: int(r["Start_Timestamp"]))
        durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "ngx_jit_final" in r["Kernel_Name"]][-n:]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for i, v in enumerate(order):
        if i < len(fetch) and "FETCH_SIZE" in fetch[i]:
            acc[v]["read"].append(2 * 1024 * fetch[i]["FETCH_SIZE"])
        if i < len(write) and "WRITE_SIZE" in write[i]:
            acc[v]["write"].append(1024 * write[i]["WRITE_SIZE"])
        if i < len(wreq):
            for k, x in wreq[i].items():
                acc[v][k].append(x)
        if i < len(durs):
            acc[v]["us"].append(durs[i])
    out = {}
    for v, info in meta["variants"].items():
        a = acc[v]
        avg = {k: sum(x) / len(x) for k, x in a.items() if x}
        must = info["rows"] * WIDTH.get(v, 0)
        out[v] = dict(rows=info["rows"], must_write=must, **avg)
        w = avg.get("write")
        print(f"{v:5s} rows {info['rows']:>10d} must {must / 1e6:8.1f} MB  write {w / 1e6 if w else float('nan'):8.1f} MB "
              f"(+{(w - must) / max(info['rows'], 1) if w else float('nan'):.2f} B/row)  read {avg.get('read', float('nan')) / 1e6:8.1f} MB  "
              + " ".join(f"{k} {x:.4g}" for k, x in avg.items() if k not in ("read", "write")))
    json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
