"""Two-lane kernel timeline of a pipelined bench run under `rocprofv3 --kernel-trace` (ngx_go_batch with
batch_pipeline: consecutive queries on two HIP streams). Prints, for a window of the timed steps, every
kernel's queue, start (us from the window start), duration and name, and per final hop the kernels of
the other queue that ran inside it.

Usage: python scripts/lanes_timeline.py gpurun_out/prof/<tag> [--skip N] [--count N]
"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--skip", type=int, default=8, help="final hops to skip (warmup, untimed)")
    ap.add_argument("--count", type=int, default=3, help="final hops to show")
    args = ap.parse_args()
    f = glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    qkey = "Queue_Id" if "Queue_Id" in rows[0] else "Stream_Id"
    finals = [i for i, r in enumerate(rows) if "ngx_jit_final" in r["Kernel_Name"] or "k_final<" in r["Kernel_Name"]]
    sel = finals[args.skip:args.skip + args.count]
    if not sel:
        print("no final hops in range")
        return
    lo = max(0, sel[0] - 12)
    hi = min(len(rows), sel[-1] + 12)
    t0 = int(rows[lo]["Start_Timestamp"])

    def us(x):
        return (int(x) - t0) / 1000

    for r in rows[lo:hi]:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ngx::", "")[:28]
        s, e = us(r["Start_Timestamp"]), us(r["End_Timestamp"])
        print(f"q{r[qkey]:>3} {s:9.1f} {e - s:7.1f}  {name}")
    for i in sel:
        fr = rows[i]
        s, e = int(fr["Start_Timestamp"]), int(fr["End_Timestamp"])
        inside = [r for r in rows if r[qkey] != fr[qkey] and int(r["Start_Timestamp"]) < e and int(r["End_Timestamp"]) > s]
        print(f"final on q{fr[qkey]} {(e - s) / 1000:.1f} us; other queue inside it: "
              + ", ".join(r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ngx::", "")[:16] for r in inside))


if __name__ == "__main__":
    main()
