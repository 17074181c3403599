"""Per-step kernel timeline of a bench run under `rocprofv3 --kernel-trace` (timed C2 steps only):
every kernel's duration and the GPU idle gap before it, in microseconds, and the gap between steps.

Usage: python scripts/timeline.py gpurun_out/prof/<tag> [--steps N]
"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=4)
    args = ap.parse_args()
    f = glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    steps, cur = [], None
    for r in rows:
        n = r["Kernel_Name"]
        if "k_seed_lookup" in n:
            cur = [r]
        elif cur is not None:
            cur.append(r)
            if "k_final_close" in n:
                steps.append(cur)
                cur = None

    def dur(r):
        return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000

    # the timed steps write compact results: their final hop is the short one
    timed = [s for s in steps if any("ngx_jit_final" in r["Kernel_Name"] and dur(r) < 350 for r in s)]
    for st in timed[2:2 + args.steps]:
        t0, prev, line = int(st[0]["Start_Timestamp"]), None, []
        busy = 0.0
        for r in st:
            s = int(r["Start_Timestamp"])
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ngx::", "")[:20]
            gap = (s - prev) / 1000 if prev else 0.0
            line.append(f"{name}:{dur(r):.1f}(+{gap:.1f})")
            busy += dur(r)
            prev = int(r["End_Timestamp"])
        print(f"span {(prev - t0) / 1000:.1f} us, kernels {busy:.1f} us: " + " ".join(line))
    for a, b in zip(timed[2:2 + args.steps], timed[3:3 + args.steps]):
        print("gap between steps %.1f us" % ((int(b[0]["Start_Timestamp"]) - int(a[-1]["End_Timestamp"])) / 1000))


if __name__ == "__main__":
    main()
