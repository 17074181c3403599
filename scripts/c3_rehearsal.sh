#!/bin/bash
# C3 rehearsal on one GPU box: WORLD ranks (default 8) of tests/c3_rehearsal_worker.py on device 0, the
# frontier exchange over gloo; checks the properties of the worker's docstring and writes
# gpurun_out/c3/summary.json. Usage: bash scripts/c3_rehearsal.sh [scale=26] [world=8] [out|in] [pull_factor]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
scale=${1:-26}; world=${2:-8}; layout=${3:-out}; pf=${4:--1}
out=gpurun_out/c3
mkdir -p "$out"
port=$((20000 + RANDOM % 20000))
pids=()
for r in $(seq 0 $((world - 1))); do
    timeout -k 10 1000 python3 -u tests/c3_rehearsal_worker.py "$r" "$world" "$port" "$out/r$r.json" "$scale" "$layout" "$pf" \
        > "$out/r$r.log" 2>&1 &
    pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=1; done
if [ $rc -ne 0 ]; then echo "a rank failed"; tail -20 "$out"/r*.log; exit 1; fi
python3 - "$out" "$world" <<'PY'
import json, sys
out, world = sys.argv[1], int(sys.argv[2])
rs = [json.load(open(f"{out}/r{r}.json")) for r in range(world)]
summ = {"world": world, "vertices": sum(r["vertices"] for r in rs), "edges": sum(r["edges"] for r in rs),
        "device_gib": sum(r["device_gib"] for r in rs), "load_s_max": max(r["load_s"] for r in rs)}
ok = True
for name in ("lt", "ge", "all"):
    assert all(r[name]["ok"] for r in rs), [r[name]["error"] for r in rs]
    hops = [sum(r[name]["hop_edges"][h] for r in rs) for h in range(len(rs[0][name]["hop_edges"]))]
    summ[name] = {"nrows": sum(r[name]["nrows"] for r in rs), "hop_edges": hops,
                  "pull_hops": [r[name]["pull_hops"] for r in rs], "ms_max": max(r[name]["ms"] for r in rs)}
bfs = rs[0]["bfs_hop_edges"]
bfs_sum = [sum(r["bfs_hop_edges"][h] for r in rs) for h in range(3)]
summ["host_bfs_hop_edges"] = bfs_sum
checks = {
    "hop_edges == host BFS": all(summ[n]["hop_edges"] == bfs_sum for n in ("lt", "ge", "all")),
    "all rows == last-hop edges": summ["all"]["nrows"] == bfs_sum[2],
    "p0<50 + p0>=50 == all": summ["lt"]["nrows"] + summ["ge"]["nrows"] == summ["all"]["nrows"],
    "same pull decisions on every rank": all(len(set(summ[n]["pull_hops"])) == 1 for n in ("lt", "ge", "all")),
}
summ["checks"] = checks
json.dump(summ, open(f"{out}/summary.json", "w"), indent=1)
print(json.dumps(summ, indent=1))
sys.exit(0 if all(checks.values()) else 1)
PY
