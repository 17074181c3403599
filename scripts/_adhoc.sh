#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
out=gpurun_out/prof/r05j_pipe; mkdir -p $out
NGX_PIPE_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace -d "$out/trace" -o run -f csv -- \
    python3 bench.py --steps 12 --warmup 3 --cpu-budget 0 > "$out/bench.json" 2> "$out/bench.err" || { echo "pipe trace failed"; tail -20 "$out/bench.err"; exit 1; }
grep -c "ngx pipe" $out/bench.err
