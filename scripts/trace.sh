#!/bin/bash
# Kernel trace + stats of a short bench run (run on the GPU box via gpurun) -> gpurun_out/prof/<tag>/trace,
# Usage: bash scripts/trace.sh <tag> [extra bench args]
set -o pipefail
tag=${1:-trace}
shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/prof/$tag
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run -f csv -- \
    python3 bench.py --steps 10 --warmup 3 --cpu-budget 0 "$@" > "$out/bench_trace.json" 2> "$out/bench_trace.err" \
    || { echo "trace failed"; tail -20 "$out/bench_trace.err"; exit 1; }
ls "$out/trace"
