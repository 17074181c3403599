#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box via gpurun):
#   1. kernel trace + stats of a short bench run           -> gpurun_out/prof/<tag>/trace
#   2. PMC pass FETCH_SIZE on the final-hop / expand kernels -> gpurun_out/prof/<tag>/fetch
#   3. PMC pass WRITE_SIZE on the same kernels              -> gpurun_out/prof/<tag>/write
# Each pass has its own time limit; the script stops at the first failing step.
# Usage: bash scripts/profile.sh <tag> [extra bench args]
set -o pipefail
tag=${1:-r01}
shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/prof/$tag
mkdir -p "$out"
args="--steps 10 --warmup 3 --cpu-budget 0 $*"
echo "[profile] trace: bench.py $args"
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats -d "$out/trace" -o run -f csv -- \
    python3 bench.py $args > "$out/bench_trace.json" 2> "$out/bench_trace.err" || { echo "trace pass failed"; tail -20 "$out/bench_trace.err"; exit 1; }
regex='ngx_jit|k_expand|k_final|k_tile|k_compact|k_lookup|k_chunk|k_pull|k_seed|k_copy'
echo "[profile] pmc FETCH_SIZE"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$regex" -d "$out/fetch" -o run -f csv -- \
    python3 bench.py $args > "$out/bench_fetch.json" 2> "$out/bench_fetch.err" || { echo "fetch pass failed"; tail -20 "$out/bench_fetch.err"; exit 1; }
echo "[profile] pmc WRITE_SIZE"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$regex" -d "$out/write" -o run -f csv -- \
    python3 bench.py $args > "$out/bench_write.json" 2> "$out/bench_write.err" || { echo "write pass failed"; tail -20 "$out/bench_write.err"; exit 1; }
if [ -n "$SQPASS" ]; then
echo "[profile] pmc SQ"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-include-regex "$regex" -d "$out/sq" -o run -f csv -- \
    python3 bench.py $args > "$out/bench_sq.json" 2> "$out/bench_sq.err" || { echo "sq pass failed"; tail -20 "$out/bench_sq.err"; exit 1; }
fi
find "$out" -name '*.csv' | head -20
echo "[profile] done"
