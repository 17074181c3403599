#!/bin/bash
# GPU parity tests + one bench line (run on the GPU box via gpurun). Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
sel=${1:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --durations=30 --timeout 300 --timeout-method thread $sel > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
