#!/bin/bash
# The full -m gpu suite as the driver runs it, with per-test durations (run on the GPU box via gpurun).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --durations=40 --timeout 600 --timeout-method thread "$@" \
    > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -45 gpurun_out/pytest_gpu.log
