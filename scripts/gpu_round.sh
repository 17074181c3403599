#!/bin/bash
# One GPU call: the compact-result tests and the bench A/B (scripts/gpu_compact_ab.sh), then the full
# -m gpu suite with per-test durations. Every step has its own limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash scripts/gpu_compact_ab.sh || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=40 --timeout 600 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -45 gpurun_out/pytest_gpu.log
