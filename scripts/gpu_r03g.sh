#!/bin/bash
# r03g: the full -m gpu suite on the final build (defaults), then bench A/B with 512-thread final workgroups.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --durations=15 --timeout 600 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
bash scripts/gpu_iter.sh - none NGX_FINAL_WG=512 || exit 1
