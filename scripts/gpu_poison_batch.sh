#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
NGX_POISON=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_poison.py tests/test_gpu_yield_only.py tests/test_gpu_configs.py -k "batch or poison or yield_only or c2" -x -q --timeout 400 --timeout-method thread > gpurun_out/poison_r05n.log 2>&1 || { tail -40 gpurun_out/poison_r05n.log; exit 1; }
tail -3 gpurun_out/poison_r05n.log
