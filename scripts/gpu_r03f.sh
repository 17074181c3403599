#!/bin/bash
# r03f: 512-thread final-hop workgroups (NGX_FINAL_WG=512): parity subset under it, then bench A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
NGX_FINAL_WG=512 timeout -k 10 600 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_configs.py tests/test_gpu_semantics.py "tests/test_gpu_parity.py" -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_r03f.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_r03f.log; exit 1; }
tail -3 gpurun_out/pytest_r03f.log
bash scripts/gpu_iter.sh - none NGX_FINAL_WG=512 || exit 1
