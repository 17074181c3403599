#!/bin/bash
# r03d: two-pass final hop. Parity subset (NBA GoTest cases on the generated kernels, compact results,
# the C2 bench step vs the oracle), then bench with and without the count pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_configs.py tests/test_gpu_semantics.py tests/test_gpu_jit_async.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/pytest_r03d.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_r03d.log; exit 1; }
tail -3 gpurun_out/pytest_r03d.log
bash scripts/gpu_iter.sh - none NGX_FINAL_2PASS=0 || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/bench_v1.json')); print('jit', d['jit']); print('roofline', d['roofline']); print('path', d['path_roofline'])"
