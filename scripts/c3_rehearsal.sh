#!/bin/bash
# C3 on one GPU box: WORLD ranks (default 8) of tests/c3_rehearsal_worker.py on device 0, the frontier
# exchange over gloo, checked by the properties of the worker's docstring; writes gpurun_out/c3/summary.json.
# Usage: bash scripts/c3_rehearsal.sh [scale=26] [world=8] [in|out] [pull_factor]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c3
timeout -k 10 900 python3 -u - "${1:-26}" "${2:-8}" "${3:-in}" "${4:--1}" <<'PY'
import json, sys
sys.path.insert(0, ".")
from tests.test_gpu_c3 import run_c3
summ, checks = run_c3("gpurun_out/c3", world=int(sys.argv[2]), scale=int(sys.argv[1]), layout=sys.argv[3],
                      pull_factor=int(sys.argv[4]))
print(json.dumps(summ, indent=1))
sys.exit(0 if all(checks.values()) else 1)
PY
