#!/bin/bash
# r03c: bench variants of the compact build (env knobs), then the rocprofv3 evidence of the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash scripts/gpu_iter.sh - none NGX_EAGER_SKIP=1 NGX_JIT_WAVES=8 NGX_JIT_WAVES=4 NGX_PULL_KH=1 NGX_PULL_WIN=1 || exit 1
bash scripts/profile.sh r03c || exit 1
