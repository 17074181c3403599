#!/bin/bash
# GPU-box half of the HBM counter calibration (tools/hbm_calib.hip): HIP-event bandwidth per pattern,
# then one rocprofv3 --pmc pass per counter (FETCH_SIZE, WRITE_SIZE), each under its own time limit.
# Summarise afterwards on the CPU side: python3 tools/calib_summary.py <tag>
set -o pipefail
tag=${1:-r04}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/calib/$tag
mkdir -p "$out"
timeout -k 10 120 ./tools/bin/hbm_calib 2048 3 > "$out/events.json" || { echo "calib run failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_calib -d "$out/fetch" -o run -f csv -- \
    ./tools/bin/hbm_calib 2048 1 > "$out/fetch.json" 2> "$out/fetch.err" || { echo "fetch pass failed"; tail -20 "$out/fetch.err"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_calib -d "$out/write" -o run -f csv -- \
    ./tools/bin/hbm_calib 2048 1 > "$out/write.json" 2> "$out/write.err" || { echo "write pass failed"; tail -20 "$out/write.err"; exit 1; }
find "$out" -name '*.csv'
echo "[calib] done"
