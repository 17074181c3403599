#!/bin/bash
# A GPU A/B of one engine flag against the default bench line, after the batch tests.
# Usage: bash scripts/gpu_ab_flag.sh NAME=VALUE
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_batch.log 2>&1 || { tail -30 gpurun_out/t_batch.log; exit 1; }
tail -2 gpurun_out/t_batch.log
for v in flag base flag2; do
  a=""; [ $v != base ] && a="--flag $1"
  timeout -k 10 300 python -u bench.py --cpu-budget 0 $a > gpurun_out/h_$v.json 2> gpurun_out/h_$v.err || { tail -20 gpurun_out/h_$v.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/h_$v.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['batch_overlaps'])"
done
