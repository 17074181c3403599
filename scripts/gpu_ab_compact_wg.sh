#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
for v in w1024 base w1024b baseb; do
  a=""; case $v in w1024*) a="--flag compact_wg=1024";; esac
  timeout -k 10 300 python -u bench.py --cpu-budget 0 $a > gpurun_out/h_$v.json 2> gpurun_out/h_$v.err || { tail -20 gpurun_out/h_$v.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/h_$v.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done
