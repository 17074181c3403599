#!/bin/bash
# End-of-round GPU call (r05n): the full -m gpu suite, the default bench line (with the CPU baseline),
# then an A/B of one engine flag against the default. Every step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
bash scripts/gpu_suite.sh || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/bench_default.json'));print('default', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline']['frac_counter'], d['batch_overlaps'], d['cpu_baseline']['value'])"
for v in nt base; do
  a=""; [ $v != base ] && a="--flag final_nt_stores=1"
  timeout -k 10 300 python -u bench.py --cpu-budget 0 $a > gpurun_out/h_$v.json 2> gpurun_out/h_$v.err || { tail -20 gpurun_out/h_$v.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/h_$v.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline']['frac_counter'], d['batch_overlaps'])"
done
