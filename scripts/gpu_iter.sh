#!/bin/bash
# Iteration run on the GPU box: a pytest selection, then bench.py once per environment variant.
# Usage: bash scripts/gpu_iter.sh "<pytest args>" "<VAR=val ...>" ["<VAR=val ...>" ...]
# ("-" as the pytest args skips the tests; "none" as a variant runs the bench with no extra env;
# "args:<bench args>" passes bench arguments instead, e.g. "args:--flag dyn_hops=1")
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
sel=${1:--}
shift || true
if [ "$sel" != "-" ]; then
    timeout -k 10 900 python -u -m pytest $sel -m gpu -x -v --timeout 300 --timeout-method thread \
        > gpurun_out/pytest_iter.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_iter.log; exit 1; }
    tail -3 gpurun_out/pytest_iter.log
fi
i=0
for v in "$@"; do
    i=$((i + 1))
    envs=""
    bargs=""
    case "$v" in
        none) ;;
        args:*) bargs="${v#args:}" ;;
        *) envs="$v" ;;
    esac
    echo "[bench $i] $envs $bargs"
    env $envs timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-budget 0 $bargs \
        > gpurun_out/bench_v$i.json 2> gpurun_out/bench_v$i.err || { echo "bench $i failed"; tail -30 gpurun_out/bench_v$i.err; exit 1; }
    python3 -c "
import json,sys
d=json.load(open('gpurun_out/bench_v$i.json'))
k=d['kernels']
print('  value %.4g ms/step %.3f dev %.3f final %.1fus' % (d['value'], d['ms_per_step'], d['device_ms_per_step'], d['roofline']['avg_launch_us']),
      ' '.join('%s=%.1fus/step' % (n, v['ms']*1e3/d['steps']) for n, v in k.items()))
"
done
