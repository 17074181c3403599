#!/bin/bash
# A/B of library builds on the GPU box: bench.py once per prebuilt libnebula_gn.so variant (copied
# over nebula_amd/libnebula_gn.so in turn; the tree's own build is restored at the end).
# Usage: bash scripts/gpu_ab.sh ab/libA.so ab/libB.so ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
cp nebula_amd/libnebula_gn.so gpurun_out/lib_tree.so
rc=0
for v in "$@"; do
    n=$(basename "$v" .so)
    cp "$v" nebula_amd/libnebula_gn.so
    echo "[ab $n]"
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-budget 0 > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err \
        || { echo "bench $n failed"; tail -30 gpurun_out/ab_$n.err; rc=1; break; }
    python3 -c "
import json
d=json.load(open('gpurun_out/ab_$n.json'))
k=d['kernels']
print('  value %.4g ms/step %.3f dev %.3f final %.1fus' % (d['value'], d['ms_per_step'], d['device_ms_per_step'], d['roofline']['avg_launch_us']),
      ' '.join('%s=%.1fus/step' % (n, v['ms']*1e3/d['steps']) for n, v in k.items()))
"
done
cp gpurun_out/lib_tree.so nebula_amd/libnebula_gn.so
exit $rc
