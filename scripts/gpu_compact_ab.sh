set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_compact.py "tests/test_gpu_configs.py::test_c2_bench_step_vs_oracle" -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/pytest_compact.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_compact.log; exit 1; }
tail -5 gpurun_out/pytest_compact.log
for v in compact wide nox; do
  extra=""; [ $v = wide ] && extra="--no-compact"; pre=""; [ $v = nox ] && pre="NGX_PULL_XCD=0"
  env $pre timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-budget 0 $extra > gpurun_out/bench_$v.json 2> gpurun_out/bench_$v.err || { echo "bench $v failed"; tail -30 gpurun_out/bench_$v.err; exit 1; }
  python3 -c "
import json
d=json.load(open('gpurun_out/bench_$v.json'))
print('$v', 'value %.4g ms/step %.3f dev %.3f final %.1fus' % (d['value'], d['ms_per_step'], d['device_ms_per_step'], d['roofline']['avg_launch_us']), ' '.join('%s=%.1f' % (n, v['ms']*1e3/d['steps']) for n, v in d['kernels'].items()))
"
done
