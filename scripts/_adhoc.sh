export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_batch.log 2>&1 || { tail -30 gpurun_out/t_batch.log; exit 1; }
tail -2 gpurun_out/t_batch.log
for v in l2 l3 l3yo; do
  a=""; [ $v = l2 ] && a="--flag batch_lanes=2"; [ $v = l3yo ] && a="--yield-only"
  timeout -k 10 400 python -u bench.py --steps 50 --warmup 5 --cpu-budget 0 $a > gpurun_out/h_$v.json 2> gpurun_out/h_$v.err || { tail -20 gpurun_out/h_$v.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/h_$v.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['batch_overlaps'])"
done
