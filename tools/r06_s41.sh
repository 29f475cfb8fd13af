# round-6 session 41: the split-pair workgroup order (KNN_XCD_ORDER=2) for
# the split filter -- split-path GPU tests under it, then mnist-real A/B
# against the default (split-major at its 6 splits)
set -o pipefail
mkdir -p gpurun_out/r06s41
KNN_XCD_ORDER=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_f32.py tests/test_golden.py tests/test_gpu_split_pack.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06s41/tests.log 2>&1 || { tail -40 gpurun_out/r06s41/tests.log; exit 1; }
tail -1 gpurun_out/r06s41/tests.log
for v in p s p s p s; do
  if [ $v = p ]; then export KNN_XCD_ORDER=2; else unset KNN_XCD_ORDER; fi
  timeout -k 10 300 python -u bench.py --workload mnist-real --steps 8 --warmup 1 --no-cpu-baseline --secondary-steps 0 > gpurun_out/r06s41/mr_$v.log 2>&1 || { tail -20 gpurun_out/r06s41/mr_$v.log; exit 1; }
  grep '^{' gpurun_out/r06s41/mr_$v.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.readline()); r = d['roofline']
print('mnist-real $v', round(d['ms_per_step'], 2), 'ms/step kernel', round(r['avg_launch_ms'], 2), 'merge', round(r.get('merge', {}).get('ms_per_step', 0), 3), d['engine']['splits'], d['check']['mismatches'], d['check_all_rows']['mismatches'])"
done
