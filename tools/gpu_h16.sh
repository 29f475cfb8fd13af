# fp16-contraction (H16) check: fp32 GPU tests, then sift bench with and without it.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32.py tests/test_golden.py -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tc_h16.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/tc_h16.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  KNN_NO_H16=$v timeout -k 10 300 python -u bench.py --workload sift --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sift_h16_$v.log 2>&1
  rc=$?; echo "sift KNN_NO_H16=$v rc=$rc"; grep '^{' gpurun_out/sift_h16_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('VALUE', round(d['value']), 'ms', round(d['ms_per_step'],1), 'dist', round(r['avg_launch_ms'],1), 'TF', round(r['achieved'],1), 'merge', round(r['exposed_merge_ms_per_step'],1), d['engine'], d['check'])"; [ $rc -eq 0 ] || exit $rc
done
