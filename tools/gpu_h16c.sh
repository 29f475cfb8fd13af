set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/tc.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/tc.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  KNN_NO_H16=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --check 64 > gpurun_out/mnist_h16_$v.log 2>&1
  rc=$?; echo "mnist KNN_NO_H16=$v rc=$rc"; grep '^{' gpurun_out/mnist_h16_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('VALUE', round(d['value']), 'ms', round(d['ms_per_step'],2), 'dist', round(r['avg_launch_ms'],2), 'TF', round(r['achieved'],1), r['mfma_input'], 'merge', round(r['exposed_merge_ms_per_step'],2), d['engine'], d['check'])"; [ $rc -eq 0 ] || exit $rc
done
