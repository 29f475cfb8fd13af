# GPU tests, then mnist and sift benches (no CPU leg) at the current build.
set -o pipefail
mkdir -p gpurun_out/ab2
timeout -k 10 400 python -u -m pytest tests/ -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/ab2/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/ab2/pytest.log; [ $rc -eq 0 ] || exit $rc
for wl in mnist sift; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab2/bench_$wl.log 2>&1
  rc=$?; echo "bench $wl rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' gpurun_out/ab2/bench_$wl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl VALUE', round(d['value']), 'ms', round(d['ms_per_step'],2), 'dist_ms', round(d['roofline']['avg_launch_ms'],2), d['engine'], d['check'])"
done
