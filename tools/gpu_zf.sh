# Survivor-mask change: GPU tests, shadow-kernel ablations, mnist + sift benches.
set -o pipefail
mkdir -p gpurun_out/zf
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/zf/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/zf/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/probe/kbench16 > gpurun_out/zf/kb16.log 2>&1 || exit 1
head -5 gpurun_out/zf/kb16.log
for wl in mnist sift; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/zf/bench_$wl.log 2>&1
  rc=$?; echo "bench $wl rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' gpurun_out/zf/bench_$wl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl VALUE', round(d['value']), 'ms', round(d['ms_per_step'],2), 'dist_ms', round(d['roofline']['avg_launch_ms'],2), d['engine'], d['check'])"
done
