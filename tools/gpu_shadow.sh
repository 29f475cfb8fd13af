set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/tc.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/tc.log; [ $rc -eq 0 ] || exit $rc
for wl in mnist sift; do for v in 0 1; do
  KNN_NO_SHADOW=$v timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --check 32 > gpurun_out/sh_${wl}_$v.log 2>&1
  rc=$?; echo -n "$wl no_shadow=$v rc=$rc "; grep '^{' gpurun_out/sh_${wl}_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('VALUE', round(d['value']), 'ms', round(d['ms_per_step'],2), 'dist', round(r['avg_launch_ms'],2), d['check'])"; [ $rc -eq 0 ] || exit $rc
done; done
