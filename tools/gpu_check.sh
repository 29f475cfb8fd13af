# GPU session: parity tests then the default bench (no CPU leg).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tc.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/tc.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bc.log 2>&1; echo "bench rc=$?"
grep '^{' gpurun_out/bc.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('VALUE', round(d['value']), 'ms', round(d['ms_per_step'],2), 'dist_ms', round(d['roofline']['avg_launch_ms'],2), 'frac', round(d['roofline']['frac'],4), d['engine'], d['check'])"
