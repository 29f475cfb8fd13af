# One tuning iteration on the GPU box: parity tests, kbench ablations, bench.
# Stops at the first failing step (no GPU work after a fault / timeout).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tc.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/tc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 ./tools/probe/kbench > gpurun_out/kb.log 2>&1
rc=$?; echo "kbench rc=$rc"; cat gpurun_out/kb.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bc.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bc.log; exit $rc; }
grep '^{' gpurun_out/bc.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('VALUE', round(d['value']), 'ms', round(d['ms_per_step'],2), 'dist_ms', round(d['roofline']['avg_launch_ms'],2), 'frac', round(d['roofline']['frac'],4), d['engine'], d['check'])"
