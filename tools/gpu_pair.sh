set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/tc.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/tc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --check 32 > gpurun_out/bc.log 2>&1
rc=$?; echo -n "bench rc=$rc "; grep '^{' gpurun_out/bc.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('VALUE', round(d['value']), 'ms', round(d['ms_per_step'],2), 'dist', round(r['avg_launch_ms'],2), d['check'])"; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
KNN_NO_PAIR=$v timeout -k 10 300 python -u tools/ring_emulate.py --steps 5 > gpurun_out/ring_emu_$v.log 2>&1
rc=$?; echo -n "emu nopair=$v rc=$rc "; grep -E '"[1248]"|rank_ms' gpurun_out/ring_emu_$v.log | tr -d '\n '; echo; [ $rc -eq 0 ] || exit $rc
done
