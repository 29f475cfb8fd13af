# HEAD check: GPU tests, smoke, default bench, ring emulation (P = 1..8).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/tc.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/tc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bc.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/bc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ring_emulate.py > gpurun_out/ring_emu.log 2>&1
rc=$?; echo "emu rc=$rc"; cat gpurun_out/ring_emu.log; exit $rc
