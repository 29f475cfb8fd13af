# round-5 session 29: a short last split filling the int8 grid's partial last round (i8_tail) -- parity, A/B, emulation
set -o pipefail
mkdir -p gpurun_out/s29
timeout -k 10 600 python -u -m pytest tests/test_gpu_i8.py tests/test_gpu_s8.py tests/test_golden.py tests/test_gpu_parity.py tests/test_gpu_fullsize_ring.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/s29/tests.log 2>&1 || { tail -40 gpurun_out/s29/tests.log; exit 1; }
tail -1 gpurun_out/s29/tests.log
for r in 1 2 3; do
for v in 1 0; do
  export KNN_I8_TAIL=$v
  timeout -k 10 200 python3 bench.py --workload mnist --steps 20 --warmup 3 --no-cpu-baseline --check 8 --secondary-steps 0 > gpurun_out/s29/mn_$v.log 2>&1 || { tail -20 gpurun_out/s29/mn_$v.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*\|"splits": [0-9]*\|"unresolved_queries": [0-9]*\|"mismatches": [0-9]*' gpurun_out/s29/mn_$v.log | tr '\n' ' '; echo " mnist TAIL=$v"
done
done
unset KNN_I8_TAIL
timeout -k 10 300 python -u tools/ring_emulate.py --workload mnist --ranks 1,2,4,8 --steps 8 > gpurun_out/s29/emu_mn.log 2>&1 || { tail -20 gpurun_out/s29/emu_mn.log; exit 1; }
grep '"P"' gpurun_out/s29/emu_mn.log | cut -c1-200
