# round-5 session 27: int8 half-tile kernel with a two-K-step A-fragment lead (barrier at the chunk start) -- int8 parity, A/B against the lead-1 build
set -o pipefail
mkdir -p gpurun_out/s27
timeout -k 10 600 python -u -m pytest tests/test_gpu_i8.py tests/test_gpu_s8.py tests/test_golden.py tests/test_gpu_parity.py tests/test_gpu_fullsize_ring.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/s27/tests.log 2>&1 || { tail -40 gpurun_out/s27/tests.log; exit 1; }
tail -1 gpurun_out/s27/tests.log
for r in 1 2; do
for v in al2 al1; do
  if [ $v = al1 ]; then export KNN_LIB_PATH=$PWD/tools/abx/libknn_al1.so; else unset KNN_LIB_PATH; fi
  timeout -k 10 200 python3 bench.py --workload mnist --steps 20 --warmup 3 --no-cpu-baseline --check 8 --secondary-steps 0 > gpurun_out/s27/mn_$v.log 2>&1 || { tail -20 gpurun_out/s27/mn_$v.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*\|"unresolved_queries": [0-9]*\|"mismatches": [0-9]*' gpurun_out/s27/mn_$v.log | tr '\n' ' '; echo " mnist $v"
done
done
unset KNN_LIB_PATH
timeout -k 10 300 python -u tools/ring_emulate.py --workload mnist --ranks 1,8 --steps 8 > gpurun_out/s27/emu_mn.log 2>&1 || { tail -20 gpurun_out/s27/emu_mn.log; exit 1; }
grep '"P"' gpurun_out/s27/emu_mn.log | cut -c1-160
