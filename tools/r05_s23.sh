# round-5 session 23: k_dist_split with the next chunk's first fragments read during the chunk before -- parity, A/B against the no-prefetch build (tools/abx)
set -o pipefail
mkdir -p gpurun_out/s23
timeout -k 10 600 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_split_pack.py tests/test_golden.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/s23/tests.log 2>&1 || { tail -40 gpurun_out/s23/tests.log; exit 1; }
tail -1 gpurun_out/s23/tests.log
for r in 1 2; do
for v in pre nopre; do
  if [ $v = nopre ]; then export KNN_LIB_PATH=$PWD/tools/abx/libknn_nopre.so; else unset KNN_LIB_PATH; fi
  timeout -k 10 200 python3 bench.py --workload mnist-real --steps 10 --warmup 3 --no-cpu-baseline --check 8 --secondary-steps 0 > gpurun_out/s23/mr_$v.log 2>&1 || { tail -20 gpurun_out/s23/mr_$v.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*\|"unresolved_queries": [0-9]*\|"mismatches": [0-9]*' gpurun_out/s23/mr_$v.log | tr '\n' ' '; echo " mnist-real $v"
done
done
for v in pre nopre; do
  if [ $v = nopre ]; then export KNN_LIB_PATH=$PWD/tools/abx/libknn_nopre.so; else unset KNN_LIB_PATH; fi
  timeout -k 10 300 python3 bench.py --workload gist --steps 3 --warmup 2 --no-cpu-baseline --check 4 > gpurun_out/s23/gist_$v.log 2>&1 || { tail -20 gpurun_out/s23/gist_$v.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*\|"unresolved_queries": [0-9]*\|"mismatches": [0-9]*' gpurun_out/s23/gist_$v.log | tr '\n' ' '; echo " gist $v"
done
