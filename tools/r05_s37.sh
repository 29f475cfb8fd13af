# round-5 session 37: k_dist_split A-fragment depth 3 (no scratch) vs 4 (16 B of scratch) for the <= 24-entry kernels
set -o pipefail
mkdir -p gpurun_out/s37
export KNN_LIB_PATH=$PWD/tools/abx/libknn_d3.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_split_pack.py tests/test_golden.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/s37/tests.log 2>&1 || { tail -30 gpurun_out/s37/tests.log; exit 1; }
echo "D=3 $(tail -1 gpurun_out/s37/tests.log)"
for r in 1 2 3; do
for v in d4 d3; do
  if [ $v = d3 ]; then export KNN_LIB_PATH=$PWD/tools/abx/libknn_d3.so; else unset KNN_LIB_PATH; fi
  timeout -k 10 200 python3 bench.py --workload mnist-real --steps 10 --warmup 3 --no-cpu-baseline --check 8 --secondary-steps 0 > gpurun_out/s37/mr_$v.log 2>&1 || { tail -20 gpurun_out/s37/mr_$v.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*\|"unresolved_queries": [0-9]*\|"mismatches": [0-9]*' gpurun_out/s37/mr_$v.log | tr '\n' ' '; echo " mnist-real $v"
done
done
