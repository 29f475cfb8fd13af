# round-5 session 3: RCCL self transport + ring-rank re-search + k_dist_split parity, then split A/B and mnist bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_s8.py tests/test_gpu_f32.py tests/test_golden.py tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/s3_tests.log 2>&1 || { tail -40 gpurun_out/s3_tests.log; exit 1; }
tail -2 gpurun_out/s3_tests.log
for v in new v1; do
  if [ $v = v1 ]; then export KNN_SPLIT_V1=1; else unset KNN_SPLIT_V1; fi
  timeout -k 10 300 python3 bench.py --workload mnist-real --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/s3_mr_$v.log 2>&1 || { tail -20 gpurun_out/s3_mr_$v.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*\|"unresolved_queries": [0-9]*\|"mismatches": [0-9]*\|"frac": [0-9.]*\|"splits": [0-9]*' gpurun_out/s3_mr_$v.log | tr '\n' ' '; echo " mnist-real $v"
  timeout -k 10 300 python3 bench.py --workload gist --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/s3_gist_$v.log 2>&1 || { tail -20 gpurun_out/s3_gist_$v.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*\|"unresolved_queries": [0-9]*\|"mismatches": [0-9]*\|"frac": [0-9.]*\|"splits": [0-9]*' gpurun_out/s3_gist_$v.log | tr '\n' ' '; echo " gist $v"
done
unset KNN_SPLIT_V1
timeout -k 10 300 python3 bench.py --workload mnist --steps 20 --warmup 5 > gpurun_out/s3_mnist.log 2>&1 || { tail -20 gpurun_out/s3_mnist.log; exit 1; }
grep '^{' gpurun_out/s3_mnist.log | tail -1
