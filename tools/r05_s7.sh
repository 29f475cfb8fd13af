# round-5 session 7: int8 two-groups-a-wave long-row kernel (KNN_I8_QG2L=1) parity + A/B; k_dist_split ablations
set -o pipefail
mkdir -p gpurun_out/s7
KNN_I8_QG2L=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_i8.py tests/test_golden.py tests/test_gpu_s8.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/s7/tests_qg2l.log 2>&1 || { tail -40 gpurun_out/s7/tests_qg2l.log; exit 1; }
tail -1 gpurun_out/s7/tests_qg2l.log
for r in 1 2; do
for v in 0 1; do
  export KNN_I8_QG2L=$v
  timeout -k 10 200 python3 bench.py --workload mnist --steps 20 --warmup 5 --no-cpu-baseline --secondary-steps 0 > gpurun_out/s7/mnist_q$v.log 2>&1 || { tail -20 gpurun_out/s7/mnist_q$v.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*\|"unresolved_queries": [0-9]*\|"mismatches": [0-9]*\|"splits": [0-9]*' gpurun_out/s7/mnist_q$v.log | tr '\n' ' '; echo " mnist QG2L=$v"
done
done
unset KNN_I8_QG2L
for v in prod noepi noepi_nodma noepi_nofrag noepi_nomfma; do
  if [ $v = prod ]; then unset KNN_LIB_PATH; else export KNN_LIB_PATH=$PWD/tools/abl5/libknn_$v.so; fi
  timeout -k 10 200 python3 bench.py --workload mnist-real --steps 5 --warmup 2 --no-cpu-baseline --check 0 --secondary-steps 0 > gpurun_out/s7/mr_$v.log 2>&1 || { tail -20 gpurun_out/s7/mr_$v.log; exit 1; }
  grep -o '"avg_launch_ms": [0-9.]*' gpurun_out/s7/mr_$v.log | tr '\n' ' '; echo " mnist-real $v"
done
