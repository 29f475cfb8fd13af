# round-5 session 8: k_dist_split v2 (queries in registers, 4-stage corpus ring, A prefetch 4 m-tiles) parity + timing + ablations
set -o pipefail
mkdir -p gpurun_out/s8
timeout -k 10 600 python -u -m pytest tests/test_gpu_f32.py tests/test_golden.py tests/test_gpu_parity.py tests/test_gpu_config4.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/s8/tests.log 2>&1 || { tail -40 gpurun_out/s8/tests.log; exit 1; }
tail -1 gpurun_out/s8/tests.log
for v in prod noepi noepi_nodma noepi_nofrag noepi_nomfma; do
  if [ $v = prod ]; then unset KNN_LIB_PATH; else export KNN_LIB_PATH=$PWD/tools/abl5/libknn_$v.so; fi
  timeout -k 10 200 python3 bench.py --workload mnist-real --steps 5 --warmup 2 --no-cpu-baseline --check 4 --secondary-steps 0 > gpurun_out/s8/mr_$v.log 2>&1 || { tail -20 gpurun_out/s8/mr_$v.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*\|"unresolved_queries": [0-9]*\|"mismatches": [0-9]*' gpurun_out/s8/mr_$v.log | tr '\n' ' '; echo " mnist-real $v"
done
unset KNN_LIB_PATH
timeout -k 10 300 python3 bench.py --workload gist --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/s8/gist.log 2>&1 || { tail -20 gpurun_out/s8/gist.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*\|"unresolved_queries": [0-9]*\|"mismatches": [0-9]*\|"frac": [0-9.]*' gpurun_out/s8/gist.log | tr '\n' ' '; echo " gist"
