# round-5 session 30: gist split kernel with and without its epilogue (timing only)
set -o pipefail
mkdir -p gpurun_out/s30
for v in prod noepi; do
  if [ $v = prod ]; then unset KNN_LIB_PATH; else export KNN_LIB_PATH=$PWD/tools/abx/libknn_$v.so; fi
  timeout -k 10 300 python3 bench.py --workload gist --steps 2 --warmup 1 --no-cpu-baseline --check 0 > gpurun_out/s30/g_$v.log 2>&1 || { tail -20 gpurun_out/s30/g_$v.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*' gpurun_out/s30/g_$v.log | tr '\n' ' '; echo " gist $v"
done
