# round-5 session 26: does the query-fragment load stall k_dist_split? noepi vs noepi + no query loads (timing only: the latter's results are wrong)
set -o pipefail
mkdir -p gpurun_out/s26
for r in 1 2; do
for v in prod noepi noepi_noq; do
  if [ $v = prod ]; then unset KNN_LIB_PATH; else export KNN_LIB_PATH=$PWD/tools/abx/libknn_$v.so; fi
  timeout -k 10 200 python3 bench.py --workload mnist-real --steps 5 --warmup 2 --no-cpu-baseline --check 0 --secondary-steps 0 > gpurun_out/s26/mr_$v.log 2>&1 || { tail -20 gpurun_out/s26/mr_$v.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*' gpurun_out/s26/mr_$v.log | tr '\n' ' '; echo " mnist-real $v"
done
done
