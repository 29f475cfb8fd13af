# round-5 session 31: gist at 1 vs 2 corpus splits (fewer lane lists, a 15.3-round grid)
set -o pipefail
mkdir -p gpurun_out/s31
for v in 1 2 3; do
  export KNN_SPLITS=$v
  timeout -k 10 300 python3 bench.py --workload gist --steps 2 --warmup 1 --no-cpu-baseline --check 4 > gpurun_out/s31/g_$v.log 2>&1 || { tail -20 gpurun_out/s31/g_$v.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*\|"unresolved_queries": [0-9]*\|"mismatches": [0-9]*' gpurun_out/s31/g_$v.log | tr '\n' ' '; echo " gist splits=$v"
done
