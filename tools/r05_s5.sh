# round-5 session 5: gist split-count / workgroup-order sweep on k_dist_split (time + FETCH_SIZE)
set -o pipefail
mkdir -p gpurun_out/s5
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in "2 0" "4 0" "8 0" "16 0" "2 1" "8 1"; do
  set -- $cfg
  export KNN_SPLITS=$1
  if [ "$2" = 1 ]; then export KNN_XCD_ORDER=1; else unset KNN_XCD_ORDER; fi
  timeout -k 10 200 python3 bench.py --workload gist --steps 2 --warmup 1 --no-cpu-baseline --check 0 > gpurun_out/s5/gist_s$1_x$2.log 2>&1 || { tail -20 gpurun_out/s5/gist_s$1_x$2.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*\|"unresolved_queries": [0-9]*\|"exposed_merge_ms_per_step": [0-9.]*' gpurun_out/s5/gist_s$1_x$2.log | tr '\n' ' '; echo " gist splits=$1 xord=$2"
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s5/pmc_s$1_x$2 -o run --pmc FETCH_SIZE -- python3 bench.py --workload gist --no-cpu-baseline --secondary-steps 0 --check 0 --steps 1 --warmup 0 > gpurun_out/s5/pmc_s$1_x$2.log 2>&1 || { tail -20 gpurun_out/s5/pmc_s$1_x$2.log; exit 1; }
done
