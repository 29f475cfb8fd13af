set -o pipefail
mkdir -p gpurun_out
ROOT=$GRAFT_REPO_ROOT
(cd /tmp && export TMPDIR=/tmp && cd "$ROOT" && KNN_SPLITS=6 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/tr6 -o run -- python3 bench.py --workload mnist --no-cpu-baseline --secondary-steps 0 --check 0 --steps 6 --warmup 2 > gpurun_out/tr6.log 2>&1) || exit 1
echo trace done
for cfg in "KNN_SPLITS=7" "KNN_SPLITS=7 KNN_NO_QSUM=1" "KNN_SPLITS=8" "KNN_SPLITS=10" "KNN_SPLITS=12" "KNN_SPLITS=8 KNN_NO_QSUM=1" "KNN_SPLITS=7 KNN_NO_RESEARCH8=1" "KNN_SPLITS=10 KNN_NO_RESEARCH8=1"; do
  env $cfg timeout -k 10 300 python -u bench.py --workload mnist --steps 20 --warmup 3 --no-cpu-baseline --secondary-steps 0 --check 0 > gpurun_out/b9.log 2>&1 || { tail -5 gpurun_out/b9.log; exit 1; }
  echo "$cfg $(grep '^{' gpurun_out/b9.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), d["engine"], round(d["roofline"]["avg_launch_ms"],4), round(d["roofline"]["exposed_merge_ms_per_step"],4))')"
done
