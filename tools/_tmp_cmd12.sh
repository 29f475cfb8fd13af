set -o pipefail
mkdir -p gpurun_out
bash tools/gpu.sh tests || exit $?
for cfg in "X=1" "KNN_SPLITS=6" "KNN_SPLITS=6 KNN_NO_RESEARCH8=1" "KNN_SPLITS=7" "KNN_SPLITS=8" "KNN_SPLITS=5"; do
  env $cfg timeout -k 10 300 python -u bench.py --workload mnist --steps 20 --warmup 3 --no-cpu-baseline --secondary-steps 0 --check 0 > gpurun_out/b12.log 2>&1 || { tail -5 gpurun_out/b12.log; exit 1; }
  echo "mnist $cfg $(grep '^{' gpurun_out/b12.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), d["engine"], round(d["roofline"]["avg_launch_ms"],4), round(d["roofline"]["exposed_merge_ms_per_step"],4))')"
done
for cfg in "X=1" "KNN_SPLITS=5" "KNN_SPLITS=4" "KNN_SPLITS=3"; do
  env $cfg timeout -k 10 300 python -u bench.py --workload sift --steps 3 --warmup 1 --no-cpu-baseline --check 0 > gpurun_out/b12.log 2>&1 || { tail -5 gpurun_out/b12.log; exit 1; }
  echo "sift $cfg $(grep '^{' gpurun_out/b12.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), d["engine"], round(d["roofline"]["avg_launch_ms"],4), round(d["roofline"]["exposed_merge_ms_per_step"],4))')"
done
