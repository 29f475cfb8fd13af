set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_s8.py tests/test_gpu_i8.py -x -q --timeout 150 --timeout-method thread > gpurun_out/pt10.log 2>&1 || { tail -20 gpurun_out/pt10.log; exit 1; }
tail -1 gpurun_out/pt10.log
for cfg in "X=1" "KNN_SPLITS=8" "KNN_SPLITS=6" "KNN_SPLITS=7"; do
  env $cfg timeout -k 10 300 python -u bench.py --workload mnist --steps 20 --warmup 3 --no-cpu-baseline --secondary-steps 0 --check 0 > gpurun_out/b10.log 2>&1 || { tail -5 gpurun_out/b10.log; exit 1; }
  echo "mnist $cfg $(grep '^{' gpurun_out/b10.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), d["engine"], round(d["roofline"]["avg_launch_ms"],4), round(d["roofline"]["exposed_merge_ms_per_step"],4))')"
done
for cfg in "X=1" "KNN_SPLITS=5" "KNN_SPLITS=3"; do
  env $cfg timeout -k 10 300 python -u bench.py --workload sift --steps 3 --warmup 1 --no-cpu-baseline --check 0 > gpurun_out/b10.log 2>&1 || { tail -5 gpurun_out/b10.log; exit 1; }
  echo "sift $cfg $(grep '^{' gpurun_out/b10.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), d["engine"], round(d["roofline"]["avg_launch_ms"],4), round(d["roofline"]["exposed_merge_ms_per_step"],4))')"
done
(cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && KNN_SPLITS=6 KNN_NO_RESEARCH8=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/tr6r -o run -- python3 bench.py --workload mnist --no-cpu-baseline --secondary-steps 0 --check 0 --steps 4 --warmup 1 > gpurun_out/tr6r.log 2>&1) || exit 1
echo trace2 done
