set -o pipefail
mkdir -p gpurun_out
for cfg in "KNN_SPLITS=5" "KNN_SPLITS=6" "KNN_SPLITS=7" "KNN_SPLITS=8" "KNN_SPLITS=10"; do
  env $cfg timeout -k 10 300 python -u bench.py --workload mnist --steps 20 --warmup 3 --no-cpu-baseline --secondary-steps 0 --check 0 > gpurun_out/b14.log 2>&1 || { tail -5 gpurun_out/b14.log; exit 1; }
  echo "mnist $cfg $(grep '^{' gpurun_out/b14.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), d["engine"], round(d["roofline"]["avg_launch_ms"],4), round(d["roofline"]["exposed_merge_ms_per_step"],4))')"
done
for cfg in "KNN_SPLITS=3" "KNN_SPLITS=4" "KNN_SPLITS=5"; do
  env $cfg timeout -k 10 300 python -u bench.py --workload sift --steps 3 --warmup 1 --no-cpu-baseline --check 0 > gpurun_out/b14.log 2>&1 || { tail -5 gpurun_out/b14.log; exit 1; }
  echo "sift $cfg $(grep '^{' gpurun_out/b14.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), d["engine"], round(d["roofline"]["avg_launch_ms"],4), round(d["roofline"]["exposed_merge_ms_per_step"],4))')"
done
timeout -k 10 400 python -u tools/ring_emulate.py --workload mnist --ranks 8 --steps 5 --splits 6,7,8 > gpurun_out/emu14.log 2>&1 || { tail -5 gpurun_out/emu14.log; exit 1; }
grep '"P"' gpurun_out/emu14.log
