set -o pipefail
mkdir -p gpurun_out
ROOT=$GRAFT_REPO_ROOT
bash tools/gpu.sh tests || exit $?
(cd /tmp && export TMPDIR=/tmp && cd "$ROOT" && KNN_SPLITS=7 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/tr7 -o run -- python3 bench.py --workload mnist --no-cpu-baseline --secondary-steps 0 --check 0 --steps 6 --warmup 2 > gpurun_out/tr7.log 2>&1) || exit 1
echo trace done
for sp in 2 3 5; do
  KNN_SPLITS=$sp KNN_NO_RESEARCH8=1 timeout -k 10 300 python -u bench.py --workload sift --steps 2 --warmup 1 --no-cpu-baseline --check 0 > gpurun_out/b8.log 2>&1 || { tail -5 gpurun_out/b8.log; exit 1; }
  echo "sift splits=$sp $(grep '^{' gpurun_out/b8.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["engine"], d["roofline"]["avg_launch_ms"])')"
done
timeout -k 10 300 python -u bench.py --workload mnist-real --steps 5 --warmup 2 --no-cpu-baseline --check 4 > gpurun_out/b8r.log 2>&1 || { tail -5 gpurun_out/b8r.log; exit 1; }
echo "mnist-real $(grep '^{' gpurun_out/b8r.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["engine"], d["check"], d["roofline"]["avg_launch_ms"], d["roofline"]["exposed_merge_ms_per_step"])')"
timeout -k 10 400 python -u tools/ring_emulate.py --workload mnist --ranks 1,8 --steps 5 --splits 4,6,8,12 > gpurun_out/emu8.log 2>&1 || { tail -5 gpurun_out/emu8.log; exit 1; }
grep '"P"' gpurun_out/emu8.log
bash tools/gpu.sh kb8:--workload+mnist+--variant+5,6+--splits+6 kb8@noepi:--workload+mnist+--variant+6+--splits+6 kb8@noepi_nodma:--workload+mnist+--variant+6+--splits+6 kb8@noepi_nodma_nobar:--workload+mnist+--variant+6+--splits+6 kb8@count:--workload+mnist+--variant+6+--splits+6+--iters+1 kb8@noepi:--workload+sift+--variant+6+--splits+3+--iters+1 kb8@count:--workload+sift+--variant+6+--splits+3+--iters+1 || exit $?
