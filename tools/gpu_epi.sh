set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tc.log 2>&1
rc=$?; tail -3 gpurun_out/tc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/probe/kbench32 && timeout -k 10 200 ./tools/probe/kbench 2>&1 | head -3
WORKLOADS="sift" bash tools/gpu_f32bench.sh 2>&1 | grep VALUE
