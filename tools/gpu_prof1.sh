set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread > gpurun_out/t3.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/t3.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b2.log 2>&1; echo "prof rc=$?"
tail -2 gpurun_out/b2.log
find gpurun_out/prof1 -name "*stats*" | head
