set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tc.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/tc.log
timeout -k 10 300 ./tools/probe/kbench
