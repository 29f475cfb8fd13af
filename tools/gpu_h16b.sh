set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/tc.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/tc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload sift --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sift.log 2>&1
rc=$?; echo "sift rc=$rc"; grep '^{' gpurun_out/sift.log; exit $rc
