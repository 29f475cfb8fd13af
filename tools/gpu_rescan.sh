# Chunked exact rescan: GPU tests, then the mnist bench with one corpus split
# (the configuration that leaves uncertified queries) and the default one.
set -o pipefail
mkdir -p gpurun_out/rescan
timeout -k 10 400 python -u -m pytest tests/ -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/rescan/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/rescan/pytest.log; [ $rc -eq 0 ] || exit $rc
KNN_SPLITS=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/rescan/bench_s1.log 2>&1
rc=$?; echo "bench s1 rc=$rc"; grep '^{' gpurun_out/rescan/bench_s1.log || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/rescan/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/rescan/bench.log
