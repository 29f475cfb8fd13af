# round-5 final check: the driver's steps on the final tree -- pytest -m gpu, smoke(), bench.py with no flags
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/final/pytest.log 2>&1 || { tail -30 gpurun_out/final/pytest.log; exit 1; }
tail -1 gpurun_out/final/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 600 python bench.py > gpurun_out/final/bench.log 2>&1 || { tail -20 gpurun_out/final/bench.log; exit 1; }
grep '^{' gpurun_out/final/bench.log | tail -1
