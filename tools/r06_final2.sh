# round-6 final check (session 2): the driver's steps on the final tree --
# pytest -m gpu, smoke(), bench.py with the driver's settings (PMC traffic
# keyed to this source, so roofline.traffic is populated)
set -o pipefail
mkdir -p gpurun_out/final6b
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/final6b/pytest.log 2>&1 || { tail -30 gpurun_out/final6b/pytest.log; exit 1; }
tail -1 gpurun_out/final6b/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final6b/smoke.log 2>&1 || { tail -20 gpurun_out/final6b/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final6b/bench.log 2>&1 || { tail -20 gpurun_out/final6b/bench.log; exit 1; }
grep '^{' gpurun_out/final6b/bench.log | tail -1 > gpurun_out/final6b/bench.json
cut -c1-400 gpurun_out/final6b/bench.json
