# Round evidence: tests, full bench (with CPU leg), kernel-trace stats, PMC traffic.
set -o pipefail
mkdir -p gpurun_out/round
timeout -k 10 400 python -u -m pytest tests/ -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/round/pytest.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/round/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/round/smoke.log 2>&1; echo "smoke rc=$?"
timeout -k 10 400 python -u bench.py > gpurun_out/round/bench.log 2>&1; echo "bench rc=$?"; grep '^{' gpurun_out/round/bench.log > gpurun_out/round/bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/round/trace -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --check 0 > gpurun_out/round/trace.log 2>&1; echo "trace rc=$?"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/round/fetch -o run --pmc FETCH_SIZE -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --check 0 > gpurun_out/round/fetch.log 2>&1; echo "fetch rc=$?"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/round/write -o run --pmc WRITE_SIZE -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --check 0 > gpurun_out/round/write.log 2>&1; echo "write rc=$?"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/round/mfma -o run --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --check 0 > gpurun_out/round/mfma.log 2>&1; echo "mfma rc=$?"
