set -o pipefail
mkdir -p gpurun_out/pmc2
timeout -k 10 300 python -u -m pytest tests/ -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tc.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/tc.log
timeout -k 10 300 ./tools/probe/kbench | tail -4
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc2/fetch -o run --pmc FETCH_SIZE -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --check 0 > gpurun_out/pmc2/fetch.log 2>&1; echo "fetch rc=$?"
