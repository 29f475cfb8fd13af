# GPU session: parity tests, then a kernel-trace profile of the default bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t3.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/t3.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1 -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b2.log 2>&1; echo "prof rc=$?"
tail -1 gpurun_out/b2.log
find gpurun_out/prof1 -name "*.csv"
