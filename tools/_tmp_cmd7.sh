set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
KNN_SPLITS=7 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/tr7 -o run -- python3 bench.py --workload mnist --no-cpu-baseline --secondary-steps 0 --check 0 --steps 6 --warmup 2 > gpurun_out/tr7.log 2>&1
