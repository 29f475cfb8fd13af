set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
KNN_SPLITS=6 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr13a -o run -- python3 bench.py --workload mnist --no-cpu-baseline --secondary-steps 0 --check 0 --steps 3 --warmup 1 > gpurun_out/tr13a.log 2>&1 || exit 1
KNN_SPLITS=6 KNN_NO_RESEARCH8=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr13b -o run -- python3 bench.py --workload mnist --no-cpu-baseline --secondary-steps 0 --check 0 --steps 3 --warmup 1 > gpurun_out/tr13b.log 2>&1 || exit 1
echo traces done
