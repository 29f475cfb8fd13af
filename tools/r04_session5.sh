# round-4 session 5: two query groups a wave (sift): bench against the one-group kernel, tests
set -o pipefail
mkdir -p gpurun_out
B="timeout -k 10 300 python -u bench.py --workload sift --steps 3 --warmup 2"
$B > gpurun_out/s5_qg2.log 2>&1 || { tail -30 gpurun_out/s5_qg2.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*\|"unresolved_queries": [0-9]*\|"mismatches": [0-9]*' gpurun_out/s5_qg2.log
KNN_I8_QG1=1 $B > gpurun_out/s5_qg1.log 2>&1 || { tail -30 gpurun_out/s5_qg1.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*\|"unresolved_queries": [0-9]*' gpurun_out/s5_qg1.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s5_tests.log 2>&1 || { tail -40 gpurun_out/s5_tests.log; exit 1; }
tail -3 gpurun_out/s5_tests.log
