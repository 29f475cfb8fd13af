# round-4 session 21: split floor of solo short-row searches (sift P = 1: 4 splits)
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu.sh bench:sift:3 emu:sift:1,8:3 || exit $?
grep -o '"ms_per_step": [0-9.]*\|"splits": [0-9]*\|"unresolved_queries": [0-9]*\|"mismatches": [0-9]*' gpurun_out/bench_sift.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_s8.py tests/test_gpu_i8.py -x -q --timeout 200 --timeout-method thread > gpurun_out/s21_tests.log 2>&1 || { tail -30 gpurun_out/s21_tests.log; exit 1; }
tail -1 gpurun_out/s21_tests.log
