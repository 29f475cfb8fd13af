# round-4 session 7: unskipped rescan + neighbour-ring cases, sift P = 8 split check
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_s8.py tests/test_gpu_ring_rotation.py -x -q --timeout 200 --timeout-method thread > gpurun_out/s7_tests.log 2>&1 || { tail -40 gpurun_out/s7_tests.log; exit 1; }
tail -2 gpurun_out/s7_tests.log
bash tools/gpu.sh emu:sift:8:3:rest:4,5 || exit $?
