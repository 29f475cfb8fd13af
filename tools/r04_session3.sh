# round-4 session 3: P=8 mnist split sweep (half-tile vs W8 kernel, fused rest vs all)
set -o pipefail
mkdir -p gpurun_out
E="timeout -k 10 240 python -u tools/ring_emulate.py --workload mnist --steps 5 --warm 5"
$E --ranks 8 --splits 6,8,12,16,24,31 > gpurun_out/s3_half.log 2>&1 || { tail -20 gpurun_out/s3_half.log; exit 1; }
KNN_I8_W8=1 $E --ranks 8 --splits 6,8,12,16,24,31 > gpurun_out/s3_w8.log 2>&1 || { tail -20 gpurun_out/s3_w8.log; exit 1; }
$E --ranks 1,8 --fuse all > gpurun_out/s3_all.log 2>&1 || { tail -20 gpurun_out/s3_all.log; exit 1; }
grep '"P"' gpurun_out/s3_*.log
bash tools/gpu.sh bench:sift:3 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_i8.py tests/test_gpu_s8.py -x -q --timeout 240 --timeout-method thread > gpurun_out/s3_tests.log 2>&1 || { tail -30 gpurun_out/s3_tests.log; exit 1; }
tail -2 gpurun_out/s3_tests.log
