# round-4 session 14: pipelined epilogue A/B, tests
set -o pipefail
mkdir -p gpurun_out
E="timeout -k 10 200 python -u tools/ring_emulate.py --workload mnist --steps 10 --warm 5"
for i in 1 2; do
$E --ranks 1,8 > gpurun_out/s14_new_$i.log 2>&1 || { tail -20 gpurun_out/s14_new_$i.log; exit 1; }
KNN_LIB_PATH=$PWD/tools/ab/libknn_prev.so $E --ranks 1,8 > gpurun_out/s14_prev_$i.log 2>&1 || { tail -20 gpurun_out/s14_prev_$i.log; exit 1; }
done
grep '"P"' gpurun_out/s14_*.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s14_tests.log 2>&1 || { tail -40 gpurun_out/s14_tests.log; exit 1; }
tail -2 gpurun_out/s14_tests.log
