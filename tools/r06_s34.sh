# round-6 session 34: 32-bit diagonal-tile check in the epilogue, 6-entry survivor buffers for 25 K-steps,
# one-chunk-tile staging for SIFT's kernels -- int8 /
# golden / byte-block / solo / ring GPU tests, then mnist bench A/B against
# the HEAD build (tools/abl7/libknn_head.so), alternating
set -o pipefail
mkdir -p gpurun_out/r06s34
timeout -k 10 600 python -u -m pytest tests/test_gpu_i8.py tests/test_golden.py tests/test_gpu_s8.py tests/test_gpu_solo.py tests/test_gpu_fullsize_ring.py tests/test_gpu_f32.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r06s34/tests.log 2>&1 || { tail -40 gpurun_out/r06s34/tests.log; exit 1; }
tail -1 gpurun_out/r06s34/tests.log
for v in new head new head new head; do
  if [ $v = head ]; then export KNN_LIB_PATH=$PWD/tools/abl7/libknn_head.so; else unset KNN_LIB_PATH; fi
  timeout -k 10 300 python -u bench.py --workload mnist --steps 20 --warmup 5 --no-cpu-baseline --secondary-steps 0 > gpurun_out/r06s34/bench_$v.log 2>&1 || { tail -20 gpurun_out/r06s34/bench_$v.log; exit 1; }
  grep '^{' gpurun_out/r06s34/bench_$v.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.readline()); r = d['roofline']
print('$v', round(d['value']/1e6, 3), 'Mq/s', round(d['ms_per_step'], 4), 'ms/step kernel', round(r['avg_launch_ms'], 4), 'frac', round(r['frac'], 4), 'rows', d['check_all_rows']['mismatches'])"
done
for v in new head new head; do
  if [ $v = head ]; then export KNN_LIB_PATH=$PWD/tools/abl7/libknn_head.so; else unset KNN_LIB_PATH; fi
  timeout -k 10 300 python -u bench.py --workload sift --steps 4 --warmup 1 --no-cpu-baseline --secondary-steps 0 > gpurun_out/r06s34/sift_$v.log 2>&1 || { tail -20 gpurun_out/r06s34/sift_$v.log; exit 1; }
  grep '^{' gpurun_out/r06s34/sift_$v.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.readline()); r = d['roofline']
print('sift $v', round(d['value']/1e6, 3), 'Mq/s', round(d['ms_per_step'], 3), 'ms/step kernel', round(r['avg_launch_ms'], 3), 'frac', round(r['frac'], 4))"
done
