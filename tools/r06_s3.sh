# round-6 session 3: the 16x16x64 int8 kernel (knn_i8x.hip) -- parity first
# (int8 tests, full-size golden rows + all-row hashes, byte blocks, P = 8
# loopback), then the mnist bench against the 32x32x32 kernel on the same box
set -o pipefail
mkdir -p gpurun_out/r06s3
timeout -k 10 600 python -u -m pytest tests/test_gpu_i8.py tests/test_golden.py tests/test_gpu_s8.py tests/test_gpu_fullsize_ring.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r06s3/tests.log 2>&1 || { tail -40 gpurun_out/r06s3/tests.log; exit 1; }
tail -2 gpurun_out/r06s3/tests.log
for v in x 12 x 12; do
  if [ $v = x ]; then unset KNN_I8_KL; else export KNN_I8_KL=$v; fi
  timeout -k 10 300 python3 bench.py --workload mnist --steps 20 --warmup 3 --no-cpu-baseline --secondary-steps 0 > gpurun_out/r06s3/bench_$v.log 2>&1 || { tail -20 gpurun_out/r06s3/bench_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/r06s3/bench_$v.log') if l.startswith('{')][-1]); r=d['roofline']; print('$v', round(d['value']/1e6,3), 'Mq/s', round(d['ms_per_step'],4), 'ms/step', round(r['avg_launch_ms'],4), 'ms kernel', round(r['frac'],4), 'frac', d['engine'], d['check_all_rows'])"
done
unset KNN_I8_KL
