# round-6 session 16: the column-major byte pack without LDS transpose or
# per-tile barriers (k_pack8_colw) against the tiled k_pack8_col
# (tools/abl6/libknn_pack_tiled.so) -- byte-block parity, then the bench A/B
set -o pipefail
mkdir -p gpurun_out/r06s16
timeout -k 10 600 python -u -m pytest tests/test_gpu_s8.py tests/test_golden.py tests/test_gpu_i8.py tests/test_gpu_solo.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r06s16/tests.log 2>&1 || { tail -40 gpurun_out/r06s16/tests.log; exit 1; }
tail -1 gpurun_out/r06s16/tests.log
for v in colw tiled colw tiled; do
  L=""; [ $v = tiled ] && L=$PWD/tools/abl6/libknn_pack_tiled.so
  KNN_LIB_PATH=$L timeout -k 10 300 python3 bench.py --workload mnist --steps 30 --warmup 5 --no-cpu-baseline --secondary-steps 0 > gpurun_out/r06s16/bench_$v.log 2>&1 || { tail -20 gpurun_out/r06s16/bench_$v.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r06s16/bench_$v.log') if l.startswith('{')][-1]); r=d['roofline']; print('$v', round(d['value']/1e6,3), 'Mq/s', round(d['ms_per_step'],4), 'ms/step', round(r['avg_launch_ms'],4), 'kernel', round(r['pack']['ms_per_step']*1000,1), 'us pack', round(r['pack']['frac'],3), d['check_all_rows']['mismatches'], 'mismatches')"
done
