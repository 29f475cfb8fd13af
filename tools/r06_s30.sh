# round-6 session 30: k_dist_split with the chunk-sum adds pinned two m-tiles
# behind their MFMA chains (no 64-VGPR temporaries, no VGPR spills) --
# split-path GPU tests, then mnist-real and gist bench A/B against the HEAD
# build (tools/abl7/libknn_head.so)
set -o pipefail
mkdir -p gpurun_out/r06s30
timeout -k 10 600 python -u -m pytest tests/test_gpu_f32.py tests/test_gpu_split_pack.py tests/test_golden.py tests/test_gpu_config4.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06s30/tests.log 2>&1 || { tail -40 gpurun_out/r06s30/tests.log; exit 1; }
tail -1 gpurun_out/r06s30/tests.log
for wl in mnist-real gist; do
for v in new head new head; do
  if [ $v = head ]; then export KNN_LIB_PATH=$PWD/tools/abl7/libknn_head.so; else unset KNN_LIB_PATH; fi
  timeout -k 10 300 python -u bench.py --workload $wl --steps 4 --warmup 1 --no-cpu-baseline --secondary-steps 0 > gpurun_out/r06s30/bench_${wl}_$v.log 2>&1 || { tail -20 gpurun_out/r06s30/bench_${wl}_$v.log; exit 1; }
  grep '^{' gpurun_out/r06s30/bench_${wl}_$v.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.readline()); r = d['roofline']
print('$wl $v', round(d['value'], 1), 'q/s', round(d['ms_per_step'], 3), 'ms/step kernel', round(r['avg_launch_ms'], 3), 'frac', round(r['frac'], 4), 'merge', round(r.get('merge', {}).get('ms_per_step', 0), 3))"
done
done
