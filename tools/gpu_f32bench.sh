# fp32 workloads (configs[3] sift, configs[4]-shaped gist) on one GPU.
set -o pipefail
mkdir -p gpurun_out
for w in ${WORKLOADS:-sift gist}; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} 2>&1 | tee gpurun_out/bench_$w.log
  rc=$?; echo "bench $w rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' gpurun_out/bench_$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w VALUE', round(d['value']), 'ms', round(d['ms_per_step'],2), 'dist_ms', round(d['roofline']['avg_launch_ms'],2), 'TF', round(d['roofline']['achieved'],1), 'frac', round(d['roofline']['frac'],4), 'merge_ms', round(d['roofline']['exposed_merge_ms_per_step'],2), d['engine'], d['check'])"
done
