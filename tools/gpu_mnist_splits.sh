# mnist bench at forced corpus split counts (KNN_SPLITS), no CPU leg.
set -o pipefail
mkdir -p gpurun_out/msplit
for v in 4 5 6 7 8 10; do
  KNN_SPLITS=$v timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/msplit/mnist_$v.log 2>&1 || exit 1
  grep '^{' gpurun_out/msplit/mnist_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('splits=$v', round(d['value']), 'ms', round(d['ms_per_step'],2), 'dist_ms', round(d['roofline']['avg_launch_ms'],3), 'merge', round(d['roofline']['exposed_merge_ms_per_step'],3), d['engine']['unresolved_queries'], d['check']['mismatches'])"
done
