# sift bench at forced corpus split counts (KNN_SPLITS), no CPU leg.
set -o pipefail
mkdir -p gpurun_out/ssplit
for v in 2 3 4; do
  KNN_SPLITS=$v timeout -k 10 200 python -u bench.py --workload sift --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ssplit/sift_$v.log 2>&1 || exit 1
  grep '^{' gpurun_out/ssplit/sift_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('splits=$v', round(d['value']), 'ms', round(d['ms_per_step'],1), 'dist_ms', round(d['roofline']['avg_launch_ms'],2), d['engine'], d['check'])"
done
