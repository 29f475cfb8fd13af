# split-count sweep on the fp16-shadow mnist kernel (diagnostic)
set -o pipefail
mkdir -p gpurun_out
for sp in 1 2 3 4 6 8; do
  KNN_SPLITS=$sp timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --check 0 > gpurun_out/sp_$sp.log 2>&1
  rc=$?; echo -n "splits=$sp rc=$rc "; grep '^{' gpurun_out/sp_$sp.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('VALUE', round(d['value']), 'ms', round(d['ms_per_step'],3), 'dist', round(r['avg_launch_ms'],3), 'merge', round(r['exposed_merge_ms_per_step'],3))"; [ $rc -eq 0 ] || exit $rc
done
