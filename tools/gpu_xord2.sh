# H16 kernels under the XCD-grouped workgroup order (A/B).
set -o pipefail
mkdir -p gpurun_out
for wl in mnist sift; do for x in 0 1; do
  KNN_XCD_ORDER=$x timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --check 0 > gpurun_out/xo_${wl}_$x.log 2>&1
  rc=$?; echo -n "$wl xord=$x rc=$rc "; grep '^{' gpurun_out/xo_${wl}_$x.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('VALUE', round(d['value']), 'dist', round(r['avg_launch_ms'],2))"; [ $rc -eq 0 ] || exit $rc
done; done
