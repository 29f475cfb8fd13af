# round-6 session 39: the XCD-grouped order as a default candidate for the
# split filter -- gist and mnist-real A/B (KNN_XCD_ORDER=1 vs unset),
# alternating, model-chosen splits
set -o pipefail
mkdir -p gpurun_out/r06s39
for wl in gist mnist-real; do
for v in x s x s x s; do
  if [ $v = x ]; then export KNN_XCD_ORDER=1; else unset KNN_XCD_ORDER; fi
  st=3; [ $wl = mnist-real ] && st=8
  timeout -k 10 300 python -u bench.py --workload $wl --steps $st --warmup 1 --no-cpu-baseline --secondary-steps 0 > gpurun_out/r06s39/${wl}_$v.log 2>&1 || { tail -20 gpurun_out/r06s39/${wl}_$v.log; exit 1; }
  grep '^{' gpurun_out/r06s39/${wl}_$v.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.readline()); r = d['roofline']
print('$wl $v', round(d['ms_per_step'], 2), 'ms/step kernel', round(r['avg_launch_ms'], 2), 'merge', round(r.get('merge', {}).get('ms_per_step', 0), 3), d['engine']['splits'], d['check']['mismatches'])"
done
done
