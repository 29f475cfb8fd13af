# round-6 session 38: gist's k_dist_split with the XCD-grouped workgroup
# order (KNN_XCD_ORDER=1: a query block's splits run side by side on one
# XCD, so its query rows are fetched once an XCD) at 2 / 4 / 8 / 16 splits,
# against the default split-major order
set -o pipefail
mkdir -p gpurun_out/r06s38
for cfg in 0:0 1:0 1:4 1:8 0:8 1:16; do
  xo=${cfg%%:*}; sp=${cfg#*:}
  if [ $xo = 1 ]; then export KNN_XCD_ORDER=1; else unset KNN_XCD_ORDER; fi
  if [ $sp = 0 ]; then unset KNN_SPLITS; else export KNN_SPLITS=$sp; fi
  timeout -k 10 300 python -u bench.py --workload gist --steps 3 --warmup 1 --no-cpu-baseline --secondary-steps 0 > gpurun_out/r06s38/gist_$xo_$sp.log 2>&1 || { tail -20 gpurun_out/r06s38/gist_$xo_$sp.log; exit 1; }
  grep '^{' gpurun_out/r06s38/gist_$xo_$sp.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.readline()); r = d['roofline']
print('xord $xo splits $sp', round(d['ms_per_step'], 1), 'ms/step kernel', round(r['avg_launch_ms'], 1), 'merge', round(r.get('merge', {}).get('ms_per_step', 0), 2), 'engine', d['engine'], 'check', d['check'])"
done
