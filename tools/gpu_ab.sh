# A/B the k_dist_topk main-loop variants (KNN_PIPE) + parity tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tc.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/tc.log
for v in 0 1 0 1; do
  KNN_PIPE=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --check 4 > gpurun_out/bab_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/bab_$v.log; exit 1; }
  grep '^{' gpurun_out/bab_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('PIPE=$v', 'ms', round(d['ms_per_step'],2), 'dist_ms', round(d['roofline']['avg_launch_ms'],2), 'frac', round(d['roofline']['frac'],4), d['check'])"
done
