# Staging A/B (default: waves 0-3 stage; KNN_STAGE_ALL=1: every wave), mnist and sift, interleaved.
set -o pipefail
mkdir -p gpurun_out/stab
for r in 1 2; do for wl in mnist sift; do for sa in 0 1; do
  KNN_STAGE_ALL=$sa timeout -k 10 300 python -u bench.py --workload $wl --steps 4 --warmup 1 --no-cpu-baseline --check 0 > gpurun_out/stab/${wl}_${sa}_$r.log 2>&1 || exit 1
  grep '^{' gpurun_out/stab/${wl}_${sa}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$wl stage_all=$sa', round(d['value']), 'dist_ms', round(d['roofline']['avg_launch_ms'],2))"
done; done; done
