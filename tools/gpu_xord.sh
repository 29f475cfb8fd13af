# k_dist_topk workgroup order (KNN_XCD_ORDER) x corpus splits (KNN_SPLITS) sweep.
set -o pipefail
mkdir -p gpurun_out/xord
one() {  # wl splits xord
  KNN_SPLITS=$2 KNN_XCD_ORDER=$3 timeout -k 10 200 python -u bench.py --workload $1 --steps 2 --warmup 1 --no-cpu-baseline --check 0 > gpurun_out/xord/$1_$2_$3.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$1 S=$2 x=$3 rc=$rc"; tail -3 gpurun_out/xord/$1_$2_$3.log; return $rc; }
  grep '^{' gpurun_out/xord/$1_$2_$3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$1 S=$2 xord=$3', 'step', round(d['ms_per_step'],2), 'dist', round(r['avg_launch_ms'],2), 'merge', round(r['exposed_merge_ms_per_step'],2), 'frac', round(r['frac'],4), d['engine']['splits'])"
}
for x in 0 1; do for s in 6 8 12; do one mnist $s $x || exit 1; done; done
for x in 0 1; do for s in 1 2 4 8; do one sift $s $x || exit 1; done; done
for x in 0 1; do for s in 2 4 8; do one gist $s $x || exit 1; done; done
