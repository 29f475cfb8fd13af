# sift k=32: default 32-slot variant vs forced 128-slot variant
set -o pipefail
mkdir -p gpurun_out
for kp in 32 128; do
  KNN_FORCE_KP=$kp timeout -k 10 300 python -u bench.py --workload sift --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sift_kp$kp.log 2>&1
  rc=$?; echo "kp $kp rc=$rc"; [ $rc -eq 0 ] || { tail -3 gpurun_out/sift_kp$kp.log; exit $rc; }
  grep '^{' gpurun_out/sift_kp$kp.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('kp $kp VALUE', round(d['value']), 'ms', round(d['ms_per_step'],2), 'dist_ms', round(d['roofline']['avg_launch_ms'],2), 'merge', round(d['roofline']['exposed_merge_ms_per_step'],2), d['engine'])"
done
