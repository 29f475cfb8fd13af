# round-6 session 35: the PF2 barrier's LDS wait only where chunk y - 2 can
# still be read (a one-K-step last chunk) -- mnist A/B against HEAD
# (tools/abl7/libknn_head.so), then the final evidence of this build: whole
# GPU suite and smoke, bench at the driver's settings, steady trace, PMC
# traffic passes, emulated ranks, and the SIFT bench / trace / PMC
set -o pipefail
mkdir -p gpurun_out/r06s35
for v in new head new head new head; do
  if [ $v = head ]; then export KNN_LIB_PATH=$PWD/tools/abl7/libknn_head.so; else unset KNN_LIB_PATH; fi
  timeout -k 10 300 python -u bench.py --workload mnist --steps 20 --warmup 5 --no-cpu-baseline --secondary-steps 0 > gpurun_out/r06s35/bench_$v.log 2>&1 || { tail -20 gpurun_out/r06s35/bench_$v.log; exit 1; }
  grep '^{' gpurun_out/r06s35/bench_$v.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.readline()); r = d['roofline']
print('$v', round(d['value']/1e6, 3), 'Mq/s', round(d['ms_per_step'], 4), 'ms/step kernel', round(r['avg_launch_ms'], 4), 'frac', round(r['frac'], 4), 'rows', d['check_all_rows']['mismatches'])"
done
unset KNN_LIB_PATH
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06s35/bench_final.log 2>&1 || { tail -20 gpurun_out/r06s35/bench_final.log; exit 1; }
grep '^{' gpurun_out/r06s35/bench_final.log | tail -1 > gpurun_out/r06s35/bench_final.json
bash tools/gpu.sh tests trace:mnist pmc:mnist:3 emu:mnist:1,2,4,8 bench:sift:3 trace:sift:4 pmc:sift:3
