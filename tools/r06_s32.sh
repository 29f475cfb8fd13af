# round-6 session 32: survivor-buffer depth NB of the 25-K-step kernel
# (4 / 5 = head / 6 / 7; tools/abl7/libknn_nb*.so built from the working
# tree with only the launch line changed) -- mnist bench and the emulated
# P = 8 rank, alternating
set -o pipefail
mkdir -p gpurun_out/r06s32
for rep in 1 2; do
for v in head nb4 nb6 nb7; do
  export KNN_LIB_PATH=$PWD/tools/abl7/libknn_$v.so
  timeout -k 10 300 python -u bench.py --workload mnist --steps 20 --warmup 5 --no-cpu-baseline --secondary-steps 0 > gpurun_out/r06s32/bench_$v.log 2>&1 || { tail -20 gpurun_out/r06s32/bench_$v.log; exit 1; }
  timeout -k 10 300 python -u tools/ring_emulate.py --workload mnist --ranks 8 --steps 5 > gpurun_out/r06s32/emu_$v.log 2>&1 || { tail -20 gpurun_out/r06s32/emu_$v.log; exit 1; }
  b=$(grep '^{' gpurun_out/r06s32/bench_$v.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.readline()); r = d['roofline']
print(round(d['ms_per_step'], 4), round(r['avg_launch_ms'], 4), d['check_all_rows']['mismatches'])")
  e=$(grep '"P"' gpurun_out/r06s32/emu_$v.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.readline()); print(round(d['rank_ms'], 4), round(d['dist_busy_ms_per_pass'], 4), d['unresolved'])")
  echo "$v bench(step kernel mism) $b  P8(rank busy unres) $e"
done
done
