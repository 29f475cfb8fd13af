# round-5 session 24: the search's last merge on its last distance stream (no merge-stream hop) -- GPU suite, mnist bench + trace gaps, P=8 emulation
set -o pipefail
mkdir -p gpurun_out/s24
bash tools/gpu.sh tests || exit 1
for v in 0 1; do
  if [ $v = 1 ]; then export KNN_END_ON_MS=1; else unset KNN_END_ON_MS; fi
  timeout -k 10 200 python3 bench.py --workload mnist --steps 20 --warmup 3 --no-cpu-baseline --check 8 --secondary-steps 0 > gpurun_out/s24/mn_$v.log 2>&1 || { tail -20 gpurun_out/s24/mn_$v.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*\|"mismatches": [0-9]*' gpurun_out/s24/mn_$v.log | tr '\n' ' '; echo " mnist END_ON_MS=$v"
  timeout -k 10 300 python -u tools/ring_emulate.py --workload mnist --ranks 1,8 --steps 8 > gpurun_out/s24/emu_mn_$v.log 2>&1 || { tail -20 gpurun_out/s24/emu_mn_$v.log; exit 1; }
  grep '"P"' gpurun_out/s24/emu_mn_$v.log | cut -c1-120
  timeout -k 10 300 python -u tools/ring_emulate.py --workload mnist-real --ranks 8 --steps 5 > gpurun_out/s24/emu_mr_$v.log 2>&1 || { tail -20 gpurun_out/s24/emu_mr_$v.log; exit 1; }
  grep '"P"' gpurun_out/s24/emu_mr_$v.log | cut -c1-120
done
unset KNN_END_ON_MS
rm -rf gpurun_out/trace_mnist
bash tools/gpu.sh trace:mnist:8
