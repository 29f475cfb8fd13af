# round-5 session 35: no caller-stream wait packet after end()'s host sync -- GPU suite, mnist bench, P=8 emulation + trace gaps
set -o pipefail
mkdir -p gpurun_out/s35
bash tools/gpu.sh tests || exit 1
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --workload mnist --steps 20 --warmup 3 --no-cpu-baseline --check 8 --secondary-steps 0 > gpurun_out/s35/mn.log 2>&1 || { tail -20 gpurun_out/s35/mn.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*\|"mismatches": [0-9]*' gpurun_out/s35/mn.log | tr '\n' ' '; echo " mnist"
done
timeout -k 10 300 python -u tools/ring_emulate.py --workload mnist --ranks 1,2,4,8 --steps 8 > gpurun_out/s35/emu_mn.log 2>&1 || { tail -20 gpurun_out/s35/emu_mn.log; exit 1; }
grep '"P"' gpurun_out/s35/emu_mn.log | cut -c1-120
timeout -k 10 300 python -u tools/ring_emulate.py --workload mnist-real --ranks 1,2,4,8 --steps 5 > gpurun_out/s35/emu_mr.log 2>&1 || { tail -20 gpurun_out/s35/emu_mr.log; exit 1; }
grep '"P"' gpurun_out/s35/emu_mr.log | cut -c1-120
timeout -k 10 400 python -u tools/ring_emulate.py --workload sift --ranks 1,8 --steps 3 > gpurun_out/s35/emu_sift.log 2>&1 || { tail -20 gpurun_out/s35/emu_sift.log; exit 1; }
grep '"P"' gpurun_out/s35/emu_sift.log | cut -c1-120
rm -rf gpurun_out/emutrace_mnist gpurun_out/trace_mnist
bash tools/gpu.sh emutrace:mnist:8 trace:mnist:8
