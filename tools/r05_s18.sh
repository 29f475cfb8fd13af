# round-5 session 18: full GPU suite + smoke at the count read-back change; ring emulation of all three workloads (profiles/r05_ring_emulation.json)
set -o pipefail
mkdir -p gpurun_out/s18
bash tools/gpu.sh tests || exit 1
for w in mnist mnist-real; do
  timeout -k 10 400 python -u tools/ring_emulate.py --workload $w --ranks 1,2,4,8 --steps 5 > gpurun_out/s18/emu_$w.log 2>&1 || { tail -20 gpurun_out/s18/emu_$w.log; exit 1; }
  echo $w; grep '"P"' gpurun_out/s18/emu_$w.log
done
timeout -k 10 400 python -u tools/ring_emulate.py --workload sift --ranks 1,8 --steps 3 > gpurun_out/s18/emu_sift.log 2>&1 || { tail -20 gpurun_out/s18/emu_sift.log; exit 1; }
echo sift; grep '"P"' gpurun_out/s18/emu_sift.log
