# round-5 session 19: own-block split count of the P=8 mnist-real rank (the shared merge fits 32 lanes at <= 3)
set -o pipefail
mkdir -p gpurun_out/s19
for v in 0 1 2 3 4 5; do
  if [ $v = 0 ]; then unset KNN_OWN_SPLITS; else export KNN_OWN_SPLITS=$v; fi
  timeout -k 10 300 python -u tools/ring_emulate.py --workload mnist-real --ranks 8 --steps 8 > gpurun_out/s19/emu_$v.log 2>&1 || { tail -20 gpurun_out/s19/emu_$v.log; exit 1; }
  echo "own splits $v"; grep '"P"' gpurun_out/s19/emu_$v.log
done
unset KNN_OWN_SPLITS
timeout -k 10 300 python -u tools/ring_emulate.py --workload mnist-real --ranks 1 --steps 5 > gpurun_out/s19/emu_p1.log 2>&1 && grep '"P"' gpurun_out/s19/emu_p1.log
