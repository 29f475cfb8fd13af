# round-5 session 17: query-ordered merge at the P=8 rank (KNN_ORDER=1) vs default, mnist-real emulation
set -o pipefail
mkdir -p gpurun_out/s17
for v in 0 1; do
  if [ $v = 1 ]; then export KNN_ORDER=1; else unset KNN_ORDER; fi
  timeout -k 10 300 python -u tools/ring_emulate.py --workload mnist-real --ranks 1,8 --steps 5 > gpurun_out/s17/emu_mr_$v.log 2>&1 || { tail -20 gpurun_out/s17/emu_mr_$v.log; exit 1; }
  echo "KNN_ORDER=$v"; grep '"P"' gpurun_out/s17/emu_mr_$v.log
done
