# P = 8 ring emulation under split-count overrides (diagnostic sweep).
set -o pipefail
mkdir -p gpurun_out
for s in 0 2 8 13 15; do
  if [ $s = 0 ]; then unset KNN_SPLITS; else export KNN_SPLITS=$s; fi
  timeout -k 10 120 python -u tools/ring_emulate.py --ranks 4,8 --steps 5 > gpurun_out/emu_s$s.log 2>&1
  rc=$?; echo "splits=$s rc=$rc"; grep -E '"(4|8)"|rank_ms|splits' gpurun_out/emu_s$s.log | tr -d '\n'; echo; [ $rc -eq 0 ] || exit $rc
done
