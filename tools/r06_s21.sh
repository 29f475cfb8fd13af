# round-6 session 21: k_merge_rank16 with 32 lanes a query for a ring rank's
# own + fused pair (<= 32 lists) -- the whole GPU suite, then the emulated
# P = 1 / 2 / 4 / 8 ranks against tools/abl6/libknn_norank16.so
set -o pipefail
mkdir -p gpurun_out/r06s21
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06s21/tests.log 2>&1 || { tail -40 gpurun_out/r06s21/tests.log; exit 1; }
tail -1 gpurun_out/r06s21/tests.log
for v in r16 norank16 r16 norank16; do
  L=""; [ $v = norank16 ] && L=$PWD/tools/abl6/libknn_norank16.so
  KNN_LIB_PATH=$L timeout -k 10 400 python -u tools/ring_emulate.py --workload mnist --ranks 1,2,4,8 --steps 5 > gpurun_out/r06s21/emu_$v.log 2>&1 || { tail -20 gpurun_out/r06s21/emu_$v.log; exit 1; }
  grep '"P"' gpurun_out/r06s21/emu_$v.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('$v', d['P'], round(d['rank_ms'], 4), round(d['exposed_merge_ms_per_pass'], 4), d['unresolved'])"
done
