# Ring emulation (one rank's compute at P = 1..8) with the default staging
# (waves 0-3 stage for all eight) and with KNN_STAGE_ALL=1, interleaved twice.
set -o pipefail
mkdir -p gpurun_out/emu_stage
for r in 1 2; do
  timeout -k 10 200 python -u tools/ring_emulate.py --steps 5 > gpurun_out/emu_stage/def_$r.log 2>&1 || exit 1
  KNN_STAGE_ALL=1 timeout -k 10 200 python -u tools/ring_emulate.py --steps 5 > gpurun_out/emu_stage/all_$r.log 2>&1 || exit 1
  for f in def_$r all_$r; do
    python3 -c "
import json
t=open('gpurun_out/emu_stage/$f.log').read(); d=json.loads(t[t.index('{'):])
print('$f', ' '.join('P%s=%.3f' % (P, v['rank_ms']) for P, v in d.items()))"
  done
done
