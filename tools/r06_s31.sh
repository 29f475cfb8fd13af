# round-6 session 31: split-count sweeps of the one-tile-ring kernel on the
# emulated ranks (P = 1: 5..9 splits; P = 8 fused: 4..16)
set -o pipefail
bash tools/gpu.sh emu:mnist:1:5:none:5,6,7,8,9 emu:mnist:8:5:rest:4,6,8,10,12,16 > gpurun_out/r06s31.log 2>&1 || { tail -30 gpurun_out/r06s31.log; exit 1; }
grep '"P"' gpurun_out/r06s31.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['P'], d['splits'], round(d['rank_ms'], 4), round(d['dist_busy_ms_per_pass'], 4), d['unresolved'])"
