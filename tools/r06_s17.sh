# round-6 session 17: k_merge_rank16 (16 lanes a query, the P = 1 fin merge)
# -- the whole GPU suite, then the bench against tools/abl6/libknn_norank16.so
# and the SQ instruction counts of both merges
set -o pipefail
mkdir -p gpurun_out/r06s17
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06s17/tests.log 2>&1 || { tail -40 gpurun_out/r06s17/tests.log; exit 1; }
tail -1 gpurun_out/r06s17/tests.log
for v in r16 norank16 r16 norank16; do
  L=""; [ $v = norank16 ] && L=$PWD/tools/abl6/libknn_norank16.so
  KNN_LIB_PATH=$L timeout -k 10 300 python3 bench.py --workload mnist --steps 30 --warmup 5 --no-cpu-baseline --secondary-steps 0 > gpurun_out/r06s17/bench_$v.log 2>&1 || { tail -20 gpurun_out/r06s17/bench_$v.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r06s17/bench_$v.log') if l.startswith('{')][-1]); r=d['roofline']; print('$v', round(d['value']/1e6,3), 'Mq/s', round(d['ms_per_step'],4), 'ms/step', round(r['avg_launch_ms'],4), 'kernel', round(r['merge']['ms_per_step']*1000,1), 'us merge', d['check_all_rows']['mismatches'], 'mismatches')"
done
for v in r16 norank16; do
  L=""; [ $v = norank16 ] && L=$PWD/tools/abl6/libknn_norank16.so
  (cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && KNN_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06s17/inst_$v -o run \
    --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -- python3 bench.py --workload mnist --no-cpu-baseline --secondary-steps 0 --check 0 --steps 1 --warmup 0 > gpurun_out/r06s17/inst_$v.log 2>&1) || exit 1
  python3 tools/pmc_breakdown.py gpurun_out/r06s17/inst_$v | python3 -c "
import json,sys; d=json.load(sys.stdin)
for k,v in d.items():
  if 'merge_rank' in k: print('$v', k, {c: round(x,3) for c,x in v.items() if c.endswith(('per_wave','frac')) or c in ('GRBM_GUI_ACTIVE','SQ_WAVES')})"
done
