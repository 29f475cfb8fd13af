# round-6 session 10: k_merge_rank's VALU work (SQ counters showed ~683 VALU
# instructions a wave, ~90% of the SIMDs' issue over the launch): product
# (tightened bound, lim from the host, shift for lpq) against the same
# without the tightened bound (tools/abl6/libknn_mr_notight.so)
set -o pipefail
mkdir -p gpurun_out/r06s10
timeout -k 10 600 python -u -m pytest tests/test_gpu_i8.py tests/test_golden.py tests/test_gpu_solo.py tests/test_gpu_s8.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r06s10/tests.log 2>&1 || { tail -40 gpurun_out/r06s10/tests.log; exit 1; }
tail -1 gpurun_out/r06s10/tests.log
for v in prod notight prod notight; do
  L=""; [ $v = notight ] && L=$PWD/tools/abl6/libknn_mr_notight.so
  KNN_LIB_PATH=$L timeout -k 10 300 python3 bench.py --workload mnist --steps 20 --warmup 3 --no-cpu-baseline --secondary-steps 0 > gpurun_out/r06s10/bench_$v.log 2>&1 || { tail -20 gpurun_out/r06s10/bench_$v.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r06s10/bench_$v.log') if l.startswith('{')][-1]); r=d['roofline']; print('$v', round(d['value']/1e6,3), 'Mq/s', round(r['avg_launch_ms'],4), 'kernel', round(r['merge']['ms_per_step']*1000,2), 'us merge', d['check_all_rows']['mismatches'], 'mismatches')"
done
for v in prod notight; do
  L=""; [ $v = notight ] && L=$PWD/tools/abl6/libknn_mr_notight.so
  (cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && KNN_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06s10/inst_$v -o run \
    --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -- python3 bench.py --workload mnist --no-cpu-baseline --secondary-steps 0 --check 0 --steps 1 --warmup 0 > gpurun_out/r06s10/inst_$v.log 2>&1) || exit 1
  python3 tools/pmc_breakdown.py gpurun_out/r06s10/inst_$v | python3 -c "
import json,sys; d=json.load(sys.stdin)
for k,v in d.items():
  if 'merge_rank' in k: print('$v', k, {c: round(x,3) for c,x in v.items() if c.endswith(('per_wave','frac')) or c=='GRBM_GUI_ACTIVE'})"
done
