# round-6 session 11: end() polls the mapped count word before its blocking
# sync (KNN_END_SPIN) -- the mnist bench with and without, then a trace
set -o pipefail
mkdir -p gpurun_out/r06s11
timeout -k 10 600 python -u -m pytest tests/test_gpu_solo.py tests/test_gpu_s8.py tests/test_gpu_ring_rotation.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r06s11/tests.log 2>&1 || { tail -40 gpurun_out/r06s11/tests.log; exit 1; }
tail -1 gpurun_out/r06s11/tests.log
for v in 1 0 1 0; do
  KNN_END_SPIN=$v timeout -k 10 300 python3 bench.py --workload mnist --steps 30 --warmup 3 --no-cpu-baseline --secondary-steps 0 > gpurun_out/r06s11/bench_$v.log 2>&1 || { tail -20 gpurun_out/r06s11/bench_$v.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r06s11/bench_$v.log') if l.startswith('{')][-1]); r=d['roofline']; print('spin=$v', round(d['value']/1e6,3), 'Mq/s', round(d['ms_per_step'],4), 'ms/step', round(r['avg_launch_ms'],4), 'kernel', d['check_all_rows']['mismatches'], 'mismatches')"
done
for v in 1 0; do
(cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && KNN_END_SPIN=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06s11/trace_$v -o run -- \
   python3 bench.py --workload mnist --no-cpu-baseline --secondary-steps 0 --check 0 --steps 10 --warmup 4 > gpurun_out/r06s11/trace_$v.log 2>&1) || exit 1
python3 - $v <<'PY'
import csv, sys, glob
f = glob.glob('gpurun_out/r06s11/trace_%s/**/run_kernel_trace.csv' % sys.argv[1], recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
pe = None
for r in rows[-14:]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print("%8.1f gap %8.1f us  %s" % (((s - pe) / 1000) if pe else 0, (e - s) / 1000, r['Kernel_Name'][:50]))
    pe = max(pe or 0, e)
PY
done
