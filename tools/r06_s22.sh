# round-6 session 22: pipelined bench steps (step i + 1's pack on a side
# stream during step i's search) -- the engine test, then the mnist bench
# with and without (KNN_BENCH_PIPELINE), then a kernel trace
set -o pipefail
mkdir -p gpurun_out/r06s22
timeout -k 10 600 python -u -m pytest tests/test_gpu_solo.py tests/test_gpu_bench_launch.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r06s22/tests.log 2>&1 || { tail -40 gpurun_out/r06s22/tests.log; exit 1; }
tail -1 gpurun_out/r06s22/tests.log
for v in 1 0 1 0; do
  KNN_BENCH_PIPELINE=$v timeout -k 10 300 python3 bench.py --workload mnist --steps 30 --warmup 5 --no-cpu-baseline --secondary-steps 0 > gpurun_out/r06s22/bench_$v.log 2>&1 || { tail -20 gpurun_out/r06s22/bench_$v.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r06s22/bench_$v.log') if l.startswith('{')][-1]); r=d['roofline']; print('pipe=$v', d['pipeline'], round(d['value']/1e6,3), 'Mq/s', round(d['ms_per_step'],4), 'ms/step', round(r['avg_launch_ms'],4), 'kernel', d['check_all_rows']['mismatches'], 'mismatches')"
done
(cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06s22/trace -o run -- \
   python3 bench.py --workload mnist --no-cpu-baseline --secondary-steps 0 --check 0 --steps 10 --warmup 4 > gpurun_out/r06s22/trace.log 2>&1) || exit 1
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r06s22/trace/**/run_kernel_trace.csv', recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
t0 = None
for r in rows[-40:-22]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    t0 = t0 or s
    print("%9.1f %8.1f q%s %s" % ((s - t0) / 1000, (e - s) / 1000, r['Queue_Id'], r['Kernel_Name'][:50]))
PY
