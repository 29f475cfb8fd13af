# round-6 session 4: k_merge_rank reading its lists in one round of loads --
# int8 / golden / ring / s8 tests, then the mnist bench (merge entry) and a
# steady rocprofv3 kernel trace
set -o pipefail
mkdir -p gpurun_out/r06s4
timeout -k 10 600 python -u -m pytest tests/test_gpu_i8.py tests/test_golden.py tests/test_gpu_s8.py tests/test_gpu_fullsize_ring.py tests/test_gpu_ring_rotation.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r06s4/tests.log 2>&1 || { tail -40 gpurun_out/r06s4/tests.log; exit 1; }
tail -2 gpurun_out/r06s4/tests.log
timeout -k 10 300 python3 bench.py --workload mnist --steps 20 --warmup 3 --no-cpu-baseline --secondary-steps 0 > gpurun_out/r06s4/bench.log 2>&1 || { tail -20 gpurun_out/r06s4/bench.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r06s4/bench.log') if l.startswith('{')][-1]); r=d['roofline']; print(round(d['value']/1e6,3), 'Mq/s', round(d['ms_per_step'],4), 'ms/step', round(r['avg_launch_ms'],4), 'kernel', r['merge'], r['pack'], d['check_all_rows'])"
bash tools/gpu.sh trace:mnist:12 && python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/trace_mnist/run_kernel_trace.csv')))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
pe = None
for r in rows[-22:]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print("%8.1f gap %8.1f us  %s" % (((s - pe) / 1000) if pe else 0, (e - s) / 1000, r['Kernel_Name'][:50]))
    pe = max(pe or 0, e)
PY
