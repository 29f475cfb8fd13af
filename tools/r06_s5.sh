# round-6 session 5: solo P = 1 searches (kernel + merge on the caller's
# stream, the meta check through knn_ctx_search_meta) -- parity, then the
# mnist bench solo / not solo on the same box, then a kernel trace
set -o pipefail
mkdir -p gpurun_out/r06s5
timeout -k 10 700 python -u -m pytest tests/test_gpu_solo.py tests/test_gpu_s8.py tests/test_golden.py tests/test_gpu_i8.py tests/test_gpu_parity.py tests/test_gpu_ring_rotation.py tests/test_gpu_rccl_self.py tests/test_gpu_f32.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r06s5/tests.log 2>&1 || { tail -40 gpurun_out/r06s5/tests.log; exit 1; }
tail -2 gpurun_out/r06s5/tests.log
for v in solo nosolo solo nosolo; do
  if [ $v = solo ]; then B="bench.py"; else B="tools/probe/bench_nosolo.py"; fi
  timeout -k 10 300 python3 $B --workload mnist --steps 30 --warmup 3 --no-cpu-baseline --secondary-steps 0 > gpurun_out/r06s5/bench_$v.log 2>&1 || { tail -20 gpurun_out/r06s5/bench_$v.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r06s5/bench_$v.log') if l.startswith('{')][-1]); r=d['roofline']; print('$v', round(d['value']/1e6,3), 'Mq/s', round(d['ms_per_step'],4), 'ms/step', round(r['avg_launch_ms'],4), 'kernel', d['check_all_rows']['mismatches'], 'mismatches')"
done
bash tools/gpu.sh trace:mnist:12 && python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/trace_mnist/run_kernel_trace.csv')))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
pe = None
for r in rows[-16:]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print("%8.1f gap %8.1f us  %s" % (((s - pe) / 1000) if pe else 0, (e - s) / 1000, r['Kernel_Name'][:50]))
    pe = max(pe or 0, e)
PY
