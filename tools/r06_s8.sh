# round-6 session 8: k_merge_rank loads in two rounds, T and the mode with the first
# of the lists' first entries) -- int8 parity, then the mnist bench twice and
# a kernel trace (k_merge_rank's average)
set -o pipefail
mkdir -p gpurun_out/r06s8
timeout -k 10 900 python -u -m pytest tests/test_gpu_solo.py tests/test_gpu_s8.py tests/test_golden.py tests/test_gpu_i8.py tests/test_gpu_parity.py tests/test_gpu_ring_rotation.py tests/test_gpu_rccl_self.py tests/test_gpu_fullsize_ring.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r06s8/tests.log 2>&1 || { tail -40 gpurun_out/r06s8/tests.log; exit 1; }
tail -2 gpurun_out/r06s8/tests.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --workload mnist --steps 30 --warmup 3 --no-cpu-baseline --secondary-steps 0 > gpurun_out/r06s8/bench_$i.log 2>&1 || { tail -20 gpurun_out/r06s8/bench_$i.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/r06s8/bench_$i.log') if l.startswith('{')][-1]); r=d['roofline']; print(round(d['value']/1e6,3), 'Mq/s', round(d['ms_per_step'],4), 'ms/step', round(r['avg_launch_ms'],4), 'kernel', r['merge'], d['check_all_rows']['mismatches'], 'mismatches')"
done
bash tools/gpu.sh trace:mnist:12 && python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open('gpurun_out/trace_mnist/run_kernel_trace.csv')))
agg = collections.defaultdict(list)
for r in rows:
    agg[r['Kernel_Name'][:60]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000)
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print("%6d  avg %9.2f us  %s" % (len(v), sum(v) / len(v), k))
PY
