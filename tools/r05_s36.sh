# round-5 session 36: k_pack8_col with 32-row workgroups (twice the workgroups) -- byte-block tests under both, mnist bench A/B, pack kernel time
set -o pipefail
mkdir -p gpurun_out/s36
for v in 64 32; do
  export KNN_PACK8_RW=$v
  timeout -k 10 400 python -u -m pytest tests/test_gpu_s8.py tests/test_golden.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/s36/tests_$v.log 2>&1 || { tail -30 gpurun_out/s36/tests_$v.log; exit 1; }
  echo "RW=$v $(tail -1 gpurun_out/s36/tests_$v.log)"
done
for r in 1 2; do
for v in 64 32; do
  export KNN_PACK8_RW=$v
  timeout -k 10 200 python3 bench.py --workload mnist --steps 20 --warmup 3 --no-cpu-baseline --check 8 --secondary-steps 0 > gpurun_out/s36/mn_$v.log 2>&1 || { tail -20 gpurun_out/s36/mn_$v.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*\|"mismatches": [0-9]*' gpurun_out/s36/mn_$v.log | tr '\n' ' '; echo " mnist RW=$v"
done
done
for v in 64 32; do
  export KNN_PACK8_RW=$v
  (cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s36/tr_$v -o run -- python3 bench.py --workload mnist --steps 10 --warmup 3 --no-cpu-baseline --check 0 --secondary-steps 0 > gpurun_out/s36/tr_$v.log 2>&1) || exit 1
  python3 - "$v" <<'PY'
import csv, glob, sys
v = sys.argv[1]
f = glob.glob("gpurun_out/s36/tr_%s/**/*kernel_stats.csv" % v, recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "pack8" in r["Name"]:
        print("RW", v, r["Name"][:40], "avg us", float(r["AverageNs"]) / 1000, "calls", r["Calls"])
PY
done
