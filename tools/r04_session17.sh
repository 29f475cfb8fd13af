# round-4 session 17: column-pack prefetch and merge query order -- A/B (kernel trace), tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_f32.py -x -q --timeout 200 --timeout-method thread > gpurun_out/s17_tests.log 2>&1 || { tail -30 gpurun_out/s17_tests.log; exit 1; }
tail -1 gpurun_out/s17_tests.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in new prev; do
  if [ $lib = prev ]; then export KNN_LIB_PATH=$PWD/tools/ab/libknn_prev.so; else unset KNN_LIB_PATH; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s17_${lib} -o run -- \
    python3 bench.py --workload mnist --steps 20 --warmup 5 --no-cpu-baseline --secondary-steps 3 \
    > gpurun_out/s17_${lib}.log 2>&1 || { tail -20 gpurun_out/s17_${lib}.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/s17_${lib}.log
  grep -h "k_pack8_col\|k_merge<\|k_order\|RadixSort\|k_dist_topk<" gpurun_out/s17_${lib}/run_kernel_stats.csv | cut -d, -f1-5
done
for lib in new prev; do
  if [ $lib = prev ]; then export KNN_LIB_PATH=$PWD/tools/ab/libknn_prev.so; else unset KNN_LIB_PATH; fi
  timeout -k 10 300 python3 bench.py --workload gist --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/s17_gist_${lib}.log 2>&1 || { tail -20 gpurun_out/s17_gist_${lib}.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*\|"exposed_merge_ms_per_step": [0-9.]*\|"unresolved_queries": [0-9]*\|"mismatches": [0-9]*' gpurun_out/s17_gist_${lib}.log
done
