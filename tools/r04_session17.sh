# round-4 session 17: column-pack prefetch A/B (kernel trace of bench.py mnist, new vs previous library)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
for lib in new prev; do
  if [ $lib = prev ]; then export KNN_LIB_PATH=$PWD/tools/ab/libknn_prev.so; else unset KNN_LIB_PATH; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s17_${lib}_$i -o run -- \
    python3 bench.py --workload mnist --steps 20 --warmup 5 --no-cpu-baseline --secondary-steps 0 \
    > gpurun_out/s17_${lib}_$i.log 2>&1 || { tail -20 gpurun_out/s17_${lib}_$i.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/s17_${lib}_$i.log
  grep -h "k_pack8_col\|k_dist_topk_i8" gpurun_out/s17_${lib}_$i/run_kernel_stats.csv | cut -d, -f1-5
done
done
