# round-6 session 2: (1) the int8 MFMA shape probe (32x32x32 vs 16x16x64 at the
# same LDS bytes per op, random data, clock stamped); (2) gist's L2 traffic
# split: TCC hits / misses / EA read requests of
# k_dist_split, two passes, beside FETCH_SIZE, on one box
set -o pipefail
mkdir -p gpurun_out/r06s2
timeout -k 10 240 tools/probe/i8_shape_probe 20000 > gpurun_out/r06s2/shape.log 2>&1 || { cat gpurun_out/r06s2/shape.log; exit 1; }
cat gpurun_out/r06s2/shape.log
for i in 1 2; do
  for g in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "FETCH_SIZE"; do
    tag=$(echo "$g" | cut -d' ' -f1 | tr 'A-Z' 'a-z')
    (cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
     timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d "gpurun_out/r06s2/gist_${tag}_$i" -o run \
       --pmc $g -- python3 bench.py --workload gist --no-cpu-baseline --secondary-steps 0 --check 0 --steps 1 --warmup 0 \
       > "gpurun_out/r06s2/gist_${tag}_$i.log" 2>&1) || { tail -20 "gpurun_out/r06s2/gist_${tag}_$i.log"; exit 1; }
    echo "pass $tag $i ok"
  done
done
