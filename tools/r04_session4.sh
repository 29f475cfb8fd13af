# round-4 session 4: sift k_dist_topk_i8 ablations (half-tile kernel, 5 splits)
set -o pipefail
mkdir -p gpurun_out
K="timeout -k 10 200 python -u tools/probe/kbench8.py --workload sift --variant 6 --splits 5 --iters 3"
true
for v in count noepi_halfdma noepi_nowait rr4s nosum norr filtonly; do
  KB8_SO=tools/probe/abl/libkbench8_$v.so $K > gpurun_out/s4_$v.log 2>&1 || { tail -20 gpurun_out/s4_$v.log; exit 1; }
done
$K --keep-qthr > gpurun_out/s4_base_keep.log 2>&1 || { tail -20 gpurun_out/s4_base_keep.log; exit 1; }
KB8_SO=tools/probe/abl/libkbench8_noepi.so $K --keep-qthr > gpurun_out/s4_noepi_keep.log 2>&1 || exit 1
for f in gpurun_out/s4_*.log; do echo "$f: $(grep '^{' $f | tail -1)"; done
