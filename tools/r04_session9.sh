# round-4 session 9: mnist half-tile kernel ablations (kbench8 variant 6, 7 splits)
set -o pipefail
mkdir -p gpurun_out
K="timeout -k 10 200 python -u tools/probe/kbench8.py --workload mnist --variant 6 --splits 7 --iters 5"
$K > gpurun_out/s9_base.log 2>&1 || { tail -20 gpurun_out/s9_base.log; exit 1; }
for v in noepi noepi_nodma noepi_nodma_nobar noepi_halfdma noepi_nowait filtonly; do
  KB8_SO=tools/probe/abl/libkbench8_$v.so $K > gpurun_out/s9_$v.log 2>&1 || { tail -20 gpurun_out/s9_$v.log; exit 1; }
done
$K --keep-qthr > gpurun_out/s9_base_keep.log 2>&1 || exit 1
for f in gpurun_out/s9_*.log; do echo "$f: $(grep -o '"ms": [0-9.]*' $f | tail -1)"; done
