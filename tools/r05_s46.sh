# the cross-split summaries at the P = 8 fused launch's shape (7500 queries
# x 60000 rows, 8 splits): kbench8 product vs nosum, cold and converged
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/s46.log
: > $L
for so in "" tools/probe/tri/libkbench8_nosum.so "" tools/probe/tri/libkbench8_nosum.so; do
  for mode in "" --keep-qthr; do
    echo "== ${so:-product} $mode" >> $L
    KB8_SO=$so timeout -k 10 300 python -u tools/probe/kbench8.py --variant 6 --splits 8 --nq 7500 --iters 10 $mode >> $L 2>&1 || { tail -20 $L; exit 1; }
  done
done
grep -E '^(==|\{)' $L
