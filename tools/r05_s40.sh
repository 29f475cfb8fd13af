# The self-join symmetry estimate: kbench8 on the product
# half-tile kernel against the upper-triangle copies (tools/probe/ablate.py
# tri / tricol, copied to tools/probe/tri/), mnist 60000 x 784, 7 splits
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/s40.log
for mode in --ideal-qthr --keep-qthr; do
  for so in "" tools/probe/tri/libkbench8_tri.so tools/probe/tri/libkbench8_tricol.so; do
    echo "== $mode ${so:-product}" >> $L
    KB8_SO=$so timeout -k 10 300 python -u tools/probe/kbench8.py --variant 6 --splits 7 --iters 10 $mode >> $L 2>&1 || exit 1
  done
done
grep -E '^(==|\{)' $L
