# what the cross-split summaries are worth (the symmetric prototype runs
# without them): kbench8 product vs nosum, cold and converged; the triangle
# copy cold (T's situation without the column path)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/s45.log
: > $L
for so in "" tools/probe/tri/libkbench8_nosum.so tools/probe/tri/libkbench8_tri.so; do
  for mode in "" --keep-qthr; do
    echo "== ${so:-product} $mode" >> $L
    KB8_SO=$so timeout -k 10 300 python -u tools/probe/kbench8.py --variant 6 --splits 7 --iters 5 $mode >> $L 2>&1 || { tail -20 $L; exit 1; }
  done
done
grep -E '^(==|\{)' $L
