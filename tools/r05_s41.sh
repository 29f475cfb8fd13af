# The self-join's symmetric launch, first GPU run (tools/probe/ksym.py):
# S + prep + T + scatter timings and neighbour coverage against the exact
# top-k of 2000 sampled queries; the product kernel cold beside it (kbench8)
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/s41.log
KSYM_SO=tools/probe/symlib/libkbench8_sym.so timeout -k 10 300 python -u tools/probe/ksym.py --splits-t 7 --iters 5 --check 2000 > $L 2>&1 || { tail -20 $L; exit 1; }
KSYM_SO=tools/probe/symlib/libkbench8_sym.so timeout -k 10 300 python -u tools/probe/ksym.py --splits-t 5,6,8 --iters 5 --check 0 >> $L 2>&1 || { tail -20 $L; exit 1; }
timeout -k 10 300 python -u tools/probe/kbench8.py --variant 6 --splits 7 --iters 5 >> $L 2>&1 || { tail -20 $L; exit 1; }
cat $L | grep '^{'
