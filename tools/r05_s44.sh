# ksym with one LDS atomic a wave and pair (the survivors as a lane mask, slots
# from a bit-sliced prefix): coverage and timings; the stores ablated
# (sym_nostore); the product kernel cold on the same box
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/s44.log
KSYM_SO=tools/probe/symlib/libkbench8_sym.so timeout -k 10 300 python -u tools/probe/ksym.py --splits-t 7,8 --iters 5 --check 2000 > $L 2>&1 || { tail -20 $L; exit 1; }
KSYM_SO=tools/probe/symlib/libkbench8_sym.so timeout -k 10 300 python -u tools/probe/ksym.py --qa 80 --splits-t 8 --iters 5 --check 2000 >> $L 2>&1 || { tail -20 $L; exit 1; }
KSYM_SO=tools/probe/symlib/libkbench8_sym_nostore.so timeout -k 10 300 python -u tools/probe/ksym.py --splits-t 8 --iters 5 --check 0 >> $L 2>&1 || { tail -20 $L; exit 1; }
timeout -k 10 300 python -u tools/probe/kbench8.py --variant 6 --splits 7 --iters 5 >> $L 2>&1 || { tail -20 $L; exit 1; }
grep '^{' $L
