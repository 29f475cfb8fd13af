# ksym after the long-row norm fix (the init words carry the thresholds):
# coverage at qa = 59, then timings over the seed size and T's split count
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/s42.log
export KSYM_SO=tools/probe/symlib/libkbench8_sym.so
timeout -k 10 300 python -u tools/probe/ksym.py --splits-t 7 --iters 5 --check 2000 > $L 2>&1 || { tail -20 $L; exit 1; }
for qa in 30 45 80; do
  timeout -k 10 300 python -u tools/probe/ksym.py --qa $qa --splits-t 6,8 --iters 5 --check 0 >> $L 2>&1 || { tail -20 $L; exit 1; }
done
grep '^{' $L
