# round-6 session 1: the whole -m gpu suite (all-row hash checks, RCCL-self
# P = 8 at full size) + smoke, the default bench line (merge / pack entries),
# the int8 kernel with a first-round stagger between the two workgroups of a
# CU (kbench8, P = 1 shape, cold and converged bounds), and last the
# noepi+nodma split ablation that faulted in r05_s8, rebuilt from one
# revision (tools/split_ablate.sh, REVISION beside the library)
set -o pipefail
mkdir -p gpurun_out/r06s1
bash tools/gpu.sh tests bench:mnist || exit $?
L=gpurun_out/r06s1/kb8.log
: > $L
for so in "" tools/probe/stag/libkbench8_stagA_1.so tools/probe/stag/libkbench8_stagA_2.so tools/probe/stag/libkbench8_stagA_3.so tools/probe/stag/libkbench8_stagB_2.so; do
  for mode in "" --keep-qthr; do
    echo "== ${so:-product} $mode" >> $L
    KB8_SO=$so timeout -k 10 200 python -u tools/probe/kbench8.py --variant 6 --splits 7 --iters 5 $mode >> $L 2>&1 || { tail -20 $L; exit 1; }
  done
done
grep -E '^(==|\{)' $L
echo "== noepi_nodma ($(cat tools/abl6/REVISION))"
KNN_LIB_PATH=$PWD/tools/abl6/libknn_noepi_nodma.so timeout -k 10 200 python3 bench.py --workload mnist-real --steps 3 --warmup 1 --no-cpu-baseline --check 0 --secondary-steps 0 > gpurun_out/r06s1/mr_noepi_nodma.log 2>&1 || { tail -20 gpurun_out/r06s1/mr_noepi_nodma.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"avg_launch_ms": [0-9.]*' gpurun_out/r06s1/mr_noepi_nodma.log | tr '\n' ' '; echo
