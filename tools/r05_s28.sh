# round-5 session 28: per-workgroup wall clock of k_dist_topk_i8 (stamp ablation build): where a P=8 rank's launches spend their fixed cost
set -o pipefail
mkdir -p gpurun_out/s28
for args in "--nq 7500 --m 7500 --splits 8" "--nq 7500 --splits 8" "--splits 7"; do
  KB8_SO=$PWD/tools/probe/libkbench8_stamp.so timeout -k 10 300 python -u tools/probe/kbench8.py --variant 6 --keep-qthr --iters 3 $args > gpurun_out/s28/kb.log 2>&1 || { tail -20 gpurun_out/s28/kb.log; exit 1; }
  grep '^{' gpurun_out/s28/kb.log
done
