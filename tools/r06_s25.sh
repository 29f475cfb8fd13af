# round-6 session 25: SQ counter groups of the PF2 int8 kernel (instruction
# mix, cycle buckets, LDS activity and bank conflicts), one pass each
set -o pipefail
bash tools/gpu.sh pmcx:mnist:inst pmcx:mnist:cyc pmcx:mnist:lds > gpurun_out/r06s25.log 2>&1 || { tail -30 gpurun_out/r06s25.log; exit 1; }
grep -v '^step' gpurun_out/r06s25.log | tail -60
