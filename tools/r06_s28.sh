# round-6 session 28: the one-tile-ring build -- whole GPU suite and smoke,
# mnist bench, SQ instruction mix and cycle buckets, emulated ranks P = 1, 8
set -o pipefail
bash tools/gpu.sh tests bench:mnist:20 pmcx:mnist:inst pmcx:mnist:cyc emu:mnist:1,8 > gpurun_out/r06s28.log 2>&1 || { tail -40 gpurun_out/r06s28.log; exit 1; }
grep -E "passed|smoke|^\{\"metric|\"P\"" gpurun_out/r06s28.log | cut -c1-400
