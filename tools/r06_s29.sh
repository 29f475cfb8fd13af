# round-6 session 29: evidence of the one-tile-ring build -- mnist bench,
# steady trace, PMC traffic passes (pmc_traffic.json follows knn_i8.hip's
# sha1), emulated ring ranks P = 1 / 2 / 4 / 8
set -o pipefail
bash tools/gpu.sh bench:mnist:20 trace:mnist pmc:mnist:3 emu:mnist:1,2,4,8
