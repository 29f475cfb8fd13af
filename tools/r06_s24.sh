# round-6 session 24: the two-deep fragment prefetch build -- whole GPU suite
# and smoke, mnist bench, steady trace and PMC passes (pmc_traffic.json is
# keyed to knn_i8.hip's sha1), emulated ring ranks P = 1 / 2 / 4 / 8
set -o pipefail
bash tools/gpu.sh tests bench:mnist:20 trace:mnist pmc:mnist:3 emu:mnist:1,2,4,8
