# round-6 session 33: kernel trace of the emulated P = 8 rank (gaps between
# the own launch, the fused launch, the merge and the count)
set -o pipefail
bash tools/gpu.sh emutrace:mnist:8
