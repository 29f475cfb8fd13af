# round-6 session 42: the emulated P = 8 rank with one fused launch of all
# eight blocks (KNN_RING_FUSE=all, the exchange exposed on a node) against
# the default own-block launch + fused rest, twice each
set -o pipefail
bash tools/gpu.sh emu:mnist:8:5:all emu:mnist:8:5:rest emu:mnist:8:5:all emu:mnist:8:5:rest
