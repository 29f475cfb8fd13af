#!/bin/bash
# Diagnostic copies of libknn with k_dist_split ablated (knn_split.hip's
# SP_ABL_* switches), under tools/abl5/ -- run them with KNN_LIB_PATH.  The
# product library (mpi-knn_amd/lib/libknn.so) is built without them.
#
# Every library here is built from ONE source revision: the committed HEAD,
# exported with `git archive` into a scratch tree, where the library's
# objects are compiled with the product Makefile and each variant's
# knn_split.o beside them.  (Round 5 linked the product tree's build/*.o,
# whatever revision they were at, and compiled only knn_split.hip fresh --
# a kernel whose arguments or block table changed between the two would
# then be launched with the wrong layout.  The r05_s8 aperture violation
# was a different defect, DESIGN.md sec.4.6, but this keeps the class out.)
# Uncommitted changes under mpi-knn_amd/ or include/ are refused: the
# ablation would not measure the source in the working tree.
set -e
HERE="$(cd "$(dirname "$0")" && pwd)"
ROOT="$(dirname "$HERE")"
cd "$ROOT"
if ! git diff --quiet HEAD -- mpi-knn_amd/csrc mpi-knn_amd/Makefile include; then
  echo "split_ablate.sh: mpi-knn_amd/csrc, its Makefile or include/ differ from HEAD; commit first" >&2
  exit 1
fi
REV=$(git rev-parse HEAD)
SCR=$(mktemp -d /tmp/split_ablate.XXXXXX)
trap 'rm -rf "$SCR"' EXIT
git archive HEAD mpi-knn_amd/csrc mpi-knn_amd/Makefile include | tar -x -C "$SCR"
make -s -j8 -C "$SCR/mpi-knn_amd" build/knn_kernels.o build/knn_i8.o build/knn_engine.o build/knn_ring.o \
  build/knn_matio.o build/knn_vote.o build/knn_compat.o build/knn_order.o
ROCM=/opt/rocm
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -I$SCR/include -I$SCR/mpi-knn_amd/csrc -I$ROCM/include"
B="$SCR/mpi-knn_amd/build"
OTHERS="$B/knn_kernels.o $B/knn_i8.o $B/knn_engine.o $B/knn_ring.o $B/knn_matio.o $B/knn_vote.o $B/knn_compat.o $B/knn_order.o"
rm -rf "$HERE/abl5"
mkdir -p "$HERE/abl5/obj"
for v in "noepi:-DSP_ABL_NOEPI=1" "noepi_nodma:-DSP_ABL_NOEPI=1 -DSP_ABL_NODMA=1" \
         "noepi_nofrag:-DSP_ABL_NOEPI=1 -DSP_ABL_NOFRAG=1" "noepi_nomfma:-DSP_ABL_NOEPI=1 -DSP_ABL_NOMFMA=1" \
         "nomfma:-DSP_ABL_NOMFMA=1" "nodma:-DSP_ABL_NODMA=1" "nopre:-DSP_NOPRE=1"; do
  name=${v%%:*}; defs=${v#*:}
  $ROCM/bin/hipcc $FL $defs -c "$SCR/mpi-knn_amd/csrc/knn_split.hip" -o "$HERE/abl5/obj/knn_split_$name.o"
  $ROCM/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$HERE/abl5/libknn_$name.so" $OTHERS \
    "$HERE/abl5/obj/knn_split_$name.o" -L$ROCM/lib -lamdhip64 -lrccl -lz -lm -Wl,-rpath,$ROCM/lib
done
echo "$REV" > "$HERE/abl5/REVISION"
ls -la "$HERE/abl5"
