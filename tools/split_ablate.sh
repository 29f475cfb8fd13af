#!/bin/bash
# Diagnostic copies of libknn with k_dist_split ablated (knn_split.hip's
# SP_ABL_* switches), under tools/abl5/ -- run them with KNN_LIB_PATH.  The
# product library (mpi-knn_amd/lib/libknn.so) is built without them.
set -e
cd "$(dirname "$0")/../mpi-knn_amd"
mkdir -p ../tools/abl5/obj
ROCM=/opt/rocm
FL="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden -I../include -Icsrc -I$ROCM/include"
OTHERS="build/knn_kernels.o build/knn_i8.o build/knn_engine.o build/knn_ring.o build/knn_matio.o build/knn_vote.o build/knn_compat.o build/knn_order.o"
for v in "noepi:-DSP_ABL_NOEPI=1" "noepi_nodma:-DSP_ABL_NOEPI=1 -DSP_ABL_NODMA=1" \
         "noepi_nofrag:-DSP_ABL_NOEPI=1 -DSP_ABL_NOFRAG=1" "noepi_nomfma:-DSP_ABL_NOEPI=1 -DSP_ABL_NOMFMA=1" \
         "nomfma:-DSP_ABL_NOMFMA=1" "nodma:-DSP_ABL_NODMA=1" "nopre:-DSP_NOPRE=1"; do
  name=${v%%:*}; defs=${v#*:}
  $ROCM/bin/hipcc $FL $defs -c csrc/knn_split.hip -o ../tools/abl5/obj/knn_split_$name.o
  $ROCM/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../tools/abl5/libknn_$name.so $OTHERS \
    ../tools/abl5/obj/knn_split_$name.o -L$ROCM/lib -lamdhip64 -lrccl -lz -lm -Wl,-rpath,$ROCM/lib
done
ls -la ../tools/abl5
