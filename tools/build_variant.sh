#!/bin/bash
# Experiment build: the library with extra flags on the candidate kernel TUs
# (the resident kernel groups and knn_cand.hip: S3 / stream kernels), as
# -mpi-knn-_amd/lib/libknn_amd_<name>.so (selected at run time with
# KNN_AMD_VARIANT=<name>).  Usage: tools/build_variant.sh nb4 -DKNN_RES_NB=4
set -e
name=$1; shift
cd "$(dirname "$0")/../-mpi-knn-_amd"
make -s -j8 >/dev/null
mkdir -p build/$name
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-honor-nans"
rm -f build/$name/res_*.o build/$name/cand.o
# VGROUPS: the resident-kernel groups to rebuild (default all); VCAND=0 keeps
# the default knn_cand.o (S3 / stream kernels)
for g in ${VGROUPS:-0 1 2 3}; do
  /opt/rocm/bin/hipcc $HIPFLAGS "$@" -DKNN_GROUP=$g -c csrc/knn_cand_res.hip -o build/$name/res_$g.o 2>/dev/null &
done
[ "${VCAND:-1}" = 0 ] || /opt/rocm/bin/hipcc $HIPFLAGS "$@" -c csrc/knn_cand.hip -o build/$name/cand.o 2>/dev/null &
rm -f build/$name/qres.o
[ "${VQRES:-1}" = 0 ] || /opt/rocm/bin/hipcc $HIPFLAGS "$@" -c csrc/knn_cand_qres.hip -o build/$name/qres.o 2>/dev/null &
wait
[ -f build/$name/cand.o ] || cp build/knn_cand.o build/$name/cand.o
[ -f build/$name/qres.o ] || cp build/knn_cand_qres.o build/$name/qres.o
# a group whose kernels do not fit the variant's geometry (LDS) keeps the
# default build's objects, so the library still links completely
for g in 0 1 2 3; do
  [ -f build/$name/res_$g.o ] || cp build/knn_cand_res_$g.o build/$name/res_$g.o
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/libknn_amd_$name.so \
  build/knn_prep.o build/$name/cand.o build/$name/qres.o build/knn_select.o build/knn_order.o build/$name/res_*.o \
  build/knn_normalize.o build/knn_api.o build/knn_group.o \
  -L/opt/rocm/lib -lamdhip64 -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built lib/libknn_amd_$name.so"
