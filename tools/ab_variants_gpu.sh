#!/bin/bash
# Cross-process A/B of library variants (lib/libknn_amd_<v>.so, "base" = the
# default build) with tools/tune.py, interleaved REPS times.
#   AB_TAG=<log prefix> AB_ARGS="<tune.py args>" AB_VARIANTS="base r3 ..." [REPS=2]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
  for v in $AB_VARIANTS; do
    if [ $v = base ]; then unset KNN_AMD_VARIANT; else export KNN_AMD_VARIANT=$v; fi
    timeout -k 10 200 python3 -u tools/tune.py $AB_ARGS > $O/${AB_TAG}_${v}_$rep.log 2>&1
    rc=$?; echo "$AB_TAG $v $rep rc=$rc"; [ $rc -lt 124 ] || exit $rc
  done
done
