#!/bin/bash
# Final-build GPU evidence, part 2: RCCL API trace of the forced one-rank
# group tests, FETCH/WRITE passes, SQ passes (tools/r5_prof.sh parts R, B, S);
# then the cfg5 A/B of the split S3 rings (lib/libknn_amd_s3s<NR><NQ>.so) with
# the S3 parity tests on the first of them.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
TAG=r5f PART=R bash tools/r5_prof.sh || exit $?
TAG=r5f PART=B bash tools/r5_prof.sh || exit $?
TAG=r5f PART=S bash tools/r5_prof.sh || exit $?
export KNN_AMD_VARIANT=s3s63
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py::test_cfg5_d960_k100 tests/test_gpu_parity.py -k "s3 or cfg5 or 784 or fp16 or bf16" > $O/s3s_tests.log 2>&1; rc=$?; tail -2 $O/s3s_tests.log; [ $rc = 0 ] || exit $rc
unset KNN_AMD_VARIANT
for rep in 1 2; do
  for v in base s3s63 s3s54 s3s72; do
    if [ $v = base ]; then unset KNN_AMD_VARIANT; else export KNN_AMD_VARIANT=$v; fi
    timeout -k 10 200 python3 -u tools/tune.py --rounds 3 --n 1000000 --m 10000 --d 960 --k 100 --data continuous auto:0:0 > $O/s3s_${v}_$rep.log 2>&1 || exit $?
    grep " cand " $O/s3s_${v}_$rep.log | sed "s/^/$v $rep /"
  done
done
