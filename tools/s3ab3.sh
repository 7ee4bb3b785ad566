#!/bin/bash
# cfg5: split S3 rings with NQ > NR, prologue fixed (both rings' leads issued);
# the S3 parity tests on the first variant, then interleaved timing
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
export KNN_AMD_VARIANT=s3s27
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py::test_cfg5_d960_k100 tests/test_gpu_parity.py -k "s3 or cfg5 or 784 or fp16 or bf16" > $O/s3s3_tests.log 2>&1; rc=$?; tail -2 $O/s3s3_tests.log; [ $rc = 0 ] || exit $rc
unset KNN_AMD_VARIANT
for rep in 1 2; do
  for v in base s3s27 s3s36 s3s45; do
    if [ $v = base ]; then unset KNN_AMD_VARIANT; else export KNN_AMD_VARIANT=$v; fi
    timeout -k 10 200 python3 -u tools/tune.py --rounds 3 --n 1000000 --m 10000 --d 960 --k 100 --data continuous auto:0:0 > $O/s3s3_${v}_$rep.log 2>&1 || exit $?
    grep " cand " $O/s3s3_${v}_$rep.log | sed "s/^/$v $rep /"
  done
done
