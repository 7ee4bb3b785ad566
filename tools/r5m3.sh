#!/bin/bash
# med3 list insertion A/B (base = KNN_MED3=1, m30 = the v_max + v_min form):
# int8 parity tests, cfg2 and the 12.5M x 96 shard interleaved across processes
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_parity.py > $O/m3_tests.log 2>&1; rc=$?; tail -2 $O/m3_tests.log; [ $rc = 0 ] || exit $rc
for rep in 1 2 3; do
  for v in base m30; do
    if [ $v = base ]; then unset KNN_AMD_VARIANT; else export KNN_AMD_VARIANT=$v; fi
    timeout -k 10 200 python3 -u tools/tune.py --rounds 6 auto:0:0 > $O/m3_cfg2_${v}_$rep.log 2>&1 || exit $?
    grep " cand " $O/m3_cfg2_${v}_$rep.log | sed "s/^/cfg2 $v $rep /"
  done
done
for rep in 1 2; do
  for v in base m30; do
    if [ $v = base ]; then unset KNN_AMD_VARIANT; else export KNN_AMD_VARIANT=$v; fi
    timeout -k 10 300 python3 -u tools/tune.py --rounds 3 --n 12500000 --d 96 auto:0:0 > $O/m3_cfg4s_${v}_$rep.log 2>&1 || exit $?
    grep " cand " $O/m3_cfg4s_${v}_$rep.log | sed "s/^/cfg4s $v $rep /"
  done
done
