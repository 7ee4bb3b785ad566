#!/bin/bash
# cfg5: split S3 rings with the longer lead on the query chunks
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
for rep in 1 2; do
  for v in base s3s45 s3s36 s3s27; do
    if [ $v = base ]; then unset KNN_AMD_VARIANT; else export KNN_AMD_VARIANT=$v; fi
    timeout -k 10 200 python3 -u tools/tune.py --rounds 3 --n 1000000 --m 10000 --d 960 --k 100 --data continuous auto:0:0 > $O/s3s2_${v}_$rep.log 2>&1 || exit $?
    grep " cand " $O/s3s2_${v}_$rep.log | sed "s/^/$v $rep /"
  done
done
