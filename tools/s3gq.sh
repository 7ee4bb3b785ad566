#!/bin/bash
# cfg5: S3 XCD grouping of query tiles (tuning s3gq: the largest gq tried) in-process A/B
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python3 -u tools/tune.py --rounds 4 --n 1000000 --m 10000 --d 960 --k 100 --data continuous \
  auto:0:0,s3gq=4 auto:0:0,s3gq=2 auto:0:0,s3gq=1 auto:0:0,s3gq=8 > $O/s3gq.log 2>&1 || exit $?
grep " cand " $O/s3gq.log
