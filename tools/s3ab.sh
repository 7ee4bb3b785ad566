#!/bin/bash
# cfg5 (d = 960, k = 100) S3 kernel: SQ counter passes and timing-only
# ablations (lib/libknn_amd_abl.so, KNN_ABLATIONS=1 on knn_cand.hip):
# 0 full, 1 no staging after the first steps, 2 no selection, 3 neither
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
TAG=${TAG:-r5s3} WLARGS="--steps 2 --warmup 1 --dim 960 --k 100" bash tools/pmc_sq2.sh || exit $?
export KNN_AMD_VARIANT=abl
timeout -k 10 300 python3 -u tools/tune.py --rounds 3 --n 1000000 --m 10000 --d 960 --k 100 --data continuous \
  auto:0:0 auto:0:0:1 auto:0:0:2 auto:0:0:3 > $O/s3abl.log 2>&1 || exit $?
grep " cand " $O/s3abl.log
