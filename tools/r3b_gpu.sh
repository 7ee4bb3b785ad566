#!/bin/bash
# round 3: full GPU suite, int8 kernel ablations at cfg2, kernel-stats profiles
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 300 \
  --timeout-method thread > gpurun_out/r3b_tests.log 2>&1 || exit $?
timeout -k 10 240 python -u tools/tune.py --rounds 6 "auto:0:0" "auto:0:0:1" "auto:0:0:2" \
  "auto:0:0:3" "auto:0:0:8" "auto:0:0:16" "auto:0:0,i8=0" > gpurun_out/r3b_abl_i8.log 2>&1 || exit $?
TAG=r3b bash tools/profile_all.sh stats cfg4 cfg5
TAG=r3b bash tools/pmc_sq2.sh
