#!/bin/bash
# round 3: int8 with 8-entry quad lists (rescan-free at k = 10?) against the default
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/tune.py --rounds 5 "auto:0:0" "auto:8:0" "auto:8:20" "auto:8:26" \
  "auto:8:32" > gpurun_out/r3h_r8.log 2>&1 || exit $?
KNN_AMD_VARIANT=cnt timeout -k 10 240 python -u tools/tune.py --rounds 3 "auto:0:0" "auto:8:0" \
  > gpurun_out/r3h_r8_cnt.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/tune.py --rounds 2 --m 1000000 "auto:0:0" "auto:8:0" "auto:8:32" \
  > gpurun_out/r3h_r8_cfg3.log 2>&1
