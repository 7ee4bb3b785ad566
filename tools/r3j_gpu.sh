#!/bin/bash
# int8: phase breakdown at 1M queries (cfg3), kernel ablations at cfg2
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/tune.py --rounds 2 --m 1000000 "auto:0:0,i8=0" "auto:0:0,i8=1" \
  > gpurun_out/r3j_cfg3.log 2>&1 || exit $?
timeout -k 10 240 python -u tools/tune.py --rounds 6 "auto:0:0,i8=1" "auto:0:0:1,i8=1" "auto:0:0:2,i8=1" \
  "auto:0:0:3,i8=1" "auto:0:0:4,i8=1" > gpurun_out/r3j_abl_i8.log 2>&1
