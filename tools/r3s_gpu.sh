#!/bin/bash
# round 3: split count of the int8 cfg2 launch (geometry only)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/tune.py --rounds 6 "auto:0:0" "auto:0:22" "auto:0:25" "auto:0:26" \
  "auto:0:32" "auto:0:51" > gpurun_out/r3s_S.log 2>&1
