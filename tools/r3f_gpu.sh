#!/bin/bash
# round 3: how much perfectly seeded thresholds would save (ablate bit 5 keeps the
# previous call's final gthr for the same queries); long-stream split counts
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/tune.py --rounds 5 "auto:0:0" "auto:0:0:32" \
  > gpurun_out/r3f_seed.log 2>&1 || exit $?
KNN_AMD_VARIANT=cnt timeout -k 10 240 python -u tools/tune.py --rounds 3 "auto:0:0" "auto:0:0:32" \
  > gpurun_out/r3f_seed_cnt.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/tune.py --rounds 2 --n 25000000 --d 96 "auto:0:0" "auto:0:64" \
  "auto:0:0:32" > gpurun_out/r3f_n25m.log 2>&1
