#!/bin/bash
# round 3: int8 selection counts with thresholds fetched at tile 0, and with perfect seeds
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
KNN_AMD_VARIANT=cnt timeout -k 10 240 python -u tools/tune.py --rounds 3 "auto:0:0" "auto:0:0:32" \
  > gpurun_out/r3m_cnt.log 2>&1 || exit $?
timeout -k 10 240 python -u tools/tune.py --rounds 5 "auto:0:0" "auto:0:0:32" \
  > gpurun_out/r3m_seed.log 2>&1
