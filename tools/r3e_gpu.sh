#!/bin/bash
# round 3: int8 selection counts, ablations, parity subset, profiles of the new default
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "i8 or int8 or golden or global" \
  > gpurun_out/r3e_parity.log 2>&1 || exit $?
KNN_AMD_VARIANT=cnt timeout -k 10 200 python -u tools/tune.py --rounds 3 "auto:0:0" \
  > gpurun_out/r3e_cnt.log 2>&1 || exit $?
KNN_AMD_VARIANT=cnt timeout -k 10 200 python -u tools/tune.py --rounds 2 --m 100000 "auto:0:0" \
  > gpurun_out/r3e_cnt_m100k.log 2>&1 || exit $?
KNN_AMD_VARIANT=abl timeout -k 10 240 python -u tools/tune.py --rounds 5 "auto:0:0" \
  "auto:0:0:2" "auto:0:0:3" "auto:0:0:8" "auto:0:0:16" > gpurun_out/r3e_abl.log 2>&1 || exit $?
TAG=r3e bash tools/profile_all.sh stats pmc cfg4 cfg5
AB_TAG=r3e_ab AB_ARGS="--rounds 5 auto:0:0" AB_VARIANTS="base xpd1" REPS=2 bash tools/ab_variants_gpu.sh
