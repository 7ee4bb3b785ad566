#!/bin/bash
# round 3: own-list threshold publish -- parity on the variant, A/B against the default
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
KNN_AMD_VARIANT=own timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r3u_parity.log 2>&1 || exit $?
AB_TAG=r3u_ab AB_ARGS="--rounds 5 auto:0:0 auto:0:0,i8=0" AB_VARIANTS="base own" REPS=2 \
  bash tools/ab_variants_gpu.sh
