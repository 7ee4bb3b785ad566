#!/bin/bash
# round 3: int8 256-row tiles as default -- GPU suite, ablations (abl build),
# exchange-period / uniform-branch A/B, default bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 300 \
  --timeout-method thread > gpurun_out/r3d_tests.log 2>&1 || exit $?
KNN_AMD_VARIANT=abl timeout -k 10 240 python -u tools/tune.py --rounds 5 "auto:0:0" "auto:0:0:1" \
  "auto:0:0:2" "auto:0:0:3" "auto:0:0:8" "auto:0:0:16" > gpurun_out/r3d_abl.log 2>&1 || exit $?
AB_TAG=r3d_ab AB_ARGS="--rounds 5 auto:0:0" AB_VARIANTS="base x4 x2 ubr" REPS=2 \
  bash tools/ab_variants_gpu.sh || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/r3d_bench.log 2>&1
