#!/bin/bash
# round 3: thresholds fetched before the first tile -- parity, A/B (int8, fp16, S3), bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 300 \
  --timeout-method thread > gpurun_out/r3l_tests.log 2>&1 || exit $?
AB_TAG=r3l_ab AB_ARGS="--rounds 5 auto:0:0 auto:0:0,i8=0" AB_VARIANTS="base xs0" REPS=2 \
  bash tools/ab_variants_gpu.sh || exit $?
AB_TAG=r3l_s3 AB_ARGS="--rounds 3 --d 960 --k 100 auto:0:0" AB_VARIANTS="base xs0" REPS=1 \
  bash tools/ab_variants_gpu.sh || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/r3l_bench.log 2>&1
