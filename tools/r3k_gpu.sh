#!/bin/bash
# int8: parity after the saturating query codes, rescan at 1M queries, tile-size A/B
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "int8 or integer or golden or nonfinite" > gpurun_out/r3k_parity.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/tune.py --rounds 2 --m 1000000 "auto:0:0,i8=1" \
  > gpurun_out/r3k_cfg3.log 2>&1 || exit $?
AB_TAG=r3k_cfg2 AB_ARGS="--rounds 6 auto:0:0,i8=1 auto:0:0:2,i8=1" AB_VARIANTS="base tpb8" REPS=2 \
  bash tools/ab_variants_gpu.sh || exit $?
AB_TAG=r3k_m100k AB_ARGS="--rounds 3 --m 100000 auto:0:0,i8=1" AB_VARIANTS="base tpb8" REPS=1 \
  bash tools/ab_variants_gpu.sh
