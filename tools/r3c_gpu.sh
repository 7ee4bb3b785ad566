#!/bin/bash
# round 3: int8 kernel ablations (quiet), staging / query-block variants: parity + A/B
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in i8qb4 i8nb3 i8tpb8 i8qb4nb3; do
  KNN_AMD_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x \
    -p no:cacheprovider --timeout 120 --timeout-method thread -k "i8 or int8" \
    > gpurun_out/r3c_parity_$v.log 2>&1 || exit $?
done
timeout -k 10 240 python -u tools/tune.py --rounds 5 "auto:0:0" "auto:0:0:1" "auto:0:0:2" \
  "auto:0:0:3" "auto:0:0:16" "auto:0:0:8" > gpurun_out/r3c_abl_i8.log 2>&1 || exit $?
AB_TAG=r3c_ab AB_ARGS="--rounds 5 auto:0:0 auto:0:0:0:4" AB_VARIANTS="base i8nb3 i8tpb8 i8qb4 i8qb4nb3" \
  REPS=2 bash tools/ab_variants_gpu.sh
