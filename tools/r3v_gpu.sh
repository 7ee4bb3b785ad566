#!/bin/bash
# round 3: denser threshold exchanges in the first 16 / 32 tiles only -- A/B
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
AB_TAG=r3v_ab AB_ARGS="--rounds 5 auto:0:0 auto:0:0,i8=0" AB_VARIANTS="base e2 e3" REPS=2 \
  bash tools/ab_variants_gpu.sh
