#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
AB_TAG=r3g_cfg5 AB_ARGS="--n 1000000 --m 10000 --d 960 --k 100 --rounds 4 fp16:0:0" \
  AB_VARIANTS="base r3 r5" bash tools/ab_variants_gpu.sh || exit $?
AB_TAG=r3g_cfg2 AB_ARGS="--rounds 6 fp16:0:0" AB_VARIANTS="base pf" REPS=3 bash tools/ab_variants_gpu.sh
