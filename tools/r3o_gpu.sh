#!/bin/bash
# round 3: seeded thresholds A/B, one seed setting per process (no sample rebuilds in the timed calls)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
for s in 0 -1 8192 16384; do
  timeout -k 10 120 python -u tools/tune.py --rounds 5 "auto:0:0,seed=$s" > gpurun_out/r3o_i8_${s}_$rep.log 2>&1 || exit $?
done
done
for s in 0 -1; do
  timeout -k 10 120 python -u tools/tune.py --rounds 5 "auto:0:0,i8=0,seed=$s" > gpurun_out/r3o_f16_${s}.log 2>&1 || exit $?
done
