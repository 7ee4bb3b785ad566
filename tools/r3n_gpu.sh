#!/bin/bash
# round 3: seeded thresholds -- parity, A/B of the sample size (int8, fp16), bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "seeded or int8 or global or targeted" \
  > gpurun_out/r3n_parity.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/tune.py --rounds 5 "auto:0:0,seed=0" "auto:0:0" "auto:0:0,seed=16384" \
  "auto:0:0,seed=65536" "auto:0:0,i8=0,seed=0" "auto:0:0,i8=0" > gpurun_out/r3n_ab.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/tune.py --rounds 2 --m 1000000 "auto:0:0,seed=0" "auto:0:0" \
  > gpurun_out/r3n_cfg3.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 300 \
  --timeout-method thread > gpurun_out/r3n_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/r3n_bench.log 2>&1
