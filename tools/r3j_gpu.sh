#!/bin/bash
# round 3: grid-stride targeted rescan -- rescan tests, full suite, rescan phase time, bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "targeted or duplicates or rescan or large_d" \
  > gpurun_out/r3j_targeted.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 300 \
  --timeout-method thread > gpurun_out/r3j_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/tune.py --rounds 5 "auto:0:0" > gpurun_out/r3j_tune.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/r3j_bench.log 2>&1
