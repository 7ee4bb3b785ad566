#!/bin/bash
# round 3: per-split certification + targeted rescan -- GPU suite and the default bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "targeted or duplicates or rescan" \
  > gpurun_out/r3i_targeted.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 300 \
  --timeout-method thread > gpurun_out/r3i_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/r3i_bench.log 2>&1
