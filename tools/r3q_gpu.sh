#!/bin/bash
# round 3: merge staging tile / rescan filter grid -- GPU suite, phase times, bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 300 \
  --timeout-method thread > gpurun_out/r3q_tests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/tune.py --rounds 5 "auto:0:0" "auto:0:0,i8=0" > gpurun_out/r3q_tune.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/r3q_bench.log 2>&1
