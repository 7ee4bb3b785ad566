#!/bin/bash
# round 3 final: GPU tests, smoke and the default bench on the committed tree
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3x_tests.log 2>&1 || exit $?
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3x_smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/r3x_bench.log 2>&1
