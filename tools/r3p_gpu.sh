#!/bin/bash
# round 3: the build with seeding off by default -- full GPU suite, smoke, bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 300 \
  --timeout-method thread > gpurun_out/r3p_tests.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3p_smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/r3p_bench.log 2>&1
