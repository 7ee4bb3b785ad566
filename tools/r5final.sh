#!/bin/bash
# Final-build GPU evidence, part 1: smoke, the whole -m gpu suite, the bench
# line (20 steps), kernel traces (profile_all.sh stats api + workloads).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/fin_smoke.log 2>&1 || exit $?
tail -1 $O/fin_smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 300 --timeout-method thread > $O/fin_tests.log 2>&1 || exit $?
tail -2 $O/fin_tests.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/fin_bench.log 2>&1 || exit $?
tail -c 600 $O/fin_bench.log
TAG=r5f PART=A bash tools/r5_prof.sh || exit $?
