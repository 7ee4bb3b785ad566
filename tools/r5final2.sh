#!/bin/bash
# Final build with the split S3 rings: smoke, the whole -m gpu suite, the bench
# line, kernel traces (PART A) and PMC traffic (PART B) of this build.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/fin3_smoke.log 2>&1 || exit $?
tail -1 $O/fin3_smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 300 --timeout-method thread > $O/fin3_tests.log 2>&1 || exit $?
tail -2 $O/fin3_tests.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/fin3_bench.log 2>&1 || exit $?
tail -c 300 $O/fin3_bench.log
TAG=r5g PART=A bash tools/r5_prof.sh || exit $?
TAG=r5g PART=B bash tools/r5_prof.sh || exit $?
echo all done
