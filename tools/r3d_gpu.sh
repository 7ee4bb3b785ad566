#!/bin/bash
# round-3 session: cfg2 split-count sweep (in-process A/B), its HBM fetch per
# variant (one FETCH_SIZE pass over the same sweep), then the default bench.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out
stop() { echo "step $1 rc=$2"; exit $2; }
V="fp16:0:0 fp16:0:24 fp16:0:32 fp16:0:40 fp16:0:48 fp16:0:64"
timeout -k 10 200 python3 -u tools/tune.py --rounds 5 $V > $O/r3d_tune_S.log 2>&1 || stop tune $?
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/r3d_fetch -o run \
  --output-format csv -- python3 tools/tune.py --rounds 1 $V > $O/r3d_fetch.log 2>&1 || stop fetch $?
timeout -k 10 600 python3 -u bench.py > $O/r3d_bench.json 2> $O/r3d_bench.log || stop bench $?
echo ok
