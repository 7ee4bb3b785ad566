#!/bin/bash
# Cross-process A/B of whole bench steps (main leg only): REPS rounds of
# every library variant in AB_VARIANTS ("base" = the default build), each a
# bench.py run of 30 timed steps -> gpurun_out/$TAG_b<variant>_<rep>.json
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
B="--steps 30 --warmup 5 --no-cpu-baseline --no-fp32-path --no-continuous --no-dropin --no-train-sharded --no-cfg5 --cfg3-queries 0 $BENCH_ARGS"
# parity gate per library before any timing (tests/test_gpu_gate.py: the
# oracle on 8 queries + brute-force optimality on 256 at cfg2)
for v in $AB_VARIANTS; do
  if [ $v = base ]; then unset KNN_AMD_VARIANT; else export KNN_AMD_VARIANT=$v; fi
  timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 240 --timeout-method thread \
      tests/test_gpu_gate.py -s > $O/${TAG}_gate_$v.log 2>&1
  rc=$?; echo "gate $v rc=$rc"; grep "^gate " $O/${TAG}_gate_$v.log
  [ $rc = 0 ] || exit 1
done
for rep in $(seq 1 ${REPS:-2}); do
  for v in $AB_VARIANTS; do
    if [ $v = base ]; then unset KNN_AMD_VARIANT; else export KNN_AMD_VARIANT=$v; fi
    timeout -k 10 300 python3 -u bench.py $B > $O/${TAG}_b${v}_$rep.json 2> $O/${TAG}_b${v}_$rep.log
    rc=$?; echo "bench $v $rep rc=$rc"
    [ $rc = 0 ] || exit $rc
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('  %.4f ms/step  %.0f q/s  kernel %.4f  prep %.4f rerank %.4f rescan %.4f resc %s' % (d['ms_per_step'], d['value'], r['kernel_ms'], r['prep_ms'], r['rerank_ms'], r['rescan_ms'], d['config']['rescanned_queries']))" $O/${TAG}_b${v}_$rep.json
  done
done
unset KNN_AMD_VARIANT
