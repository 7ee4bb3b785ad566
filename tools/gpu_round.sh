#!/bin/bash
# One GPU call of the build/measure loop (every round's one-shot scripts are
# folded into it).  Steps, each with its own time limit, stopping at the
# first failure:
#   SMOKE=1        __graft_entry__.smoke()         -> gpurun_out/$TAG_smoke.log
#   TESTS=1        the whole -m gpu suite          -> gpurun_out/$TAG_tests.log
#   TESTS="<args>" those pytest arguments instead
#   AB_VARIANTS    cross-process A/B of lib/libknn_amd_<v>.so ("base" = default)
#                  with tools/tune.py $AB_ARGS, REPS rounds -> $TAG_ab_<v>_<rep>.log;
#                  every library first passes the parity gate (tests/test_gpu_gate.py:
#                  the oracle on 8 queries + brute-force optimality on 256, for each
#                  tuning variant named in $AB_ARGS; GATE=0 skips) -> $TAG_gate_<v>.log,
#                  and tune.py itself gates each variant before timing it
#   BENCH=1        bench.py --steps 20 --warmup 5 -> $TAG_bench.log / .json
#   PROF=1         rocprofv3 kernel trace + stats of a short bench -> $TAG_prof/
#   PROF_PARTS     "A R B S": tools/prof_round.sh parts (kernel traces of every
#                  workload, RCCL API trace, FETCH/WRITE passes, SQ passes)
#                  -> gpurun_out/prof_$TAG, pmc_sq_$TAG*; tools/profiles_commit.py
#                  --tag $TAG turns them into profiles/
# Usage: TAG=r4b TESTS=1 AB_VARIANTS="base fl" AB_ARGS="--rounds 5 auto:0:0" \
#        bash tools/gpu_round.sh
#        TAG=r4x AB_SETS="--order 0 auto:0:0;--order -1 auto:0:0" bash tools/gpu_round.sh
#        TAG=r4y BENCH_SETS="--order 0;--order -1" bash tools/gpu_round.sh
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
TAG=${TAG:-run}
if [ -n "$SMOKE" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 $O/${TAG}_smoke.log
  [ $rc = 0 ] || exit $rc
fi
if [ -n "$TESTS" ]; then
  args="tests"
  [ "$TESTS" = 1 ] || args="$TESTS"
  timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest -x -q -m gpu --timeout 300 \
      --timeout-method thread $args > $O/${TAG}_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -5 $O/${TAG}_tests.log
  [ $rc = 0 ] || exit $rc
fi
# gate_env: KNN_GATE* variables from a tune.py argument string (its variants
# and workload); timing-only ablation variants (bits 1/2/8/16) are skipped
gate_env() {
  local g="" prev="" t
  GN=1000000; GM=10000; GD=128; GK=10; GDATA=grid; GORD=-1
  for t in $1; do
    case "$prev" in --n) GN=$t;; --m) GM=$t;; --d) GD=$t;; --k) GK=$t;; --data) GDATA=$t;; --order) GORD=$t;; esac
    case "$t" in
      *:*:*) a=$(echo "$t" | cut -d, -f1 | cut -d: -f4); a=${a:-0}
             [ $((a & 27)) = 0 ] && g="$g;$t";;
    esac
    prev=$t
  done
  echo "KNN_GATE='${g#;}' KNN_GATE_N=$GN KNN_GATE_M=$GM KNN_GATE_D=$GD KNN_GATE_K=$GK KNN_GATE_DATA=$GDATA KNN_GATE_ORDER=$GORD"
}
run_gate() {  # $1 variant library ("base" = default), $2 tune.py arguments
  [ "${GATE:-1}" = 0 ] && return 0
  if [ $1 = base ]; then unset KNN_AMD_VARIANT; else export KNN_AMD_VARIANT=$1; fi
  eval "$(gate_env "$2")" timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 240 \
      --timeout-method thread tests/test_gpu_gate.py -s > $O/${TAG}_gate_$1.log 2>&1
  local rc=$?; echo "gate $1 rc=$rc"; grep "^gate " $O/${TAG}_gate_$1.log
  unset KNN_AMD_VARIANT
  return $rc
}
if [ -n "$AB_VARIANTS" ]; then
  for v in $AB_VARIANTS; do run_gate $v "$AB_ARGS" || exit 1; done
  for rep in $(seq 1 ${REPS:-2}); do
    for v in $AB_VARIANTS; do
      if [ $v = base ]; then unset KNN_AMD_VARIANT; else export KNN_AMD_VARIANT=$v; fi
      timeout -k 10 200 python3 -u tools/tune.py $AB_ARGS > $O/${TAG}_ab_${v}_$rep.log 2>&1
      rc=$?; echo "ab $v $rep rc=$rc"; grep " cand " $O/${TAG}_ab_${v}_$rep.log
      [ $rc = 0 ] || exit $rc
    done
  done
  unset KNN_AMD_VARIANT
fi
# AB_SETS: tune.py argument sets separated by ';' (e.g. train layouts, which
# are fixed per process: "--order 0 auto:0:0;--order -1 auto:0:0"), REPS
# rounds of all sets in turn -> $TAG_set<i>_<rep>.log
if [ -n "$AB_SETS" ]; then
  for rep in $(seq 1 ${REPS:-2}); do
    i=0
    IFS=';' read -ra sets <<< "$AB_SETS"
    for a in "${sets[@]}"; do
      i=$((i + 1))
      [ $rep = 1 ] && { run_gate base "$a" || exit 1; }
      timeout -k 10 300 python3 -u tools/tune.py $a > $O/${TAG}_set${i}_$rep.log 2>&1
      rc=$?; echo "set $i ($a) $rep rc=$rc"; grep " cand " $O/${TAG}_set${i}_$rep.log
      [ $rc = 0 ] || exit $rc
    done
  done
fi
# AB_PAIRS: "<variant>|<tune.py arguments>" pairs separated by ';' (a library
# variant with arguments of its own, e.g. a tuning only that build has),
# each gated first, then REPS interleaved rounds -> $TAG_pair<i>_<rep>.log
if [ -n "$AB_PAIRS" ]; then
  IFS=';' read -ra pairs <<< "$AB_PAIRS"
  for p in "${pairs[@]}"; do run_gate "${p%%|*}" "${p#*|}" || exit 1; done
  for rep in $(seq 1 ${REPS:-2}); do
    i=0
    for p in "${pairs[@]}"; do
      i=$((i + 1)); v=${p%%|*}
      if [ $v = base ]; then unset KNN_AMD_VARIANT; else export KNN_AMD_VARIANT=$v; fi
      timeout -k 10 300 python3 -u tools/tune.py ${p#*|} > $O/${TAG}_pair${i}_$rep.log 2>&1
      rc=$?; echo "pair $i ($p) $rep rc=$rc"; grep " cand " $O/${TAG}_pair${i}_$rep.log
      [ $rc = 0 ] || exit $rc
    done
  done
  unset KNN_AMD_VARIANT
fi
# BENCH_SETS: bench.py argument sets separated by ';' (20 timed steps each,
# main leg only), REPS rounds -> $TAG_bset<i>_<rep>.json
if [ -n "$BENCH_SETS" ]; then
  B="--steps 30 --warmup 5 --no-cpu-baseline --no-fp32-path --no-continuous --no-dropin --no-train-sharded --no-cfg5 --cfg3-queries 0"
  for rep in $(seq 1 ${REPS:-2}); do
    i=0
    IFS=';' read -ra sets <<< "$BENCH_SETS"
    for a in "${sets[@]}"; do
      i=$((i + 1))
      timeout -k 10 240 python3 -u bench.py $B $a > $O/${TAG}_bset${i}_$rep.json 2> $O/${TAG}_bset${i}_$rep.log
      rc=$?; echo "bench set $i ($a) $rep rc=$rc"; tail -c 300 $O/${TAG}_bset${i}_$rep.json
      [ $rc = 0 ] || exit $rc
    done
  done
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 ${BENCH_LIMIT:-400} python3 -u bench.py --steps 20 --warmup 5 ${BENCH_ARGS} \
      > $O/${TAG}_bench.json 2> $O/${TAG}_bench.log
  rc=$?; echo "bench rc=$rc"; tail -c 600 $O/${TAG}_bench.json
  [ $rc = 0 ] || exit $rc
fi
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${TAG}_prof -o prof -- \
      python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fp32-path --no-continuous --no-dropin --no-train-sharded --cfg3-queries 0 > $O/${TAG}_prof.log 2>&1
  rc=$?; echo "prof rc=$rc"
  [ $rc = 0 ] || exit $rc
fi
if [ -n "$PROF_PARTS" ]; then
  TAG=$TAG PART="$PROF_PARTS" bash tools/prof_round.sh || exit $?
fi
exit 0
