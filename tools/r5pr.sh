#!/bin/bash
# A/B: slow-path issue priority (prio = setprio 2, prio1 = 1) on the int8
# metric-6 kernel (cfg2, 12.5M x 96 shard); S3 row stream non-temporal (s3nt)
# at cfg5, time and FETCH_SIZE per launch.  Interleaved processes.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
ab() {  # ab <tag> <variant> <tune args...>
  local tag=$1 v=$2; shift 2
  if [ $v = base ]; then unset KNN_AMD_VARIANT; else export KNN_AMD_VARIANT=$v; fi
  timeout -k 10 240 python3 -u tools/tune.py "$@" > $O/pr_${tag}_${v}.log 2>&1 || exit $?
  grep " cand " $O/pr_${tag}_${v}.log | sed "s/^/$tag $v /"
  unset KNN_AMD_VARIANT
}
for rep in 1 2 3; do for v in base prio prio1; do ab cfg2_$rep $v --rounds 6 auto:0:0 || exit $?; done; done
for rep in 1 2; do for v in base prio; do ab cfg4s_$rep $v --rounds 3 --n 12500000 --d 96 auto:0:0 || exit $?; done; done
for rep in 1 2; do for v in base s3nt; do ab cfg5_$rep $v --rounds 3 --n 1000000 --m 10000 --d 960 --k 100 --data continuous auto:0:0 || exit $?; done; done
B="--steps 2 --warmup 1 --dim 960 --k 100 --no-cpu-baseline --no-fp32-path --no-continuous --cfg3-queries 0 --no-dropin --no-train-sharded --no-cfg5"
for v in base s3nt; do
  if [ $v = base ]; then unset KNN_AMD_VARIANT; else export KNN_AMD_VARIANT=$v; fi
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pr_fetch_$v -o run --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" $B > $O/pr_fetch_$v.log 2>&1 || exit $?
  echo "fetch $v done"
done
