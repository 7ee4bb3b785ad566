#!/bin/bash
# GPU-box profiling of the bench workloads (run through gpurun):
#   stats  rocprofv3 --kernel-trace --stats of bench.py (cfg2 / cfg4 / cfg5)
#   pmc    FETCH_SIZE and WRITE_SIZE in separate passes (MI355X_MICROARCH.md,
#          HBM section; each pass its own run, --kernel-trace only)
#   api    rocprofv3 --hip-trace of a short cfg2 bench: the HIP calls made
#          inside the timed knn_classify_device loop (no stream syncs)
# Usage: TAG=r2 tools/profile_all.sh [stats] [pmc] [api] [cfg4] [cfg4s] [cfg5] [cfg5q] [cfg2c] [cfg2f32]
# Outputs under gpurun_out/prof_$TAG/; tools/profiles_commit.py turns them
# into the committed profiles/ files.  Every GPU step has its own time limit
# and a failing step ends the script.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-r2}
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
# the source identity of the build being profiled (tools/profiles_commit.py
# refuses to stamp a different tree's sha onto these results)
python3 -c "import sys; sys.path.insert(0, '$GRAFT_REPO_ROOT'); import bench; print(bench.kernel_src_sha())" > "$OUT/src_sha.txt"
BENCH_COMMON="--no-cpu-baseline --no-fp32-path --no-continuous --cfg3-queries 0 --no-dropin --no-train-sharded --no-cfg5"
declare -A WL
WL[cfg2]="--steps 10 --warmup 2"
WL[cfg4]="--steps 3 --warmup 1 --mode train --n-train 100000000 --dim 96 --queries 10000"
WL[cfg5]="--steps 4 --warmup 1 --dim 960 --k 100"
# cfg5 on the query-resident fp16 kernel (tuning "qres" 1; AUTO keeps S3)
WL[cfg5q]="--steps 4 --warmup 1 --dim 960 --k 100 --tune qres=1"
# the general-data kernels: fp16 on continuous (min-max normalised) data and
# the fp32 path, each as the main leg
WL[cfg2c]="--steps 10 --warmup 2 --data continuous"
WL[cfg2f32]="--steps 4 --warmup 1 --precision fp32"
# configs[3] at the 8-GPU shard size (100M / 8 rows per rank)
WL[cfg4s]="--steps 5 --warmup 1 --mode train --n-train 12500000 --dim 96 --queries 10000"
run() {  # run <name> <limit> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "== $name"
  timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -2 "$OUT/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
cfgs="cfg2"
for a in "$@"; do case $a in cfg4|cfg5|cfg5q|cfg4s|cfg2c|cfg2f32) cfgs="$cfgs $a" ;; esac; done
for a in "$@"; do
  case $a in
    stats)
      for c in $cfgs; do
        run stats_$c 600 rocprofv3 --kernel-trace --stats -d "$OUT/stats_$c" -o run \
          --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" ${WL[$c]} $BENCH_COMMON
        cp "$OUT/stats_$c.log" "$OUT/stats_$c/bench_line.txt"
      done ;;
    pmc)
      for c in $cfgs; do
        run fetch_$c 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/fetch_$c" -o run \
          --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" ${WL[$c]} $BENCH_COMMON
        run write_$c 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/write_$c" -o run \
          --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" ${WL[$c]} $BENCH_COMMON
      done ;;
    api)
      run api_cfg2 600 rocprofv3 --hip-trace --kernel-trace -d "$OUT/api_cfg2" -o run \
        --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 \
        $BENCH_COMMON ;;
  esac
done
