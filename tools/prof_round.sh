#!/bin/bash
# Profiling evidence of one build (any round; TAG names it), each step its own
# time limit (a failing step ends the call):
#   PART=A  kernel trace + stats of cfg2 / cfg4s (12.5M x 96 shard) / cfg5 and
#           of the general-data kernels (cfg2c: fp16 on continuous data,
#           cfg2f32: the fp32 path); HIP API trace of cfg2
#   PART=R  RCCL API + kernel trace of the forced one-rank RCCL group tests
#           (ncclSend / ncclRecv of the tie all-to-all included)
#   PART=B  FETCH_SIZE / WRITE_SIZE passes of the same workloads
#   PART=S  the two SQ passes over cfg2 and over the cfg4s shard
#   PART=Q  cfg5 on the query-resident kernel: trace, FETCH/WRITE, SQ passes
# Outputs under gpurun_out/prof_$TAG and gpurun_out/pmc_sq_$TAG[_cfg4s];
# tools/profiles_commit.py --tag $TAG turns them into profiles/.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-prof}
export TAG
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
for part in ${PART:-A}; do
case "$part" in
  A) bash tools/profile_all.sh stats api cfg4s cfg5 cfg2c cfg2f32 || exit $? ;;
  # (the query-resident cfg5 kernel: trace, traffic and SQ passes)
  Q) bash tools/profile_all.sh stats pmc cfg5q || exit $?
     TAG=${TAG}_cfg5q WLARGS="--steps 2 --warmup 1 --dim 960 --k 100 --tune qres=1" bash tools/pmc_sq2.sh || exit $? ;;
  R) timeout -k 10 300 rocprofv3 --rccl-trace --kernel-trace --stats -d "$OUT/rccl" -o run --output-format csv -- \
       python3 -m pytest -x -q -m gpu --timeout 200 tests/test_gpu_sharded.py -k True \
       > "$OUT/rccl.log" 2>&1 || exit $?
     echo "rccl trace ok"; tail -3 "$OUT/rccl.log" ;;
  B) bash tools/profile_all.sh pmc cfg4s cfg5 cfg2c cfg2f32 || exit $? ;;
  S) bash tools/pmc_sq2.sh || exit $?
     TAG=${TAG}_cfg4s WLARGS="--steps 3 --warmup 1 --mode train --n-train 12500000 --dim 96 --queries 10000" \
       bash tools/pmc_sq2.sh || exit $?
     TAG=${TAG}_cfg2c WLARGS="--steps 3 --warmup 1 --data continuous" bash tools/pmc_sq2.sh || exit $?
     TAG=${TAG}_cfg5 WLARGS="--steps 2 --warmup 1 --dim 960 --k 100" bash tools/pmc_sq2.sh || exit $? ;;
  *) echo "unknown PART $part"; exit 2 ;;
esac
done
