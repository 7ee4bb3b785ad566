#!/bin/bash
# Round-4 evidence in two GPU calls (each step its own time limit; a failing
# step ends the call):
#   PART=A  kernel trace + stats of cfg2 / cfg4s (12.5M x 96 shard) / cfg5;
#           HIP API trace of cfg2; RCCL API + kernel trace of the forced
#           one-rank RCCL group tests (PART=R: that step alone)
#   PART=B  FETCH_SIZE / WRITE_SIZE passes (cfg2, cfg4s, cfg5) and the two SQ
#           passes over cfg2
# Outputs under gpurun_out/prof_$TAG and gpurun_out/pmc_sq_$TAG;
# tools/profiles_commit.py --tag $TAG turns them into profiles/.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-r4}
export TAG
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
if [ "$PART" = A ] || [ "$PART" = R ]; then
  [ "$PART" = R ] || bash tools/profile_all.sh stats api cfg4s cfg5 || exit $?
  timeout -k 10 300 rocprofv3 --rccl-trace --kernel-trace --stats -d "$OUT/rccl" -o run --output-format csv -- \
    python3 -m pytest -x -q -m gpu --timeout 200 tests/test_gpu_sharded.py -k True \
    > "$OUT/rccl.log" 2>&1 || exit $?
  echo "rccl trace ok"; tail -3 "$OUT/rccl.log"
else
  bash tools/profile_all.sh pmc cfg4s cfg5 || exit $?
  bash tools/pmc_sq2.sh || exit $?
fi
