#!/bin/bash
# A/B of staging-geometry variant libraries (tools/build_variant.sh) on the
# cfg2 shape through tools/tune.py; one process per variant library, the
# variants inside a process interleaved.  Usage (GPU box):
#   tools/ab_geom.sh "base nb4 t2nb4" "fp16:0:0 fp16:0:0:0:16"
cd "$GRAFT_REPO_ROOT" || exit 1
libs=${1:-base}
specs=${2:-fp16:0:0}
rounds=${ROUNDS:-9}
for pass in 1 2; do
  for v in $libs; do
    if [ "$v" = base ]; then unset KNN_AMD_VARIANT; else export KNN_AMD_VARIANT=$v; fi
    echo "== pass $pass lib $v"
    timeout -k 10 150 python tools/tune.py --rounds "$rounds" $specs 2>&1 | grep -v amdgpu.ids
    rc=${PIPESTATUS[0]}
    [ "$rc" -eq 0 ] || exit "$rc"
  done
done
