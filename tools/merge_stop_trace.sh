#!/bin/bash
# Where the merge kernel's time goes: kernel traces of the timing-only
# KNN_MERGE_STOP builds (lib/libknn_amd_ms<N>.so: 1 = loads + error bound,
# 2 = + selection, 3 = + exact re-rank and sort; results invalid, so no
# gate) beside the default build, cfg2 via tools/tune.py.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
for v in base ms1 ms2 ms3; do
  if [ $v = base ]; then unset KNN_AMD_VARIANT; else export KNN_AMD_VARIANT=$v; fi
  timeout -k 10 240 rocprofv3 --kernel-trace -d $O/${TAG:-ms}_$v -o run --output-format csv -- \
    python3 tools/tune.py --rounds 3 --gate 0 auto:0:0 > $O/${TAG:-ms}_$v.log 2>&1 || exit $?
  echo "trace $v done"
done
