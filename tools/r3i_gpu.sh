#!/bin/bash
# int8 candidate pass: parity, in-process A/B against fp16, default bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "int8 or integer or golden" > gpurun_out/r3i_parity.log 2>&1 || exit $?
timeout -k 10 240 python -u tools/tune.py --rounds 6 "auto:0:0,i8=0" "auto:0:0,i8=1" \
  > gpurun_out/r3i_ab_cfg2.log 2>&1 || exit $?
timeout -k 10 240 python -u tools/tune.py --rounds 4 --m 100000 "auto:0:0,i8=0" "auto:0:0,i8=1" \
  > gpurun_out/r3i_ab_cfg2_100k.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > gpurun_out/r3i_bench.log 2>&1
