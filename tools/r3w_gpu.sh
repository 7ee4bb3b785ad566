#!/bin/bash
# round 3: 16-wave int8 workgroups (512 queries share each staged tile) -- A/B
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/tune.py --rounds 6 "auto:0:0" "auto:0:0:0:16" > gpurun_out/r3w_nw16.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/tune.py --rounds 2 --m 100000 "auto:0:0" "auto:0:0:0:16" > gpurun_out/r3w_nw16_m100k.log 2>&1
