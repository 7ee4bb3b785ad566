#!/bin/bash
# GPU tests, then cfg5 / cfg2 candidate-kernel A/B, then the default bench.
# Any step ending by a signal / time limit ends the script.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out
step() {  # step <name> <limit> <cmd...>: stop on signals/timeouts (rc >= 124)
  local n=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "$n rc=$rc"
  [ $rc -lt 124 ] || exit $rc
}
step r3e_tests 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread
step r3e_cfg5 200 python3 -u tools/tune.py --n 1000000 --m 10000 --d 960 --k 100 --rounds 4 fp16:0:0
step r3e_cfg2S 200 python3 -u tools/tune.py --rounds 5 fp16:0:0 fp16:0:24 fp16:0:32 fp16:0:40 fp16:0:48 fp16:0:64
step r3e_bench 600 python3 -u bench.py
