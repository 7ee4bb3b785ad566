#!/bin/bash
# Two SQ counter passes (<= 8 SQ counters each, their own runs) over a short
# cfg2 bench (or the WLARGS workload): issue/wait breakdown of the candidate kernel.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-r2k}
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_sq_$TAG
mkdir -p "$OUT"
# WLARGS: another workload's bench arguments (default: cfg2)
B="${WLARGS:---steps 3 --warmup 1} --no-cpu-baseline --no-fp32-path --no-continuous --cfg3-queries 0 --no-dropin --no-train-sharded --no-cfg5"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
  --kernel-trace -d "$OUT/p1" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" $B \
  > "$OUT/p1.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_BRANCH \
  SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
  --kernel-trace -d "$OUT/p2" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" $B \
  > "$OUT/p2.log" 2>&1 || exit $?
echo done
