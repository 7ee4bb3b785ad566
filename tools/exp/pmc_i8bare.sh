#!/bin/bash
# SQ counter passes over the int8 bare-loop experiment (tools/exp/i8bare.hip
# builds i8bare_<v>), one rocprofv3 run per pass.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_i8bare
mkdir -p "$OUT"
for v in ${VARIANTS:-pf0}; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
    --kernel-trace -d "$OUT/${v}_p1" -o run --output-format csv -- ./tools/exp/i8bare_$v 40 \
    > "$OUT/${v}_p1.log" 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_BRANCH \
    SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
    --kernel-trace -d "$OUT/${v}_p2" -o run --output-format csv -- ./tools/exp/i8bare_$v 40 \
    > "$OUT/${v}_p2.log" 2>&1 || exit $?
done
echo done
