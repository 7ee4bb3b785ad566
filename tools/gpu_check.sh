#!/bin/bash
# GPU-box check script (run through gpurun).  Stages: smoke tests bench prof
# pmc; each GPU step has its own time limit; a crash/timeout (rc not 0/1)
# stops the script so nothing else touches the GPU after a fault.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r1}
if [ $# -eq 0 ]; then set -- smoke tests bench; fi
step() {  # step <name> <limit-seconds> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$lim" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -3 "gpurun_out/${TAG}_${name}.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
nc=0
for s in "$@"; do
  case $s in
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step tests 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 300 --timeout-method thread ;;
    testsall) step testsall 900 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
    bench) step bench 600 python bench.py --steps 10 --warmup 2 ;;
    prof)
      export TMPDIR=/tmp
      step prof 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" \
        -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 1 \
        --no-cpu-baseline ;;
    pmc)
      export TMPDIR=/tmp
      step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_fetch_$TAG" \
        -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 \
        --no-cpu-baseline
      step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_write_$TAG" \
        -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 \
        --no-cpu-baseline ;;
    pmcsq)
      export TMPDIR=/tmp
      step pmc_sq 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU \
        SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace \
        -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_sq_$TAG" -o run --output-format csv -- \
        python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline ;;
    tune) step tune 600 python tools/tune.py ${TUNE_ARGS:-} ;;
    *) nc=$((nc+1)); step custom$nc 600 bash -c "$s" ;;
  esac
done
