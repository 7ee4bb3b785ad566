# A/B of the fp16 candidate-kernel MFMA layouts (run through gpurun):
# parity first, then in-process timing of each layout.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
[ -n "$NOPARITY" ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/w_par.log 2>&1; rc=$?; [ -n "$NOPARITY" ] || tail -3 gpurun_out/w_par.log; [ $rc -eq 0 ] || exit $rc
for v in ${VARIANTS:-base}; do
  if [ $v = base ]; then unset KNN_AMD_VARIANT; else export KNN_AMD_VARIANT=$v; fi
  echo "variant $v"
  timeout -k 10 150 python tools/tune.py --rounds 5 ${TUNE_ARGS:-fp16:0:0 f16l:0:0 f16l:4:0 f16l:8:0} > gpurun_out/ab_$v.log 2>&1
  rc=$?
  grep "cand " gpurun_out/ab_$v.log
  [ $rc -eq 0 ] || { tail -5 gpurun_out/ab_$v.log; exit $rc; }
done
