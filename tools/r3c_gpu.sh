set -o pipefail
cd $GRAFT_REPO_ROOT 2>/dev/null || true
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread > gpurun_out/r3c_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/r3c_tests.log
for v in base s3old s3r6; do
  if [ $v = base ]; then unset KNN_AMD_VARIANT; else export KNN_AMD_VARIANT=$v; fi
  timeout -k 10 150 python -u tools/tune.py --n 1000000 --m 10000 --d 960 --k 100 --rounds 5 fp16:0:0 > gpurun_out/r3c_s3_$v.log 2>&1 || { echo "tune $v failed rc=$?"; break; }
done
