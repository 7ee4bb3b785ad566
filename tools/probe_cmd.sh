cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r2_tests_i.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r2_tests_i.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 tools/tune.py --rounds 3 --d 960 --k 100 --m 10000 "fp16:0:0" "fp16:8:64" > gpurun_out/r2_tune_cfg5j.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r2_tune_cfg5j.log
