cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r2_tests_n.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/r2_tests_n.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 tools/tune.py --rounds 3 --d 960 --k 100 "fp16:0:0" "fp16:0:0:4" > gpurun_out/r2_tune_cfg5n.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r2_tune_cfg5n.log
