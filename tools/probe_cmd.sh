cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "large_d or 960 or 784 or 520 or 300" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2_tests_l.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r2_tests_l.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 tools/tune.py --rounds 3 --d 960 --k 100 --m 10000 "fp16:0:0" > gpurun_out/r2_tune_cfg5m.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r2_tune_cfg5m.log
