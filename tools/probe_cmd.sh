cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "scan" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r2_scan_tests.log 2>&1
echo "tests rc=$?"; tail -5 gpurun_out/r2_scan_tests.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_scan2 -o run --output-format csv -- python3 tools/tune.py --rounds 5 "fp16:0:0,scan=0" "fp16:0:0,scan=1" "fp16:0:25,scan=1" "fp16:0:0,scan=1,scan_a=512" "fp16:0:0,scan=1,scan_a=1024" > gpurun_out/r2_tune_scan2.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r2_tune_scan2.log | grep -v rocprofv3 | grep -v "^[WE]2026"
