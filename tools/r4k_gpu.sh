# Region order after the centroid-transpose / batched-mapping cut: GPU tests
# (order + parity subset), then cfg2 A/B (order 0 vs auto, 2 reps).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_order.py tests/test_gpu_parity.py -k "order or ord or targeted" > $O/r4k_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/r4k_tests.log; [ $rc = 0 ] || exit $rc
for rep in 1 2; do
for o in 0 -1; do
  timeout -k 10 200 python3 -u tools/tune.py --rounds 5 --order $o auto:0:0 > $O/r4k_ab_o${o}_$rep.log 2>&1
  rc=$?; echo "order $o rc=$rc"; grep " cand \|phases" $O/r4k_ab_o${o}_$rep.log; [ $rc = 0 ] || exit $rc
done
done
