# Region order after the per-call overhead cut: its GPU tests, then A/B of
# the train layout on cfg2 (grid, int8), continuous data (fp16) and 100K queries.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v -m gpu --timeout 200 --timeout-method thread tests/test_gpu_order.py > $O/r4j_order_tests.log 2>&1
rc=$?; echo "order tests rc=$rc"; tail -3 $O/r4j_order_tests.log; [ $rc = 0 ] || exit $rc
for rep in 1 2; do
for o in 0 -1; do
  timeout -k 10 200 python3 -u tools/tune.py --rounds 5 --order $o auto:0:0 > $O/r4j_ab_o${o}_$rep.log 2>&1
  rc=$?; echo "order $o rc=$rc"; grep " cand \|phases" $O/r4j_ab_o${o}_$rep.log; [ $rc = 0 ] || exit $rc
done
done
for o in 0 64; do
  timeout -k 10 200 python3 -u tools/tune.py --rounds 5 --order $o --data continuous fp16:0:0 > $O/r4jc_ab_o${o}.log 2>&1
  rc=$?; echo "continuous order $o rc=$rc"; grep " cand \|phases" $O/r4jc_ab_o${o}.log; [ $rc = 0 ] || exit $rc
  timeout -k 10 200 python3 -u tools/tune.py --rounds 3 --order $o --m 100000 auto:0:0 > $O/r4jm_ab_o${o}.log 2>&1
  rc=$?; echo "100k order $o rc=$rc"; grep " cand \|phases" $O/r4jm_ab_o${o}.log; [ $rc = 0 ] || exit $rc
done
