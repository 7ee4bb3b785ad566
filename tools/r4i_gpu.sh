# Region order: its GPU tests, then cross-process A/B of the train layout
# (order 0 / auto / 64 regions) with the query streams' start at the region
# or at one of 8 phases (cfg2 and a 12.5M x 96 shard).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v -m gpu --timeout 200 --timeout-method thread tests/test_gpu_order.py > $O/r4i_order_tests.log 2>&1
rc=$?; echo "order tests rc=$rc"; tail -8 $O/r4i_order_tests.log; [ $rc = 0 ] || exit $rc
for o in 0 -1 64; do
  timeout -k 10 200 python3 -u tools/tune.py --rounds 5 --order $o auto:0:0 auto:0:0,ophase=8 > $O/r4i_ab_o${o}.log 2>&1
  rc=$?; echo "order $o rc=$rc"; grep " cand " $O/r4i_ab_o${o}.log; [ $rc = 0 ] || exit $rc
done
for o in 0 -1; do
  timeout -k 10 240 python3 -u tools/tune.py --rounds 3 --order $o --n 12500000 --d 96 auto:0:0 auto:0:0,ophase=8 > $O/r4i4_ab_o${o}.log 2>&1
  rc=$?; echo "cfg4 order $o rc=$rc"; grep " cand " $O/r4i4_ab_o${o}.log; [ $rc = 0 ] || exit $rc
done
timeout -k 10 300 python3 -u tools/tune.py --rounds 3 --d 960 --k 100 --data continuous auto:0:0,s3gq=4 auto:0:0,s3gq=8 > $O/r4i5_ab.log 2>&1
rc=$?; echo "cfg5 rc=$rc"; grep " cand " $O/r4i5_ab.log; [ $rc = 0 ] || exit $rc
