# Region order with 8 stream-start phases on the fp16 pass (continuous data,
# forced 64 regions) and at 100K queries (int8, auto), against train order.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4r; mkdir -p $O
for o in 0 64; do
  timeout -k 10 200 python3 -u tools/tune.py --rounds 5 --order $o --data continuous fp16:0:0 > $O/c_o$o.log 2>&1
  rc=$?; echo "continuous order $o rc=$rc"; grep " cand " $O/c_o$o.log; [ $rc = 0 ] || exit $rc
done
for o in 0 -1; do
  timeout -k 10 200 python3 -u tools/tune.py --rounds 3 --order $o --m 100000 auto:0:0 > $O/m_o$o.log 2>&1
  rc=$?; echo "100k order $o rc=$rc"; grep " cand " $O/m_o$o.log; [ $rc = 0 ] || exit $rc
done
