# Region order with the MFMA assignment: order tests, bench A/B (order 0 /
# auto, 2 reps), and a kernel trace of the ordered cfg2 step.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O/r4n
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_order.py > $O/r4n_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/r4n_tests.log; [ $rc = 0 ] || exit $rc
B="--steps 30 --warmup 5 --no-cpu-baseline --no-fp32-path --no-continuous --no-dropin --no-train-sharded --no-cfg5 --cfg3-queries 0"
for rep in 1 2; do
for o in 0 -1; do
  timeout -k 10 240 python3 -u bench.py $B --order $o > $O/r4n_b_o${o}_$rep.json 2> $O/r4n_b_o${o}_$rep.log
  rc=$?; echo "order $o rc=$rc"; python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(j['ms_per_step'], j['value'], j['roofline']['achieved'], j['roofline']['frac'])" $O/r4n_b_o${o}_$rep.json; [ $rc = 0 ] || exit $rc
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r4n/o1 -o run --output-format csv -- python3 -u bench.py $B --steps 10 --order -1 > $O/r4n/o1.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc = 0 ] || exit $rc
grep -h "region\|sort_\|fill\|merge_rerank\|cand_kernel" $(find $O/r4n/o1 -name "*kernel_stats.csv") | cut -c1-60,200-400 | head
