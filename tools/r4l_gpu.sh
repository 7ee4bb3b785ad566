# bench.py main leg (pipelined classify calls) with the train layout in
# train order and in region order, alternating, 2 reps each.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
B="--steps 30 --warmup 5 --no-cpu-baseline --no-fp32-path --no-continuous --no-dropin --no-train-sharded --no-cfg5 --cfg3-queries 0"
for rep in 1 2; do
for o in 0 -1; do
  timeout -k 10 240 python3 -u bench.py $B --order $o > $O/r4l_b_o${o}_$rep.json 2> $O/r4l_b_o${o}_$rep.log
  rc=$?; echo "order $o rc=$rc"; python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(j['ms_per_step'], j['value'], j['roofline']['achieved'], j['roofline']['frac'])" $O/r4l_b_o${o}_$rep.json; [ $rc = 0 ] || exit $rc
done
done
