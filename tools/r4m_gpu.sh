# Kernel trace + stats of the cfg2 main leg with the region order (which
# kernels the per-call query ordering costs).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4m; mkdir -p $O
B="--steps 10 --warmup 2 --no-cpu-baseline --no-fp32-path --no-continuous --no-dropin --no-train-sharded --no-cfg5 --cfg3-queries 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/o1 -o run --output-format csv -- python3 -u bench.py $B --order -1 > $O/o1.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc = 0 ] || exit $rc
f=$(find $O/o1 -name "*kernel_stats.csv" | head -1); head -30 "$f"
