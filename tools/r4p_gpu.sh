# Region order: query streams starting at the region (ophase 0) or at one of
# 8 / 4 phases (query tiles of a phase share their streams' start, hence the
# staged tiles in L2): candidate time (interleaved A/B) and L2-miss traffic
# (FETCH_SIZE / WRITE_SIZE passes, one variant per run).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4p; mkdir -p $O
timeout -k 10 200 python3 -u tools/tune.py --rounds 7 auto:0:0,ophase=0 auto:0:0,ophase=8 auto:0:0,ophase=4 > $O/ab.log 2>&1
rc=$?; echo "ab rc=$rc"; grep " cand " $O/ab.log; [ $rc = 0 ] || exit $rc
for ph in 0 8 4; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $O/${c}_$ph -o run --output-format csv -- python3 -u tools/tune.py --rounds 2 auto:0:0,ophase=$ph > $O/${c}_$ph.log 2>&1
    rc=$?; echo "$c $ph rc=$rc"; [ $rc = 0 ] || exit $rc
  done
  python3 tools/pmc_summary.py $O/FETCH_SIZE_$ph cand_kernel | grep FETCH
  python3 tools/pmc_summary.py $O/WRITE_SIZE_$ph cand_kernel | grep WRITE
done
