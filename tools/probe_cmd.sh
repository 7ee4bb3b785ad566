cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in base spread base spread; do
  if [ $v = base ]; then unset KNN_AMD_VARIANT; else export KNN_AMD_VARIANT=$v; fi
  echo "variant $v"
  timeout -k 10 200 python tools/tune.py --rounds 3 --d 960 --k 100 fp16:0:0 2>&1 | grep -v amdgpu.ids | grep cand || exit 1
done
