for v in base te s4 t4 all base all; do
  if [ $v = base ]; then unset KNN_AMD_VARIANT; else export KNN_AMD_VARIANT=$v; fi
  echo "variant $v"
  timeout -k 10 120 python tools/tune.py --rounds 7 fp16:0:0 2>&1 | grep -v amdgpu.ids || exit 1
done
