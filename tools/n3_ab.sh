set -u
out=gpurun_out/n3; mkdir -p $out
for v in ${VARIANTS:-head cur}; do
  if [ $v = cur ]; then unset RGAN_LIB; else export RGAN_LIB=$PWD/tools/variants/librgan_$v.so; fi
  echo "== $v"
  timeout -k 10 120 python -u tools/narrow3_micro.py 50 2>&1 | grep -v amdgpu.ids || exit 1
done
