out=gpurun_out/r6h; mkdir -p $out
for v in base cur c8b2 base cur; do
  if [ $v = cur ]; then unset RGAN_LIB; else export RGAN_LIB=$PWD/tools/variants/librgan_$v.so; fi
  echo "== $v" >> $out/narrow.txt
  NARROW_SHAPE=C3 timeout -k 10 120 python -u tools/narrow_micro.py 30 >> $out/narrow.txt 2>&1 || exit 1
  timeout -k 10 120 python -u tools/narrow_micro.py 30 >> $out/narrow.txt 2>&1 || exit 1
done
unset RGAN_LIB
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "narrow or image or convt or patch" -q --timeout 300 --timeout-method thread -p no:cacheprovider > $out/ktest.log 2>&1; echo ktest rc=$?; tail -2 $out/ktest.log
grep -v amdgpu.ids $out/narrow.txt
