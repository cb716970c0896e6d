#!/bin/bash
# r5g: narrow ConvT two-half pipeline (npipe): correctness, then micro A/B at C1 and C3 shapes
set -u
out=gpurun_out/r5g; mkdir -p $out
V=$PWD/tools/variants
RGAN_LIB=$V/librgan_npipe.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "narrow or convt or image or full_size" --timeout 120 --timeout-method thread -p no:cacheprovider > $out/kt.txt 2>&1 || { echo "kt rc=$?"; tail -30 $out/kt.txt; exit 1; }
tail -1 $out/kt.txt
for v in base npipe base npipe; do
  if [ $v = base ]; then unset RGAN_LIB; else export RGAN_LIB=$V/librgan_$v.so; fi
  timeout -k 10 120 python -u tools/narrow_micro.py 30 > $out/micro_$v.txt 2>&1 || exit 1
  NARROW_SHAPE=C3 timeout -k 10 120 python -u tools/narrow_micro.py 20 >> $out/micro_$v.txt 2>&1 || exit 1
  echo "== $v"; cat $out/micro_$v.txt
done
unset RGAN_LIB
timeout -k 10 400 tools/ab_lib.sh r5g C1 npipe 20 || exit 1
