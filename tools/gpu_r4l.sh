#!/bin/bash
# narrow ConvT halo offsets per tile: kernel tests of the narrow paths, micro timing at the C3
# and C1/C2 shapes against the previous build (nmold), VALU count pass
set -u
out=gpurun_out/${1:-r4l}; mkdir -p "$out"
stop() { case $1 in 124|134|137|139) echo "STOP: rc=$1 at $2"; exit "$1" ;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x -k "narrow or image or full_size" --timeout 120 \
  --timeout-method thread -p no:cacheprovider > "$out/kern.log" 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -2 "$out/kern.log"; stop $rc kern; [ $rc -eq 0 ] || exit $rc
for v in base nmold base nmold; do
  if [ $v = base ]; then unset RGAN_LIB; else export RGAN_LIB=$PWD/tools/variants/librgan_$v.so; fi
  echo "== $v"; NARROW_SHAPE=C3 timeout -k 10 120 python -u tools/narrow_micro.py 30 2>/dev/null | grep -v amdgpu.ids; stop $? micro
  timeout -k 10 120 python -u tools/narrow_micro.py 30 2>/dev/null | grep -v amdgpu.ids; stop $? micro2
done
