#!/bin/bash
# WGRAD staging with 16-B LDS stores: WGRAD kernel tests, micro A/B against the previous build
# (wgold), C3 / C1 bench A/B
set -u
out=gpurun_out/${1:-r4n}; mkdir -p "$out"
stop() { case $1 in 124|134|137|139) echo "STOP: rc=$1 at $2"; exit "$1" ;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gp_gpu.py -m gpu -q -x --timeout 120 \
  --timeout-method thread -p no:cacheprovider > "$out/kern.log" 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -2 "$out/kern.log"; stop $rc kern; [ $rc -eq 0 ] || exit $rc
for v in base wgold base wgold; do
  if [ $v = base ]; then unset RGAN_LIB; else export RGAN_LIB=$PWD/tools/variants/librgan_$v.so; fi
  echo "== $v"; timeout -k 10 120 python -u tools/gemm_micro.py 20 wgrad,convtw 2>/dev/null | grep -v amdgpu.ids
done
unset RGAN_LIB
timeout -k 10 500 tools/ab_lib.sh "$(basename $out)" C3 wgold 20; rc=$?; stop $rc abC3
timeout -k 10 300 tools/ab_lib.sh "$(basename $out)" C1 wgold 20; rc=$?; stop $rc abC1
