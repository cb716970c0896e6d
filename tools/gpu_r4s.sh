#!/bin/bash
# split-K BN reduce with 4 splits' loads in flight: kernel tests, then A/B against the previous build (old)
set -u
out=gpurun_out/${1:-r4s}; mkdir -p "$out"
stop() { case $1 in 124|134|137|139) echo "STOP: rc=$1 at $2"; exit "$1" ;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x --timeout 120 \
  --timeout-method thread -p no:cacheprovider > "$out/kern.log" 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -2 "$out/kern.log"; stop $rc kern; [ $rc -eq 0 ] || exit $rc
for wl in C4 C1 C2; do
  timeout -k 10 400 tools/ab_lib.sh "$(basename $out)" $wl old 20; rc=$?; stop $rc ab_$wl; [ $rc -eq 0 ] || exit $rc
done
