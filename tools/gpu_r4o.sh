#!/bin/bash
# one-launch small channel sum: kernel + GP tests, C4 bench against the previous build (csold)
set -u
out=gpurun_out/${1:-r4o}; mkdir -p "$out"
stop() { case $1 in 124|134|137|139) echo "STOP: rc=$1 at $2"; exit "$1" ;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gp_gpu.py -m gpu -q -x --timeout 120 \
  --timeout-method thread -p no:cacheprovider > "$out/kern.log" 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -2 "$out/kern.log"; stop $rc kern; [ $rc -eq 0 ] || exit $rc
RGAN_PARITY_AUDIT=$out/audit timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -m gpu -q -x -k "arch1 or wgangp" \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$out/parity.log" 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 "$out/parity.log"; stop $rc parity; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 tools/ab_lib.sh "$(basename $out)" C4 csold 20; rc=$?; stop $rc abC4
